# Round-4 GPU call: the given GPU tests first, then the whole gpu suite, smoke(), the
# headline bench (round protocol) and the self-launched 2-rank rehearsal (gloo, ranks
# sharing cuda:0). Usage: bash scripts/gpu_r4.sh TAG [BENCH=0|1] test_ids...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
if [ $# -gt 0 ]; then
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -60 gpurun_out/newtests_$TAG.log; exit 1; }
tail -3 gpurun_out/newtests_$TAG.log
fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 2; }
tail -2 gpurun_out/smoke_$TAG.log
if [ "${BENCH:-1}" = "1" ]; then
timeout -k 10 900 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 3; }
python -c "import json,sys; d=json.load(open('gpurun_out/bench_$TAG.json')); print({k: d.get(k) for k in ('value','ms_per_step','round_phases_ms_per_step','kernels')}); print('parity', d.get('parity_mode',{}).get('ms_per_step'), 'config2', d.get('config2',{}).get('ms_per_step'))"
NOF_BENCH_BACKEND=gloo NOF_BENCH_SHARE_GPU=1 timeout -k 10 600 python bench.py --gpus 2 --no-extras --no-cpu-baseline > gpurun_out/bench_dp2_$TAG.json 2> gpurun_out/bench_dp2_$TAG.err || { tail -20 gpurun_out/bench_dp2_$TAG.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/bench_dp2_$TAG.json')); print('dp2', d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'])"
fi
if [ "${SPROF:-0}" = "1" ]; then
bash scripts/gpu_small_prof.sh $TAG || exit 6
cp gpurun_out/sprof_$TAG/run_kernel_stats.csv gpurun_out/kernel_stats_parity_$TAG.csv
fi
