# Round-3 GPU call (second form): A/B of the timing builds (ABL_ONLY / LIBS as gpu_r3.sh), the given
# GPU tests, then the config-5 global-refine bench line. Usage: bash scripts/gpu_r3b.sh TAG test_ids...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
LIBS="${LIBS:-libnof_ablate.so}" FRAMES=64 ABL_ONLY="${ABL_ONLY:-full}" bash scripts/gpu_ab.sh $TAG || exit 5
timeout -k 10 400 python -u -m pytest "$@" -x -v --timeout 200 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -40 gpurun_out/newtests_$TAG.log; exit 1; }
tail -3 gpurun_out/newtests_$TAG.log
timeout -k 10 600 python bench.py --workload global_refine --steps 501 > gpurun_out/bench_gr_$TAG.json 2> gpurun_out/bench_gr_$TAG.err || { tail -20 gpurun_out/bench_gr_$TAG.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_gr_$TAG.json')); print({k: d[k] for k in ('value','ms_per_step','round_phases_ms_per_step','kernels')})"
