set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -m pytest tests/test_gpu_step.py -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_step_ap.log 2>&1 || { tail -30 gpurun_out/gpu_step_ap.log; exit 1; }
tail -1 gpurun_out/gpu_step_ap.log
ONLY=full,no_backward_level,no_scatter_atomics,flush_no_hbm timeout -k 10 400 python scripts/ablate.py > gpurun_out/ablate_ap.jsonl 2> gpurun_out/ablate_ap.err || { tail -20 gpurun_out/ablate_ap.err; exit 1; }
cat gpurun_out/ablate_ap.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_ap.json 2> gpurun_out/bench_ap.err || { tail -20 gpurun_out/bench_ap.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_ap.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['scatter_hbm_atomics'], d['loss'])"
