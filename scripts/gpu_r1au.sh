set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py --steps 20 --warmup 30 --blocks-per-cu 1 --no-cpu-baseline > gpurun_out/bench_au.json 2> gpurun_out/bench_au.err || { tail -20 gpurun_out/bench_au.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/bench_au.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
