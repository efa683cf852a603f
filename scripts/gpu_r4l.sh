# Round-4 validation: scripts/gpu_r4.sh (given tests, the whole GPU suite, smoke, headline bench,
# 2-rank rehearsal), then BASELINE config 5's per-GPU shape (bench --workload global_refine).
# Usage: bash scripts/gpu_r4l.sh TAG tests...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1
BENCH=1 bash scripts/gpu_r4.sh "$@" || exit $?
timeout -k 10 900 python bench.py --workload global_refine --no-cpu-baseline --no-extras > gpurun_out/bench_gr_$TAG.json 2> gpurun_out/bench_gr_$TAG.err || { tail -20 gpurun_out/bench_gr_$TAG.err; exit 8; }
python -c "import json; d=json.load(open('gpurun_out/bench_gr_$TAG.json')); print('global_refine', d['value'], d['ms_per_step'], {k: v.get('ms') for k, v in d.get('kernels', {}).items()})"
