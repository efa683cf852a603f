# Block-order experiment: default bench (no extras) with dispatch vs XCD-contiguous block order.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for X in ${XCD_LIST:-0 1 2 3}; do
  NOF_XCD_ORDER=$X timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_xcd$X.json 2> gpurun_out/bench_xcd$X.err || { tail -20 gpurun_out/bench_xcd$X.err; exit 3; }
  python -c "import json; d=json.load(open('gpurun_out/bench_xcd$X.json')); print($X, d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
