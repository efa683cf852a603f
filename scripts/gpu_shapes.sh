# Per-rank shapes of the strong-scaling headline at N = 2, 4, 8 (64/N frames per rank), timed at
# N = 1 on one GPU (the rank's whole step without the exchange), for DESIGN §6's modelled scaling.
# Usage: bash scripts/gpu_shapes.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-shapes}
for F in 32 16 8; do
  timeout -k 10 300 python bench.py --frames-per-gpu $F --no-extras --no-cpu-baseline > gpurun_out/shape_${TAG}_f$F.json 2> gpurun_out/shape_${TAG}_f$F.err || { tail -20 gpurun_out/shape_${TAG}_f$F.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/shape_${TAG}_f$F.json')); print($F, d['ms_per_step'], d['value'], {k: v['ms'] for k, v in d['kernels'].items()})"
done
