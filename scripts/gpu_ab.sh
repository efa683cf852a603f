# A/B timing of two library builds on the same box: scripts/ablate.py (variants in ABL_ONLY)
# with NOF_LIB = each of LIBS, at FRAMES frames (16: config 2, 64: headline pool).
# Usage: LIBS="libnof_prev.so libnof_ablate.so" FRAMES=64 bash scripts/gpu_ab.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-ab}
for L in ${LIBS:-libnof_prev.so libnof_ablate.so}; do
  for F in ${FRAMES:-16 64}; do
   for SKV in ${SKS:-0}; do
    SK=$SKV FRAMES=$F NOF_LIB=$R/bundlesdf_amd/$L ONLY=${ABL_ONLY:-full} timeout -k 10 300 python scripts/ablate.py >> gpurun_out/ab_$TAG.jsonl 2> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
   done
  done
done
python -c "
import json
for l in open('gpurun_out/ab_$TAG.jsonl'):
    d = json.loads(l); print(d['lib'], d['frames'], 'sk', d.get('sk'), d['variant'], d['field_ms_median'], d['kernels'])"
