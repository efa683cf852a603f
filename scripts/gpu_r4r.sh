# Round-4: scatter group size / table size at the headline pool with the final build (production lib).
# Usage: bash scripts/gpu_r4r.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1
for v in LPW=8 LPW=4 LPW=16 LPW=8,SLOTS=256 LPW=8; do
  env ${v//,/ } FRAMES=64 NOF_LIB=$R/bundlesdf_amd/libnof.so ONLY=full timeout -k 10 300 python scripts/ablate.py >> gpurun_out/ab_$TAG.jsonl 2>> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
done
python -c "
import json
for l in open('gpurun_out/ab_$TAG.jsonl'):
    d = json.loads(l); print('lpw', d.get('lpw'), 'slots', d.get('slots'), d['field_ms_median'], d['kernels'].get('k_scatter'))"
