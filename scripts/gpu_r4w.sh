# Round-4: hybrid scatter (coarse levels level-serial, the rest run-scan) with few level-serial
# levels, same box as the default run-scan kernel (production build, headline pool).
# Usage: bash scripts/gpu_r4w.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-r4w}
run() {  # SK LSL LPW
  SK=$1 LSL=$2 LPW=$3 FRAMES=64 NOF_LIB=$R/bundlesdf_amd/libnof.so ONLY=full timeout -k 10 300 python scripts/ablate.py \
    >> gpurun_out/ab_$TAG.jsonl 2>> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
}
run 0 0 0
run 3 2 7
run 3 3 7
run 3 4 6
run 0 0 0
run 3 2 7
run 3 3 7
python -c "
import json
for l in open('gpurun_out/ab_$TAG.jsonl'):
    d = json.loads(l); print('sk', d.get('sk'), 'lsl', d.get('lsl'), 'lpw', d.get('lpw'), d['field_ms_median'], d['kernels'])"
