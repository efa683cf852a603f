# Level-serial scatter sweep at the headline pool (same box): LDS slots per wave x waves per ray,
# against the run-scan scatter. Usage: bash scripts/gpu_sweep_ls.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-sweep}
run() { env "$@" FRAMES=64 ONLY=full timeout -k 10 300 python scripts/ablate.py >> gpurun_out/ab_$TAG.jsonl 2>> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }; }
run SK=2
run SK=3 LSL=8
run SK=3 LSL=6
run SK=3 LSL=10
run SK=1 WPR=1 SLOTS=1024
run SK=1 WPR=2 SLOTS=1024
run SK=1 WPR=4 SLOTS=512
python -c "
import json
for l in open('gpurun_out/ab_$TAG.jsonl'):
    d = json.loads(l); print('sk', d.get('sk'), 'lsl', d.get('lsl'), 'wpr', d.get('wpr'), 'slots', d.get('slots'), d['field_ms_median'], d['kernels'])"
