# Round-4: new GPU tests, same-box A/B (libnof.so, FLATS x LPWS) at the headline pool, the 2048-ray
# step under SWEEP. Usage: FLATS="0 1" bash scripts/gpu_r4h.sh TAG tests...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
if [ $# -gt 0 ]; then
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -60 gpurun_out/newtests_$TAG.log; exit 1; }
tail -3 gpurun_out/newtests_$TAG.log
fi
for LP in ${LPWS:-0}; do
LPW=$LP LIBS=libnof.so FRAMES="${AB_FRAMES:-64}" ABL_ONLY=full bash scripts/gpu_ab.sh $TAG > /dev/null || exit 5
done
python -c "
import json
for l in open('gpurun_out/ab_$TAG.jsonl'):
    d = json.loads(l); print(d['frames'], 'lpw', d.get('lpw'), 'flat', d.get('flat'), d['field_ms_median'], d['kernels'])"
for v in ${SWEEP:-FLAT=0 FLAT=1}; do
  env ${v//,/ } timeout -k 10 200 python scripts/small_batch_prof.py 501 2>>gpurun_out/sweep_$TAG.err | grep "small batch" | tee -a gpurun_out/sweep_$TAG.txt || exit 2
done
