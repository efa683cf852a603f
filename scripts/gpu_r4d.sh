# Round-4: GPU step tests, then the NerfRunner.train()-sized step under the MLP backward flush /
# scatter shapes (scripts/gpu_small_sweep.sh). Usage: bash scripts/gpu_r4d.sh TAG [tests...]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
if [ $# -gt 0 ]; then
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -60 gpurun_out/newtests_$TAG.log; exit 1; }
tail -3 gpurun_out/newtests_$TAG.log
fi
SWEEP="${SWEEP:-BWDF=1 BWDF=2 BWDF=2,SLOTS=128 BWDF=2,SLOTS=256 BWDF=2,SLOTS=128,LPW=1 BWDF=2,SLOTS=256,LPW=4}"
for v in $SWEEP; do
  env ${v//,/ } timeout -k 10 200 python scripts/small_batch_prof.py 501 2>>gpurun_out/sweep_$TAG.err | grep "small batch" | tee -a gpurun_out/sweep_$TAG.txt || exit 2
done
