# NerfRunner.train()-sized step (2048 rays, graph replay, whole round) under scatter shapes.
# Usage: bash scripts/gpu_small_sweep.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
for v in ${SWEEP:-"SLOTS=0" "SLOTS=128" "SLOTS=256" "SLOTS=128 LPW=1" "SLOTS=256 LPW=4"}; do
  env $v timeout -k 10 200 python scripts/small_batch_prof.py 501 2>/dev/null | grep "small batch" || exit 1
done
