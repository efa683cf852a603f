# Round-4: same-box A/B of the scatter kernels (level-serial 1 vs run-scan 2) at the headline
# pool, then scripts/gpu_r4.sh (tests, suite, smoke, bench). Usage: bash scripts/gpu_r4b.sh TAG tests...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1
LIBS=libnof.so FRAMES="${AB_FRAMES:-64}" SKS="1 2" ESIGS="0 1" ABL_ONLY=full bash scripts/gpu_ab.sh $TAG || exit 5
bash scripts/gpu_r4.sh "$@"
