# Round-4: ablation A/B (timing build; ABL_ONLY variants, ESIGS / SKS) at the headline pool, then
# scripts/gpu_r4.sh (tests, suite, smoke, bench). Usage: ABL_ONLY=full,x bash scripts/gpu_r4e.sh TAG tests...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1
LIBS=libnof_ablate.so FRAMES="${AB_FRAMES:-64}" SKS="${SKS:-0}" ESIGS="${ESIGS:-0}" ABL_ONLY=${ABL_ONLY:-full} bash scripts/gpu_ab.sh $TAG || exit 5
bash scripts/gpu_r4.sh "$@"
