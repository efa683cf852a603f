# Round-4: timing-build ablations (ABL_ONLY) at the headline pool, then the headline profile
# (scripts/gpu_prof_r3.sh: kernel stats + PMC traffic / MFMA / SQ). Usage: ABL_ONLY=... bash scripts/gpu_r4i.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1
LIBS=libnof_ablate.so FRAMES="${AB_FRAMES:-64}" ABL_ONLY=${ABL_ONLY:-full} bash scripts/gpu_ab.sh $TAG || exit 5
if [ "${PROF:-1}" = "1" ]; then
bash scripts/gpu_prof_r3.sh $TAG || exit 6
rm -rf gpurun_out/prof_$TAG
fi
