# Round-4: GPU tests, then same-box A/B prev (HEAD) vs working tree (timing builds), the working
# tree's ablations (ABL_ONLY), the headline profile. Usage: ABL_ONLY=... bash scripts/gpu_r4j.sh TAG tests...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
if [ $# -gt 0 ]; then
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -60 gpurun_out/newtests_$TAG.log; exit 1; }
tail -3 gpurun_out/newtests_$TAG.log
fi
LIBS="libnof_prev.so libnof_ablate.so" FRAMES="${AB_FRAMES:-64}" ABL_ONLY=full bash scripts/gpu_ab.sh ${TAG}_ab || exit 5
if [ -n "$ABL_ONLY" ]; then
LIBS=libnof_ablate.so FRAMES="${AB_FRAMES:-64}" ABL_ONLY=$ABL_ONLY bash scripts/gpu_ab.sh ${TAG}_abl || exit 6
fi
if [ "${PROF:-1}" = "1" ]; then
bash scripts/gpu_prof_r3.sh $TAG || exit 7
rm -rf gpurun_out/prof_$TAG
fi
