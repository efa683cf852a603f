# Round-4: GPU tests, same-box A/B of two production builds (libnof_prev.so = HEAD's field_step,
# libnof.so = the working tree) at the headline pool, and the 2048-ray step of both.
# Usage: bash scripts/gpu_r4k.sh TAG tests...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
if [ $# -gt 0 ]; then
timeout -k 10 600 python -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > gpurun_out/newtests_$TAG.log 2>&1 || { tail -60 gpurun_out/newtests_$TAG.log; exit 1; }
tail -3 gpurun_out/newtests_$TAG.log
fi
LIBS="libnof_prev.so libnof.so libnof_prev.so libnof.so" FRAMES="${AB_FRAMES:-64}" ABL_ONLY=full bash scripts/gpu_ab.sh ${TAG} || exit 5
for L in libnof_prev.so libnof.so; do
  NOF_LIB=$R/bundlesdf_amd/$L timeout -k 10 200 python scripts/small_batch_prof.py 501 2>>gpurun_out/sweep_$TAG.err | sed "s/^/$L /" | grep "small batch" | tee -a gpurun_out/sweep_$TAG.txt || exit 2
done
