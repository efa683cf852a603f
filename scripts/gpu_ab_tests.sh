# A/B timing of libnof_prev.so vs libnof_ablate.so at the 64-frame pool (ABL_ONLY variants), then the
# given GPU tests with the product library. Usage: ABL_ONLY=full,... bash scripts/gpu_ab_tests.sh TAG tests...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1; shift
LIBS="${LIBS:-libnof_prev.so libnof_ablate.so}" FRAMES=64 ABL_ONLY="${ABL_ONLY:-full}" bash scripts/gpu_ab.sh $TAG || exit 5
if [ $# -gt 0 ]; then
  timeout -k 10 500 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
  tail -2 gpurun_out/tests_$TAG.log
fi
