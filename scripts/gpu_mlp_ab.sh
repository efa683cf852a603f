# Same-box A/B of MLP-backward builds: the previous commit's (libnof_prev.so) against the working
# tree's (libnof.so), alternating, then the step parity tests on the working tree's build.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-mlpab}
LIBS=${LIBS_AB:-"libnof_prev.so libnof.so libnof_prev.so libnof.so libnof_prev.so libnof.so"} FRAMES=${FRAMES_AB:-64} bash scripts/gpu_ab.sh $T || exit 2
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_headline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 3; }
tail -1 gpurun_out/tests_$T.log
