# Same-box A/B of k_scatter builds: the previous commit's (libnof_prev.so), the working tree's
# (libnof.so) and a variant build (libnof_v2.so), alternating twice, then the scatter parity tests on
# the working tree's build.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-scatab}
LIBS=${LIBS_AB:-"libnof_prev.so libnof.so libnof_v2.so libnof_prev.so libnof.so libnof_v2.so"} FRAMES=64 bash scripts/gpu_ab.sh $T || exit 2
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -m gpu -x -q -k "matches_oracle or reference_train_loop or ragged" --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 3; }
tail -1 gpurun_out/tests_$T.log
