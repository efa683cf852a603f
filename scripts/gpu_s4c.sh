# GPU: new-feature tests first (hand-off, ray pool), then the full gpu suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-s4c}
timeout -k 10 300 python -u -m pytest tests/test_gpu_handoff.py -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_ho_$TAG.log 2>&1 || { tail -60 gpurun_out/tests_ho_$TAG.log; exit 1; }
tail -8 gpurun_out/tests_ho_$TAG.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 2; }
tail -3 gpurun_out/tests_$TAG.log
