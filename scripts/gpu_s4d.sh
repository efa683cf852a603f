# GPU: texture kernels + runner texture e2e, then the full gpu suite.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-s4d}
timeout -k 10 300 python -u -m pytest tests/test_gpu_texture.py "tests/test_gpu_runner.py::test_texture_from_train_images" -x -v -s --timeout 200 --timeout-method thread > gpurun_out/tests_tx_$TAG.log 2>&1 || { tail -60 gpurun_out/tests_tx_$TAG.log; exit 1; }
tail -6 gpurun_out/tests_tx_$TAG.log
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 2; }
tail -3 gpurun_out/tests_$TAG.log
