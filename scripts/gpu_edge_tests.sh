set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py -m gpu -v -k "ragged" --timeout 200 --timeout-method thread > gpurun_out/tests_r6x.log 2>&1 || { tail -60 gpurun_out/tests_r6x.log; exit 2; }
tail -12 gpurun_out/tests_r6x.log
