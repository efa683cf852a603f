set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_all_ak.log 2>&1 || { tail -50 gpurun_out/gpu_all_ak.log; exit 1; }
tail -2 gpurun_out/gpu_all_ak.log
