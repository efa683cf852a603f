set -o pipefail
timeout -k 10 300 python -m pytest tests/test_gpu_runner.py -m gpu -x -q -s -p no:cacheprovider -k extract_mesh > gpurun_out/gpu_mesh_al.log 2>&1 || { tail -50 gpurun_out/gpu_mesh_al.log; exit 1; }
grep -E "mesh:|passed|failed" gpurun_out/gpu_mesh_al.log
