set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_boundary.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_n.log 2>&1 || { tail -40 gpurun_out/gpu_step_n.log; exit 1; }
tail -2 gpurun_out/gpu_step_n.log
for NC in 1 2 3; do for SL in 64 128; do
NC=$NC SLOTS=$SL ONLY=full,no_scatter_atomics,no_backward_level timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_n.err | tr '\n' ' ' || exit 4; echo
done; done
