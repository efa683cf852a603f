set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_l.log 2>&1 || { tail -40 gpurun_out/gpu_step_l.log; exit 1; }
tail -2 gpurun_out/gpu_step_l.log
for NC in 1 2 3; do for SL in 32 64 128; do
NC=$NC SLOTS=$SL ONLY=full,no_scatter_atomics timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_l.err | tr '\n' ' ' || exit 4; echo
done; done
