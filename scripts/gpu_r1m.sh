set -o pipefail
for NC in 1; do for SL in 64 128; do
NC=$NC SLOTS=$SL ONLY=full,no_scatter_atomics,flush_no_hbm,no_backward_level timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_m.err | tr '\n' ' ' || exit 4; echo
done; done
