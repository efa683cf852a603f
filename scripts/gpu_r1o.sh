set -o pipefail
for NC in 1; do for SL in 128; do
NC=$NC SLOTS=$SL ONLY=full,no_scatter_atomics,no_backward_level,no_lds_ops,no_lds_no_flush,flush_no_hbm timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_o.err | tr '\n' ' ' || exit 4; echo
done; done
