set -o pipefail
for SL in 256 512; do
SLOTS=$SL ONLY=full,flush_no_hbm,ident_hash,ident_hash_no_hbm,seg_hash,seg_hash_no_hbm timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_s.err | tr '\n' ' ' || exit 4; echo
done
