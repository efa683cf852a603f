set -o pipefail
for cfg in "1 64" "1 128" "2 32" "2 64" "2 128"; do set -- $cfg
NC=$1 SLOTS=$2 ONLY=full,no_lds_ops timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_p.err | tr '\n' ' ' || exit 4; echo
done
