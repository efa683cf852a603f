set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r6h}
VARIANTS='{"base": {}, "s256": {"scatter_slots": 256}, "s128": {"scatter_slots": 128}, "lpw1": {"scatter_levels_per_wave": 1}, "lpw1_s128": {"scatter_levels_per_wave": 1, "scatter_slots": 128}, "lpw4_s128": {"scatter_levels_per_wave": 4, "scatter_slots": 128}}' \
  timeout -k 10 500 python scripts/parity_ab.py > gpurun_out/parity_$T.jsonl 2> gpurun_out/parity_$T.err || { tail -20 gpurun_out/parity_$T.err; exit 3; }
cat gpurun_out/parity_$T.jsonl
