set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r6g}
VARIANTS='{"fuse_off": {"scatter_fuse_levels": 1}, "fuse_p1": {"scatter_fuse_levels": 0}}' ROUNDS=5 \
  timeout -k 10 500 python scripts/knob_ab.py > gpurun_out/knob_$T.jsonl 2> gpurun_out/knob_$T.err || { tail -20 gpurun_out/knob_$T.err; exit 3; }
cat gpurun_out/knob_$T.jsonl
