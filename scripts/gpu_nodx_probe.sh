# Upper bound of the scatter's input-gradient share: the headline field pass with frozen poses
# (skip_pose_grad: no corner re-gather, no slopes) against the default, same box, interleaved.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
VARIANTS='{"base": {}, "nodx": {"pose_grad": false}}' ROUNDS=6 \
  timeout -k 10 400 python scripts/knob_ab.py > gpurun_out/knob_nodx.jsonl 2> gpurun_out/knob_nodx.err || { tail -20 gpurun_out/knob_nodx.err; exit 3; }
cat gpurun_out/knob_nodx.jsonl
