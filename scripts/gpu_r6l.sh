set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r6l}
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -m gpu -v -k "quad_mirror" --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -40 gpurun_out/tests_$T.log; exit 2; }
tail -1 gpurun_out/tests_$T.log
VARIANTS='{"quad16": {}, "cell32": {"quad_layout": 1}}' ROUNDS=6 \
  timeout -k 10 400 python scripts/knob_ab.py > gpurun_out/knob_$T.jsonl 2> gpurun_out/knob_$T.err || { tail -20 gpurun_out/knob_$T.err; exit 3; }
cat gpurun_out/knob_$T.jsonl
VARIANTS='{"quad16": {}, "cell32": {"quad_layout": 1}}' REPS=4 STEPS=100 \
  timeout -k 10 400 python scripts/chunk_ab.py > gpurun_out/step_$T.jsonl 2> gpurun_out/step_$T.err || { tail -20 gpurun_out/step_$T.err; exit 4; }
cat gpurun_out/step_$T.jsonl
