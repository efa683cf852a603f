set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r6i}
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -m gpu -v -k "sampler_kernel or g4amp or matches_reference_train_loop" --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 2; }
tail -1 gpurun_out/tests_$T.log
VARIANTS='{"base": {}, "samp": {"encode_wpb": 256}}' ROUNDS=6 \
  timeout -k 10 400 python scripts/knob_ab.py > gpurun_out/knob_$T.jsonl 2> gpurun_out/knob_$T.err || { tail -20 gpurun_out/knob_$T.err; exit 3; }
cat gpurun_out/knob_$T.jsonl
VARIANTS='{"base": {}, "s256": {"scatter_slots": 256}, "s128": {"scatter_slots": 128}, "lpw1": {"scatter_levels_per_wave": 1}, "lpw1_s128": {"scatter_levels_per_wave": 1, "scatter_slots": 128}, "samp": {"encode_wpb": 256}}' \
  timeout -k 10 500 python scripts/parity_ab.py > gpurun_out/parity_$T.jsonl 2> gpurun_out/parity_$T.err || { tail -20 gpurun_out/parity_$T.err; exit 4; }
cat gpurun_out/parity_$T.jsonl
