# Round 6: pass-1 multi-tile parity + same-box A/B, deferred optimiser on / off on the bench's side lines.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r6c}
timeout -k 10 600 python -u -m pytest tests/test_gpu_step.py -m gpu -v -k "mlp_pass1" --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 2; }
tail -2 gpurun_out/tests_$T.log
VARIANTS='{"p1_1": {"mlp_pass1_tiles": 1}, "p1_12": {"mlp_pass1_tiles": 12}, "p1_13": {"mlp_pass1_tiles": 13}, "p1_22": {"mlp_pass1_tiles": 22}}' \
  timeout -k 10 400 python scripts/knob_ab.py > gpurun_out/knob_$T.jsonl 2> gpurun_out/knob_$T.err || { tail -20 gpurun_out/knob_$T.err; exit 3; }
cat gpurun_out/knob_$T.jsonl
for D in 1 0; do
  NOF_DEFER_OPT=$D timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/bench_${T}_defer$D.json 2> gpurun_out/bench_${T}_defer$D.err \
    || { tail -20 gpurun_out/bench_${T}_defer$D.err; exit 4; }
  python -c "import json; d=json.load(open('gpurun_out/bench_${T}_defer$D.json')); print('defer $D', d['value'], d['ms_per_step'], d['other_execution']['ms_per_step'], 'parity', d['parity_mode']['ms_per_step'], d['parity_mode']['eager']['ms_per_step'], 'config2', d['config2']['ms_per_step'], 'config1', d['config1']['ms_per_step'])"
done
