# NerfRunner.train()'s step: graph_step_epoch (slice read on the device) against graph_step_ids (a
# per-step id copy), same process, alternating; then the graph / runner / headline tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-epochab}
VARIANTS='{"ids_copy": {"_path": "ids"}, "epoch": {}}' REPS=4 STEPS=300 \
  timeout -k 10 400 python scripts/parity_ab.py > gpurun_out/parity_$T.jsonl 2> gpurun_out/parity_$T.err || { tail -20 gpurun_out/parity_$T.err; exit 2; }
cat gpurun_out/parity_$T.jsonl
timeout -k 10 500 python -u -m pytest tests/test_gpu_graph.py tests/test_gpu_runner.py tests/test_gpu_headline.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 3; }
tail -1 gpurun_out/tests_$T.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$T.json 2> gpurun_out/bench_$T.err || { tail -20 gpurun_out/bench_$T.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/bench_$T.json')); print(d['value'], d['ms_per_step'], d['parity_mode']['ms_per_step'], d['config2']['ms_per_step'])"
