set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r6j}
timeout -k 10 300 python -u -m pytest tests/test_gpu_headline.py -m gpu -v -k "pipelined" --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -40 gpurun_out/tests_$T.log; exit 2; }
tail -1 gpurun_out/tests_$T.log
VARIANTS='{"one": {}, "c2": {"field_chunks": 2}, "c2s": {"field_chunks": 2, "field_split": 3}, "c3s": {"field_chunks": 4, "field_split": 3}, "c4": {"field_chunks": 4}}' REPS=4 STEPS=100 \
  timeout -k 10 400 python scripts/chunk_ab.py > gpurun_out/chunk_$T.jsonl 2> gpurun_out/chunk_$T.err || { tail -20 gpurun_out/chunk_$T.err; exit 3; }
cat gpurun_out/chunk_$T.jsonl
