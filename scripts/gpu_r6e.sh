set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-r6e}
timeout -k 10 900 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_headline.py tests/test_gpu_graph.py -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$T.log 2>&1; rc=$?
grep -E "^(FAILED|ERROR)" gpurun_out/tests_$T.log | head; tail -1 gpurun_out/tests_$T.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
VARIANTS='{"fuse_on": {"scatter_fuse_levels": 0}, "fuse_off": {"scatter_fuse_levels": 1}}' ROUNDS=6 \
  timeout -k 10 400 python scripts/knob_ab.py > gpurun_out/knob_$T.jsonl 2> gpurun_out/knob_$T.err || { tail -20 gpurun_out/knob_$T.err; exit 3; }
cat gpurun_out/knob_$T.jsonl
exit $rc
