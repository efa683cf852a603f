# Same-box A/B of two library builds on whole graph-replayed steps (for kernels outside the field
# pass): NerfRunner.train()'s 2048-ray step (scripts/parity_ab.py) and the headline step
# (scripts/chunk_ab.py), each build in its own process, alternating; then the step tests.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-steplib}
for rep in 1 2 3; do
  for L in libnof_prev.so libnof.so; do
    NOF_LIB=$GRAFT_REPO_ROOT/bundlesdf_amd/$L VARIANTS="{\"$L\": {}}" REPS=2 STEPS=300 timeout -k 10 200 python scripts/parity_ab.py >> gpurun_out/steplib_$T.jsonl 2>> gpurun_out/steplib_$T.err || { tail -20 gpurun_out/steplib_$T.err; exit 2; }
    NOF_LIB=$GRAFT_REPO_ROOT/bundlesdf_amd/$L VARIANTS="{\"$L\": {}}" REPS=2 STEPS=60 timeout -k 10 200 python scripts/chunk_ab.py >> gpurun_out/steplib_$T.jsonl 2>> gpurun_out/steplib_$T.err || { tail -20 gpurun_out/steplib_$T.err; exit 3; }
  done
done
cat gpurun_out/steplib_$T.jsonl
timeout -k 10 400 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_boundary.py tests/test_gpu_graph.py tests/test_gpu_runner.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_$T.log 2>&1 || { tail -30 gpurun_out/tests_$T.log; exit 4; }
tail -1 gpurun_out/tests_$T.log
