# Round-1 final: all GPU tests, then the rocprofv3 kernel-trace summary of the default bench
# command, then the default bench line (each step under its own time limit, stop at the first failure).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_final.log 2>&1 || { tail -30 gpurun_out/tests_final.log; exit 1; }
tail -3 gpurun_out/tests_final.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_final -o run -- python $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_final.log 2>&1 || { tail -20 $R/gpurun_out/prof_final.log; exit 3; }
cd $R && timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -20 gpurun_out/bench_final.err; exit 6; }
cat gpurun_out/bench_final.json
