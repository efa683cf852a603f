set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py -k quad -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/tests_r3s2t.log 2>&1 || { tail -30 gpurun_out/tests_r3s2t.log; exit 1; }
tail -2 gpurun_out/tests_r3s2t.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_r3s2t -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-extras > $GRAFT_REPO_ROOT/gpurun_out/prof_r3s2t.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/prof_r3s2t.log; exit 3; }
grep -h "k_quad_mirror\|k_encode\|k_scatter" $GRAFT_REPO_ROOT/gpurun_out/prof_r3s2t/run_kernel_stats.csv | cut -c1-160
