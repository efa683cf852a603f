set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_boundary.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_f.log 2>&1 || { tail -40 gpurun_out/gpu_step_f.log; exit 1; }
tail -3 gpurun_out/gpu_step_f.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_f.json 2> gpurun_out/bench_f.err || { tail -30 gpurun_out/bench_f.err; exit 3; }
cat gpurun_out/bench_f.json
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_f -o run -- python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_f.log 2>&1 || exit 4
head -8 $(find $R/gpurun_out/prof_f -name "*kernel_stats.csv" | sort | tail -1) | cut -c1-150
