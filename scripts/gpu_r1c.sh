set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_boundary.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_c.log 2>&1 || { tail -40 gpurun_out/gpu_step_c.log; exit 1; }
tail -3 gpurun_out/gpu_step_c.log
timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_c.jsonl 2> gpurun_out/ablate_c.err || exit 2
cat gpurun_out/ablate_c.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_c.json 2> gpurun_out/bench_c.err || exit 3
cat gpurun_out/bench_c.json
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_c -o run -- python $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_c.log 2>&1 || exit 4
find $R/gpurun_out/prof_c -name "*kernel_stats.csv" | head -1 | xargs cat | head -20
