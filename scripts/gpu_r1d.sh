set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_boundary.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_d.log 2>&1 || { tail -40 gpurun_out/gpu_step_d.log; exit 1; }
tail -3 gpurun_out/gpu_step_d.log
timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_d.jsonl 2> gpurun_out/ablate_d.err || exit 2
cat gpurun_out/ablate_d.jsonl
SLOTS=512 timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_d512.jsonl 2> gpurun_out/ablate_d512.err || exit 2
head -1 gpurun_out/ablate_d512.jsonl
SLOTS=2048 timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_d2048.jsonl 2> gpurun_out/ablate_d2048.err || exit 2
head -1 gpurun_out/ablate_d2048.jsonl
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_d -o run -- python $R/bench.py --steps 20 --warmup 5 > $R/gpurun_out/prof_d.log 2>&1 || exit 4
cat $(find $R/gpurun_out/prof_d -name "*kernel_stats.csv" | sort | tail -1)
