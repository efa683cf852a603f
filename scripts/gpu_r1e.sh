set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_boundary.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_e.log 2>&1 || { tail -40 gpurun_out/gpu_step_e.log; exit 1; }
tail -3 gpurun_out/gpu_step_e.log
for B in 1 2; do for SL in 512 1024; do
BPC=$B SLOTS=$SL timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_e_${B}_${SL}.jsonl 2> gpurun_out/ablate_e.err || exit 2
echo "BPC=$B SLOTS=$SL"; head -1 gpurun_out/ablate_e_${B}_${SL}.jsonl
done; done
cat gpurun_out/ablate_e_2_512.jsonl
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_e -o run -- python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/prof_e.log 2>&1 || exit 4
head -8 $(find $R/gpurun_out/prof_e -name "*kernel_stats.csv" | sort | tail -1) | cut -c1-150
