set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_h.log 2>&1 || { tail -40 gpurun_out/gpu_step_h.log; exit 1; }
tail -2 gpurun_out/gpu_step_h.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_h.json 2> gpurun_out/bench_h.err || { tail -30 gpurun_out/bench_h.err; exit 3; }
cat gpurun_out/bench_h.json
for B in 1 2; do BPC=$B timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_h_$B.jsonl 2> gpurun_out/ablate_h.err || exit 4; done
cat gpurun_out/ablate_h_1.jsonl | head -1; cat gpurun_out/ablate_h_2.jsonl
