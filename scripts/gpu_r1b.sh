set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_boundary.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_2.log 2>&1 || { tail -40 gpurun_out/gpu_step_2.log; exit 1; }
tail -3 gpurun_out/gpu_step_2.log
timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_r1b.jsonl 2> gpurun_out/ablate_r1b.err || exit 2
cat gpurun_out/ablate_r1b.jsonl
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r1b.json 2> gpurun_out/bench_r1b.err || exit 3
cat gpurun_out/bench_r1b.json
