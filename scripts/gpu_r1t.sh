set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_runner.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_t.log 2>&1 || { tail -40 gpurun_out/gpu_step_t.log; exit 1; }
tail -1 gpurun_out/gpu_step_t.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_t.json 2> gpurun_out/bench_t.err || { tail -30 gpurun_out/bench_t.err; exit 3; }
cat gpurun_out/bench_t.json
