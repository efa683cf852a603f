set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_all_u.log 2>&1 || { tail -40 gpurun_out/gpu_all_u.log; exit 1; }
tail -1 gpurun_out/gpu_all_u.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_u.json 2> gpurun_out/bench_u.err || { tail -30 gpurun_out/bench_u.err; exit 3; }
cat gpurun_out/bench_u.json
