set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_w.log 2>&1 || { tail -40 gpurun_out/gpu_step_w.log; exit 1; }
tail -1 gpurun_out/gpu_step_w.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_w.json 2> gpurun_out/bench_w.err || { tail -30 gpurun_out/bench_w.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_w.json')); print(d['value'], d['ms_per_step'], d['kernels'])"
