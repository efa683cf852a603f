set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_z.log 2>&1 || { tail -40 gpurun_out/gpu_step_z.log; exit 1; }
tail -1 gpurun_out/gpu_step_z.log
for B in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --blocks-per-cu $B > gpurun_out/bench_z$B.json 2> gpurun_out/bench_z.err || { tail -30 gpurun_out/bench_z.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_z$B.json')); print($B, d['value'], d['ms_per_step'], d['kernels'])"
done
