set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_aj.log 2>&1 || { tail -40 gpurun_out/gpu_step_ae.log; exit 1; }
tail -1 gpurun_out/gpu_step_aj.log
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_aj$i.json 2> gpurun_out/bench_aj.err || { tail -30 gpurun_out/bench_aj.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_aj$i.json')); print(d['value'], d['ms_per_step'], d['field_step_ms'], d['host_enqueue_ms_per_step'], d['kernels'])"
done
