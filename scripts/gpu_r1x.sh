set -o pipefail
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_x$i.json 2> gpurun_out/bench_x.err || { tail -30 gpurun_out/bench_x.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_x$i.json')); print(d['value'], d['ms_per_step'], d['field_step_ms'], d['kernels'])"
done
