set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_aa.log 2>&1 || { tail -40 gpurun_out/gpu_step_aa.log; exit 1; }
tail -1 gpurun_out/gpu_step_aa.log
for B in 2 2 1; do
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --blocks-per-cu $B > gpurun_out/bench_aa.json 2> gpurun_out/bench_aa.err || { tail -30 gpurun_out/bench_aa.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_aa.json')); print($B, d['value'], d['ms_per_step'], d['field_step_ms'], d['host_enqueue_ms_per_step'])"
done
