set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_ac.log 2>&1 || { tail -40 gpurun_out/gpu_step_ac.log; exit 1; }
tail -1 gpurun_out/gpu_step_ac.log
for SL in 256 512; do
SLOTS=$SL ONLY=full,fib_hash,no_lds_ops,flush_no_hbm timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_ac.err | tr '\n' ' ' || exit 4; echo
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_ac.json 2> gpurun_out/bench_ac.err || { tail -30 gpurun_out/bench_ac.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_ac.json')); print(d['value'], d['ms_per_step'], d['field_step_ms'], d['kernels'], d['scatter_hbm_atomics'])"
