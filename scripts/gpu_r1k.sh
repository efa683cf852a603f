set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_step.py tests/test_gpu_runner.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_k.log 2>&1 || { tail -40 gpurun_out/gpu_step_i.log; exit 1; }
tail -2 gpurun_out/gpu_step_k.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_k.json 2> gpurun_out/bench_k.err || { tail -30 gpurun_out/bench_k.err; exit 3; }
cat gpurun_out/bench_k.json
for SL in 64 128 256; do SLOTS=$SL timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_k_$SL.jsonl 2> gpurun_out/ablate_k.err || exit 4; echo SLOTS=$SL; head -2 gpurun_out/ablate_k_$SL.jsonl; done
cat gpurun_out/ablate_k_128.jsonl
