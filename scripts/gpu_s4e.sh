# GPU: fused MLP backward+dW path — step parity tests, then bench fused vs records.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-s4e}
timeout -k 10 300 python -u -m pytest tests/test_gpu_step.py tests/test_gpu_runner.py -x -v --timeout 200 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -60 gpurun_out/tests_$TAG.log; exit 1; }
tail -4 gpurun_out/tests_$TAG.log
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 20 > gpurun_out/bench_fused_$TAG.json 2> gpurun_out/bench_fused_$TAG.err || { tail -20 gpurun_out/bench_fused_$TAG.err; exit 2; }
NOF_MLP_PATH=records timeout -k 10 200 python bench.py --no-cpu-baseline --steps 50 --warmup 20 > gpurun_out/bench_rec_$TAG.json 2> gpurun_out/bench_rec_$TAG.err || { tail -20 gpurun_out/bench_rec_$TAG.err; exit 3; }
python - <<'PY'
import json,sys
for n in ("fused","rec"):
    d=json.load(open(f"gpurun_out/bench_{n}_{sys.argv[1] if len(sys.argv)>1 else 's4e'}.json"))
    print(n, d["value"], d["ms_per_step"], {k: v["ms"] for k, v in d["kernels"].items()}, d["loss"])
PY
