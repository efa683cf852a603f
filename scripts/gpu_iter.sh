# Iteration check: scatter ablation breakdown (timing build), the step / optimiser parity
# tests, then the headline bench line without the extra lines. Usage: bash scripts/gpu_iter.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-iter}
NOF_LIB=$R/bundlesdf_amd/libnof_ablate.so ONLY=${ABL_ONLY:-full,no_scatter_atomics,no_backward_level,f32_lds} timeout -k 10 300 python scripts/ablate.py > gpurun_out/ablate_$TAG.jsonl 2> gpurun_out/ablate_$TAG.err || { tail -20 gpurun_out/ablate_$TAG.err; exit 1; }
cat gpurun_out/ablate_$TAG.jsonl
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_gpu_step.py tests/test_gpu_optim.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -30 gpurun_out/tests_$TAG.log; exit 2; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['roofline'])"
