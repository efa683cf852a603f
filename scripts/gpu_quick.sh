# Quick iteration: the step / optimiser / graph parity tests, then the headline bench line
# without the side configurations. Usage: bash scripts/gpu_quick.sh TAG [bench args...]
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-quick}
shift || true
timeout -k 10 500 python -u -m pytest ${TESTS:-tests/test_gpu_step.py tests/test_gpu_optim.py tests/test_gpu_graph.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 2; }
tail -2 gpurun_out/tests_$TAG.log
timeout -k 10 300 python bench.py --no-extras --no-cpu-baseline "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 3; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['roofline']['frac'])"
