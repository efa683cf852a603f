# Whole GPU suite without -x (every failure reported), then — only if pytest ended normally
# (0: green, 1: some tests failed; not a fault / abort / time limit) — smoke and the quick bench.
# Usage: bash scripts/gpu_suite_then_bench.sh TAG [pytest files...]
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
TAG=${1:?tag}; shift
FILES=${*:-tests}
timeout -k 10 1000 python -u -m pytest $FILES -m gpu -v --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/tests_$TAG.log | grep -v "^FAILED\|^ERROR" | awk '{print $NF, $1}' | sort | uniq -c | sort -rn | head -3
grep -E "^(FAILED|ERROR)" gpurun_out/tests_$TAG.log | head -20
tail -1 gpurun_out/tests_$TAG.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
  || { tail -20 gpurun_out/smoke_$TAG.log; exit 3; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 400 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_$TAG.json \
  2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 4; }
python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['roofline']['frac'])"
exit $rc
