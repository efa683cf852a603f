# One parameterised GPU launcher (replaces the per-experiment gpu_r*.sh scripts).
# Usage: bash scripts/gpu_run.sh TAG STEPS...   where each step is one of
#   tests[=FILES]   pytest -m gpu on FILES (default: the whole suite)
#   smoke           __graft_entry__.smoke()
#   quick           bench.py --no-extras --no-cpu-baseline (headline line only)
#   bench           the default bench.py line (all side lines, cpu baseline)
#   prof            rocprofv3 kernel-trace summary + PMC passes of the headline (scripts/gpu_prof_headline.sh)
#   sprof           rocprofv3 kernel stats of NerfRunner.train()-sized steps (scripts/gpu_small_prof.sh)
#   ab=LIBS         same-box A/B of library builds (scripts/gpu_ab.sh; FRAMES / ABL_ONLY from the env)
# Every GPU step runs under its own time limit; the script stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:?tag}
shift
for step in "$@"; do
  case "$step" in
    tests|tests=*)
      files=${step#tests}; files=${files#=}; files=${files:-tests}
      timeout -k 10 900 python -u -m pytest ${files//,/ } -m gpu -x -v --timeout 300 --timeout-method thread \
        > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 2; }
      tail -3 gpurun_out/tests_$TAG.log ;;
    smoke)
      timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 \
        || { tail -20 gpurun_out/smoke_$TAG.log; exit 3; }
      tail -2 gpurun_out/smoke_$TAG.log ;;
    quick)
      timeout -k 10 400 python bench.py --no-extras --no-cpu-baseline > gpurun_out/bench_$TAG.json \
        2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 4; }
      python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['roofline']['frac'])" ;;
    bench)
      timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err \
        || { tail -20 gpurun_out/bench_$TAG.err; exit 5; }
      python -c "import json; d=json.load(open('gpurun_out/bench_$TAG.json')); print(d['value'], d['ms_per_step'], {k: v['ms'] for k, v in d['kernels'].items()}, d['roofline']['frac'], d['parity_mode']['ms_per_step'], d['config2']['ms_per_step'])" ;;
    prof)
      bash scripts/gpu_prof_headline.sh $TAG || exit 6 ;;
    sprof)
      bash scripts/gpu_small_prof.sh $TAG > gpurun_out/sprof_top_$TAG.txt 2>&1 || { tail -20 gpurun_out/sprof_top_$TAG.txt; exit 8; }
      cp gpurun_out/sprof_$TAG/run_kernel_stats.csv gpurun_out/kernel_stats_parity_$TAG.csv
      head -12 gpurun_out/sprof_top_$TAG.txt ;;
    ab=*)
      LIBS="${step#ab=}" bash scripts/gpu_ab.sh $TAG || exit 7 ;;
    *) echo "unknown step $step"; exit 9 ;;
  esac
done
echo "gpu_run $TAG done"
