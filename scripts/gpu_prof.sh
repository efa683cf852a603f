# rocprofv3 kernel-trace summary of the default (headline) bench command (no extras / CPU legs),
# then separate FETCH_SIZE and WRITE_SIZE PMC passes of the same command (MI355X_MICROARCH.md).
# Usage: bash scripts/gpu_prof.sh TAG [pmc]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-prof}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 20 --warmup 20 --no-cpu-baseline --no-extras > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 3; }
find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $R/gpurun_out/kernel_stats_$TAG.csv
if [ "$2" = "pmc" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python $R/bench.py --steps 10 --warmup 20 --no-cpu-baseline --no-extras > $R/gpurun_out/pmc_fetch_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_fetch_$TAG.log; exit 4; }
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- python $R/bench.py --steps 10 --warmup 20 --no-cpu-baseline --no-extras > $R/gpurun_out/pmc_write_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_write_$TAG.log; exit 5; }
fi
echo done
