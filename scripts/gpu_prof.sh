# rocprofv3 kernel-trace summary of the headline bench command (no extras / CPU legs), then
# (with "pmc") separate FETCH_SIZE, WRITE_SIZE and MFMA-busy PMC passes of the same command
# (MI355X_MICROARCH.md: one counter group per pass, no trace domains with --pmc).
# Usage: bash scripts/gpu_prof.sh TAG [pmc]
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-prof}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py --steps 20 --warmup 20 --no-cpu-baseline --no-extras > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 3; }
find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $R/gpurun_out/kernel_stats_$TAG.csv
if [ "$2" = "pmc" ]; then
  CMD="--steps 10 --warmup 20 --no-cpu-baseline --no-extras"
  timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_fetch_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_fetch_$TAG.log; exit 4; }
  timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_write_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_write_$TAG.log; exit 5; }
  timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mfma_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_mfma_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_mfma_$TAG.log; exit 6; }
  cd $R
  python scripts/pmc_traffic.py $(find gpurun_out/pmc_fetch_$TAG -name "*counter_collection.csv" | head -1) $(find gpurun_out/pmc_write_$TAG -name "*counter_collection.csv" | head -1) gpurun_out/pmc_traffic_$TAG.json > /dev/null
  python scripts/pmc_mfma.py $(find gpurun_out/pmc_mfma_$TAG -name "*counter_collection.csv" | head -1) gpurun_out/pmc_mfma_$TAG.json > /dev/null
fi
echo done
