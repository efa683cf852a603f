# Headline profile (the round protocol): rocprofv3 kernel-trace summary, FETCH_SIZE / WRITE_SIZE /
# MFMA-busy PMC passes (one counter group per pass, no trace
# domains with --pmc: MI355X_MICROARCH.md), and two SQ passes over the field kernels.
# Usage: bash scripts/gpu_prof_headline.sh TAG (or: bash scripts/gpu_run.sh TAG prof)
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-prof}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
CMD="--warmup 20 --no-cpu-baseline --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/prof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/prof_$TAG.log; exit 3; }
find $R/gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $R/gpurun_out/kernel_stats_$TAG.csv
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_fetch_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_fetch_$TAG.log; exit 4; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_write_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_write_$TAG.log; exit 5; }
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmc_mfma_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_mfma_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_mfma_$TAG.log; exit 6; }
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-include-regex "k_mlp|k_scatter|k_encode" --output-format csv -d $R/gpurun_out/pmc_sq1_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_sq1_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq1_$TAG.log; exit 7; }
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS_ATOMIC SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SALU --kernel-include-regex "k_mlp|k_scatter|k_encode" --output-format csv -d $R/gpurun_out/pmc_sq2_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_sq2_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq2_$TAG.log; exit 8; }
cd $R
python scripts/pmc_traffic.py $(find gpurun_out/pmc_fetch_$TAG -name "*counter_collection.csv" | head -1) $(find gpurun_out/pmc_write_$TAG -name "*counter_collection.csv" | head -1) gpurun_out/pmc_traffic_$TAG.json --last 501 --cmd "bench.py $CMD" > /dev/null
python scripts/pmc_mfma.py $(find gpurun_out/pmc_mfma_$TAG -name "*counter_collection.csv" | head -1) gpurun_out/pmc_mfma_$TAG.json --last 501 --cmd "bench.py $CMD" > /dev/null
python scripts/pmc_sq_summary.py $TAG 501 > gpurun_out/pmc_sq_$TAG.txt
rm -rf gpurun_out/pmc_fetch_$TAG gpurun_out/pmc_write_$TAG gpurun_out/pmc_mfma_$TAG gpurun_out/pmc_sq1_$TAG gpurun_out/pmc_sq2_$TAG
echo done
