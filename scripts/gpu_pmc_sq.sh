# SQ counters of the kernels matching REGEX on the headline bench command (two 8-counter
# passes, no trace domains). Usage: bash scripts/gpu_pmc_sq.sh TAG REGEX
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
TAG=${1:-sq}
RX=${2:-k_encode|k_mlp|k_scatter}
CMD="--steps 3 --warmup 20 --no-cpu-baseline --no-extras --no-graph"
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU --kernel-include-regex "$RX" --output-format csv -d $R/gpurun_out/pmc_sq1_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_sq1_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq1_$TAG.log; exit 3; }
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "$RX" --output-format csv -d $R/gpurun_out/pmc_sq2_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_sq2_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq2_$TAG.log; exit 4; }
echo done
