set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU --kernel-include-regex "k_scatter|k_mlp|k_encode|k_dw" --output-format csv -d $R/gpurun_out/pmc_sq -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_sq.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq.log; exit 3; }
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_LDS_IDX_ACTIVE SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY --kernel-include-regex "k_scatter|k_mlp|k_encode|k_dw" --output-format csv -d $R/gpurun_out/pmc_sq2 -o run -- python $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $R/gpurun_out/pmc_sq2.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq2.log; exit 4; }
echo done
