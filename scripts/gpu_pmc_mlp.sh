# SQ counters of the MLP / scatter kernels (one 8-counter pass): where their waves wait.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SMEM --kernel-include-regex "k_mlp|k_scatter|k_encode" --output-format csv -d $R/gpurun_out/pmc_sq_$1 -o run -- python $R/bench.py --steps 3 --warmup 20 --no-cpu-baseline --no-extras > $R/gpurun_out/pmc_sq_$1.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq_$1.log; exit 3; }
echo done
