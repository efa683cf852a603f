set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAVES --kernel-include-regex "k_scatter|k_mlp|k_encode|k_dw|k_compact" --output-format csv -d $R/gpurun_out/pmc_av -o run -- python $R/bench.py --steps 5 --warmup 30 --no-cpu-baseline > $R/gpurun_out/pmc_av.log 2>&1 || { tail -20 $R/gpurun_out/pmc_av.log; exit 3; }
echo done
