# Round 6: deferred-optimiser same-box A/B; SQ counters of the pass-1 MLP backward shapes (knob_ab variants).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
T=${1:-r6d}
timeout -k 10 500 python scripts/defer_ab.py > gpurun_out/defer_$T.jsonl 2> gpurun_out/defer_$T.err || { tail -20 gpurun_out/defer_$T.err; exit 2; }
cat gpurun_out/defer_$T.jsonl
cd /tmp && export TMPDIR=/tmp
export VARIANTS='{"p1_1": {"mlp_pass1_tiles": 1}, "p1_12": {"mlp_pass1_tiles": 12}, "p1_22": {"mlp_pass1_tiles": 22}}'
export ROUNDS=2 WARM=10
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU --kernel-include-regex "k_mlp_bwd" --output-format csv -d $R/gpurun_out/pmc_sq1_$T -o run -- python $R/scripts/knob_ab.py > $R/gpurun_out/pmc_sq1_$T.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq1_$T.log; exit 3; }
timeout -s KILL 240 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INST_CYCLES_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA --kernel-include-regex "k_mlp_bwd" --output-format csv -d $R/gpurun_out/pmc_sq2_$T -o run -- python $R/scripts/knob_ab.py > $R/gpurun_out/pmc_sq2_$T.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sq2_$T.log; exit 4; }
cd $R && python scripts/pmc_sq_summary.py $T 6
