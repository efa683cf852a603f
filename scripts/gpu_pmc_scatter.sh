# SQ counters of k_scatter on the headline bench command (two 8-counter passes).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
TAG=${1:-sc}
timeout -k 10 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS --kernel-include-regex "k_scatter" --output-format csv -d $R/gpurun_out/pmc_sc1_$TAG -o run -- python $R/bench.py --steps 3 --warmup 20 --no-cpu-baseline --no-extras > $R/gpurun_out/pmc_sc1_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sc1_$TAG.log; exit 3; }
timeout -k 10 240 rocprofv3 --pmc SQ_INSTS_LDS_ATOMIC SQ_LDS_ATOMIC_RETURN SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM --kernel-include-regex "k_scatter" --output-format csv -d $R/gpurun_out/pmc_sc2_$TAG -o run -- python $R/bench.py --steps 3 --warmup 20 --no-cpu-baseline --no-extras > $R/gpurun_out/pmc_sc2_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_sc2_$TAG.log; exit 4; }
echo done
