set -o pipefail
cd $GRAFT_REPO_ROOT
ONLY=full,no_scatter_atomics,flush_no_hbm,no_lds_ops,no_lds_no_flush,no_backward_level,no_lds_table,f32_lds timeout -k 10 400 python scripts/ablate.py > gpurun_out/ablate_ao.jsonl 2> gpurun_out/ablate_ao.err || { tail -20 gpurun_out/ablate_ao.err; exit 1; }
cat gpurun_out/ablate_ao.jsonl
