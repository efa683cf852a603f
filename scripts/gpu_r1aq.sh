set -o pipefail
cd $GRAFT_REPO_ROOT
ONLY=full,no_passA,no_mlp_bwd,passB_fwd_only timeout -k 10 400 python scripts/ablate.py > gpurun_out/ablate_aq.jsonl 2> gpurun_out/ablate_aq.err || { tail -20 gpurun_out/ablate_aq.err; exit 1; }
cat gpurun_out/ablate_aq.jsonl
