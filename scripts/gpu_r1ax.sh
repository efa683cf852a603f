set -o pipefail
cd $GRAFT_REPO_ROOT
ONLY=full,no_mlp_bwd timeout -k 10 400 python scripts/ablate.py > gpurun_out/ablate_ax.jsonl 2> gpurun_out/ablate_ax.err || { tail -20 gpurun_out/ablate_ax.err; exit 1; }
cat gpurun_out/ablate_ax.jsonl
