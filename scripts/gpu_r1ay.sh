set -o pipefail
cd $GRAFT_REPO_ROOT
ONLY=full,no_insert,cas_only,add_only timeout -k 10 400 python scripts/ablate.py > gpurun_out/ablate_ay.jsonl 2> gpurun_out/ablate_ay.err || { tail -20 gpurun_out/ablate_ay.err; exit 1; }
python -c "
import json
for l in open('gpurun_out/ablate_ay.jsonl'):
    d = json.loads(l); print(d['variant'], d['kernels']['k_scatter'])
"
