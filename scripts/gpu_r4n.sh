# Round-4: the MLP backward flush modes at the headline pool (64 frames), production lib, twice
# interleaved. Usage: bash scripts/gpu_r4n.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1
for rep in 1 2; do for B in 1 2; do
  BWDF=$B FRAMES=64 NOF_LIB=$R/bundlesdf_amd/libnof.so ONLY=full timeout -k 10 300 python scripts/ablate.py >> gpurun_out/ab_$TAG.jsonl 2>> gpurun_out/ab_$TAG.err || { tail -20 gpurun_out/ab_$TAG.err; exit 1; }
done; done
python -c "
import json
for l in open('gpurun_out/ab_$TAG.jsonl'):
    d = json.loads(l); print(d['frames'], 'bwdf', d.get('bwdf'), d['field_ms_median'], d['kernels'])"
