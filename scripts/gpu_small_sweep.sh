# Small-batch (NerfRunner.train()-sized, 2048 rays) knob sweep: scripts/small_batch_prof.py timing lines
# for each "VAR=VALUE ..." set given as an argument (one process each). Usage:
#   bash scripts/gpu_small_sweep.sh TAG "" "LPW=1" "SLOTS=256" ...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:?tag}
shift
for v in "$@"; do
  env $v timeout -k 10 240 python scripts/small_batch_prof.py 300 >> gpurun_out/small_sweep_$TAG.txt 2> gpurun_out/small_sweep_$TAG.err \
    || { tail -20 gpurun_out/small_sweep_$TAG.err; exit 1; }
done
cat gpurun_out/small_sweep_$TAG.txt
