# Round-4 session 3: same-box A/B of the forward layouts (encode_sigma 1 tiles / 2 off / 3 per-ray)
# x scatter kernels (2 run-scan, 3 hybrid) at the headline pool, then scripts/gpu_r4.sh.
# Usage: bash scripts/gpu_r4c.sh TAG tests...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=$1
LIBS=libnof.so FRAMES="${AB_FRAMES:-64}" SKS="${SKS:-2 3}" ESIGS="${ESIGS:-1 2 3}" ABL_ONLY=full bash scripts/gpu_ab.sh $TAG || exit 5
bash scripts/gpu_r4.sh "$@"
