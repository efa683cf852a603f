# Same-box A/B of k_encode builds: the previous commit's production library (scripts/build_prev.py
# PROD=1 -> libnof_prev.so) against the working tree's (libnof.so), alternating, then the encode's
# two-level gather group (encode_group 2) against the default on the working tree's build.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-encab}
LIBS="libnof_prev.so libnof.so libnof_prev.so libnof.so libnof_prev.so libnof.so" FRAMES=64 bash scripts/gpu_ab.sh $T || exit 2
VARIANTS='{"g1": {}}' ROUNDS=1 \
  timeout -k 10 400 python scripts/knob_ab.py > gpurun_out/knob_$T.jsonl 2> gpurun_out/knob_$T.err || { tail -20 gpurun_out/knob_$T.err; exit 3; }
cat gpurun_out/knob_$T.jsonl
