# Same-box knob A/B on the working tree's build (scripts/knob_ab.py); VARIANTS from the environment.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-knob}
ROUNDS=${ROUNDS:-6} timeout -k 10 500 python scripts/knob_ab.py > gpurun_out/knob_$T.jsonl 2> gpurun_out/knob_$T.err || { tail -20 gpurun_out/knob_$T.err; exit 3; }
cat gpurun_out/knob_$T.jsonl
