# Same-box knob A/B on NerfRunner.train()'s 2048-ray step (scripts/parity_ab.py); VARIANTS from the env.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
T=${1:-pknob}
REPS=${REPS:-4} STEPS=${STEPS:-300} timeout -k 10 500 python scripts/parity_ab.py > gpurun_out/parity_$T.jsonl 2> gpurun_out/parity_$T.err || { tail -20 gpurun_out/parity_$T.err; exit 3; }
cat gpurun_out/parity_$T.jsonl
