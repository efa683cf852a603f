set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_q.log 2>&1 || { tail -40 gpurun_out/gpu_step_q.log; exit 1; }
tail -1 gpurun_out/gpu_step_q.log
for cfg in "1 256" "1 512" "1 1024" "2 256" "2 512"; do set -- $cfg
NC=$1 SLOTS=$2 ONLY=full,no_lds_ops,flush_no_hbm timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_q.err | tr '\n' ' ' || exit 4; echo
done
