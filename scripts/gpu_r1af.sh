set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_af.log 2>&1 || { tail -40 gpurun_out/gpu_step_af.log; exit 1; }
tail -1 gpurun_out/gpu_step_af.log
bash scripts/gpu_pmc_sq.sh
