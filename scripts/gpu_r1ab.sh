set -o pipefail
timeout -k 10 400 python -m pytest tests/test_gpu_step.py -x -q -p no:cacheprovider > gpurun_out/gpu_step_ab.log 2>&1 || { tail -40 gpurun_out/gpu_step_ab.log; exit 1; }
tail -1 gpurun_out/gpu_step_ab.log
for SL in 512 1024; do
SLOTS=$SL ONLY=full,f32_lds,ident_hash,f32_lds_ident,no_lds_ops,flush_no_hbm timeout -k 10 300 python scripts/ablate.py 2> gpurun_out/ablate_ab.err | tr '\n' ' ' || exit 4; echo
done
