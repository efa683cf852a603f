set -o pipefail
mkdir -p gpurun_out
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/gpu_all_g.log 2>&1 || { tail -40 gpurun_out/gpu_all_g.log; exit 1; }
tail -3 gpurun_out/gpu_all_g.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_g.log 2>&1 || { tail -30 gpurun_out/smoke_g.log; exit 2; }
cat gpurun_out/smoke_g.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/pmc_fetch.log 2>&1 || { tail -20 $R/gpurun_out/pmc_fetch.log; exit 3; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/pmc_write.log 2>&1 || { tail -20 $R/gpurun_out/pmc_write.log; exit 4; }
ls -R $R/gpurun_out/pmc_fetch | head
