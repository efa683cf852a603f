# GPU: gpu tests, smoke, bench, MFMA-busy PMC pass over the MLP kernels.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
TAG=${1:-s4a}
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/tests_$TAG.log 2>&1 || { tail -40 gpurun_out/tests_$TAG.log; exit 1; }
tail -3 gpurun_out/tests_$TAG.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -20 gpurun_out/smoke_$TAG.log; exit 2; }
tail -2 gpurun_out/smoke_$TAG.log
timeout -k 10 300 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 3; }
cat gpurun_out/bench_$TAG.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-include-regex "k_mlp|k_dw" --output-format csv -d $R/gpurun_out/pmc_mfma_$TAG -o run -- python $R/bench.py --steps 10 --warmup 20 --no-cpu-baseline > $R/gpurun_out/pmc_mfma_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_mfma_$TAG.log; exit 4; }
echo pmc done
