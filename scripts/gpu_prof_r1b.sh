set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_b -o run -- python $R/bench.py --no-cpu-baseline > $R/gpurun_out/prof_b.log 2>&1 || { tail -20 $R/gpurun_out/prof_b.log; exit 3; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pmc_fetch_b -o run -- python $R/bench.py --steps 10 --warmup 20 --no-cpu-baseline > $R/gpurun_out/pmc_fetch_b.log 2>&1 || { tail -20 $R/gpurun_out/pmc_fetch_b.log; exit 4; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pmc_write_b -o run -- python $R/bench.py --steps 10 --warmup 20 --no-cpu-baseline > $R/gpurun_out/pmc_write_b.log 2>&1 || { tail -20 $R/gpurun_out/pmc_write_b.log; exit 5; }
cd $R && timeout -k 10 300 python bench.py > gpurun_out/bench_b.json 2> gpurun_out/bench_b.err || { tail -20 gpurun_out/bench_b.err; exit 6; }
cat gpurun_out/bench_b.json
