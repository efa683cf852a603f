set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_r1.json 2> gpurun_out/bench_r1.err || exit $?
cat gpurun_out/bench_r1.json
R=$PWD
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_r1 -o run -- python $R/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $R/gpurun_out/prof_r1.log 2>&1 || exit $?
ls -R $R/gpurun_out/prof_r1 | head -20
