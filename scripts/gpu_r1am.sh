set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/kt_am -o run -- python $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $R/gpurun_out/kt_am.log 2>&1 || { tail -20 $R/gpurun_out/kt_am.log; exit 3; }
find $R/gpurun_out/kt_am -name "*.csv" | head
