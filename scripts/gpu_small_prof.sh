# rocprofv3 kernel stats of NerfRunner.train()-sized steps (scripts/small_batch_prof.py). Usage: bash scripts/gpu_small_prof.sh TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${1:-small}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sprof_$TAG -o run -- python $R/scripts/small_batch_prof.py 501 > $R/gpurun_out/sprof_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/sprof_$TAG.log; exit 3; }
grep "small batch" $R/gpurun_out/sprof_$TAG.log
python - <<PY
import csv
rows = list(csv.DictReader(open("$R/gpurun_out/sprof_$TAG/run_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:24]:
    print(r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 1), "us")
PY
