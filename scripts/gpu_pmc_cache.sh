# L2 (TCC) hit / miss and L1 (TCP) request counters of the field kernels on the headline bench
# command (one pass, no trace domains). Usage: bash scripts/gpu_pmc_cache.sh TAG [REGEX]
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
TAG=${1:-cache}
RX=${2:-k_encode|k_mlp|k_scatter}
CMD="--steps 3 --warmup 20 --no-cpu-baseline --no-extras --no-graph"
timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --kernel-include-regex "$RX" --output-format csv -d $R/gpurun_out/pmc_cache_$TAG -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_cache_$TAG.log 2>&1 || { tail -20 $R/gpurun_out/pmc_cache_$TAG.log; exit 3; }
cd $R && python - <<PY
import collections, csv, glob
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob("gpurun_out/pmc_cache_$TAG/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in vals.items():
    m = {n: sum(v[-3:]) / len(v[-3:]) for n, v in c.items()}
    hit = m.get("TCC_HIT_sum", 0); miss = m.get("TCC_MISS_sum", 0)
    print(k, {n: f"{v:.3g}" for n, v in sorted(m.items())}, "L2 hit", round(hit / max(hit + miss, 1), 3))
PY
