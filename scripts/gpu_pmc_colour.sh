set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
CMD="--warmup 20 --no-cpu-baseline --no-extras"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS --kernel-include-regex "k_colour|k_mlp_bwd_tr" --output-format csv -d $R/gpurun_out/pmc_col -o run -- python $R/bench.py $CMD > $R/gpurun_out/pmc_col.log 2>&1 || { tail -20 $R/gpurun_out/pmc_col.log; exit 4; }
cd $R && python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/pmc_col/**/*counter_collection.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    agg[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in agg.items():
    print(k, {c: "%.3g" % (sum(v[-501:]) / len(v[-501:])) for c, v in d.items()})
PY
