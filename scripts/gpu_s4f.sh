# GPU: why is k_mlp_bwdw slow — ablation (no dW) + SQ PMC pass on the fused kernel.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R && mkdir -p gpurun_out
ONLY=full,bwdw_no_dw WARM=30 timeout -k 10 200 python scripts/ablate.py > gpurun_out/ablate_s4f.jsonl 2> gpurun_out/ablate_s4f.err || { tail -20 gpurun_out/ablate_s4f.err; exit 1; }
cat gpurun_out/ablate_s4f.jsonl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU SQ_INSTS_VMEM --kernel-include-regex "k_mlp_bwd" --output-format csv -d $R/gpurun_out/pmc_bwdw -o run -- python $R/bench.py --steps 5 --warmup 20 --no-cpu-baseline > $R/gpurun_out/pmc_bwdw.log 2>&1 || { tail -20 $R/gpurun_out/pmc_bwdw.log; exit 2; }
python - <<'PY'
import csv, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open('/root/repo/gpurun_out/pmc_bwdw/run_counter_collection.csv')):
    v[(r['Kernel_Name'][:40], r['Counter_Name'])].append(float(r['Counter_Value']))
for k, x in sorted(v.items()): print(k, sum(x[-5:]) / len(x[-5:]))
PY
