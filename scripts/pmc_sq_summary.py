"""Per-kernel (per template instance) means of SQ counters from scripts/gpu_pmc_sq.sh
output, over the last N dispatches. Usage: python scripts/pmc_sq_summary.py TAG [N]"""
import collections
import csv
import glob
import sys

tag = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 3
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"gpurun_out/pmc_sq[12]_{tag}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        vals[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in vals.items():
    m = {n: sum(v[-last:]) / len(v[-last:]) for n, v in c.items()}
    print(k)
    print("   " + " ".join(f"{n}={v:.3g}" for n, v in sorted(m.items())))
