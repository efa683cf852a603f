"""Steady-state per-kernel means from a rocprofv3 kernel trace of bench.py: the rocprof
stats summary averages over every dispatch, including the warm-up steps (the first steps of a
round run slower); this takes the mean of each field kernel's LAST n dispatches (the
timed steps), which is what the bench's HIP-event breakdown measures.
Usage: python scripts/steady_kernel_stats.py run_kernel_trace.csv N out.json"""
import csv
import json
import sys
from collections import defaultdict

path, n, out = sys.argv[1], int(sys.argv[2]), sys.argv[3]
durs = defaultdict(list)
for row in csv.DictReader(open(path)):
    name = row["Kernel_Name"]
    for k in ("k_encode", "k_mlp_fwd", "k_mlp_bwd", "k_scatter", "k_adam"):
        if f"nof{len(k)}{k}" in name or f"nof::{k}(" in name:
            key = k
            if k == "k_mlp_bwd":
                key += "_pass1" if "Li2ELi1E" in name or "Li1ELi1E" in name else "_pass0"
            durs[key].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
res = {}
for k, v in sorted(durs.items()):
    v.sort()
    last = [d for _, d in v[-n:]]
    res[k] = {"dispatches": len(v), "steady_mean_ms": round(sum(last) / len(last) / 1e6, 4), "steady_n": len(last),
              "all_mean_ms": round(sum(d for _, d in v) / len(v) / 1e6, 4)}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
