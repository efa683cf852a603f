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
# longest names first: k_mlp_bwd_tr must not be taken for k_mlp_bwd
KERNELS = ("k_mlp_bwd_tr", "k_mlp_bwd", "k_encode", "k_colour", "k_ray_final", "k_scatter", "k_adam")


def kernel_key(name):
    """Field-kernel key of a rocprof kernel name (mangled or demangled); the amp MLP backward
    (k_mlp_bwd_tr<lpw, pass, ff>) and the fp32 one are split into their two passes."""
    for k in KERNELS:
        if f"nof{len(k)}{k}I" in name or f"nof{len(k)}{k}E" in name or f"nof::{k}(" in name or f"nof::{k}<" in name:
            if k.startswith("k_mlp_bwd"):
                p1 = ("Li1E" in name.split(k, 1)[1][:12]) if f"{k}I" in name else (", 1" in name.split(k, 1)[1][:8])
                return "k_mlp_bwd_pass1" if p1 else "k_mlp_bwd_pass0"
            return k
    return None


for row in csv.DictReader(open(path)):
    key = kernel_key(row["Kernel_Name"])
    if key is not None:
        durs[key].append((int(row["Start_Timestamp"]), int(row["End_Timestamp"]) - int(row["Start_Timestamp"])))
res = {}
for k, v in sorted(durs.items()):
    v.sort()
    last = [d for _, d in v[-n:]]
    res[k] = {"dispatches": len(v), "steady_mean_ms": round(sum(last) / len(last) / 1e6, 4), "steady_n": len(last),
              "all_mean_ms": round(sum(d for _, d in v) / len(v) / 1e6, 4)}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res))
