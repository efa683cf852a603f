"""MFMA utilisation of the MLP kernels from one rocprofv3 PMC pass
(`--pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE` over the bench
command). Per MI355X_MICROARCH.md: SQ_VALU_MFMA_BUSY_CYCLES counts cycles an
MFMA unit is busy, summed over the chip's SIMDs; GRBM_GUI_ACTIVE is the kernel's
GPU-active cycles summed over the 8 XCDs. Utilisation = MFMA-busy cycles /
(1024 SIMDs x GRBM_GUI_ACTIVE / 8). Averages over the last `--last` dispatches.
Writes the JSON that bench.py reports as mlp_mfma.pmc_mfma_busy."""
import argparse
import collections
import csv
import json

# k_colour: the tile-parallel colour forward (the sigma net runs inside k_encode, whose MFMA-busy share
# is reported as well); k_mlp_bwd: both passes of the MLP backward (k_mlp_bwd_tr<lpw, pass, ff> in amp),
# also split into k_mlp_bwd_pass0 / _pass1


def _pass(name, p):
    tail = name.split("k_mlp_bwd", 1)[1][:16]
    return f"Li{p}E" in tail if "ILi" in tail else f", {p}" in tail


KERNELS = {"k_colour": lambda n: "k_colour" in n, "k_encode": lambda n: "k_encode" in n,
           "k_mlp_bwd": lambda n: "k_mlp_bwd" in n,
           "k_mlp_bwd_pass0": lambda n: "k_mlp_bwd" in n and _pass(n, 0),
           "k_mlp_bwd_pass1": lambda n: "k_mlp_bwd" in n and _pass(n, 1),
           "k_query_sdf": lambda n: "k_query_sdf" in n}
N_SIMD = 256 * 4


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("out")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--cmd", default="bench.py --steps 10 --warmup 20 --no-cpu-baseline --no-extras")
    ap.add_argument("--workload", default="headline:64")
    a = ap.parse_args()
    # per (kernel, template instance): a kernel launched as several instances per step
    # (k_mlp_bwd's two passes) is summed over its instances, each averaged over its last dispatches
    vals = collections.defaultdict(lambda: collections.defaultdict(lambda: collections.defaultdict(list)))
    for r in csv.DictReader(open(a.csv)):
        for name, match in KERNELS.items():
            if match(r["Kernel_Name"]) and "pack" not in r["Kernel_Name"]:
                vals[name][r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, inst in vals.items():
        m = collections.defaultdict(float)
        for c in inst.values():
            for n, v in c.items():
                m[n] += sum(v[-a.last:]) / len(v[-a.last:])
        busy, active = m.get("SQ_VALU_MFMA_BUSY_CYCLES"), m.get("GRBM_GUI_ACTIVE")
        e = {n: round(v, 1) for n, v in m.items()}
        if busy is not None and active:
            e["mfma_util"] = round(busy / (N_SIMD * active / 8), 4)
        res[k] = e
    res["_workload"] = a.workload
    res["_method"] = ("rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE over "
                      f"'{a.cmd}'; per template instance the mean of its last {a.last} dispatches, summed over "
                      "the instances one step launches; "
                      "mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE/8)")
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
