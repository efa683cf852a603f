"""Per-launch HBM traffic of the field-step kernels from two rocprofv3 PMC
passes (FETCH_SIZE and WRITE_SIZE in separate runs of the same bench command,
MI355X_MICROARCH.md 'HBM' + 'rocprofv3 PMC slots'): counter values are KiB;
gfx950 FETCH_SIZE is doubled (it tallies 128-B requests at 64 B); WRITE_SIZE
is exact. Averages over the last `--last` dispatches (the timed steps).
Writes a JSON summary that bench.py reports as roofline.traffic."""
import argparse
import csv
import collections
import json

KERNELS = {"k_encode": "k_encode", "k_colour": "k_colour", "k_mlp_bwd": "k_mlp_bwd", "k_compact": "k_compact",
           "k_scatter": "k_scatter", "k_adam": "k_adam", "k_trace": "k_trace"}


def load(path, last):
    """Per kernel: the mean of the last `last` dispatches of each template instance, summed
    over the instances one step launches (k_mlp_bwd's two passes)."""
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        for name, key in KERNELS.items():
            if key in n and "pack" not in n:
                d[name][n].append(float(r["Counter_Value"]))
    return {k: sum(sum(v[-last:]) / len(v[-last:]) for v in inst.values()) for k, inst in d.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("out")
    ap.add_argument("--last", type=int, default=10)
    ap.add_argument("--cmd", default="bench.py --steps 10 --warmup 20 --no-cpu-baseline --no-extras")
    ap.add_argument("--workload", default="headline:64", help="bench workload:frames_per_gpu the passes ran")
    a = ap.parse_args()
    f, w = load(a.fetch_csv, a.last), load(a.write_csv, a.last)
    res = {"_workload": a.workload}
    for k in KERNELS:
        if k not in f or k not in w:
            continue
        fk, wk = f[k], w[k]
        res[k] = {"fetch_size_KiB": round(fk, 1), "write_size_KiB": round(wk, 1),
                  "traffic_bytes": int((2 * fk + wk) * 1024)}
    res["_method"] = ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over "
                      f"'{a.cmd}'; per template instance the mean of its last {a.last} dispatches, summed over "
                      "the instances one step launches; "
                      "traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 (gfx950 FETCH_SIZE correction)")
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
