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

KERNELS = {"k_encode": "k_encode", "k_mlp_fwd": "k_mlp_fwd", "k_mlp_bwd": "k_mlp_bwd", "k_compact": "k_compact",
           "k_scatter": "k_scatter", "k_dw": "k_dwI", "k_adam": "k_adam", "k_trace": "k_trace"}


def load(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        n = r["Kernel_Name"]
        for name, key in KERNELS.items():
            if key in n and "pack" not in n:
                d[name].append(float(r["Counter_Value"]))
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("out")
    ap.add_argument("--last", type=int, default=10)
    a = ap.parse_args()
    f, w = load(a.fetch_csv), load(a.write_csv)
    res = {}
    for k in KERNELS:
        if not f.get(k) or not w.get(k):
            continue
        fk = sum(f[k][-a.last:]) / len(f[k][-a.last:])
        wk = sum(w[k][-a.last:]) / len(w[k][-a.last:])
        res[k] = {"fetch_size_KiB": round(fk, 1), "write_size_KiB": round(wk, 1),
                  "traffic_bytes": int((2 * fk + wk) * 1024)}
    res["_method"] = ("rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes) over "
                      f"'bench.py --steps 10 --warmup 20 --no-cpu-baseline'; mean of the last {a.last} dispatches; "
                      "traffic = (2*FETCH_SIZE + WRITE_SIZE) KiB * 1024 (gfx950 FETCH_SIZE correction)")
    json.dump(res, open(a.out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
