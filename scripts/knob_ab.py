"""Same-box A/B of FusedStep knobs (production library, no timing-build ablation bits): the headline
pool (FRAMES frames x 2048 rays, amp), every variant a dict of FusedStep attributes, the variants
interleaved over ROUNDS rounds of 3 eager steps each from the same state; one JSON line per variant
with the median of each field-kernel bucket (HIP events inside the C ABI).
Usage: VARIANTS='{"slots512": {}, "slots256": {"scatter_slots": 256}}' python scripts/knob_ab.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    frames = int(os.environ.get("FRAMES", "64"))
    variants = json.loads(os.environ["VARIANTS"])
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, frames, dict(amp=True), dev)
    enc, net, pa = bench.make_models(cfg, frames, dev)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start,
                   time_kernels=True)
    for it in range(int(os.environ.get("WARM", "40"))):
        fs.step(ids=fs.sample_ids(2048, it))
    torch.cuda.synchronize()
    fs.field_kernel_breakdown()
    P0, M0, V0, E0 = fs.P.clone(), fs.M.clone(), fs.V.clone(), fs.emb16.clone()
    per = {k: [] for k in variants}
    for rnd in range(int(os.environ.get("ROUNDS", "5"))):
        for name, knobs in variants.items():
            fs.P.copy_(P0); fs.M.copy_(M0); fs.V.copy_(V0); fs.emb16.copy_(E0)
            old = {k: fs.__dict__.get(k, KeyError) for k in knobs}
            for k, v in knobs.items():
                setattr(fs, k, v)
            for it in range(3):
                fs.step(ids=fs.sample_ids(2048, 100 + it))
            torch.cuda.synchronize()
            bd, _ = fs.field_kernel_breakdown()
            c = fs.scatter_atomic_counts()   # last step's scatter HBM atomics (table flush, probe overflow)
            bd = dict(bd, flush_atomics=float(c[0]), overflow_atomics=float(c[1]))
            per[name].append(bd)
            for k, v in old.items():
                if v is KeyError:
                    delattr(fs, k)
                else:
                    setattr(fs, k, v)
    for name in variants:
        tot = [sum(v for k, v in b.items() if k.startswith("k_")) for b in per[name]]
        print(json.dumps({"variant": name, "knobs": variants[name], "frames": frames,
                          "field_ms_median": round(float(np.median(tot)), 4), "field_ms_min": round(float(np.min(tot)), 4),
                          "kernels": {k: round(float(np.median([b[k] for b in per[name]])), 4) for k in per[name][0]}}),
              flush=True)


if __name__ == "__main__":
    main()
