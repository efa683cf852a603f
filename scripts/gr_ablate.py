"""Timing ablation on the BASELINE config-5 (global refine) per-GPU shape: 63 frames x 4096 rays,
S = 64 + 256, hashed top levels, frame features 2, amp (diagnostic only: ablated runs compute
wrong results). Prints one JSON line per variant with the median field-kernel breakdown.
Usage: NOF_LIB=.../libnof_ablate.so ONLY=full,... python scripts/gr_ablate.py"""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402

MASKS = {"full": 0, "no_ff_atomics": 512}


def main():
    dev = torch.device("cuda", 0)
    frames, rpf = 63, 4096
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, frames, dict(amp=True, **bench.GLOBAL_REFINE), dev)
    enc, net, pa, fa = bench.make_models(cfg, frames, dev, with_features=True)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start,
                   feature_array=fa, time_kernels=True)
    if os.environ.get("LPW"):   # k_scatter levels per wave (0: the library's choice by batch size)
        fs.scatter_levels_per_wave = int(os.environ["LPW"])
    for it in range(int(os.environ.get("WARM", "20"))):
        fs.step(ids=fs.sample_ids(rpf, it))
    torch.cuda.synchronize()
    fs.field_kernel_breakdown()
    fs.wait_exchange()   # emb16 may be an all-gather target still in flight (N > 1)
    P0, M0, V0, E0 = fs.P.clone(), fs.M.clone(), fs.V.clone(), fs.emb16.clone()
    only = os.environ.get("ONLY")
    masks = {k: v for k, v in MASKS.items() if not only or k in only.split(",")}
    per = {k: [] for k in masks}
    for rnd in range(2):
        for name, m in masks.items():
            fs.wait_exchange()
            fs.P.copy_(P0); fs.M.copy_(M0); fs.V.copy_(V0); fs.emb16.copy_(E0)
            fs.ablate = m
            for it in range(3):
                fs.step(ids=fs.sample_ids(rpf, 100 + it))
            torch.cuda.synchronize()
            bd, _ = fs.field_kernel_breakdown()
            per[name].append(bd)
    for name in masks:
        print(json.dumps({"variant": name, "mask": masks[name], "workload": "global_refine", "lpw": os.environ.get("LPW", "0"), 
                          "lib": os.path.basename(os.environ.get("NOF_LIB", "libnof.so")),
                          "kernels": {k: round(float(np.median([b[k] for b in per[name]])), 4) for k in per[name][0]}}),
              flush=True)


if __name__ == "__main__":
    main()
