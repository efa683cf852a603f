"""Same-box A/B of FusedStep knobs on NerfRunner.train()'s step (2048-ray DataLoader batches over the
64-frame pool, graph replay, amp): the variants (dicts of FusedStep attributes, env VARIANTS) alternate
over REPS repetitions, each timing STEPS replays from the same initial parameters after 5 warm-up
replays (which capture). Prints the median ms/step per variant. The step is NerfRunner.train()'s:
graph_step_epoch on the DataLoader's permutation (no per-step id copy)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402
from bundlesdf_amd.nerf_runner import DataLoader  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    reps, steps = int(os.environ.get("REPS", "4")), int(os.environ.get("STEPS", "300"))
    frames = int(os.environ.get("FRAMES", "64"))
    batch = int(os.environ.get("BATCH", "2048"))
    variants = json.loads(os.environ["VARIANTS"])
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, frames, dict(amp=True), dev)
    enc, net, pa = bench.make_models(cfg, frames, dev)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start)
    P0 = fs.P.detach().clone()
    torch.manual_seed(0)
    dl = DataLoader(pool, batch)
    res = {k: [] for k in variants}
    for rep in range(reps):
        for name, knobs in variants.items():
            knobs = dict(knobs)
            # "_path": "ids" replays graph_step_ids (a per-step copy of the slice) instead
            path = knobs.pop("_path", "epoch")
            for k, v in knobs.items():
                setattr(fs, k, v)
            fs.reset_state(P0)
            if path == "ids":
                step = lambda: fs.graph_step_ids(dl.next_ids())   # noqa: E731
            else:
                step = lambda: fs.graph_step_epoch(*dl.next_slice(), batch)   # noqa: E731
            for _ in range(5):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                step()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / steps * 1e3)
            for k in knobs:
                delattr(fs, k)
    for name, v in res.items():
        print(json.dumps({"variant": name, "knobs": variants[name], "batch": batch, "ms_per_step_median":
                          round(float(np.median(v)), 4), "ms_per_step": [round(x, 4) for x in v]}), flush=True)


if __name__ == "__main__":
    main()
