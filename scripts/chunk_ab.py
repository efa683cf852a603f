"""Same-box A/B of FusedStep knobs on the bench's own step (round 6: the pipelined field pass,
field_chunks / field_split, measured here and removed — profiles/r6/ab_r6jk_*): graph replay of the headline step (FRAMES frames x RPF rays, amp, device-drawn
batches), the variants (dicts of FusedStep attributes, env VARIANTS) alternating over REPS
repetitions, each timing STEPS replays from the same initial state after 5 warm-up replays (which
capture). Prints the median ms/step per variant and the last replay's loss."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    reps, steps = int(os.environ.get("REPS", "4")), int(os.environ.get("STEPS", "100"))
    frames, rpf = int(os.environ.get("FRAMES", "64")), int(os.environ.get("RPF", "2048"))
    variants = json.loads(os.environ["VARIANTS"])
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, frames, dict(amp=True), dev)
    enc, net, pa = bench.make_models(cfg, frames, dev)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start)
    P0 = fs.P.detach().clone()
    res = {k: [] for k in variants}
    loss = {}
    for rep in range(reps):
        for name, knobs in variants.items():
            for k, v in knobs.items():
                setattr(fs, k, v)
            fs.reset_state(P0)
            for it in range(5):
                fs.graph_step(rpf, seed_base=rep)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for it in range(steps):
                out = fs.graph_step(rpf, seed_base=rep)
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / steps * 1e3)
            loss[name] = [round(float(x), 6) for x in out["loss_terms"][:4].tolist()]
            for k in knobs:
                delattr(fs, k)
    for name, v in res.items():
        print(json.dumps({"variant": name, "knobs": variants[name], "rays": frames * rpf, "ms_per_step_median":
                          round(float(np.median(v)), 4), "ms_per_step": [round(x, 4) for x in v],
                          "loss_last": loss[name]}), flush=True)


if __name__ == "__main__":
    main()
