"""Same-box A/B of the graph replay's deferred optimiser (FusedStep.defer_opt): the variants alternate
over REPS repetitions in one process, each timing STEPS graph replays (after a few warm-up replays,
which also capture) from the same initial parameters. Workloads: NerfRunner.train()'s 2048-ray
DataLoader batches over the 64-frame pool (parity) and the headline throughput step (64 x 2048 rays)."""
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
    reps, steps = int(os.environ.get("REPS", "4")), int(os.environ.get("STEPS", "200"))
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, 64, dict(amp=True), dev)
    enc, net, pa = bench.make_models(cfg, 64, dev)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start)
    P0 = fs.P.detach().clone()
    torch.manual_seed(0)
    dl = DataLoader(pool, 2048)
    work = {"parity": lambda: fs.graph_step_ids(dl.next_ids()), "headline": lambda: fs.graph_step(2048)}
    res = {(w, d): [] for w in work for d in (1, 0)}
    for rep in range(reps):
        for w, fn in work.items():
            for d in (1, 0):
                fs.defer_opt = bool(d)
                fs.reset_state(P0)
                for _ in range(5):
                    fn()
                fs.settle()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    fn()
                fs.settle()
                torch.cuda.synchronize()
                res[(w, d)].append((time.perf_counter() - t0) / steps * 1e3)
    for (w, d), v in res.items():
        print(json.dumps({"workload": w, "defer_opt": d, "ms_per_step_median": round(float(np.median(v)), 4),
                          "ms_per_step": [round(x, 4) for x in v], "steps": steps}), flush=True)


if __name__ == "__main__":
    main()
