"""Lane utilisation of k_scatter's (level, chunk) iterations on the bench workload
(timing build libnof_ablate.so, ablate bit 1<<25 turns the HBM-atomic counters into
active-lane / busy-iteration-lane counts; the step's results are not used)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402

dev = torch.device("cuda", 0)
frames = int(os.environ.get("FRAMES", "64"))
cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, frames, dict(amp=True), dev)
enc, net, pa = bench.make_models(cfg, frames, dev)
fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start)
fs.count_atomics = True   # scatter_atomic_counts below
for it in range(40):
    fs.step(ids=fs.sample_ids(2048, it))
fs.ablate = 1 << 25
fs.step(ids=fs.sample_ids(2048, 41))
torch.cuda.synchronize()
act, busy = fs.scatter_atomic_counts().tolist()
R = frames * 2048
print({"frames": frames, "active_lane_iters": act, "busy_lane_iters": busy, "utilisation": act / max(busy, 1),
       "active_per_ray_level": act / R / cfg.get("num_levels", 16), "n_bwd": float(fs.loss_acc[5])})
