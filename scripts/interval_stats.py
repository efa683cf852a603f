"""Interval-list statistics of the headline ray batch (diagnostic): the traced intervals per ray
and, per sampler tile (32 octree samples), the interval index the walk reaches."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402

dev = torch.device("cuda:0")
cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, 64, dict(amp=True), dev)
enc, net, pa = bench.make_models(cfg, 64, dev)
fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start)
fs.step(ids=fs.sample_ids(2048, 3))
torch.cuda.synchronize()
cnt = fs.counts.cpu().numpy()
iv = fs.intervals.cpu().numpy()
tot = fs.totals.cpu().numpy()
print("Kmax", fs.Kmax, "rays", cnt.size, "counts mean %.2f median %d p90 %d max %d zero %.3f" % (
    cnt.mean(), np.median(cnt), np.percentile(cnt, 90), cnt.max(), (cnt == 0).mean()))
lens = iv[..., 1] - iv[..., 0]
print("interval length mean %.4f (z units), total mean %.3f" % (lens[iv[..., 0] > 0].mean(), tot.mean()))
