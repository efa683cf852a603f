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
for it in range(int(os.environ.get("WARM", "40"))):   # the bench's steady state (ablate.py's warm-up)
    fs.step(ids=fs.sample_ids(2048, it))
torch.cuda.synchronize()
cnt = fs.counts.cpu().numpy()
iv = fs.intervals.cpu().numpy()
tot = fs.totals.cpu().numpy()
print("Kmax", fs.Kmax, "rays", cnt.size, "counts mean %.2f median %d p90 %d max %d zero %.3f" % (
    cnt.mean(), np.median(cnt), np.percentile(cnt, 90), cnt.max(), (cnt == 0).mean()))
lens = iv[..., 1] - iv[..., 0]
print("interval length mean %.4f (z units), total mean %.3f" % (lens[iv[..., 0] > 0].mean(), tot.mean()))

# per ray: the scatter's compacted backward samples (gradient-mask bits of flagged tiles)
offs, nt = fs._ws_offsets()
ws = fs.workspace
flags = ws[offs["tile_bwd"]:offs["tile_bwd"] + nt].cpu().numpy()
gm = ws[offs["gmask"]:offs["gmask"] + 4 * nt].view(torch.int32).cpu().numpy().view(np.uint32)
cnt = ws[offs["n_tiles"]:offs["n_tiles"] + 12].view(torch.int32).tolist()
bits = np.unpackbits(gm.view(np.uint8)).reshape(-1, 32).sum(1)
bits = np.where((flags == 1) | (flags == 2), bits, 0)
nact = bits.reshape(fs._R, -1).sum(1)
hit = nact[nact > 0]
print("tile counts: colour-bwd %d colour %d sigma-only %d" % (cnt[0], cnt[1], cnt[2]))
print("rays with backward samples %d, n_act mean %.1f" % (hit.size, hit.mean()))
edges = [0, 16, 32, 48, 64, 80, 96, 128, 160, 192, 320]
h, _ = np.histogram(hit, bins=edges)
print("n_act histogram", {f"{edges[i]+1}-{edges[i+1]}": int(h[i]) for i in range(len(h))})
for w in (64, 32):
    it = np.ceil(hit / w) * (64 // w) / 2 if w == 32 else np.ceil(hit / 64)
    print("iterations per level pair-equivalent, chunk %d: %.3f" % (w, it.mean()))
