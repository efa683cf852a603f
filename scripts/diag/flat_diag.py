"""Diagnostic: the run-scan scatter with and without scatter_flat on the frame-feature amp case
(config-5 shape) — table-gradient entries that differ, with their level and row. (Found the
neighbour-exchange level tags breaking runs; the item-index boundary flags replaced them.)"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import test_gpu_step as T  # noqa: E402

dev = torch.device("cuda", 0)
cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, ff = T._ff_case()
cfg["amp"] = True
res = {}
for knobs in (dict(scatter_kernel=2, scatter_levels_per_wave=4, scatter_flat=0, ablate=0),
              dict(scatter_kernel=2, scatter_levels_per_wave=1, scatter_flat=1, ablate=0),
              dict(scatter_kernel=2, scatter_levels_per_wave=4, scatter_flat=1, ablate=0),
              dict(scatter_kernel=2, scatter_levels_per_wave=8, scatter_flat=1, ablate=0),
              dict(scatter_kernel=2, scatter_levels_per_wave=16, scatter_flat=1, ablate=0)):
    fs, fa = T._ff_fused(dev, cfg, seq, batch, occ, mlp_w, emb, pose, ff, amp=True)
    for k, v in knobs.items():
        setattr(fs, k, v)
    fs.scale.fill_(1024.0)
    R = batch.shape[0]
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
    torch.cuda.synchronize()
    g = fs.split(out["grads"].cpu())["embeddings"].numpy().reshape(-1, 2)
    res[tuple(knobs.values())] = (g, fs.scatter_atomic_counts().tolist())
base = res[(2, 4, 0, 0)][0]
offs = np.asarray(offs)
for k, (g, cnt) in res.items():
    d = np.abs(g - base)
    rel = d / (np.abs(base) + 1e-6 * np.abs(base).max())
    bad = np.where((rel > 0.05).any(1))[0]
    print(k, "atomics", cnt, "entries differing > 5 %:", len(bad))
    for row in bad[:12]:
        lv = int(np.searchsorted(offs, row, side="right") - 1)
        print("   row", row, "level", lv, "base", base[row], "got", g[row])
