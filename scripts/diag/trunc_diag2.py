"""Diagnostic (GPU): split dL/dfeature of one sample (r258 s64 of the seed-29
linear-truncation case) into its colour and sdf-loss parts, fused vs oracle."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from tests.test_gpu_step import _scene_case, _run_fused, _oracle_ref  # noqa: E402

dev = torch.device("cuda", 0)
base = _scene_case(seed=29)
S = 192


def dfeat(fs, R):
    n = R * S
    al = lambda b: (b + 255) & ~255  # noqa: E731
    off = al(n * 32 * 4)
    df = fs.workspace[off:off + n * 32 * 4].view(torch.float32).view(n, 32).cpu().numpy()
    perm = np.zeros(32, int)
    for s_ in range(2):
        for h in range(2):
            for q in range(4):
                lv = 8 * s_ + 4 * (q >> 1) + 2 * h + (q & 1)
                for c in range(2):
                    perm[(s_ * 2 + h) * 8 + 2 * q + c] = lv * 2 + c
    return df[:, np.argsort(perm)]


k = 258 * S + 64
for name, over in (("all", {}), ("colour only", dict(trunc_weight=0, fs_weight=0)), ("sdf only", dict(rgb_weight=0))):
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = base
    cfg = dict(cfg)
    cfg.update(trunc_decay_type="linear", trunc_start=0.03, trunc=0.01, n_step=100, **over)
    fs, enc, out = _run_fused(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, dev, global_step=12)
    ref = _oracle_ref(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, enc, step=12)
    g = dfeat(fs, batch.shape[0])[k]
    r = ref["d_feat"].numpy()[k]
    print(f"{name:12s} fused {g[:4]} oracle {r[:4]} maxdiff {np.abs(g - r).max():.3e}")
    if name == "all":
        tile = 258 * 6 + 2
        zz = out["dbg"]["z"].cpu().numpy()[258]
        print("   z of ray 258 samples 60..70:", zz[60:71] - batch[258, 6])
        print("   ref weights 60..70:", ref["weights"].numpy()[258, 60:71])
