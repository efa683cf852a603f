"""Diagnostic (GPU): amp step 0 on the G4 batch — per-sample dL/dfeature of the
fused step (workspace, fp16, scaled) vs the oracle's autocast restatement, and
the worst table-gradient entries with the samples feeding them."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import nerf_step as NS  # noqa: E402
from tests.test_gpu_optim import _build  # noqa: E402

g = np.load(os.path.join(ROOT, "tests/golden/train_step.npz"))
cfg = json.loads(str(g["cfg_json"]))
cfg.update(amp=True, n_step=24)
dev = torch.device("cuda", 0)
fs, batch = _build(dev, g, cfg)
R = batch.shape[0]
S = cfg["N_samples"] + cfg["N_samples_around_depth"]
meta = (g["offsets"], float(np.log2(g["per_level_scale"][0])), cfg["base_res"])
rng = np.random.default_rng(0)
t_rand = rng.uniform(size=(R, S)).astype(np.float32)
P0 = {k: v.clone() for k, v in fs.split(fs.P.detach().cpu().clone()).items()}
scale = float(fs.scale.item())
out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
torch.cuda.synchronize()
ref = NS.train_step(P0, batch, torch.from_numpy(g["c2w"]), g["occ"], cfg, torch.from_numpy(t_rand), meta, amp=True,
                    loss_scale=scale)
print("loss", float(out["loss_terms"][:4].sum()), ref["loss"])
raw_g, raw_r = out["dbg"]["raw"].cpu().numpy(), ref["raw"].numpy()
vr = ref["valid"].numpy()
print("raw max diff", np.abs(raw_g - raw_r)[vr].max(), "rgb", np.abs(out["dbg"]["rgb"].cpu().numpy() - ref["rgb_map"].numpy()).max())
n = R * S
al = lambda b: (b + 255) & ~255  # noqa: E731
off = al(n * 32 * 2)
df = fs.workspace[off:off + n * 32 * 2].view(torch.float16).view(n, 32).float().cpu().numpy() / scale
perm = np.zeros(32, int)
for s_ in range(2):
    for h in range(2):
        for q in range(4):
            lv = 8 * s_ + 4 * (q >> 1) + 2 * h + (q & 1)
            for c in range(2):
                perm[(s_ * 2 + h) * 8 + 2 * q + c] = lv * 2 + c
L = cfg["num_levels"]
dfg = np.zeros((n, 2 * L))
for e in range(32):
    if perm[e] < 2 * L:
        dfg[:, perm[e]] = df[:, e]
flags = fs.workspace[2 * off + al(n * 4):2 * off + al(n * 4) + R * (S // 32)].cpu().numpy()
sflag = np.repeat(flags, 32)
dfg[sflag == 0] = 0.0
dfr = ref["d_feat"].numpy()
d = np.abs(dfg - dfr)
rel = d.max(1) / (np.abs(dfr).max(1) + 1e-3 * np.abs(dfr).max())
print("dfeat max |ref|", np.abs(dfr).max(), "max abs diff", d.max(), "worst rel", rel.max())
for i in np.argsort(-rel)[:8]:
    r_, s_ = divmod(i, S)
    print(f"  r{r_} s{s_} tileflag {flags[r_ * (S // 32) + s_ // 32]} valid {vr[r_, s_]} ref {dfr[i, :4]} got {dfg[i, :4]}")
G = fs.split(out["grads"].cpu())
got, want = G["embeddings"].numpy().ravel(), ref["grads"]["embeddings"].numpy().ravel()
A = ref["g_emb_abs"].numpy().ravel()
r2 = np.abs(got - want) / (5e-2 * np.abs(want) + 2e-2 * A + 1e-12)
print("table worst", r2.max(), "entry", r2.argmax(), got[r2.argmax()], want[r2.argmax()], A[r2.argmax()])
