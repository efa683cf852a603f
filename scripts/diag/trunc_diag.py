"""Diagnostic (GPU): the truncation-schedule case of test_gpu_step (seed 29, linear,
global_step 12): per-sample dL/dfeature vs the oracle, and the table-gradient entry
that disagrees, with the samples / corners that feed it."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import nerf_step as NS  # noqa: E402
from oracle import kernels as K  # noqa: E402
from tests.test_gpu_step import _scene_case, _run_fused, _oracle_ref  # noqa: E402

dev = torch.device("cuda", 0)
cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=29)
cfg.update(trunc_decay_type="linear", trunc_start=0.03, trunc=0.01, n_step=100)
slots = int(sys.argv[1]) if len(sys.argv) > 1 else 0
fs, enc, out = _run_fused(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, dev, global_step=12, slots=slots)
ref = _oracle_ref(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, enc, step=12)
R, S = batch.shape[0], 192
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
dfg = df[:, np.argsort(perm)]
flags = fs.workspace[2 * off + al(n * 4):2 * off + al(n * 4) + R * (S // 32)].cpu().numpy()
dfg[np.repeat(flags, 32) == 0] = 0.0
dfr = ref["d_feat"].numpy()
print("dfeat max |ref|", np.abs(dfr).max(), "max abs diff", np.abs(dfg - dfr).max())
G = fs.split(out["grads"].cpu())
got, want = G["embeddings"].numpy().ravel(), ref["grads"]["embeddings"].numpy().ravel()
A = ref["g_emb_abs"].numpy().ravel()
i = int(np.argmax(np.abs(got - want) / (5e-3 * np.abs(want) + 1e-4 * A + 1e-12)))
row, ch = divmod(i, 2)
lv = int(np.searchsorted(offs, row, side="right") - 1)
print(f"entry {i}: level {lv} row {row - offs[lv]} ch {ch}: got {got[i]:.6e} want {want[i]:.6e} A {A[i]:.3e}")
# the table gradient recomputed from the FUSED per-sample dL/dfeature with the oracle's backward
valid = ref["valid"].numpy().reshape(-1)
x = None
# positions of the valid samples from the oracle
import json  # noqa: E402,F401
P = fs.split(fs.P.detach().cpu())
tfw = ref["tf"].numpy()
zr = ref["z_vals"].numpy()
d = batch[:, 0:3]
pts = d[:, None, :] * zr[:, :, None]
xw = np.einsum("rij,rsj->rsi", tfw[:, :3, :3], pts) + tfw[:, None, :3, 3]
x01 = ((xw.reshape(-1, 3) + 1) / 2).astype(np.float32)[valid]
gl = dfg[valid].reshape(-1, 16, 2).transpose(1, 0, 2).copy().astype(np.float32)
gemb, _ = K.grid_encode_backward(gl, x01, offs, int(offs[-1]), float(np.log2(enc.per_level_scale)), 16)
print("oracle backward of the FUSED dL/dfeature at that entry:", gemb.ravel()[i],
      " (fused kernel:", got[i], ", oracle:", want[i], ")")
diff = np.abs(gemb.ravel() - got)
print("max |oracle-bwd(fused dfeat) - fused table grad| =", diff.max(), "at", diff.argmax(), "; its A", A[diff.argmax()])
print("scatter atomics", fs.scatter_atomic_counts().tolist())

# ---- the samples whose dL/dfeature disagree most
ds = np.abs(dfg - dfr).max(1)
tr = NS.truncation(cfg, 12)
zg = out["dbg"]["z"].cpu().numpy().ravel()
raw_g, raw_r = out["dbg"]["raw"].cpu().numpy().reshape(n, 4), ref["raw"].numpy().reshape(n, 4)
wr = ref["weights"].numpy().ravel()
dd = np.repeat(batch[:, 6], S)
aux_off = 2 * off + al(n * 4) + al(R * (S // 32)) + al(R * (S // 32) * 4) + al(4) + al(R * 8 * 4)
aux = fs.workspace[aux_off:aux_off + R * (S // 32) * 128 * 16].view(torch.float32).view(R * (S // 32), 128, 4).cpu().numpy()
ray_aux_off = 2 * off + al(n * 4) + al(R * (S // 32)) + al(R * (S // 32) * 4) + al(4)
ray_aux = fs.workspace[ray_aux_off:ray_aux_off + R * 8 * 4].view(torch.float32).view(R, 8).cpu().numpy()
print("trunc", tr)
for k in np.argsort(-ds)[:10]:
    r_, s_ = divmod(int(k), S)
    a4 = aux[r_ * (S // 32) + s_ // 32, 64 + s_ % 32]
    print(f"  r{r_} s{s_}: |d dfeat| {ds[k]:.2e} (|ref| {np.abs(dfr[k]).max():.2e}) z-d {zg[k] - dd[k]:+.5f} "
          f"sdf g {raw_g[k, 3]:+.6f} r {raw_r[k, 3]:+.6f} logit diff {np.abs(raw_g[k, :3] - raw_r[k, :3]).max():.1e} "
          f"w_ref {wr[k]:.3e} aux(dsdf {a4[0]:+.3e}, w' {a4[1]:.3e}, sv {a4[2]}) wtot {ray_aux[r_, 3]:.4e} "
          f"drgb {ray_aux[r_, :3]}")
