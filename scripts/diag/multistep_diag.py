"""Diagnostic (GPU): follow the oracle's deterministic parameter trajectory on
the G4 batch (as tests/test_gpu_optim.py does) and report, at each step, the
worst table-gradient entries of the fused step vs the oracle and the samples
where the two disagree (validity, masks, raw)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import nerf_step as NS  # noqa: E402
from tests.test_gpu_optim import _build, _keys  # noqa: E402

g = np.load(os.path.join(ROOT, "tests/golden/train_step.npz"))
cfg = json.loads(str(g["cfg_json"]))
cfg.update(amp=False, n_step=24)
dev = torch.device("cuda", 0)
fs, batch = _build(dev, g, cfg)
R = batch.shape[0]
S = cfg["N_samples"] + cfg["N_samples_around_depth"]
meta = (g["offsets"], float(np.log2(g["per_level_scale"][0])), cfg["base_res"])
rng = np.random.default_rng(0)
ids = torch.arange(R, dtype=torch.int32, device=dev)
traj = {k: v.clone() for k, v in fs.split(fs.P.detach().cpu().clone()).items()}
ost, o_t = None, 0
lr = {k: cfg["lrate"] for k in traj}
for t in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    t_rand = rng.uniform(size=(R, S)).astype(np.float32)
    flat = torch.cat([traj[k].reshape(-1) for k in _keys(fs)]).to(dev)
    with torch.no_grad():
        fs.P.copy_(flat)
    out = fs.step(ids=ids, t_rand=torch.from_numpy(t_rand), debug=True)
    torch.cuda.synchronize()
    ref = NS.train_step({k: v.clone() for k, v in traj.items()}, batch, torch.from_numpy(g["c2w"]), g["occ"], cfg,
                        torch.from_numpy(t_rand), meta, step=t)
    G = fs.split(out["grads"].cpu())
    print(f"step {t}: loss fused {float(out['loss_terms'][:4].sum()):.7f} oracle {ref['loss']:.7f}")
    for k in ["embeddings", "pose"] + NS.MLP_KEYS:
        got, want = G[k].numpy().ravel(), ref["grads"][k].numpy().ravel()
        scale = np.abs(want) + 1e-3 * np.abs(want).max()
        rel = np.abs(got - want) / scale
        print(f"   {k}: max rel {rel.max():.3e} (entry {rel.argmax()}: got {got[rel.argmax()]:.4e} "
              f"want {want[rel.argmax()]:.4e}, max|ref| {np.abs(want).max():.3e})")
        if k == "embeddings" and rel.max() > 5e-3:
            offs = g["offsets"]
            for i in np.argsort(-rel)[:6]:
                row = i // 2
                lv = int(np.searchsorted(offs, row, side="right") - 1)
                print(f"      entry {i} level {lv} row {row - offs[lv]}: got {got[i]:.6e} want {want[i]:.6e}")
    dz = np.abs(out["dbg"]["z"].cpu().numpy() - ref["z_vals"].numpy())
    vg, vr = out["dbg"]["valid"].cpu().numpy().astype(bool), ref["valid"].numpy()
    raw_g, raw_r = out["dbg"]["raw"].cpu().numpy(), ref["raw"].numpy()
    print(f"   z max diff {dz.max():.3e}, valid flips {(vg != vr).sum()}, raw max diff {np.abs(raw_g - raw_r)[vr].max():.3e}")
    rg, rr = out["dbg"]["rgb"].cpu().numpy(), ref["rgb_map"].numpy()
    print(f"   rgb max diff {np.abs(rg - rr).max():.3e}")
    sdf = raw_r[..., 3]
    for name, thr in (("one", 1.0), ("fs_sdf", cfg["fs_sdf"])):
        flip = vr & ((raw_g[..., 3] < thr) != (sdf < thr))
        print(f"   sdf<{name} flips {flip.sum()}; min |sdf-thr| {np.abs(sdf - thr)[vr].min():.3e}")
    if t == 2:
        # per-sample dL/dfeature: fused workspace (fragment order, scaled by 1) vs the oracle's
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
        L = cfg["num_levels"]
        dfg = np.zeros((n, 2 * L))
        for e in range(32):
            if perm[e] < 2 * L:
                dfg[:, perm[e]] = df[:, e]
        dfr = ref["d_feat"].numpy()
        diff = np.abs(dfg - dfr).max(1)
        flags = fs.workspace[2 * off + al(n * 4):2 * off + al(n * 4) + R * (S // 32)].cpu().numpy()
        sc = np.abs(dfr).max()
        print(f"   dfeat max |ref| {sc:.3e}; samples with |diff| > 1e-3 max: {(diff > 1e-3 * sc).sum()}")
        zr = ref["z_vals"].numpy().ravel()
        d = np.repeat(batch[:, 6].numpy(), S)
        for i in np.argsort(-diff)[:10]:
            r_, s_ = divmod(i, S)
            print(f"      sample r{r_} s{s_}: diff {diff[i]:.3e} |ref| {np.abs(dfr[i]).max():.3e} |got| "
                  f"{np.abs(dfg[i]).max():.3e} z {zr[i]:.5f} depth {d[i]:.5f} sdf {raw_r[r_, s_, 3]:.6f} "
                  f"valid {vr[r_, s_]} type {batch[r_, 9].item()} tileflag {flags[r_ * (S // 32) + s_ // 32]} "
                  f"w {ref['weights'][r_, s_].item():.3e}")
    traj, ost = NS.adam_step(traj, ref["grads"], ost, o_t, lr)
    o_t += 1
