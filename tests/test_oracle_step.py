"""CPU: pin oracle/nerf_step.py (the CPU restatement of one training step)
against G4 — the reference's own NerfRunner.train_loop executed from
/root/reference on CPU with the oracle kernels substituted for its CUDA
extensions (tests/golden/train_step.npz, make_golden.py:gen_train_step) —
and the smaller G3 fixtures (raw2outputs / get_sdf_loss / NeRFSmall / SH /
sample_rays_uniform)."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import nerf_step as NS


@pytest.fixture(scope="module")
def g4(golden_dir):
    return np.load(os.path.join(golden_dir, "train_step.npz"))


def _params_from(g, prefix):
    P = {"embeddings": torch.from_numpy(g["emb0" if prefix == "w0_" else "emb1"]),
         "pose": torch.from_numpy(g["pose0" if prefix == "w0_" else "pose1"])}
    for k in NS.MLP_KEYS:
        P[k] = torch.from_numpy(g[prefix + k])
    return P


def test_train_step_matches_reference_train_loop(g4):
    cfg = json.loads(str(g4["cfg_json"]))
    P0 = _params_from(g4, "w0_")
    offs = g4["offsets"]
    meta = (offs, float(np.log2(g4["per_level_scale"][0])), cfg["base_res"])
    out = NS.train_step(P0, torch.from_numpy(g4["batch"]), torch.from_numpy(g4["c2w"]), g4["occ"], cfg,
                        torch.from_numpy(g4["t_rand"]), meta, step=0,
                        lr={k: cfg["lrate"] if k != "pose" else cfg["lrate_pose"] for k in P0})
    np.testing.assert_allclose(out["z_vals"].numpy(), g4["z_vals"], rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(out["valid"].numpy(), g4["valid"])
    np.testing.assert_allclose(out["raw"].numpy(), g4["raw"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["weights"].numpy(), g4["weights"], rtol=1e-5, atol=1e-7)
    np.testing.assert_allclose(out["rgb_map"].numpy(), g4["rgb_map"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(out["loss"], float(g4["loss"]), rtol=1e-5)
    G = out["grads"]
    np.testing.assert_allclose(G["embeddings"].numpy(), g4["g_emb"], rtol=1e-3, atol=1e-7)
    for k in NS.MLP_KEYS:
        np.testing.assert_allclose(G[k].numpy(), g4["g_" + k], rtol=1e-3, atol=1e-6, err_msg=k)
    np.testing.assert_allclose(G["pose"].numpy(), g4["g_pose"], rtol=1e-3, atol=1e-6)
    P1 = _params_from(g4, "w1_")
    for k, v in out["params"].items():
        # Adam's first step moves every param with a nonzero grad by ~lr; compare the update
        np.testing.assert_allclose(v.numpy(), P1[k].numpy(), rtol=1e-4, atol=2e-5, err_msg=k)


@pytest.fixture(scope="module")
def g4amp(golden_dir):
    return np.load(os.path.join(golden_dir, "train_step_amp.npz"))


def _amp_step(g, **kw):
    cfg = json.loads(str(g["cfg_json"]))
    assert cfg["amp"] is True and float(g["found_inf"][0]) == 0.0
    P0 = _params_from(g, "w0_")
    meta = (g["offsets"], float(np.log2(g["per_level_scale"][0])), cfg["base_res"])
    return NS.train_step(P0, torch.from_numpy(g["batch"]), torch.from_numpy(g["c2w"]), g["occ"], cfg,
                         torch.from_numpy(g["t_rand"]), meta, step=0, amp=True, loss_scale=float(g["loss_scale"][0]),
                         lr={k: cfg["lrate"] if k != "pose" else cfg["lrate_pose"] for k in P0}, **kw)


@pytest.mark.parametrize("table_accum", ["fp16_serial", "fp32"])
def test_amp_train_step_matches_reference_amp_train_loop(g4amp, table_accum):
    """G4-amp: the reference's own train_loop with cfg amp = True (the config.yml default the headline
    runs) under autocast — run on CPU with torch.autocast("cpu", float16) for its
    torch.cuda.amp.autocast regions (nerf_runner.py:1254,1288), the fp16 table cast of grid.py:50-51,
    and a real GradScaler (:159, :757-760) at scale 1024 (make_golden.py:gen_train_step(amp=True)).

    fp16_serial: the oracle with the reference kernel's rounding (every sample-corner term added into
    the fp16 table gradient one by one, in the serial order the golden ran) reproduces it to one fp16
    ulp: forward bit-exact, MLP / pose gradients, the Adam update.
    fp32 (the oracle mode every GPU amp parity test compares against): the same fp16 terms summed in
    fp32 — the order-free value the reference's unordered __half2 atomics approximate. Only the table
    gradient differs, by the fp16 accumulation error of the reference's own sum: each entry within
    0.02 of the absolute sum A of its terms (serial fp16 summation of n terms errs by up to ~n·2^-11·A)
    plus the scaled-fp16 subnormal floor 2^-14 / scale, normwise within 1 %."""
    g = g4amp
    out = _amp_step(g, fp16_table_accum=table_accum == "fp16_serial")
    np.testing.assert_allclose(out["z_vals"].numpy(), g["z_vals"], rtol=1e-6, atol=1e-6)
    np.testing.assert_array_equal(out["valid"].numpy(), g["valid"])
    np.testing.assert_allclose(out["raw"].numpy(), g["raw"], rtol=1e-6, atol=0)      # fp16 Linear chain: exact
    np.testing.assert_allclose(out["rgb_map"].numpy(), g["rgb_map"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(out["loss"], float(g["loss"]), rtol=1e-6)
    G = out["grads"]
    for k in NS.MLP_KEYS:
        ref = g["g_" + k]
        np.testing.assert_allclose(G[k].numpy(), ref, rtol=1e-3, atol=1e-4 * np.abs(ref).max(), err_msg=k)
    np.testing.assert_allclose(G["pose"].numpy(), g["g_pose"], rtol=1e-4, atol=1e-6 * np.abs(g["g_pose"]).max())
    got, ref = G["embeddings"].numpy().astype(np.float64), g["g_emb"].astype(np.float64)
    sub = 2.0 ** -14 / float(g["loss_scale"][0])
    if table_accum == "fp16_serial":
        assert (np.abs(got - ref) <= 2.0 ** -10 * np.abs(ref) + sub).all()
        P1 = out["params"]
        np.testing.assert_allclose(P1["embeddings"].numpy(), g["emb1"], atol=1e-7)
        np.testing.assert_allclose(P1["pose"].numpy(), g["pose1"], atol=1e-7)
        for k in NS.MLP_KEYS:
            np.testing.assert_allclose(P1[k].numpy(), g["w1_" + k], atol=1e-7, err_msg=k)
    else:
        A = out["g_emb_abs"].numpy().astype(np.float64)
        assert (np.abs(got - ref) <= 0.02 * A + sub).all()
        assert np.linalg.norm(got - ref) <= 1e-2 * np.linalg.norm(ref)


def test_amp_reference_step_differs_from_fp32(g4, g4amp):
    """G4 and G4-amp run the same inputs: the autocast step is a distinct computation (fp16 table
    read, fp16 Linear results), so a test passing on G4-amp is not passing on fp32 numerics."""
    np.testing.assert_array_equal(g4["t_rand"], g4amp["t_rand"])
    r16, r32 = g4amp["raw"], g4["raw"]
    assert (r16.astype(np.float16).astype(np.float32) == r16).all()      # autocast Linear outputs: fp16 values
    assert (r32.astype(np.float16).astype(np.float32) != r32).mean() > 0.5
    assert float(g4["loss"]) != float(g4amp["loss"])


def test_render_and_losses(golden_dir):
    g = np.load(os.path.join(golden_dir, "render_loss.npz"))
    sc, trunc_m, lam, ntr, near, far, fs_sdf, ew = g["cfg"]
    z = torch.from_numpy(g["z"])
    depth = torch.from_numpy(g["depth"])
    raw = torch.from_numpy(g["raw"]).requires_grad_(True)
    valid = torch.from_numpy(g["valid"])
    t = float(g["trunc"][0])
    d = depth.view(-1, 1)
    u = (d - z) / t
    w = torch.sigmoid(u * lam) * torch.sigmoid(-u * lam)
    inv = (d > far * sc).reshape(-1)
    m = (z - d <= t * ntr) & (z - d >= -t)
    w = torch.where(inv[:, None], torch.zeros_like(w), w * m)
    w = w / (w.sum(-1, keepdim=True) + 1e-10) * valid
    rgb = (w[..., None] * torch.sigmoid(raw[..., :3])).sum(-2)
    rgb.backward(torch.from_numpy(g["g_rgb"]))
    np.testing.assert_allclose(w.detach().numpy(), g["weights"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(rgb.detach().numpy(), g["rgb_map"], rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(raw.grad.numpy(), g["d_raw"], rtol=1e-5, atol=1e-7)


def test_mlp_matches_reference(golden_dir):
    g = np.load(os.path.join(golden_dir, "mlp.npz"))
    W = {k: torch.from_numpy(g["w_" + k]).requires_grad_(True) for k in NS.MLP_KEYS}
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    out = NS.nerf_small(x, W)
    out.backward(torch.from_numpy(g["gout"]))
    np.testing.assert_allclose(out.detach().numpy(), g["out"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(x.grad.numpy(), g["dx"], rtol=1e-5, atol=1e-6)
    for k in NS.MLP_KEYS:
        np.testing.assert_allclose(W[k].grad.numpy(), g["g_" + k], rtol=1e-4, atol=1e-5)


def test_sh_and_stratified(golden_dir):
    g = np.load(os.path.join(golden_dir, "helpers.npz"))
    np.testing.assert_allclose(NS.sh3(torch.from_numpy(g["dirs"])).numpy(), g["sh3"], rtol=0, atol=0)
    near, far = torch.from_numpy(g["near"]), torch.from_numpy(g["far"])
    for N in (128, 64, 7):
        z = NS.sample_rays_uniform(N, near, far, torch.from_numpy(g[f"t_rand{N}"]))
        np.testing.assert_array_equal(z.numpy(), g[f"z_perturb{N}"])


def test_se3_identity_and_orthonormal():
    x = torch.zeros(3, 6)
    T = NS.se3_exp_map(x)
    np.testing.assert_allclose(T.numpy(), np.broadcast_to(np.eye(4), (3, 4, 4)), atol=1e-7)
    x = torch.randn(5, 6, generator=torch.Generator().manual_seed(0), dtype=torch.float64) * 0.3
    T = NS.se3_exp_map(x)
    R = T[:, :3, :3]
    np.testing.assert_allclose((R @ R.transpose(1, 2)).numpy(), np.broadcast_to(np.eye(3), (5, 3, 3)), atol=1e-12)
    # rotation block is the Rodrigues matrix: about z by a, column 0 = (cos a, sin a, 0)
    a = 0.4
    T = NS.se3_exp_map(torch.tensor([[0.1, 0.2, 0.3, 0, 0, a]], dtype=torch.float64))
    np.testing.assert_allclose(T[0, :3, 0].numpy(), [np.cos(a), np.sin(a), 0], atol=1e-12)
    assert T[0, 3, 3] == 1 and np.all(T[0, :3, 3].numpy() == 0)      # translation lives in the last row


@pytest.mark.parametrize("fixture", ["train_step", "train_step_amp"])
def test_loss_terms_f64_matches_reference_loss(golden_dir, fixture):
    """oracle.nerf_step.loss_terms_f64 (the float64 loss recomputation the headline-size GPU test
    applies to the production step's per-sample records) on G4 / G4-amp's own forward records
    reproduces the loss the reference's train_loop computed."""
    g = np.load(os.path.join(golden_dir, fixture + ".npz"))
    cfg = json.loads(str(g["cfg_json"]))
    f = NS.loss_terms_f64(torch.from_numpy(g["batch"]), torch.from_numpy(g["z_vals"]), torch.from_numpy(g["raw"]),
                          torch.from_numpy(g["valid"]), cfg, NS.truncation(cfg))
    np.testing.assert_allclose(f["rgb_loss"] + f["fs_loss"] + f["sdf_loss"], float(g["loss"]), rtol=2e-6)
    np.testing.assert_allclose(f["rgb"].numpy(), g["rgb_map"], rtol=0, atol=1e-6)
