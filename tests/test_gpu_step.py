"""GPU parity of the fused training step (bundlesdf_amd.fused.FusedStep over
nof_trace_rays / nof_field_step / nof_adam_step) against
  * G4 — the reference's own NerfRunner.train_loop executed on CPU
    (tests/golden/train_step.npz), and
  * the CPU oracle step (oracle/nerf_step.py) on a BASELINE-config-2-shaped
    case (L=16, 2^22 table, 192 samples/ray).

Tolerances (fp32 mode, amp off): z_vals / valid bit-exact or 1 ulp-level
(atol 2e-6: sigmoid/exp and the per-voxel slab test use device libm);
raw rtol 1e-4; rgb_map / losses rtol 1e-4; every parameter-gradient entry
within GRAD_TOL of |ref| + 1e-3 max|ref| (a max over entries, so a bug in one
level's rows or in the scatter's overflow path fails) — the MLP runs as f32
MFMA chains and the table gradient is summed with device atomics, so only the
summation order differs from the oracle. A gradient entry is a sum of
many terms of both signs, so its summation-order error scales with the sum of
their absolute values A, and the sample positions (z from the DDA intervals,
x = tf p) agree with the oracle to ~1e-6, which moves an entry by up to its
position sensitivity D times that (the oracle returns both: g_emb_abs,
g_emb_dpos; for the MLP weights A = |dL/dy|^T |x|, g_mlp_abs): each entry
within GRAD_TOL |ref| + KAPPA32 A (+ DPOS D for the table; KAPPA_AMP A in amp
mode, where both the reference and the kernels round through fp16). Adam-updated parameters atol 2e-5
(lr = 0.01 steps). amp mode (fp16 table mirror + f16 MFMA, GradScaler) against
the oracle's autocast restatement (amp=True: fp16 table reads / accumulation,
fp16 Linear operands and results, scaled fp16 gradients): losses rtol
AMP_LOSS_TOL, every gradient entry within AMP_GRAD_TOL of |ref| + 1e-2 max|ref|
(the reference accumulates the fp16 table gradient per sample and corner; the
kernels sum DPP runs of consecutive samples in fp32 and add each run to the
ray's LDS row table in fp16).

Each check also records its worst entry in gpurun_out/parity_metrics.json."""
import json
import os

import numpy as np
import pytest
import torch

from oracle import nerf_step as NS

pytestmark = pytest.mark.gpu


def _build(dev, cfg, emb, mlp_w, pose, n_levels, log2T, finest, base_res=16):
    from bundlesdf_amd.grid import GridEncoder
    from bundlesdf_amd.nerf_helpers import NeRFSmall, PoseArray
    enc = GridEncoder(3, n_levels, 2, base_res, log2T, finest).to(dev)
    enc.embeddings.data.copy_(torch.as_tensor(emb))
    net = NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3, hidden_dim_color=64,
                    input_ch=n_levels * 2, input_ch_views=9).to(dev)
    net.load_state_dict({k: torch.as_tensor(v) for k, v in mlp_w.items()})
    pa = PoseArray(pose.shape[0], cfg["max_trans"] * cfg["sc_factor"], cfg["max_rot"]).to(dev)
    pa.data.data.copy_(torch.as_tensor(pose))
    return enc, net, pa


GRAD_TOL = 5e-3
AMP_LOSS_TOL = 5e-3
AMP_GRAD_TOL = 1.25e-2
KAPPA32 = 1e-4
KAPPA_AMP = 2.5e-2  # amp: fp16 rounding points differ between autocast and the MFMA chains. Round 6: 4x
                    # tighter than round 5's 5e-2 / 0.1, whose worst entry used 0.083 of its allowance
                    # (colour-net weight, frame-feature case; the table 0.036; gpurun_out/parity_metrics.json)
DPOS = 4e-6          # sample-position agreement with the oracle, in x01 units
EXEMPT = 16          # entries allowed past the tight bound (ReLU-kink / loss-mask neighbours, see _check_grad)
EXEMPT_TABLE = 512   # one sample reaches 16 levels x 8 corners x 2 channels = 256 table entries
_METRICS = {}


def _max_rel(got, ref, eps=1e-3):
    """max over entries of |got - ref| / (|ref| + eps max|ref|)."""
    got, ref = np.asarray(got, np.float64).ravel(), np.asarray(ref, np.float64).ravel()
    scale = np.abs(ref) + eps * (np.abs(ref).max() + 1e-30)
    return float((np.abs(got - ref) / scale).max())


def _check_grad(name, got, ref, tol=GRAD_TOL, eps=1e-3, absum=None, kappa=KAPPA32, dpos=None, floor=1e-5,
                exempt=EXEMPT, kink=None):
    """Every entry: |got - ref| <= tol (|ref| + eps max|ref|), or with its conditioning
    A (absolute sum of the accumulated terms) and, for the table, D (position
    sensitivity): <= tol |ref| + kappa A + DPOS D + floor tol max|ref|; plus, when given, K
    (kink): the terms of samples whose ReLU pre-activation lies within rounding distance of 0
    (oracle _mlp_kink: another implementation may take the other side of the kink there and add
    or drop such a term whole)."""
    got, ref = np.asarray(got, np.float64).ravel(), np.asarray(ref, np.float64).ravel()
    m = np.abs(ref).max() + 1e-30
    if absum is None:
        allowed = tol * (np.abs(ref) + eps * m)
    else:
        allowed = tol * np.abs(ref) + kappa * np.asarray(absum, np.float64).ravel() + floor * tol * m
        if dpos is not None:
            allowed = allowed + DPOS * np.asarray(dpos, np.float64).ravel()
    if kink is not None:
        allowed = allowed + np.asarray(kink, np.float64).ravel()
    err = np.abs(got - ref)
    r = err / allowed
    # A handful of entries may sit next to a sample that takes the other side of a ReLU kink
    # (pre-activation within fp32 rounding of 0: MFMA vs CPU summation order) or of a loss
    # mask: that sample's whole contribution moves. Up to EXEMPT such entries may exceed the
    # tight allowance, but every entry stays within 10 % of |ref| + its conditioning.
    coarse = 0.1 * (np.abs(ref) + (np.asarray(absum, np.float64).ravel() if absum is not None else eps * m)) + \
        allowed
    over = int((r > 1.0).sum())
    _METRICS[name] = float(np.sort(r)[-exempt - 1]) if r.size > exempt else 0.0
    _METRICS[name + "/over"] = over
    i = int(r.argmax())
    assert (err <= coarse).all(), f"{name}: entry {i} got {got[i]:.6e} want {ref[i]:.6e} beyond the coarse bound"
    assert over <= exempt, (f"{name}: {over} entries beyond their allowance (worst: entry {i} got {got[i]:.6e} "
                            f"want {ref[i]:.6e}, {r[i]:.2f}x its allowance {allowed[i]:.3e})")


def mask_flips(dbg, ref, batch, cfg, trunc):
    """Samples on which the fused step and the oracle take a different branch of a
    discontinuous loss mask (train_loop / get_sdf_loss / raw2outputs: validity, front /
    back / sdf band |z - d| <= t, sdf < fs_sdf, sdf < 1) because their z or sdf differ by
    rounding right at the threshold. A flip moves that sample's gradient by a finite
    amount, so entry-wise parity holds only on inputs without one."""
    zg, zr = dbg["z"].cpu().numpy(), ref["z_vals"].numpy()
    sg, sr = dbg["raw"].cpu().numpy()[..., 3], ref["raw"].numpy()[..., 3]
    vg, vr = dbg["valid"].cpu().numpy().astype(bool), ref["valid"].numpy()
    d = np.asarray(batch)[:, 6:7]
    sc = cfg["sc_factor"]

    def masks(z, sdf):
        return [z < d - trunc, z > d + trunc * cfg["neg_trunc_ratio"], sdf < cfg["fs_sdf"], sdf < 1.0,
                (z - d <= trunc * cfg["neg_trunc_ratio"]) & (z - d >= -trunc), (d >= cfg["near"] * sc) & (d <= cfg["far"] * sc)]
    flip = vg != vr
    for a_, b_ in zip(masks(zg, sg), masks(zr, sr)):
        flip |= vr & (a_ != b_)
    return int(flip.sum())


FLIP_MAX = 8   # samples allowed on the other side of a loss-mask threshold (of R x S >= 70 K)


def aligned_ref(prefix, dbg, ref_fn, batch, cfg, trunc):
    """The oracle step on the fused step's own inputs, with its discontinuous masks aligned
    to the branches the kernels took: run the oracle, count the samples whose mask decision
    differs (mask_flips: fp16 / fp32 rounding right at a threshold), bound that count, and —
    when there are any — re-run the oracle with mask_from = the kernels' (z, sdf), so those
    samples are evaluated on the kernels' branch and every gradient entry stays comparable.
    Validity (|x| <= 1) flips cannot be aligned and must not occur."""
    ref = ref_fn()
    np.testing.assert_array_equal(dbg["valid"].cpu().numpy().astype(bool), ref["valid"].numpy(),
                                  err_msg=f"{prefix}: validity")
    n = mask_flips(dbg, ref, batch, cfg, trunc)
    _METRICS[f"{prefix}/mask_flips"] = n
    assert n <= FLIP_MAX, f"{prefix}: {n} samples on the other side of a loss-mask threshold"
    if n:
        ref = ref_fn(mask_from=(dbg["z"].cpu(), dbg["raw"][..., 3].cpu()))
    return ref


def _check_all(prefix, G, ref, keys=None, amp=False):
    tol = AMP_GRAD_TOL if amp else GRAD_TOL
    eps = 1e-2 if amp else 1e-3
    for k in keys or (["embeddings", "pose"] + NS.MLP_KEYS):
        emb = k == "embeddings"
        absum = ref.get("g_emb_abs") if emb else (ref.get("g_mlp_abs") or {}).get(k)
        kink = ref.get("g_emb_kink") if emb else (ref.get("g_mlp_kink") or {}).get(k)
        _check_grad(f"{prefix}/{k}", G[k].numpy(), ref["grads"][k].numpy(), tol=tol, eps=eps,
                    absum=absum, dpos=ref.get("g_emb_dpos") if emb else None,
                    kappa=KAPPA_AMP if amp else KAPPA32, floor=eps if amp else 1e-5,
                    exempt=EXEMPT_TABLE if emb else EXEMPT, kink=None if kink is None else kink.numpy())


@pytest.fixture(scope="module", autouse=True)
def _write_metrics():
    yield
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(root, exist_ok=True)
    with open(os.path.join(root, "parity_metrics.json"), "w") as f:
        json.dump({k: float(v) for k, v in _METRICS.items()}, f, indent=1, sort_keys=True)


# k_scatter shapes (nof_field_desc.scatter_levels_per_wave): one wave per ray over all 16 levels
# (config 5's 258 K rays) and 4 levels per wave (16-32 K rays); the headline's 8 levels per wave run in
# HEADLINE_SCATTER below, NerfRunner.train's 2 in test_gpu_runner / test_gpu_graph
SHAPES = {"per_ray": dict(scatter_levels_per_wave=16),
          "split": dict(scatter_levels_per_wave=4)}
# the amp tests add the 2-level-group shape (NerfRunner.train's small batches)
AMP_SHAPES = dict(SHAPES, split2=dict(scatter_levels_per_wave=2))


def _shape(fs, shape):
    for k, v in AMP_SHAPES[shape].items():
        setattr(fs, k, v)


@pytest.mark.parametrize("shape", list(SHAPES))
def test_fused_step_matches_reference_train_loop(golden_dir, cuda_device, shape):
    from bundlesdf_amd.fused import FusedStep
    g = np.load(os.path.join(golden_dir, "train_step.npz"))
    cfg = json.loads(str(g["cfg_json"]))
    dev = cuda_device
    mlp_w = {k: g["w0_" + k] for k in NS.MLP_KEYS}
    enc, net, pa = _build(dev, cfg, g["emb0"], mlp_w, g["pose0"], cfg["num_levels"], cfg["log2_hashmap_size"],
                          cfg["finest_res"])
    pool = torch.from_numpy(g["batch"]).to(dev)
    R = pool.shape[0]
    fs = FusedStep(cfg, pool, torch.from_numpy(g["c2w"]), torch.from_numpy(g["occ"]), enc, net, pa, amp=False)
    _shape(fs, shape)
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(g["t_rand"]),
                  debug=True)
    torch.cuda.synchronize()
    dbg = out["dbg"]
    np.testing.assert_allclose(dbg["z"].cpu().numpy(), g["z_vals"], rtol=1e-6, atol=2e-6)
    np.testing.assert_array_equal(dbg["valid"].cpu().numpy().astype(bool), g["valid"])
    np.testing.assert_allclose(dbg["raw"].cpu().numpy(), g["raw"], rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(dbg["rgb"].cpu().numpy(), g["rgb_map"], rtol=1e-4, atol=1e-5)
    lt = out["loss_terms"].cpu().numpy()[:4]
    np.testing.assert_allclose(lt.sum(), float(g["loss"]), rtol=1e-4)
    G = fs.split(out["grads"].cpu())
    # conditioning of the table-gradient entries from the oracle (pinned to G4) on the same inputs
    P0 = {"embeddings": torch.from_numpy(g["emb0"]), "pose": torch.from_numpy(g["pose0"])}
    P0.update({k: torch.from_numpy(g["w0_" + k]) for k in NS.MLP_KEYS})
    meta = (g["offsets"], float(np.log2(g["per_level_scale"][0])), cfg["base_res"])
    o = NS.train_step(P0, torch.from_numpy(g["batch"]), torch.from_numpy(g["c2w"]), g["occ"], cfg,
                      torch.from_numpy(g["t_rand"]), meta)
    ref = {"grads": {"embeddings": torch.from_numpy(g["g_emb"]), "pose": torch.from_numpy(g["g_pose"])},
           "g_emb_abs": o["g_emb_abs"], "g_emb_dpos": o["g_emb_dpos"], "g_mlp_abs": o["g_mlp_abs"],
           "g_mlp_kink": o["g_mlp_kink"], "g_emb_kink": o["g_emb_kink"]}
    ref["grads"].update({k: torch.from_numpy(g["g_" + k]) for k in NS.MLP_KEYS})
    _check_all("g4", G, ref)
    P = fs.split(fs.P.detach().cpu())
    np.testing.assert_allclose(P["embeddings"].numpy(), g["emb1"], atol=2e-5)
    for k in NS.MLP_KEYS:
        np.testing.assert_allclose(P[k].numpy(), g["w1_" + k], atol=2e-5, err_msg=k)
    np.testing.assert_allclose(P["pose"].numpy(), g["pose1"], atol=2e-5)


G4AMP_TABLE_KAPPA = 2e-2   # the reference's own serial fp16 table sum vs the order-free one (test_oracle_step)
AMP_SHAPES_G4 = {"split": dict(scatter_levels_per_wave=4), "split2": dict(scatter_levels_per_wave=2)}


@pytest.mark.parametrize("shape", list(AMP_SHAPES_G4))
def test_fused_step_amp_matches_reference_amp_train_loop(golden_dir, cuda_device, shape):
    """G4-amp (tests/golden/train_step_amp.npz): the reference's own NerfRunner.train_loop with
    cfg amp = True — its autocast regions (nerf_runner.py:1254,1288) run as CPU fp16 autocast,
    the fp16 table cast of grid.py:50-51, a real GradScaler at scale 1024 — against
    FusedStep(amp=True) on the same inputs: z / validity, the fp16 raw outputs, rgb, the loss,
    and every gradient entry (table, MLP, pose) within the amp allowances. The golden's table
    gradient is the reference kernel's fp16 sum (serial order), which itself differs from the
    order-free value by up to G4AMP_TABLE_KAPPA of each entry's absolute term sum A
    (test_oracle_step pins that): the table allowance adds it to KAPPA_AMP."""
    from bundlesdf_amd.fused import FusedStep
    g = np.load(os.path.join(golden_dir, "train_step_amp.npz"))
    cfg = json.loads(str(g["cfg_json"]))
    assert cfg["amp"] is True and float(g["found_inf"][0]) == 0.0
    dev = cuda_device
    mlp_w = {k: g["w0_" + k] for k in NS.MLP_KEYS}
    enc, net, pa = _build(dev, cfg, g["emb0"], mlp_w, g["pose0"], cfg["num_levels"], cfg["log2_hashmap_size"],
                          cfg["finest_res"])
    R = g["batch"].shape[0]
    fs = FusedStep(cfg, torch.from_numpy(g["batch"]).to(dev), torch.from_numpy(g["c2w"]), torch.from_numpy(g["occ"]),
                   enc, net, pa, amp=True)
    for k, v in AMP_SHAPES_G4[shape].items():
        setattr(fs, k, v)
    fs.scale.fill_(float(g["loss_scale"][0]))
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(g["t_rand"]), debug=True)
    torch.cuda.synchronize()
    dbg = out["dbg"]
    prefix = f"g4amp_{shape}"
    np.testing.assert_allclose(dbg["z"].cpu().numpy(), g["z_vals"], rtol=1e-6, atol=2e-6)
    np.testing.assert_array_equal(dbg["valid"].cpu().numpy().astype(bool), g["valid"])
    raw = dbg["raw"].cpu().numpy()
    # the reference's raw are fp16 Linear outputs; the MFMA chains accumulate in another order
    ulp = np.spacing(np.abs(g["raw"]).astype(np.float16)).astype(np.float32)
    _METRICS[f"{prefix}/raw_fp16_ulps"] = float((np.abs(raw - g["raw"]) / ulp).max())
    np.testing.assert_allclose(raw, g["raw"], rtol=1e-2, atol=2e-3)
    np.testing.assert_allclose(dbg["rgb"].cpu().numpy(), g["rgb_map"], rtol=2e-3, atol=1e-4)
    ref_fwd = {"z_vals": torch.from_numpy(g["z_vals"]), "raw": torch.from_numpy(g["raw"]),
               "valid": torch.from_numpy(g["valid"])}
    flips = mask_flips(dbg, ref_fwd, g["batch"], cfg, NS.truncation(cfg))
    _METRICS[f"{prefix}/mask_flips"] = flips
    assert flips == 0, f"{flips} samples on the other side of a loss-mask threshold than the reference"
    lt = out["loss_terms"].cpu().numpy()[:4]
    _METRICS[f"{prefix}/loss"] = abs(float(lt.sum()) - float(g["loss"])) / float(g["loss"])
    np.testing.assert_allclose(lt.sum(), float(g["loss"]), rtol=AMP_LOSS_TOL)
    G = fs.split(out["grads"].cpu())
    # conditioning (absolute term sums) from the oracle's amp step on the same inputs (pinned to G4-amp)
    P0 = {"embeddings": torch.from_numpy(g["emb0"]), "pose": torch.from_numpy(g["pose0"])}
    P0.update({k: torch.from_numpy(g["w0_" + k]) for k in NS.MLP_KEYS})
    meta = (g["offsets"], float(np.log2(g["per_level_scale"][0])), cfg["base_res"])
    o = NS.train_step(P0, torch.from_numpy(g["batch"]), torch.from_numpy(g["c2w"]), g["occ"], cfg,
                      torch.from_numpy(g["t_rand"]), meta, amp=True, loss_scale=float(g["loss_scale"][0]))
    ref = {"grads": {"embeddings": torch.from_numpy(g["g_emb"]), "pose": torch.from_numpy(g["g_pose"])},
           "g_emb_abs": o["g_emb_abs"] * (1.0 + G4AMP_TABLE_KAPPA / KAPPA_AMP), "g_emb_dpos": o["g_emb_dpos"],
           "g_mlp_abs": o["g_mlp_abs"], "g_mlp_kink": o["g_mlp_kink"], "g_emb_kink": o["g_emb_kink"]}
    ref["grads"].update({k: torch.from_numpy(g["g_" + k]) for k in NS.MLP_KEYS})
    _check_all(prefix, G, ref, amp=True)


def _scene_case(n_frames=4, R=384, seed=0, L=16, log2T=22, finest=128):
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.octree import build_occupancy, coarsen
    seq = SY.make_sequence(n_frames, seed=seed)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"], num_levels=L,
                         log2_hashmap_size=log2T, finest_res=finest, amp=False)
    sc = cfg["sc_factor"]
    pool = SY.build_pool(seq, cfg)
    max_level = int(np.ceil(np.log2(2.0 / (cfg["octree_smallest_voxel_size"] * sc))))
    level = int(np.floor(np.log2(2.0 / (cfg["octree_raytracing_voxel_size"] * sc))))
    occ = coarsen(build_occupancy(torch.from_numpy(seq["octree_pts"]).float(), max_level, 1),
                  2 ** (max_level - level)).numpy()
    rng = np.random.default_rng(seed)
    ids = rng.choice(len(pool), R, replace=False)
    batch = pool[ids]
    t_rand = rng.uniform(size=(R, 192)).astype(np.float32)
    torch.manual_seed(seed)
    from bundlesdf_amd.nerf_helpers import NeRFSmall
    net = NeRFSmall(2, 64, 15, 3, 64, input_ch=2 * L, input_ch_views=9)
    mlp_w = {k: v.detach().numpy() for k, v in net.state_dict().items()}
    from bundlesdf_amd.grid import level_layout
    _, offs = level_layout(3, L, 2, 16, log2T, finest)
    emb = np.random.default_rng(seed + 1).uniform(-1e-4, 1e-4, (int(offs[-1]), 2)).astype(np.float32)
    emb[: min(len(emb), 200000)] *= 1000          # make table values matter at init scale
    pose = (np.random.default_rng(seed + 2).standard_normal((n_frames, 6)) * 0.05).astype(np.float32)
    return cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs


@pytest.mark.parametrize("shape", list(SHAPES))
def test_fused_step_matches_oracle_config2(cuda_device, shape):
    from bundlesdf_amd.fused import FusedStep
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case()
    dev = cuda_device
    enc, net, pa = _build(dev, cfg, emb, mlp_w, pose, 16, 22, 128)
    R = batch.shape[0]
    fs = FusedStep(cfg, torch.from_numpy(batch).to(dev), torch.from_numpy(np.asarray(seq["poses"], np.float32)),
                   torch.from_numpy(occ), enc, net, pa, amp=False)
    _shape(fs, shape)
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
    torch.cuda.synchronize()
    P0 = {"embeddings": torch.from_numpy(emb), "pose": torch.from_numpy(pose)}
    P0.update({k: torch.from_numpy(v) for k, v in mlp_w.items()})
    meta = (offs, float(np.log2(enc.per_level_scale)), 16)
    ref = NS.train_step(P0, torch.from_numpy(batch), torch.from_numpy(np.asarray(seq["poses"], np.float32)), occ, cfg,
                        torch.from_numpy(t_rand), meta)
    dbg = out["dbg"]
    np.testing.assert_allclose(dbg["z"].cpu().numpy(), ref["z_vals"].numpy(), rtol=1e-6, atol=2e-6)
    np.testing.assert_array_equal(dbg["valid"].cpu().numpy().astype(bool), ref["valid"].numpy())
    np.testing.assert_allclose(dbg["raw"].cpu().numpy(), ref["raw"].numpy(), rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(dbg["rgb"].cpu().numpy(), ref["rgb_map"].numpy(), rtol=1e-4, atol=1e-5)
    lt = out["loss_terms"].cpu().numpy()[:4]
    np.testing.assert_allclose(lt.sum(), ref["loss"], rtol=1e-4)
    G = fs.split(out["grads"].cpu())
    _check_all("config2", G, ref)


def test_fused_step_amp_close_to_fp32(cuda_device):
    from bundlesdf_amd.fused import FusedStep
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=3)
    dev = cuda_device
    res = {}
    for amp in (False, True):
        enc, net, pa = _build(dev, cfg, emb, mlp_w, pose, 16, 22, 128)
        R = batch.shape[0]
        fs = FusedStep(cfg, torch.from_numpy(batch).to(dev), torch.from_numpy(np.asarray(seq["poses"], np.float32)),
                       torch.from_numpy(occ), enc, net, pa, amp=amp)
        out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
        torch.cuda.synchronize()
        res[amp] = (out["loss_terms"].cpu().numpy()[:4], out["grads"].cpu().numpy(), fs)
    np.testing.assert_allclose(res[True][0], res[False][0], rtol=2e-2, atol=1e-6)
    g32, g16 = res[False][1], res[True][1]
    cos = float(np.dot(g32, g16) / (np.linalg.norm(g32) * np.linalg.norm(g16)))
    assert cos > 0.99, cos


def test_amp_encode_quad_mirror_bit_identical(cuda_device):
    """Large amp batches (R >= 32768) encode from the xy-quad mirror (k_quad_mirror, two 16-B loads
    per level instead of four 8-B pair loads): same corner values, same arithmetic, so the forward
    (z, validity, raw sdf / colour logits, composited rgb) is bit-identical to the pair-load encode."""
    from bundlesdf_amd.fused import FusedStep
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(n_frames=4, R=32768, seed=5)
    cfg = dict(cfg, amp=True)
    dev = cuda_device
    R = batch.shape[0]
    dbg, quads, grads = {}, {}, {}
    for use in (True, False):
        enc, net, pa = _build(dev, cfg, emb, mlp_w, pose, 16, 22, 128)
        fs = FusedStep(cfg, torch.from_numpy(batch).to(dev), torch.from_numpy(np.asarray(seq["poses"], np.float32)),
                       torch.from_numpy(occ), enc, net, pa, amp=True)
        fs.use_quads = use
        fs.quads.zero_()
        out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
        torch.cuda.synchronize()
        dbg[use] = {k: v.cpu().numpy() for k, v in out["dbg"].items()}
        quads[use] = int(torch.count_nonzero(fs.quads).item())
        G = fs.split(out["grads"].cpu())
        grads[use] = {k: v.numpy().astype(np.float64) for k, v in G.items()}
    assert quads[True] > 0 and quads[False] == 0, quads   # the quad path ran, and only where enabled
    for k in ("z", "valid", "raw", "rgb"):
        np.testing.assert_array_equal(dbg[True][k], dbg[False][k], err_msg=k)
    # the backward is unchanged (the scatter re-gathers from the pair table): the gradients differ
    # only by the order of the atomics — fp16 adds for the table (each rounds at 2^-11 relative),
    # fp32 for the rest. A wrong corner in the input-gradient path moved the pose gradient by 0.8.
    for k, g in grads[True].items():
        ref = grads[False][k]
        err = float(np.abs(g - ref).max()) / max(float(np.abs(ref).max()), 1e-30)
        assert err < (2e-2 if k == "embeddings" else 2e-3), (k, err)


def test_fused_training_decreases_loss(cuda_device):
    """Throughput mode (per-frame uniform rays, device RNG): 30 amp steps reduce the loss."""
    from bundlesdf_amd.fused import FusedStep
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(n_frames=4, R=64, seed=5)
    from bundlesdf_amd import synthetic as SY
    cfg["amp"] = True
    pool = SY.build_pool(seq, cfg)
    frame_start = np.searchsorted(pool[:, 8], np.arange(5))
    dev = cuda_device
    enc, net, pa = _build(dev, cfg, np.random.default_rng(0).uniform(-1e-4, 1e-4, emb.shape).astype(np.float32),
                          mlp_w, np.zeros_like(pose), 16, 22, 128)
    fs = FusedStep(cfg, torch.from_numpy(pool).to(dev), torch.from_numpy(np.asarray(seq["poses"], np.float32)),
                   torch.from_numpy(occ), enc, net, pa, amp=True, frame_start=frame_start)
    losses = []
    for it in range(30):
        ids = fs.sample_ids(512, seed=it)
        out = fs.step(ids=ids)
        losses.append(float(out["loss_terms"][:4].sum().item()))
    assert np.isfinite(losses).all()
    assert np.mean(losses[-5:]) < 0.7 * np.mean(losses[:3]), losses


@pytest.mark.parametrize("shape", list(SHAPES))
def test_fused_step_matches_oracle_hashed_levels(cuda_device, shape):
    """Config-5-like grid: finest 512 with a 2^19 table, so the top levels hash
    (fast_hash + modulo, gridencoder.cu:46-83) — the fused encode/scatter take
    the per-corner grid_row path there."""
    from bundlesdf_amd.fused import FusedStep
    from bundlesdf_amd.grid import level_layout
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=7, R=256, log2T=19, finest=512)
    pls, _ = level_layout(3, 16, 2, 16, 19, 512)
    res = [int(np.ceil(16 * pls ** l)) for l in range(16)]
    assert any((r + 1) ** 3 > 2 ** 19 for r in res), "case must contain hashed levels"
    dev = cuda_device
    enc, net, pa = _build(dev, cfg, emb, mlp_w, pose, 16, 19, 512)
    R = batch.shape[0]
    fs = FusedStep(cfg, torch.from_numpy(batch).to(dev), torch.from_numpy(np.asarray(seq["poses"], np.float32)),
                   torch.from_numpy(occ), enc, net, pa, amp=False)
    _shape(fs, shape)
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
    torch.cuda.synchronize()
    P0 = {"embeddings": torch.from_numpy(emb), "pose": torch.from_numpy(pose)}
    P0.update({k: torch.from_numpy(v) for k, v in mlp_w.items()})
    meta = (offs, float(np.log2(enc.per_level_scale)), 16)
    ref = NS.train_step(P0, torch.from_numpy(batch), torch.from_numpy(np.asarray(seq["poses"], np.float32)), occ, cfg,
                        torch.from_numpy(t_rand), meta)
    np.testing.assert_allclose(out["dbg"]["raw"].cpu().numpy(), ref["raw"].numpy(), rtol=1e-4, atol=2e-5)
    np.testing.assert_allclose(out["loss_terms"].cpu().numpy()[:4].sum(), ref["loss"], rtol=1e-4)
    G = fs.split(out["grads"].cpu())
    _check_all("hashed", G, ref)


def _ff_case(seed=11, R=192, n_frames=4, n_ff=2):
    """BASELINE config 5 shape (run_custom.py:122-133): frame_features=2,
    N_samples=64 + N_samples_around_depth=256 (S=320), hashed top levels."""
    cfg, seq, batch, occ, _, _, emb, pose, offs = _scene_case(seed=seed, R=R, n_frames=n_frames, log2T=19,
                                                              finest=512)
    cfg.update(frame_features=n_ff, N_samples=64, N_samples_around_depth=256, feature_reg_weight=0.1)
    rng = np.random.default_rng(seed + 10)
    t_rand = rng.uniform(size=(R, 320)).astype(np.float32)
    torch.manual_seed(seed)
    from bundlesdf_amd.nerf_helpers import NeRFSmall
    net = NeRFSmall(2, 64, 15, 3, 64, input_ch=32, input_ch_views=9 + n_ff)
    mlp_w = {k: v.detach().numpy() for k, v in net.state_dict().items()}
    ff = rng.standard_normal((n_frames, n_ff)).astype(np.float32)   # FeatureArray init N(0, 1)
    return cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, ff


def _ff_fused(dev, cfg, seq, batch, occ, mlp_w, emb, pose, ff, amp):
    from bundlesdf_amd.fused import FusedStep
    from bundlesdf_amd.grid import GridEncoder
    from bundlesdf_amd.nerf_helpers import FeatureArray, NeRFSmall, PoseArray
    enc = GridEncoder(3, 16, 2, 16, 19, 512).to(dev)
    enc.embeddings.data.copy_(torch.as_tensor(emb))
    net = NeRFSmall(2, 64, 15, 3, 64, input_ch=32, input_ch_views=9 + ff.shape[1]).to(dev)
    net.load_state_dict({k: torch.as_tensor(v) for k, v in mlp_w.items()})
    pa = PoseArray(pose.shape[0], cfg["max_trans"] * cfg["sc_factor"], cfg["max_rot"]).to(dev)
    pa.data.data.copy_(torch.as_tensor(pose))
    fa = FeatureArray(ff.shape[0], ff.shape[1]).to(dev)
    fa.data.data.copy_(torch.as_tensor(ff))
    return FusedStep(cfg, torch.from_numpy(batch).to(dev), torch.from_numpy(np.asarray(seq["poses"], np.float32)),
                     torch.from_numpy(occ), enc, net, pa, amp=amp, feature_array=fa), fa


def test_fused_step_frame_features_matches_oracle(cuda_device):
    """frame_features=2 (FeatureArray latent code in the colour-net input,
    nerf_runner.py:221,1268-1277; reg_features :743-746) at S=320: raw, losses,
    every gradient incl. the feature gradient, and the Adam update vs the oracle."""
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, ff = _ff_case()
    dev = cuda_device
    fs, fa = _ff_fused(dev, cfg, seq, batch, occ, mlp_w, emb, pose, ff, amp=False)
    R = batch.shape[0]
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
    torch.cuda.synchronize()
    P0 = {"embeddings": torch.from_numpy(emb), "pose": torch.from_numpy(pose), "features": torch.from_numpy(ff)}
    P0.update({k: torch.from_numpy(v) for k, v in mlp_w.items()})
    from bundlesdf_amd.grid import GridEncoder
    meta = (offs, float(np.log2(GridEncoder(3, 16, 2, 16, 19, 512).per_level_scale)), 16)
    lr = {k: cfg["lrate"] for k in P0}
    lr["pose"] = cfg["lrate_pose"]
    ref = NS.train_step(P0, torch.from_numpy(batch), torch.from_numpy(np.asarray(seq["poses"], np.float32)), occ, cfg,
                        torch.from_numpy(t_rand), meta, lr=lr)
    assert out["dbg"]["z"].shape[1] == 320
    np.testing.assert_allclose(out["dbg"]["z"].cpu().numpy(), ref["z_vals"].numpy(), rtol=1e-6, atol=2e-6)
    np.testing.assert_allclose(out["dbg"]["raw"].cpu().numpy(), ref["raw"].numpy(), rtol=1e-4, atol=2e-5)
    lt = out["loss_terms"].cpu().numpy()
    np.testing.assert_allclose(lt[6], ref["reg_features"], rtol=1e-5)
    np.testing.assert_allclose(lt[:4].sum() + lt[6], ref["loss"], rtol=1e-4)
    G = fs.split(out["grads"].cpu())
    _check_all("features", G, ref, keys=["embeddings", "pose", "features"] + NS.MLP_KEYS)
    # the data term of the feature gradient (through the colour net) on its own, without reg_features
    reg = 2 * cfg["feature_reg_weight"] * ff / ff.size
    g_data, r_data = G["features"].numpy() - reg, ref["grads"]["features"].numpy() - reg
    assert np.abs(r_data).max() > 0.1 * np.abs(reg).max()
    np.testing.assert_allclose(g_data, r_data, rtol=2e-3, atol=2e-3 * np.abs(r_data).max())
    P1 = fs.split(fs.P.detach().cpu())
    for k in ["features", "color_net.0.weight"]:
        np.testing.assert_allclose(P1[k].numpy(), ref["params"][k].numpy(), atol=2e-5, err_msg=k)
    assert fa.data.data_ptr() == fs.P.data_ptr() + 4 * fs.feat_off   # the module parameter is a view


@pytest.mark.parametrize("shape", list(AMP_SHAPES))
def test_fused_step_frame_features_amp_matches_oracle_amp(cuda_device, shape):
    """BASELINE config 5's real numerics (run_custom.py:122-133: amp with the fp16 table,
    frame_features 2, hashed top levels, S = 64 + 256) against the oracle's autocast
    restatement, entry by entry: losses (incl. reg_features) and every gradient — table,
    MLP, pose and the FeatureArray — within the amp allowances of the module docstring,
    at both k_scatter shapes. Samples whose fp16 sdf sits on a loss-mask threshold (1.0 /
    fs_sdf) are counted and bounded, and the oracle takes the kernels' branch there
    (aligned_ref)."""
    from bundlesdf_amd.grid import GridEncoder
    dev = cuda_device
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, ff = _ff_case(seed=13)
    cfg["amp"] = True
    fs, fa = _ff_fused(dev, cfg, seq, batch, occ, mlp_w, emb, pose, ff, amp=True)
    fs.scale.fill_(1024.0)          # the case's fp16 weight gradients overflow at 2^16 (the step would skip)
    _shape(fs, shape)
    R = batch.shape[0]
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
    torch.cuda.synchronize()
    P0 = {"embeddings": torch.from_numpy(emb), "pose": torch.from_numpy(pose), "features": torch.from_numpy(ff)}
    P0.update({k: torch.from_numpy(v) for k, v in mlp_w.items()})
    meta = (offs, float(np.log2(GridEncoder(3, 16, 2, 16, 19, 512).per_level_scale)), 16)
    ref = aligned_ref(f"ff_amp_{shape}", out["dbg"], lambda **kw: NS.train_step(
        P0, torch.from_numpy(batch), torch.from_numpy(np.asarray(seq["poses"], np.float32)), occ, cfg,
        torch.from_numpy(t_rand), meta, amp=True, loss_scale=1024.0, **kw), batch, cfg, NS.truncation(cfg))
    assert all(torch.isfinite(v).all() for v in ref["grads"].values())
    assert out["dbg"]["z"].shape[1] == 320
    lt = out["loss_terms"].cpu().numpy()
    for i, k in enumerate(["rgb_loss", "fs_loss", None, "sdf_loss"]):
        if k is None:
            continue
        got = lt[i] + (lt[2] if k == "fs_loss" else 0.0)
        _METRICS[f"ff_amp_{shape}/{k}"] = abs(got - ref[k]) / abs(ref[k])
        np.testing.assert_allclose(got, ref[k], rtol=AMP_LOSS_TOL, err_msg=k)
    np.testing.assert_allclose(lt[6], ref["reg_features"], rtol=1e-5)
    np.testing.assert_allclose(out["dbg"]["raw"].cpu().numpy(), ref["raw"].numpy(), rtol=1e-2, atol=2e-3)
    G = fs.split(out["grads"].cpu())
    _check_all(f"ff_amp_{shape}", G, ref, keys=["embeddings", "pose", "features"] + NS.MLP_KEYS, amp=True)


def test_fused_step_pose_reg_matches_oracle(cuda_device):
    """pose_reg_weight > 0 (nerf_runner.py:748-751): pose_reg value and the pose gradient vs the oracle."""
    from bundlesdf_amd.fused import FusedStep
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=17, R=128)
    cfg["pose_reg_weight"] = 0.5
    dev = cuda_device
    enc, net, pa = _build(dev, cfg, emb, mlp_w, pose, 16, 22, 128)
    R = batch.shape[0]
    fs = FusedStep(cfg, torch.from_numpy(batch).to(dev), torch.from_numpy(np.asarray(seq["poses"], np.float32)),
                   torch.from_numpy(occ), enc, net, pa, amp=False)
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
    torch.cuda.synchronize()
    P0 = {"embeddings": torch.from_numpy(emb), "pose": torch.from_numpy(pose)}
    P0.update({k: torch.from_numpy(v) for k, v in mlp_w.items()})
    meta = (offs, float(np.log2(enc.per_level_scale)), 16)
    ref = NS.train_step(P0, torch.from_numpy(batch), torch.from_numpy(np.asarray(seq["poses"], np.float32)), occ, cfg,
                        torch.from_numpy(t_rand), meta)
    lt = out["loss_terms"].cpu().numpy()
    np.testing.assert_allclose(lt[7], ref["pose_reg"], rtol=1e-5)
    np.testing.assert_allclose(lt[:4].sum() + lt[7], ref["loss"], rtol=1e-4)
    G = fs.split(out["grads"].cpu())
    _check_grad("pose_reg/pose", G["pose"].numpy(), ref["grads"]["pose"].numpy())


def _oracle_ref(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, enc, **kw):
    P0 = {"embeddings": torch.from_numpy(emb), "pose": torch.from_numpy(pose)}
    P0.update({k: torch.from_numpy(v) for k, v in mlp_w.items()})
    meta = (offs, float(np.log2(enc.per_level_scale)), 16)
    return NS.train_step(P0, torch.from_numpy(batch), torch.from_numpy(np.asarray(seq["poses"], np.float32)), occ, cfg,
                         torch.from_numpy(t_rand), meta, **kw)


def _run_fused(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, dev, amp=False, global_step=0, slots=0, L=16, log2T=22,
               finest=128, scale=None, shape=None, knobs=None, blocks_per_cu=0):
    from bundlesdf_amd.fused import FusedStep
    enc, net, pa = _build(dev, cfg, emb, mlp_w, pose, L, log2T, finest)
    R = batch.shape[0]
    fs = FusedStep(cfg, torch.from_numpy(batch).to(dev), torch.from_numpy(np.asarray(seq["poses"], np.float32)),
                   torch.from_numpy(occ), enc, net, pa, amp=amp, blocks_per_cu=blocks_per_cu)
    for k, v in (knobs or {}).items():
        setattr(fs, k, v)
    if fs.quads is not None:
        fs.quads.zero_()          # a non-zero quad table afterwards proves the quad encode ran
    fs.global_step = global_step
    if slots:
        fs.scatter_slots = slots
    if scale is not None:
        fs.scale.fill_(scale)
    if shape is not None:
        _shape(fs, shape)
    out = fs.step(ids=torch.arange(R, dtype=torch.int32, device=dev), t_rand=torch.from_numpy(t_rand), debug=True)
    torch.cuda.synchronize()
    return fs, enc, out


def test_scatter_probe_overflow_path_matches_oracle(cuda_device):
    """64 LDS slots per wave: k_scatter's probe chains overflow and those rows go to
    HBM atomics directly (lds_probe) — the table gradient must still match the oracle
    entry by entry."""
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=19)
    fs, enc, out = _run_fused(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, cuda_device, slots=64, shape="per_ray")
    n_overflow = float(fs.scatter_atomic_counts()[1].item())
    assert n_overflow > 0, "the case must drive the probe-overflow path"
    ref = _oracle_ref(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, enc)
    G = fs.split(out["grads"].cpu())
    _check_all("overflow", G, ref)
    _METRICS["overflow/n_direct_atomics"] = n_overflow


def _amp_vs_oracle(prefix, dev, shape=None, knobs=None, blocks_per_cu=0, seed=3, R=384):
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=seed, R=R)
    cfg["amp"] = True
    # loss scale 1024: at the GradScaler's initial 2^16 the reference's fp16 weight gradients of this
    # case overflow (the step would be skipped; test_gpu_optim covers that path)
    fs, enc, out = _run_fused(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, dev, amp=True, scale=1024.0,
                              shape=shape, knobs=knobs, blocks_per_cu=blocks_per_cu)
    ref = aligned_ref(prefix, out["dbg"], lambda **kw: _oracle_ref(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs,
                                                                    enc, amp=True, loss_scale=1024.0, **kw),
                      batch, cfg, NS.truncation(cfg))
    assert all(torch.isfinite(v).all() for v in ref["grads"].values())
    lt = out["loss_terms"].cpu().numpy()
    for i, k in enumerate(["rgb_loss", "fs_loss", None, "sdf_loss"]):
        if k is None:
            continue
        got = lt[i] + (lt[2] if k == "fs_loss" else 0.0)
        _METRICS[f"{prefix}/{k}"] = abs(got - ref[k]) / abs(ref[k])
        np.testing.assert_allclose(got, ref[k], rtol=AMP_LOSS_TOL, err_msg=k)
    np.testing.assert_allclose(out["dbg"]["raw"].cpu().numpy(), ref["raw"].numpy(), rtol=1e-2, atol=2e-3)
    G = fs.split(out["grads"].cpu())
    _check_all(prefix, G, ref, amp=True)
    return fs


@pytest.mark.parametrize("shape", list(AMP_SHAPES))
def test_fused_step_amp_matches_oracle_amp(cuda_device, shape):
    """amp (the shipped config.yml setting) against the oracle's autocast restatement:
    losses and every gradient entry (fp16-class tolerance, see module doc)."""
    _amp_vs_oracle("amp" if shape == "split" else f"amp_{shape}", cuda_device, shape=shape)


# the default MLP weight-gradient flush is block-reduced at every size; bwd_flush 1 keeps the
# per-wave flush under test. compact_per_block 4096: the compaction's 16-flags-per-thread branch
# (one 16-B load per thread), which the library selects only from 262,144 tiles (R >= 43,691)
HEADLINE_SCATTER = {"scan8": dict(scatter_levels_per_wave=8, compact_per_block=4096),
                    "scan8_wave_flush": dict(scatter_levels_per_wave=8, bwd_flush=1)}


@pytest.mark.parametrize("scatter", list(HEADLINE_SCATTER))
def test_headline_kernel_instances_amp_match_oracle_amp(cuda_device, scatter):
    """The kernel instances the headline (64 frames x 2048 rays, amp) runs, forced on an
    oracle-sized batch and checked entry by entry against the oracle's autocast step
    (VERDICT r3, r4): the scatter at its headline shape (run-scan, 8 levels per wave), the
    quad-mirror encode (quads_min_rays lowered from 32,768) and the tile compaction's
    16-flags-per-thread branch (compact_per_block 4096, the headline's). Two batch sizes:
    384 rays, and 1,024 rays (several persistent tiles per backward wave); the tile lists
    must hold every flagged tile (a dropped tile zeroes its gradients)."""
    dev = cuda_device
    for R, seed in ((384, 3), (1024, 43)):
        fs = _amp_vs_oracle(f"headline_{scatter}_R{R}", dev, knobs=dict(HEADLINE_SCATTER[scatter], quads_min_rays=1),
                            seed=seed, R=R)
        assert int(torch.count_nonzero(fs.quads).item()) > 0, "the quad-mirror encode did not run"
        bl, cl = fs.tile_lists()
        offs, nt = fs._ws_offsets()
        flags = fs.workspace[offs["tile_bwd"]:offs["tile_bwd"] + nt].cpu().numpy()
        want_b = np.nonzero((flags == 1) | (flags == 2))[0]
        want_c = np.nonzero((flags == 1) | (flags == 3))[0]
        got_b = np.sort(bl.cpu().numpy() & 0x7fffffff) >> 5
        np.testing.assert_array_equal(got_b, want_b)
        np.testing.assert_array_equal(cl.cpu().numpy() >> 5, want_c)


def test_fs_rgb_loss_matches_oracle(cuda_device):
    """cfg fs_rgb_weight > 0 (train_loop :728-731): front samples' colour pulled to
    white; value and every gradient vs the oracle."""
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=23)
    cfg["fs_rgb_weight"] = 10.0
    fs, enc, out = _run_fused(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, cuda_device)
    ref = _oracle_ref(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, enc)
    assert ref["fs_rgb_loss"] > 0
    np.testing.assert_allclose(float(out["fs_rgb_loss"].item()), ref["fs_rgb_loss"], rtol=1e-4)   # unweighted metric
    lt = out["loss_terms"].cpu().numpy()
    np.testing.assert_allclose(lt[:4].sum() + 10.0 * float(out["fs_rgb_loss"].item()), ref["loss"], rtol=1e-4)
    assert mask_flips(out["dbg"], ref, batch, cfg, NS.truncation(cfg)) == 0
    G = fs.split(out["grads"].cpu())
    _check_all("fs_rgb", G, ref)


@pytest.mark.parametrize("kind", ["linear", "exp"])
def test_truncation_schedule_matches_oracle(cuda_device, kind):
    """trunc_decay_type (get_truncation nerf_runner.py:661-674) at global_step 12 of a
    100-step round (the exp schedule reaches trunc at n_step / 4): sampling band,
    compositing weights, losses and gradients. Samples on a loss-mask threshold are counted,
    bounded and evaluated on the kernels' branch by the oracle (aligned_ref)."""
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=29)
    cfg.update(trunc_decay_type=kind, trunc_start=0.03, trunc=0.01, n_step=100)
    fs, enc, out = _run_fused(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, cuda_device, global_step=12)
    ref = aligned_ref(f"trunc_{kind}", out["dbg"],
                      lambda **kw: _oracle_ref(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, enc, step=12, **kw),
                      batch, cfg, NS.truncation(cfg, 12))
    assert NS.truncation(cfg, 12) > 1.2 * NS.truncation(cfg, 100)     # the band is still annealing
    np.testing.assert_allclose(out["dbg"]["z"].cpu().numpy(), ref["z_vals"].numpy(), rtol=1e-6, atol=2e-6)
    np.testing.assert_allclose(out["dbg"]["rgb"].cpu().numpy(), ref["rgb_map"].numpy(), rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(out["loss_terms"].cpu().numpy()[:4].sum(), ref["loss"], rtol=1e-4)
    G = fs.split(out["grads"].cpu())
    _check_all(f"trunc_{kind}", G, ref)


def test_frozen_poses_skip_input_gradient(golden_dir, cuda_device):
    """cfg optimize_poses = 0 (NerfRunner freezes the pose array): the fused step skips
    the input gradient (no corner re-gather, no dL/dtf — the reference's grid backward
    computes dy_dx only when its inputs need grad). Every other gradient is unchanged:
    the table / MLP gradients equal the pose-optimising step's up to float-atomic order,
    the pose gradient is zero."""
    from bundlesdf_amd.fused import FusedStep
    g = np.load(os.path.join(golden_dir, "train_step.npz"))
    cfg = json.loads(str(g["cfg_json"]))
    dev = cuda_device
    L = cfg["num_levels"]
    mlp_w = {k: g["w0_" + k] for k in NS.MLP_KEYS}
    t_rand = torch.from_numpy(g["t_rand"]).to(dev)
    grads = {}
    for opt in (1, 0):
        c = dict(cfg, optimize_poses=opt)
        enc, net, pa = _build(dev, c, g["emb0"], mlp_w, g["pose0"], L, cfg["log2_hashmap_size"], cfg["finest_res"])
        fs = FusedStep(c, torch.from_numpy(g["batch"]).to(dev), torch.from_numpy(g["c2w"]), torch.from_numpy(g["occ"]),
                       enc, net, pa, amp=False)
        assert fs.pose_grad == bool(opt)
        out = fs.step(ids=torch.arange(g["batch"].shape[0], dtype=torch.int32, device=dev), t_rand=t_rand, debug=True)
        grads[opt] = fs.split(out["grads"].cpu())
    for k, ref in grads[1].items():
        got = grads[0][k]
        if k == "pose":
            assert float(got.abs().max()) == 0.0
            assert float(ref.abs().max()) > 0.0
        else:
            # two runs of the same sums in a different float-atomic order
            np.testing.assert_allclose(got.numpy(), ref.numpy(), rtol=1e-4, atol=1e-6 * float(ref.abs().max()) + 1e-30,
                                       err_msg=k)


def test_fused_step_rejects_level_resolution_beyond_scatter_keys(golden_dir, cuda_device):
    """k_scatter's run keys hold 10 bits per cell coordinate: a grid whose finest level
    exceeds resolution 1023 is refused at construction instead of merging neighbouring cells' runs."""
    from bundlesdf_amd.fused import FusedStep
    g = np.load(os.path.join(golden_dir, "train_step.npz"))
    cfg = json.loads(str(g["cfg_json"]))
    dev = cuda_device
    mlp_w = {k: g["w0_" + k] for k in NS.MLP_KEYS}
    for finest, ok in ((1000, True), (2048, False)):
        from bundlesdf_amd.grid import GridEncoder
        enc = GridEncoder(3, cfg["num_levels"], 2, 16, 19, finest).to(dev)
        _, net, pa = _build(dev, cfg, g["emb0"], mlp_w, g["pose0"], cfg["num_levels"], cfg["log2_hashmap_size"],
                            cfg["finest_res"])
        make = lambda: FusedStep(cfg, torch.from_numpy(g["batch"]).to(dev), torch.from_numpy(g["c2w"]),  # noqa: E731
                                 torch.from_numpy(g["occ"]), enc, net, pa, amp=False)
        if ok:
            make()
        else:
            with pytest.raises(ValueError, match="10-bit cell keys"):
                make()


# Ragged and empty batches (the parity bar's "empty and ragged inputs"): batch sizes that are not
# multiples of any block / wave / chunk size, a single ray, rays of the reference's type 1 (invalid
# depth, nerf_runner.py:253-255: no loss weight, train_loop :692,722) mixed in with depths beyond far
# (the free-space branch), and a batch with no loss-carrying ray at all (empty tile lists: every
# persistent backward wave and the scatter have nothing to do, every gradient must be exactly zero).
EDGE_CASES = {"ragged37": dict(R=37, seed=31), "single": dict(R=64, seed=37), "mixed45": dict(R=45, seed=41),
              "no_backward64": dict(R=64, seed=43)}


@pytest.mark.parametrize("amp", [False, True], ids=["fp32", "amp"])
@pytest.mark.parametrize("case", list(EDGE_CASES))
def test_fused_step_ragged_and_empty_batches_match_oracle(cuda_device, case, amp):
    R, seed = EDGE_CASES[case]["R"], EDGE_CASES[case]["seed"]
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs = _scene_case(seed=seed, R=R)
    batch = batch.copy()
    if case == "single":   # one object ray (type 0, mask set, depth inside [near, far]) of the drawn 64
        sc = cfg["sc_factor"]
        ok = np.nonzero((batch[:, 9] == 0) & (batch[:, 7] > 0) & (batch[:, 6] > cfg["near"] * sc) &
                        (batch[:, 6] < cfg["far"] * sc))[0]
        batch, t_rand = batch[ok[:1]].copy(), t_rand[ok[:1]].copy()
    if case == "mixed45":
        batch[1::3, 9] = 1.0                                            # invalid-depth rays
        batch[2::5, 6] = 2.0 * cfg["far"] * cfg["sc_factor"]            # depth beyond far: free space
    if case == "no_backward64":
        batch[:, 9] = 1.0
    cfg["amp"] = amp
    scale = 1024.0 if amp else None
    fs, enc, out = _run_fused(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, cuda_device, amp=amp, scale=scale)
    kw = dict(amp=True, loss_scale=1024.0) if amp else {}
    prefix = f"edge_{case}_{'amp' if amp else 'fp32'}"
    ref = aligned_ref(prefix, out["dbg"], lambda **k2: _oracle_ref(cfg, seq, batch, occ, t_rand, mlp_w, emb, pose,
                                                                    offs, enc, **kw, **k2),
                      batch, cfg, NS.truncation(cfg))
    dbg = out["dbg"]
    np.testing.assert_allclose(dbg["z"].cpu().numpy(), ref["z_vals"].numpy(), rtol=1e-6, atol=2e-6)
    if amp:
        np.testing.assert_allclose(dbg["raw"].cpu().numpy(), ref["raw"].numpy(), rtol=1e-2, atol=2e-3)
        np.testing.assert_allclose(dbg["rgb"].cpu().numpy(), ref["rgb_map"].numpy(), rtol=2e-3, atol=1e-4)
    else:
        np.testing.assert_allclose(dbg["raw"].cpu().numpy(), ref["raw"].numpy(), rtol=1e-4, atol=2e-5)
        np.testing.assert_allclose(dbg["rgb"].cpu().numpy(), ref["rgb_map"].numpy(), rtol=1e-4, atol=1e-5)
    lt = out["loss_terms"].cpu().numpy().astype(np.float64)
    assert np.isfinite(lt[:8]).all()
    got = {"rgb_loss": lt[0], "fs_loss": lt[1] + lt[2], "sdf_loss": lt[3]}
    for k, v in got.items():
        np.testing.assert_allclose(v, float(ref[k]), rtol=AMP_LOSS_TOL if amp else 1e-4, atol=1e-9, err_msg=k)
    G = fs.split(out["grads"].cpu())
    if case != "no_backward64":   # a case that exercises the backward (its ray(s) carry loss gradients)
        assert float(ref["loss"]) > 0 and int(torch.count_nonzero(ref["grads"]["embeddings"])) > 0
        assert int(torch.count_nonzero(G["embeddings"])) > 0
    if case == "no_backward64":
        assert float(ref["loss"]) == 0.0
        for k, g in G.items():
            assert int(torch.count_nonzero(g)) == 0, k
        assert fs.n_tile_records() == 0
        return
    _check_all(prefix, G, ref, amp=amp)
