"""GPU: the optimiser state machine of the fused trainer over many steps —
GradScaler (init 2^16, backoff 0.5, growth x2 every `growth_interval` clean
steps, skip on inf/NaN with the Adam step count not advanced), Adam(betas
(0.9, 0.999), eps 1e-15) with the 'basic' / 'pose_array' groups, and the
schedule_lr decay every 10 steps (nerf_runner.py:159,490-502,577-581,755-762)
— against the reference's own objects: torch.optim.Adam and
torch.amp.GradScaler on the same device, fed each step with the gradients the
fused step produced (so the comparison has no feedback and stays tight).
Each step's gradients are also checked against the CPU oracle
(oracle/nerf_step.py, fp32 or its autocast restatement) at the same parameters,
worst entry within the tolerances of test_gpu_step.py."""
import json
import math
import os

import numpy as np
import pytest
import torch

from oracle import nerf_step as NS
from tests.test_gpu_step import _METRICS, AMP_GRAD_TOL, GRAD_TOL, _check_all, _check_grad, mask_flips

pytestmark = pytest.mark.gpu

K_STEPS = 25
INF_STEP = 12


def _build(dev, g, cfg):
    from bundlesdf_amd.fused import FusedStep
    from bundlesdf_amd.grid import GridEncoder
    from bundlesdf_amd.nerf_helpers import NeRFSmall, PoseArray
    L = cfg["num_levels"]
    enc = GridEncoder(3, L, 2, cfg["base_res"], cfg["log2_hashmap_size"], cfg["finest_res"]).to(dev)
    enc.embeddings.data.copy_(torch.from_numpy(g["emb0"]))
    net = NeRFSmall(2, 64, 15, 3, 64, input_ch=2 * L, input_ch_views=9).to(dev)
    net.load_state_dict({k: torch.from_numpy(g["w0_" + k]) for k in NS.MLP_KEYS})
    pa = PoseArray(g["pose0"].shape[0], cfg["max_trans"] * cfg["sc_factor"], cfg["max_rot"]).to(dev)
    pa.data.data.copy_(torch.from_numpy(g["pose0"]))
    batch = torch.from_numpy(g["batch"])
    fs = FusedStep(cfg, batch.to(dev), torch.from_numpy(g["c2w"]), torch.from_numpy(g["occ"]), enc, net, pa,
                   amp=cfg["amp"])
    return fs, batch


@pytest.mark.parametrize("amp", [False, True], ids=["fp32", "amp"])
def test_multi_step_optimizer_state_machine(golden_dir, cuda_device, amp):
    """25 steps. The parameter trajectory is the oracle's own (deterministic: each step
    starts from the oracle's parameters, written into the fused trainer's flat buffer),
    so the per-step gradient checks are reproducible; the fused optimiser state (Adam
    moments, step count, GradScaler scale / tracker) evolves from the fused gradients
    and is compared with torch.optim.Adam + torch.amp.GradScaler fed the same ones."""
    g = np.load(os.path.join(golden_dir, "train_step.npz"))
    cfg = json.loads(str(g["cfg_json"]))
    cfg.update(amp=amp, n_step=K_STEPS - 1)              # N_iters = 25: schedule_lr after steps 10 and 20
    dev = cuda_device
    fs, batch = _build(dev, g, cfg)
    fs.growth_interval = 5                                 # exercise GradScaler growth inside 25 steps
    assert fs.P.numel() % 4 != 0, "the Adam kernel's tail loop must run"
    R = batch.shape[0]
    S = cfg["N_samples"] + cfg["N_samples_around_depth"]
    meta = (g["offsets"], float(np.log2(g["per_level_scale"][0])), cfg["base_res"])
    # the reference optimiser (nerf_runner.py:490-502) over the flat parameters
    basic = torch.nn.Parameter(fs.P[:fs.pose_off].detach().clone())
    pose = torch.nn.Parameter(fs.P[fs.pose_off:].detach().clone())
    opt = torch.optim.Adam([{"params": [basic], "lr": cfg["lrate"]}, {"params": [pose], "lr": cfg["lrate_pose"]}],
                           betas=(0.9, 0.999), eps=1e-15, weight_decay=0, foreach=False)
    init_lr = [cfg["lrate"], cfg["lrate_pose"]]
    scaler = torch.amp.GradScaler("cuda", init_scale=65536.0, growth_factor=2.0, backoff_factor=0.5,
                                  growth_interval=5, enabled=amp)
    scaler.scale(torch.zeros((), device=dev))             # materialises the scale tensor (lazy in torch)
    # the oracle's trajectory
    traj = fs.split(fs.P.detach().cpu().clone())
    traj = {k: v.clone() for k, v in traj.items()}
    ostate = None
    o_lr = {k: cfg["lrate"] for k in traj}
    o_lr["pose"] = cfg["lrate_pose"]
    o_t = 0
    rng = np.random.default_rng(0)
    worst = {"param": 0.0}
    n_skips = 0
    n_flip_steps = 0         # steps with a sample on a loss-mask threshold (entry-wise check undefined there)
    ids = torch.arange(R, dtype=torch.int32, device=dev)
    for t in range(K_STEPS):
        t_rand = rng.uniform(size=(R, S)).astype(np.float32)
        flat = torch.cat([traj[k].reshape(-1) for k in _keys(fs)]).to(dev)
        with torch.no_grad():
            fs.P.copy_(flat)
        fs.refresh_half_table()
        scale_before = float(fs.scale.item())
        adam_t_before = int(fs.adam_t.item())

        def poison(f):
            f.G[f.mlp_off + 7] = float("inf")              # a non-finite gradient entry (scaled, fp32 MLP part)
        out = fs.step(ids=ids, t_rand=torch.from_numpy(t_rand), debug=True,
                      grad_hook=poison if (amp and t == INF_STEP) else None)
        torch.cuda.synchronize()
        grads = out["grads"]                               # unscaled, [table | mlp | pose]
        # gradient parity with the oracle at the same parameters, every step
        ref = NS.train_step({k: v.clone() for k, v in traj.items()}, batch, torch.from_numpy(g["c2w"]), g["occ"], cfg,
                            torch.from_numpy(t_rand), meta, step=t, amp=amp, loss_scale=scale_before)
        poisoned = amp and t == INF_STEP
        # under autocast the reference's weight gradients are fp16: at a large scale they overflow
        # and its GradScaler skips the step — the fused trainer must skip the same steps
        ref_overflow = amp and not all(bool(torch.isfinite(v).all()) for v in ref["grads"].values())
        skipped = int(fs.adam_t.item()) == adam_t_before
        assert skipped == (poisoned or ref_overflow), (t, skipped, poisoned, ref_overflow)
        n_skips += skipped
        flips = mask_flips(out["dbg"], ref, batch, cfg, NS.truncation(cfg, t))
        n_flip_steps += flips > 0
        if not skipped and flips == 0:
            G = fs.split(grads.cpu())
            pre = f"{'amp' if amp else 'fp32'}/step{t}"
            _check_all(pre, G, ref, keys=["embeddings"] + ([] if amp else NS.MLP_KEYS), amp=amp)
            if amp:
                # along an amp trajectory, hidden units whose fp16 pre-activations sit at 0 flip
                # their ReLU between the autocast reference and the MFMA chains (different fp16
                # rounding points), which moves single weight-gradient entries by O(1); the first
                # step is checked entry by entry (test_gpu_step), later steps by relative L2 norm
                for k in NS.MLP_KEYS:
                    a_, b_ = G[k].double(), ref["grads"][k].double()
                    e = float((a_ - b_).norm() / (b_.norm() + 1e-30))
                    _METRICS[f"{pre}/{k}/rel_l2"] = e
                    assert e < 5e-2, (t, k, e)
            # the pose gradient sums dL/dx over every sample, and dL/dx (the trilinear derivative
            # dy_dx) jumps where a sample crosses a cell face: once training has grown the table, a
            # sample within rounding distance of a face moves the pose gradient by ~1e-2 of its scale
            _check_grad(f"{pre}/pose", G["pose"].numpy(), ref["grads"]["pose"].numpy(),
                        tol=AMP_GRAD_TOL if amp else GRAD_TOL, eps=5.0)
        # the reference optimiser on the same gradients (scaled as the backward produced them),
        # from the same parameters
        with torch.no_grad():
            basic.copy_(flat[:fs.pose_off])
            pose.copy_(flat[fs.pose_off:])
        gs = grads.to(dev) * scaler.get_scale() if amp else grads.to(dev)
        if amp:   # the reference holds the NeRFSmall weight gradients in fp16: beyond its range they are inf
            # (frame features, when present, are fp32 parameters summed in fp32: [mlp_off, feat_off) only)
            seg = gs[fs.mlp_off:fs.feat_off]
            seg[seg.abs() >= 65520.0] = float("inf")
        basic.grad = gs[:fs.pose_off].clone()
        pose.grad = gs[fs.pose_off:].clone()
        scaler.step(opt)
        scaler.update()
        if t % 10 == 0 and t > 0:                          # schedule_lr (nerf_runner.py:577-581, :761-762)
            for i, pg in enumerate(opt.param_groups):
                pg["lr"] = init_lr[i] * cfg["decay_rate"] ** (float(t) / (cfg["n_step"] + 1))
        got = fs.P.detach()
        if skipped:
            # skipped step: parameters unchanged, scale backed off, Adam step count not advanced
            assert torch.equal(got, flat)
            assert float(fs.scale.item()) == scale_before * 0.5
            assert int(fs.tracker.item()) == 0
        assert float(fs.scale.item()) == float(scaler.get_scale())
        err = float((got - torch.cat([basic.detach(), pose.detach()])).abs().max().item())
        worst["param"] = max(worst["param"], err)
        assert err <= 2e-6, (t, err)
        # optimiser bookkeeping: gradients cleared, fp16 table mirror refreshed
        assert float(fs.G.abs().max().item()) == 0.0
        if amp:
            assert float(fs.G16.float().abs().max().item()) == 0.0
            assert torch.equal(fs.emb16, fs.P[:fs.n_emb].half())
        # next oracle state: Adam on the oracle's gradients with the reference schedule
        if not skipped:
            traj, ostate = NS.adam_step(traj, ref["grads"], ostate, o_t, o_lr)
            o_t += 1
        if t % 10 == 0 and t > 0:
            o_lr = {k: (cfg["lrate_pose"] if k == "pose" else cfg["lrate"]) *
                    cfg["decay_rate"] ** (float(t) / (cfg["n_step"] + 1)) for k in traj}
    if amp:
        assert n_skips >= 1 and float(fs.scale.item()) != 65536.0   # backed off and grew during the run
    worst["skipped_steps"] = n_skips
    worst["mask_flip_steps"] = n_flip_steps
    # fp16 sdf values sit exactly on the thresholds (1.0, fs_sdf) far more often than fp32 ones
    assert n_flip_steps <= (K_STEPS // 2 if amp else K_STEPS // 5), n_flip_steps
    lr_now = [pg["lr"] for pg in opt.param_groups]
    assert math.isclose(lr_now[0], cfg["lrate"] * cfg["decay_rate"] ** (20 / 25))
    root = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    os.makedirs(root, exist_ok=True)
    pre = f"{'amp' if amp else 'fp32'}/"
    worst["grad"] = max(v for k, v in _METRICS.items() if k.startswith(pre))
    with open(os.path.join(root, f"optim_metrics_{'amp' if amp else 'fp32'}.json"), "w") as f:
        json.dump(worst, f)


def _keys(fs):
    from bundlesdf_amd import mlp_layout as ML
    return ["embeddings"] + list(ML.MLP_KEYS) + ["pose"]


def test_amp_overflow_range_excludes_frame_features(cuda_device):
    """amp with frame_features > 0: the NeRFSmall weight gradients are fp16 under autocast
    (an entry at or beyond 65520 scaled is inf -> GradScaler skips), the FeatureArray
    gradient is an fp32 parameter gradient (summed in fp32: a large finite value steps
    normally). The kernel's overflow range is [mlp_off, feat_off)."""
    from tests.test_gpu_step import _ff_case, _ff_fused
    dev = cuda_device
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, ff = _ff_case(seed=43, R=64)
    cfg["amp"] = True
    R = batch.shape[0]
    ids = torch.arange(R, dtype=torch.int32, device=dev)
    for where, want_skip in (("features", False), ("mlp", True)):
        fs, _ = _ff_fused(dev, cfg, seq, batch, occ, mlp_w, emb, pose, ff, amp=True)
        fs.scale.fill_(1024.0)

        def poison(f):
            o = f.feat_off if where == "features" else f.mlp_off + 3
            f.G[o] = 70000.0                       # finite in fp32, beyond the fp16 range
        P0 = fs.P.detach().clone()
        fs.step(ids=ids, t_rand=torch.from_numpy(t_rand), grad_hook=poison)
        torch.cuda.synchronize()
        skipped = int(fs.adam_t.item()) == 0
        assert skipped == want_skip, (where, skipped)
        assert float(fs.scale.item()) == (512.0 if want_skip else 1024.0)
        assert torch.equal(fs.P, P0) == want_skip


def test_amp_inf_in_fp16_table_gradient_skips_step(cuda_device):
    """amp: the hash-table gradient is accumulated in fp16 (G16, as the reference's __half2
    atomics, gridencoder.cu:319-327); an inf or nan anywhere in it — first entry, middle, the
    last entry (past the kernel's 8-wide vector loads when the length is not a multiple of 8)
    — makes k_unscale_check skip the step exactly as GradScaler does; a large finite value
    does not."""
    from tests.test_gpu_step import _ff_case, _ff_fused
    dev = cuda_device
    cfg, seq, batch, occ, t_rand, mlp_w, emb, pose, offs, ff = _ff_case(seed=43, R=64)
    cfg["amp"] = True
    ids = torch.arange(batch.shape[0], dtype=torch.int32, device=dev)
    cases = []
    for where in ("first", "middle", "last"):
        for val in (float("inf"), float("-inf"), float("nan")):
            cases.append((where, val, True))
    cases.append(("middle", 60000.0, False))
    for where, val, want_skip in cases:
        fs, _ = _ff_fused(dev, cfg, seq, batch, occ, mlp_w, emb, pose, ff, amp=True)
        fs.scale.fill_(1024.0)
        n = fs.G16.numel()
        o = {"first": 0, "middle": n // 2 + 3, "last": n - 1}[where]

        def poison(f, o=o, val=val):
            f.G16[o] = val
        P0 = fs.P.detach().clone()
        fs.step(ids=ids, t_rand=torch.from_numpy(t_rand), grad_hook=poison)
        torch.cuda.synchronize()
        skipped = int(fs.adam_t.item()) == 0
        assert skipped == want_skip, (where, val, skipped)
        assert float(fs.scale.item()) == (512.0 if want_skip else 1024.0), (where, val)
        assert torch.equal(fs.P, P0) == want_skip, (where, val)


@pytest.mark.parametrize("amp", [False, True], ids=["fp32", "amp"])
def test_adam_active_flags_bit_identical_to_dense(cuda_device, amp):
    """k_adam's touched-group flags (one per 256 parameters; never-touched groups are
    neither read nor written) against the dense update (active=None) on the same gradients, over
    4 steps: P, M, V and the fp16 mirror bit-identical. Groups: never touched; touched at step 0
    and zero afterwards (must keep moving on its moments); touched every step; touched from step 2
    on; plus a partly-touched group and a tail past the last full group (n % 4 != 0)."""
    from bundlesdf_amd import _lib
    dev = cuda_device
    G = 256
    n = 10 * G + 7
    gen = torch.Generator().manual_seed(5)
    P0 = (torch.randn(n, generator=gen) * 0.1).to(dev)
    scale = torch.tensor([1024.0 if amp else 1.0], device=dev)
    st = {}
    for mode in ("dense", "flags"):
        P, M, V = P0.clone(), torch.zeros(n, device=dev), torch.zeros(n, device=dev)
        Gf = torch.zeros(n, device=dev)
        mirror = P0.half() if amp else None
        G16 = torch.zeros(n, dtype=torch.float16, device=dev) if amp else None
        act = torch.zeros(int(_lib.lib().nof_adam_active_bytes(n)), dtype=torch.uint8, device=dev) \
            if mode == "flags" else None
        t = torch.zeros(1, dtype=torch.int32, device=dev)
        inf = torch.zeros(1, dtype=torch.int32, device=dev)
        for k in range(4):
            g = torch.zeros(n)
            gk = torch.Generator().manual_seed(100 + k)
            g[1 * G:2 * G] = torch.randn(G, generator=gk) if k == 0 else 0.0      # touched, then zero
            g[2 * G:3 * G] = torch.randn(G, generator=gk)                          # every step
            if k >= 2:
                g[4 * G:5 * G] = torch.randn(G, generator=gk)                      # from step 2
            g[6 * G + 17] = 0.5 * (k + 1)                                          # one entry of a group
            g[10 * G + 5] = -0.25                                                  # the tail loop (n % 4)
            if amp:   # the table part as the scaled fp16 gradient, the rest fp32
                G16.copy_((g * scale.cpu()).half().to(dev))
            else:
                Gf.copy_(g.to(dev))
            _lib.check(_lib.lib().nof_adam_step(
                _lib.ptr(P), _lib.ptr(Gf), _lib.ptr(M), _lib.ptr(V), n, n - 5, 0.01, 0.001, 0.9, 0.999, 1e-15,
                _lib.ptr(t), _lib.ptr(inf), _lib.ptr(mirror), n if amp else 0, _lib.ptr(G16), _lib.ptr(scale),
                None, _lib.ptr(act), _lib.stream_of(P)), "adam")
            t += 1
        torch.cuda.synchronize()
        st[mode] = {k: v.cpu().numpy() for k, v in dict(P=P, M=M, V=V).items()}
        if amp:
            st[mode]["mirror"] = mirror.cpu().numpy()
            assert int(torch.count_nonzero(G16).item()) == 0          # cleared for the next step
        if mode == "flags":
            flags = act.cpu().numpy()
            assert flags[0] == 0 and flags[3] == 0 and flags[1] == 1 and flags[2] == 1 and flags[4] == 1
    for k in st["dense"]:
        np.testing.assert_array_equal(st["flags"][k], st["dense"][k], err_msg=k)
    P1 = st["dense"]["P"]
    P0h = P0.cpu().numpy()
    np.testing.assert_array_equal(P1[0:G], P0h[0:G])                      # never touched
    assert (P1[G:2 * G] != P0h[G:2 * G]).all()                            # moved at step 0 and after
    if amp:
        np.testing.assert_array_equal(st["dense"]["mirror"], P1.astype(np.float16))
