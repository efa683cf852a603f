"""Generate golden fixtures from the REFERENCE's own Python code.

Runs only in the build container (needs /root/reference, read-only); the
committed .npz files are what the GPU box and the CPU test-suite use. No
reference source is copied: the reference modules are imported from
/root/reference and executed; only their inputs/outputs are stored.

Third-party packages the reference imports at module level but that are absent
here (trimesh, open3d, cv2, kaolin, pytorch3d, ruamel, skimage, imageio,
transformations, matplotlib, PIL) and the CUDA extension modules
(gridencoder, mycuda) are replaced by empty module objects: none of the
functions exercised below calls into them.

Usage:  python tests/golden/make_golden.py [fixture ...]   (writes tests/golden/*.npz)
"""
import json
import os
import sys
import types

import numpy as np
import torch

REF = "/root/reference"
OUT = os.path.dirname(os.path.abspath(__file__))


def _stub_modules():
    names = ["trimesh", "imageio", "open3d", "cv2", "transformations", "ruamel", "ruamel.yaml", "kaolin",
             "pytorch3d", "pytorch3d.transforms", "skimage", "mycuda", "gridencoder", "matplotlib",
             "matplotlib.pyplot", "PIL", "PIL.Image"]
    for m in names:
        if m not in sys.modules:
            sys.modules[m] = types.ModuleType(m)
    sys.modules["ruamel.yaml"].YAML = lambda *a, **k: None
    sys.modules["ruamel"].yaml = sys.modules["ruamel.yaml"]
    t = sys.modules["pytorch3d.transforms"]
    t.so3_log_map = t.so3_exp_map = t.se3_exp_map = None
    sys.modules["PIL"].Image = sys.modules["PIL.Image"]


def _import_reference():
    if not os.path.isdir(REF):
        raise SystemExit("make_golden.py needs the read-only reference at /root/reference")
    _stub_modules()
    sys.path.insert(0, REF)
    sys.path.insert(0, os.path.join(REF, "mycuda", "torch_ngp_grid_encoder"))
    import grid as ref_grid  # noqa: E402
    sys.modules["mycuda"].__path__ = []
    tng = types.ModuleType("mycuda.torch_ngp_grid_encoder")
    tng.__path__ = []
    tng.grid = ref_grid
    sys.modules["mycuda.torch_ngp_grid_encoder"] = tng
    sys.modules["mycuda.torch_ngp_grid_encoder.grid"] = ref_grid
    import nerf_helpers as ref_helpers  # noqa: E402
    import nerf_runner as ref_runner  # noqa: E402
    return ref_grid, ref_helpers, ref_runner


GRID_CONFIGS = [  # (input_dim, n_levels, level_dim, base_res, log2_hashmap, finest)
    (3, 16, 2, 16, 22, 128),   # BASELINE config 2
    (3, 4, 2, 16, 22, 128),    # config.yml default (num_levels 4)
    (3, 16, 2, 16, 22, 256),   # global refine (run_custom.py:122-133): 3 hashed levels
    (3, 16, 2, 16, 19, 512),   # deep hashing
    (3, 8, 4, 8, 15, 64),
    (2, 6, 1, 4, 12, 64),
]


def gen_grid_layout(ref_grid):
    out = {}
    for i, (D, L, C, H, T, fin) in enumerate(GRID_CONFIGS):
        enc = ref_grid.GridEncoder(input_dim=D, n_levels=L, level_dim=C, base_resolution=H, log2_hashmap_size=T,
                                   desired_resolution=fin)
        out[f"cfg{i}"] = np.array([D, L, C, H, T, fin], np.int64)
        out[f"offsets{i}"] = enc.offsets.numpy().astype(np.int32)
        out[f"per_level_scale{i}"] = np.array([enc.per_level_scale], np.float64)
        out[f"n_params{i}"] = np.array([int(enc.n_params)], np.int64)
    np.savez_compressed(os.path.join(OUT, "grid_layout.npz"), **out)


class _FakeRunner:
    def __init__(self, cfg):
        self.cfg = cfg

    def get_truncation(self):
        return self.cfg["trunc"] * self.cfg["sc_factor"]


CFG = dict(trunc=0.01, sc_factor=6.0, sdf_lambda=5, neg_trunc_ratio=1, near=0.1, far=2.0, fs_sdf=0.001,
           empty_weight=0.01, trunc_decay_type="")


def _ray_case(R=48, S=192, seed=0):
    g = torch.Generator().manual_seed(seed)
    sc = CFG["sc_factor"]
    t = CFG["trunc"] * sc
    depth = 0.3 * sc + 0.1 * sc * torch.rand(R, generator=g)
    depth[::5] = 99 * sc                         # background rays (BAD_DEPTH*sc)
    depth[3] = 0.05 * sc                         # below near
    z_oct = torch.sort(depth[:, None] * (0.6 + 0.8 * torch.rand(R, 128, generator=g)), dim=1)[0]
    z_dep = torch.sort(depth[:, None] - t + 2 * t * torch.rand(R, 64, generator=g), dim=1)[0]
    z = torch.cat([z_oct, z_dep], 1)
    raw = torch.randn(R, S, 4, generator=g)
    rays_d = torch.cat([torch.randn(R, 2, generator=g) * 0.3, -torch.ones(R, 1)], 1)
    valid = torch.rand(R, S, generator=g) > 0.05
    valid[7] = False
    return depth, z, raw, rays_d, valid


def gen_render_loss(ref_helpers, ref_runner):
    depth, z, raw, rays_d, valid = _ray_case()
    fake = _FakeRunner(dict(CFG))
    raw_req = raw.clone().requires_grad_(True)
    rgb_map, weights = ref_runner.NerfRunner.raw2outputs(fake, raw_req, z, rays_d, valid_samples=valid, depth=depth)
    g_rgb = torch.randn_like(rgb_map, generator=torch.Generator().manual_seed(3))
    rgb_map.backward(g_rgb)
    R, S = z.shape
    sdf = raw[..., 3].clone().requires_grad_(True)
    sample_w = torch.rand(R, S, generator=torch.Generator().manual_seed(4)) * valid
    trunc = fake.get_truncation()
    fs, sdf_l, front, sdfm = ref_helpers.get_sdf_loss(z, depth.reshape(-1, 1).expand(-1, S), sdf, trunc, fake.cfg,
                                                      return_mask=True, sample_weights=sample_w, rays_d=rays_d)
    (fs + sdf_l).backward()
    np.savez_compressed(
        os.path.join(OUT, "render_loss.npz"), depth=depth.numpy(), z=z.numpy(), raw=raw.numpy(),
        rays_d=rays_d.numpy(), valid=valid.numpy(), g_rgb=g_rgb.numpy(), rgb_map=rgb_map.detach().numpy(),
        weights=weights.detach().numpy(), d_raw=raw_req.grad.numpy(), sample_w=sample_w.numpy(),
        fs_loss=np.array([fs.item()]), sdf_loss=np.array([sdf_l.item()]), front=front.numpy(), sdf_mask=sdfm.numpy(),
        d_sdf=sdf.grad.numpy(), trunc=np.array([trunc]),
        cfg=np.array([CFG["sc_factor"], CFG["trunc"], CFG["sdf_lambda"], CFG["neg_trunc_ratio"], CFG["near"],
                      CFG["far"], CFG["fs_sdf"], CFG["empty_weight"]]))


def gen_mlp(ref_helpers):
    torch.manual_seed(0)
    net = ref_helpers.NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3,
                                hidden_dim_color=64, input_ch=32, input_ch_views=9)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(333, 41, generator=g).requires_grad_(True)
    out = net(x)
    gout = torch.randn(out.shape, generator=g)
    out.backward(gout)
    d = {"x": x.detach().numpy(), "out": out.detach().numpy(), "gout": gout.numpy(), "dx": x.grad.numpy()}
    for k, v in net.state_dict().items():
        d["w_" + k] = v.numpy()
    for k, p in net.named_parameters():
        d["g_" + k] = p.grad.numpy()
    sdf = net.forward_sdf(x.detach()[:, :32])
    d["sdf"] = sdf.detach().numpy()
    np.savez_compressed(os.path.join(OUT, "mlp.npz"), **d)


def gen_sh_and_samplers(ref_helpers, ref_runner):
    g = torch.Generator().manual_seed(2)
    dirs = torch.nn.functional.normalize(torch.randn(200, 3, generator=g), dim=-1)
    d = {"dirs": dirs.numpy()}
    for deg in (1, 2, 3, 4, 5):
        d[f"sh{deg}"] = ref_helpers.SHEncoder(degree=deg)(dirs).numpy()
    near = torch.rand(50, 1, generator=g) + 0.1
    far = near + torch.rand(50, 1, generator=g) + 0.01
    for N in (128, 64, 7):
        torch.manual_seed(123 + N)
        zp = ref_runner.sample_rays_uniform(N, near, far, lindisp=False, perturb=True)
        torch.manual_seed(123 + N)
        d[f"t_rand{N}"] = torch.rand(50, N).numpy()
        d[f"z_perturb{N}"] = zp.numpy()
        d[f"z_plain{N}"] = ref_runner.sample_rays_uniform(N, near, far, lindisp=False, perturb=False).numpy()
    d["near"], d["far"] = near.numpy(), far.numpy()
    H, W = 12, 16
    K = np.array([[20.0, 0, 7.5], [0, 21.0, 5.5], [0, 0, 1]])
    d["cam_rays"] = ref_helpers.get_camera_rays_np(H, W, K)
    o = torch.randn(100, 3, generator=g, dtype=torch.float64) * 2
    dd = torch.randn(100, 3, generator=g, dtype=torch.float64)
    tmin, tmax = ref_helpers.ray_box_intersection_batch(o, dd, torch.tensor([[-1.0, -1, -1], [1, 1, 1]],
                                                                            dtype=torch.float64))
    d["box_o"], d["box_d"], d["box_tmin"], d["box_tmax"] = o.numpy(), dd.numpy(), tmin.numpy(), tmax.numpy()
    np.savez_compressed(os.path.join(OUT, "helpers.npz"), **d)




# ---------------------------------------------------------------------------
# G4: one full reference training step (NerfRunner.train_loop, executed from
# /root/reference on CPU). The reference's CUDA extensions and kaolin are
# replaced by the oracle restatements (oracle/kernels.py) and pytorch3d's
# se3_exp_map by its restated algorithm; everything else — render_rays,
# run_network, raw2outputs, the losses, autograd, Adam — is the reference's
# own code.
# ---------------------------------------------------------------------------
G4_CFG = dict(num_levels=4, log2_hashmap_size=12, finest_res=32, base_res=16, N_rand=96, amp=False)


def _install_oracle_extensions():
    repo = os.path.dirname(os.path.dirname(OUT))
    sys.path.insert(0, repo)
    from oracle import kernels as K
    from oracle import nerf_step as NS

    ge = sys.modules["gridencoder"]

    def grid_encode_forward(inputs, embeddings, offsets, outputs, B, D, C, L, S, H, cgi, dy_dx, gt, ac):
        out, dd = K.grid_encode_forward(inputs.detach().numpy(), embeddings.detach().numpy(), offsets.numpy(), S, H,
                                        calc_grad_inputs=cgi, gridtype=gt, align_corners=ac)
        outputs.copy_(torch.from_numpy(out))
        if cgi:
            dy_dx.copy_(torch.from_numpy(dd))

    def grid_encode_backward(grad, inputs, embeddings, offsets, gemb, B, D, C, L, S, H, cgi, dy_dx, gin, gt, ac):
        g, gi = K.grid_encode_backward(grad.numpy(), inputs.detach().numpy(), offsets.numpy(), gemb.shape[0], S, H,
                                       calc_grad_inputs=cgi, dy_dx=dy_dx.numpy() if cgi else None, gridtype=gt,
                                       align_corners=ac)
        gemb.copy_(torch.from_numpy(g))
        if cgi:
            gin.copy_(torch.from_numpy(gi))

    ge.grid_encode_forward = grid_encode_forward
    ge.grid_encode_backward = grid_encode_backward
    common = types.ModuleType("mycuda.common")

    def sampleRaysUniformOccupiedVoxels(z_in_out, z_sampled, z_vals):
        z, err = K.sample_occupied(z_in_out.numpy(), z_sampled.numpy(), z_vals.numpy())
        assert err == 0
        z_vals.copy_(torch.from_numpy(z))
        return z_vals

    common.sampleRaysUniformOccupiedVoxels = sampleRaysUniformOccupiedVoxels
    sys.modules["mycuda"].common = common
    sys.modules["mycuda.common"] = common
    sys.modules["pytorch3d.transforms"].se3_exp_map = NS.se3_exp_map
    return K, NS


class _OracleOctree:
    def __init__(self, K, occ):
        self.K, self.occ = K, occ

    def ray_trace(self, rays_o, rays_d, level, debug=False):
        assert 2 ** level == self.occ.shape[0]
        dio, counts = self.K.octree_ray_trace(self.occ, rays_o.detach().numpy(), rays_d.detach().numpy(),
                                              3 * self.occ.shape[0])
        k = max(1, int(counts.max()))
        dio = torch.from_numpy(dio[:, :k].copy())
        return dio[:, 0, 0:1], dio[:, :, 1].max(-1)[0][:, None], None, dio


class _Scaler:
    def __init__(self):
        self.losses = []

    def scale(self, loss):
        self.losses.append(loss.detach().clone())
        return loss

    def step(self, opt):
        opt.step()

    def update(self):
        pass


class _CpuAutocast:
    """G4-amp harness substitutions for the CUDA-only autocast entry points the reference
    calls: torch.cuda.amp.autocast(enabled=...) (nerf_runner.py:1254,1288) becomes
    torch.autocast("cpu", dtype=torch.float16, enabled=...), and torch.is_autocast_enabled()
    without a device (grid.py:50) reports the CPU state, so the encoder casts its table to
    fp16 as it does under CUDA autocast. Calls with a device argument pass through."""

    def __enter__(self):
        self._ac, self._ie = torch.cuda.amp.autocast, torch.is_autocast_enabled
        ie = self._ie
        torch.cuda.amp.autocast = lambda enabled=True, dtype=torch.float16, cache_enabled=True: torch.autocast(
            "cpu", dtype=torch.float16, enabled=enabled)
        torch.is_autocast_enabled = lambda *a: ie(*a) if a else ie("cpu")
        return self

    def __exit__(self, *exc):
        torch.cuda.amp.autocast, torch.is_autocast_enabled = self._ac, self._ie


class _RecordingGradScaler(torch.amp.GradScaler):
    """The reference's GradScaler (nerf_runner.py:159, :757-760) on the CPU device, recording
    the unscaled loss it is handed."""

    def __init__(self, init_scale):
        super().__init__("cpu", init_scale=init_scale)
        self.losses = []

    def scale(self, loss):
        self.losses.append(loss.detach().clone())
        return super().scale(loss)


G4_AMP_SCALE = 1024.0      # torch GradScaler init_scale is 2^16, at which this step's fp16 MLP gradients overflow (the reference would skip it and back off); 1024 = the amp parity tests' scale


def gen_train_step(ref_helpers, ref_runner, amp=False):
    """G4 (amp=False, train_step.npz) / G4-amp (amp=True, train_step_amp.npz): the same inputs, the
    reference's train_loop with cfg amp as given; amp runs under _CpuAutocast with a real GradScaler."""
    K, NS = _install_oracle_extensions()
    ref_helpers.se3_exp_map = NS.se3_exp_map       # bound at import time (nerf_helpers.py:15)
    ref_runner.common = sys.modules["mycuda.common"]  # Utils.py:28-31 import fell through at load time
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.octree import build_occupancy, coarsen
    torch.Tensor.cuda = lambda self, *a, **k: self
    seq = SY.make_sequence(3, seed=1)
    import yaml
    with open(os.path.join(REF, "config.yml")) as f:
        cfg = yaml.safe_load(f)                     # the reference's own defaults
    cfg.update(sc_factor=seq["sc_factor"], translation=seq["translation"], **G4_CFG)
    cfg["amp"] = bool(amp)
    sc = cfg["sc_factor"]
    from oracle import ray_pool as RP
    pool = RP.build_pool(range(3), seq["rgbs"], seq["depths"], seq["masks"], seq["poses"], seq["K"], cfg)
    max_level = int(np.ceil(np.log2(2.0 / (cfg["octree_smallest_voxel_size"] * sc))))
    level = int(np.floor(np.log2(2.0 / (cfg["octree_raytracing_voxel_size"] * sc))))
    occ_f = build_occupancy(torch.from_numpy(seq["octree_pts"]).float(), max_level, 1)
    occ = coarsen(occ_f, 2 ** (max_level - level)).numpy()
    rng = np.random.default_rng(5)
    obj = np.where(pool[:, 6] <= cfg["far"] * sc)[0]
    bg = np.where(pool[:, 6] > cfg["far"] * sc)[0]
    ids = np.concatenate([rng.choice(obj, 64, replace=False), rng.choice(bg, 32, replace=False)])
    rng.shuffle(ids)
    batch = torch.from_numpy(pool[ids])

    torch.manual_seed(0)
    runner = object.__new__(ref_runner.NerfRunner)
    runner.cfg = cfg
    runner.octree_m = None
    runner.images = seq["rgbs"]
    runner.create_nerf(device=torch.device("cpu"))
    runner.models["pose_array"].data.data = torch.randn(3, 6, generator=torch.Generator().manual_seed(9)) * 0.05
    runner.create_optimizer()
    runner.octree_m = _OracleOctree(K, occ)
    runner.amp_scaler = _RecordingGradScaler(G4_AMP_SCALE) if amp else _Scaler()
    runner.global_step = 0
    runner.N_iters = cfg["n_step"] + 1
    runner.c2w_array = torch.tensor(seq["poses"]).float()
    runner.ray_dir_slice, runner.ray_rgb_slice, runner.ray_depth_slice, runner.ray_mask_slice = [0, 1, 2], [3, 4, 5], 6, 7
    runner.ray_frame_id_slice, runner.ray_type_slice, runner.ray_near_slice, runner.ray_far_slice = 8, 9, 10, 11
    runner.data_loader = types.SimpleNamespace(batch_ray_ids=torch.from_numpy(ids))
    runner._run = None
    params0 = {k: v.detach().clone() for k, v in runner.models["model"].state_dict().items()}
    emb0 = runner.models["embed_fn"].embeddings.detach().clone()
    pose0 = runner.models["pose_array"].data.detach().clone()

    draws = []
    gen = torch.Generator().manual_seed(77)
    real_rand = torch.rand

    def rec_rand(*shape, **kw):
        kw.pop("device", None)
        kw.pop("generator", None)
        t = real_rand(*shape, generator=gen, **kw)
        draws.append(t.clone())
        return t

    captured = {}
    real_render = runner.render

    def rec_render(*a, **kw):
        rgb, extras = real_render(*a, **kw)
        captured["rgb"], captured["extras"] = rgb.detach().clone(), {k: v.detach().clone() for k, v in
                                                                     extras.items()}
        return rgb, extras

    runner.render = rec_render
    torch.rand = rec_rand
    try:
        if amp:
            with _CpuAutocast():
                runner.train_loop(batch)
        else:
            runner.train_loop(batch)
    finally:
        torch.rand = real_rand
    # assemble t_rand [R, N + N_around] from the three draws (render_rays :1060,:1070,:1074)
    N, Na = cfg["N_samples"], cfg["N_samples_around_depth"]
    depth = batch[:, 6]
    vmask = (depth >= cfg["near"] * sc) & (depth <= cfg["far"] * sc)
    t_rand = torch.zeros(len(ids), N + Na)
    t_rand[:, :N] = draws[0]
    t_rand[vmask, N:] = draws[1]
    if (~vmask).any():
        t_rand[~vmask, N:] = draws[2]
    net = runner.models["model"]
    d = dict(batch=batch.numpy(), c2w=np.asarray(seq["poses"], np.float32), occ=occ, t_rand=t_rand.numpy(),
             emb0=emb0.numpy(), offsets=runner.models["embed_fn"].offsets.numpy(),
             per_level_scale=np.array([runner.models["embed_fn"].per_level_scale]), pose0=pose0.numpy(),
             loss=runner.amp_scaler.losses[0].numpy(), rgb_map=captured["rgb"].numpy(),
             z_vals=captured["extras"]["z_vals"].numpy(), raw=captured["extras"]["raw"].numpy(),
             valid=captured["extras"]["valid_samples"].numpy(), weights=captured["extras"]["weights"].numpy(),
             g_emb=runner.models["embed_fn"].embeddings.grad.numpy(),
             g_pose=runner.models["pose_array"].data.grad.numpy(),
             emb1=runner.models["embed_fn"].embeddings.detach().numpy(),
             pose1=runner.models["pose_array"].data.detach().numpy(),
             cfg_json=np.array(json.dumps({k: v for k, v in cfg.items() if not isinstance(v, np.ndarray)},
                                          default=float)))
    for k, v in params0.items():
        d["w0_" + k] = v.numpy()
    for k, p in net.named_parameters():
        d["g_" + k] = p.grad.numpy()
        d["w1_" + k] = p.detach().numpy()
    if amp:
        # GradScaler.step unscaled the .grad tensors in place (the stored gradients are unscaled);
        # the scale the backward ran at, and whether the step was skipped for a non-finite gradient
        sc_ = runner.amp_scaler
        d["loss_scale"] = np.array([G4_AMP_SCALE])
        d["scale_after"] = np.array([sc_.get_scale()])
        d["found_inf"] = np.array([float(d["scale_after"][0] < G4_AMP_SCALE)])   # update() backs off on inf
        assert d["found_inf"][0] == 0, "G4-amp: the reference step overflowed at the initial scale"
        # the reference's fp16 table read: the encoder's outputs are the fp16 kernel's (grid.py:50-61)
        assert captured["extras"]["raw"].dtype == torch.float32
    np.savez_compressed(os.path.join(OUT, "train_step_amp.npz" if amp else "train_step.npz"), **d)


# ---------------------------------------------------------------------------
# G5: ray-pool construction — the reference's own NerfRunner.make_frame_rays
# (nerf_runner.py:244-314, with compute_near_far_and_filter_rays and
# ray_box_intersection_batch) executed from /root/reference on CPU. cv2.dilate
# (absent) is restated as oracle.ray_pool.dilate; kaolin's trace is the oracle
# dense-grid trace. The denoise step (inline in the reference's __init__) is
# oracle.ray_pool.denoise, so "pool_denoised" is restatement-pinned only.
# ---------------------------------------------------------------------------
def gen_ray_pool(ref_helpers, ref_runner):
    K, _ = _install_oracle_extensions()
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.octree import build_occupancy, coarsen
    from oracle import ray_pool as RP
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.modules["cv2"].dilate = lambda m, kernel, iterations=1: RP.dilate(m, kernel.shape[0])
    ref_runner.cv2 = sys.modules["cv2"]
    seq = SY.make_sequence(3, seed=2)
    r = 4                                             # down_scale_ratio: 160x120 frames, 15 px dilation
    import yaml
    with open(os.path.join(REF, "config.yml")) as f:
        cfg = yaml.safe_load(f)
    cfg.update(sc_factor=seq["sc_factor"], translation=seq["translation"], down_scale_ratio=r)
    sc = cfg["sc_factor"]
    images = np.ascontiguousarray(seq["rgbs"][:, ::r, ::r])
    depths = np.ascontiguousarray(seq["depths"][:, ::r, ::r]).copy()
    masks = np.ascontiguousarray(seq["masks"][:, ::r, ::r])
    N, H, W = images.shape[:3]
    Km = seq["K"].copy()
    Km[0] *= W / seq["rgbs"].shape[2]
    Km[1] *= H / seq["rgbs"].shape[1]
    rng = np.random.default_rng(3)
    for f in range(N):                                # invalid depth inside the mask -> type 1 (dropped)
        vs, us = np.where(masks[f, ..., 0] > 0)
        pick = rng.choice(len(vs), 40, replace=False)
        depths[f, vs[pick[:20]], us[pick[:20]], 0] = 0.05 * sc      # < near*sc
        depths[f, vs[pick[20:]], us[pick[20:]], 0] = 2.5 * sc       # > far*sc
    occ_masks = np.zeros((N, H, W), np.uint8)
    occ_masks[2, 40:70, 60:100] = 1
    max_level = int(np.ceil(np.log2(2.0 / (cfg["octree_smallest_voxel_size"] * sc))))
    level = RP.trace_level(cfg)
    occ_f = build_occupancy(torch.from_numpy(seq["octree_pts"]).float(), max_level, 1)
    occ = coarsen(occ_f, 2 ** (max_level - level)).numpy()
    runner = object.__new__(ref_runner.NerfRunner)
    runner.cfg, runner.H, runner.W, runner.K = cfg, H, W, Km
    runner.images, runner.depths, runner.masks = images, depths, masks
    runner.normal_maps, runner.occ_masks, runner.poses = None, occ_masks, seq["poses"]
    runner.octree_m = _OracleOctree(K, occ)
    per_frame = [runner.make_frame_rays(f) for f in range(N)]
    pool = np.concatenate(per_frame, 0)
    # denoise against a cloud with the box half removed: depth points there become type 1
    cloud = seq["octree_pts"][seq["octree_pts"][:, 0] < (0.06 + seq["translation"][0]) * sc]
    den = RP.denoise(pool, seq["poses"], cloud, cfg)
    d = dict(images=images, depths=depths, masks=masks, occ_masks=occ_masks, poses=seq["poses"], K=Km, occ=occ,
             cloud=cloud, pool=pool.astype(np.float32), pool_denoised=den.astype(np.float32),
             frame_counts=np.array([len(p) for p in per_frame], np.int64),
             cfg_json=json.dumps({k: (v.tolist() if isinstance(v, np.ndarray) else v) for k, v in cfg.items()}))
    np.savez_compressed(os.path.join(OUT, "ray_pool.npz"), **d)
    print("ray_pool:", len(pool), "rays,", len(den), "after denoise")


# ---------------------------------------------------------------------------
# G6: online hand-off helpers — the reference's own Utils.depth2xyzmap,
# Utils.get_optimized_poses_in_real_world (PoseArray from nerf_helpers with
# pytorch3d's se3_exp_map restated, as G4), tool.find_biggest_cluster and
# tool.compute_translation_scales (sklearn DBSCAN, installed here).
# ---------------------------------------------------------------------------
def gen_handoff(ref_helpers, ref_runner):
    _, NS = _install_oracle_extensions()
    ref_helpers.se3_exp_map = NS.se3_exp_map
    import Utils as ref_utils
    import tool as ref_tool
    rng = np.random.default_rng(11)
    d = {}
    depth = rng.uniform(0.05, 1.5, (48, 64))
    depth[5:9, 10:20] = 0.0
    K = np.array([[600.0, 0, 31.5], [0, 600.0, 23.5], [0, 0, 1]])
    d["depth"], d["K"] = depth, K
    d["xyz"] = ref_utils.depth2xyzmap(depth, K)
    # three clusters of different sizes + scattered noise (metres)
    c = [rng.normal([0, 0, 0.5], 0.02, (700, 3)), rng.normal([0.3, 0, 0.5], 0.015, (250, 3)),
         rng.normal([0, 0.4, 0.6], 0.01, (90, 3)), rng.uniform(-1, 1, (40, 3))]
    pts = np.concatenate(c)[rng.permutation(1080)]
    d["cloud"] = pts
    for ms in (1, 3):
        _, keep = ref_tool.find_biggest_cluster(pts, eps=0.06, min_samples=ms)
        d[f"keep_ms{ms}"] = keep
    t, sc, keep = ref_tool.compute_translation_scales(pts, eps=0.06, min_samples=1)
    d["translation"], d["sc_factor"], d["keep_ts"] = t, np.array([sc]), keep
    # optimised poses back to the real world
    poses = np.stack([np.eye(4) for _ in range(5)])
    for i in range(5):
        a = rng.normal(size=3) * 0.3
        Kx = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        th = np.linalg.norm(a)
        poses[i, :3, :3] = np.eye(3) + np.sin(th) / th * Kx + (1 - np.cos(th)) / th ** 2 * Kx @ Kx
        poses[i, :3, 3] = rng.normal(size=3) * 0.5
    pa = ref_helpers.PoseArray(5, max_trans=0.02 * 6.6, max_rot=20)
    pa.data.data = torch.from_numpy(rng.normal(size=(5, 6)).astype(np.float32) * 0.3)
    opt, off = ref_utils.get_optimized_poses_in_real_world(poses, pa, 6.6, np.array([0.01, -0.02, 0.03]))
    d["poses"], d["pose_data"], d["opt_poses"], d["offset"] = poses, pa.data.data.numpy(), opt, off
    np.savez_compressed(os.path.join(OUT, "handoff.npz"), **d)
    print("handoff: biggest cluster sizes", int(d["keep_ms1"].sum()), int(d["keep_ms3"].sum()))


# ---------------------------------------------------------------------------
# G7: the trainer's seeding and batch order — the reference's own
# NerfRunner.__init__ (set_seed(0), build_octree, create_nerf, create_optimizer,
# make_frame_rays, the denoise, DataLoader's CPU randperm), NerfRunner.train()
# (set_seed(0) + next(data_loader) per step; train_loop replaced by a recorder of
# the batch ids: on a GPU the step consumes no CPU random numbers) and the call
# bundlesdf.py:223 makes, add_new_frames(..., new_pcd=, reuse_weights=False),
# followed by train() again — executed from /root/reference on CPU. kaolin's
# OctreeManager is the dense occupancy of the reference's own dilated, quantised
# points with the oracle trace; open3d's voxel_down_sample and cv2.dilate are the
# oracle restatements. Stored: initial parameters (both rounds), pool sizes, every
# step's batch ids, the octree build cloud after the hand-off.
# ---------------------------------------------------------------------------
G7_SEQ = dict(n_frames=5, seed=4, n_init=3)
G7_CFG = dict(down_scale_ratio=4, N_rand=1100, n_step=24, frame_features=2, num_levels=4, log2_hashmap_size=11,
              finest_res=32, amp=True, save_octree_clouds=False, save_dir="/tmp")


def g7_clouds(seq):
    """(initial octree build cloud, the cloud handed over with the new frames) in normalised space."""
    pts = seq["octree_pts"]
    rng = np.random.default_rng(7)
    new = pts[rng.permutation(len(pts))[:25000]] + rng.normal(0, 0.002, (25000, 3))
    return pts, new


def gen_runner_seed(ref_helpers, ref_runner):
    K, _ = _install_oracle_extensions()
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.octree import OctreeManager as DenseOctree
    from oracle import ray_pool as RP
    from oracle import scene_bounds as SB
    torch.Tensor.cuda = lambda self, *a, **k: self
    sys.modules["cv2"].dilate = lambda m, kernel, iterations=1: RP.dilate(m, kernel.shape[0])
    ref_runner.cv2 = sys.modules["cv2"]

    class _Octree:   # kaolin SPC stand-in (Utils.OctreeManager(pts, max_level))
        def __init__(self, pts, max_level):
            self.dense = DenseOctree(pts.float(), max_level)          # quantised points, no further dilation

        def ray_trace(self, rays_o, rays_d, level, debug=False):
            return _OracleOctree(K, self.dense.occupancy(level).numpy()).ray_trace(rays_o, rays_d, level)

    class _Pcd:      # open3d PointCloud stand-in: .points, voxel_down_sample (oracle restatement)
        def __init__(self, pts):
            self.points = np.asarray(pts, np.float64)

        def voxel_down_sample(self, v):
            return _Pcd(SB.voxel_down_sample(self.points, None, v)[0])

    ref_runner.OctreeManager = _Octree
    ref_runner.NerfRunner.create_nerf.__defaults__ = (torch.device("cpu"),)
    seq = SY.make_sequence(G7_SEQ["n_frames"], seed=G7_SEQ["seed"])
    import yaml
    with open(os.path.join(REF, "config.yml")) as f:
        cfg = yaml.safe_load(f)
    cfg.update(sc_factor=seq["sc_factor"], translation=seq["translation"].tolist(), **G7_CFG)
    n0 = G7_SEQ["n_init"]
    cloud0, cloud1 = g7_clouds(seq)
    ids_log = []

    def record(self, batch):
        ids_log.append(self.data_loader.batch_ray_ids.numpy().astype(np.int32).copy())
    ref_runner.NerfRunner.train_loop = record

    def state(r):
        m = r.models
        d = {"embeddings": m["embed_fn"].embeddings.detach().numpy().copy(),
             "pose": m["pose_array"].data.detach().numpy().copy(),
             "features": m["feature_array"].data.detach().numpy().copy()}
        d.update({k: v.detach().numpy().copy() for k, v in m["model"].state_dict().items()})
        return d
    runner = ref_runner.NerfRunner(dict(cfg), seq["rgbs"][:n0], seq["depths"][:n0], seq["masks"][:n0], None,
                                   seq["poses"][:n0], seq["K"], build_octree_pcd=_Pcd(cloud0))
    d = {f"r0_{k}": v for k, v in state(runner).items()}
    d["r0_pool"] = np.array([len(runner.rays)])
    d["r0_perm_head"] = runner.data_loader.ids[:2048].numpy().astype(np.int32)
    runner.train()
    d["r0_ids"] = np.stack(ids_log)
    ids_log.clear()
    runner.add_new_frames(seq["rgbs"][n0:], seq["depths"][n0:], seq["masks"][n0:], None, seq["poses"], occ_masks=None,
                          new_pcd=_Pcd(cloud1), reuse_weights=False)
    d.update({f"r1_{k}": v for k, v in state(runner).items()})
    d["r1_pool"] = np.array([len(runner.rays)])
    bp = np.ascontiguousarray(runner.build_octree_pts, np.float64)
    import hashlib
    d["r1_octree_n"] = np.array([len(bp)])
    d["r1_octree_sha"] = np.array(hashlib.sha256(bp.tobytes()).hexdigest())
    d["r1_octree_head"] = bp[:64]
    runner.train()
    d["r1_ids"] = np.stack(ids_log)
    d["inputs_checksum"] = np.array([float(np.sum(seq["rgbs"], dtype=np.float64)),
                                     float(np.sum(seq["depths"], dtype=np.float64)),
                                     float(np.sum(seq["masks"], dtype=np.float64))])
    d["cfg_json"] = np.array(json.dumps(cfg))
    d["seq_json"] = np.array(json.dumps(G7_SEQ))
    np.savez_compressed(os.path.join(OUT, "runner_seed.npz"), **d)
    print("runner_seed: pools", int(d["r0_pool"][0]), int(d["r1_pool"][0]), "ids", d["r0_ids"].shape)


def main():
    ref_grid, ref_helpers, ref_runner = _import_reference()
    only = set(sys.argv[1:])                  # e.g. `make_golden.py ray_pool` regenerates one fixture
    gens = [("grid_layout", lambda: gen_grid_layout(ref_grid)),
            ("render_loss", lambda: gen_render_loss(ref_helpers, ref_runner)),
            ("mlp", lambda: gen_mlp(ref_helpers)),
            ("helpers", lambda: gen_sh_and_samplers(ref_helpers, ref_runner)),
            ("train_step", lambda: gen_train_step(ref_helpers, ref_runner)),
            ("train_step_amp", lambda: gen_train_step(ref_helpers, ref_runner, amp=True)),
            ("ray_pool", lambda: gen_ray_pool(ref_helpers, ref_runner)),
            ("handoff", lambda: gen_handoff(ref_helpers, ref_runner)),
            ("runner_seed", lambda: gen_runner_seed(ref_helpers, ref_runner))]
    for name, fn in gens:
        if not only or name in only:
            fn()
    print("golden fixtures written to", OUT)


if __name__ == "__main__":
    main()
