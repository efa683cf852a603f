"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(), bench.py
cpu_baseline). CPU fp32 restatement of one BundleSDF NeRF training step:

  NerfRunner.train_loop        nerf_runner.py:677-762
    render_rays                 :1013-1128   (N_importance = 0 path)
    sample_rays_uniform_occupied_voxels :979-1010
    sample_rays_uniform         :67-87
    run_network                 :1226-1303
    raw2outputs                 :1131-1168
    get_sdf_loss / get_masks    nerf_helpers.py:367-399
    PoseArray.get_matrices      nerf_helpers.py:143-154
    NeRFSmall                   nerf_helpers.py:243-321
    SHEncoder (degree 3)        nerf_helpers.py:22-105
    Adam(eps=1e-15)             nerf_runner.py:490-502
  with the kernels of oracle/kernels.py (grid encoder, samplers, ray trace).

amp=True restates the reference's autocast step (nerf_runner.py:159,685-760,
grid.py:50-51): the hash table read as fp16 with the reference kernel's fp16
accumulation (grid_oracle.c half mode; the fp16 table-gradient terms are summed
in fp32, the order-free value the reference's __half2 atomics approximate), every
nn.Linear with fp16 inputs / weights / outputs and fp32 accumulation (its
backward rounds dX / dW to fp16), the loss scaled by the GradScaler scale before
the backward and the gradients unscaled after it.

Randomness is injected: t_rand [R, N_samples + N_samples_around_depth] holds
the stratification draws ([:, :N] for the octree samples, [:, N:] for the
around-depth samples of valid-depth rays or the octree samples of
invalid-depth rays) — the three torch.rand calls of render_rays.
The pose correction uses the restated se3_exp_map (pytorch3d not installed:
parity unpinned at non-identity poses)."""
import numpy as np
import torch

from . import kernels as K

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]


def linspace01(n):
    """torch.linspace(0,1,n) in float32 (symmetric two-sided formula)."""
    return torch.linspace(0.0, 1.0, steps=n, dtype=torch.float32)


def sample_rays_uniform(N, near, far, t_rand, perturb=True):
    """nerf_runner.py:67-87 with injected t_rand."""
    t = linspace01(N).reshape(1, -1)
    z = near * (1. - t) + far * t
    if perturb:
        mids = .5 * (z[..., 1:] + z[..., :-1])
        upper = torch.cat([mids, z[..., -1:]], -1)
        lower = torch.cat([z[..., :1], mids], -1)
        z = lower + (upper - lower) * t_rand
        z = torch.clip(z, near, far)
    return z


def _hat(v):
    x, y, z = v.unbind(-1)
    o = torch.zeros_like(x)
    return torch.stack([o, -z, y, z, o, -x, -y, x, o], -1).view(*v.shape[:-1], 3, 3)


def se3_exp_map(log_transform, eps=1e-4):
    """pytorch3d.transforms.se3_exp_map (published algorithm; row-vector convention)."""
    t, w = log_transform[..., :3], log_transform[..., 3:6]
    ang = torch.clamp((w * w).sum(-1), eps).sqrt()
    inv = 1.0 / ang
    fac1 = inv * ang.sin()
    fac2 = inv * inv * (1.0 - ang.cos())
    Kh = _hat(w)
    K2 = Kh @ Kh
    eye = torch.eye(3, dtype=log_transform.dtype)
    R = fac1[..., None, None] * Kh + fac2[..., None, None] * K2 + eye
    V = eye + Kh * ((1 - torch.cos(ang)) / ang ** 2)[..., None, None] + K2 * ((ang - torch.sin(ang)) / ang ** 3)[
        ..., None, None]
    T = (V @ t[..., None])[..., 0]
    out = torch.zeros((*log_transform.shape[:-1], 4, 4), dtype=log_transform.dtype)
    out[..., :3, :3] = R
    out[..., 3, :3] = T
    out[..., 3, 3] = 1.0
    return out


def pose_matrices(pose_data, ids, max_trans, max_rot):
    """PoseArray.get_matrices (nerf_helpers.py:143-154)."""
    theta = torch.tanh(pose_data)
    trans = theta[:, :3] * max_trans
    rot = theta[:, 3:6] * max_rot / 180.0 * np.pi
    Ts_data = se3_exp_map(torch.cat((trans, rot), dim=-1)).permute(0, 2, 1)
    Ts = torch.eye(4).reshape(1, 4, 4).repeat(len(ids), 1, 1)
    mask = ids != 0
    Ts[mask] = Ts_data[ids[mask]]
    return Ts


def sh3(d):
    """SHEncoder(degree=3) forward."""
    x, y, z = d.unbind(-1)
    xx, yy, zz = x * x, y * y, z * z
    return torch.stack([torch.full_like(x, SH_C0), -SH_C1 * y, SH_C1 * z, -SH_C1 * x, SH_C2[0] * (x * y),
                        SH_C2[1] * (y * z), SH_C2[2] * (2.0 * zz - xx - yy), SH_C2[3] * (x * z),
                        SH_C2[4] * (xx - yy)], -1)


class _GridFn(torch.autograd.Function):
    """grid.py:31-99 over the C oracle: fp32, or (half=True) the autocast path —
    the fp16 table copy, fp16 outputs / dy_dx / gradients (gridencoder.cu in half)."""

    @staticmethod
    def forward(ctx, x01, emb, offsets, S, H, half=False, fp16_accum=False):
        e = emb.detach().numpy()
        if half:
            e = e.astype(np.float16)
        out, dydx = K.grid_encode_forward(x01.detach().numpy(), e, offsets, S, H, calc_grad_inputs=True)
        L, B, C = out.shape
        ctx.save_for_backward(x01)
        ctx.dydx, ctx.offsets, ctx.S, ctx.H, ctx.nrows, ctx.half = dydx, offsets, S, H, emb.shape[0], half
        ctx.fp16_accum = fp16_accum
        return torch.from_numpy(out.astype(np.float32)).permute(1, 0, 2).reshape(B, L * C)

    @staticmethod
    def backward(ctx, g):
        (x01,) = ctx.saved_tensors
        B = x01.shape[0]
        L = len(ctx.offsets) - 1
        C = g.shape[1] // L
        gl = g.view(B, L, C).permute(1, 0, 2).contiguous().numpy()
        dydx = ctx.dydx
        if ctx.half and ctx.fp16_accum:
            # the reference kernel's own rounding: every sample-corner term added into the fp16
            # table gradient (and the input gradient) one by one, here in serial order
            # (gridencoder.cu:319-327 with its atomics serialised; grid_oracle.c half mode)
            gemb, gin = K.grid_encode_backward(gl.astype(np.float16), x01.detach().numpy(), ctx.offsets, ctx.nrows,
                                               ctx.S, ctx.H, calc_grad_inputs=True, dy_dx=dydx)
            return (torch.from_numpy(gin.astype(np.float32)), torch.from_numpy(gemb.astype(np.float32)), None, None,
                    None, None, None)
        if ctx.half:
            # autocast hands the encoder dL/dfeature in fp16; the reference then adds each
            # sample's terms into the fp16 table gradient with __half2 atomics, whose result
            # depends on the (unspecified) atomic order — the oracle sums those same fp16
            # terms in fp32 (the order-free value they approximate)
            gl = gl.astype(np.float16).astype(np.float32)
            dydx = dydx.astype(np.float32)
        gemb, gin = K.grid_encode_backward(gl, x01.detach().numpy(), ctx.offsets, ctx.nrows, ctx.S, ctx.H,
                                           calc_grad_inputs=True, dy_dx=dydx)
        return (torch.from_numpy(gin.astype(np.float32)), torch.from_numpy(gemb.astype(np.float32)), None, None, None,
                None, None)


def _h(t):
    """Round to fp16 and back (forward); its autograd rounds the gradient to fp16 too."""
    return t.half().float()


def nerf_small(x, W, amp=False, acts=None):
    """NeRFSmall(num_layers=2, hidden 64, geo 15, colour 3 layers) forward; W = state dict.
    amp: autocast Linear = fp16 operands, fp32 accumulation, fp16 result.
    acts: optional dict, filled with name -> (layer input, layer output) (output keeps its grad) and,
    for the ReLU layers, name + ".relu" -> the ReLU output (keeps its grad: the unmasked gradient)."""
    def relu(y, name):
        r = torch.relu(y)
        if acts is not None and r.requires_grad:
            r.retain_grad()
            acts[name + ".relu"] = r
        return r

    def lin(h, name):
        if amp:
            y = _h(_h(h) @ _h(W[f"{name}.weight"]).t() + _h(W[f"{name}.bias"]))
        else:
            y = h @ W[f"{name}.weight"].t() + W[f"{name}.bias"]
        if acts is not None and y.requires_grad:
            y.retain_grad()
            acts[name] = (h, y)
        return y
    n_in = W["sigma_net.0.weight"].shape[1]
    pts, views = x[:, :n_in], x[:, n_in:]
    h = lin(relu(lin(pts, "sigma_net.0"), "sigma_net.0"), "sigma_net.2")
    sigma, geo = h[:, 0], h[:, 1:]
    c = torch.cat([views, geo], -1)
    c = lin(relu(lin(relu(lin(c, "color_net.0"), "color_net.0"), "color_net.2"), "color_net.2"), "color_net.4")
    return torch.cat([c, sigma[:, None]], -1)


MLP_KEYS = ["sigma_net.0.weight", "sigma_net.0.bias", "sigma_net.2.weight", "sigma_net.2.bias",
            "color_net.0.weight", "color_net.0.bias", "color_net.2.weight", "color_net.2.bias",
            "color_net.4.weight", "color_net.4.bias"]


def truncation(cfg, global_step=0):
    """get_truncation (nerf_runner.py:661-674) at training step global_step."""
    kind = cfg.get("trunc_decay_type", "") or ""
    if kind == "linear":
        t = cfg["trunc_start"] - (cfg["trunc_start"] - cfg["trunc"]) * float(global_step) / cfg["n_step"]
    elif kind == "exp":
        lamb = np.log(cfg["trunc"] / cfg["trunc_start"]) / (cfg["n_step"] / 4)
        t = max(cfg["trunc_start"] * np.exp(global_step * lamb), cfg["trunc"])
    else:
        t = cfg["trunc"]
    return float(t) * cfg["sc_factor"]


def trace_and_sample(batch, tf, occ, cfg, t_rand, kmax=None, trunc=None):
    """render_rays :1043-1080 up to z_vals (no grad). batch [R,12] reference columns.
    Returns z_vals [R, N+N_around] and the per-ray z_in_out intervals."""
    with torch.no_grad():
        sc = cfg["sc_factor"]
        R = batch.shape[0]
        N, Na = cfg["N_samples"], cfg["N_samples_around_depth"]
        rays_d = batch[:, 0:3]
        viewdirs = rays_d / rays_d.norm(dim=-1, keepdim=True)
        rays_o_w = tf[:, :3, 3]
        viewdirs_w = (tf[:, :3, :3] @ viewdirs[:, :, None])[:, :, 0]
        nres = occ.shape[0]
        kb = 3 * nres if kmax is None else kmax
        dio, counts = K.octree_ray_trace(occ, rays_o_w.numpy(), viewdirs_w.numpy(), kb)
        k = max(1, int(counts.max()))
        dio = torch.from_numpy(dio[:, :k].copy())
        depth = batch[:, 6]
        trunc = truncation(cfg) if trunc is None else trunc

        def occupied(dio_sub, vdirs, depths, n, tr):
            z_in_out = dio_sub * torch.abs(vdirs[:, 2]).reshape(-1, 1, 1)
            if depths is not None:
                d = depths.reshape(-1, 1)
                valid = (d >= cfg["near"] * sc) & (d <= cfg["far"] * sc).expand(-1, z_in_out.shape[1])
                valid = valid & (z_in_out > 0).all(dim=-1)
                hi = (d.reshape(-1, 1, 1).expand(-1, z_in_out.shape[1], 2)[valid] + trunc)
                z_in_out[valid] = torch.clip(z_in_out[valid], min=torch.zeros_like(z_in_out[valid]), max=hi)
            lens = z_in_out[:, :, 1] - z_in_out[:, :, 0]
            total = _seqsum(lens)
            zc = sample_rays_uniform(n, torch.zeros_like(total).reshape(-1, 1), total.reshape(-1, 1), tr)
            zv, err = K.sample_occupied(z_in_out.numpy(), zc.numpy())
            assert err == 0, "sampler error"
            return torch.from_numpy(zv)

        z = occupied(dio, viewdirs, depth, N, t_rand[:, :N])
        vmask = (depth >= cfg["near"] * sc) & (depth <= cfg["far"] * sc)
        za = torch.zeros((R, Na))
        if vmask.any():
            za[vmask] = sample_rays_uniform(Na, (depth[vmask] - trunc).reshape(-1, 1),
                                            (depth[vmask] + trunc * cfg["neg_trunc_ratio"]).reshape(-1, 1),
                                            t_rand[vmask, N:])
        inv = ~vmask
        if inv.any():
            za[inv] = occupied(dio[inv], viewdirs[inv], None, Na, t_rand[inv, N:])
        return torch.cat([z, za], -1), dio


def _seqsum(lens):
    """Row sums accumulated left to right in float32 (the HIP kernel's order)."""
    acc = torch.zeros(lens.shape[0], dtype=torch.float32)
    for k in range(lens.shape[1]):
        acc = acc + lens[:, k]
    return acc


def train_step(params, batch, c2w, occ, cfg, t_rand, grid_meta, step=0, lr=None, adam_state=None, kmax=None,
               amp=False, loss_scale=65536.0, mask_from=None, fp16_table_accum=False):
    """One train_loop iteration. params: dict with 'embeddings' [T,C], MLP_KEYS, 'pose' [F,6]
    and, for cfg frame_features > 0, 'features' [F, frame_features] (FeatureArray.data).
    `step` is the round's global_step (truncation schedule, Adam bias correction).
    amp: the autocast / GradScaler step (module docstring); the returned grads are unscaled.
    fp16_table_accum (amp): sum the table / input gradient in fp16 term by term in serial order, the
    reference kernel's rounding as G4-amp ran it (tests/golden/train_step_amp.npz), instead of the
    order-free fp32 sum of the same fp16 terms (the default, what the GPU parity tests compare with).
    mask_from (test infrastructure): (z [R,S], sdf [R,S]) of another implementation of the
    step — the discontinuous loss / compositing masks (the |z - d| band, front / back,
    sdf < fs_sdf, sdf < 1) are taken from THOSE values while every loss value and gradient
    is computed from this step's own z and sdf, so a sample whose rounding put it on the
    other side of a threshold there is evaluated on the same branch here (the parity tests
    count and bound such samples instead of searching for inputs without one).
    Returns dict of losses, intermediates, grads and updated params."""
    sc = cfg["sc_factor"]
    P = {k: v.detach().clone().float().requires_grad_(True) for k, v in params.items()}
    R = batch.shape[0]
    frame_ids = batch[:, 8].long()
    max_trans = cfg["max_trans"] * sc
    poses = pose_matrices(P["pose"], frame_ids, max_trans, cfg["max_rot"])
    tf = poses @ c2w[frame_ids]
    trunc = truncation(cfg, step)
    z, z_in_out = trace_and_sample(batch, tf.detach(), occ, cfg, t_rand, kmax, trunc)
    S = z.shape[1]
    rays_d = batch[:, 0:3]
    viewdirs = rays_d / rays_d.norm(dim=-1, keepdim=True)
    pts = rays_d[:, None, :] * z[:, :, None]
    tf_flat = tf[:, None].expand(-1, S, -1, -1).reshape(-1, 4, 4)
    x = (tf_flat[:, :3, :3] @ pts.reshape(-1, 3)[:, :, None] + tf_flat[:, :3, 3:])[:, :, 0]
    valid = (torch.abs(x) <= 1).all(dim=-1).view(R, S)
    offsets, S_log, H = grid_meta
    emb_out = torch.zeros((R * S, (len(offsets) - 1) * P["embeddings"].shape[1]))
    vflat = valid.reshape(-1)
    x01 = (x[vflat] + 1) / 2
    emb_out[vflat] = _GridFn.apply(x01, P["embeddings"], offsets, S_log, H, amp, fp16_table_accum)
    emb_out.retain_grad()
    input_dirs = (tf[:, :3, :3] @ viewdirs[:, :, None])[:, :, 0]
    sh = sh3(input_dirs)
    parts = [emb_out]
    if "features" in P:   # FeatureArray latent code per frame (nerf_runner.py:1268-1277), before the SH dirs
        ff = P["features"][frame_ids]
        parts.append(ff[:, None].expand(-1, S, -1).reshape(R * S, -1))
    parts.append(sh[:, None].expand(-1, S, -1).reshape(R * S, -1))
    feat = torch.cat(parts, -1)
    acts = {}
    raw = nerf_small(feat, P, amp, acts).view(R, S, 4)
    depth = batch[:, 6]
    # raw2outputs (:1131-1168)
    d = depth.view(-1, 1)
    zm, sm = (z, raw[..., 3].detach()) if mask_from is None else (torch.as_tensor(mask_from[0]).float(),
                                                                    torch.as_tensor(mask_from[1]).float())
    u = (d - z) / trunc
    w = torch.sigmoid(u * cfg["sdf_lambda"]) * torch.sigmoid(-u * cfg["sdf_lambda"])
    invalid = (d > cfg["far"] * sc).reshape(-1)
    m = (zm - d <= trunc * cfg["neg_trunc_ratio"]) & (zm - d >= -trunc)
    w = torch.where(invalid[:, None], torch.zeros_like(w), w * m)
    w = w / (w.sum(dim=-1, keepdim=True) + 1e-10)
    w = w * valid
    rgb_map = torch.sum(w[..., None] * torch.sigmoid(raw[..., :3]), -2)
    # train_loop losses (:687-751)
    sdf = raw[..., 3]
    ray_type = batch[:, 9]
    valid_rays = valid.any(dim=-1) & (ray_type == 0)
    rw = torch.ones(R)
    rw[frame_ids == 0] = cfg["first_frame_weight"]
    rw = rw * valid_rays
    sw = rw.view(R, 1).expand(-1, S) * valid
    sw = torch.where((ray_type == 1)[:, None], torch.zeros_like(sw), sw)
    rgb_loss = cfg["rgb_weight"] * ((rgb_map - batch[:, 3:6]) ** 2 * rw.view(-1, 1)).mean()
    td = d.expand(-1, S)
    front = zm < td - trunc
    back = zm > td + trunc * cfg["neg_trunc_ratio"]
    vdm = (td >= cfg["near"] * sc) & (td <= cfg["far"] * sc)
    sdfm = (1.0 - front.float()) * (1.0 - back.float()) * vdm
    fsm = (td > cfg["far"] * sc) & (sm < cfg["fs_sdf"])
    fs = torch.mean(((sdf - cfg["fs_sdf"]) * fsm) ** 2 * sw) * 0.5
    em = front & (td <= cfg["far"] * sc) & (sm < 1)
    empty = torch.mean(torch.abs(sdf - 1) * em * sw) * cfg["empty_weight"]
    fs_loss = (fs + empty) * cfg["fs_weight"]
    sdf_loss = torch.mean(((z + sdf * trunc) * sdfm - td * sdfm) ** 2 * sw) * 0.5 * cfg["trunc_weight"]
    loss = rgb_loss + fs_loss + sdf_loss
    fs_rgb_loss = torch.zeros(())
    if cfg.get("fs_rgb_weight", 0) > 0:   # train_loop :728-731 (front_mask of get_masks, sample weights)
        fs_rgb_loss = ((((torch.sigmoid(raw[..., :3]) - 1) * front[..., None]) ** 2) * sw[..., None]).mean()
        loss = loss + fs_rgb_loss * cfg["fs_rgb_weight"]
    reg_features = torch.zeros(())
    if "features" in P:   # feature_reg_weight * mean(data^2) (nerf_runner.py:743-746)
        reg_features = cfg.get("feature_reg_weight", 0.1) * (P["features"] ** 2).mean()
        loss = loss + reg_features
    pose_reg = torch.zeros(())
    if cfg.get("pose_reg_weight", 0):   # pose_reg_weight * ||pose_array.data[1:]|| (nerf_runner.py:748-751)
        pose_reg = cfg["pose_reg_weight"] * P["pose"][1:].norm()
        loss = loss + pose_reg
    (loss * loss_scale if amp else loss).backward()
    grads = {k: v.grad.detach().clone() if v.grad is not None else torch.zeros_like(v) for k, v in P.items()}
    if amp:
        grads = {k: v / loss_scale for k, v in grads.items()}
    # conditioning of each table-gradient entry: the sum of the absolute values of the terms
    # it is accumulated from (sum over samples and corners of w |dL/dfeature|), in fp32 —
    # the scale of the summation-order (and fp16 accumulation) error any implementation has
    g_emb_abs = g_emb_dpos = None
    if emb_out.grad is not None and bool(vflat.any()):
        d = emb_out.grad[vflat].abs() / (loss_scale if amp else 1.0)
        if amp and "sigma_net.0" in acts and acts["sigma_net.0"][1].grad is not None:
            # fp16 dL/dfeature = W1^T dH1 rounded from fp16 operands: its noise follows the
            # absolute GEMM |dH1| |W1| (one fp16 unit of it, 2^-11, doubled), not |dL/dfeature|
            n1 = acts["sigma_net.0"][1].grad.detach().abs() @ P["sigma_net.0.weight"].detach().abs()
            d = d + 2.0 ** -10 * n1[vflat] / loss_scale
        ga, gd = table_sensitivity(x01.detach().numpy(), d.numpy(), offsets, S_log, H, P["embeddings"].shape[0])
        g_emb_abs, g_emb_dpos = torch.from_numpy(ga), torch.from_numpy(gd)
    g_mlp_kink, e_x = _mlp_kink(acts, P, amp, loss_scale)
    g_emb_kink = None
    if e_x is not None and bool(vflat.any()):
        gk, _ = table_sensitivity(x01.detach().numpy(), e_x[vflat].numpy(), offsets, S_log, H,
                                  P["embeddings"].shape[0])
        g_emb_kink = torch.from_numpy(gk)
    out = dict(loss=loss.item(), rgb_loss=rgb_loss.item(), fs_loss=fs_loss.item(), sdf_loss=sdf_loss.item(),
               reg_features=reg_features.item(), pose_reg=pose_reg.item(), fs_rgb_loss=fs_rgb_loss.item(),
               z_vals=z.detach(), valid=valid, raw=raw.detach(), rgb_map=rgb_map.detach(), weights=w.detach(),
               d_feat=None if emb_out.grad is None else emb_out.grad.detach() / (loss_scale if amp else 1.0),
               g_emb_abs=g_emb_abs, g_emb_dpos=g_emb_dpos, g_mlp_abs=_mlp_abs(acts, amp, loss_scale),
               g_mlp_kink=g_mlp_kink, g_emb_kink=g_emb_kink,
               grads=grads, tf=tf.detach())
    if lr is not None:
        out["params"], out["adam_state"] = adam_step(params, grads, adam_state, step, lr)
    return out


def loss_terms_f64(batch, z, raw, valid, cfg, trunc):
    """The train_loop losses (nerf_runner.py:687-731, raw2outputs :1131-1168, get_sdf_loss
    nerf_helpers.py:367-399) recomputed in float64 from another implementation's per-sample
    forward records — z [R,S], raw [R,S,4], valid [R,S] — on the device they live on. Returns
    the float64 rgb / fs (free-space + empty) / sdf losses and the composited rgb [R,3]; a check
    of how that implementation reduced its records into the step's loss, at any batch size."""
    f = torch.float64
    z, raw, batch = z.to(f), raw.to(f), batch.to(f)
    valid = valid.bool()
    sc = cfg["sc_factor"]
    R, S = z.shape
    d = batch[:, 6:7]
    u = (d - z) / trunc
    w = torch.sigmoid(u * cfg["sdf_lambda"]) * torch.sigmoid(-u * cfg["sdf_lambda"])
    m = (z - d <= trunc * cfg["neg_trunc_ratio"]) & (z - d >= -trunc)
    w = torch.where((d > cfg["far"] * sc), torch.zeros_like(w), w * m)
    w = w / (w.sum(-1, keepdim=True) + 1e-10) * valid
    rgb = (w[..., None] * torch.sigmoid(raw[..., :3])).sum(-2)
    frame_ids, ray_type = batch[:, 8], batch[:, 9]
    rw = torch.where(frame_ids == 0, torch.full_like(frame_ids, cfg["first_frame_weight"]), torch.ones_like(frame_ids))
    rw = rw * (valid.any(-1) & (ray_type == 0))
    sw = rw[:, None] * valid
    sw = torch.where((ray_type == 1)[:, None], torch.zeros_like(sw), sw)
    rgb_loss = cfg["rgb_weight"] * ((rgb - batch[:, 3:6]) ** 2 * rw[:, None]).mean()
    sdf = raw[..., 3]
    front = z < d - trunc
    back = z > d + trunc * cfg["neg_trunc_ratio"]
    vdm = (d >= cfg["near"] * sc) & (d <= cfg["far"] * sc)
    sdfm = (~front) & (~back) & vdm
    fsm = (d > cfg["far"] * sc) & (sdf < cfg["fs_sdf"])
    fs = (((sdf - cfg["fs_sdf"]) * fsm) ** 2 * sw).mean() * 0.5
    em = front & (d <= cfg["far"] * sc) & (sdf < 1)
    empty = ((sdf - 1).abs() * em * sw).mean() * cfg["empty_weight"]
    sdf_loss = ((((z + sdf * trunc) - d) * sdfm) ** 2 * sw).mean() * 0.5 * cfg["trunc_weight"]
    return dict(rgb_loss=float(rgb_loss), fs_loss=float((fs + empty) * cfg["fs_weight"]), sdf_loss=float(sdf_loss),
                rgb=rgb)


KINK_REL = {True: 2.0 ** -9, False: 2.0 ** -20}


def _mlp_kink(acts, W, amp, loss_scale):
    """ReLU-kink conditioning of the MLP and table gradients (test tolerances, not part of the
    reference step). A sample whose pre-activation y of a ReLU unit lies within rounding distance
    of the kink — |y| <= c (|W| |x| + |b|) for that unit, c = 2^-9 in amp (two implementations'
    layer inputs differ by up to an fp16 ulp, 2^-11 relative) and 2^-20 in fp32 — can take the
    other side of it in another implementation, which then adds or drops that sample's whole term
    of the unit's gradient (ReLU backward passes all or nothing). Returns (K, E_x): K[param] bounds
    the resulting change of each MLP parameter-gradient entry — the flippable samples' unmasked
    terms |dL/dh| |x|, propagated to the earlier layers through |W| — and E_x [samples, n_in] the
    change of each sample's dL/dfeature (for the table's bound, through table_sensitivity)."""
    if not acts or "color_net.4" not in acts:
        return {}, None
    c = KINK_REL[bool(amp)]
    sc = loss_scale if amp else 1.0
    K = {}

    def wabs(name):
        return W[f"{name}.weight"].detach().abs()

    def flippable(name):
        x, y = acts[name]
        r = acts.get(name + ".relu")
        if r is None or r.grad is None:
            return 0.0
        delta = c * (x.detach().abs() @ wabs(name).t() + W[f"{name}.bias"].detach().abs())
        return r.grad.detach().abs() / sc * (y.detach().abs() <= delta)

    def add(name, E):
        K[f"{name}.weight"] = E.t() @ acts[name][0].detach().abs()
        K[f"{name}.bias"] = E.sum(0)
        return E @ wabs(name)          # bound on the change of dL/d(the layer's input)

    n = acts["color_net.4"][0].shape[0]
    e = add("color_net.4", torch.zeros(n, acts["color_net.4"][1].shape[1]))
    e = add("color_net.2", e + flippable("color_net.2"))
    e = add("color_net.0", e + flippable("color_net.0"))
    n_geo = acts["sigma_net.2"][1].shape[1] - 1        # cat([views, geo]): geo are the last columns
    e = add("sigma_net.2", torch.cat([torch.zeros(n, 1), e[:, -n_geo:]], 1))
    e = add("sigma_net.0", e + flippable("sigma_net.0"))
    return K, e


def _mlp_abs(acts, amp, loss_scale):
    """Conditioning of the MLP weight / bias gradients: |dL/dy|^T |x| and sum |dL/dy| per
    layer — the absolute sums of the terms each gradient entry accumulates."""
    out = {}
    for name, hy in acts.items():
        if name.endswith(".relu"):
            continue
        h, y = hy
        if y.grad is None:
            continue
        gy = y.grad.detach().abs() / (loss_scale if amp else 1.0)
        out[f"{name}.weight"] = gy.t() @ h.detach().abs()
        out[f"{name}.bias"] = gy.sum(0)
    return out


def table_sensitivity(x01, g_abs, offsets, S, H, n_rows):
    """Conditioning of each table-gradient entry (test tolerances, not part of the
    reference step): for samples at x01 [B,3] with |dL/dfeature| g_abs [B, L*C],
      A[row, c] = sum over samples / corners of w |g_c|            (the terms' absolute sum)
      D[row, c] = sum over samples / corners of |grad_x01 w|_1 |g_c| (its sensitivity to the
                  sample position: a position perturbed by dx moves the entry by <= D dx)
    with the kernel_grid corner rows and trilinear weights (gridencoder.cu:46-83,160-195)."""
    x01 = np.asarray(x01, np.float32)
    B = x01.shape[0]
    L = len(offsets) - 1
    C = g_abs.shape[1] // L
    g = np.asarray(g_abs, np.float64).reshape(B, L, C)
    scales, res = K.level_params(L, S, H)
    A = np.zeros((n_rows, C))
    Dp = np.zeros((n_rows, C))
    primes = np.array([1, 2654435761, 805459861], np.uint64)
    for lv in range(L):
        T = int(offsets[lv + 1] - offsets[lv])
        pos = (x01 * scales[lv] + np.float32(0.5)).astype(np.float32)
        pg = np.floor(pos).astype(np.int64)
        f = (pos - pg).astype(np.float64)
        rs = int(res[lv]) + 1
        dense = rs ** 3 <= T
        for idx in range(8):
            bits = [(idx >> d) & 1 for d in range(3)]
            fac = np.stack([f[:, d] if bits[d] else 1 - f[:, d] for d in range(3)], 1)
            w = fac.prod(1)
            dw = sum(np.prod(np.delete(fac, d, axis=1), axis=1) for d in range(3)) * float(scales[lv])
            pl = pg + np.array(bits)
            if dense:
                row = pl[:, 0] + pl[:, 1] * rs + pl[:, 2] * rs * rs
            else:
                h = np.zeros(B, np.uint64)
                for d in range(3):
                    h ^= (pl[:, d].astype(np.uint64) * primes[d]) & np.uint64(0xFFFFFFFF)
                row = h.astype(np.int64)
            row = row % T + int(offsets[lv])
            for c in range(C):
                np.add.at(A[:, c], row, w * g[:, lv, c])
                np.add.at(Dp[:, c], row, dw * g[:, lv, c])
    return A.astype(np.float32), Dp.astype(np.float32)


def adam_step(params, grads, state, step, lr, betas=(0.9, 0.999), eps=1e-15):
    """torch.optim.Adam (single-tensor) update, t = step+1; lr per key (dict) or scalar."""
    state = {} if state is None else state
    new, st = {}, {}
    t = step + 1
    b1, b2 = betas
    for k, p in params.items():
        g = grads[k].float()
        m, v = state.get(k, (torch.zeros_like(p), torch.zeros_like(p)))
        m = m * b1 + g * (1 - b1)
        v = v * b2 + g * g * (1 - b2)
        bc1 = 1 - b1 ** t
        bc2 = 1 - b2 ** t
        lr_k = lr[k] if isinstance(lr, dict) else lr
        step_size = lr_k / bc1
        denom = v.sqrt() / np.sqrt(bc2) + eps
        new[k] = p - step_size * m / denom
        st[k] = (m, v)
    return new, st
