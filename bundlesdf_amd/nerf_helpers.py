"""Torch-level mirror of the reference's nerf_helpers.py (same names,
signatures and semantics), used by the drop-in NerfRunner and by callers that
`from nerf_runner import *` (bundlesdf.py:11 needs preprocess_data).

The hot path of a training step does not run these torch modules: it runs the
fused HIP kernels in libnof (see nerf_runner.py / fused.py), which consume the
parameters these modules own (same parameter names, shapes and init).
"""
import numpy as np
import torch
import torch.nn as nn

BAD_DEPTH = 99      # Utils.py:33
BAD_COLOR = 128     # Utils.py:34

to8b = lambda x: (255 * np.clip(x, 0, 1)).astype(np.uint8)  # noqa: E731  (nerf_helpers.py:18)


class SHEncoder(nn.Module):
    """nerf_helpers.py:22-105 — real spherical harmonics up to `degree` (out_dim = degree^2)."""

    C0 = 0.28209479177387814
    C1 = 0.4886025119029199
    C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
    C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
          1.445305721320277, -0.5900435899266435]
    C4 = [2.5033429417967046, -1.7701307697799304, 0.9461746957575601, -0.6690465435572892, 0.10578554691520431,
          -0.6690465435572892, 0.47308734787878004, -1.7701307697799304, 0.6258357354491761]

    def __init__(self, input_dim=3, degree=4):
        super().__init__()
        assert input_dim == 3 and 1 <= degree <= 5
        self.input_dim = input_dim
        self.degree = degree
        self.out_dim = degree ** 2

    def forward(self, input, **kwargs):
        out = torch.empty((*input.shape[:-1], self.out_dim), dtype=input.dtype, device=input.device)
        x, y, z = input.unbind(-1)
        out[..., 0] = self.C0
        if self.degree > 1:
            out[..., 1] = -self.C1 * y
            out[..., 2] = self.C1 * z
            out[..., 3] = -self.C1 * x
            if self.degree > 2:
                xx, yy, zz = x * x, y * y, z * z
                xy, yz, xz = x * y, y * z, x * z
                out[..., 4] = self.C2[0] * xy
                out[..., 5] = self.C2[1] * yz
                out[..., 6] = self.C2[2] * (2.0 * zz - xx - yy)
                out[..., 7] = self.C2[3] * xz
                out[..., 8] = self.C2[4] * (xx - yy)
                if self.degree > 3:
                    out[..., 9] = self.C3[0] * y * (3 * xx - yy)
                    out[..., 10] = self.C3[1] * xy * z
                    out[..., 11] = self.C3[2] * y * (4 * zz - xx - yy)
                    out[..., 12] = self.C3[3] * z * (2 * zz - 3 * xx - 3 * yy)
                    out[..., 13] = self.C3[4] * x * (4 * zz - xx - yy)
                    out[..., 14] = self.C3[5] * z * (xx - yy)
                    out[..., 15] = self.C3[6] * x * (xx - 3 * yy)
                    if self.degree > 4:
                        out[..., 16] = self.C4[0] * xy * (xx - yy)
                        out[..., 17] = self.C4[1] * yz * (3 * xx - yy)
                        out[..., 18] = self.C4[2] * xy * (7 * zz - 1)
                        out[..., 19] = self.C4[3] * yz * (7 * zz - 3)
                        out[..., 20] = self.C4[4] * (zz * (35 * zz - 30) + 3)
                        out[..., 21] = self.C4[5] * xz * (7 * zz - 3)
                        out[..., 22] = self.C4[6] * (xx - yy) * (7 * zz - 1)
                        out[..., 23] = self.C4[7] * xz * (xx - 3 * yy)
                        out[..., 24] = self.C4[8] * (xx * (xx - 3 * yy) - yy * (3 * xx - yy))
        return out


class FeatureArray(nn.Module):
    """nerf_helpers.py:108-124 — per-frame latent code."""

    def __init__(self, num_frames, num_channels):
        super().__init__()
        self.num_frames = num_frames
        self.num_channels = num_channels
        self.data = nn.parameter.Parameter(torch.normal(0, 1, size=[num_frames, num_channels]).float(),
                                           requires_grad=True)

    def __call__(self, ids):
        return self.data[ids]


def _hat(v):
    x, y, z = v.unbind(-1)
    o = torch.zeros_like(x)
    return torch.stack([o, -z, y, z, o, -x, -y, x, o], -1).view(*v.shape[:-1], 3, 3)


def se3_exp_map(log_transform, eps=1e-4):
    """Restatement of pytorch3d.transforms.se3_exp_map (pytorch3d@stable, pinned by
    docker/dockerfile:79; not installed here — PARITY UNPINNED against the library,
    pinned only at the identity and by SE(3) properties in tests). Row-vector
    convention: rotation in [:3,:3], translation in the last ROW."""
    t = log_transform[..., :3]
    w = log_transform[..., 3:6]
    nrms = (w * w).sum(-1)
    ang = torch.clamp(nrms, eps).sqrt()
    ang_inv = 1.0 / ang
    fac1 = ang_inv * ang.sin()
    fac2 = ang_inv * ang_inv * (1.0 - ang.cos())
    K = _hat(w)
    K2 = K @ K
    eye = torch.eye(3, dtype=log_transform.dtype, device=log_transform.device)
    R = fac1[..., None, None] * K + fac2[..., None, None] * K2 + eye
    V = (eye + K * ((1 - torch.cos(ang)) / (ang ** 2))[..., None, None]
         + K2 * ((ang - torch.sin(ang)) / (ang ** 3))[..., None, None])
    T = (V @ t[..., None])[..., 0]
    out = torch.zeros((*log_transform.shape[:-1], 4, 4), dtype=log_transform.dtype, device=log_transform.device)
    out[..., :3, :3] = R
    out[..., 3, :3] = T
    out[..., 3, 3] = 1.0
    return out


class PoseArray(nn.Module):
    """nerf_helpers.py:127-154 — per-frame pose correction (tanh-bounded se(3))."""

    def __init__(self, num_frames, max_trans, max_rot):
        super().__init__()
        self.num_frames = num_frames
        self.max_trans = max_trans
        self.max_rot = max_rot
        self.data = nn.parameter.Parameter(torch.zeros([num_frames, 6]).float(), requires_grad=True)

    def frame_matrices(self):
        """[F,4,4] corrections for every frame (frame 0 forced identity)."""
        theta = torch.tanh(self.data)
        trans = theta[:, :3] * self.max_trans
        rot = theta[:, 3:6] * self.max_rot / 180.0 * np.pi
        Ts = se3_exp_map(torch.cat((trans, rot), dim=-1)).permute(0, 2, 1)
        eye = torch.eye(4, device=self.data.device, dtype=Ts.dtype)[None]
        first = torch.zeros(self.num_frames, 1, 1, device=self.data.device, dtype=Ts.dtype)
        first[0] = 1
        return first * eye + (1 - first) * Ts

    def get_matrices(self, ids):
        if not torch.is_tensor(ids):
            ids = torch.tensor(ids).long()
        theta = torch.tanh(self.data)
        trans = theta[:, :3] * self.max_trans
        rot = theta[:, 3:6] * self.max_rot / 180.0 * np.pi
        Ts_data = se3_exp_map(torch.cat((trans, rot), dim=-1)).permute(0, 2, 1)
        Ts = torch.eye(4, device=self.data.device).reshape(1, 4, 4).repeat(len(ids), 1, 1)
        mask = ids != 0
        Ts[mask] = Ts_data[ids[mask]]
        return Ts


class Embedder(nn.Module):
    """nerf_helpers.py:157-188 — positional encoding (not used by the default config)."""

    def __init__(self, **kwargs):
        super().__init__()
        self.kwargs = kwargs
        d = kwargs["input_dims"]
        fns, out_dim = [], 0
        if kwargs["include_input"]:
            fns.append(lambda x: x)
            out_dim += d
        max_freq, n = kwargs["max_freq_log2"], kwargs["num_freqs"]
        bands = 2. ** torch.linspace(0., max_freq, steps=n) if kwargs["log_sampling"] else \
            torch.linspace(2. ** 0., 2. ** max_freq, steps=n)
        for freq in bands:
            for p_fn in kwargs["periodic_fns"]:
                fns.append(lambda x, p_fn=p_fn, freq=freq: p_fn(x * freq))
                out_dim += d
        self.embed_fns, self.out_dim = fns, out_dim

    def forward(self, inputs):
        return torch.cat([fn(inputs) for fn in self.embed_fns], -1)


def get_embedder(multires, cfg, i=0, octree_m=None):
    """nerf_helpers.py:191-214."""
    if i == -1:
        return nn.Identity(), 3
    if i == 0:
        embed = Embedder(include_input=True, input_dims=3, max_freq_log2=multires - 1, num_freqs=multires,
                         log_sampling=True, periodic_fns=[torch.sin, torch.cos])
        return embed, embed.out_dim
    if i == 1:
        from .grid import GridEncoder
        embed = GridEncoder(input_dim=3, n_levels=cfg["num_levels"], log2_hashmap_size=cfg["log2_hashmap_size"],
                            desired_resolution=cfg["finest_res"], base_resolution=cfg["base_res"],
                            level_dim=cfg["feature_grid_dim"])
        return embed, embed.out_dim
    if i == 2:
        embed = SHEncoder(degree=cfg["multires_views"])
        return embed, embed.out_dim
    raise ValueError(f"unsupported embedder {i}")


def preprocess_data(rgbs, depths, masks, normal_maps, poses, sc_factor, translation):
    """nerf_helpers.py:218-240."""
    depths[depths < 0.1] = BAD_DEPTH
    if masks is not None:
        rgbs[masks == 0] = BAD_COLOR
        depths[masks == 0] = BAD_DEPTH
        if normal_maps is not None:
            normal_maps[..., [1, 2]] *= -1
            normal_maps[masks == 0] = 0
        masks = masks[..., None]
    rgbs = (rgbs / 255.0).astype(np.float32)
    depths *= sc_factor
    depths = depths[..., None]
    poses[:, :3, 3] += translation
    poses[:, :3, 3] *= sc_factor
    return rgbs, depths, masks, normal_maps, poses


class NeRFSmall(nn.Module):
    """nerf_helpers.py:243-321 — sigma MLP (input_ch -> hidden -> 1+geo) and colour MLP."""

    def __init__(self, num_layers=3, hidden_dim=64, geo_feat_dim=15, num_layers_color=4, hidden_dim_color=64,
                 input_ch=3, input_ch_views=3):
        super().__init__()
        self.input_ch = input_ch
        self.input_ch_views = input_ch_views
        self.num_layers = num_layers
        self.hidden_dim = hidden_dim
        self.geo_feat_dim = geo_feat_dim
        sigma_net = []
        for l in range(num_layers):
            in_dim = self.input_ch if l == 0 else hidden_dim
            out_dim = 1 + self.geo_feat_dim if l == num_layers - 1 else hidden_dim
            sigma_net.append(nn.Linear(in_dim, out_dim, bias=True))
            if l != num_layers - 1:
                sigma_net.append(nn.ReLU(inplace=True))
        self.sigma_net = nn.Sequential(*sigma_net)
        torch.nn.init.constant_(self.sigma_net[-1].bias, 0.1)
        self.num_layers_color = num_layers_color
        self.hidden_dim_color = hidden_dim_color
        color_net = []
        for l in range(num_layers_color):
            in_dim = self.input_ch_views + self.geo_feat_dim if l == 0 else hidden_dim
            out_dim = 3 if l == num_layers_color - 1 else hidden_dim
            color_net.append(nn.Linear(in_dim, out_dim, bias=True))
            if l != num_layers_color - 1:
                color_net.append(nn.ReLU(inplace=True))
        self.color_net = nn.Sequential(*color_net)

    def forward_sdf(self, x):
        h = self.sigma_net(x)
        return h[..., 0]

    def forward(self, x):
        x = x.float()
        input_pts, input_views = torch.split(x, [self.input_ch, self.input_ch_views], dim=-1)
        h = self.sigma_net(input_pts)
        sigma, geo_feat = h[..., 0], h[..., 1:]
        color = self.color_net(torch.cat([input_views, geo_feat], dim=-1))
        return torch.cat([color, sigma.unsqueeze(dim=-1)], -1)


def sample_pdf(bins, weights, N_samples, det=False):
    """nerf_helpers.py:324-354 (hierarchical sampling; dead with N_importance=0)."""
    weights = weights + 1e-5
    pdf = weights / torch.sum(weights, -1, keepdim=True)
    cdf = torch.cumsum(pdf, -1)
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    if det:
        u = torch.linspace(0., 1., steps=N_samples, device=bins.device)
        u = u.expand(list(cdf.shape[:-1]) + [N_samples])
    else:
        u = torch.rand(list(cdf.shape[:-1]) + [N_samples], device=bins.device)
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=True)
    below = torch.max(torch.zeros_like(inds - 1), inds - 1)
    above = torch.min((cdf.shape[-1] - 1) * torch.ones_like(inds), inds)
    inds_g = torch.stack([below, above], -1)
    matched_shape = [inds_g.shape[0], inds_g.shape[1], cdf.shape[-1]]
    cdf_g = torch.gather(cdf.unsqueeze(1).expand(matched_shape), 2, inds_g)
    bins_g = torch.gather(bins.unsqueeze(1).expand(matched_shape), 2, inds_g)
    denom = cdf_g[..., 1] - cdf_g[..., 0]
    denom = torch.where(denom < 1e-5, torch.ones_like(denom), denom)
    t = (u - cdf_g[..., 0]) / denom
    return bins_g[..., 0] + t * (bins_g[..., 1] - bins_g[..., 0])


def get_camera_rays_np(H, W, K):
    """nerf_helpers.py:358-363 — GL-convention camera rays (z = -1)."""
    i, j = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
    return np.stack([(i - K[0, 2]) / K[0, 0], -(j - K[1, 2]) / K[1, 1], -np.ones_like(i)], axis=-1)


def get_masks(z_vals, target_d, truncation, cfg, dir_norm=None):
    """nerf_helpers.py:367-379."""
    valid_depth_mask = (target_d >= cfg["near"] * cfg["sc_factor"]) & (target_d <= cfg["far"] * cfg["sc_factor"])
    front_mask = z_vals < target_d - truncation
    back_mask = z_vals > target_d + truncation * cfg["neg_trunc_ratio"]
    sdf_mask = (1.0 - front_mask.float()) * (1.0 - back_mask.float()) * valid_depth_mask
    fs_weight = 0.5
    return front_mask.bool(), sdf_mask.bool(), fs_weight, 1.0 - fs_weight


def get_sdf_loss(z_vals, target_d, predicted_sdf, truncation, cfg, return_mask=False, sample_weights=None,
                 rays_d=None):
    """nerf_helpers.py:382-399."""
    front_mask, sdf_mask, fs_weight, sdf_weight = get_masks(z_vals, target_d, truncation, cfg)
    mask = (target_d > cfg["far"] * cfg["sc_factor"]) & (predicted_sdf < cfg["fs_sdf"])
    fs_loss = torch.mean(((predicted_sdf - cfg["fs_sdf"]) * mask) ** 2 * sample_weights) * fs_weight
    mask = front_mask & (target_d <= cfg["far"] * cfg["sc_factor"]) & (predicted_sdf < 1)
    empty_loss = torch.mean(torch.abs(predicted_sdf - 1) * mask * sample_weights) * cfg["empty_weight"]
    fs_loss = fs_loss + empty_loss
    sdf_loss = torch.mean(((z_vals + predicted_sdf * truncation) * sdf_mask - target_d * sdf_mask) ** 2
                          * sample_weights) * sdf_weight
    if return_mask:
        return fs_loss, sdf_loss, front_mask, sdf_mask
    return fs_loss, sdf_loss


def ray_box_intersection_batch(origins, dirs, bounds):
    """nerf_helpers.py:403-446."""
    if not torch.is_tensor(origins):
        origins = torch.tensor(origins)
        dirs = torch.tensor(dirs)
    if not torch.is_tensor(bounds):
        bounds = torch.tensor(bounds)
    dirs = dirs / (torch.norm(dirs, dim=-1, keepdim=True) + 1e-10)
    inv_dirs = 1 / dirs
    bounds = bounds[None].expand(len(dirs), -1, -1).to(dirs.dtype)
    sign = (inv_dirs < 0).long()

    def g(axis, idx):
        return torch.gather(bounds[..., axis], dim=1, index=idx.reshape(-1, 1)).reshape(-1)

    tmin = (g(0, sign[:, 0]) - origins[:, 0]) * inv_dirs[:, 0]
    tmin[tmin < 0] = 0
    tmax = (g(0, 1 - sign[:, 0]) - origins[:, 0]) * inv_dirs[:, 0]
    tymin = (g(1, sign[:, 1]) - origins[:, 1]) * inv_dirs[:, 1]
    tymin[tymin < 0] = 0
    tymax = (g(1, 1 - sign[:, 1]) - origins[:, 1]) * inv_dirs[:, 1]
    ishit = torch.ones(len(dirs)).bool().to(dirs.device)
    ishit[(tmin > tymax) | (tymin > tmax)] = 0
    tmin[tymin > tmin] = tymin[tymin > tmin]
    tmax[tymax < tmax] = tymax[tymax < tmax]
    tzmin = (g(2, sign[:, 2]) - origins[:, 2]) * inv_dirs[:, 2]
    tzmin[tzmin < 0] = 0
    tzmax = (g(2, 1 - sign[:, 2]) - origins[:, 2]) * inv_dirs[:, 2]
    ishit[(tmin > tzmax) | (tzmin > tmax)] = 0
    tmin[tzmin > tmin] = tzmin[tzmin > tmin]
    tmax[tzmax < tmax] = tzmax[tzmax < tmax]
    tmin[ishit == 0] = -1
    tmax[ishit == 0] = -1
    return tmin, tmax
