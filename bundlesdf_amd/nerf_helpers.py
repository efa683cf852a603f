"""The module-level names the trainer boundary needs from the reference's
nerf_helpers.py: the parameter-owning modules (NeRFSmall,
PoseArray, FeatureArray — same parameter names, shapes and init, so state
dicts interchange), the embedder factory, and preprocess_data (bundlesdf.py
reaches it through `from nerf_runner import *`).

The training step never runs these modules: the fused HIP kernels (fused.py,
libnof) read their parameters from the trainer's flat buffer. The samplers,
losses and compositing of the reference module (get_masks, get_sdf_loss,
sample_pdf, ray_box_intersection_batch) live in the kernels and, as test
infrastructure, in oracle/; they are not part of this module.
"""
import math

import numpy as np
import torch
import torch.nn as nn

BAD_DEPTH = 99      # Utils.py:33 (invalid / background depth, before sc_factor)
BAD_COLOR = 128     # Utils.py:34


def to8b(x):
    """[0,1] float image -> uint8 (nerf_helpers.py:18)."""
    return (np.clip(x, 0, 1) * 255).astype(np.uint8)


# Real spherical harmonics as sums of monomials c * x^a y^b z^d, one list per
# output channel, degrees 0..4 (the reference encoder's basis and sign
# convention, nerf_helpers.py:22-105; 25 channels for degree 5).
def _sh_table():
    c0 = 0.28209479177387814
    c1 = 0.4886025119029199
    c2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
    c3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
          1.445305721320277, -0.5900435899266435)
    c4 = (2.5033429417967046, -1.7701307697799304, 0.9461746957575601, -0.6690465435572892, 0.10578554691520431,
          -0.6690465435572892, 0.47308734787878004, -1.7701307697799304, 0.6258357354491761)
    t = [[(c0, (0, 0, 0))],
         [(-c1, (0, 1, 0))], [(c1, (0, 0, 1))], [(-c1, (1, 0, 0))],
         [(c2[0], (1, 1, 0))], [(c2[1], (0, 1, 1))],
         [(2 * c2[2], (0, 0, 2)), (-c2[2], (2, 0, 0)), (-c2[2], (0, 2, 0))],
         [(c2[3], (1, 0, 1))], [(c2[4], (2, 0, 0)), (-c2[4], (0, 2, 0))],
         [(3 * c3[0], (2, 1, 0)), (-c3[0], (0, 3, 0))], [(c3[1], (1, 1, 1))],
         [(4 * c3[2], (0, 1, 2)), (-c3[2], (2, 1, 0)), (-c3[2], (0, 3, 0))],
         [(2 * c3[3], (0, 0, 3)), (-3 * c3[3], (2, 0, 1)), (-3 * c3[3], (0, 2, 1))],
         [(4 * c3[4], (1, 0, 2)), (-c3[4], (3, 0, 0)), (-c3[4], (1, 2, 0))],
         [(c3[5], (2, 0, 1)), (-c3[5], (0, 2, 1))], [(c3[6], (3, 0, 0)), (-3 * c3[6], (1, 2, 0))],
         [(c4[0], (3, 1, 0)), (-c4[0], (1, 3, 0))], [(3 * c4[1], (2, 1, 1)), (-c4[1], (0, 3, 1))],
         [(7 * c4[2], (1, 1, 2)), (-c4[2], (1, 1, 0))], [(7 * c4[3], (0, 1, 3)), (-3 * c4[3], (0, 1, 1))],
         [(35 * c4[4], (0, 0, 4)), (-30 * c4[4], (0, 0, 2)), (3 * c4[4], (0, 0, 0))],
         [(7 * c4[5], (1, 0, 3)), (-3 * c4[5], (1, 0, 1))],
         [(7 * c4[6], (2, 0, 2)), (-c4[6], (2, 0, 0)), (-7 * c4[6], (0, 2, 2)), (c4[6], (0, 2, 0))],
         [(c4[7], (3, 0, 1)), (-3 * c4[7], (1, 2, 1))],
         [(c4[8], (4, 0, 0)), (-6 * c4[8], (2, 2, 0)), (c4[8], (0, 4, 0))]]
    return t


_SH = _sh_table()


class SHEncoder(nn.Module):
    """View-direction encoder (nerf_helpers.py:22-105): real SH up to `degree`,
    out_dim = degree^2. The fused kernels evaluate degree 3 per ray in the
    MLP kernel (sh_frag); this module serves the API and host-side tools."""

    def __init__(self, input_dim=3, degree=4):
        super().__init__()
        if input_dim != 3 or not 1 <= degree <= 5:
            raise ValueError("SHEncoder: input_dim 3, degree 1..5")
        self.input_dim, self.degree, self.out_dim = input_dim, degree, degree ** 2

    def forward(self, input, **kwargs):
        x, y, z = input.unbind(-1)
        pw = [[torch.ones_like(x)], [torch.ones_like(y)], [torch.ones_like(z)]]
        for k in range(1, 5):
            pw[0].append(pw[0][-1] * x)
            pw[1].append(pw[1][-1] * y)
            pw[2].append(pw[2][-1] * z)
        chans = []
        for terms in _SH[:self.out_dim]:
            acc = None
            for c, (a, b, d) in terms:
                v = c * (pw[0][a] * pw[1][b] * pw[2][d])
                acc = v if acc is None else acc + v
            chans.append(acc)
        return torch.stack(chans, -1)


class FeatureArray(nn.Module):
    """Per-frame latent code (nerf_helpers.py:108-124): data [F, C] ~ N(0, 1)."""

    def __init__(self, num_frames, num_channels):
        super().__init__()
        self.num_frames, self.num_channels = num_frames, num_channels
        self.data = nn.Parameter(torch.normal(0, 1, size=[num_frames, num_channels]).float(), requires_grad=True)

    def __call__(self, ids):
        return self.data[ids]


class PoseArray(nn.Module):
    """Per-frame pose correction (nerf_helpers.py:127-154): data [F, 6] =
    (translation, axis-angle) before a tanh bound of max_trans / max_rot deg;
    frame 0 is held at the identity. The training step evaluates it on the device
    (nof_pose_forward, with its Jacobian); get_matrices serves the hand-off tools."""

    def __init__(self, num_frames, max_trans, max_rot):
        super().__init__()
        self.num_frames, self.max_trans, self.max_rot = num_frames, max_trans, max_rot
        self.data = nn.Parameter(torch.zeros(num_frames, 6), requires_grad=True)

    def _all_matrices(self):
        """[F,4,4] corrections of every frame (column-vector convention)."""
        d = self.data.detach().float().contiguous()
        F = d.shape[0]
        if d.is_cuda:
            from . import _lib
            L = _lib.lib()
            eye = torch.eye(4, device=d.device).expand(F, 4, 4).contiguous()
            tf = torch.empty(F, 16, device=d.device)
            jac = torch.empty(F, 12, 6, device=d.device)
            _lib.check(L.nof_pose_forward(_lib.ptr(d), _lib.ptr(eye), F, float(self.max_trans),
                                          float(self.max_rot * math.pi / 180.0), _lib.ptr(tf), _lib.ptr(jac),
                                          _lib.stream_of(d)), "pose_forward")
            return tf.view(F, 4, 4)
        # host tools on CPU tensors. pytorch3d's se3_exp_map (row-vector form, transposed by
        # the reference) gives rotation exp(hat(w))^T and translation V(w) t, V the left
        # Jacobian of SO(3): both read off the matrix exponential of the 4x4 generator
        # [[hat(w), t], [0, 0]] (pytorch3d clamps |w|^2 at 1e-4: a ~1e-7 difference here)
        th = torch.tanh(d.double())
        t = th[:, :3] * self.max_trans
        w = th[:, 3:] * (self.max_rot * math.pi / 180.0)
        G = torch.zeros(F, 4, 4, dtype=torch.float64)
        G[:, 0, 1], G[:, 0, 2], G[:, 1, 2] = -w[:, 2], w[:, 1], -w[:, 0]
        G[:, 1, 0], G[:, 2, 0], G[:, 2, 1] = w[:, 2], -w[:, 1], w[:, 0]
        G[:, :3, 3] = t
        E = torch.linalg.matrix_exp(G)
        T = torch.eye(4, dtype=torch.float64).repeat(F, 1, 1)
        T[:, :3, :3] = E[:, :3, :3].transpose(1, 2)
        T[:, :3, 3] = E[:, :3, 3]
        T = T.float()
        T[0] = torch.eye(4)
        return T

    def get_matrices(self, ids):
        if not torch.is_tensor(ids):
            ids = torch.as_tensor(ids)
        T = self._all_matrices()
        return T[ids.long().to(T.device)]


def get_embedder(multires, cfg, i=0, octree_m=None):
    """nerf_helpers.py:191-214 for the encoders the fused trainer runs:
    i=1 hash grid (GridEncoder), i=2 spherical harmonics; -1 identity."""
    if i == -1:
        return nn.Identity(), 3
    if i == 1:
        from .grid import GridEncoder
        enc = GridEncoder(input_dim=3, n_levels=cfg["num_levels"], level_dim=cfg["feature_grid_dim"],
                          base_resolution=cfg["base_res"], log2_hashmap_size=cfg["log2_hashmap_size"],
                          desired_resolution=cfg["finest_res"])
        return enc, enc.out_dim
    if i == 2:
        enc = SHEncoder(degree=cfg["multires_views"])
        return enc, enc.out_dim
    raise NotImplementedError(f"embedder {i}: the fused MI355X trainer runs the hash grid (1) and SH (2)")


def preprocess_data(rgbs, depths, masks, normal_maps, poses, sc_factor, translation):
    """nerf_helpers.py:218-240 (in place where the reference is): depths < 0.1
    and pixels outside the mask -> BAD_DEPTH, colour outside the mask -> BAD_COLOR,
    normals flipped to GL (y, z) and zeroed outside the mask, rgb to [0,1] f32,
    depth and camera translation normalised by (+translation) * sc_factor."""
    depths[depths < 0.1] = BAD_DEPTH
    if masks is not None:
        off = masks == 0
        rgbs[off] = BAD_COLOR
        depths[off] = BAD_DEPTH
        if normal_maps is not None:
            normal_maps[..., 1:3] = -normal_maps[..., 1:3]
            normal_maps[off] = 0
        masks = masks[..., None]
    rgbs = (rgbs / 255.0).astype(np.float32)
    depths *= sc_factor
    depths = depths[..., None]
    poses[:, :3, 3] = (poses[:, :3, 3] + translation) * sc_factor
    return rgbs, depths, masks, normal_maps, poses


def get_camera_rays_np(H, W, K):
    """Pixel rays in the GL camera frame (x right, y up, z = -1), nerf_helpers.py:358-363."""
    u = np.arange(W, dtype=np.float32)[None, :].repeat(H, 0)
    v = np.arange(H, dtype=np.float32)[:, None].repeat(W, 1)
    return np.stack([(u - K[0][2]) / K[0][0], (K[1][2] - v) / K[1][1], -np.ones((H, W), np.float32)], -1)


class NeRFSmall(nn.Module):
    """The SDF + colour network (nerf_helpers.py:243-321): parameters
    sigma_net.{0,2,..}, color_net.{0,2,..} of nn.Linear layers with ReLUs in
    between; the last sigma bias is initialised to 0.1. Output [rgb logits(3), sdf].
    The fused kernels run it on MFMA (bundlesdf_amd/mlp_layout.py packs these
    parameters); forward() is the plain torch evaluation for host-side use."""

    def __init__(self, num_layers=3, hidden_dim=64, geo_feat_dim=15, num_layers_color=4, hidden_dim_color=64,
                 input_ch=3, input_ch_views=3):
        super().__init__()
        self.input_ch, self.input_ch_views = input_ch, input_ch_views
        self.num_layers, self.hidden_dim, self.geo_feat_dim = num_layers, hidden_dim, geo_feat_dim
        self.num_layers_color, self.hidden_dim_color = num_layers_color, hidden_dim_color
        self.sigma_net = self._chain([input_ch] + [hidden_dim] * (num_layers - 1) + [1 + geo_feat_dim])
        nn.init.constant_(self.sigma_net[-1].bias, 0.1)
        self.color_net = self._chain([input_ch_views + geo_feat_dim] + [hidden_dim] * (num_layers_color - 1) + [3])

    @staticmethod
    def _chain(widths):
        mods = []
        for k in range(len(widths) - 1):
            if k:
                mods.append(nn.ReLU(inplace=True))
            mods.append(nn.Linear(widths[k], widths[k + 1]))
        return nn.Sequential(*mods)

    def forward_sdf(self, x):
        return self.sigma_net(x)[..., 0]

    def forward(self, x):
        x = x.float()
        h = self.sigma_net(x[..., :self.input_ch])
        rgb = self.color_net(torch.cat([x[..., self.input_ch:self.input_ch + self.input_ch_views], h[..., 1:]], -1))
        return torch.cat([rgb, h[..., :1]], -1)
