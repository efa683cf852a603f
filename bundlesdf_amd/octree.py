"""Occupancy "octree" for ray marching — replaces the kaolin-SPC OctreeManager
(Utils.py:359-475) on the hot path.

MI355X design: instead of a pointer/SPC octree walked per ray, the occupied
set is a dense uint8 grid per level (the finest grid at the reference's
octree_smallest_voxel_size is 2^max_level per side: 32^3..512^3 bytes, i.e.
kilobytes to 134 MB — resident in HBM/L2), and the ray trace is a branch-light
3-D DDA kernel (csrc/ray_sampling.hip). Coarser levels are OR-reductions of
the finest one, which is exactly which SPC nodes exist at that level.
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import _lib


def quantize(pts, level):
    """kaolin.ops.spc.quantize_points: floor((p+1)/2 * 2^level) clamped to the grid."""
    n = 2 ** level
    return torch.clamp(torch.floor((pts + 1) / 2 * n), 0, n - 1).long()


def build_occupancy(pts, max_level, dilate_radius=1):
    """nerf_runner.py:441-474 + Utils.py:362-363: quantize points at the finest
    voxel size, dilate by `dilate_radius` 27-neighbourhood steps, return the
    dense occupancy [N,N,N] (z,y,x; x fastest) at max_level. Out-of-range
    dilated cells clamp into the border (the reference clips to [-1,1] before
    re-quantising); those cells are already covered by the dilation itself,
    so a max-pool dilation is equivalent."""
    n = 2 ** max_level
    vox = 2.0 / n
    coords = torch.clamp(torch.floor((pts.double() + 1) / vox), 0, n - 1).long()
    occ = torch.zeros((n, n, n), dtype=torch.float32, device=pts.device)
    occ[coords[:, 2], coords[:, 1], coords[:, 0]] = 1.0
    for _ in range(max(1, int(dilate_radius))):
        occ = F.max_pool3d(occ[None, None], kernel_size=3, stride=1, padding=1)[0, 0]
    return occ.to(torch.uint8)


def coarsen(occ, factor):
    if factor == 1:
        return occ
    n = occ.shape[0] // factor
    return occ.view(n, factor, n, factor, n, factor).amax(dim=(1, 3, 5))


def ray_trace_dense(occ, rays_o, rays_d, kmax):
    """Front-to-back [t_in,t_out] of occupied voxels per ray, zero padded to kmax
    (nof_octree_ray_trace). Returns (depths_in_out [R,kmax,2], counts [R] i32)."""
    if not (occ.is_cuda and rays_o.is_cuda and rays_d.is_cuda):
        raise RuntimeError("ray_trace_dense: tensors must be on the HIP device")
    occ = occ.contiguous()
    rays_o = rays_o.contiguous().float()
    rays_d = rays_d.contiguous().float()
    R = rays_o.shape[0]
    out = torch.empty((R, kmax, 2), dtype=torch.float32, device=rays_o.device)
    counts = torch.empty(R, dtype=torch.int32, device=rays_o.device)
    rc = _lib.lib().nof_octree_ray_trace(_lib.ptr(occ), int(occ.shape[0]), _lib.ptr(rays_o), _lib.ptr(rays_d), int(R),
                                         int(kmax), _lib.ptr(out), _lib.ptr(counts), _lib.stream_of(rays_o))
    _lib.check(rc, "octree_ray_trace")
    return out, counts


class OctreeManager:
    """API subset of Utils.OctreeManager used by the trainer (Utils.py:359-475)."""

    def __init__(self, pts=None, max_level=None, octree=None, dilate_radius=0):
        if octree is not None:
            self.occ_finest = octree.to(torch.uint8)
            self.max_level = int(round(np.log2(self.occ_finest.shape[0])))
        else:
            self.max_level = int(max_level)
            if dilate_radius:
                self.occ_finest = build_occupancy(pts, self.max_level, dilate_radius)
            else:
                n = 2 ** self.max_level
                q = quantize(pts, self.max_level)
                occ = torch.zeros((n, n, n), dtype=torch.uint8, device=pts.device)
                occ[q[:, 2], q[:, 1], q[:, 0]] = 1
                self.occ_finest = occ
        self.octree = self.occ_finest            # serialisable state (save_weights key 'octree')
        self.n_level = self.max_level + 1
        self._levels = {}

    def occupancy(self, level):
        if level not in self._levels:
            self._levels[level] = coarsen(self.occ_finest, 2 ** (self.max_level - level)).contiguous()
        return self._levels[level]

    def get_center_ids(self, x, level):
        """Utils.py:392-394: voxel id at `level` or -1 if unoccupied."""
        occ = self.occupancy(level)
        q = quantize(x, level)
        n = occ.shape[0]
        lin = (q[:, 2] * n + q[:, 1]) * n + q[:, 0]
        inside = (x.abs() <= 1).all(dim=-1)
        ok = inside & (occ.view(-1)[lin] > 0)
        return torch.where(ok, lin, torch.full_like(lin, -1))

    def ray_trace(self, rays_o, rays_d, level, debug=False, kmax=None):
        """Utils.py:443-475: returns (near, far, pid, depths_in_out [R,K,2]) in travel
        distance t along unit rays_d. K = max hits in the batch (one host sync, as the
        reference's counts.max().item()) unless kmax is given."""
        occ = self.occupancy(level)
        n = occ.shape[0]
        bound = 3 * n if kmax is None else kmax
        out, counts = ray_trace_dense(occ, rays_o, rays_d, bound)
        if kmax is None:
            k = max(1, int(counts.max().item()))
            out = out[:, :k].contiguous()
        near = out[:, 0, 0].reshape(-1, 1)
        far = out[:, :, 1].max(dim=-1)[0].reshape(-1, 1)
        pid = torch.where(counts > 0, torch.zeros_like(counts), -torch.ones_like(counts)).reshape(-1, 1)
        return near, far, pid, out
