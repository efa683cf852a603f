"""Ray-pool construction on the device.

Replaces the per-frame host loop of the reference — NerfRunner.make_frame_rays
(nerf_runner.py:244-314) with compute_near_far_and_filter_rays (:39-65),
ray_box_intersection_batch (nerf_helpers.py:403-446), the octree filter
(:300-312) — and the cKDTree denoise of the concatenated pool (:175-194,
:408-423) with five HIP launches per frame batch (csrc/ray_pool.hip):
separable mask dilation, per-pixel selection (box near/far + dense-grid
trace + uniform-grid radius test), block-count scan and ordered compaction.
The pool is produced directly in HBM in the reference's row order and
12-column layout; the host only uploads the frames.

No CPU fallback: every entry point raises if libnof.so cannot run.
"""
import ctypes

import numpy as np
import torch

from . import _lib

POOL_MAX_PIXELS = 1 << 26        # frames per launch: F*H*W <= 64 M pixels (~3.2 GB of [P,12] f32 rows)


class PointGrid:
    """Uniform grid of the octree point cloud for the denoise radius test
    (nof_point_grid_build). cell >= radius, so a radius query visits the
    3x3x3 cells around the query point."""

    def __init__(self, points, radius, device):
        pts = np.ascontiguousarray(np.asarray(points, np.float64).reshape(-1, 3))
        if len(pts) == 0:
            raise ValueError("PointGrid: empty point cloud")
        self.radius = float(radius)
        lo, hi = pts.min(0), pts.max(0)
        cell = self.radius
        while True:
            dims = np.floor((hi - lo) / cell).astype(np.int64) + 3
            if int(np.prod(dims)) <= (1 << 26):
                break
            cell *= 1.25
        self.cell = float(cell)
        self.origin = (lo - cell).astype(np.float64)
        self.dims = dims.astype(np.int32)
        nc = int(np.prod(self.dims))
        L = _lib.lib()
        p = torch.from_numpy(pts).to(device)
        self.cell_start = torch.empty(nc + 1, dtype=torch.int32, device=device)
        self.cell_points = torch.empty_like(p)
        ws = torch.empty(int(L.nof_point_grid_workspace_bytes(nc)), dtype=torch.uint8, device=device)
        org = (ctypes.c_double * 3)(*self.origin.tolist())
        dm = (ctypes.c_int32 * 3)(*self.dims.tolist())
        rc = L.nof_point_grid_build(_lib.ptr(p), int(len(pts)), org, dm, ctypes.c_double(self.cell),
                                    _lib.ptr(self.cell_start), _lib.ptr(self.cell_points), None, _lib.ptr(ws),
                                    _lib.stream_of(p))
        _lib.check(rc, "point_grid_build")
        self._keep = (p, ws)


def make_pool_rays(frames, images, depths, masks, poses, K, cfg, occ_masks=None, occ=None, point_grid=None,
                   device=None, index_base=0):
    """Rays of `frames` (consecutive ascending global ids) -> [n,12] f32 on `device`,
    equal to the reference's make_frame_rays over those frames, concatenated,
    then denoised when `point_grid` is given (cfg['denoise_depth_use_octree_cloud']).

    images [N,H,W,3] in [0,1]; depths [N,H,W,1] (sc-scaled); masks [N,H,W,1];
    occ_masks [N,H,W] or None; poses [N,4,4] normalised GL cam-in-object;
    occ: dense occupancy [n,n,n] u8 at the trace level (device tensor) or None.
    index_base: global id of row 0 of the frame arrays (a rank holding frames
    lo..hi of a sharded sequence passes lo); `frames` are global ids (column 8,
    and frame 0's 100 px dilation, follow them)."""
    frames = list(frames)
    if not frames:
        return torch.empty((0, 12), dtype=torch.float32, device=device)
    if frames != list(range(frames[0], frames[0] + len(frames))):
        raise ValueError("make_pool_rays: frames must be consecutive ids")
    device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    L = _lib.lib()
    H, W = images.shape[1:3]
    sc = float(cfg["sc_factor"])
    k32 = np.asarray(K, np.float64).astype(np.float32)
    bbox = np.asarray(cfg["bounding_box"], np.float64).reshape(6)
    if occ is not None:
        if not (occ.is_cuda and occ.dtype == torch.uint8 and occ.dim() == 3):
            raise RuntimeError("make_pool_rays: occ must be a [n,n,n] uint8 device tensor")
        occ = occ.contiguous()
    per = max(1, POOL_MAX_PIXELS // (H * W))
    out = []
    for c0 in range(0, len(frames), per):
        fs = frames[c0:c0 + per]
        a, b = fs[0] - index_base, fs[-1] + 1 - index_base
        if a < 0 or b > len(images):
            raise ValueError(f"make_pool_rays: frames {fs[0]}..{fs[-1]} outside the arrays (index_base {index_base})")
        F = b - a
        rgb = torch.from_numpy(np.ascontiguousarray(images[a:b], np.float32)).to(device)
        dep = torch.from_numpy(np.ascontiguousarray(np.asarray(depths[a:b]).reshape(F, H, W), np.float32)).to(device)
        msk = torch.from_numpy(np.ascontiguousarray(np.asarray(masks[a:b]).reshape(F, H, W) > 0, np.uint8)).to(device)
        om = None
        if occ_masks is not None:
            om = torch.from_numpy(np.ascontiguousarray(np.asarray(occ_masks[a:b]).reshape(F, H, W) > 0,
                                                       np.uint8)).to(device)
        T = torch.from_numpy(np.ascontiguousarray(np.asarray(poses[a:b], np.float64))).to(device)
        P = F * H * W
        rays = torch.empty((P, 12), dtype=torch.float32, device=device)
        n_out = torch.zeros(1, dtype=torch.int64, device=device)
        ws = torch.empty(int(L.nof_ray_pool_workspace_bytes(F, H, W)), dtype=torch.uint8, device=device)
        d = _lib.RayPoolDesc()
        d.rgb, d.depth, d.mask, d.occ_mask, d.cam_in_world = (_lib.ptr(rgb).value, _lib.ptr(dep).value,
                                                              _lib.ptr(msk).value, _lib.ptr(om).value,
                                                              _lib.ptr(T).value)
        d.F, d.H, d.W, d.first_frame_id = F, H, W, fs[0]
        d.dilate_first, d.dilate_other = 100, 60 // int(cfg["down_scale_ratio"])
        d.fx, d.fy, d.cx, d.cy = float(k32[0, 0]), float(k32[1, 1]), float(k32[0, 2]), float(k32[1, 2])
        d.near_sc = float(np.float32(cfg["near"] * sc))
        d.far_sc = float(np.float32(cfg["far"] * sc))
        d.far_sc64 = cfg["far"] * sc
        d.bbox[:] = bbox.tolist()
        d.occ, d.occ_n = (_lib.ptr(occ).value, int(occ.shape[0])) if occ is not None else (None, 0)
        if point_grid is not None:
            d.cell_start, d.cell_points = _lib.ptr(point_grid.cell_start).value, _lib.ptr(point_grid.cell_points).value
            d.grid_origin[:] = point_grid.origin.tolist()
            d.grid_dims[:] = point_grid.dims.tolist()
            d.grid_cell, d.grid_radius = point_grid.cell, point_grid.radius
        d.workspace, d.rays, d.n_out = _lib.ptr(ws).value, _lib.ptr(rays).value, _lib.ptr(n_out).value
        _lib.check(L.nof_make_frame_rays(ctypes.byref(d), _lib.stream_of(rays)), "make_frame_rays")
        n = int(n_out.item())
        out.append(rays[:n].clone())
        del rays, ws
    return out[0] if len(out) == 1 else torch.cat(out, 0)
