"""Online hand-off between the tracker and the NeRF process,
device-resident: the point-cloud / scene-bounds / pose helpers that
bundlesdf.py imports from Utils.py and tool.py around the NerfRunner calls
(bundlesdf.py:87-260).

  toOpen3dCloud                  Utils.py:207-215  -> PointCloud (below)
  depth2xyzmap                   Utils.py:219-231
  compute_scene_bounds_worker    tool.py:42-63
  compute_scene_bounds           tool.py:67-131
  compute_translation_scales     tool.py:27-39
  find_biggest_cluster           tool.py:18-24     (sklearn DBSCAN -> nof_dbscan)
  get_optimized_poses_in_real_world  Utils.py:476-505
  mesh_to_real_world             Utils.py:508-514

PointCloud stands in for the open3d.geometry.PointCloud the hand-off uses:
points / colors (numpy views, f64), `+` / `+=`, voxel_down_sample (open3d
VoxelDownSample: voxel origin = min bound - size/2, per-voxel mean in point
order; device sort + nof_segment_mean), remove_statistical_outlier (open3d
RemoveStatisticalOutliers: mean distance to the k nearest points, the point
itself included, kept if 0 < d < mean + ratio * std; nof_knn_mean_dist),
select_by_index and transform (homogeneous, f64). Points live on the device;
numpy is produced only when .points / .colors are read.

MI355X-first differences: voxel_down_sample returns voxels in (x, y, z) index
order (open3d: hash-map order — a permutation of the same points); DBSCAN
border points join the cluster of their lowest-index core neighbour (sklearn:
the first cluster whose expansion reaches them); both are documented in
DESIGN.md and covered by tests/test_gpu_handoff.py.
"""
import ctypes
import logging
import os

import numpy as np
import torch

from . import _lib
from .mesh import mesh_to_real_world  # noqa: F401  (Utils.py:508 re-export)

GLCAM_IN_CVCAM = np.array([[1, 0, 0, 0], [0, -1, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]], dtype=np.float64)

__all__ = ["PointCloud", "toOpen3dCloud", "depth2xyzmap", "compute_scene_bounds_worker", "compute_scene_bounds",
           "compute_translation_scales", "find_biggest_cluster", "dbscan_labels", "get_optimized_poses_in_real_world",
           "mesh_to_real_world", "GLCAM_IN_CVCAM"]


def _dev(device=None):
    return torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())


class PointCloud:
    """Device point cloud with the open3d.geometry.PointCloud surface the hand-off uses."""

    def __init__(self, points=None, colors=None, device=None):
        self.device = _dev(device)
        self._p = self._as_dev(points) if points is not None else torch.zeros((0, 3), dtype=torch.float64,
                                                                                  device=self.device)
        self._c = self._as_dev(colors) if colors is not None else None

    def _as_dev(self, a):
        t = a if torch.is_tensor(a) else torch.from_numpy(np.ascontiguousarray(np.asarray(a, np.float64)))
        return t.to(self.device, torch.float64).reshape(-1, 3).contiguous()

    # -- open3d-style attributes
    @property
    def points(self):
        return self._p.cpu().numpy()

    @points.setter
    def points(self, v):
        self._p = self._as_dev(v)

    @property
    def colors(self):
        return self._c.cpu().numpy() if self._c is not None else np.zeros((0, 3))

    @colors.setter
    def colors(self, v):
        self._c = self._as_dev(v)

    def has_points(self):
        return len(self._p) > 0

    def has_colors(self):
        return self._c is not None and len(self._c) > 0

    def __len__(self):
        return len(self._p)

    def __add__(self, other):
        out = PointCloud(device=self.device)
        out._p = torch.cat([self._p, other._p.to(self.device)], 0)
        if self.has_colors() and other.has_colors():
            out._c = torch.cat([self._c, other._c.to(self.device)], 0)
        return out

    def __iadd__(self, other):
        r = self + other
        self._p, self._c = r._p, r._c
        return self

    def select_by_index(self, indices, invert=False):
        """open3d SelectByIndex: the selected points in their original order."""
        keep = torch.zeros(len(self._p), dtype=torch.bool, device=self.device)
        ids = torch.as_tensor(np.asarray(indices, np.int64), device=self.device)
        keep[ids] = True
        if invert:
            keep = ~keep
        out = PointCloud(device=self.device)
        out._p = self._p[keep].contiguous()
        out._c = self._c[keep].contiguous() if self.has_colors() else None
        return out

    def transform(self, T):
        """open3d Transform: p <- (T [p; 1])[:3] / w, f64; returns self."""
        T = torch.as_tensor(np.asarray(T, np.float64), device=self.device)
        ph = torch.cat([self._p, torch.ones((len(self._p), 1), dtype=torch.float64, device=self.device)], 1)
        q = ph @ T.T
        self._p = (q[:, :3] / q[:, 3:4]).contiguous()
        return self

    def voxel_down_sample(self, voxel_size):
        """open3d VoxelDownSample: mean point (and colour) of each occupied voxel of
        edge voxel_size, the grid anchored at min bound - voxel_size/2. Voxels are
        returned in (x, y, z) index order."""
        if voxel_size <= 0:
            raise ValueError("voxel_down_sample: voxel_size must be > 0")
        out = PointCloud(device=self.device)
        if len(self._p) == 0:
            return out
        vmin = self._p.min(0).values - voxel_size * 0.5
        idx = torch.floor((self._p - vmin) / voxel_size).to(torch.int64)
        dims = idx.max(0).values + 1
        key = (idx[:, 0] * dims[1] + idx[:, 1]) * dims[2] + idx[:, 2]
        skey, perm = torch.sort(key, stable=True)
        _, counts = torch.unique_consecutive(skey, return_counts=True)
        starts = torch.zeros(len(counts) + 1, dtype=torch.int64, device=self.device)
        starts[1:] = torch.cumsum(counts, 0)
        out._p = _segment_mean(self._p, perm, starts)
        out._c = _segment_mean(self._c, perm, starts) if self.has_colors() else None
        return out

    def remove_statistical_outlier(self, nb_neighbors, std_ratio):
        """open3d RemoveStatisticalOutliers -> (cloud, kept indices)."""
        n = len(self._p)
        if n == 0 or nb_neighbors < 1 or std_ratio <= 0:
            return PointCloud(device=self.device), []
        d = torch.empty(n, dtype=torch.float64, device=self.device)
        _lib.check(_lib.lib().nof_knn_mean_dist(_lib.ptr(self._p), n, int(nb_neighbors), _lib.ptr(d),
                                                _lib.stream_of(d)), "knn_mean_dist")
        # cloud statistics: sequential f64 sums in point order, as open3d's std::accumulate
        # / std::inner_product (n scalars: host side)
        dh = d.cpu().numpy()
        valid = dh > 0
        nv = int(valid.sum())
        mean = float(np.add.accumulate(dh[valid])[-1]) / nv if nv else 0.0
        sq = float(np.add.accumulate((dh[valid] - mean) * (dh[valid] - mean))[-1]) if nv else 0.0
        std = np.sqrt(sq / (nv - 1)) if nv > 1 else 0.0
        thr = mean + std_ratio * std
        ind = np.nonzero(valid & (dh < thr))[0]
        return self.select_by_index(ind), ind.tolist()


def _segment_mean(vals, perm, starts):
    S = len(starts) - 1
    C = vals.shape[1]
    out = torch.empty((S, C), dtype=torch.float64, device=vals.device)
    vals = vals.contiguous()
    _lib.check(_lib.lib().nof_segment_mean(_lib.ptr(vals), C, _lib.ptr(perm.contiguous()), _lib.ptr(starts), S,
                                           _lib.ptr(out), _lib.stream_of(vals)), "segment_mean")
    return out


def toOpen3dCloud(points, colors=None, normals=None, device=None):
    """Utils.py:207-215: f64 points; colours scaled by 1/255 when their max exceeds 1.
    Normals are accepted and dropped (the hand-off never reads them)."""
    pc = PointCloud(np.asarray(points, np.float64), device=device)
    if colors is not None:
        colors = np.asarray(colors)
        if len(colors) and colors.max() > 1:
            colors = colors / 255.0
        pc.colors = np.asarray(colors, np.float64)
    return pc


def depth2xyzmap(depth, K, device=None):
    """Utils.py:219-231 on the device: camera-frame xyz per pixel (f64 math,
    f32 result), zeros where depth < 0.1. Returns a [H,W,3] f32 tensor."""
    dev = _dev(device)
    z = torch.as_tensor(np.asarray(depth, np.float64), device=dev).reshape(depth.shape[0], depth.shape[1])
    H, W = z.shape
    vs = torch.arange(H, dtype=torch.float64, device=dev)[:, None].expand(H, W)
    us = torch.arange(W, dtype=torch.float64, device=dev)[None, :].expand(H, W)
    K = np.asarray(K, np.float64)
    xs = (us - K[0, 2]) * z / K[0, 0]
    ys = (vs - K[1, 2]) * z / K[1, 1]
    xyz = torch.stack([xs, ys, z], -1).to(torch.float32)
    xyz[z < 0.1] = 0
    return xyz


def compute_scene_bounds_worker(color_file, K, glcam_in_world, use_mask, rgb=None, depth=None, mask=None,
                                device=None):
    """tool.py:42-63: masked depth points of one frame, voxel_down_sample(0.01),
    remove_statistical_outlier(30, 2.0), to world (glcam_in_world @ glcam_in_cvcam).
    Returns (points [n,3] f64, colors [n,3] f64) or None."""
    if rgb is None:
        raise NotImplementedError("compute_scene_bounds_worker: reading frames from files is out of scope; "
                                  "pass rgb / depth / mask arrays")
    dev = _dev(device)
    depth = np.asarray(depth).reshape(np.asarray(depth).shape[:2])
    xyz = depth2xyzmap(depth, K, dev)
    valid = torch.as_tensor(depth >= 0.1, device=dev)
    if use_mask:
        valid &= torch.as_tensor(np.asarray(mask).reshape(depth.shape) > 0, device=dev)
    if not bool(valid.any()):
        return None
    pts = xyz[valid].reshape(-1, 3)
    colors = torch.as_tensor(np.asarray(rgb)[..., :3], device=dev)[valid].reshape(-1, 3).to(torch.float64)
    pc = PointCloud(pts, device=dev)
    if len(colors) and float(colors.max()) > 1:
        colors = colors / 255.0
    pc._c = colors.contiguous()
    pc = pc.voxel_down_sample(0.01)
    pc, _ = pc.remove_statistical_outlier(nb_neighbors=30, std_ratio=2.0)
    pc.transform(np.asarray(glcam_in_world, np.float64) @ GLCAM_IN_CVCAM)
    return pc.points.copy(), pc.colors.copy()


def dbscan_labels(pts, eps, min_samples=1, device=None):
    """sklearn.cluster.DBSCAN(eps, min_samples).fit(pts).labels_ on the device
    (nof_dbscan): clusters numbered 0.. in the order of their lowest core-point
    index, -1 = noise."""
    dev = _dev(device)
    p = torch.as_tensor(np.ascontiguousarray(np.asarray(pts, np.float64).reshape(-1, 3)), device=dev)
    n = len(p)
    if n == 0:
        return np.zeros(0, np.int64)
    lo = p.min(0).values.cpu().numpy() - eps
    hi = p.max(0).values.cpu().numpy()
    dims = (np.floor((hi - lo) / eps).astype(np.int64) + 2).astype(np.int32)
    nc = int(np.prod(dims.astype(np.int64)))
    L = _lib.lib()
    ws = torch.empty(int(L.nof_dbscan_workspace_bytes(n, nc)), dtype=torch.uint8, device=dev)
    roots = torch.empty(n, dtype=torch.int32, device=dev)
    org = (ctypes.c_double * 3)(*lo.tolist())
    dm = (ctypes.c_int32 * 3)(*dims.tolist())
    _lib.check(L.nof_dbscan(_lib.ptr(p), n, ctypes.c_double(eps), int(min_samples), org, dm, _lib.ptr(roots),
                            _lib.ptr(ws), _lib.stream_of(p)), "dbscan")
    roots = roots.long()
    clustered = roots >= 0
    uniq = torch.unique(roots[clustered])                      # sorted root indices = cluster order
    labels = torch.full_like(roots, -1)
    labels[clustered] = torch.searchsorted(uniq, roots[clustered])
    return labels.cpu().numpy()


def find_biggest_cluster(pts, eps=0.06, min_samples=1, device=None):
    """tool.py:18-24: points of the most populated DBSCAN label (noise included as
    a label, as the reference's np.unique over labels_) and the keep mask. Ties go
    to the larger label (numpy's argsort keeps equal counts in label order)."""
    labels = dbscan_labels(pts, eps, min_samples, device)
    ids, cnts = np.unique(labels, return_counts=True)
    best = ids[np.lexsort((ids, cnts))[-1]]
    keep = labels == best
    return np.asarray(pts)[keep], keep


def compute_translation_scales(pts, max_dim=2, cluster=True, eps=0.06, min_samples=1, device=None):
    """tool.py:27-39."""
    if cluster:
        pts, keep = find_biggest_cluster(pts, eps, min_samples, device)
    else:
        keep = np.ones(len(pts), dtype=bool)
    mx, mn = pts.max(axis=0), pts.min(axis=0)
    center = (mx + mn) / 2
    sc_factor = max_dim / (mx - mn).max() * 0.9
    return -center, sc_factor, keep


def _make_tf(translation, sc_factor):
    tf = np.eye(4)
    tf[:3, 3] = translation
    tf1 = np.eye(4)
    tf1[:3, :3] *= sc_factor
    return tf1 @ tf


def _write_ply(path, pts, colors=None):
    pts = np.asarray(pts, np.float64)
    with open(path, "wb") as f:
        hdr = ["ply", "format binary_little_endian 1.0", f"element vertex {len(pts)}", "property double x",
               "property double y", "property double z"]
        if colors is not None:
            hdr += ["property uchar red", "property uchar green", "property uchar blue"]
        f.write(("\n".join(hdr + ["end_header"]) + "\n").encode())
        if colors is None:
            f.write(pts.astype("<f8").tobytes())
        else:
            rec = np.zeros(len(pts), dtype=[("p", "<f8", 3), ("c", "u1", 3)])
            rec["p"] = pts
            rec["c"] = np.clip(np.round(np.asarray(colors) * 255), 0, 255).astype(np.uint8)
            f.write(rec.tobytes())


def compute_scene_bounds(color_files, glcam_in_worlds, K, use_mask=True, base_dir=None, rgbs=None, depths=None,
                         masks=None, cluster=True, translation_cvcam=None, sc_factor=None, eps=0.06, min_samples=1,
                         device=None):
    """tool.py:67-131: fuse the masked frames (worker per frame), voxel_down_sample(eps/5),
    biggest DBSCAN cluster -> (sc_factor, translation_cvcam, pcd_real_scale, pcd_normalized).
    With base_dir, writes naive_fusion.ply, naive_fusion_biggest_cluster.ply and
    normalization.yml like the reference."""
    assert color_files is None or rgbs is None
    if rgbs is None:
        raise NotImplementedError("compute_scene_bounds: reading frames from files is out of scope; pass rgbs/depths/masks")
    dev = _dev(device)
    pcd_all = None
    for i in range(len(rgbs)):
        r = compute_scene_bounds_worker(None, K, glcam_in_worlds[i], use_mask, rgbs[i], depths[i], masks[i], dev)
        if r is None:
            continue
        pc = toOpen3dCloud(r[0], r[1], device=dev)
        pcd_all = pc if pcd_all is None else pcd_all + pc
    if pcd_all is None:
        raise RuntimeError("compute_scene_bounds: no valid depth point in any frame")
    pcd = pcd_all.voxel_down_sample(eps / 5)
    if base_dir is not None:
        os.makedirs(base_dir, exist_ok=True)
        _write_ply(f"{base_dir}/naive_fusion.ply", pcd.points, pcd.colors)
    pts = pcd.points.copy()
    if translation_cvcam is None:
        translation_cvcam, sc_factor, keep = compute_translation_scales(pts, cluster=cluster, eps=eps,
                                                                        min_samples=min_samples, device=dev)
        tf = _make_tf(translation_cvcam, sc_factor)
    else:
        tf = _make_tf(translation_cvcam, sc_factor)
        tmp = PointCloud(pts, device=dev).transform(tf)
        keep = (np.abs(tmp.points) < 1).all(axis=-1)
    pcd = toOpen3dCloud(pts[keep], pcd.colors[keep], device=dev)
    if base_dir is not None:
        import yaml
        _write_ply(f"{base_dir}/naive_fusion_biggest_cluster.ply", pcd.points, pcd.colors)
        with open(f"{base_dir}/normalization.yml", "w") as ff:
            yaml.dump({"translation_cvcam": np.asarray(translation_cvcam).tolist(), "sc_factor": float(sc_factor)}, ff)
    logging.info(f"translation_cvcam={translation_cvcam}, sc_factor={sc_factor}")
    pcd_real_scale = toOpen3dCloud(pcd.points, pcd.colors, device=dev)
    pcd.transform(tf)
    return sc_factor, translation_cvcam, pcd_real_scale, pcd


def get_optimized_poses_in_real_world(poses_normalized, pose_array, sc_factor, translation):
    """Utils.py:476-505: pose corrections applied to the normalised GL cam-in-object
    poses, back to metres, re-anchored on frame 0, OpenCV convention.
    Returns (optimized cvcam_in_ob [N,4,4] f32, offset [4,4])."""
    original = np.array(poses_normalized, copy=True)
    original[:, :3, 3] /= sc_factor
    original[:, :3, 3] -= translation
    ids = torch.arange(len(poses_normalized), device=pose_array.data.device)
    with torch.no_grad():
        tf = pose_array.get_matrices(ids).reshape(-1, 4, 4).detach().cpu().numpy()
    opt = np.array(tf @ poses_normalized).astype(np.float32)
    opt[:, :3, 3] /= sc_factor
    opt[:, :3, 3] -= translation
    offset = np.linalg.inv(opt[0].copy()) @ original[0]
    for i in range(len(opt)):
        opt[i] = opt[i] @ offset
        opt[i] = opt[i] @ GLCAM_IN_CVCAM
    return opt, offset
