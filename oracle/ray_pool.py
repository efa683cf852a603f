"""ORACLE — test infrastructure only (tests/, make_golden.py). numpy
restatement of the reference's ray-pool construction, the checker for
bundlesdf_amd.ray_pool (nof_make_frame_rays):

  NerfRunner.make_frame_rays              nerf_runner.py:244-314
  compute_near_far_and_filter_rays        nerf_runner.py:39-65
  ray_box_intersection_batch              nerf_helpers.py:403-446
  get_camera_rays_np                      nerf_helpers.py:358-363
  octree-cloud denoise                    nerf_runner.py:175-194 (__init__),
                                          :408-423 (add_new_frames)

Pinned by tests/golden/ray_pool.npz, which runs the reference's own
make_frame_rays (from /root/reference) with cv2.dilate restated as a square
maximum filter and kaolin's trace replaced by oracle.kernels.octree_ray_trace
(the dense-grid trace, itself parity-unpinned against kaolin — SURVEY §8c).
The denoise step is inline in the reference's __init__, so it is restated
here (cKDTree nearest neighbour, as the reference) and not golden-pinned.

Numerics follow the reference's era (numpy 1.x value-based casting):
get_camera_rays_np computes in float32 with the float64 intrinsics rounded to
float32; everything after the concatenation with the float64 frame-id column
is float64; the pool is rounded to float32 at the end (torch.tensor(...,
dtype=float)).
"""
import numpy as np
from scipy import ndimage
from scipy.spatial import cKDTree

from . import kernels as K

BAD_DEPTH = 99


def camera_rays(H, W, Kmat):
    """get_camera_rays_np (nerf_helpers.py:358-363), float32 arithmetic."""
    i, j = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
    k = np.asarray(Kmat, np.float64).astype(np.float32)
    return np.stack([(i - k[0, 2]) / k[0, 0], -(j - k[1, 2]) / k[1, 1], -np.ones_like(i)], axis=-1)


def dilate(mask, k):
    """cv2.dilate(mask, np.ones((k,k)), iterations=1): window [u - k//2, u + k-1-k//2],
    borders never add (scipy's maximum_filter with origin 0 has the same window)."""
    k = 3 if k <= 0 else k
    return ndimage.maximum_filter(mask, size=(k, k), mode="constant", cval=0)


def ray_box(origins, dirs, bounds):
    """ray_box_intersection_batch (nerf_helpers.py:403-446), float64, same clamps."""
    n = np.sqrt((dirs * dirs).sum(-1, keepdims=True)) + 1e-10
    d = dirs / n
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1 / d
    bmin, bmax = np.asarray(bounds, np.float64).reshape(2, 3)
    neg = inv < 0
    lo = (np.where(neg, bmax, bmin) - origins) * inv
    hi = (np.where(neg, bmin, bmax) - origins) * inv
    tmin, tmax = lo[:, 0].copy(), hi[:, 0].copy()
    tmin[tmin < 0] = 0
    tymin, tymax = lo[:, 1].copy(), hi[:, 1]
    tymin[tymin < 0] = 0
    hit = ~((tmin > tymax) | (tymin > tmax))
    tmin = np.where(tymin > tmin, tymin, tmin)
    tmax = np.where(tymax < tmax, tymax, tmax)
    tzmin, tzmax = lo[:, 2].copy(), hi[:, 2]
    tzmin[tzmin < 0] = 0
    hit &= ~((tmin > tzmax) | (tzmin > tmax))
    tmin = np.where(tzmin > tmin, tzmin, tmin)
    tmax = np.where(tzmax < tmax, tzmax, tmax)
    tmin[~hit] = -1
    tmax[~hit] = -1
    return tmin, tmax


def near_far_filter(cam_in_world, rays, cfg):
    """compute_near_far_and_filter_rays (nerf_runner.py:39-65): rays [n,D] f64 in
    camera frame -> hits only, with |near|, |far| (z units) appended."""
    du = rays[:, :3] / np.linalg.norm(rays[:, :3], axis=-1).reshape(-1, 1)
    dirs = rays[:, :3] @ cam_in_world[:3, :3].T
    origins = np.broadcast_to(cam_in_world[:3, 3], dirs.shape)
    tmin, tmax = ray_box(origins, dirs, cfg["bounding_box"])
    hit = tmin >= 0
    near = np.abs(du[:, 2] * tmin)[hit]
    far = np.abs(du[:, 2] * tmax)[hit]
    return np.concatenate([rays[hit], near[:, None], far[:, None]], -1)


def trace_level(cfg):
    return int(np.floor(np.log2(2.0 / (cfg["octree_raytracing_voxel_size"] * cfg["sc_factor"]))))


def make_frame_rays(frame_id, images, depths, masks, poses, Kmat, cfg, occ_masks=None, occ=None):
    """NerfRunner.make_frame_rays (nerf_runner.py:244-314) without normal maps.
    occ: dense occupancy [n,n,n] u8 at trace_level(cfg) (None = no octree filter).
    Returns [n,12] float64: dir(3) rgb(3) depth mask frame_id type near far."""
    sc = cfg["sc_factor"]
    H, W = images.shape[1:3]
    mask = np.asarray(masks[frame_id, ..., 0]).copy()
    depth = depths[frame_id, ..., 0]
    rays = np.concatenate([camera_rays(H, W, Kmat), images[frame_id], depths[frame_id], masks[frame_id] > 0,
                           frame_id * np.ones(depths[frame_id].shape)], -1)
    invalid = ((depth < cfg["near"] * sc) | (depth > cfg["far"] * sc)) & (mask > 0)
    types = np.zeros((H, W, 1))
    types[invalid] = 1
    rays = np.concatenate([rays, types], -1)
    k = 100 if frame_id == 0 else 60 // int(cfg["down_scale_ratio"])
    mask = dilate(mask, k)
    if occ_masks is not None:
        mask[occ_masks[frame_id] > 0] = 0
    if cfg["rays_valid_depth_only"]:
        mask[invalid] = 0
    vs, us = np.where(mask > 0)
    cur = rays[vs, us].reshape(-1, 10)
    cur = cur[cur[:, 9] == 0]
    cur = near_far_filter(poses[frame_id], cur, cfg)
    if occ is not None and len(cur):
        T = poses[frame_id]
        o = np.broadcast_to(T[:3, 3], (len(cur), 3)).astype(np.float32)
        du = cur[:, :3] / np.linalg.norm(cur[:, :3], axis=-1).reshape(-1, 1)
        d = (du @ T[:3, :3].T).astype(np.float32)
        dio, _ = K.octree_ray_trace(occ, o, d, 1)
        cur = cur[dio[:, 0, 0] > 0]
    return cur


def denoise(rays, poses, cloud, cfg):
    """nerf_runner.py:175-194: depth points (mask > 0, depth <= far*sc) farther than
    0.02*sc from every octree-cloud point become type 1 and are dropped."""
    sc = cfg["sc_factor"]
    m = (rays[:, 7] > 0) & (rays[:, 6] <= cfg["far"] * sc)
    p = rays[m][:, :3] * rays[m][:, 6].reshape(-1, 1)
    fid = rays[m][:, 8].astype(int)
    ph = np.concatenate([p, np.ones((len(p), 1))], -1)
    pw = (poses[fid] @ ph[..., None])[:, :3, 0]
    rays = rays.copy()
    if len(pw):
        dists, _ = cKDTree(cloud).query(pw, k=1)
        bad = np.arange(len(rays))[m][dists > 0.02 * sc]
        rays[bad, 6] = BAD_DEPTH * sc
        rays[bad, 9] = 1
    return rays[rays[:, 9] == 0]


def build_pool(frames, images, depths, masks, poses, Kmat, cfg, occ_masks=None, occ=None, cloud=None):
    """Reference pool for `frames`: per-frame rays, concatenated, denoised (if
    cfg['denoise_depth_use_octree_cloud'] and a cloud is given), float32."""
    rays = np.concatenate([make_frame_rays(f, images, depths, masks, poses, Kmat, cfg, occ_masks, occ)
                           for f in frames], 0)
    if cfg.get("denoise_depth_use_octree_cloud") and cloud is not None:
        rays = denoise(rays, poses, cloud, cfg)
    return rays.astype(np.float32)
