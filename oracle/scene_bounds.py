"""ORACLE — test infrastructure only (tests/). CPU restatement of the online
hand-off's point-cloud path, the checker for bundlesdf_amd.handoff:

  voxel_down_sample            open3d PointCloud::VoxelDownSample (published
                               algorithm: voxel origin = min bound - size/2,
                               floor index, per-voxel mean accumulated in point
                               order) — open3d is not installed: PARITY
                               UNPINNED against open3d itself
  remove_statistical_outlier   open3d PointCloud::RemoveStatisticalOutliers
                               (kNN incl. the point itself, sequential mean /
                               std, keep 0 < d < mean + ratio*std) — kNN by
                               scipy cKDTree; PARITY UNPINNED against open3d
  dbscan_labels                sklearn.cluster.DBSCAN — the reference's own
                               dependency (tool.py:11,19), installed here
  depth2xyzmap                 Utils.py:219-231 (golden-pinned, G6)
  find_biggest_cluster /
  compute_translation_scales   tool.py:18-39 (golden-pinned, G6)
  compute_scene_bounds(_worker) tool.py:42-131 composed from the above
"""
import numpy as np
from scipy.spatial import cKDTree

GLCAM_IN_CVCAM = np.array([[1, 0, 0, 0], [0, -1, 0, 0], [0, 0, -1, 0], [0, 0, 0, 1]], dtype=np.float64)


def voxel_down_sample(points, colors, voxel):
    """-> (points, colors) of the occupied voxels in (x, y, z) index order."""
    points = np.asarray(points, np.float64)
    vmin = points.min(0) - voxel * 0.5
    idx = np.floor((points - vmin) / voxel).astype(np.int64)
    acc = {}
    for i in range(len(points)):
        k = tuple(idx[i])
        if k not in acc:
            acc[k] = [np.zeros(3), np.zeros(3), 0]
        a = acc[k]
        for d in range(3):                      # sequential f64 sums in point order
            a[0][d] += points[i, d]
            if colors is not None:
                a[1][d] += colors[i, d]
        a[2] += 1
    keys = sorted(acc)
    p = np.array([acc[k][0] / acc[k][2] for k in keys])
    c = np.array([acc[k][1] / acc[k][2] for k in keys]) if colors is not None else None
    return p, c


def knn_mean_dist(points, k):
    points = np.asarray(points, np.float64)
    ke = min(k, len(points))
    d, _ = cKDTree(points).query(points, k=ke)
    d = d.reshape(len(points), ke)
    return np.array([np.add.accumulate(row)[-1] / ke for row in d])


def remove_statistical_outlier(points, nb_neighbors, std_ratio):
    """-> kept indices (ascending)."""
    d = knn_mean_dist(points, nb_neighbors)
    valid = d > 0
    nv = int(valid.sum())
    mean = float(np.add.accumulate(d[valid])[-1]) / nv
    sq = float(np.add.accumulate((d[valid] - mean) * (d[valid] - mean))[-1])
    std = np.sqrt(sq / (nv - 1)) if nv > 1 else 0.0
    return np.nonzero(valid & (d < mean + std_ratio * std))[0]


def dbscan_labels(points, eps, min_samples):
    from sklearn.cluster import DBSCAN
    return DBSCAN(eps=eps, min_samples=min_samples).fit(np.asarray(points, np.float64)).labels_


def depth2xyzmap(depth, K):
    invalid = depth < 0.1
    H, W = depth.shape[:2]
    vs, us = np.meshgrid(np.arange(0, H), np.arange(0, W), sparse=False, indexing="ij")
    zs = depth.reshape(-1)
    xs = (us.reshape(-1) - K[0, 2]) * zs / K[0, 0]
    ys = (vs.reshape(-1) - K[1, 2]) * zs / K[1, 1]
    xyz = np.stack((xs, ys, zs), 1).reshape(H, W, 3).astype(np.float32)
    xyz[invalid] = 0
    return xyz


def find_biggest_cluster(pts, eps=0.06, min_samples=1):
    labels = dbscan_labels(pts, eps, min_samples)
    ids, cnts = np.unique(labels, return_counts=True)
    best = ids[cnts.argsort()[-1]]
    keep = labels == best
    return pts[keep], keep


def compute_translation_scales(pts, max_dim=2, cluster=True, eps=0.06, min_samples=1):
    if cluster:
        pts, keep = find_biggest_cluster(pts, eps, min_samples)
    else:
        keep = np.ones(len(pts), dtype=bool)
    mx, mn = pts.max(axis=0), pts.min(axis=0)
    center = (mx + mn) / 2
    return -center, max_dim / (mx - mn).max() * 0.9, keep


def transform(points, T):
    ph = np.concatenate([points, np.ones((len(points), 1))], 1)
    q = ph @ np.asarray(T, np.float64).T
    return q[:, :3] / q[:, 3:4]


def scene_bounds_worker(K, glcam_in_world, rgb, depth, mask, use_mask=True):
    xyz = depth2xyzmap(depth, K)
    valid = depth >= 0.1
    if use_mask:
        valid = valid & (mask > 0)
    pts = xyz[valid].reshape(-1, 3).astype(np.float64)
    if len(pts) == 0:
        return None
    colors = rgb[valid].reshape(-1, 3).astype(np.float64)
    if colors.max() > 1:
        colors = colors / 255.0
    p, c = voxel_down_sample(pts, colors, 0.01)
    keep = remove_statistical_outlier(p, 30, 2.0)
    return transform(p[keep], glcam_in_world @ GLCAM_IN_CVCAM), c[keep]


def compute_scene_bounds(glcam_in_worlds, K, rgbs, depths, masks, eps=0.06, min_samples=1):
    P, C = [], []
    for i in range(len(rgbs)):
        r = scene_bounds_worker(K, glcam_in_worlds[i], rgbs[i], depths[i], masks[i])
        if r is not None:
            P.append(r[0])
            C.append(r[1])
    p, c = voxel_down_sample(np.concatenate(P), np.concatenate(C), eps / 5)
    t, sc, keep = compute_translation_scales(p, eps=eps, min_samples=min_samples)
    tf = np.eye(4)
    tf[:3, 3] = t
    s = np.eye(4)
    s[:3, :3] *= sc
    return sc, t, p[keep], c[keep], transform(p[keep], s @ tf)
