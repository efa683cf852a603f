"""GPU: the device hand-off path (bundlesdf_amd.handoff: voxel down-sampling via
nof_segment_mean, statistical-outlier statistic via nof_knn_mean_dist, DBSCAN
via nof_dbscan) against the oracle (oracle/scene_bounds.py: open3d's published
algorithms restated, sklearn DBSCAN) and the G6 golden (the reference's own
tool.py / Utils.py functions). Voxel means, kept indices and cluster masks are
exact; kNN mean distances within 1e-12 (summation order)."""
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "handoff.npz")


def test_voxel_down_sample_exact(cuda_device):
    from bundlesdf_amd.handoff import PointCloud
    from oracle import scene_bounds as SB
    rng = np.random.default_rng(1)
    pts = rng.normal(0, 0.1, (20000, 3))
    col = rng.uniform(0, 1, (20000, 3))
    pc = PointCloud(pts, col, device=cuda_device)
    for vox in (0.01, 0.037):
        d = pc.voxel_down_sample(vox)
        p, c = SB.voxel_down_sample(pts, col, vox)
        np.testing.assert_array_equal(d.points, p)
        np.testing.assert_array_equal(d.colors, c)
    assert len(PointCloud(np.zeros((0, 3)), device=cuda_device).voxel_down_sample(0.01)) == 0


def test_statistical_outlier_and_knn(cuda_device):
    from bundlesdf_amd import _lib
    from bundlesdf_amd.handoff import PointCloud
    from oracle import scene_bounds as SB
    rng = np.random.default_rng(2)
    pts = np.concatenate([rng.normal(0, 0.05, (3000, 3)), rng.uniform(-1, 1, (30, 3)), np.zeros((2, 3))])
    for k in (1, 5, 30):
        t = torch.from_numpy(pts).to(cuda_device)
        d = torch.empty(len(pts), dtype=torch.float64, device=cuda_device)
        _lib.check(_lib.lib().nof_knn_mean_dist(_lib.ptr(t), len(pts), k, _lib.ptr(d), _lib.stream_of(t)))
        np.testing.assert_allclose(d.cpu().numpy(), SB.knn_mean_dist(pts, k), rtol=1e-12, atol=1e-15)
    pc, ind = PointCloud(pts, device=cuda_device).remove_statistical_outlier(30, 2.0)
    np.testing.assert_array_equal(np.array(ind), SB.remove_statistical_outlier(pts, 30, 2.0))
    np.testing.assert_array_equal(pc.points, pts[ind])
    # fewer points than neighbours: k clamps to n
    small = pts[:7]
    _, ind = PointCloud(small, device=cuda_device).remove_statistical_outlier(30, 2.0)
    np.testing.assert_array_equal(np.array(ind), SB.remove_statistical_outlier(small, 30, 2.0))


def test_dbscan_matches_sklearn_and_reference(cuda_device):
    from bundlesdf_amd.handoff import compute_translation_scales, dbscan_labels, find_biggest_cluster
    from oracle import scene_bounds as SB
    g = np.load(GOLD)
    pts = g["cloud"]
    np.testing.assert_array_equal(dbscan_labels(pts, 0.06, 1, cuda_device), SB.dbscan_labels(pts, 0.06, 1))
    lab = dbscan_labels(pts, 0.06, 3, cuda_device)
    ref = SB.dbscan_labels(pts, 0.06, 3)
    np.testing.assert_array_equal(lab == -1, ref == -1)      # noise / core-reachable sets agree
    for ms in (1, 3):
        _, keep = find_biggest_cluster(pts, 0.06, ms, cuda_device)
        np.testing.assert_array_equal(keep, g[f"keep_ms{ms}"])
    t, sc, keep = compute_translation_scales(pts, eps=0.06, min_samples=1, device=cuda_device)
    np.testing.assert_array_equal(t, g["translation"])
    assert sc == g["sc_factor"][0]
    # a larger random cloud: chain-like components exercise several union-find rounds
    rng = np.random.default_rng(3)
    walk = np.cumsum(rng.normal(0, 0.01, (5000, 3)), 0)
    big = np.concatenate([walk, rng.uniform(-3, 3, (3000, 3))])
    np.testing.assert_array_equal(dbscan_labels(big, 0.05, 1, cuda_device), SB.dbscan_labels(big, 0.05, 1))


def test_depth2xyz_and_scene_bounds(cuda_device):
    from bundlesdf_amd import handoff as HO
    from bundlesdf_amd import synthetic as SY
    from oracle import scene_bounds as SB
    g = np.load(GOLD)
    np.testing.assert_array_equal(HO.depth2xyzmap(g["depth"], g["K"], cuda_device).cpu().numpy(), g["xyz"])
    poses = SY.camera_poses(3, seed=5)
    rgbs, depths, masks = [], [], []
    for T in poses:
        rgb, depth, mask = SY.render_frame(T)
        rgbs.append(rgb)
        depths.append(depth)
        masks.append(mask)
    rgbs, depths, masks = np.stack(rgbs), np.stack(depths), np.stack(masks)
    sc, t, real, real_c, norm = SB.compute_scene_bounds(poses, SY.K_CAM, rgbs, depths, masks)
    sc2, t2, pcd_real, pcd_norm = HO.compute_scene_bounds(None, poses, SY.K_CAM, rgbs=rgbs, depths=depths,
                                                          masks=masks, eps=0.06, min_samples=1, device=cuda_device)
    assert abs(sc2 - sc) <= 1e-12 * sc
    np.testing.assert_allclose(t2, t, rtol=0, atol=1e-12)
    assert pcd_real.points.shape == real.shape
    np.testing.assert_allclose(pcd_real.points, real, rtol=0, atol=1e-12)
    np.testing.assert_allclose(pcd_real.colors, real_c, rtol=0, atol=1e-12)
    np.testing.assert_allclose(pcd_norm.points, norm, rtol=0, atol=1e-9)
    assert np.abs(pcd_norm.points).max() < 1.0


def test_optimized_poses_device(cuda_device):
    from bundlesdf_amd.handoff import get_optimized_poses_in_real_world
    from bundlesdf_amd.nerf_helpers import PoseArray
    g = np.load(GOLD)
    pa = PoseArray(5, max_trans=0.02 * 6.6, max_rot=20).to(cuda_device)
    pa.data.data = torch.from_numpy(g["pose_data"]).to(cuda_device)
    opt, off = get_optimized_poses_in_real_world(g["poses"], pa, 6.6, np.array([0.01, -0.02, 0.03]))
    np.testing.assert_allclose(opt, g["opt_poses"], rtol=1e-5, atol=1e-6)
