"""CPU: the hand-off oracle (oracle/scene_bounds.py) against the G6 golden —
the reference's own Utils.depth2xyzmap, tool.find_biggest_cluster,
tool.compute_translation_scales (sklearn DBSCAN) — and the host-side
get_optimized_poses_in_real_world of bundlesdf_amd.handoff (PoseArray on CPU)
against the reference's Utils.get_optimized_poses_in_real_world."""
import os

import numpy as np
import pytest
import torch

from oracle import scene_bounds as SB

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "handoff.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def test_depth2xyzmap(g):
    np.testing.assert_array_equal(SB.depth2xyzmap(g["depth"], g["K"]), g["xyz"])


def test_biggest_cluster_and_scales(g):
    for ms in (1, 3):
        _, keep = SB.find_biggest_cluster(g["cloud"], eps=0.06, min_samples=ms)
        np.testing.assert_array_equal(keep, g[f"keep_ms{ms}"])
    t, sc, keep = SB.compute_translation_scales(g["cloud"], eps=0.06, min_samples=1)
    np.testing.assert_array_equal(t, g["translation"])
    assert sc == g["sc_factor"][0]
    np.testing.assert_array_equal(keep, g["keep_ts"])


def test_voxel_and_outlier_restatement():
    rng = np.random.default_rng(0)
    pts = np.concatenate([rng.normal(0, 0.05, (400, 3)), rng.uniform(-2, 2, (5, 3))])
    p, c = SB.voxel_down_sample(pts, pts * 0.5, 0.02)
    assert len(p) < len(pts) and np.allclose(c, p * 0.5)
    vmin = pts.min(0) - 0.01
    vid = np.floor((p - vmin) / 0.02)                   # each mean lies in its own voxel
    assert len(np.unique(vid, axis=0)) == len(p)
    keep = SB.remove_statistical_outlier(pts, 30, 2.0)
    assert set(range(400, 405)).isdisjoint(keep) and len(keep) > 350


def test_optimized_poses_host(g):
    from bundlesdf_amd.handoff import get_optimized_poses_in_real_world
    from bundlesdf_amd.nerf_helpers import PoseArray
    pa = PoseArray(5, max_trans=0.02 * 6.6, max_rot=20)
    pa.data.data = torch.from_numpy(g["pose_data"])
    opt, off = get_optimized_poses_in_real_world(g["poses"], pa, 6.6, np.array([0.01, -0.02, 0.03]))
    assert opt.dtype == np.float32
    np.testing.assert_allclose(opt, g["opt_poses"], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(off, g["offset"], rtol=1e-5, atol=1e-6)
