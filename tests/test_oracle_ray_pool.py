"""CPU: the ray-pool oracle (oracle/ray_pool.py) against the G5 golden — the
reference's own NerfRunner.make_frame_rays (nerf_runner.py:244-314) run on the
same frames (tests/golden/make_golden.py gen_ray_pool) — and the host-side
compute_near_far_and_filter_rays re-export."""
import json
import os

import numpy as np
import pytest

from oracle import ray_pool as RP

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ray_pool.npz")


@pytest.fixture(scope="module")
def g():
    return np.load(GOLD)


def _cfg(g):
    return json.loads(str(g["cfg_json"]))


def test_oracle_matches_reference_make_frame_rays(g):
    cfg = _cfg(g)
    got = RP.build_pool(range(len(g["images"])), g["images"], g["depths"], g["masks"], g["poses"], g["K"], cfg,
                        occ_masks=g["occ_masks"], occ=g["occ"], cloud=None)
    ref = g["pool"]
    assert got.shape == ref.shape
    np.testing.assert_array_equal(got[:, :10], ref[:, :10])
    np.testing.assert_allclose(got[:, 10:], ref[:, 10:], rtol=2e-7, atol=0)


def test_oracle_denoise(g):
    cfg = _cfg(g)
    den = RP.denoise(g["pool"].astype(np.float64), g["poses"], g["cloud"], cfg).astype(np.float32)
    np.testing.assert_array_equal(den, g["pool_denoised"])
    assert 0 < len(den) < len(g["pool"])


def test_pool_semantics(g):
    """Row order (frame-major, row-major pixels), only type-0 rays, frame 0 uses the
    100 px dilation (more background rays than the others), occluded pixels absent."""
    pool, counts = g["pool"], g["frame_counts"]
    assert counts.sum() == len(pool)
    fid = pool[:, 8].astype(int)
    assert (np.diff(fid) >= 0).all() and (pool[:, 9] == 0).all()
    assert (pool[:, 10] <= pool[:, 11]).all() and (pool[:, 10] >= 0).all()
    bg = [(pool[fid == f, 7] == 0).sum() for f in range(3)]
    assert bg[0] > bg[1] and bg[0] > bg[2]
    # occluded rectangle of frame 2 (rows 40:70, cols 60:100) contributes no ray
    K = g["K"]
    u = np.rint(pool[fid == 2, 0] * K[0, 0] + K[0, 2]).astype(int)
    v = np.rint(-pool[fid == 2, 1] * K[1, 1] + K[1, 2]).astype(int)
    assert not ((v >= 40) & (v < 70) & (u >= 60) & (u < 100)).any()


def test_near_far_box_filter():
    from bundlesdf_amd import nerf_runner as NR
    cfg = {"bounding_box": [[-1, -1, -1], [1, 1, 1]]}
    T = np.eye(4)
    T[:3, 3] = [0, 0, 3.0]                    # camera at z=3 looking down -z (GL)
    rays = np.zeros((3, 10), np.float64)
    rays[0, :3] = [0, 0, -1]                  # hits the cube: t in [2, 4]
    rays[1, :3] = [1, 0, -0.01]               # misses
    rays[2, :3] = [0.2, 0.1, -1]
    out = NR.compute_near_far_and_filter_rays(T, rays, cfg)
    assert out.shape == (2, 12)
    np.testing.assert_allclose(out[0, 10:], [2.0, 4.0], rtol=1e-6)
    assert out[1, 10] > 0 and out[1, 11] > out[1, 10]
    ref = RP.near_far_filter(T, rays, cfg)
    np.testing.assert_allclose(out, ref, rtol=1e-12)
