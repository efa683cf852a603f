"""GPU: device ray-pool construction (nof_make_frame_rays via
bundlesdf_amd.ray_pool) against the reference's make_frame_rays (G5 golden,
tests/golden/ray_pool.npz) and against the numpy oracle (oracle/ray_pool.py)
on full 640x480 synthetic frames. Columns 0-9 (camera dir, rgb, depth, mask,
frame id, type) must be bit-exact and the row set / order identical; near/far
(float64 box test rounded to f32, the reference's float64 numpy/torch path)
within 2 ulp (rtol 2e-7) — the only freedom is the summation order of the
reference's 3x3 BLAS rotation."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "ray_pool.npz")


def _check(got, ref):
    got = got.cpu().numpy() if torch.is_tensor(got) else got
    assert got.shape == ref.shape, (got.shape, ref.shape)
    np.testing.assert_array_equal(got[:, :10], ref[:, :10])
    np.testing.assert_allclose(got[:, 10:], ref[:, 10:], rtol=2e-7, atol=0)


def test_pool_matches_reference_golden(cuda_device):
    from bundlesdf_amd.ray_pool import PointGrid, make_pool_rays
    g = np.load(GOLD)
    cfg = json.loads(str(g["cfg_json"]))
    occ = torch.from_numpy(g["occ"]).to(cuda_device)
    args = (range(3), g["images"], g["depths"], g["masks"], g["poses"], g["K"], cfg)
    got = make_pool_rays(*args, occ_masks=g["occ_masks"], occ=occ, device=cuda_device)
    _check(got, g["pool"])
    grid = PointGrid(g["cloud"], 0.02 * cfg["sc_factor"], cuda_device)
    den = make_pool_rays(*args, occ_masks=g["occ_masks"], occ=occ, point_grid=grid, device=cuda_device)
    _check(den, g["pool_denoised"])
    # frames one at a time (first_frame_id > 0 path) concatenate to the same pool
    parts = [make_pool_rays([f], *args[1:], occ_masks=g["occ_masks"], occ=occ, device=cuda_device)
             for f in range(3)]
    _check(torch.cat(parts), g["pool"])


def test_pool_full_frames_vs_oracle(cuda_device):
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.octree import OctreeManager
    from bundlesdf_amd.ray_pool import PointGrid, make_pool_rays
    from oracle import ray_pool as RP
    seq = SY.make_sequence(4, seed=3)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"])
    sc = cfg["sc_factor"]
    max_level = int(np.ceil(np.log2(2.0 / (cfg["octree_smallest_voxel_size"] * sc))))
    om = OctreeManager(torch.from_numpy(seq["octree_pts"]).float().to(cuda_device), max_level, dilate_radius=1)
    occ = om.occupancy(RP.trace_level(cfg))
    cloud = seq["octree_pts"][::3]
    ref = RP.build_pool(range(4), seq["rgbs"], seq["depths"], seq["masks"], seq["poses"], seq["K"], cfg,
                        occ=occ.cpu().numpy(), cloud=cloud)
    got = make_pool_rays(range(4), seq["rgbs"], seq["depths"], seq["masks"], seq["poses"], seq["K"], cfg, occ=occ,
                         point_grid=PointGrid(cloud, 0.02 * sc, cuda_device), device=cuda_device)
    assert len(ref) > 100000
    _check(got, ref)


def test_pool_edge_cases(cuda_device):
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.ray_pool import make_pool_rays
    from oracle import ray_pool as RP
    seq = SY.make_sequence(2, seed=4)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"], down_scale_ratio=2)
    masks = seq["masks"].copy()
    masks[1] = 0                                         # empty mask: no ray from frame 1
    rgbs, depths = seq["rgbs"][:, :37, :53], seq["depths"][:, :37, :53]   # ragged, non-multiple-of-64 frame
    masks = np.ascontiguousarray(masks[:, :37, :53])
    masks[0, 10:20, 10:20] = 1
    got = make_pool_rays([1], rgbs, depths, masks, seq["poses"], seq["K"], cfg, device=cuda_device)
    assert got.shape == (0, 12)
    got = make_pool_rays(range(2), rgbs, depths, masks, seq["poses"], seq["K"], cfg, device=cuda_device)
    ref = RP.build_pool(range(2), rgbs, depths, masks, seq["poses"], seq["K"], cfg)
    _check(got, ref)
    assert make_pool_rays([], rgbs, depths, masks, seq["poses"], seq["K"], cfg, device=cuda_device).shape == (0, 12)
    wide = np.zeros((1, 2, 5000, 3), np.float32)
    with pytest.raises(RuntimeError, match="frames up to"):
        make_pool_rays([0], wide, wide[..., :1], wide[..., :1], seq["poses"], seq["K"], cfg, device=cuda_device)
