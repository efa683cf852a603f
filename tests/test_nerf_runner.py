"""CPU tests of the NerfRunner drop-in's host logic (bundlesdf_amd/nerf_runner.py):
ray-pool construction (make_frame_rays, nerf_runner.py:244-314), the box
near/far filter (:39-65) and the DataLoader epoch semantics (:90-107)."""
import numpy as np
import torch

from bundlesdf_amd import nerf_runner as NR
from bundlesdf_amd import synthetic as SY


def _seq():
    return SY.make_sequence(2, seed=0)


def test_make_frame_rays_layout_and_filters():
    seq = _seq()
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"])
    for f in range(2):
        r = NR.make_frame_rays(f, seq["rgbs"], seq["depths"], seq["masks"], seq["poses"], seq["K"], cfg)
        assert r.dtype == np.float32 and r.shape[1] == 12
        assert (r[:, 8] == f).all() and (r[:, 9] == 0).all()
        assert (r[:, 10] <= r[:, 11]).all() and (r[:, 10] >= 0).all()
        # every ray is inside the dilated mask: object pixels (mask 1) are a strict subset
        n_obj = int((seq["masks"][f] > 0).sum())
        assert (r[:, 7] > 0).sum() == n_obj
        assert len(r) > n_obj
        # rgb / depth columns are the frame's pixels
        assert r[:, 3:6].min() >= 0 and r[:, 3:6].max() <= 1
    # frame 0 uses the 100 px dilation, others 60 px
    r0 = NR.make_frame_rays(0, seq["rgbs"], seq["depths"], seq["masks"], seq["poses"], seq["K"], cfg)
    r1 = NR.make_frame_rays(1, seq["rgbs"], seq["depths"], seq["masks"], seq["poses"], seq["K"], cfg)
    assert len(r0) - int((r0[:, 7] > 0).sum()) > len(r1) - int((r1[:, 7] > 0).sum())


def test_near_far_box_filter():
    cfg = {}
    T = np.eye(4)
    T[:3, 3] = [0, 0, 3.0]                    # camera at z=3 looking down -z (GL)
    rays = np.zeros((3, 10), np.float32)
    rays[0, :3] = [0, 0, -1]                  # hits the cube: t in [2, 4]
    rays[1, :3] = [1, 0, -0.01]               # misses
    rays[2, :3] = [0.2, 0.1, -1]
    out = NR.compute_near_far_and_filter_rays(T, rays, cfg)
    assert out.shape == (2, 12)
    np.testing.assert_allclose(out[0, 10:], [2.0, 4.0], rtol=1e-6)
    assert out[1, 10] > 0 and out[1, 11] > out[1, 10]


def test_dataloader_epochs():
    rays = torch.arange(10).float()[:, None]
    g = torch.Generator()
    g.manual_seed(0)
    dl = NR.DataLoader(rays, 4, generator=g)
    a, b = dl.next_ids(), dl.next_ids()
    assert len(a) == 4 and len(b) == 4 and not set(a.tolist()) & set(b.tolist())
    c = dl.next_ids()                           # 8 + 4 >= 10 -> reshuffle, first slice of a new perm
    assert dl.pos == 4 and len(set(c.tolist())) == 4
    batch = next(dl)
    assert batch.shape == (4, 1)


def test_reexports_for_bundlesdf():
    # bundlesdf.py does `from nerf_runner import *` and uses preprocess_data
    ns = {}
    exec("from bundlesdf_amd.nerf_runner import *", ns)
    for name in ("NerfRunner", "preprocess_data", "DataLoader", "BAD_DEPTH"):
        assert name in ns


def test_unsupported_configs_fail_loudly():
    import pytest
    for over in (dict(frame_features=2), dict(N_importance=64), dict(i_embed=0)):
        cfg = SY.default_cfg(sc_factor=1.0, translation=np.zeros(3), **over)
        with pytest.raises(NotImplementedError):
            NR._check_supported(cfg)
