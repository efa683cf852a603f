"""CPU tests of the NerfRunner drop-in's host logic (bundlesdf_amd/nerf_runner.py):
the DataLoader epoch semantics (:90-107), re-exports and config gating. The
ray pool (make_frame_rays) is built on the device: its oracle is checked in
test_oracle_ray_pool.py and the HIP path in test_gpu_ray_pool.py."""
import numpy as np
import torch

from bundlesdf_amd import nerf_runner as NR
from bundlesdf_amd import synthetic as SY


def _seq():
    return SY.make_sequence(2, seed=0)


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
    NR._check_supported(SY.default_cfg(sc_factor=1.0, translation=np.zeros(3), frame_features=2))   # global refine
    for over in (dict(frame_features=4), dict(N_importance=64), dict(i_embed=0)):
        cfg = SY.default_cfg(sc_factor=1.0, translation=np.zeros(3), **over)
        with pytest.raises(NotImplementedError):
            NR._check_supported(cfg)
