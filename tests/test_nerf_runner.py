"""CPU tests of the NerfRunner drop-in's host logic (bundlesdf_amd/nerf_runner.py):
the DataLoader epoch semantics (:90-107), re-exports and config gating. The
ray pool (make_frame_rays) is built on the device: its oracle is checked in
test_oracle_ray_pool.py and the HIP path in test_gpu_ray_pool.py."""
import numpy as np
import torch

from bundlesdf_amd import nerf_runner as NR
from bundlesdf_amd import synthetic as SY


def _reference_lr_trace(cfg, base, n):
    """The reference's learning rate per step: Adam runs with the group lr, then
    schedule_lr (nerf_runner.py:577-581) fires after steps with global_step % 10 == 0
    and global_step > 0 (:761-762), lr = init * decay ^ (global_step / N_iters)."""
    lr, out, n_iters = base, [], cfg["n_step"] + 1
    for gs in range(n):
        out.append(lr)
        if gs % 10 == 0 and gs > 0:
            lr = base * cfg["decay_rate"] ** (float(gs) / n_iters)
    return out


def test_lr_schedule_matches_reference():
    from bundlesdf_amd.fused import lr_at
    for n_step in (24, 500, 2000):
        cfg = SY.default_cfg(sc_factor=1.0, translation=np.zeros(3), n_step=n_step)
        want = _reference_lr_trace(cfg, 0.01, 45)
        got = [lr_at(cfg, gs, 0.01) for gs in range(45)]
        assert got == want


def test_truncation_schedule_matches_oracle():
    from bundlesdf_amd.fused import truncation
    from oracle import nerf_step as NS
    for kind in ("", "linear", "exp"):
        cfg = SY.default_cfg(sc_factor=3.7, translation=np.zeros(3), trunc_decay_type=kind, trunc_start=0.05,
                             trunc=0.01, n_step=200)
        vals = [truncation(cfg, gs) for gs in range(0, 201, 7)]
        assert vals == [NS.truncation(cfg, gs) for gs in range(0, 201, 7)]
        assert vals[-1] >= 0.01 * 3.7 - 1e-12
        if kind:
            assert vals[0] == 0.05 * 3.7 and all(a >= b for a, b in zip(vals, vals[1:]))


def _seq():
    return SY.make_sequence(2, seed=0)


def test_dataloader_epochs():
    rays = torch.arange(10).float()[:, None]
    torch.manual_seed(0)
    dl = NR.DataLoader(rays, 4)
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
    for over in (dict(frame_features=4), dict(N_importance=64), dict(i_embed=0), dict(depth_weight=0.1),
                 dict(eikonal_weight=0.1), dict(trunc_decay_type="cosine"), dict(mode="density"),
                 dict(finest_res=2048)):
        cfg = SY.default_cfg(sc_factor=1.0, translation=np.zeros(3), **over)
        with pytest.raises(NotImplementedError):
            NR._check_supported(cfg)
