"""GPU: the NerfRunner drop-in trains end to end through the fused HIP path
(constructor -> octree -> ray pool -> train), exposes models['pose_array'],
and continues after add_new_frames (reuse_weights=True)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_nerf_runner_trains_and_adds_frames(cuda_device):
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.nerf_runner import NerfRunner
    seq = SY.make_sequence(4, seed=1)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"], n_step=40, N_rand=1024,
                         num_levels=16, amp=True)
    nr = NerfRunner(cfg, seq["rgbs"][:3], seq["depths"][:3], seq["masks"][:3], None, seq["poses"][:3], seq["K"],
                    build_octree_pcd=seq["octree_pts"])
    assert nr.rays.is_cuda and nr.rays.shape[1] == 12
    assert set(np.unique(nr.rays[:, 8].cpu().numpy()).astype(int)) == {0, 1, 2}
    losses = []
    for _ in range(3):
        nr.N_iters = 15
        out = nr.train()
        losses.append(float(out["loss_terms"][:4].sum()))
    assert np.isfinite(losses).all() and losses[-1] < losses[0], losses
    pa = nr.models["pose_array"]
    assert pa.data.shape == (3, 6) and torch.isfinite(pa.data).all()
    assert pa.get_matrices(torch.arange(3, device=cuda_device)).shape == (3, 4, 4)
    n_before = nr.rays.shape[0]
    nr.add_new_frames(seq["rgbs"][3:], seq["depths"][3:], seq["masks"][3:], None, seq["poses"], reuse_weights=True)
    assert nr.rays.shape[0] > n_before and nr.models["pose_array"].data.shape == (4, 6)
    nr.N_iters = 10
    out = nr.train()
    assert np.isfinite(float(out["loss_terms"][:4].sum()))
