"""GPU: nof_pose_forward / nof_pose_backward against torch autograd through the
oracle's PoseArray.get_matrices restatement (oracle/nerf_step.py pose_matrices,
nerf_helpers.py:127-154, pytorch3d se3_exp_map restated) and tf = T @ c2w
(nerf_runner.py:1050-1052): tf and the pose gradient within fp32 tolerance
(rtol 1e-5 / 1e-4), frame 0 identity with zero gradient, small-angle branch of
se3_exp_map (clamped norm) included."""
import math

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_pose_forward_backward_matches_autograd(cuda_device):
    from bundlesdf_amd import _lib
    from bundlesdf_amd.nerf_helpers import PoseArray
    dev = cuda_device
    F, R = 7, 5000
    g = torch.Generator().manual_seed(0)
    pa = PoseArray(F, 0.02 * 6.6, 20.0)
    data = torch.randn(F, 6, generator=g) * 0.5
    data[2] = 1e-4 * torch.randn(6, generator=g)          # clamped-norm branch
    pa.data.data.copy_(data)
    c2w = torch.eye(4).repeat(F, 1, 1)
    c2w[:, :3, :3] = torch.linalg.qr(torch.randn(F, 3, 3, generator=g))[0]
    c2w[:, :3, 3] = torch.randn(F, 3, generator=g)
    # reference: autograd on CPU
    from oracle import nerf_step as NS
    T = NS.pose_matrices(pa.data, torch.arange(F), pa.max_trans, pa.max_rot)
    tf = T @ c2w
    frames = torch.randint(0, F, (R,), generator=g)
    ray_grad = torch.randn(R, 12, generator=g)
    fg = torch.zeros(F, 12).index_add_(0, frames, ray_grad)
    gp, = torch.autograd.grad(tf[:, :3, :].reshape(F, 12), pa.data, fg)
    # device
    L = _lib.lib()
    d_data = pa.data.detach().to(dev).contiguous()
    d_c2w = c2w.to(dev).contiguous()
    tf_out = torch.empty(F, 16, device=dev)
    jac = torch.empty(F, 12, 6, device=dev)
    _lib.check(L.nof_pose_forward(_lib.ptr(d_data), _lib.ptr(d_c2w), F, float(pa.max_trans),
                                  float(pa.max_rot / 180.0 * math.pi), _lib.ptr(tf_out), _lib.ptr(jac),
                                  _lib.stream_of(d_data)), "pose_forward")
    rays = torch.zeros(R, 12)
    rays[:, 8] = frames.float()
    d_rays, d_rg = rays.to(dev), ray_grad.to(dev)
    d_fg = torch.zeros(F, 12, device=dev)      # scratch: zero on entry, left zero
    d_gp = torch.zeros(F, 6, device=dev)
    _lib.check(L.nof_pose_backward(_lib.ptr(d_rg), _lib.ptr(d_rays), R, _lib.ptr(jac), F, _lib.ptr(d_fg),
                                   _lib.ptr(d_gp), _lib.stream_of(d_rg)), "pose_backward")
    torch.cuda.synchronize()
    np.testing.assert_allclose(tf_out.cpu().view(F, 4, 4).numpy(), tf.detach().numpy(), rtol=1e-5, atol=1e-6)
    assert float(d_fg.abs().max()) == 0.0          # the per-frame sums were consumed and cleared
    np.testing.assert_allclose(d_gp.cpu().numpy(), gp.numpy(), rtol=1e-4, atol=1e-4)
    assert (d_gp[0] == 0).all() and (jac[0] == 0).all()
    # PoseArray.get_matrices on the device runs the same kernel (c2w = identity)
    pa_d = PoseArray(F, pa.max_trans, pa.max_rot).to(dev)
    pa_d.data.data.copy_(pa.data.data)
    ids = torch.tensor([3, 0, 5, 5, 1])
    np.testing.assert_allclose(pa_d.get_matrices(ids).cpu().numpy(), T[ids].detach().numpy(), rtol=1e-5, atol=1e-6)
    # and the host (CPU) evaluation used by the hand-off tools agrees with both
    np.testing.assert_allclose(pa.get_matrices(ids).numpy(), T[ids].detach().numpy(), rtol=1e-5, atol=1e-6)
