"""GPU parity of the drop-in boundary (gridencoder / common modules over the
libnof C ABI) against the CPU oracle, on identical seeded inputs.

Tolerances: forward fp32 and input-grad fp32 are bit-exact (the kernels
restate nvcc's FMA contraction explicitly); fp16 forward is bit-exact too
(c10::Half rounding restated); grid backward uses device atomics like the
reference, so only the summation order differs: rtol 1e-5 / atol 1e-6 (fp32)
and 2 half-ulps per add (fp16). Samplers are bit-exact."""
import numpy as np
import pytest
import torch

from oracle import kernels as K

pytestmark = pytest.mark.gpu


def _setup(D, L, C, H, T, fin, B, seed, dtype=torch.float32, spread=1.0):
    from bundlesdf_amd.grid import level_layout
    pls, offs = level_layout(D, L, C, H, T, fin)
    rng = np.random.default_rng(seed)
    x = rng.uniform(-0.02, 1.02, (B, D)).astype(np.float32)
    x[:8] = np.clip(x[:8], 0, 1)
    x[8] = 1.0
    x[9] = 0.0
    emb = rng.uniform(-spread, spread, (int(offs[-1]), C)).astype(np.float32)
    if dtype == torch.float16:
        emb = emb.astype(np.float16)
    return pls, offs, x, emb


CONFIGS = [(3, 16, 2, 16, 22, 128, 20000), (3, 4, 2, 16, 22, 128, 5000), (3, 16, 2, 16, 19, 512, 8000),
           (3, 8, 4, 8, 15, 64, 3000), (2, 6, 1, 4, 12, 64, 3000), (5, 3, 8, 4, 14, 16, 1000)]


@pytest.mark.parametrize("cfg", CONFIGS)
def test_grid_forward_fp32_bitexact(cfg, cuda_device):
    from bundlesdf_amd import gridencoder
    D, L, C, H, T, fin, B = cfg
    pls, offs, x, emb = _setup(D, L, C, H, T, fin, B, seed=1)
    S = np.log2(pls)
    o_out, o_dd = K.grid_encode_forward(x, emb, offs, S, H, calc_grad_inputs=True)
    xi = torch.from_numpy(x).to(cuda_device)
    e = torch.from_numpy(emb).to(cuda_device)
    of = torch.from_numpy(offs).to(cuda_device)
    out = torch.empty(L, B, C, device=cuda_device)
    dd = torch.empty(B, L * D * C, device=cuda_device)
    gridencoder.grid_encode_forward(xi, e, of, out, B, D, C, L, S, H, True, dd, 0, False)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(out.cpu().numpy(), o_out)
    np.testing.assert_array_equal(dd.cpu().numpy(), o_dd)


def test_grid_forward_fp16_matches_half_semantics(cuda_device):
    from bundlesdf_amd import gridencoder
    D, L, C, H, T, fin, B = 3, 16, 2, 16, 22, 128, 10000
    pls, offs, x, emb = _setup(D, L, C, H, T, fin, B, seed=2, dtype=torch.float16, spread=1e-2)
    S = np.log2(pls)
    o_out, o_dd = K.grid_encode_forward(x, emb, offs, S, H, calc_grad_inputs=True)
    out = torch.empty(L, B, C, device=cuda_device, dtype=torch.float16)
    dd = torch.empty(B, L * D * C, device=cuda_device, dtype=torch.float16)
    gridencoder.grid_encode_forward(torch.from_numpy(x).to(cuda_device), torch.from_numpy(emb).to(cuda_device),
                                    torch.from_numpy(offs).to(cuda_device), out, B, D, C, L, S, H, True, dd, 0, False)
    np.testing.assert_array_equal(out.cpu().numpy().view(np.uint16), o_out.view(np.uint16))
    np.testing.assert_array_equal(dd.cpu().numpy().view(np.uint16), o_dd.view(np.uint16))


@pytest.mark.parametrize("cfg", CONFIGS[:4])
def test_grid_backward_fp32(cfg, cuda_device):
    from bundlesdf_amd import gridencoder
    D, L, C, H, T, fin, B = cfg
    pls, offs, x, emb = _setup(D, L, C, H, T, fin, B, seed=3)
    S = np.log2(pls)
    _, o_dd = K.grid_encode_forward(x, emb, offs, S, H, calc_grad_inputs=True)
    g = np.random.default_rng(4).standard_normal((L, B, C)).astype(np.float32)
    o_gemb, o_gin = K.grid_encode_backward(g, x, offs, int(offs[-1]), S, H, calc_grad_inputs=True, dy_dx=o_dd)
    dev = cuda_device
    gemb = torch.zeros(int(offs[-1]), C, device=dev)
    gin = torch.zeros(B, D, device=dev)
    gridencoder.grid_encode_backward(torch.from_numpy(g).to(dev), torch.from_numpy(x).to(dev),
                                     torch.from_numpy(emb).to(dev), torch.from_numpy(offs).to(dev), gemb, B, D, C, L,
                                     S, H, True, torch.from_numpy(o_dd).to(dev), gin, 0, False)
    np.testing.assert_allclose(gemb.cpu().numpy(), o_gemb, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal(gin.cpu().numpy(), o_gin)


def test_grid_backward_fp16(cuda_device):
    from bundlesdf_amd import gridencoder
    D, L, C, H, T, fin, B = 3, 16, 2, 16, 22, 128, 4000
    pls, offs, x, emb = _setup(D, L, C, H, T, fin, B, seed=5, dtype=torch.float16, spread=1e-2)
    S = np.log2(pls)
    _, o_dd = K.grid_encode_forward(x, emb, offs, S, H, calc_grad_inputs=True)
    g = (np.random.default_rng(6).standard_normal((L, B, C)) * 0.1).astype(np.float16)
    o_gemb, o_gin = K.grid_encode_backward(g, x, offs, int(offs[-1]), S, H, calc_grad_inputs=True, dy_dx=o_dd)
    dev = cuda_device
    gemb = torch.zeros(int(offs[-1]), C, device=dev, dtype=torch.float16)
    gin = torch.zeros(B, D, device=dev, dtype=torch.float16)
    gridencoder.grid_encode_backward(torch.from_numpy(g).to(dev), torch.from_numpy(x).to(dev),
                                     torch.from_numpy(emb).to(dev), torch.from_numpy(offs).to(dev), gemb, B, D, C, L,
                                     S, H, True, torch.from_numpy(o_dd).to(dev), gin, 0, False)
    np.testing.assert_allclose(gemb.cpu().numpy().astype(np.float32), o_gemb.astype(np.float32), rtol=4e-3,
                               atol=2e-4)
    np.testing.assert_array_equal(gin.cpu().numpy().view(np.uint16), o_gin.view(np.uint16))


def test_grid_module_autograd(cuda_device):
    """GridEncoder (grid.py:106-171 API) fwd+bwd through autograd vs the oracle."""
    from bundlesdf_amd.grid import GridEncoder
    torch.manual_seed(0)
    enc = GridEncoder(input_dim=3, n_levels=16, level_dim=2, base_resolution=16, log2_hashmap_size=22,
                      desired_resolution=128).to(cuda_device)
    assert enc.embeddings.shape == (6512256, 2) and enc.out_dim == 32
    x = (torch.rand(3000, 3, device=cuda_device) * 2 - 1).requires_grad_(True)
    y = enc(x)
    g = torch.randn_like(y)
    y.backward(g)
    S = np.log2(enc.per_level_scale)
    x01 = ((x.detach() + 1) / 2).cpu().numpy()
    emb = enc.embeddings.detach().cpu().numpy()
    offs = enc.offsets.cpu().numpy()
    o_out, o_dd = K.grid_encode_forward(x01, emb, offs, S, 16, calc_grad_inputs=True)
    np.testing.assert_array_equal(y.detach().cpu().numpy(), o_out.transpose(1, 0, 2).reshape(3000, 32))
    gl = g.view(3000, 16, 2).permute(1, 0, 2).contiguous().cpu().numpy()
    o_gemb, o_gin = K.grid_encode_backward(gl, x01, offs, emb.shape[0], S, 16, calc_grad_inputs=True, dy_dx=o_dd)
    np.testing.assert_allclose(enc.embeddings.grad.cpu().numpy(), o_gemb, rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(x.grad.cpu().numpy(), o_gin * 0.5, rtol=1e-6, atol=1e-7)


def test_grid_errors(cuda_device):
    from bundlesdf_amd import gridencoder
    dev = cuda_device
    x = torch.rand(10, 3, device=dev)
    e = torch.rand(100, 3, device=dev)
    offs = torch.tensor([0, 100], dtype=torch.int32, device=dev)
    out = torch.empty(1, 10, 3, device=dev)
    with pytest.raises(RuntimeError, match="C must be 1, 2, 4, or 8"):
        gridencoder.grid_encode_forward(x, e, offs, out, 10, 3, 3, 1, 0.0, 4, False, out, 0, False)
    with pytest.raises(RuntimeError, match="must be a CUDA tensor"):
        gridencoder.grid_encode_forward(x.cpu(), e, offs, out, 10, 3, 3, 1, 0.0, 4, False, out, 0, False)
    with pytest.raises(RuntimeError, match="int tensor"):
        gridencoder.grid_encode_forward(x, e, offs.long(), out, 10, 3, 3, 1, 0.0, 4, False, out, 0, False)


def test_sampler_bitexact(cuda_device):
    from bundlesdf_amd import common
    rng = np.random.default_rng(9)
    R, Kb, S = 777, 12, 128
    z_in_out = np.zeros((R, Kb, 2), np.float32)
    totals = np.zeros(R, np.float32)
    for r in range(R):
        n = rng.integers(0, Kb + 1)
        if r % 50 == 0:
            n = Kb
        t = 0.5 + rng.uniform(0, 0.2)
        for k in range(n):
            a = t + rng.uniform(0, 0.1)
            b = a + rng.uniform(0, 0.3)
            z_in_out[r, k] = (a, b)
            t = b
        totals[r] = (z_in_out[r, :, 1] - z_in_out[r, :, 0]).sum()
    u = (np.sort(rng.uniform(0, 1, (R, S)), 1) * totals[:, None]).astype(np.float32)
    o_z, o_err = K.sample_occupied(z_in_out, u)
    dev = cuda_device
    z = torch.zeros(R, S, device=dev)
    common.reset_sampler_errors(dev)
    common.sampleRaysUniformOccupiedVoxels(torch.from_numpy(z_in_out).to(dev), torch.from_numpy(u).to(dev), z)
    np.testing.assert_array_equal(z.cpu().numpy(), o_z)
    assert common.sampler_error_count(dev) == o_err


def test_postprocess_exact(cuda_device):
    from bundlesdf_amd import common
    rng = np.random.default_rng(10)
    R = 500
    counts = rng.integers(0, 9, R)
    ray_index = np.repeat(np.arange(R), counts).astype(np.int64)
    M = len(ray_index)
    depth = rng.uniform(0.1, 3, (M, 2)).astype(np.float32)
    depth[::7, 1] = depth[::7, 0] + 5e-5
    uniq, start, cnt = np.unique(ray_index, return_index=True, return_counts=True)
    o = K.postprocess_octree(ray_index, depth, uniq, start, int(cnt.max()), R)
    dev = cuda_device
    out = common.postprocessOctreeRayTracing(torch.from_numpy(ray_index).to(dev), torch.from_numpy(depth).to(dev),
                                             torch.from_numpy(uniq.astype(np.int64)).to(dev),
                                             torch.from_numpy(start.astype(np.int64)).to(dev), int(cnt.max()), R)
    assert out.device == dev
    np.testing.assert_array_equal(out.cpu().numpy(), o)


def test_octree_ray_trace_matches_oracle(cuda_device):
    from bundlesdf_amd import octree
    rng = np.random.default_rng(11)
    N = 16
    occ = (rng.uniform(size=(N, N, N)) < 0.3).astype(np.uint8)
    o = rng.normal(size=(4000, 3))
    o = (o / np.linalg.norm(o, axis=1, keepdims=True) * 3).astype(np.float32)
    d = rng.uniform(-0.7, 0.7, (4000, 3)) - o
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    d[:10, 1:] = 0
    d[:10, 0] = 1
    o[:10, 0] = -3
    ref, cnt = K.octree_ray_trace(occ, o, d, 3 * N)
    dev = cuda_device
    out, counts = octree.ray_trace_dense(torch.from_numpy(occ).to(dev), torch.from_numpy(o).to(dev),
                                         torch.from_numpy(d).to(dev), 3 * N)
    np.testing.assert_array_equal(counts.cpu().numpy(), cnt)
    np.testing.assert_array_equal(out.cpu().numpy(), ref)
