"""CPU: pin the grid-encoder oracle (oracle/grid_oracle.c) and the host-side
layout of bundlesdf_amd.grid against the reference's own Python
(tests/golden/grid_layout.npz) and against algebraic properties of
gridencoder.cu:106-365 (the CUDA source itself is unbuildable here)."""
import os

import numpy as np
import pytest

from oracle import kernels as K
from bundlesdf_amd.grid import level_layout


@pytest.fixture(scope="module")
def layout(golden_dir):
    return np.load(os.path.join(golden_dir, "grid_layout.npz"))


def _cfgs(layout):
    i = 0
    while f"cfg{i}" in layout:
        yield i, [int(v) for v in layout[f"cfg{i}"]]
        i += 1


def test_offsets_match_reference_python(layout):
    for i, (D, L, C, H, T, fin) in _cfgs(layout):
        pls, offs = level_layout(D, L, C, H, T, fin)
        np.testing.assert_array_equal(offs, layout[f"offsets{i}"])
        assert pls == layout[f"per_level_scale{i}"][0]
        assert int(offs[-1]) * C == int(layout[f"n_params{i}"][0])


def test_kernel_resolution_trap():
    """at L=16/finest=128 the kernel's float32 resolution is 32/64/128 at
    levels 5/10/15 while grid.py's float64 layout uses 33/65/129."""
    pls, offs = level_layout(3, 16, 2, 16, 22, 128)
    sc, res = K.level_params(16, np.float32(np.log2(pls)), 16)
    assert list(res) == [16, 19, 22, 25, 28, 32, 37, 43, 49, 56, 64, 74, 85, 98, 112, 128]
    py_res = [int(np.ceil(16 * pls ** i)) for i in range(16)]
    assert (py_res[5], py_res[10], py_res[15]) == (33, 65, 129)
    # every level is dense at this config: (res+1)^3 fits the level's rows
    rows = np.diff(offs)
    assert all((int(r) + 1) ** 3 <= int(n) for r, n in zip(res, rows))


def _table(offs, C, seed=0, dtype=np.float32):
    rng = np.random.default_rng(seed)
    return rng.uniform(-1, 1, size=(int(offs[-1]), C)).astype(dtype)


def test_forward_partition_of_unity():
    """Constant table -> every in-range encoding equals the constant (trilinear weights sum to 1)."""
    pls, offs = level_layout(3, 6, 2, 4, 12, 64)
    emb = np.full((int(offs[-1]), 2), 0.375, np.float32)
    rng = np.random.default_rng(1)
    x = rng.uniform(0, 1, size=(500, 3)).astype(np.float32)
    out, _ = K.grid_encode_forward(x, emb, offs, np.log2(pls), 4)
    np.testing.assert_allclose(out, 0.375, rtol=0, atol=2e-7)


def test_forward_oob_and_nodes():
    pls, offs = level_layout(3, 4, 2, 8, 19, 32)
    emb = _table(offs, 2)
    x = np.array([[-1e-3, 0.5, 0.5], [0.5, 1.0001, 0.2], [0, 0, 0], [1, 1, 1]], np.float32)
    out, dydx = K.grid_encode_forward(x, emb, offs, np.log2(pls), 8, calc_grad_inputs=True)
    assert np.all(out[:, 0] == 0) and np.all(out[:, 1] == 0)
    assert np.all(dydx[0] == 0) and np.all(dydx[1] == 0)
    # x=0 maps to pos=0.5 (align_corners=False): average of corner rows 0 and 1 in x, etc.
    assert np.all(np.isfinite(out))


def test_dense_index_formula_level0():
    """Level 0 (dense): a point exactly between grid nodes reads the expected 8 rows."""
    pls, offs = level_layout(3, 2, 1, 4, 12, 8)
    sc, res = K.level_params(2, np.float32(np.log2(pls)), 4)
    emb = np.zeros((int(offs[-1]), 1), np.float32)
    r = int(res[0]) + 1
    gx, gy, gz = 1, 2, 0
    for dx in (0, 1):
        for dy in (0, 1):
            for dz in (0, 1):
                emb[(gx + dx) + (gy + dy) * r + (gz + dz) * r * r, 0] = 8.0
    # choose x so that pos = x*scale + 0.5 = g + 0.5 exactly
    x = np.array([[(gx + 0.0) / sc[0], (gy + 0.0) / sc[0], (gz + 0.0) / sc[0]]], np.float32)
    out, _ = K.grid_encode_forward(x, emb, offs, np.log2(pls), 4)
    assert abs(out[0, 0, 0] - 8.0) < 1e-5


def test_hash_levels_use_fast_hash():
    """Config with hashed fine levels: encoding of a table equal to row index mod prime structure
    is finite and different rows are reached (sanity of the hash branch)."""
    pls, offs = level_layout(3, 16, 2, 16, 19, 512)
    sc, res = K.level_params(16, np.float32(np.log2(pls)), 16)
    rows = np.diff(offs)
    hashed = [l for l in range(16) if (int(res[l]) + 1) ** 3 > int(rows[l])]
    assert len(hashed) > 0
    emb = _table(offs, 2, seed=3)
    x = np.random.default_rng(2).uniform(0, 1, (300, 3)).astype(np.float32)
    out, _ = K.grid_encode_forward(x, emb, offs, np.log2(pls), 16)
    assert np.all(np.isfinite(out)) and np.abs(out[hashed[-1]]).max() > 0


def test_dydx_matches_finite_difference():
    pls, offs = level_layout(3, 4, 2, 8, 19, 32)
    emb = _table(offs, 2, seed=5).astype(np.float64).astype(np.float32)
    rng = np.random.default_rng(7)
    x = rng.uniform(0.1, 0.9, (64, 3)).astype(np.float32)
    out, dydx = K.grid_encode_forward(x, emb, offs, np.log2(pls), 8, calc_grad_inputs=True)
    L, B, C = out.shape
    dd = dydx.reshape(B, L, 3, C)
    h = 1e-3
    for d in range(3):
        xp, xm = x.copy(), x.copy()
        xp[:, d] += h
        xm[:, d] -= h
        op, _ = K.grid_encode_forward(xp, emb, offs, np.log2(pls), 8)
        om, _ = K.grid_encode_forward(xm, emb, offs, np.log2(pls), 8)
        fd = (op.astype(np.float64) - om) / (2 * h)           # [L,B,C]
        an = dd[:, :, d, :].transpose(1, 0, 2)
        # piecewise-linear: FD is exact unless the stencil crosses a cell face
        ok = np.isclose(fd, an, rtol=1e-2, atol=5e-2)
        assert ok.mean() > 0.9


def test_backward_partition_and_input_grad():
    pls, offs = level_layout(3, 5, 2, 8, 19, 64)
    rng = np.random.default_rng(11)
    B = 256
    x = rng.uniform(0, 1, (B, 3)).astype(np.float32)
    x[:4] = [[1.2, 0.5, 0.5], [0.5, -0.1, 0.5], [0.3, 0.3, 0.3], [0.9, 0.1, 0.4]]
    emb = _table(offs, 2, seed=12)
    out, dydx = K.grid_encode_forward(x, emb, offs, np.log2(pls), 8, calc_grad_inputs=True)
    g = rng.standard_normal(out.shape).astype(np.float32)
    gemb, gin = K.grid_encode_backward(g, x, offs, int(offs[-1]), np.log2(pls), 8, calc_grad_inputs=True,
                                       dy_dx=dydx)
    inb = np.all((x >= 0) & (x <= 1), axis=1)
    # sum of scattered grads per level/channel equals sum of incoming grads (weights sum to 1)
    for l in range(out.shape[0]):
        seg = gemb[offs[l]:offs[l + 1]]
        np.testing.assert_allclose(seg.sum(0), g[l][inb].sum(0), rtol=1e-4, atol=1e-4)
    # linearity: <grad_out, enc(E)> == <grad_emb, E>
    np.testing.assert_allclose((g * out).sum(), (gemb * emb).sum(), rtol=1e-4)
    # input grad = sum_l,c g * dy_dx
    L, B_, C = out.shape
    ref = np.einsum("lbc,bldc->bd", g.astype(np.float64), dydx.reshape(B_, L, 3, C).astype(np.float64))
    np.testing.assert_allclose(gin, ref, rtol=1e-4, atol=1e-5)


def test_half_path_close_to_float():
    pls, offs = level_layout(3, 6, 2, 8, 19, 64)
    emb = (_table(offs, 2, seed=4) * 1e-2).astype(np.float16)
    x = np.random.default_rng(8).uniform(0, 1, (200, 3)).astype(np.float32)
    oh, dh = K.grid_encode_forward(x, emb, offs, np.log2(pls), 8, calc_grad_inputs=True)
    of, df = K.grid_encode_forward(x, emb.astype(np.float32), offs, np.log2(pls), 8, calc_grad_inputs=True)
    assert oh.dtype == np.float16
    np.testing.assert_allclose(oh.astype(np.float32), of, rtol=0, atol=2e-5)
    np.testing.assert_allclose(dh.astype(np.float32), df, rtol=2e-2, atol=2e-3)
