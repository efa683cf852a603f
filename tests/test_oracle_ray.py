"""CPU: pin the ray-sampling oracle (oracle/ray_oracle.c) — the restatement of
common.cu:40-167 — with the known-answer vectors recorded in SURVEY.md §8c
(produced there from the reference kernel bodies) and edge cases; check the
(parity-unpinned) dense ray trace against analytic geometry."""
import numpy as np

from oracle import kernels as K


def _pad(boxes, K_):
    out = np.zeros((len(boxes), K_, 2), np.float32)
    for i, b in enumerate(boxes):
        if len(b):
            out[i, :len(b)] = b
    return out


def test_sampler_known_answers():
    z_in_out = _pad([[[1, 1.2], [1.5, 1.6], [2, 2.5]], [[.5, .7], [.9, 1.0]]], 3)
    u = np.array([[0, .2, .4, .6, .8], np.linspace(0, 0.3, 5)], np.float32)
    z, err = K.sample_occupied(z_in_out, u)
    assert err == 0
    np.testing.assert_allclose(z[0], [1.0, 1.2, 2.1, 2.3, 2.5], atol=1e-6)
    np.testing.assert_allclose(z[1], [.5, .575, .65, .925, 1.0], atol=1e-6)


def test_sampler_edge_cases():
    # ray without intersections keeps its initial value; eps tail snaps to last exit
    z_in_out = _pad([[], [[1, 2]], [[1, 2]], [[1, 1.5], [3, 3.5]]], 2)
    u = np.array([[0.3, 0.5], [1.00005, 0.0], [1.5, 0.2], [1.0 + 5e-5, 1.2]], np.float32)
    init = np.full(u.shape, -7.0, np.float32)
    z, err = K.sample_occupied(z_in_out, u, init)
    assert z[0, 0] == -7 and z[0, 1] == -7                  # common.cu:54
    assert z[1, 0] == 2.0                                   # K exhausted, z_remain <= eps (:58-62)
    assert z[2, 1] == np.float32(1.2)
    assert z[2, 0] == -7                                    # overflow: reference hangs, oracle counts
    assert z[3, 0] == np.float32(3.5)
    assert z[3, 1] == -7                                    # beyond total length -> error
    assert err == 2


def test_postprocess_known_answer():
    ray_index = np.array([0, 0, 0, 2, 2, 2, 2, 5], np.int64)
    depth = np.array([[1, 2], [2, 2.00001], [2.5, 3], [0.5, 0.4], [0.6, 0.9], [1.0, 1.1], [0, 1.3], [4, 5]],
                     np.float32)
    uniq = np.array([0, 2, 5], np.int64)
    start = np.array([0, 3, 7], np.int64)
    out = K.postprocess_octree(ray_index, depth, uniq, start, 4, 6)
    np.testing.assert_array_equal(out[0, :2], np.float32([[1, 2], [2.5, 3]]))       # degenerate dropped
    np.testing.assert_array_equal(out[0, 2:], 0)
    np.testing.assert_array_equal(out[2, :2], np.float32([[0.6, 0.9], [1.0, 1.1]]))  # reversed dropped, zero -> stop
    np.testing.assert_array_equal(out[5, 0], [4, 5])
    assert np.all(out[[1, 3, 4]] == 0)


def _box_chord(o, d):
    tn, tf = -np.inf, np.inf
    for a in range(3):
        if d[a] == 0:
            continue
        t1, t2 = (-1 - o[a]) / d[a], (1 - o[a]) / d[a]
        tn, tf = max(tn, min(t1, t2)), min(tf, max(t1, t2))
    return max(tn, 0), tf


def test_ray_trace_full_grid_tiles_chord():
    rng = np.random.default_rng(0)
    N = 8
    occ = np.ones((N, N, N), np.uint8)
    o = rng.normal(size=(200, 3)).astype(np.float32)
    o = (o / np.linalg.norm(o, axis=1, keepdims=True) * 2.5).astype(np.float32)
    target = rng.uniform(-0.5, 0.5, (200, 3)).astype(np.float32)
    d = target - o
    d = (d / np.linalg.norm(d, axis=1, keepdims=True)).astype(np.float32)
    out, counts = K.octree_ray_trace(occ, o, d, 3 * N)
    for r in range(200):
        t0, t1 = _box_chord(o[r].astype(np.float64), d[r].astype(np.float64))
        iv = out[r, :counts[r]]
        assert counts[r] > 0
        assert np.all(np.diff(iv[:, 0]) > 0)                 # front to back
        assert abs(iv[0, 0] - t0) < 1e-5 and abs(iv[-1, 1] - t1) < 1e-5
        gaps = iv[1:, 0] - iv[:-1, 1]
        assert np.all(np.abs(gaps) < 1e-4 + 1e-5)           # contiguous up to dropped slivers
        assert np.all(out[r, counts[r]:] == 0)


def test_ray_trace_single_voxel_slab():
    N = 4
    occ = np.zeros((N, N, N), np.uint8)
    occ[2, 1, 3] = 1                                         # z=2, y=1, x=3  (x fastest)
    lo = np.array([-1 + 3 * 0.5, -1 + 1 * 0.5, -1 + 2 * 0.5])
    c = lo + 0.25
    o = np.array([[-3.0, -2.0, -1.5]], np.float32)
    d = (c - o[0])
    d = (d / np.linalg.norm(d))[None].astype(np.float32)
    out, counts = K.octree_ray_trace(occ, o, d, 12)
    assert counts[0] == 1
    tn = max(min((lo[a] - o[0, a]) / d[0, a], (lo[a] + 0.5 - o[0, a]) / d[0, a]) for a in range(3))
    tf = min(max((lo[a] - o[0, a]) / d[0, a], (lo[a] + 0.5 - o[0, a]) / d[0, a]) for a in range(3))
    np.testing.assert_allclose(out[0, 0], [tn, tf], rtol=1e-6)


def test_ray_trace_miss_and_parallel():
    N = 4
    occ = np.ones((N, N, N), np.uint8)
    o = np.array([[3, 3, 3], [-3, 0.1, 0.1]], np.float32)
    d = np.array([[1, 0, 0], [1, 0, 0]], np.float32)
    out, counts = K.octree_ray_trace(occ, o, d, 12)
    assert counts[0] == 0 and counts[1] == N
    np.testing.assert_allclose(out[1, :N, 0], [2.0, 2.5, 3.0, 3.5], atol=1e-6)
