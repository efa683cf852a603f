"""GPU: the throughput-mode batch draw (nof_sample_batch, FusedStep.sample_ids): per frame,
rays_per_frame draws with replacement from the frame's contiguous pool segment, produced in
ascending pool order (the sorted draws are generated as uniform order statistics from
exponential spacings). Checks the layout (in range, ascending per frame, deterministic per
seed) and the distribution (uniform over the frame: mean / quartiles of the positions, the
number of distinct draws of k samples from n with replacement)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_sample_batch_sorted_uniform_per_frame(cuda_device):
    from bundlesdf_amd import _lib
    dev = cuda_device
    rng = np.random.default_rng(5)
    counts = rng.integers(3000, 40000, size=24)
    counts[3] = 1                                           # a one-ray frame
    fs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    frame_start = torch.from_numpy(fs).to(dev)
    F = len(counts)
    pos = []
    for k in (2048, 4096, 100):
        ids = torch.empty(F * k, dtype=torch.int32, device=dev)
        L = _lib.lib()
        _lib.check(L.nof_sample_batch(_lib.ptr(frame_start), F, k, 1234, _lib.ptr(ids), None,
                                      _lib.stream_of(ids)), "sample_batch")
        ids2 = torch.empty_like(ids)
        _lib.check(L.nof_sample_batch(_lib.ptr(frame_start), F, k, 1234, _lib.ptr(ids2), None,
                                      _lib.stream_of(ids)), "sample_batch")
        torch.cuda.synchronize()
        a = ids.cpu().numpy().reshape(F, k).astype(np.int64)
        assert np.array_equal(a, ids2.cpu().numpy().reshape(F, k))          # deterministic per seed
        for f in range(F):
            lo, hi = fs[f], fs[f + 1]
            assert a[f].min() >= lo and a[f].max() < hi, f
            assert np.all(np.diff(a[f]) >= 0), f                            # ascending pool order
            n = hi - lo
            if n > 1000 and k >= 2048:
                u = (a[f] - lo + 0.5) / n
                pos.append(u)
                # distinct draws of k from n with replacement: n (1 - (1 - 1/n)^k), sd ~ sqrt of it
                want = n * (1 - (1 - 1 / n) ** k)
                assert abs(len(np.unique(a[f])) - want) < 6 * np.sqrt(want) + 5, (f, len(np.unique(a[f])), want)
    u = np.concatenate(pos)
    assert abs(u.mean() - 0.5) < 0.01
    q = np.quantile(u, [0.25, 0.5, 0.75])
    assert np.allclose(q, [0.25, 0.5, 0.75], atol=0.01), q
