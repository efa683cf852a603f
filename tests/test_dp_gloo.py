"""CPU (world_size 2 and 8, gloo) tests of the data-parallel path:
frame-sharded equal batches + one mean all-reduce of the flat fp32 bucket
reproduce the full-batch gradient of the reference's train_loop (G4), in fp32
mode and in amp mode (fp16 table gradients moved into the fp32 bucket);
replicas end bit-identical; bench's rank scenes partition the frames."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests import _dp_worker


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module", params=[2, 8], ids=["w2", "w8"])
def dp_results(request, golden_dir, tmp_path_factory):
    world = request.param
    out = tmp_path_factory.mktemp(f"dp{world}")
    mp.spawn(_dp_worker.run, args=(world, _free_port(), os.path.join(golden_dir, "train_step.npz"), str(out)),
             nprocs=world, join=True)
    return [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(world)]


def test_sharded_fp32_bucket_equals_full_batch_gradient(dp_results):
    r0 = dp_results[0]
    for r in dp_results[1:]:
        np.testing.assert_array_equal(r0["fp32"], r["fp32"])          # replicas identical
    ref = r0["ref"]
    n_emb = int(r0["n_emb"])
    # max over every entry; same tolerance as the oracle-vs-G4 pin (summation order differs only)
    np.testing.assert_allclose(r0["fp32"][n_emb:], ref[n_emb:], rtol=1e-3, atol=1e-6)
    np.testing.assert_allclose(r0["fp32"][:n_emb], ref[:n_emb], rtol=1e-3, atol=1e-7)


def test_sharded_amp_bucket(dp_results):
    """amp: fp16 table gradients summed as fp32 (SURVEY §8e flat fp32 bucket): every entry
    within the fp16 roundings of the local gradients (2^-11 relative each, bounded by
    2^-10 of the mean absolute local value) of the full-batch gradient."""
    r0 = dp_results[0]
    for r in dp_results[1:]:
        np.testing.assert_array_equal(r0["amp"], r["amp"])
    n_emb = int(r0["n_emb"])
    ref, got = r0["ref"], r0["amp"]
    np.testing.assert_allclose(got[n_emb:], ref[n_emb:], rtol=1e-3, atol=1e-6)
    bound = 1e-3 * np.abs(ref[:n_emb]) + 2.0 ** -10 * r0["abs_table"] + 1e-7 * np.abs(ref[:n_emb]).max()
    excess = np.abs(got[:n_emb] - ref[:n_emb]) - bound
    assert excess.max() <= 0, f"worst entry exceeds its bound by {excess.max():.3e}"


def test_rank_scenes_partition_frames():
    """Each rank renders only its own frames (global ids lo..hi-1, which the device
    pool writes into column 8 via index_base) and holds every pose."""
    import bench
    spans = []
    for rank in range(2):
        cfg, seq, poses, pts, lo, hi = bench.rank_frames(rank, 2, 1, dict(amp=True))
        assert seq["rgbs"].shape[0] == hi - lo == 1 and poses.shape[0] == 2
        np.testing.assert_array_equal(seq["poses"], poses[lo:hi])
        spans.append((lo, hi))
    assert spans == [(0, 1), (1, 2)]


def test_sharded_exchange_fp16_reduce_scatter(dp_results):
    """amp through the production sharded exchange (fp16 table gradient pre-scaled by 1/W2,
    reduce-scattered in fp16 — the reference's own fp16 accumulation, gridencoder.cu:319-327 —
    plus the rest-bucket all-reduce): replicas identical, the MLP / pose gradient as the
    fp32 bucket, every table entry within the fp16 roundings of the local gradients plus
    one fp16 rounding per reduction hop (W2 x 2^-11 of the mean absolute local value)."""
    r0 = dp_results[0]
    world = len(dp_results)
    for r in dp_results[1:]:
        np.testing.assert_array_equal(r0["sharded"], r["sharded"])
    n_emb = int(r0["n_emb"])
    ref, got = r0["ref"], r0["sharded"]
    np.testing.assert_allclose(got[n_emb:], ref[n_emb:], rtol=1e-3, atol=1e-6)
    w2 = 1 << (world - 1).bit_length()
    bound = (1e-3 * np.abs(ref[:n_emb]) + (2.0 ** -10 + w2 * 2.0 ** -11) * r0["abs_table"] +
             1e-7 * np.abs(ref[:n_emb]).max())
    excess = np.abs(got[:n_emb] - ref[:n_emb]) - bound
    assert excess.max() <= 0, f"worst entry exceeds its bound by {excess.max():.3e}"
