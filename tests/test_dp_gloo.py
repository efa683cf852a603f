"""CPU (world_size 2, gloo) tests of the data-parallel path:
frame-sharded equal batches + one mean all-reduce per bucket reproduce the
full-batch gradient of the reference's train_loop (G4), in fp32 and amp
bucket layouts; replicas end bit-identical; bench's rank scenes partition
the frames."""
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


@pytest.fixture(scope="module")
def dp_results(golden_dir, tmp_path_factory):
    out = tmp_path_factory.mktemp("dp")
    world = 2
    mp.spawn(_dp_worker.run, args=(world, _free_port(), os.path.join(golden_dir, "train_step.npz"), str(out)),
             nprocs=world, join=True)
    return [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(world)]


def _rel_err_q(got, ref, q=0.99):
    scale = np.abs(ref) + 1e-3 * (np.abs(ref).max() + 1e-30)
    return np.quantile(np.abs(got - ref) / scale, q)


def test_sharded_fp32_bucket_equals_full_batch_gradient(dp_results):
    r0, r1 = dp_results
    np.testing.assert_array_equal(r0["fp32"], r1["fp32"])          # replicas identical
    ref = r0["ref"]
    n_emb = int(r0["n_emb"])
    # same tolerance as the oracle-vs-G4 pin (summation order differs only)
    np.testing.assert_allclose(r0["fp32"][n_emb:], ref[n_emb:], rtol=1e-3, atol=1e-6)
    np.testing.assert_allclose(r0["fp32"][:n_emb], ref[:n_emb], rtol=1e-3, atol=1e-7)


def test_sharded_amp_buckets(dp_results):
    r0, r1 = dp_results
    np.testing.assert_array_equal(r0["amp_table"], r1["amp_table"])
    np.testing.assert_array_equal(r0["amp_tail"], r1["amp_tail"])
    n_emb = int(r0["n_emb"])
    ref = r0["ref"]
    np.testing.assert_allclose(r0["amp_tail"], ref[n_emb:], rtol=1e-3, atol=1e-6)
    # fp16 table bucket: within fp16 resolution of the scaled values
    assert _rel_err_q(r0["amp_table"], ref[:n_emb]) < 2e-3


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
