"""CPU (gloo, world size 8 and 3) test of the sharded exchange (bundlesdf_amd/
exchange.py: fp16 reduce-scatter of the table gradient pre-scaled by 1/W2, Adam on
each rank's shard, all-gather of the fp16 mirror, the local inf verdict riding in
the rest bucket) against the replicated exchange (one fp32 all-reduce, the whole
Adam everywhere), both run by tests/_exchange_worker.py through the product
protocol code. With small dyadic gradients every summation order is exact, so the
two must be bit-identical: master parameters, Adam moments, fp16 mirror,
GradScaler state — including steps where one rank's table shard holds an inf
produced on another rank while the rest bucket is finite (every rank skips)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from tests import _exchange_worker as W


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world", [8, 3])
def test_sharded_exchange_bit_identical_to_replicated(tmp_path, world):
    mp.spawn(W.run, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    ranks = [dict(np.load(os.path.join(tmp_path, f"rank{r}.npz"))) for r in range(world)]
    r0 = ranks[0]
    for step in range(W.STEPS):
        for k in ("P", "M", "V", "mirror", "scale", "adam_t", "tracker"):
            rep, sh = r0[f"replicated/{step}/{k}"], r0[f"sharded/{step}/{k}"]
            np.testing.assert_array_equal(sh, rep, err_msg=f"step {step} {k}")
            for r in ranks[1:]:       # replicas identical
                np.testing.assert_array_equal(r[f"sharded/{step}/{k}"], sh)
                np.testing.assert_array_equal(r[f"replicated/{step}/{k}"], rep)
    # the inf steps skipped on every rank: parameters unchanged, scale backed off, count held
    for s in (W.INF_STEP, W.INF_STEP2):
        for r in ranks:
            np.testing.assert_array_equal(r[f"sharded/{s}/P"], r[f"sharded/{s - 1}/P"])
            assert float(r[f"sharded/{s}/scale"][0]) == 0.5 * float(r[f"sharded/{s - 1}/scale"][0])
            assert int(r[f"sharded/{s}/adam_t"][0]) == int(r[f"sharded/{s - 1}/adam_t"][0])
    # the other steps moved the parameters
    assert not np.array_equal(r0["sharded/4/P"], r0["sharded/3/P"])
    assert not np.array_equal(r0["sharded/2/P"], r0["sharded/1/P"])
    assert int(r0[f"sharded/{W.STEPS - 1}/adam_t"][0]) == W.STEPS - 2
    # the overlapped schedule (mirror all-gather left in flight into the next step, waited for before
    # the field pass): the same states, and every step's forward saw the previous step's mirror
    for r in ranks:
        for step in range(W.STEPS):
            for k in ("P", "M", "V", "mirror", "scale", "adam_t", "tracker"):
                np.testing.assert_array_equal(r[f"overlap/{step}/{k}"], r[f"sharded/{step}/{k}"],
                                              err_msg=f"overlap step {step} {k}")
            if step:
                np.testing.assert_array_equal(r[f"overlap/{step}/seen"], r[f"sharded/{step - 1}/mirror"])


def test_shard_plan_covers_the_table():
    from bundlesdf_amd.exchange import ShardPlan
    for n, world in ((13024512, 8), (1000, 3), (7, 8), (64 * 8, 8)):
        plans = [ShardPlan(n, world, r) for r in range(world)]
        assert plans[0].sh % 64 == 0 and plans[0].n_pad == plans[0].sh * world >= n
        assert sum(p.cnt for p in plans) == n
        assert all(p.lo == min(n, r * p.sh) for r, p in enumerate(plans))
