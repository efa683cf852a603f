"""GPU: the N>1 data-parallel training step (BASELINE config 4's code
path) against the single-process step on the whole batch.

Two ranks (tests/_dp_gpu_worker.py, gloo, both on cuda:0) each run
FusedStep(world_size=2) on one half of a fixed batch — the G4 batch and a
config-2-shaped scene case (L=16, 2^22 table, S=192) — for 3 steps with
injected stratification draws, in fp32 and amp, eager and from the captured
two-graph split (field graph | all-reduce | optimiser graph). This exercises
exactly what differs at N>1: the fp16 table gradient widened into the fp32
bucket (nof_grad16_to_f32), the unscale / Adam branch that reads the table
gradient from the bucket, and the all-reduce between the two graphs.

Checks, per case / precision / execution:
  * replicas bit-identical (P, M, V, GradScaler scale / tracker, Adam count);
  * mean of the ranks' losses = the whole-batch losses;
  * step 0: the exchanged gradient = the single-process gradient entry by entry,
    within the summation-order allowance of tests/test_gpu_step.py (conditioning
    from the oracle on the same inputs: both runs evaluate identical samples, only
    the grouping of the sums differs — and in amp the fp16 accumulation of each
    half); the Adam update equal wherever the gradient sign is determined (at step
    1 with eps 1e-15 Adam moves every entry by lr sign(g), so an entry whose
    gradient is within its summation noise of 0 may move either way);
  * step 2: P / M / V within 3x the run-to-run spread of two single-process runs
    (or 2e-3 relative L2), scale / Adam count / tracker equal;
  * a non-finite gradient on one rank makes every replica skip (P unchanged,
    scale backed off, Adam count not advanced)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from oracle import nerf_step as NS
from tests import _dp_gpu_worker as W
from tests.test_gpu_step import _METRICS, _check_all

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture(scope="module")
def dp_ranks(tmp_path_factory):
    out = tmp_path_factory.mktemp("dp_gpu")
    mp.spawn(W.run, args=(2, _free_port(), str(out)), nprocs=2, join=True)
    return [dict(np.load(os.path.join(out, f"rank{r}.npz"))) for r in range(2)]


def _single(dev, c, amp, runs=2):
    """Single-process FusedStep on the whole batch: `runs` independent runs of K_STEPS, and a
    trainer of the same layout (for split())."""
    R = c[1].shape[0]
    S = c[0]["N_samples"] + c[0]["N_samples_around_depth"]
    out = []
    for _ in range(runs):
        fs = W.make_step(dev, c, amp, 0, R, 1, None)
        out.append(W.run_steps(fs, "eager", 0, R, R, S))
        del fs
    return out, W.make_step(dev, c, amp, 0, 8, 1, None)


def _flat_abs(ref_o, lay):
    """The oracle's per-entry conditioning A in the flat [table | mlp | pose] layout."""
    parts = [ref_o["g_emb_abs"].numpy().ravel()]
    from bundlesdf_amd import mlp_layout as ML
    for k in ML.MLP_KEYS:
        parts.append(ref_o["g_mlp_abs"][k].numpy().ravel())
    parts.append(np.zeros(lay.P.numel() - lay.pose_off))
    A = np.concatenate(parts)
    assert A.size == lay.P.numel()
    return A


def _oracle_conditioning(c, amp):
    cfg, batch, c2w, occ, emb, mlp_w, pose, (L, log2T, finest, base) = c
    from bundlesdf_amd.grid import GridEncoder
    P0 = {"embeddings": torch.from_numpy(emb), "pose": torch.from_numpy(pose)}
    P0.update({k: torch.from_numpy(v) for k, v in mlp_w.items()})
    pls = GridEncoder(3, L, 2, base, log2T, finest).per_level_scale
    from bundlesdf_amd.grid import level_layout
    _, offs = level_layout(3, L, 2, base, log2T, finest)
    S = cfg["N_samples"] + cfg["N_samples_around_depth"]
    ref = NS.train_step(P0, torch.from_numpy(batch), torch.from_numpy(c2w), occ, dict(cfg, amp=amp),
                        torch.from_numpy(W.t_rand_of(0, batch.shape[0], S)), (offs, float(np.log2(pls)), base),
                        amp=amp, loss_scale=W.AMP_SCALE)
    return ref


def _rel(a, b):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    return float(np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-30))


@pytest.mark.parametrize("name", ["g4", "scene"])
@pytest.mark.parametrize("amp", [False, True], ids=["fp32", "amp"])
def test_dp2_step_matches_single_process(dp_ranks, cuda_device, name, amp):
    r0, r1 = dp_ranks
    c = W.case(name)
    single, lay = _single(cuda_device, c, amp)
    s1, s2 = single
    ref_o = _oracle_conditioning(c, amp)
    pre = f"{name}/{int(amp)}"
    for mode in [m for a, m, _ in W.MODES if a == amp]:
        for k in range(W.K_STEPS):
            key = f"{pre}/{mode}/{k}"
            # replicas identical after the exchange + Adam
            for f in ("P", "M", "V", "scale", "adam_t", "tracker"):
                np.testing.assert_array_equal(r0[f"{key}/{f}"], r1[f"{key}/{f}"], err_msg=f"{key}/{f}")
            # losses: equal halves -> the whole-batch means are the means of the local ones (step 0:
            # the same samples; later steps start from parameters that moved by lr at the entries
            # whose gradient sign is undetermined, see below)
            np.testing.assert_allclose(0.5 * (r0[f"{key}/loss"] + r1[f"{key}/loss"]), s1[k]["loss"],
                                       rtol=2e-5 if k == 0 else 2e-3, atol=1e-9, err_msg=f"{key}/loss")
            for f in ("scale", "adam_t", "tracker"):
                assert float(r0[f"{key}/{f}"]) == float(s1[k][f]), (key, f)
        # step 0: the exchanged gradient, entry by entry
        if mode.startswith("eager"):
            g_dp = torch.from_numpy(r0[f"{pre}/{mode}/0/grads"])
            ref = {"grads": lay.split(torch.from_numpy(s1[0]["grads"])), "g_emb_abs": ref_o["g_emb_abs"],
                   "g_mlp_abs": ref_o["g_mlp_abs"]}
            _check_all(f"dp2/{pre}", lay.split(g_dp), ref, amp=amp)
        # step 0: Adam moved every entry by lr sign(g); entries whose gradient sign differs
        # between the two groupings must be within their summation noise of 0
        g1 = s1[0]["grads"]
        dP = np.abs(r0[f"{pre}/{mode}/0/P"].astype(np.float64) - s1[0]["P"])
        moved = dP > 1e-6
        A = _flat_abs(ref_o, lay)
        noise = (5e-2 if amp else 1e-4) * np.abs(g1) + (1e-1 if amp else 1e-4) * A + 1e-9 * np.abs(g1).max()
        if amp:   # fp16 resolution of the scaled gradient near 0 (subnormals)
            noise = noise + 2.0 ** -13 / W.AMP_SCALE
        bad = moved & (np.abs(g1) > noise)
        _METRICS[f"dp2/{pre}/{mode}/sign_flips"] = int(moved.sum())
        assert not bad.any(), f"{pre}/{mode}: {int(bad.sum())} determined entries updated differently"
        # step K-1: the MLP / pose part within the run-to-run spread of the single-process step
        k = W.K_STEPS - 1
        ne = lay.n_emb
        for f in ("P", "M", "V"):
            rel = _rel(r0[f"{pre}/{mode}/{k}/{f}"][ne:], s1[k][f][ne:])
            spread = _rel(s2[k][f][ne:], s1[k][f][ne:])
            _METRICS[f"dp2/{pre}/{mode}/{f}_rel"] = rel
            assert rel < max(2e-3, 3 * spread), (pre, mode, f, rel, spread)
        # ... and the table: every entry that moved differently had a gradient within its noise
        # of 0 at some step (Adam with eps 1e-15 moves such an entry by a full lr either way). In
        # amp the table gradient is summed in fp16 — per rank here, over the whole batch in the
        # single-process step — so the noise includes fp16 rounding of the scaled gradient near 0
        # (2^-14 resolution of subnormals)
        # (classified on both trajectories' gradients: after step 0 they sit at slightly different
        # parameters; the graph run's trajectory is the eager one's up to float-atomic order)
        undet = np.zeros(ne, bool)
        for j in range(W.K_STEPS):
            for gj in (s1[j]["grads"][:ne], r0[f"{pre}/eager/{j}/grads"][:ne]):
                nz = (5e-2 if amp else 1e-4) * np.abs(gj) + (1e-1 if amp else 1e-4) * A[:ne] + \
                    1e-9 * np.abs(gj).max()
                if amp:
                    nz = nz + 2.0 ** -13 / W.AMP_SCALE
                undet |= np.abs(gj) <= nz
        # (a sign-level difference is ~lr = 1e-2; determined entries differ by at most ~lr times the
        # relative difference of their gradient histories)
        dPt = np.abs(r0[f"{pre}/{mode}/{k}/P"][:ne].astype(np.float64) - s1[k]["P"][:ne])
        moved_t = dPt > 1e-3
        _METRICS[f"dp2/{pre}/{mode}/table_moved_differently"] = int(moved_t.sum())
        _METRICS[f"dp2/{pre}/{mode}/table_undetermined"] = int(undet.sum())
        # a handful of determined entries may still move apart by > 10 % of lr: their gradient
        # history at the later steps differs because neighbouring entries moved (training
        # dynamics, not the exchange) — at most 1 % of the differently-moved entries in the
        # replicated exchange. The sharded amp exchange's fp16 reduce-scatter adds one fp16
        # rounding of every summed table-gradient entry (the reference's own fp16 accumulation
        # class; bounded per entry at step 0 by test_dp2_sharded_fp16_sum_per_entry), which the
        # trajectories then carry: measured 24 of 1,193 (2.0 %) on the scene case, so the bound
        # there is 3 % (1.5x the measurement)
        n_bad = int((moved_t & ~undet).sum())
        _METRICS[f"dp2/{pre}/{mode}/table_determined_moved"] = n_bad
        frac = 0.03 if (amp and mode in ("eager", "graph")) else 0.01
        assert n_bad <= max(8, int(frac * moved_t.sum())), (pre, mode, n_bad, int(moved_t.sum()))


def _ulp16(x):
    """fp16 spacing at |x| (2^-24 in the subnormal range)."""
    ax = np.abs(np.asarray(x, np.float64))
    e = np.floor(np.log2(np.maximum(ax, 2.0 ** -14)))
    return 2.0 ** (e - 10)


@pytest.mark.parametrize("name", ["g4", "scene"])
def test_dp2_sharded_fp16_sum_per_entry(dp_ranks, name):
    """the sharded exchange pre-scales each rank's fp16 table gradient by 1/W2 and
    sums the ranks' fp16 values in the reduce-scatter; the replicated exchange widens them to
    fp32 first. On the SAME step-0 local gradients (captured on each rank as they enter the
    exchange, real-scale), every exchanged table entry must be the exact mean of the two ranks'
    fp16 values within one fp16 ulp of the (scaled) sum plus the subnormal term of the halving
    (2^-25 per rank): the exchange adds one fp16 rounding, nothing more."""
    r0, r1 = dp_ranks
    key = f"{name}/1/eager/0"
    g0, g1 = r0[f"{key}/local16"].astype(np.float64), r1[f"{key}/local16"].astype(np.float64)
    scale = W.AMP_SCALE
    n = g0.size
    got = r0[f"{key}/grads"][:n].astype(np.float64) * scale        # the exchanged gradient, scaled back
    exact = 0.5 * (g0 + g1)
    allowed = _ulp16(exact) + 2 * 2.0 ** -25
    err = np.abs(got - exact)
    _METRICS[f"dp2/{name}/sharded_sum_worst_ulps"] = float((err / _ulp16(exact)).max())
    assert np.count_nonzero(g0) > 1000 and np.count_nonzero(g1) > 1000
    assert (err <= allowed).all(), (int((err > allowed).sum()), float((err / allowed).max()))
    # both ranks hold the same exchanged gradient
    np.testing.assert_array_equal(r0[f"{key}/grads"], r1[f"{key}/grads"])


@pytest.mark.parametrize("where", ["mlp", "table"])
def test_dp2_inf_on_one_rank_skips_everywhere(dp_ranks, where):
    """amp, sharded exchange: rank 1 poisons an MLP gradient entry (reaches rank 0 through
    the rest bucket's sum) or a table row of its own shard (rank 0 learns it only from the
    shard's inf flag in the rest bucket): both ranks skip the step."""
    r0, r1 = dp_ranks
    p = f"inf_{where}"
    for r in (r0, r1):
        assert int(r[f"{p}/0/adam_t"]) == 1
        assert int(r[f"{p}/1/adam_t"]) == 1                  # skipped: Adam count not advanced
        assert int(r[f"{p}/2/adam_t"]) == 2
        np.testing.assert_array_equal(r[f"{p}/1/P"], r[f"{p}/0/P"])
        assert float(r[f"{p}/1/scale"]) == 0.5 * float(r[f"{p}/0/scale"])
        assert int(r[f"{p}/1/tracker"]) == 0
    for k in range(W.K_STEPS):
        np.testing.assert_array_equal(r0[f"{p}/{k}/P"], r1[f"{p}/{k}/P"])


def test_dp2_reset_state_then_skipped_step_keeps_fresh_mirror(dp_ranks):
    """amp, sharded exchange: reset_state(P0) after some steps, then a first step that
    skips (non-finite gradient): the all-gathered fp16 table both ranks' forward reads must be
    to_half(P0) — reset_state re-copies the rank's mirror shard, so the all-gather cannot bring
    back the previous round's table."""
    for r in dp_ranks:
        assert int(r["reset_skip/adam_t"]) == 0
        np.testing.assert_array_equal(r["reset_skip/emb16"], r["reset_skip/want"])
