"""The production step at BASELINE's headline size: 64 frames x 2048
rays = 131,072 rays per step, 192 samples/ray, L=16 (finest 128, 2^22), amp — the shape
bench.py times, with every size-selected branch the library takes only there (the
16-flags-per-thread tile compaction from 262,144 tiles, the quad-mirror encode from 32 K
rays, 8 scatter levels per wave from 32 K rays, the block-reduced MLP flush).

The oracle cannot run this size in test time, so the checks are size-independent
properties of the same step:
  * the tile lists hold exactly the flagged tiles under the headline compaction (4096 flags
    per block) and under the small-batch one (512): same counts, same sets;
  * the two runs' gradients agree entry by entry within float-atomic order (the lists'
    order differs, so the MLP weight-gradient atomics and the fp16 table adds land in another
    order);
  * the losses are finite and the forward is bit-identical between them (per-tile records
    summed in tile order: no float atomics; only the per-block loss-row adds reorder);
  * one captured-graph replay of the step equals the eager step on the same batch.
"""
import os
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def headline(cuda_device):
    import bench
    from bundlesdf_amd.fused import FusedStep
    dev = cuda_device
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, 64, dict(amp=True), dev)
    enc, net, pa, fa = bench.make_models(cfg, 64, dev, with_features=True)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start,
                   feature_array=fa)
    P0 = fs.P.detach().clone()
    ids = fs.sample_ids(2048, seed=7).clone()
    assert ids.numel() == 131072
    yield fs, P0, ids
    del fs
    torch.cuda.empty_cache()


def _eager(fs, P0, ids, per):
    fs.reset_state(P0)
    fs.compact_per_block = per
    out = fs.step(ids=ids, seed=11, debug=True)
    torch.cuda.synchronize()
    bl, cl = fs.tile_lists()
    return dict(loss=out["loss_terms"].cpu().numpy().copy(), grads=out["grads"].cpu().numpy().astype(np.float64),
                rgb=out["dbg"]["rgb"].cpu().numpy(), raw=out["dbg"]["raw"].cpu().numpy(),
                blist=bl.cpu().numpy(), clist=cl.cpu().numpy(), P=fs.P.detach().cpu().numpy().copy())


def test_headline_step_compaction_paths_agree(headline):
    fs, P0, ids = headline
    a = _eager(fs, P0, ids, 0)        # by batch size: 4096 flags per block (16 per thread) at this size
    b = _eager(fs, P0, ids, 512)      # the small-batch compaction
    assert np.isfinite(a["loss"][:8]).all() and np.isfinite(b["loss"][:8]).all()
    assert a["loss"][:4].sum() > 0
    # the forward does not depend on the lists' order: bit-identical
    np.testing.assert_array_equal(a["raw"], b["raw"])
    np.testing.assert_array_equal(a["rgb"], b["rgb"])
    # the loss terms: per-ray sums in tile order, then per-block float adds into the loss rows
    np.testing.assert_allclose(a["loss"][:4], b["loss"][:4], rtol=1e-5)
    # the same tiles listed (a dropped tile would silently zero its gradients)
    assert a["blist"].size > 100000 and a["clist"].size > 0
    np.testing.assert_array_equal(a["blist"], b["blist"])
    np.testing.assert_array_equal(a["clist"], b["clist"])
    # every listed tile is a flagged one and every flagged tile is listed (headline path)
    offs, nt = fs._ws_offsets()
    flags = fs.workspace[offs["tile_bwd"]:offs["tile_bwd"] + nt].cpu().numpy()
    np.testing.assert_array_equal(np.sort(b["blist"] & 0x7fffffff) >> 5, np.nonzero((flags == 1) | (flags == 2))[0])
    np.testing.assert_array_equal(b["clist"] >> 5, np.nonzero((flags == 1) | (flags == 3))[0])
    # gradients: the same sums in another float-atomic order. The fp16 table gradient rounds each
    # add at 2^-11 relative (the reference's __half2 accumulation class), fp32 elsewhere
    ga, gb = a["grads"], b["grads"]
    n_emb = fs.n_emb
    for name, sl, tol in (("table", slice(0, n_emb), 2e-2), ("rest", slice(n_emb, None), 2e-3)):
        x, y = ga[sl], gb[sl]
        scale = max(float(np.abs(y).max()), 1e-30)
        err = float(np.abs(x - y).max()) / scale
        assert err < tol, (name, err)
        assert np.count_nonzero(x) > 0
    # the MLP weight gradients entry by entry (fp32 atomics: relative order error only)
    mlp = slice(n_emb, fs.feat_off)
    np.testing.assert_allclose(ga[mlp], gb[mlp], rtol=1e-3, atol=1e-4 * float(np.abs(gb[mlp]).max()))


def test_headline_quad_mirror_fork_equals_inline(headline):
    """The quad mirror rebuilt on the side stream beside the prologue and trace (nof_quad_mirror,
    the default) and inside the field pass (quads_prebuilt 0) give a bit-identical forward."""
    fs, P0, ids = headline
    try:
        fs.quad_fork = False
        a = _eager(fs, P0, ids, 0)
        fs.quad_fork = True
        fs.quads.fill_(-1)   # a stale or partial rebuild would show in the forward
        b = _eager(fs, P0, ids, 0)
    finally:
        fs.quad_fork = True
    assert np.isfinite(b["loss"][:8]).all()
    np.testing.assert_array_equal(a["raw"], b["raw"])
    np.testing.assert_array_equal(a["rgb"], b["rgb"])


def test_headline_step_subset_matches_oracle(headline):
    """The 131,072-ray production step (quad-mirror encode, 16-flag compaction, k_colour at headline
    occupancy, 8 scatter levels per wave) with injected stratification draws, checked against the
    oracle:
      * forward: rays are independent in the forward, so 512 rays spread over the 64 frames are
        compared with the oracle's amp step on those rays alone — z (2e-6), validity (exact), the
        fp16 raw outputs and rgb (the amp forward tolerances of test_gpu_step);
      * loss: the step's rgb / free-space / sdf loss terms against the same losses recomputed in
        float64 from the whole batch's per-sample records (oracle.nerf_step.loss_terms_f64), so the
        kernels' reduction of 25 M samples into the reported loss is checked at full size."""
    from oracle import nerf_step as NS
    fs, P0, ids = headline
    fs.reset_state(P0)
    fs.compact_per_block = 0
    cfg = fs.cfg
    R = ids.numel()
    S = cfg["N_samples"] + cfg["N_samples_around_depth"]
    t_rand = torch.rand(R, S, generator=torch.Generator().manual_seed(5))
    out = fs.step(ids=ids, t_rand=t_rand, debug=True)
    torch.cuda.synchronize()
    dbg = out["dbg"]
    lt = out["loss_terms"].cpu().numpy().astype(np.float64)
    batch_full = fs.pool[ids.long()]
    trunc = NS.truncation(cfg, 0)
    f64 = NS.loss_terms_f64(batch_full, dbg["z"], dbg["raw"], dbg["valid"], cfg, trunc)
    np.testing.assert_allclose(lt[0], f64["rgb_loss"], rtol=1e-4)
    np.testing.assert_allclose(lt[1] + lt[2], f64["fs_loss"], rtol=1e-4)
    np.testing.assert_allclose(lt[3], f64["sdf_loss"], rtol=1e-4)
    np.testing.assert_allclose(dbg["rgb"].double().cpu().numpy(), f64["rgb"].cpu().numpy(), rtol=0, atol=2e-6)
    assert f64["rgb_loss"] > 0 and f64["sdf_loss"] > 0 and f64["fs_loss"] > 0
    # forward subset: 8 rays from every frame (the batch is frame-sorted, 2048 rays per frame)
    sel = (np.arange(64)[:, None] * 2048 + np.random.default_rng(3).choice(2048, 8, replace=False)[None]).ravel()
    sel_t = torch.from_numpy(sel).to(ids.device)
    batch = fs.pool[ids.long()[sel_t]].cpu()
    P = {k: v.clone() for k, v in fs.split(P0.cpu()).items()}
    offs = fs.grid.offsets.cpu().numpy()
    meta = (offs, float(np.log2(fs.grid.per_level_scale)), int(fs.grid.base_resolution))
    ref = NS.train_step(P, batch, fs.c2w.cpu(), fs.occ.cpu().numpy(), cfg, t_rand[sel], meta, amp=True,
                        loss_scale=65536.0, kmax=fs.Kmax)
    z, raw = dbg["z"][sel_t].cpu().numpy(), dbg["raw"][sel_t].cpu().numpy()
    np.testing.assert_allclose(z, ref["z_vals"].numpy(), rtol=1e-6, atol=2e-6)
    np.testing.assert_array_equal(dbg["valid"][sel_t].cpu().numpy().astype(bool), ref["valid"].numpy())
    assert ref["valid"].numpy().mean() > 0.2
    np.testing.assert_allclose(raw, ref["raw"].numpy(), rtol=1e-2, atol=2e-3)
    np.testing.assert_allclose(dbg["rgb"][sel_t].cpu().numpy(), ref["rgb_map"].numpy(), rtol=2e-3, atol=1e-4)
    fs.reset_state(P0)


def test_headline_graph_replay_equals_eager(headline):
    fs, P0, ids = headline
    fs.compact_per_block = 0
    fs.reset_state(P0)
    out = fs.step(ids=ids, seed=11)
    torch.cuda.synchronize()
    loss_e = out["loss_terms"].cpu().numpy().copy()
    P_e = fs.P.detach().cpu().numpy().copy()
    fs.reset_state(P0)
    out = fs.graph_step_ids(ids, seed_base=11)
    torch.cuda.synchronize()
    loss_g = out["loss_terms"].cpu().numpy().copy()
    P_g = fs.P.detach().cpu().numpy().copy()
    assert np.isfinite(loss_g[:8]).all()
    # same batch, same seed: the same forward (the loss rows' per-block adds may reorder)
    np.testing.assert_allclose(loss_g[:4], loss_e[:4], rtol=1e-5)
    # Adam's first step moves every touched parameter by exactly +-lr (m / sqrt(v) = sign(g)):
    # graph and eager differ only where a gradient's sign depends on float-atomic order
    lr = fs.cfg["lrate"]
    d = np.abs(P_g.astype(np.float64) - P_e)
    moved = np.abs(P_e.astype(np.float64) - P0.cpu().numpy()) > 0
    assert moved.sum() > 100000
    assert d.max() <= 2.0 * lr * 1.0001 + 1e-7
    n_diff = int((d > 1e-6).sum())
    assert n_diff <= 1e-3 * moved.sum(), (n_diff, int(moved.sum()))
    fs.reset_state(P0)
