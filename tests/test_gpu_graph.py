"""GPU: the captured step (FusedStep.graph_step: one hipGraph holding the device
schedule, the batch draw, the field pass and the optimiser) replays the eager
step. Two trainers start from the same parameters; one runs eager steps
with host-side schedule values (lr_at / truncation / seeds of global_step), the
other replays its graph, which computes them on the device (nof_step_schedule).
The exp truncation anneal and the schedule_lr decay (every 10 steps) both move
inside the 14 steps, so a schedule read at capture time instead of replay time
would show: every step's device block is compared with the host schedule, the
batch draws must be identical, and losses / parameters agree up to the
run-to-run spread of the float atomics."""
import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS = 14
RPF = 512


def _trainer(dev, scene, amp):
    import bench
    from bundlesdf_amd.fused import FusedStep
    cfg, pool, frame_start, c2w, occ = scene
    enc, net, pa = bench.make_models(cfg, len(frame_start) - 1, dev)   # seeded init: identical trainers
    return FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=amp, frame_start=frame_start)


@pytest.mark.parametrize("amp", [True, False], ids=["amp", "fp32"])
def test_graph_replay_matches_eager(cuda_device, amp):
    import bench
    from bundlesdf_amd import _lib
    from bundlesdf_amd.fused import lr_at, truncation
    dev = cuda_device
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(
        0, 1, 4, dict(amp=amp, trunc_decay_type="exp", trunc_start=0.03, n_step=40), dev)
    scene = (cfg, pool, frame_start, c2w, occ)
    eager, graph = _trainer(dev, scene, amp), _trainer(dev, scene, amp)
    eager2 = _trainer(dev, scene, amp)   # run-to-run spread of the eager step itself (float atomics)
    assert torch.equal(eager.P, graph.P)
    assert truncation(cfg, 0) != truncation(cfg, STEPS - 1)
    assert lr_at(cfg, 1, 1.0) != lr_at(cfg, STEPS, 1.0)
    for gs in range(STEPS):
        oe = eager.step(ids=eager.sample_ids(RPF, 50 + gs), seed=3)
        eager2.step(ids=eager2.sample_ids(RPF, 50 + gs), seed=3)
        og = graph.graph_step(RPF, seed_base=3, batch_seed_base=50)
        # the device schedule block of this step equals the host schedule of global_step gs
        sp = _lib.StepParams.from_buffer_copy(bytes(graph.step_params.cpu().numpy()))
        assert sp.step == gs
        assert sp.seed == (gs * 0x9E3779B1 + 3) & 0xFFFFFFFF and sp.batch_seed == 50 + gs
        assert sp.lr0 == pytest.approx(lr_at(cfg, gs, cfg["lrate"]), rel=1e-12)
        assert sp.lr1 == pytest.approx(lr_at(cfg, gs, cfg["lrate_pose"]), rel=1e-12)
        assert sp.trunc == pytest.approx(truncation(cfg, gs), rel=1e-6)
        assert torch.equal(graph.ids, eager.ids), f"batch draw, step {gs}"
        # float atomics (table / weight gradient sums) make two runs of the same step differ
        # in the last bits, and training amplifies that a little from step to step
        torch.testing.assert_close(og["loss_terms"][:6], oe["loss_terms"][:6], rtol=2e-3, atol=1e-6)
    torch.cuda.synchronize()
    assert graph.global_step == eager.global_step == STEPS
    assert int(graph.step_dev.item()) == STEPS            # the device counter advanced once per replay
    for name in ("scale", "adam_t", "tracker"):
        assert torch.equal(getattr(graph, name), getattr(eager, name)), name
    # Adam (eps 1e-15) turns last-bit differences of near-zero gradients into full-size
    # updates: the graph must stay within 4x the spread of two eager runs (or 4e-3; one sample
    # of that spread: amp measured rel 2.1e-3 against a spread of 0.64e-3 once the scatter summed
    # its runs in fp16 — a schedule or capture error moves P by far more)
    for name in ("P", "M", "V"):
        a, b = getattr(graph, name), getattr(eager, name)
        rel = float((a - b).norm() / b.norm().clamp_min(1e-30))
        spread = float((getattr(eager2, name) - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < max(4e-3, 4 * spread), (name, rel, spread)


def test_graph_recaptures_when_a_knob_changes(cuda_device):
    """A captured graph bakes host values in (kernel shape knobs, loss weights): changing
    one between two graph steps must capture again, so graph and eager steps stay the
    same computation (the key used to hold only the call's arguments)."""
    import bench
    dev = cuda_device
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, 2, dict(amp=True), dev)
    fs = _trainer(dev, (cfg, pool, frame_start, c2w, occ), True)
    fs.graph_step(256)
    g0 = fs._graphs[1][0]
    fs.graph_step(256)
    assert fs._graphs[1][0] is g0                          # same knobs: replayed
    fs.scatter_levels_per_wave = 4
    fs.graph_step(256)
    g1 = fs._graphs[1][0]
    assert g1 is not g0                                    # kernel shape knob: captured again
    cfg["fs_rgb_weight"] = 10.0
    fs.graph_step(256)
    assert fs._graphs[1][0] is not g1                      # loss weight: captured again
    torch.cuda.synchronize()


@pytest.mark.parametrize("amp", [True, False], ids=["amp", "fp32"])
def test_graph_step_ids_matches_eager(cuda_device, amp):
    """NerfRunner.train()'s batches (pool-uniform randperm slices, DataLoader) through the
    captured step (graph_step_ids) replay the eager step on the same ids; an eager step of
    another batch size in between re-allocates the buffers and forces a re-capture."""
    import bench
    from bundlesdf_amd.nerf_runner import DataLoader
    dev = cuda_device
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(
        0, 1, 4, dict(amp=amp, trunc_decay_type="linear", trunc_start=0.03, n_step=40), dev)
    scene = (cfg, pool, frame_start, c2w, occ)
    eager, graph = _trainer(dev, scene, amp), _trainer(dev, scene, amp)
    eager2 = _trainer(dev, scene, amp)   # run-to-run spread of the eager step itself (float atomics)
    torch.manual_seed(0)
    dl = DataLoader(pool, 1024)
    for gs in range(STEPS):
        ids = dl.next_ids()
        if gs == 7:   # an eager step of another size on both: buffers re-allocated
            other = dl.next_ids()[:300]
            eager.step(ids=other, seed=3)
            eager2.step(ids=other, seed=3)
            graph.step(ids=other, seed=3)
            assert graph._graphs is None
        oe = eager.step(ids=ids, seed=3)
        eager2.step(ids=ids, seed=3)
        og = graph.graph_step_ids(ids, seed_base=3)
        torch.testing.assert_close(og["loss_terms"][:6], oe["loss_terms"][:6], rtol=2e-3, atol=1e-6)
    torch.cuda.synchronize()
    assert graph.global_step == eager.global_step == STEPS + 1
    for name in ("scale", "adam_t", "tracker"):
        assert torch.equal(getattr(graph, name), getattr(eager, name)), name
    # Adam (eps 1e-15) turns last-bit differences of near-zero gradients into full-size
    # updates, so parameters drift apart over the steps even between two eager runs: the
    # graph must stay within 3x that spread (or 2e-3)
    for name in ("P", "M", "V"):
        b = getattr(eager, name)
        rel = float((getattr(graph, name) - b).norm() / b.norm().clamp_min(1e-30))
        spread = float((getattr(eager2, name) - b).norm() / b.norm().clamp_min(1e-30))
        assert rel < max(2e-3, 3 * spread), (name, rel, spread)


@pytest.mark.parametrize("amp", [True, False], ids=["amp", "fp32"])
def test_graph_step_epoch_matches_graph_step_ids(cuda_device, amp):
    """NerfRunner.train()'s captured step reading its batch slice on the device
    (graph_step_epoch -> nof_trace_rays_epoch: slice step - epoch_step0 of the DataLoader's one
    permutation buffer, no per-step id copy) against graph_step_ids on the same DataLoader draws,
    through two epoch reshuffles (a 5,000-ray permutation: 4 slices of 1,024 per epoch): the same
    batch rows gathered every step (bit-identical), the same losses."""
    import bench
    from bundlesdf_amd.nerf_runner import DataLoader
    dev = cuda_device
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, 4, dict(amp=amp, n_step=40), dev)
    scene = (cfg, pool, frame_start, c2w, occ)
    a, b = _trainer(dev, scene, amp), _trainer(dev, scene, amp)
    torch.manual_seed(0)
    dl_a = DataLoader(pool[:5000], 1024)
    torch.manual_seed(0)
    dl_b = DataLoader(pool[:5000], 1024)
    firsts = 0
    for it in range(11):
        if it == 6:   # a reset step count mid-epoch (bench.py's re-initialisation): the slice index rules
            a.reset_state(a.P.detach().clone())
            b.reset_state(b.P.detach().clone())
        st = torch.get_rng_state()   # both loaders draw their epoch reshuffles from the same CPU state
        ids = dl_a.next_ids()
        oa = a.graph_step_ids(ids, seed_base=3)
        torch.set_rng_state(st)
        perm, k = dl_b.next_slice()
        firsts += int(k == 0)
        ob = b.graph_step_epoch(perm, k, 1024, seed_base=3)
        torch.cuda.synchronize()
        assert torch.equal(a.rays, b.rays), it
        torch.testing.assert_close(ob["loss_terms"][:6], oa["loss_terms"][:6], rtol=2e-3, atol=1e-6)
    assert firsts == 3 and b.global_step == a.global_step
    # a slice past the permutation is refused on the host (the device would read past the buffer)
    with pytest.raises(RuntimeError, match="outside"):
        b.graph_step_epoch(perm, 4, 1024, seed_base=3)


def test_trace_rays_epoch_abi_reads_the_step_slice(cuda_device):
    """nof_trace_rays_epoch through the C ABI: with the device step block at step 7 and epoch_step0 = 5 it
    traces slice 2 of the permutation — the same rays, intervals, totals and counts as nof_trace_rays on
    that slice given explicitly; NULL step block or epoch_step0 is refused (NOF_EINVAL)."""
    import bench
    from bundlesdf_amd import _lib
    from bundlesdf_amd.fused import truncation
    dev = cuda_device
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, 4, dict(amp=True), dev)
    fs = _trainer(dev, (cfg, pool, frame_start, c2w, occ), True)
    fs._prologue()
    R, n = 512, int(fs.pool.shape[0])
    perm = torch.randperm(n, generator=torch.Generator().manual_seed(3)).to(torch.int32).to(dev)
    spc = _lib.StepParams(lr0=1e-2, lr1=1e-3, trunc=float(truncation(cfg, 0)), seed=1, batch_seed=2, step=7)
    sp = torch.frombuffer(bytearray(bytes(spc)), dtype=torch.uint8).to(dev)
    step0 = torch.tensor([5], dtype=torch.int32, device=dev)
    L = _lib.lib()
    sc = cfg["sc_factor"]

    def outs():
        return (torch.zeros(R, 12, device=dev), torch.full((R, fs.Kmax, 2), -1.0, device=dev), torch.zeros(R, device=dev),
                torch.zeros(R, dtype=torch.int32, device=dev))

    common = (_lib.ptr(fs.tf_buf), _lib.ptr(fs.occ), fs.Nocc, fs.Kmax, cfg["near"] * sc, cfg["far"] * sc, 0.0)
    a = outs()
    _lib.check(L.nof_trace_rays_epoch(_lib.ptr(fs.pool), _lib.ptr(perm), _lib.ptr(step0), R, *common,
                                      *[_lib.ptr(t) for t in a], _lib.ptr(sp), _lib.stream_of(fs.pool)), "epoch")
    b = outs()
    ids = perm[2 * R:3 * R].contiguous()
    _lib.check(L.nof_trace_rays(_lib.ptr(fs.pool), _lib.ptr(ids), R, *common, *[_lib.ptr(t) for t in b],
                                _lib.ptr(sp), _lib.stream_of(fs.pool)), "slice")
    torch.cuda.synchronize()
    assert int(a[3].sum()) > 0
    torch.testing.assert_close(a[0], fs.pool[ids.long()], rtol=0, atol=0)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
    for bad in ((_lib.ptr(step0), None), (None, _lib.ptr(sp))):
        rc = L.nof_trace_rays_epoch(_lib.ptr(fs.pool), _lib.ptr(perm), bad[0], R, *common, *[_lib.ptr(t) for t in a],
                                    bad[1], _lib.stream_of(fs.pool))
        assert rc != 0 and b"epoch_step0" in L.nof_last_error()
