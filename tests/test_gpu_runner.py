"""GPU: the NerfRunner drop-in trains end to end through the fused HIP path
(constructor -> octree -> ray pool -> train), exposes models['pose_array'],
and continues after add_new_frames (reuse_weights=True)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_nerf_runner_trains_and_adds_frames(cuda_device):
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.nerf_runner import NerfRunner
    seq = SY.make_sequence(4, seed=1)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"], n_step=40, N_rand=1024,
                         num_levels=16, amp=True)
    nr = NerfRunner(cfg, seq["rgbs"][:3], seq["depths"][:3], seq["masks"][:3], None, seq["poses"][:3], seq["K"],
                    build_octree_pcd=seq["octree_pts"])
    assert nr.rays.is_cuda and nr.rays.shape[1] == 12
    assert set(np.unique(nr.rays[:, 8].cpu().numpy()).astype(int)) == {0, 1, 2}
    losses = []
    for _ in range(3):
        nr.N_iters = 15
        out = nr.train()
        losses.append(float(out["loss_terms"][:4].sum()))
    assert np.isfinite(losses).all() and losses[-1] < losses[0], losses
    pa = nr.models["pose_array"]
    assert pa.data.shape == (3, 6) and torch.isfinite(pa.data).all()
    assert pa.get_matrices(torch.arange(3, device=cuda_device)).shape == (3, 4, 4)
    n_before = nr.rays.shape[0]
    nr.add_new_frames(seq["rgbs"][3:], seq["depths"][3:], seq["masks"][3:], None, seq["poses"], reuse_weights=True)
    assert nr.rays.shape[0] > n_before and nr.models["pose_array"].data.shape == (4, 6)
    nr.N_iters = 10
    out = nr.train()
    assert np.isfinite(float(out["loss_terms"][:4].sum()))


def test_query_sdf_matches_oracle(cuda_device):
    """nof_query_sdf (fused encode + sigma net) vs the CPU oracle (grid encode +
    NeRFSmall forward) in fp32, points and grid mode, occupancy fill."""
    import json
    import os
    from bundlesdf_amd.fused import FusedStep
    from bundlesdf_amd.grid import GridEncoder
    from bundlesdf_amd.nerf_helpers import NeRFSmall, PoseArray
    from oracle import kernels as K
    from oracle import nerf_step as NS
    golden = os.path.join(os.path.dirname(__file__), "golden", "train_step.npz")
    g = np.load(golden)
    cfg = json.loads(str(g["cfg_json"]))
    dev = cuda_device
    L = cfg["num_levels"]
    enc = GridEncoder(3, L, 2, cfg["base_res"], cfg["log2_hashmap_size"], cfg["finest_res"]).to(dev)
    enc.embeddings.data.copy_(torch.from_numpy(g["emb0"]) * 300)
    net = NeRFSmall(2, 64, 15, 3, 64, input_ch=2 * L, input_ch_views=9).to(dev)
    net.load_state_dict({k: torch.from_numpy(g["w0_" + k]) for k in NS.MLP_KEYS})
    pa = PoseArray(g["pose0"].shape[0], 0.1, 20.0).to(dev)
    fs = FusedStep(cfg, torch.from_numpy(g["batch"]).to(dev), torch.from_numpy(g["c2w"]), torch.from_numpy(g["occ"]),
                   enc, net, pa, amp=False)
    rng = np.random.default_rng(0)
    pts = rng.uniform(-1.1, 1.1, (3000, 3)).astype(np.float32)
    got = fs.query_sdf(points=torch.from_numpy(pts)).cpu().numpy()
    x01 = (np.clip(pts, -1, 1) + 1) / 2
    feat, _ = K.grid_encode_forward(x01, enc.embeddings.detach().cpu().numpy(), enc.offsets.cpu().numpy(),
                                    float(np.log2(enc.per_level_scale)), cfg["base_res"])
    feat = torch.from_numpy(feat.transpose(1, 0, 2).reshape(len(pts), -1))
    W = {k: v.detach().cpu() for k, v in net.state_dict().items()}
    ref = NS.nerf_small(torch.cat([feat, torch.zeros(len(pts), 9)], -1), W)[:, 3].numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-5)
    # grid mode + occupancy fill
    ax = [np.linspace(-0.9, 0.9, 7), np.linspace(-0.8, 0.8, 5), np.linspace(-0.7, 0.7, 6)]
    occ = torch.zeros(4, 4, 4, dtype=torch.uint8)
    occ[:, :, :2] = 1          # x < 0 occupied
    sg = fs.query_sdf(axes=ax, occ=occ).cpu().numpy().reshape(7, 5, 6)
    q = np.stack(np.meshgrid(*ax, indexing="ij"), -1).astype(np.float32).reshape(-1, 3)
    sp = fs.query_sdf(points=torch.from_numpy(q)).cpu().numpy().reshape(7, 5, 6)
    xs = ax[0][:, None, None] * np.ones((1, 5, 6))
    # linspace's middle sample is -1e-16, not 0: it lands in voxel 2 (free), so split at +-0.1
    np.testing.assert_allclose(sg[xs < -0.1], sp[xs < -0.1], rtol=1e-6)
    assert (sg[xs > -0.1] == 1.0).all()


def test_extract_mesh_after_training(cuda_device, tmp_path):
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.nerf_runner import NerfRunner
    seq = SY.make_sequence(3, seed=2)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"], n_step=150, N_rand=2048,
                         num_levels=16, amp=True)
    nr = NerfRunner(cfg, seq["rgbs"], seq["depths"], seq["masks"], None, seq["poses"], seq["K"],
                    build_octree_pcd=seq["octree_pts"])
    nr.train()
    mesh = nr.extract_mesh(voxel_size=0.004)
    assert mesh is not None and len(mesh.faces) > 100
    assert np.abs(mesh.vertices).max() <= 1.0 + 1e-6
    # the surface sits on the synthetic object: distance of the vertices (back in
    # world metres) to the analytic sphere-union-box surface
    from bundlesdf_amd.mesh import largest_component, mesh_to_real_world
    mesh = largest_component(mesh)        # bundlesdf.py:748-759
    pw = mesh_to_real_world(mesh, np.eye(4), seq["translation"], seq["sc_factor"]).vertices
    d_sph = np.linalg.norm(pw, axis=1) - SY.SPHERE_R
    q = np.abs(pw - SY.BOX_C) - SY.BOX_H
    d_box = np.linalg.norm(np.maximum(q, 0), axis=1) + np.minimum(q.max(1), 0)
    err = np.abs(np.minimum(d_sph, d_box))
    print(f"mesh: {len(mesh.vertices)} verts, |sdf| median {np.median(err) * 1e3:.2f} mm, "
          f"p90 {np.percentile(err, 90) * 1e3:.2f} mm, within 3 mm {np.mean(err < 3e-3):.2f}")
    # the tail is the inner shell where the trained (negative) sdf meets the 1.0
    # fill of empty octree voxels inside the object — the reference's mesh has it too
    assert np.median(err) < 2e-3
    mesh, sigma, q = nr.extract_mesh(voxel_size=0.008, return_sigma=True)
    assert sigma.ndim == 3 and q.shape[-1] == 3
    mesh.export(str(tmp_path / "m.ply"))


def test_texture_from_train_images(cuda_device, tmp_path):
    """mesh_texture_from_train_images end to end on the extracted mesh: the baked
    texels hold the frames' colours (procedural albedo of the synthetic object)."""
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.nerf_runner import NerfRunner
    seq = SY.make_sequence(3, seed=2)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"], n_step=100, N_rand=2048,
                         num_levels=16, amp=True)
    nr = NerfRunner(cfg, seq["rgbs"], seq["depths"], seq["masks"], None, seq["poses"], seq["K"],
                    build_octree_pcd=seq["octree_pts"])
    nr.train()
    mesh = nr.extract_mesh(voxel_size=0.006)
    raw = (seq["rgbs"] * 255).astype(np.float32)
    tm = nr.mesh_texture_from_train_images(mesh, raw, tex_res=512)
    assert tm.uv.shape == (len(tm.vertices), 2) and tm.texture.shape == (512, 512, 3)
    filled = tm.texture.reshape(-1, 3).max(1) > 0
    assert filled.mean() > 0.02, filled.mean()
    tm.export(str(tmp_path / "tex.obj"))
    assert (tmp_path / "tex.png").stat().st_size > 1000 and (tmp_path / "tex.mtl").exists()


def test_nerf_runner_global_refine_frame_features(cuda_device, tmp_path):
    """Global-refine settings (run_custom.py:122-133: S = 64 + 256, finest 256,
    frame_features 2, rgb_weight 100): the FeatureArray is created (nerf_runner.py:234-235),
    trained through the fused path, saved, and re-created for new frames (:384-385)."""
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.nerf_runner import NerfRunner
    seq = SY.make_sequence(4, seed=2)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"], n_step=20, N_rand=1024,
                         num_levels=16, amp=True, N_samples=64, N_samples_around_depth=256, finest_res=256,
                         first_frame_weight=1, fs_sdf=0.1, frame_features=2, rgb_weight=100)
    nr = NerfRunner(cfg, seq["rgbs"][:3], seq["depths"][:3], seq["masks"][:3], None, seq["poses"][:3], seq["K"],
                    build_octree_pcd=seq["octree_pts"])
    fa = nr.models["feature_array"]
    assert fa is not None and fa.data.shape == (3, 2)
    assert nr.models["model"].color_net[0].weight.shape == (64, 2 + 9 + 15)
    f0 = fa.data.detach().clone()
    out = nr.train()
    lt = out["loss_terms"].cpu().numpy()
    assert np.isfinite(lt).all() and lt[6] > 0                      # reg_features reported
    f1 = nr.models["feature_array"].data.detach()
    assert torch.isfinite(f1).all() and (f1 - f0).abs().max() > 1e-4   # the latent code trains
    nr.save_weights(str(tmp_path / "w.pth"))
    sd = torch.load(str(tmp_path / "w.pth"), weights_only=False)   # written by this test
    assert sd["feature_array"]["data"].shape == (3, 2)
    # load_weights restores the frame codes in place (nerf_runner.py:537-538)
    with torch.no_grad():
        nr.models["feature_array"].data.zero_()
    nr.load_weights(str(tmp_path / "w.pth"))
    torch.testing.assert_close(nr.models["feature_array"].data.detach(), f1)
    nr.add_new_frames(seq["rgbs"][3:], seq["depths"][3:], seq["masks"][3:], None, seq["poses"], reuse_weights=True)
    fa2 = nr.models["feature_array"]
    assert fa2.data.shape == (4, 2)
    # the trained codes of the first 3 frames carry over (:384-386); the new frame's row is new
    torch.testing.assert_close(fa2.data.detach()[:3], f1)
    assert fa2.data.data_ptr() == nr.trainer.P.data_ptr() + 4 * nr.trainer.feat_off
    nr.N_iters = 5
    out = nr.train()
    assert np.isfinite(out["loss_terms"].cpu().numpy()).all()


def test_add_new_frames_reuse_weights_frozen_poses(cuda_device):
    """optimize_poses = 0 (the trainer keeps a frozen identity stand-in PoseArray):
    add_new_frames(reuse_weights=True) resizes it with the frame count and training
    continues; the network weights carry over."""
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.nerf_runner import NerfRunner
    seq = SY.make_sequence(4, seed=3)
    cfg = SY.default_cfg(sc_factor=seq["sc_factor"], translation=seq["translation"], n_step=10, N_rand=512,
                         num_levels=8, amp=True, optimize_poses=0)
    nr = NerfRunner(cfg, seq["rgbs"][:2], seq["depths"][:2], seq["masks"][:2], None, seq["poses"][:2], seq["K"],
                    build_octree_pcd=seq["octree_pts"])
    nr.train()
    w = nr.models["model"].sigma_net[0].weight.detach().clone()
    nr.add_new_frames(seq["rgbs"][2:], seq["depths"][2:], seq["masks"][2:], None, seq["poses"], reuse_weights=True)
    assert nr.models["pose_array"].data.shape == (4, 6)
    torch.testing.assert_close(nr.models["model"].sigma_net[0].weight.detach(), w)
    nr.N_iters = 3
    out = nr.train()
    assert np.isfinite(out["loss_terms"].cpu().numpy()).all()
    assert float(nr.models["pose_array"].data.abs().max()) == 0.0     # frozen: lrate_pose 0


def test_runner_seed_and_batches_match_reference(cuda_device, golden_dir):
    """A1 + the online call path, against G7 (tests/golden/runner_seed.npz: the reference's
    own NerfRunner run from /root/reference, make_golden.py gen_runner_seed): the device
    NerfRunner built from the same frames starts from the reference's initial parameters bit
    for bit, builds a pool of the same size and trains on the reference's batches, index for
    index, through an epoch reshuffle. Then the call bundlesdf.py:223 makes —
    add_new_frames(..., new_pcd=cloud, reuse_weights=False) — re-initialises the networks
    exactly as the reference's create_nerf does at that point of the generator sequence,
    rebuilds the octree from the down-sampled new cloud (nerf_runner.py:372-375), and
    train() again runs the reference's batches."""
    import hashlib
    import json
    import os
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.nerf_runner import NerfRunner
    from bundlesdf_amd.octree import build_occupancy
    from tests.golden.make_golden import g7_clouds
    from tests.test_runner_seed import check_state, state_of
    g = np.load(os.path.join(golden_dir, "runner_seed.npz"))
    cfg, sq = json.loads(str(g["cfg_json"])), json.loads(str(g["seq_json"]))
    seq = SY.make_sequence(sq["n_frames"], seed=sq["seed"])
    np.testing.assert_allclose([float(np.sum(seq[k], dtype=np.float64)) for k in ("rgbs", "depths", "masks")],
                               g["inputs_checksum"], rtol=1e-12)
    n0 = sq["n_init"]
    cloud0, cloud1 = g7_clouds(seq)
    nr = NerfRunner(dict(cfg), seq["rgbs"][:n0], seq["depths"][:n0], seq["masks"][:n0], None, seq["poses"][:n0],
                    seq["K"], build_octree_pcd=cloud0)
    check_state("r0_", state_of(nr.models), g)
    assert nr.rays.shape[0] == int(g["r0_pool"][0])
    np.testing.assert_array_equal(nr.data_loader.ids[:2048].cpu().numpy(), g["r0_perm_head"])

    def recorded_train():
        log, real = [], nr.data_loader.next_ids

        def rec():
            ids = real()
            log.append(ids.cpu().numpy().copy())
            return ids
        nr.data_loader.next_ids = rec
        out = nr.train()
        return np.stack(log), out
    ids0, out = recorded_train()
    np.testing.assert_array_equal(ids0, g["r0_ids"])
    assert np.isfinite(out["loss_terms"][:4].cpu().numpy()).all()
    occ_before = nr.octree_m.occ_finest.clone()
    nr.add_new_frames(seq["rgbs"][n0:], seq["depths"][n0:], seq["masks"][n0:], None, seq["poses"], occ_masks=None,
                      new_pcd=cloud1, reuse_weights=False)
    check_state("r1_", state_of(nr.models), g)
    bp = np.ascontiguousarray(nr.build_octree_pts, np.float64)
    assert len(bp) == int(g["r1_octree_n"][0])
    np.testing.assert_array_equal(bp[:64], g["r1_octree_head"])
    assert hashlib.sha256(bp.tobytes()).hexdigest() == str(g["r1_octree_sha"])
    # the octree was rebuilt from the new cloud
    dil = max(1, int(np.ceil(cfg["octree_dilate_size"] / cfg["octree_smallest_voxel_size"])))
    want = build_occupancy(torch.as_tensor(bp, dtype=torch.float32, device=cuda_device), nr.octree_m.max_level, dil)
    assert torch.equal(nr.octree_m.occ_finest, want) and not torch.equal(occ_before, want)
    assert nr.rays.shape[0] == int(g["r1_pool"][0])
    ids1, out = recorded_train()
    np.testing.assert_array_equal(ids1, g["r1_ids"])
    assert np.isfinite(out["loss_terms"][:4].cpu().numpy()).all()
