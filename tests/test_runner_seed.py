"""A1 index-exactness (CPU): under set_seed(0) the drop-in trainer consumes the
CPU generator in the reference's order, so its initial parameters and every
batch of ray ids are the reference's own — pinned by G7
(tests/golden/runner_seed.npz: the reference's NerfRunner.__init__ / train() /
add_new_frames(reuse_weights=False) / train() run from /root/reference by
tests/golden/make_golden.py). This test drives the same generator sequence
through this package's create_nerf and DataLoader on the CPU (no device); the
GPU test tests/test_gpu_runner.py::test_runner_seed_and_batches_match_reference
runs the whole NerfRunner on the device against the same fixture."""
import json
import os

import numpy as np
import torch

from bundlesdf_amd import nerf_runner as NR


def _fixture(golden_dir):
    g = np.load(os.path.join(golden_dir, "runner_seed.npz"))
    return g, json.loads(str(g["cfg_json"]))


def state_of(models):
    d = {"embeddings": models["embed_fn"].embeddings.detach().cpu().numpy(),
         "pose": models["pose_array"].data.detach().cpu().numpy(),
         "features": models["feature_array"].data.detach().cpu().numpy()}
    d.update({k: v.detach().cpu().numpy() for k, v in models["model"].state_dict().items()})
    return d


def check_state(prefix, got, g):
    keys = [k[len(prefix):] for k in g.files if k.startswith(prefix) and k[len(prefix):] in got]
    assert {"embeddings", "pose", "features", "sigma_net.0.weight", "color_net.4.bias"} <= set(keys)
    for k in keys:
        np.testing.assert_array_equal(got[k], g[prefix + k], err_msg=prefix + k)


def _cpu_runner(cfg, n_frames):
    r = object.__new__(NR.NerfRunner)
    r.cfg, r.images, r.octree_m, r.device = dict(cfg), [None] * n_frames, None, torch.device("cpu")
    return r


def _train_ids(dl, n_iters):
    NR.set_seed(0)                              # NerfRunner.train (nerf_runner.py:855)
    return np.stack([dl.next_ids().numpy() for _ in range(n_iters)])


def test_seed_order_reproduces_reference_init_and_batches(golden_dir):
    g, cfg = _fixture(golden_dir)
    seq = json.loads(str(g["seq_json"]))
    n_iters = cfg["n_step"] + 1
    # round 0: NerfRunner.__init__ — set_seed(0), create_nerf, the pool's DataLoader
    NR.set_seed(0)
    r = _cpu_runner(cfg, seq["n_init"])
    r.create_nerf()
    check_state("r0_", state_of(r.models), g)
    dl = NR.DataLoader(torch.empty(int(g["r0_pool"][0]), 12), cfg["N_rand"])
    np.testing.assert_array_equal(dl.ids[:2048].numpy(), g["r0_perm_head"])
    np.testing.assert_array_equal(_train_ids(dl, n_iters), g["r0_ids"])
    # round 1: add_new_frames(reuse_weights=False) re-creates the networks from the generator
    # state train() left (bundlesdf.py:223, nerf_runner.py:379-380), then a new DataLoader
    r.images = [None] * seq["n_frames"]
    r.create_nerf()
    check_state("r1_", state_of(r.models), g)
    dl = NR.DataLoader(torch.empty(int(g["r1_pool"][0]), 12), cfg["N_rand"])
    np.testing.assert_array_equal(_train_ids(dl, n_iters), g["r1_ids"])
    # the batches run through an epoch boundary (a reshuffle) in both rounds
    assert n_iters * cfg["N_rand"] > max(int(g["r0_pool"][0]), int(g["r1_pool"][0]))
