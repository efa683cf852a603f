"""Worker for tests/test_dp_gloo.py (one process per rank, gloo on CPU).

Each rank runs the CPU oracle training step on its equal-sized shard of the
G4 ray batch, flattens the parameter gradients into the [table | mlp | pose]
bucket layout FusedStep uses, and calls the production exchange
(bundlesdf_amd.fused.allreduce_gradients). The result must equal the
full-batch gradient of the reference's own train_loop (G4)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def _flat(G, keys):
    return torch.cat([G["embeddings"].reshape(-1)] + [G[k].reshape(-1) for k in keys] + [G["pose"].reshape(-1)])


def _sharded_amp(G, n_emb, n_mlp, world, rank, scale):
    import types
    from bundlesdf_amd import exchange as EX
    from tests._exchange_worker import TorchOps
    N = G.numel()
    fs = types.SimpleNamespace(n_emb=n_emb, mlp_off=n_emb, feat_off=n_emb + n_mlp, pose_off=n_emb + n_mlp, amp=True,
                               growth_interval=2000, global_step=0,
                               cfg=dict(n_step=500, lrate=0.01, lrate_pose=0.01, decay_rate=0.1))
    fs.P = torch.zeros(N)
    fs.M, fs.V = torch.zeros(N), torch.zeros(N)
    fs.Gbuf = torch.zeros(N + 1)
    fs.G = fs.Gbuf[:N]
    fs.G16 = torch.zeros(n_emb, dtype=torch.float16)
    fs.scale = torch.tensor([scale])
    fs.found_inf, fs.tracker, fs.adam_t = (torch.zeros(1, dtype=torch.int32) for _ in range(3))
    ex = EX.ShardedExchange(fs, TorchOps(fs), world, rank)
    fs.G16.copy_((G[:n_emb] * scale).half())
    fs.G[n_emb:] = G[n_emb:] * scale
    grads = ex.step(debug=True)
    assert int(fs.adam_t.item()) == 1        # not skipped
    return grads


def run(rank, world, port, golden, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from bundlesdf_amd.fused import allreduce_gradients
    from oracle import nerf_step as NS
    g = np.load(golden)
    cfg = json.loads(str(g["cfg_json"]))
    R = g["batch"].shape[0]
    lo, hi = rank * R // world, (rank + 1) * R // world
    P0 = {"embeddings": torch.from_numpy(g["emb0"]), "pose": torch.from_numpy(g["pose0"])}
    for k in NS.MLP_KEYS:
        P0[k] = torch.from_numpy(g["w0_" + k])
    meta = (g["offsets"], float(np.log2(g["per_level_scale"][0])), cfg["base_res"])
    out = NS.train_step(P0, torch.from_numpy(g["batch"][lo:hi]), torch.from_numpy(g["c2w"]), g["occ"], cfg,
                        torch.from_numpy(g["t_rand"][lo:hi]), meta, step=0)
    G = _flat(out["grads"], NS.MLP_KEYS).float().contiguous()
    n_emb = out["grads"]["embeddings"].numel()
    n_mlp = sum(out["grads"][k].numel() for k in NS.MLP_KEYS)
    # fp32 mode: the flat [table | mlp | pose] bucket
    Gf = G.clone()
    allreduce_gradients(Gf, world)
    # amp mode, as FusedStep does it: every gradient carries the GradScaler scale; the
    # table gradient was accumulated in fp16 (G16) and is moved into the fp32 bucket
    # (nof_grad16_to_f32) before the one all-reduce; unscaled afterwards
    scale = 1024.0
    G16 = (G[:n_emb] * scale).half()
    Ga = G * scale
    Ga[:n_emb] = G16.float()
    allreduce_gradients(Ga, world)
    Ga /= scale
    # amp through the production sharded exchange (exchange.ShardedExchange over the torch
    # restatements of the optimiser kernels): fp16 table gradient pre-scaled by 1/W2 and
    # reduce-scattered in fp16, rest bucket all-reduced, unscaled (debug returns the gradient)
    Gsh = _sharded_amp(G, n_emb, n_mlp, world, rank, scale)
    # per-entry bound of the fp16 roundings: sum over ranks of |local table gradient|
    A = G[:n_emb].abs().clone()
    torch.distributed.all_reduce(A)
    A /= world
    ref = np.concatenate([g["g_emb"].ravel()] + [g["g_" + k].ravel() for k in NS.MLP_KEYS] + [g["g_pose"].ravel()])
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), fp32=Gf.numpy(), amp=Ga.numpy(), abs_table=A.numpy(),
             ref=ref, n_emb=n_emb, n_mlp=n_mlp, sharded=Gsh.numpy())
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
