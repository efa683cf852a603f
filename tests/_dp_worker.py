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
    # per-entry bound of the fp16 roundings: sum over ranks of |local table gradient|
    A = G[:n_emb].abs().clone()
    torch.distributed.all_reduce(A)
    A /= world
    ref = np.concatenate([g["g_emb"].ravel()] + [g["g_" + k].ravel() for k in NS.MLP_KEYS] + [g["g_pose"].ravel()])
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), fp32=Gf.numpy(), amp=Ga.numpy(), abs_table=A.numpy(),
             ref=ref, n_emb=n_emb, n_mlp=n_mlp)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
