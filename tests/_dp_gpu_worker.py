"""Worker for tests/test_gpu_dp.py: one rank of the N=2 data-parallel training
step (BASELINE config 4's code path) on the GPU. Both ranks share
cuda:0 and exchange over gloo (RCCL needs one GPU per rank; the production
collective is the same torch.distributed.all_reduce call).

Each rank builds FusedStep(world_size=2) on its half of a fixed batch and runs
K_STEPS steps with injected stratification draws (t_rand rows of its half),
eager or replayed from the captured two-graph split (field graph | RCCL/gloo
all-reduce | optimiser graph), in fp32 and amp. After every step it saves the
exchanged (unscaled) gradient and the optimiser state for the parent test,
which compares them with a single-process FusedStep on the whole batch."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

K_STEPS = 3
# (amp, execution[_variant], exchange): fp32 all-reduces; amp shards the table's optimiser state
# (exchange.py) by default, and its replicated all-reduce variant is kept covered too
MODES = [(False, "eager", "allreduce"), (False, "graph", "allreduce"), (True, "eager", "sharded"),
         (True, "graph", "sharded"), (True, "eager_ar", "allreduce")]
W_SCALE_RESET = 65536.0   # reset_state's scale (the first step of a round)
AMP_SCALE = 1024.0       # the scene case's fp16 weight gradients overflow at the GradScaler's initial 2^16


def case(name):
    """(cfg, batch [R,12], c2w, occ, emb, mlp_w, pose, grid shape) of a named parity case."""
    from oracle import nerf_step as NS
    if name == "g4":
        import json
        g = np.load(os.path.join(ROOT, "tests", "golden", "train_step.npz"))
        cfg = json.loads(str(g["cfg_json"]))
        mlp_w = {k: g["w0_" + k] for k in NS.MLP_KEYS}
        return (cfg, g["batch"], np.asarray(g["c2w"], np.float32), g["occ"], g["emb0"], mlp_w, g["pose0"],
                (cfg["num_levels"], cfg["log2_hashmap_size"], cfg["finest_res"], cfg["base_res"]))
    from tests.test_gpu_step import _scene_case
    cfg, seq, batch, occ, _, mlp_w, emb, pose, _ = _scene_case(seed=47, R=256)
    return cfg, batch, np.asarray(seq["poses"], np.float32), occ, emb, mlp_w, pose, (16, 22, 128, 16)


def t_rand_of(step, R, S):
    return np.random.default_rng(1000 + step).uniform(size=(R, S)).astype(np.float32)


def make_step(dev, c, amp, lo, hi, world, pg, exchange=None):
    from bundlesdf_amd.fused import FusedStep
    from tests.test_gpu_step import _build
    cfg, batch, c2w, occ, emb, mlp_w, pose, (L, log2T, finest, base) = c
    cfg = dict(cfg, amp=amp)
    enc, net, pa = _build(dev, cfg, emb, mlp_w, pose, L, log2T, finest, base)
    fs = FusedStep(cfg, torch.from_numpy(np.ascontiguousarray(batch[lo:hi])).to(dev), torch.from_numpy(c2w),
                   torch.from_numpy(occ), enc, net, pa, amp=amp, process_group=pg, world_size=world,
                   exchange=exchange)
    if amp:
        fs.scale.fill_(AMP_SCALE)
    return fs


def run_steps(fs, mode, lo, hi, R_all, S, poison_step=None, poison="mlp", capture_local=False):
    """K_STEPS steps of the rows [lo, hi) of an R_all-ray batch (t_rand rows likewise);
    returns per-step dicts of host arrays. capture_local: step 0 also returns the rank's LOCAL
    (scaled) fp16 table gradient as it enters the exchange (grad_hook: after the backward)."""
    ids = torch.arange(hi - lo, dtype=torch.int32, device=fs.dev)
    out = []
    for k in range(K_STEPS):
        tr = torch.from_numpy(np.ascontiguousarray(t_rand_of(k, R_all, S)[lo:hi]))
        hook = None
        local = {}
        if poison_step is not None and k == poison_step:
            def hook(f):
                if poison == "mlp":
                    f.G[f.mlp_off + 5] = float("inf")
                else:   # a row of the last table shard (rank 1 owns it; rank 0 learns of it from the flag)
                    f.G16[f.n_emb - 3] = float("inf")
        elif capture_local and k == 0:
            def hook(f):
                local["g16"] = f.G16.float().cpu().numpy()
        if mode == "graph" and hook is None:
            o = fs.graph_step_ids(ids, t_rand=tr)
            grads = None
        else:
            o = fs.step(ids=ids, t_rand=tr, debug=True, grad_hook=hook)
            grads = o["grads"].cpu().numpy()
        torch.cuda.synchronize()
        P = fs.master_params()              # the sharded exchange keeps 1/W of the table per rank
        M, V = fs.optimizer_state()
        out.append(dict(grads=grads, P=P.cpu().numpy(), M=M.cpu().numpy(), V=V.cpu().numpy(),
                        scale=float(fs.scale.item()), adam_t=int(fs.adam_t.item()), tracker=int(fs.tracker.item()),
                        loss=o["loss_terms"][:4].cpu().numpy(), local16=local.get("g16")))
    return out


def run(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    pg = torch.distributed.group.WORLD
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    res = {}
    for name in ("g4", "scene"):
        c = case(name)
        R = c[1].shape[0]
        S = c[0]["N_samples"] + c[0]["N_samples_around_depth"]
        lo, hi = rank * R // world, (rank + 1) * R // world
        for amp, mode, exchange in MODES:
            fs = make_step(dev, c, amp, lo, hi, world, pg, exchange)
            assert fs.exchange == exchange
            steps = run_steps(fs, mode.split("_")[0], lo, hi, R, S, capture_local=amp and mode == "eager")
            for k, st in enumerate(steps):
                for key, v in st.items():
                    if v is not None:
                        res[f"{name}/{int(amp)}/{mode}/{k}/{key}"] = np.asarray(v)
            del fs
        if name == "g4":
            # one rank's non-finite gradient reaches every replica through the exchange: all skip
            # (an MLP entry: the rest bucket's sum; a table entry: the shard's flag slot)
            for where in ("mlp", "table"):
                fs = make_step(dev, c, True, lo, hi, world, pg)
                steps = run_steps(fs, "eager", lo, hi, R, S, poison_step=1 if rank == 1 else None, poison=where)
                for k, st in enumerate(steps):
                    for key in ("P", "scale", "adam_t", "tracker"):
                        res[f"inf_{where}/{k}/{key}"] = np.asarray(st[key])
                del fs
            # a new round on the same buffers (reset_state, as bench.py does per round) whose first
            # step skips: the all-gathered fp16 mirror must be the fresh table, not the last round's
            fs = make_step(dev, c, True, lo, hi, world, pg)
            P0 = fs.P.detach().clone()
            run_steps(fs, "eager", lo, hi, R, S)
            fs.reset_state(P0)
            fs.scale.fill_(W_SCALE_RESET)
            ids = torch.arange(hi - lo, dtype=torch.int32, device=dev)

            def poison(f):
                f.G[f.mlp_off + 5] = float("inf")
            fs.step(ids=ids, t_rand=torch.from_numpy(np.ascontiguousarray(t_rand_of(0, R, S)[lo:hi])),
                    grad_hook=poison)
            torch.cuda.synchronize()
            fs.wait_exchange()   # the step left the mirror all-gather in flight
            res["reset_skip/adam_t"] = np.asarray(int(fs.adam_t.item()))
            res["reset_skip/emb16"] = fs.emb16.cpu().numpy()
            res["reset_skip/want"] = P0[:fs.n_emb].half().cpu().numpy()
            del fs
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
