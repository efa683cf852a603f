"""Worker for tests/test_exchange_gloo.py: one rank (gloo, CPU) running the
product exchange protocols of bundlesdf_amd/exchange.py — replicated and
sharded — over torch restatements of the optimiser kernels (the ops interface
FusedStep fills with libnof kernels). Gradients are dyadic and small (k / 1024,
|k| < 200: exact in fp16 after the sharded exchange's 1/W2 pre-scale, and their
sum over up to 8 ranks is exact in fp16 as well as fp32 in any order), so the two
protocols must end bit-identical whatever order the collectives add in."""
import os
import sys
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

N_EMB, N_MLP, N_FEAT, N_POSE = 1000, 37, 6, 12
STEPS = 5
INF_STEP, INF_RANK = 1, 3      # an inf in rank 0's table shard, produced on rank INF_RANK
INF_STEP2 = 3                  # an inf in the LAST rank's table shard, produced on rank 0 (rest finite)


class TorchOps:
    """fp32 torch restatement of k_grad16_to_f32 / k_unscale_check / k_adam / k_scaler_update
    (bundlesdf_amd/csrc/optim.hip) — the CPU stand-in behind the ops interface."""

    def __init__(self, fs):
        self.fs = fs

    def grad16_to_f32(self, src16, dst32, n):
        dst32[:n] = src16[:n].float()
        src16.zero_()

    def check16(self, g16, n):
        if not bool(torch.isfinite(g16[:n].float()).all()):
            self.fs.found_inf.fill_(1)

    def unscale_check(self, g, n, f16_lo=0, f16_hi=0):
        fs = self.fs
        raw = g[:n].clone()
        v = raw * (1.0 / fs.scale)
        g[:n] = v
        bad = ~torch.isfinite(v)
        if f16_hi > f16_lo:
            bad[f16_lo:f16_hi] |= raw[f16_lo:f16_hi].abs() >= 65520.0
        if bool(bad.any()):
            fs.found_inf.fill_(1)

    def adam(self, p, g, m, v, n, group1_start, mirror, sp, g16=None, active=None):
        from bundlesdf_amd.fused import lr_at
        fs = self.fs
        gi = g[:n].clone()
        g[:n] = 0.0
        if int(fs.found_inf.item()):
            return
        t = fs.adam_t.item() + 1
        b1, b2, eps = 0.9, 0.999, 1e-15
        bc1, bc2 = 1.0 - b1 ** t, 1.0 - b2 ** t
        lr0 = lr_at(fs.cfg, fs.global_step, fs.cfg["lrate"])
        lr1 = lr_at(fs.cfg, fs.global_step, fs.cfg["lrate_pose"])
        f32 = lambda x: float(np.float32(x))   # noqa: E731  (kernel scalars are float32)
        mm = m[:n] + f32(1.0 - b1) * (gi - m[:n])
        vv = v[:n] * f32(b2) + f32(1.0 - b2) * gi * gi
        denom = vv.sqrt() / f32(np.sqrt(bc2)) + f32(eps)
        ss = torch.full((n,), f32(lr0 / bc1))
        ss[group1_start:] = f32(lr1 / bc1)
        p[:n] = p[:n] + (-ss) * (mm / denom)
        m[:n], v[:n] = mm, vv
        if mirror is not None:
            mirror[:] = p[:mirror.numel()].half()

    def scaler_update(self):
        fs = self.fs
        inf = int(fs.found_inf.item())
        if not inf:
            fs.adam_t += 1
        if inf:
            fs.scale *= 0.5
            fs.tracker.zero_()
        else:
            fs.tracker += 1
            if int(fs.tracker.item()) == fs.growth_interval:
                fs.scale *= 2.0
                fs.tracker.zero_()
        fs.found_inf.zero_()


def make_fs(P0):
    fs = types.SimpleNamespace()
    fs.n_emb, fs.mlp_off = N_EMB, N_EMB
    fs.feat_off = N_EMB + N_MLP
    fs.pose_off = fs.feat_off + N_FEAT
    fs.P = P0.clone()
    fs.M, fs.V = torch.zeros_like(fs.P), torch.zeros_like(fs.P)
    fs.Gbuf = torch.zeros(fs.P.numel() + 1)
    fs.G = fs.Gbuf[:fs.P.numel()]
    fs.G16 = torch.zeros(N_EMB, dtype=torch.float16)
    fs.emb16 = fs.P[:N_EMB].half()
    fs.amp = True
    fs.scale = torch.tensor([1024.0])
    fs.found_inf = torch.zeros(1, dtype=torch.int32)
    fs.tracker = torch.zeros(1, dtype=torch.int32)
    fs.adam_t = torch.zeros(1, dtype=torch.int32)
    fs.growth_interval = 3
    fs.cfg = dict(n_step=10, lrate=0.01, lrate_pose=0.005, decay_rate=0.1)
    fs.global_step = 0
    return fs


def local_grads(rank, step, world):
    """This rank's scaled gradients of one step: dyadic, fp16-exact table part."""
    g = torch.Generator().manual_seed(1000 * step + rank)
    tab = torch.randint(-200, 200, (N_EMB,), generator=g).float() / 1024.0
    tab[torch.randint(0, N_EMB, (200,), generator=g)] = 0.0          # untouched rows
    rest = torch.randint(-4000, 4000, (N_MLP + N_FEAT + N_POSE,), generator=g).float() / 1024.0
    if step == INF_STEP and rank == min(INF_RANK, world - 1):
        tab[17] = float("inf")                                        # one rank's fp16 table overflow
    if step == INF_STEP2 and rank == 0:
        tab[N_EMB - 1] = float("inf")
    return tab.half(), rest


def run(rank, world, port, out_dir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    from bundlesdf_amd import exchange as EX
    P0 = torch.randn(N_EMB + N_MLP + N_FEAT + N_POSE, generator=torch.Generator().manual_seed(5)) * 0.1
    res = {}
    for kind in ("replicated", "sharded", "overlap"):
        fs = make_fs(P0)
        ops = TorchOps(fs)
        if kind in ("sharded", "overlap"):
            ex = EX.ShardedExchange(fs, ops, world, rank)
            ex.mirror_pad[:N_EMB].copy_(fs.emb16)
            fs.emb16 = ex.mirror_pad[:N_EMB]
            p = ex.plan
            ex.mirror_shard[:p.cnt].copy_(fs.emb16[p.lo:p.hi])
        else:
            ex = EX.ReplicatedExchange(fs, ops, world)
        for step in range(STEPS):
            if kind == "overlap":
                # FusedStep's overlapped schedule: the previous step's mirror all-gather is still in
                # flight while the next step's prologue / trace run; it is waited for right before the
                # field pass reads the mirror
                ex.wait_mirror()
                res[f"{kind}/{step}/seen"] = fs.emb16.float().clone().numpy()
            tab16, rest = local_grads(rank, step, world)
            fs.G16.copy_(tab16)
            fs.G[fs.mlp_off:] = rest
            ex.step(overlap=kind == "overlap")
            fs.global_step += 1
            if kind == "overlap":
                ex.wait_mirror()   # the host reads below (the test's view), not the schedule's
            if kind in ("sharded", "overlap"):
                P = torch.cat([ex.gather(fs.P), fs.P[N_EMB:]])
                M = torch.cat([ex.gather(fs.M), fs.M[N_EMB:]])
                V = torch.cat([ex.gather(fs.V), fs.V[N_EMB:]])
            else:
                P, M, V = fs.P, fs.M, fs.V
            for k, t in (("P", P), ("M", M), ("V", V), ("mirror", fs.emb16.float()), ("scale", fs.scale),
                         ("adam_t", fs.adam_t), ("tracker", fs.tracker)):
                res[f"{kind}/{step}/{k}"] = t.clone().numpy()
    np.savez(os.path.join(out_dir, f"rank{rank}.npz"), **res)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
