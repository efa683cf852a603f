"""Data-parallel gradient exchange + optimiser step of one training iteration
(SURVEY §8e): the host-side protocol that FusedStep runs between its captured
device segments, written once against an `ops` interface so the same code
drives the HIP kernels (FusedStep) and, in the CPU tests, torch restatements
of them (tests/test_exchange_gloo.py).

The reference trains on one GPU (no exchange, nerf_runner.py:755-762); its
step is GradScaler.unscale_ + inf check, Adam(eps 1e-15) over the dense
parameters, GradScaler.update. Two exchanges build the same step over W ranks
whose equal-sized, frame-sharded batches make the global gradient the mean of
the local ones:

  replicated  one all-reduce (sum, x 1/W) of the flat fp32 bucket
              [table | mlp | features | pose]; every rank runs the whole Adam.
  sharded     (amp) the fp16 table gradient is reduce-scattered AS fp16 (the
              reference accumulates it in fp16 __half2 atomics itself,
              gridencoder.cu:319-327) -> each rank's 1/W shard, issued together
              with the all-reduce of the small rest bucket [mlp | features |
              pose | inf flag]; Adam on the rank's table shard + the replicated
              rest; all-gather of the fp16 table mirror the amp forward reads.
              Moves (W-1)/W x (2 + 2) B per table parameter instead of the
              all-reduce's 2 (W-1)/W x 4 B (half), in two collective phases, and
              runs 1/W of the table's Adam per rank. The fp32 master table is
              then sharded: FusedStep.master_params() assembles it.

Overflow-free fp16 sum: before the reduce-scatter every rank scales its fp16
table gradient by 1/W2 (W2 = the power of two >= W, exact in fp16 outside the
subnormals), so the sum of W such values is at most 65504 in magnitude and the
reduction cannot overflow (fp16 round-to-nearest never exceeds a representable
bound of the exact sum); after widening the shard to fp32 it is multiplied by
W2/W (1 for W a power of two). So the table's non-finite verdict is decided on
each rank's LOCAL fp16 gradient before the exchange and rides in the rest
bucket's flag slot (summed): every replica skips together, with no extra
collective and no check of the summed shard needed.

found_inf contract (the optimiser kernels, optim.hip): k_unscale_check ORs into
found_inf (it never clears it), k_adam reads it to skip, and k_scaler_update —
the only writer that clears it — also advances Adam's step count. So post()
merges the ranks' verdict into found_inf, runs every unscale_check, then BOTH
Adam calls, and only then scaler_update; a kernel that reset found_inf, or a
scaler update between the two Adam calls, would let one rank step while another
skips (the replicas would diverge silently).

Failure diagnosis (the first multi-GPU contact is the driver's 8-GPU run): every
collective is issued through `collective(phase, fn)`, which records the rank / step /
phase it is in (logged on stderr for the first steps and every 100th), and turns any
error raised by the collective — a gloo timeout, an RCCL error surfaced by the async
error handling, a peer that left — into a CollectiveError naming that rank, step and
phase. The process group's timeout (COLLECTIVE_TIMEOUT_S, bench.py) bounds every wait;
bench.py ends the rank with a non-zero status on a CollectiveError (no retry)."""
import os
import sys
import time

import torch
import torch.distributed as dist

# seconds any collective may wait for its peers (init_process_group(timeout=...) in bench.py)
COLLECTIVE_TIMEOUT_S = float(os.environ.get("NOF_COLLECTIVE_TIMEOUT_S", "120"))


class CollectiveError(RuntimeError):
    """A collective failed or timed out; the message names the rank, step and phase."""


class _Where:
    rank, step, phase, t = None, -1, "init", 0.0


_WHERE = _Where()


def where():
    """'rank r step s phase p' of the last collective this process entered."""
    r = _WHERE.rank
    if r is None:
        r = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
    return f"rank {r} step {_WHERE.step} phase {_WHERE.phase}"


def collective(phase, fn, step=-1):
    """Run the collective call fn() (issue, or issue + wait) as `phase` of training step `step`:
    record where this rank is, log the first steps' and every 100th step's phases, and convert
    any failure into a CollectiveError that says where."""
    _WHERE.step, _WHERE.phase, _WHERE.t = step, phase, time.time()
    if os.environ.get("NOF_COLLECTIVE_LOG", "1") != "0" and (0 <= step < 2 or step % 100 == 0):
        print(f"[exchange] {where()}", file=sys.stderr, flush=True)
    try:
        return fn()
    except Exception as e:           # gloo / RCCL errors are RuntimeError subclasses (DistBackendError, ...)
        raise CollectiveError(f"{where()}: {type(e).__name__}: {e}") from e


def allreduce_mean(G, world_size, group=None, step=-1):
    """The replicated exchange's collective: ONE all-reduce (sum) of the flat fp32 bucket
    G = [table | mlp | features | pose] over RCCL (xGMI) on GPU (gloo in the CPU tests), then
    x 1/W: equal local batches make the mean of the local gradients the global one. The
    scaled gradient is summed, so one rank's inf / NaN reaches every rank and all replicas
    skip the step together; pose / feature rows are non-zero only on their owning rank."""
    collective("all_reduce", lambda: dist.all_reduce(G, group=group), step)
    G.mul_(1.0 / world_size)


def pow2_at_least(w):
    p = 1
    while p < w:
        p *= 2
    return p


class ShardPlan:
    """Table shard of rank `rank` of `world`: [lo, hi) of n entries; every shard is
    `sh` entries (a multiple of `align`, so shard pointers stay 16-B aligned for the
    vectorised kernels), the padded table n_pad = W sh."""

    def __init__(self, n, world, rank, align=64):
        per = -(-n // world)
        self.sh = -(-per // align) * align
        self.n_pad = self.sh * world
        self.lo = min(n, rank * self.sh)
        self.hi = min(n, self.lo + self.sh)
        self.cnt = self.hi - self.lo
        self.n, self.world, self.rank = n, world, rank


class ShardedExchange:
    """Buffers and collectives of the sharded exchange. `fs` holds the flat fp32
    buffers P / M / V (length N), the gradient buffer Gbuf (length N + 1: the last
    element is the inf-flag slot), G16 (fp16 table gradient, replaced here by a view of
    a zero-padded n_pad buffer: the reduce-scatter's input) and the offsets n_emb /
    mlp_off / feat_off / pose_off; `ops` provides the device operations (widen,
    unscale_check, adam, scaler_update)."""

    def __init__(self, fs, ops, world, rank, group=None):
        self.fs, self.ops, self.world, self.group = fs, ops, world, group
        dev = fs.P.device
        self.plan = p = ShardPlan(fs.n_emb, world, rank)
        self.w2 = pow2_at_least(world)
        self.G16pad = torch.zeros(p.n_pad, dtype=torch.float16, device=dev)
        self.G16pad[:fs.n_emb].copy_(fs.G16)
        fs.G16 = self.G16pad[:fs.n_emb]        # the field pass accumulates into the padded buffer
        self.Gs16 = torch.zeros(p.sh, dtype=torch.float16, device=dev)    # this rank's summed shard (fp16)
        self.Gs = torch.zeros(p.sh, dtype=torch.float32, device=dev)      # ... widened, mean, unscaled
        self.mirror_pad = torch.zeros(p.n_pad, dtype=torch.float16, device=dev)
        self.mirror_shard = torch.zeros(p.sh, dtype=torch.float16, device=dev)
        # Adam's touched-group flags of the shard (ops.active_flags; None: every group updated)
        self.active_shard = ops.active_flags(p.sh, dev) if hasattr(ops, "active_flags") else None

    # ---- end of device segment 1 (after the field pass): the local table verdict into the
    # flag slot, the fp16 table gradient pre-scaled by 1/W2 (the sum cannot overflow)
    def prep(self):
        fs = self.fs
        self.ops.check16(fs.G16, fs.n_emb)
        fs.Gbuf[-1:].copy_(fs.found_inf.to(torch.float32))
        if self.w2 > 1:
            self.G16pad.mul_(1.0 / self.w2)

    # ---- collective phase 1: fp16 table reduce-scatter + rest-bucket all-reduce, issued together
    def reduce(self):
        fs = self.fs
        step = getattr(fs, "global_step", -1)

        def run():
            w1 = dist.reduce_scatter_tensor(self.Gs16, self.G16pad, group=self.group, async_op=True)
            w2 = dist.all_reduce(fs.Gbuf[fs.mlp_off:], group=self.group, async_op=True)
            w1.wait()
            w2.wait()
        collective("reduce_scatter+all_reduce", run, step)

    # ---- device segment 2: the optimiser on the shard and the rest (found_inf contract above)
    def post(self, sp=None, debug=False):
        fs, p = self.fs, self.plan
        N = fs.P.numel()
        self.G16pad.zero_()                              # the next step's accumulator
        self.ops.grad16_to_f32(self.Gs16, self.Gs, p.sh)
        if self.w2 != self.world:
            self.Gs.mul_(self.w2 / self.world)
        # a non-finite local table gradient on any rank: every rank skips
        fs.found_inf.copy_(torch.maximum(fs.found_inf, (fs.Gbuf[-1:] > 0).to(torch.int32)))
        self.ops.unscale_check(self.Gs, p.cnt, f16_lo=0, f16_hi=0)
        rest = fs.Gbuf[fs.mlp_off:N]
        rest.mul_(1.0 / self.world)
        # the NeRFSmall gradients are fp16 under autocast in the reference: beyond its range = overflow
        self.ops.unscale_check(rest, N - fs.mlp_off, f16_lo=0, f16_hi=fs.feat_off - fs.mlp_off)
        grads = None
        if debug:
            full = torch.empty(p.n_pad, dtype=torch.float32, device=fs.P.device)
            collective("debug_all_gather", lambda: dist.all_gather_into_tensor(full, self.Gs, group=self.group),
                       getattr(fs, "global_step", -1))
            grads = torch.cat([full[:fs.n_emb], rest.clone()])
        self.ops.adam(fs.P[p.lo:p.hi], self.Gs[:p.cnt], fs.M[p.lo:p.hi], fs.V[p.lo:p.hi], p.cnt, p.cnt,
                      self.mirror_shard[:p.cnt], sp, active=self.active_shard)
        self.ops.adam(fs.P[fs.mlp_off:], rest, fs.M[fs.mlp_off:], fs.V[fs.mlp_off:], N - fs.mlp_off,
                      fs.pose_off - fs.mlp_off, None, sp)
        self.ops.scaler_update()                         # clears found_inf, advances adam_t: after both Adams
        return grads

    # ---- collective phase 2: the fp16 table mirror the amp forward reads. Overlapped (async_op):
    # issued at the end of the step and waited for just before the next step's field pass — the
    # next step's prologue (pose forward, MLP packing), batch draw and ray trace do not read the
    # table, so on RCCL the gather runs on its own stream beside them (wait() only orders the
    # compute stream behind it; the host does not block). Every reader or writer of the mirror
    # outside the field pass calls wait_mirror() first (FusedStep.wait_exchange).
    def all_gather_mirror(self, async_op=False):
        self.wait_mirror()
        w = collective("all_gather_mirror", lambda: dist.all_gather_into_tensor(
            self.mirror_pad, self.mirror_shard, group=self.group, async_op=async_op), getattr(self.fs, "global_step", -1))
        self._pending = w if async_op else None

    def all_gather_mirror_async(self):
        self.all_gather_mirror(async_op=True)

    def wait_mirror(self):
        w = getattr(self, "_pending", None)
        if w is not None:
            self._pending = None
            collective("wait_mirror", w.wait, getattr(self.fs, "global_step", -1))

    def gather(self, t):
        """Full [0, n_emb) of a sharded fp32 table buffer (P / M / V) from every rank's shard."""
        p = self.plan
        sh = torch.zeros(p.sh, dtype=t.dtype, device=t.device)
        sh[:p.cnt].copy_(t[p.lo:p.hi])
        full = torch.empty(p.n_pad, dtype=t.dtype, device=t.device)
        collective("gather_shards", lambda: dist.all_gather_into_tensor(full, sh, group=self.group))
        return full[:p.n]

    def step(self, sp=None, debug=False, overlap=False):
        """The eager sequence (FusedStep.step); graph replay runs the same device
        segments from captured graphs with the two collective phases between them.
        overlap: the mirror all-gather is left in flight (wait_mirror() before the mirror
        is read)."""
        self.prep()
        self.reduce()
        grads = self.post(sp, debug)
        self.all_gather_mirror(async_op=overlap)
        return grads


class ReplicatedExchange:
    """One all-reduce of the flat fp32 bucket; the whole optimiser on every rank."""

    def __init__(self, fs, ops, world, group=None):
        self.fs, self.ops, self.world, self.group = fs, ops, world, group

    def wait_mirror(self):
        """Nothing in flight between steps (Adam writes the mirror itself)."""

    def prep(self):
        fs = self.fs
        if fs.amp:   # the fp16 table gradient joins the fp32 bucket: nothing is summed in fp16
            self.ops.grad16_to_f32(fs.G16, fs.G, fs.n_emb)

    def all_reduce(self):
        allreduce_mean(self.fs.G, self.world, self.group, getattr(self.fs, "global_step", -1))

    def post(self, sp=None, debug=False):
        fs = self.fs
        N = fs.P.numel()
        if fs.amp:
            self.ops.unscale_check(fs.G, N, f16_lo=fs.mlp_off, f16_hi=fs.feat_off)
        grads = fs.G.clone() if debug else None
        self.ops.adam(fs.P, fs.G, fs.M, fs.V, N, fs.pose_off, fs.emb16 if fs.amp else None, sp,
                      active=getattr(fs, "adam_active", None))
        self.ops.scaler_update()
        return grads

    def step(self, sp=None, debug=False, overlap=False):
        self.prep()
        self.all_reduce()
        return self.post(sp, debug)
