"""FusedStep — one NeRF training iteration on MI355X (the body of
NerfRunner.train_loop, nerf_runner.py:677-762) as a short, sync-free sequence
of libnof kernels on the current HIP stream:

  1+3. nof_step_prologue  pose corrections -> per-frame world_from_cam tf [F,16] + d tf / d pose,
                         MLP params -> MFMA operand fragments (and, graph replay, the step schedule)
                         in one launch (= nof_pose_forward + nof_pack_mlp [+ nof_step_schedule])
  2. nof_trace_rays      gather batch, ray setup, DDA trace, clip, lengths
  4. nof_field_step      sample/encode/MLP/composite/loss + full backward
  5. nof_pose_backward   per-ray dL/dtf -> per frame -> pose gradient (Jacobian from step 1)
  6. GradScaler unscale + inf check, Adam (+ fp16 table mirror), scaler update

Parameters live in ONE flat fp32 buffer [embeddings | NeRFSmall | PoseArray];
the nn.Parameters of the modules are views of it, so state_dict keys and
shapes are the reference's (grid.py / nerf_helpers.py).
"""
import ctypes
import math

import numpy as np
import torch

from . import _lib
from . import exchange as EX
from . import mlp_layout as ML

_F32, _F16 = 0, 1
MAX_LEVEL_RES = 1023      # k_scatter's run keys: 10 bits per cell coordinate (field_step.hip)
QUADS_MIN_RAYS = 32768    # nof_field_step's default quads_min_rays (the xy-quad mirror encode from this batch)


def lr_at(cfg, global_step, base):
    """schedule_lr (nerf_runner.py:577-581), applied every 10 steps after the step (:761-762)."""
    n_iters = cfg["n_step"] + 1
    if global_step <= 10:
        return base
    last = 10 * ((global_step - 1) // 10)
    return base * (cfg["decay_rate"] ** (float(last) / n_iters))


def truncation(cfg, global_step):
    """get_truncation (nerf_runner.py:661-674): the truncation band, annealed from
    trunc_start to trunc over the round when trunc_decay_type is 'linear' / 'exp',
    times sc_factor. Host double arithmetic as the reference; the kernels take it
    as float32."""
    kind = cfg.get("trunc_decay_type", "") or ""
    if kind == "linear":
        t = cfg["trunc_start"] - (cfg["trunc_start"] - cfg["trunc"]) * float(global_step) / cfg["n_step"]
    elif kind == "exp":
        lamb = np.log(cfg["trunc"] / cfg["trunc_start"]) / (cfg["n_step"] / 4)
        t = max(cfg["trunc_start"] * np.exp(global_step * lamb), cfg["trunc"])
    elif kind == "":
        t = cfg["trunc"]
    else:
        raise NotImplementedError(f"trunc_decay_type {kind!r} (the reference knows '', 'linear', 'exp')")
    return float(t) * cfg["sc_factor"]


# the replicated exchange's collective (exchange.py), kept under its r1 name for callers
allreduce_gradients = EX.allreduce_mean


class _HipOps:
    """exchange.py's device operations on the libnof kernels, on the current HIP stream of
    the trainer's buffers (graph-capture safe)."""

    def __init__(self, fs):
        self.fs = fs

    def grad16_to_f32(self, src16, dst32, n):
        _lib.check(_lib.lib().nof_grad16_to_f32(_lib.ptr(src16), _lib.ptr(dst32), n, _lib.stream_of(dst32)),
                   "grad16_to_f32")

    def unscale_check(self, g, n, f16_lo=0, f16_hi=0):
        fs = self.fs
        _lib.check(_lib.lib().nof_unscale_check(_lib.ptr(g), n, _lib.ptr(fs.scale), _lib.ptr(fs.found_inf), None, 0,
                                                f16_lo, f16_hi, _lib.stream_of(g)), "unscale")

    def check16(self, g16, n):
        """Non-finite check of an fp16 gradient (ORed into found_inf), no unscale."""
        fs = self.fs
        _lib.check(_lib.lib().nof_unscale_check(None, 0, _lib.ptr(fs.scale), _lib.ptr(fs.found_inf), _lib.ptr(g16), n,
                                                0, 0, _lib.stream_of(g16)), "check16")

    def adam(self, p, g, m, v, n, group1_start, mirror, sp, g16=None, active=None):
        """Adam over n entries of p (group 'basic' before group1_start, 'pose_array' after),
        refreshing the fp16 mirror of its first mirror.numel() entries; g16: the fp16 table
        gradient (scaled) for those entries instead of g; active: the touched-group flags of
        this p (adam_active_flags(n), zeroed with m / v) — untouched groups are skipped."""
        fs = self.fs
        lr0 = lr_at(fs.cfg, fs.global_step, fs.cfg["lrate"])
        lr1 = lr_at(fs.cfg, fs.global_step, fs.cfg["lrate_pose"])
        mn = 0 if mirror is None else int(mirror.numel())
        _lib.check(_lib.lib().nof_adam_step(_lib.ptr(p), _lib.ptr(g), _lib.ptr(m), _lib.ptr(v), n, group1_start, lr0, lr1,
                                            0.9, 0.999, 1e-15, _lib.ptr(fs.adam_t), _lib.ptr(fs.found_inf),
                                            _lib.ptr(mirror), mn, _lib.ptr(g16), _lib.ptr(fs.scale),
                                            _lib.ctypes.c_void_p(sp), _lib.ptr(active), _lib.stream_of(p)), "adam")

    @staticmethod
    def active_flags(n, dev):
        return torch.zeros(int(_lib.lib().nof_adam_active_bytes(n)), dtype=torch.uint8, device=dev)

    def scaler_update(self):
        fs = self.fs
        _lib.check(_lib.lib().nof_scaler_update(_lib.ptr(fs.scale), _lib.ptr(fs.tracker), _lib.ptr(fs.found_inf),
                                                _lib.ptr(fs.adam_t), 2.0, 0.5, fs.growth_interval,
                                                1 if fs.amp else 0, _lib.stream_of(fs.scale)), "scaler")


class FusedStep:
    def __init__(self, cfg, pool, c2w, occ, grid, mlp, pose_array, amp=None, frame_start=None, blocks_per_cu=0,
                 process_group=None, world_size=1, time_kernels=False, feature_array=None, exchange=None):
        dev = pool.device
        if dev.type != "cuda":
            raise RuntimeError("FusedStep needs a HIP device (no CPU fallback)")
        _lib.lib()
        self.cfg, self.dev = cfg, dev
        self.amp = bool(cfg["amp"] if amp is None else amp)
        self.pool = pool.contiguous().float()
        self.c2w = c2w.to(dev).float().contiguous()
        self.F = self.c2w.shape[0]
        self.occ = occ.to(dev).to(torch.uint8).contiguous()
        self.Nocc = int(self.occ.shape[0])
        self.Kmax = 3 * self.Nocc
        self.grid, self.mlp, self.pose_array = grid, mlp, pose_array
        self.L, self.C = grid.n_levels, grid.level_dim
        self.n_in = self.L * self.C
        assert self.C == 2 and self.n_in <= 32, "fused path: C=2, L<=16"
        self.blocks_per_cu = blocks_per_cu
        self.frame_start = None
        if frame_start is not None:
            fst = np.asarray(frame_start, np.int64).ravel()
            # k_sample_batch maps a frame's draws into [start, start + count): an empty frame
            # would hand out the next frame's first ray (or one past the pool)
            if fst.size < 2 or fst[0] != 0 or (np.diff(fst) <= 0).any() or fst[-1] > self.pool.shape[0]:
                raise ValueError("frame_start must be an increasing prefix [0, ..., <= N_pool] with no empty frame")
            self.frame_start = torch.as_tensor(fst, dtype=torch.int64, device=dev)
        # ---- flat parameter buffer, module params become views
        emb = grid.embeddings.data.reshape(-1)
        sd = dict(mlp.named_parameters())
        mlp_flat = torch.cat([sd[k].data.reshape(-1).float() for k in ML.MLP_KEYS])
        # cfg frame_features: FeatureArray [F, n_ff] fed to the colour net (nerf_runner.py:221,234-235,1268-1277)
        self.feature_array = feature_array
        self.n_ff = 0 if feature_array is None else int(feature_array.data.shape[1])
        if not 0 <= self.n_ff <= 3:
            raise ValueError(f"fused path: frame_features must be <= 3 (got {self.n_ff})")
        assert mlp_flat.numel() == ML.offsets(self.n_in, self.n_ff)[1]
        pose = pose_array.data.data.reshape(-1)
        feat = (torch.zeros(0) if feature_array is None else feature_array.data.data.reshape(-1).float())
        if feature_array is not None and feature_array.data.shape[0] != self.F:
            raise ValueError("feature_array rows must match the number of frames")
        self.n_emb, self.n_mlp, self.n_pose = emb.numel(), mlp_flat.numel(), pose.numel()
        self.n_feat = feat.numel()
        # flat [table | mlp | frame features | pose]: Adam's 'basic' group (lrate) is everything before pose_off
        self.P = torch.cat([emb.to(dev), mlp_flat.to(dev), feat.to(dev), pose.to(dev)]).contiguous()
        self.mlp_off = self.n_emb
        self.feat_off = self.n_emb + self.n_mlp
        self.pose_off = self.feat_off + self.n_feat
        grid.embeddings.data = self.P[:self.n_emb].view(-1, self.C)
        o = self.mlp_off
        for k in ML.MLP_KEYS:
            n = sd[k].numel()
            sd[k].data = self.P[o:o + n].view(sd[k].shape)
            o += n
        pose_array.data.data = self.P[self.pose_off:].view(self.F, 6)
        if feature_array is not None:
            feature_array.data.data = self.P[self.feat_off:self.pose_off].view(self.F, self.n_ff)
        # gradient bucket: N entries + one slot (the sharded exchange's inf flag, exchange.py)
        self.Gbuf = torch.zeros(self.P.numel() + 1, dtype=torch.float32, device=dev)
        self.G = self.Gbuf[:self.P.numel()]
        self.M = torch.zeros_like(self.P)
        self.V = torch.zeros_like(self.P)
        # k_adam's touched-group flags for the whole-buffer update (N = 1 / replicated exchange)
        self.adam_active = _HipOps.active_flags(self.P.numel(), dev)
        # emb16: the fp16 table mirror the amp kernels read. Under the sharded exchange (N > 1) it is the
        # target of the mirror all-gather that runs on into the next step: code outside this class must
        # call wait_exchange() before reading or writing it (the library's own readers do)
        self.emb16 = torch.empty(self.n_emb, dtype=torch.float16, device=dev) if self.amp else None
        # amp: the table gradient is accumulated in fp16 (packed fp16x2 atomics), as the reference's
        # grid_encode_backward does for half embeddings (gridencoder.cu:319-327)
        self.G16 = torch.zeros(self.n_emb, dtype=torch.float16, device=dev) if self.amp else None
        # amp: k_encode's xy-quad mirror of emb16 (16 B per table row, rebuilt inside every large field pass)
        self.quads = torch.empty(self.n_emb * 2, dtype=torch.int32, device=dev) if self.amp else None
        # its rebuild runs on this side stream, overlapping the prologue and trace (_fork_quad_mirror)
        self._side = torch.cuda.Stream(dev) if self.amp else None
        self.quad_fork = __import__("os").environ.get("NOF_QUAD_FORK", "1") != "0"   # 0: rebuilt in the step
        if self.amp:
            _lib.check(_lib.lib().nof_to_half(_lib.ptr(self.P), _lib.ptr(self.emb16), self.n_emb,
                                              _lib.stream_of(self.P)), "to_half")
        # ---- MLP fragment image
        idx, _, nfr = ML.pack_table(self.n_in, self.n_ff)
        self.pack_idx = torch.from_numpy(idx).to(dev)
        self.n_frag_elems = nfr * 64 * 8
        self.frags = torch.empty(self.n_frag_elems, dtype=torch.float16 if self.amp else torch.float32, device=dev)
        self.bias = torch.empty(5 * 64, dtype=torch.float32, device=dev)
        # ---- level table
        offs = grid.offsets.cpu().numpy().astype(np.int32)
        lt = np.zeros((self.L, 4), np.float32)
        S_log = float(np.log2(grid.per_level_scale))
        _lib.lib().nof_level_table(self.L, np.float32(S_log), int(grid.base_resolution),
                                   offs.ctypes.data_as(_lib.ctypes.c_void_p), lt.ctypes.data_as(_lib.ctypes.c_void_p))
        # k_scatter's run keys pack a sample's cell coordinates into 10 bits each (field_step.hip, the
        # run-key comment): a level whose resolution exceeds 1023 would alias neighbouring cells' keys
        # and merge their runs (the reference's configs stop at 512)
        res = lt.view(np.int32)[:, 1]
        if int(res.max()) > MAX_LEVEL_RES:
            raise ValueError(f"fused path: level resolution {int(res.max())} > {MAX_LEVEL_RES} "
                             "(k_scatter's 10-bit cell keys)")
        self.levels = torch.from_numpy(lt).to(dev)
        # ---- GradScaler / Adam device state
        self.scale = torch.tensor([65536.0 if self.amp else 1.0], dtype=torch.float32, device=dev)
        self.tracker = torch.zeros(1, dtype=torch.int32, device=dev)
        self.found_inf = torch.zeros(1, dtype=torch.int32, device=dev)
        self.adam_t = torch.zeros(1, dtype=torch.int32, device=dev)
        # rgb, fs, empty, sdf, n_valid, n_bwd, scatter HBM atomics (table flush, probe overflow)
        self.loss_acc = torch.zeros(8 + 128 + 8, dtype=torch.float32, device=dev)
        # graph_step_epoch: the global step that took the current epoch's first slice (device int)
        self.epoch_step0 = torch.zeros(1, dtype=torch.int32, device=dev)
        self.process_group, self.world_size = process_group, world_size
        self.time_kernels = time_kernels
        self._c_timing = False
        self.kernel_ms = []
        self.tf_buf = torch.empty(self.F, 16, dtype=torch.float32, device=dev)
        self.pose_jac = torch.empty(self.F, 12, 6, dtype=torch.float32, device=dev)
        self.pose_fg = torch.zeros(self.F, 12, dtype=torch.float32, device=dev)   # nof_pose_backward leaves it zero
        self.global_step = 0
        self.growth_interval = 2000        # GradScaler(growth_interval) of the reference (nerf_runner.py:159)
        # XCD-contiguous block order for k_encode (bit 0; measured faster on sorted batches) and
        # k_scatter (bit 1; measured slower): NOF_XCD_ORDER overrides for experiments
        self.xcd_order = int(__import__("os").environ.get("NOF_XCD_ORDER", "1"))
        self._R = None
        # graph replay (graph_step): device step counter + the step block nof_step_schedule writes
        self.step_dev = torch.zeros(1, dtype=torch.int32, device=dev)
        self._step_dev_at = 0         # the value step_dev holds (host view), or None when unknown
        self.step_params = torch.zeros(ctypes.sizeof(_lib.StepParams), dtype=torch.uint8, device=dev)
        self._graphs = None
        self._inflight = []
        self._capturing = False
        # cfg optimize_poses = 0 (NerfRunner freezes the pose array): no pose gradient at all —
        # the reference's grid backward skips dy_dx then (its inputs need no grad)
        self.pose_grad = bool(cfg.get("optimize_poses", 1))
        # ---- data-parallel exchange (exchange.py): amp shards the table's optimiser state
        # (reduce-scatter + Adam on the shard + all-gather of the fp16 mirror), fp32 all-reduces
        self.ex = None
        self.exchange = "local"
        if world_size > 1:
            if exchange not in (None, "sharded", "allreduce"):
                raise ValueError(f"exchange {exchange!r}: 'sharded' (amp default) or 'allreduce'")
            ops = _HipOps(self)
            if exchange == "sharded" and not self.amp:
                raise ValueError("exchange='sharded' needs amp (it shards the fp16 table mirror); "
                                 "use exchange='allreduce' or None for fp32")
            if self.amp and exchange in (None, "sharded"):
                self.exchange = "sharded"
                rank = torch.distributed.get_rank(process_group)
                self.ex = EX.ShardedExchange(self, ops, world_size, rank, process_group)
                self.ex.mirror_pad[:self.n_emb].copy_(self.emb16)
                self.emb16 = self.ex.mirror_pad[:self.n_emb]    # the all-gather lands where the kernels read
                self._shard_mirror()
            else:
                self.exchange = "allreduce"
                self.ex = EX.ReplicatedExchange(self, ops, world_size, process_group)

    def _shard_mirror(self):
        if self.exchange == "sharded":
            p = self.ex.plan
            self.ex.mirror_shard[:p.cnt].copy_(self.emb16[p.lo:p.hi])

    def master_params(self):
        """The flat fp32 parameters [table | mlp | features | pose] with the table assembled
        from every rank's shard when the optimiser state is sharded (a collective: every rank
        calls it); the buffer itself otherwise."""
        if self.exchange != "sharded":
            return self.P
        return torch.cat([self.ex.gather(self.P), self.P[self.n_emb:]])

    def optimizer_state(self):
        """(M, V) Adam moments, assembled like master_params()."""
        if self.exchange != "sharded":
            return self.M, self.V
        return (torch.cat([self.ex.gather(self.M), self.M[self.n_emb:]]),
                torch.cat([self.ex.gather(self.V), self.V[self.n_emb:]]))

    def sync_master_params(self):
        """Write the assembled master table back into P on every rank (before a checkpoint
        or any host read of the full table under the sharded exchange)."""
        if self.exchange == "sharded":
            with torch.no_grad():
                self.P[:self.n_emb].copy_(self.ex.gather(self.P))

    def reset_state(self, P=None):
        """Start a new training round on the same buffers: parameters from P (flat, e.g. a
        copy of the initial self.P), gradients / Adam moments zero, GradScaler at its
        initial scale, step counters 0 — what bundlesdf.py's add_new_frames(reuse_weights=
        False) does through create_nerf + create_optimizer (nerf_runner.py:379-380,396-399).
        Captured graphs stay valid (same addresses). Stream-ordered: no host sync."""
        self.wait_exchange()
        with torch.no_grad():
            if P is not None:
                self.P.copy_(P)
            self.Gbuf.zero_()
            self.M.zero_()
            self.V.zero_()
            self.adam_active.zero_()
            if self.amp:
                self.G16.zero_()
                self.refresh_half_table()
            if self.exchange == "sharded":
                self.ex.Gs.zero_()
                self.ex.Gs16.zero_()
                self.ex.active_shard.zero_()
            self.scale.fill_(65536.0 if self.amp else 1.0)
            self.tracker.zero_()
            self.found_inf.zero_()
            self.adam_t.zero_()
            self.step_dev.zero_()
        self.global_step = 0
        self._step_dev_at = 0

    # ------------------------------------------------------------------
    def _alloc(self, R):
        if self._R == R:
            return
        d = self.dev
        self.rays = torch.empty(R, 12, device=d)
        self.intervals = torch.empty(R, self.Kmax, 2, device=d)
        self.totals = torch.empty(R, device=d)
        self.counts = torch.empty(R, dtype=torch.int32, device=d)
        self.ray_grad = torch.empty(R, 12, device=d)
        self.ids = torch.empty(R, dtype=torch.int32, device=d)
        S = self.cfg["N_samples"] + self.cfg["N_samples_around_depth"]
        nbytes = _lib.lib().nof_field_workspace_bytes(R, S, _F16 if self.amp else _F32)
        self.workspace = torch.empty(nbytes, dtype=torch.uint8, device=d)
        self._R = R
        self._graphs = None   # captured graphs hold the old buffers' addresses

    def sample_ids(self, rays_per_frame, seed):
        """Throughput mode: rays_per_frame uniform rays from every frame of the (local) pool."""
        nf = int(self.frame_start.numel()) - 1
        R = nf * rays_per_frame
        self._alloc(R)
        _lib.check(_lib.lib().nof_sample_batch(_lib.ptr(self.frame_start), nf, rays_per_frame, seed & 0xFFFFFFFF,
                                               _lib.ptr(self.ids), None, _lib.stream_of(self.ids)), "sample_batch")
        return self.ids

    def step(self, ids=None, t_rand=None, debug=False, seed=None, perturb=True, grad_hook=None):
        """One training iteration on the batch pool[ids]. t_rand [R,S] injects the
        stratification draws (parity tests); debug returns z / raw / valid / rgb and the
        unscaled gradients. grad_hook(self), when given, runs after the backward and
        before the exchange / optimiser (tests inject non-finite gradients there)."""
        if ids is None:
            raise ValueError("step(ids=...) or sample_ids() first")
        ids = ids.to(self.dev).to(torch.int32).contiguous()
        R = ids.numel()
        self._alloc(R)
        if ids.data_ptr() != self.ids.data_ptr():
            self.ids.copy_(ids)
        dbg = self._field_part(R, None, t_rand, debug, seed, perturb)
        if grad_hook is not None:
            grad_hook(self)
        grads = self._exchange_and_optimize(debug)
        self.global_step += 1
        out = {"loss_terms": self.loss_acc[:8], "fs_rgb_loss": self.loss_acc[140]}
        if debug:
            out.update(dbg=dbg, grads=grads)
        return out

    def _prologue(self, sched=None):
        """Steps 1 and 3 in one launch (nof_step_prologue): pose corrections (PoseArray.get_matrices,
        nerf_helpers.py:143-154) and tf = T @ c2w (:1050-1052) with d tf / d pose for step 5, the MLP
        fragment packing, and — graph replay, sched given — the device step schedule first."""
        L = _lib.lib()
        sd = None if sched is None else _lib.ctypes.byref(sched)
        _lib.check(L.nof_step_prologue(sd, _lib.ptr(self.step_dev) if sched is not None else None,
                                       _lib.ptr(self.step_params) if sched is not None else None,
                                       _lib.ctypes.c_void_p(self.P.data_ptr() + 4 * self.pose_off), _lib.ptr(self.c2w),
                                       self.F, float(self.pose_array.max_trans),
                                       float(self.pose_array.max_rot / 180.0 * math.pi), _lib.ptr(self.tf_buf),
                                       _lib.ptr(self.pose_jac),
                                       _lib.ctypes.c_void_p(self.P.data_ptr() + 4 * self.mlp_off),
                                       _lib.ptr(self.pack_idx), self.n_frag_elems, 5 * 64, _lib.ptr(self.frags),
                                       _lib.ptr(self.bias), _F16 if self.amp else _F32, _lib.stream_of(self.P)),
                   "step_prologue")

    def _trace(self, R, sp):
        """Step 2: gather the batch, ray setup, DDA trace, clip, lengths (nof_trace_rays; while an
        epoch graph is captured, nof_trace_rays_epoch on the step's slice of the permutation)."""
        cfg = self.cfg
        sc = cfg["sc_factor"]
        perm = getattr(self, "_trace_perm", None)
        if perm is not None and sp is not None:
            _lib.check(_lib.lib().nof_trace_rays_epoch(
                _lib.ptr(self.pool), _lib.ptr(perm), _lib.ptr(self.epoch_step0), R, _lib.ptr(self.tf_buf),
                _lib.ptr(self.occ), self.Nocc, self.Kmax, cfg["near"] * sc, cfg["far"] * sc,
                truncation(cfg, self.global_step), _lib.ptr(self.rays), _lib.ptr(self.intervals),
                _lib.ptr(self.totals), _lib.ptr(self.counts), _lib.ctypes.c_void_p(sp), _lib.stream_of(self.P)),
                "trace_rays_epoch")
            return
        _lib.check(_lib.lib().nof_trace_rays(_lib.ptr(self.pool), _lib.ptr(self.ids), R, _lib.ptr(self.tf_buf),
                                             _lib.ptr(self.occ), self.Nocc, self.Kmax, cfg["near"] * sc,
                                             cfg["far"] * sc, truncation(cfg, self.global_step), _lib.ptr(self.rays),
                                             _lib.ptr(self.intervals), _lib.ptr(self.totals), _lib.ptr(self.counts),
                                             _lib.ctypes.c_void_p(sp), _lib.stream_of(self.P)), "trace_rays")

    def wait_exchange(self):
        """Order the current stream behind the data-parallel exchange's collective still in flight
        (the sharded exchange leaves the fp16 mirror all-gather running into the next step, which
        waits for it right before its field pass): call before reading or writing the fp16 table
        mirror outside the step. No-op at N = 1."""
        if self.ex is not None:
            self.ex.wait_mirror()

    def _uses_quads(self):
        return self.quads is not None and getattr(self, "use_quads", True)

    def _fork_quad_mirror(self, R):
        """Launch the encode's xy-quad mirror rebuild (nof_quad_mirror) on the side stream, forked from
        the current one, so that it overlaps the prologue / batch draw / trace; returns the join (the
        current stream waits for it) to call before the field pass, or None when the step rebuilds the
        mirror itself: no quads, the per-kernel timing pass (its encode bucket includes the rebuild), or
        the sharded exchange (the mirror all-gather lands only right before the field pass)."""
        if (not self._uses_quads() or not self.quad_fork or self.time_kernels or R == 0
                or (self.ex is not None and self.exchange == "sharded")):
            return None
        # below the library's quad threshold (nof_field_step: quads_min_rays, default 32,768 rays) the
        # encode reads the pair table and nof_quad_mirror does nothing: no fork / join nodes at all
        if R < (int(getattr(self, "quads_min_rays", 0)) or QUADS_MIN_RAYS):
            return None
        D = _lib.FieldDesc()
        D.R, D.L, D.C, D.D = R, self.L, self.C, 3
        D.table, D.levels = self.emb16.data_ptr(), self.levels.data_ptr()
        D.table_dtype = D.mlp_dtype = _F16
        D.table_quads, D.table_rows = self.quads.data_ptr(), self.n_emb // 2
        D.quads_min_rays = int(getattr(self, "quads_min_rays", 0))
        D.ablate = getattr(self, "ablate", 0)
        main = torch.cuda.current_stream(self.dev)
        self._side.wait_stream(main)
        with torch.cuda.stream(self._side):
            _lib.check(_lib.lib().nof_quad_mirror(_lib.ctypes.byref(D), _lib.stream_of(self.P)), "quad_mirror")
        return lambda: main.wait_stream(self._side)

    def _field_part(self, R, sp, t_rand=None, debug=False, seed=None, perturb=True, prologue=True, trace=True,
                    join_quads=None):
        """Steps 1-5 of one iteration on the batch in self.ids[:R]: pose forward + MLP pack (the
        prologue, unless the caller launched it), trace (unless launched), the fused field pass, pose
        backward, regularisers. sp: device step block (graph replay) or None (host scalars of
        self.global_step). join_quads: the caller forked the quad mirror rebuild (_fork_quad_mirror)."""
        cfg = self.cfg
        L = _lib.lib()
        st = _lib.stream_of(self.P)
        sc = cfg["sc_factor"]
        trunc = truncation(cfg, self.global_step)
        S = cfg["N_samples"] + cfg["N_samples_around_depth"]
        # 1 + 3. pose corrections with their Jacobian, MLP fragments (one launch); the quad mirror
        # rebuild beside them
        if prologue:
            if join_quads is None:
                join_quads = self._fork_quad_mirror(R)
            self._prologue()
        # 2. trace
        if trace:
            self._trace(R, sp)
        # the previous step's mirror all-gather (sharded exchange) lands before the field pass reads it
        if not self._capturing:
            self.wait_exchange()
        if join_quads is not None:
            join_quads()
        # 4. field pass (nof_field_step zeroes loss_acc itself)
        if R == 0:
            self.loss_acc.zero_()
        dbg = None
        if debug:
            dbg = dict(z=torch.zeros(R, S, device=self.dev), raw=torch.zeros(R, S, 4, device=self.dev),
                       valid=torch.zeros(R, S, dtype=torch.uint8, device=self.dev),
                       rgb=torch.zeros(R, 3, device=self.dev))
        D = _lib.FieldDesc()
        D.rays, D.tf, D.intervals, D.totals = self.rays.data_ptr(), self.tf_buf.data_ptr(), \
            self.intervals.data_ptr(), self.totals.data_ptr()
        if t_rand is not None:
            t_rand = t_rand.to(self.dev).float().contiguous()
            self._t_rand = t_rand
            D.t_rand = t_rand.data_ptr()
        D.seed = (self.global_step * 0x9E3779B1 + (0 if seed is None else seed)) & 0xFFFFFFFF
        D.R, D.Kmax, D.N_oct, D.N_dep, D.S = R, self.Kmax, cfg["N_samples"], cfg["N_samples_around_depth"], S
        D.perturb = 1 if perturb else 0
        D.near_sc, D.far_sc, D.trunc = cfg["near"] * sc, cfg["far"] * sc, trunc
        D.neg_trunc_ratio, D.sdf_lambda, D.fs_sdf = cfg["neg_trunc_ratio"], cfg["sdf_lambda"], cfg["fs_sdf"]
        D.first_frame_weight, D.rgb_weight, D.fs_weight = cfg["first_frame_weight"], cfg["rgb_weight"], cfg["fs_weight"]
        D.empty_weight, D.trunc_weight = cfg["empty_weight"], cfg["trunc_weight"]
        D.fs_rgb_weight = float(cfg.get("fs_rgb_weight", 0) or 0)
        D.loss_scale = self.scale.data_ptr()
        D.table = (self.emb16 if self.amp else self.P).data_ptr()
        D.levels = self.levels.data_ptr()
        D.L, D.C, D.D = self.L, self.C, 3
        D.table_dtype = D.mlp_dtype = _F16 if self.amp else _F32
        D.frags, D.bias = self.frags.data_ptr(), self.bias.data_ptr()
        D.grad_table, D.grad_mlp = self.G.data_ptr(), self.G.data_ptr() + 4 * self.mlp_off
        D.grad_table16 = self.G16.data_ptr() if self.amp else None
        D.ray_grad, D.loss_acc = self.ray_grad.data_ptr(), self.loss_acc.data_ptr()
        if dbg is not None:
            D.dbg_z, D.dbg_raw, D.dbg_valid, D.dbg_rgb = (dbg["z"].data_ptr(), dbg["raw"].data_ptr(),
                                                          dbg["valid"].data_ptr(), dbg["rgb"].data_ptr())
        D.blocks_per_cu = self.blocks_per_cu
        D.ablate = getattr(self, "ablate", 0)
        D.workspace = self.workspace.data_ptr()
        D.scatter_slots = getattr(self, "scatter_slots", 0)
        D.xcd_order = int(self.xcd_order)
        D.step_params = sp
        D.skip_pose_grad = 0 if self.pose_grad else 1
        # 0 = by batch size; tests force the per-ray (large-batch) or split scatter shape
        D.scatter_levels_per_wave = int(getattr(self, "scatter_levels_per_wave", 0))
        D.bwd_flush = int(getattr(self, "bwd_flush", 0))
        # table-gradient scatter: 0 / 2 the run-scan k_scatter (the only one left)
        D.scatter_kernel = int(getattr(self, "scatter_kernel", 0))
        # 0 = by batch size; tests force the 16-flags-per-thread compaction (4096) on small batches
        D.compact_per_block = int(getattr(self, "compact_per_block", 0))
        D.encode_group = int(getattr(self, "encode_group", 0))
        # HBM-atomic counters of the scatter (scatter_atomic_counts): debug steps, the kernel-timing
        # pass, or on request (count_atomics); off in the timed path (they cost 9 us at 2048 rays)
        D.count_atomics = 1 if (debug or self.time_kernels or getattr(self, "count_atomics", False)) else 0
        if self._uses_quads():
            D.table_quads, D.table_rows = self.quads.data_ptr(), self.n_emb // 2
            # 0: the library's batch-size threshold; tests force the quad encode on small batches
            D.quads_min_rays = int(getattr(self, "quads_min_rays", 0))
            D.quads_prebuilt = 0 if join_quads is None else 1
        D.n_ff = self.n_ff
        if self.n_ff:
            D.ff = self.P.data_ptr() + 4 * self.feat_off
            D.grad_ff = self.G.data_ptr() + 4 * self.feat_off
        if self.time_kernels:
            if not self._c_timing:
                L.nof_field_timing(1)
                self._c_timing = True
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        _lib.check(L.nof_field_step(_lib.ctypes.byref(D), st), "field_step")
        if self.time_kernels:
            ev1.record()
            self.kernel_ms.append((ev0, ev1))
        # 5. pose gradient: per-ray dL/dtf -> per-frame sums -> jac^T (nof_pose_backward)
        if self.pose_grad:
            _lib.check(L.nof_pose_backward(_lib.ptr(self.ray_grad), _lib.ptr(self.rays), R, _lib.ptr(self.pose_jac),
                                           self.F, _lib.ptr(self.pose_fg),
                                           _lib.ctypes.c_void_p(self.G.data_ptr() + 4 * self.pose_off), st),
                       "pose_backward")
        if self.n_ff:
            # reg_features = feature_reg_weight * mean(data^2) (nerf_runner.py:743-746): value in loss_terms[6],
            # gradient 2 w data / n (times the GradScaler scale, like the kernel gradients)
            w = float(cfg.get("feature_reg_weight", 0.1))
            f = self.P[self.feat_off:self.pose_off]
            self.loss_acc[6:7].copy_(w * (f * f).mean().view(1))
            self.G[self.feat_off:self.pose_off].add_(f * (self.scale * (2.0 * w / self.n_feat)))
        wp = float(cfg.get("pose_reg_weight", 0.0))
        if wp:
            # pose_reg = pose_reg_weight * ||pose_array.data[1:]|| (nerf_runner.py:748-751): value in loss_terms[7],
            # gradient w p / ||p|| (0 at p = 0), scaled like the kernel gradients
            p = self.P[self.pose_off + 6:]
            nrm = p.norm()
            self.loss_acc[7:8].copy_((wp * nrm).view(1))
            self.G[self.pose_off + 6:].add_(p * (self.scale * wp / nrm.clamp_min(1e-30)))
        return dbg

    def _exchange_and_optimize(self, debug=False):
        """(N>1) the data-parallel exchange + optimiser (exchange.py), else the optimiser."""
        if self.ex is not None:
            return self.ex.step(None, debug, overlap=True)
        return self._optimize(None, debug)

    def _optimize(self, sp, debug=False):
        """(N=1) GradScaler unscale + inf check, Adam with the scheduled learning rates (host
        values of self.global_step, or the device step block sp), GradScaler update;
        returns the unscaled gradients when debug. The fp16 table gradient (amp) is checked
        in place and unscaled inside the Adam kernel."""
        L = _lib.lib()
        st = _lib.stream_of(self.P)
        grads = None
        if self.amp:
            # the NeRFSmall gradients are fp16 in the reference (autocast Linear): out-of-range = overflow
            _lib.check(L.nof_unscale_check(_lib.ctypes.c_void_p(self.G.data_ptr() + 4 * self.mlp_off),
                                           self.P.numel() - self.mlp_off, _lib.ptr(self.scale), _lib.ptr(self.found_inf),
                                           _lib.ptr(self.G16), self.n_emb, 0, self.feat_off - self.mlp_off, st),
                       "unscale")
            if debug:
                grads = self.G.clone()
                grads[:self.n_emb] = self.G16.float() / self.scale
        elif debug:
            grads = self.G.clone()
        ops = _HipOps(self)
        ops.adam(self.P, self.G, self.M, self.V, self.P.numel(), self.pose_off, self.emb16 if self.amp else None, sp,
                 g16=self.G16 if self.amp else None, active=self.adam_active)
        ops.scaler_update()
        return grads

    # ------------------------------------------------------------------ graph replay
    def schedule_desc(self, seed_base=0, batch_seed_base=0):
        """nof_schedule_desc of this config (the device form of lr_at / truncation)."""
        cfg = self.cfg
        kind = cfg.get("trunc_decay_type", "") or ""
        kinds = {"": 0, "linear": 1, "exp": 2}
        if kind not in kinds:
            raise NotImplementedError(f"trunc_decay_type {kind!r} (the reference knows '', 'linear', 'exp')")
        return _lib.ScheduleDesc(lrate=cfg["lrate"], lrate_pose=cfg["lrate_pose"], decay_rate=cfg["decay_rate"],
                                 trunc=cfg["trunc"], trunc_start=cfg.get("trunc_start", cfg["trunc"]),
                                 sc_factor=cfg["sc_factor"], trunc_decay=kinds[kind], n_step=int(cfg["n_step"]),
                                 seed_base=seed_base & 0xFFFFFFFF, batch_seed_base=batch_seed_base & 0xFFFFFFFF)

    def _graph_body(self, part, rays_per_frame, sched, R=None, t_rand=None):
        """One captured step. rays_per_frame: the batch is drawn on the device (throughput
        mode); None: the batch is whatever self.ids[:R] holds at replay (graph_step_ids).
        t_rand: a fixed [R,S] buffer of injected stratification draws read at replay."""
        L = _lib.lib()
        st = _lib.stream_of(self.P)
        sp = self.step_params.data_ptr()
        if rays_per_frame is not None:
            R = (int(self.frame_start.numel()) - 1) * rays_per_frame
        # the quad mirror rebuild forked beside the prologue and trace (not under the sharded exchange,
        # whose "pre" part runs before the mirror all-gather has landed)
        join = self._fork_quad_mirror(R) if part in ("all", "field") else None
        if part in ("all", "field", "pre"):
            # the step schedule, pose forward and MLP packing: one launch; then the batch draw and trace
            # (none of them reads the fp16 table mirror: under the sharded exchange they overlap the
            # previous step's mirror all-gather)
            self._prologue(sched)
            if rays_per_frame is not None:
                nf = int(self.frame_start.numel()) - 1
                _lib.check(L.nof_sample_batch(_lib.ptr(self.frame_start), nf, rays_per_frame, 0, _lib.ptr(self.ids),
                                              _lib.ctypes.c_void_p(sp), st), "sample_batch")
            self._trace(R, sp)
        if part in ("all", "field", "main"):
            self._field_part(R, sp, t_rand, prologue=False, trace=False, join_quads=join)
            if self.ex is not None:
                self.ex.prep()
        if part == "all":
            self._optimize(sp)
        elif part == "optimize":
            self.ex.post(sp)

    def _replay_plan(self):
        """The captured segments and the host collectives between them, in order."""
        if self.ex is None:
            return [("graph", "all")]
        if self.exchange == "sharded":
            # the mirror all-gather is issued at the end of the step and waited for between the next
            # step's trace and its field pass (overlapped with the prologue, batch draw and trace)
            return [("graph", "pre"), ("wait", self.ex.wait_mirror), ("graph", "main"), ("coll", self.ex.reduce),
                    ("graph", "optimize"), ("coll", self.ex.all_gather_mirror_async)]
        return [("graph", "field"), ("coll", self.ex.all_reduce), ("graph", "optimize")]

    def _graph_key(self, *key):
        """Capture key: the call's own arguments plus every host value a captured graph
        bakes in (kernel shape knobs, scaler interval, the loss / regulariser weights of
        cfg) — change any of them and the next graph step captures again."""
        knobs = (self.xcd_order, getattr(self, "scatter_levels_per_wave", 0), getattr(self, "scatter_slots", 0),
                 getattr(self, "use_quads", True), getattr(self, "quads_min_rays", 0),
                 getattr(self, "bwd_flush", 0), getattr(self, "compact_per_block", 0), getattr(self, "scatter_kernel", 0),
                 getattr(self, "encode_group", 0), self.quad_fork,
                 bool(getattr(self, "count_atomics", False)),
                 getattr(self, "ablate", 0), self.blocks_per_cu, self.pose_grad, self.growth_interval)
        return key + knobs + tuple(self.cfg.get(k) for k in self._CAPTURED_CFG)

    # cfg entries the step reads on the host (descriptor scalars, regulariser weights, schedule)
    _CAPTURED_CFG = ("near", "far", "sc_factor", "N_samples", "N_samples_around_depth", "neg_trunc_ratio",
                     "sdf_lambda", "fs_sdf", "first_frame_weight", "rgb_weight", "fs_weight", "empty_weight",
                     "trunc_weight", "fs_rgb_weight", "feature_reg_weight", "pose_reg_weight", "lrate", "lrate_pose",
                     "decay_rate", "trunc", "trunc_start", "trunc_decay_type", "n_step")

    def _capture(self, key, R, rays_per_frame, sched, t_rand=None):
        self._alloc(R)
        self.wait_exchange()
        torch.cuda.synchronize(self.dev)
        plan = []
        for kind, what in self._replay_plan():
            if kind == "graph":
                g = torch.cuda.CUDAGraph()
                self._capturing = True
                try:
                    with torch.cuda.graph(g):
                        self._graph_body(what, rays_per_frame, sched, R, t_rand)
                finally:
                    self._capturing = False
                plan.append(("graph", g))
            else:
                plan.append((kind, what))
        self._graphs = (key, [g for k, g in plan if k == "graph"], sched, plan)

    def _replay(self):
        # bounded run-ahead: the host waits for the replay GRAPH_INFLIGHT steps back before
        # enqueueing another (a GPU-bound step loses nothing; an unbounded queue of graph
        # launches is not relied on)
        if len(self._inflight) >= self.GRAPH_INFLIGHT:
            self._inflight.pop(0).synchronize()
        if self._step_dev_at != self.global_step:
            # the device step counter (k_step_schedule advances it in the graph) is re-synced only
            # after an eager step or an outside change of global_step: one launch fewer per replay
            self.step_dev.fill_(self.global_step)
        for kind, what in self._graphs[3]:
            if kind == "graph":
                what.replay()
            else:          # the exchange's collective between two captured segments
                what()
        ev = torch.cuda.Event()
        ev.record()
        self._inflight.append(ev)
        self.global_step += 1
        self._step_dev_at = self.global_step
        return {"loss_terms": self.loss_acc[:8], "fs_rgb_loss": self.loss_acc[140]}

    def graph_step_ids(self, ids, seed_base=0, t_rand=None):
        """NerfRunner.train()'s iteration (a DataLoader batch of pool ids, nerf_runner.py:854-862)
        replayed from a captured graph: the batch is copied into the fixed id buffer (stream
        order keeps it behind the previous replay), then one graph runs the schedule, the
        field pass and the optimiser. Equivalent to step(ids, seed=seed_base) — or, with
        t_rand [R,S] (injected draws, parity tests), to step(ids, t_rand=t_rand)."""
        if self.time_kernels:
            raise ValueError("graph_step_ids: HIP timing events are not capturable (time_kernels=False)")
        R = int(ids.numel())
        key = self._graph_key("ids", R, seed_base, t_rand is not None)
        if self._graphs is None or self._graphs[0] != key:
            buf = None
            if t_rand is not None:
                S = self.cfg["N_samples"] + self.cfg["N_samples_around_depth"]
                self._t_rand_graph = torch.empty(R, S, dtype=torch.float32, device=self.dev)
                buf = self._t_rand_graph
            self._capture(key, R, None, self.schedule_desc(seed_base, 0), buf)
        self.ids[:R].copy_(ids.to(self.dev).to(torch.int32))
        if t_rand is not None:
            self._t_rand_graph.copy_(torch.as_tensor(t_rand).to(self.dev).float())
        return self._replay()

    GRAPH_INFLIGHT = 4

    def graph_step_epoch(self, perm, k, R, seed_base=0):
        """NerfRunner.train()'s iteration without a per-step id copy: perm is the DataLoader's epoch
        permutation buffer (one device buffer for every epoch), k the index of this step's R-slice
        (DataLoader.next_slice). The captured trace reads slice (step - epoch_step0) of perm on the
        device (nof_trace_rays_epoch); the host rewrites the device epoch_step0 only when that no
        longer names slice k (a new epoch, a reset step count). Equivalent to
        graph_step_ids(perm[k R:(k + 1) R], seed_base)."""
        if self.time_kernels:
            raise ValueError("graph_step_epoch: HIP timing events are not capturable (time_kernels=False)")
        if k < 0 or (k + 1) * R > perm.numel():
            raise RuntimeError(f"graph_step_epoch: slice {k} of {R} ids is outside the {perm.numel()}-id permutation")
        if getattr(self, "_epoch_step0_host", None) != self.global_step - k:
            self._epoch_step0_host = self.global_step - k
            self.epoch_step0.fill_(self._epoch_step0_host)
        key = self._graph_key("epoch", R, perm.data_ptr(), int(perm.numel()), seed_base)
        if self._graphs is None or self._graphs[0] != key:
            self._trace_perm = perm
            try:
                self._capture(key, R, None, self.schedule_desc(seed_base, 0))
            finally:
                self._trace_perm = None
        return self._replay()

    def graph_step(self, rays_per_frame, seed_base=0, batch_seed_base=0):
        """One training iteration replayed from captured HIP graphs (throughput mode:
        rays_per_frame draws per frame, as sample_ids). The whole step — schedule,
        batch draw, field pass, optimiser — is one graph (N=1); with N>1 the RCCL
        all-reduce runs between two graphs. Equivalent to
        step(sample_ids(rays_per_frame, batch_seed_base + global_step), seed=seed_base)."""
        if self.frame_start is None:
            raise ValueError("graph_step needs frame_start (throughput mode)")
        if self.time_kernels:
            raise ValueError("graph_step: HIP timing events are not capturable (time_kernels=False)")
        key = self._graph_key(rays_per_frame, seed_base, batch_seed_base)
        if self._graphs is None or self._graphs[0] != key:
            nf = int(self.frame_start.numel()) - 1
            self._capture(key, nf * rays_per_frame, rays_per_frame, self.schedule_desc(seed_base, batch_seed_base))
        return self._replay()

    # the four timed buckets of nof_field_step: encode (+ quad mirror, sigma net), the colour forward
    # (compaction, k_colour, k_ray_final), the MLP backward (two passes), the scatter
    FIELD_KERNELS = ("k_encode", "k_colour", "k_mlp_bwd", "k_scatter")

    def field_kernel_breakdown(self):
        """Mean duration (ms) of each nof_field_step kernel over the timed calls
        since the last collect (HIP events recorded inside the C ABI between the
        launches, on the launch stream). Returns (dict, n_calls)."""
        buf = (_lib.ctypes.c_float * 8)()
        n = _lib.ctypes.c_int32(0)
        _lib.check(_lib.lib().nof_field_timing_collect(buf, 8, _lib.ctypes.byref(n)), "field_timing_collect")
        k = max(n.value, 1)
        return {name: buf[i] / k for i, name in enumerate(self.FIELD_KERNELS)}, n.value

    def tile_counters(self):
        """Executed work of the last step (the forward's counters): 32-sample tiles that ran
        the sigma net / the colour net, backward records with / without the colour net."""
        c = self.loss_acc[136:140].tolist()
        return {"tiles_sigma": int(c[0]), "tiles_colour": int(c[1]), "records_colour": int(c[2]),
                "records_sigma": int(c[3])}

    def scatter_atomic_counts(self):
        """HBM atomics k_scatter issued in the last step: (table flush, probe overflow). Counted in
        debug steps, the kernel-timing pass (time_kernels) and when count_atomics is set; zero
        otherwise."""
        return self.loss_acc[8:136].view(64, 2).sum(0)

    def pack_mlp(self):
        """Re-pack the MLP fragments from the current parameters (after an optimiser step)."""
        _lib.check(_lib.lib().nof_pack_mlp(_lib.ctypes.c_void_p(self.P.data_ptr() + 4 * self.mlp_off),
                                           _lib.ptr(self.pack_idx), self.n_frag_elems, 5 * 64, _lib.ptr(self.frags),
                                           _lib.ptr(self.bias), _F16 if self.amp else _F32, _lib.stream_of(self.P)),
                   "pack_mlp")

    def query_sdf(self, points=None, axes=None, occ=None):
        """SDF of the current field (run_network_density, nerf_runner.py:1306-1346) at
        points [n,3] or on the grid axes (gx, gy, gz) in meshgrid 'ij' order; points in
        empty voxels of `occ` (dense u8 [N,N,N]) read 1.0 as in extract_mesh."""
        self.wait_exchange()
        self.pack_mlp()
        dev = self.dev
        out_n = None
        gx = gy = gz = None
        nx = ny = nz = 0
        if points is not None:
            pts = torch.as_tensor(points, dtype=torch.float32, device=dev).reshape(-1, 3).contiguous()
            out_n = pts.shape[0]
        else:
            gx, gy, gz = (torch.as_tensor(np.asarray(a, np.float64).astype(np.float32), device=dev) for a in axes)
            nx, ny, nz = len(gx), len(gy), len(gz)
            out_n = nx * ny * nz
            pts = None
        sdf = torch.empty(out_n, dtype=torch.float32, device=dev)
        occ_t = None if occ is None else occ.to(dev).to(torch.uint8).contiguous()
        dt = _F16 if self.amp else _F32
        _lib.check(_lib.lib().nof_query_sdf(
            _lib.ptr(self.emb16 if self.amp else self.P), dt, _lib.ptr(self.levels), self.L, _lib.ptr(self.frags),
            _lib.ptr(self.bias), dt, self.n_in, None if pts is None else _lib.ptr(pts), out_n,
            None if gx is None else _lib.ptr(gx), None if gy is None else _lib.ptr(gy),
            None if gz is None else _lib.ptr(gz), nx, ny, nz, None if occ_t is None else _lib.ptr(occ_t),
            0 if occ_t is None else int(occ_t.shape[0]), _lib.ptr(sdf), _lib.stream_of(sdf)), "query_sdf")
        return sdf

    def refresh_half_table(self):
        """Re-derive the fp16 table mirror after the fp32 table was written from outside (load_weights,
        reset_state). Under the sharded exchange the rank's mirror shard is re-copied as well: the
        all-gather after every step rebuilds emb16 from the shards, and k_adam does not write the
        shard on a skipped step, so a stale shard would overwrite the fresh table."""
        self.wait_exchange()
        if self.amp:
            _lib.check(_lib.lib().nof_to_half(_lib.ptr(self.P), _lib.ptr(self.emb16), self.n_emb,
                                              _lib.stream_of(self.P)), "to_half")
            self._shard_mirror()

    WS_SECTIONS = ("feat", "dfeat", "zbuf", "tile_bwd", "tile_sid", "n_tiles", "ray_aux", "tile_aux", "rctx", "gmask",
                   "rrec", "ctile", "total")

    def _ws_offsets(self):
        """Byte offsets of the workspace sections the host reads, from the library's own layout
        (nof_field_workspace_offsets: FieldWorkspace in field_step.hip), and the tile count."""
        R = self._R
        S = self.cfg["N_samples"] + self.cfg["N_samples_around_depth"]
        o = np.zeros(len(self.WS_SECTIONS), np.uint64)
        _lib.check(_lib.lib().nof_field_workspace_offsets(R, S, _F16 if self.amp else _F32,
                                                          o.ctypes.data_as(ctypes.c_void_p), len(o)),
                   "field_workspace_offsets")
        offs = {k: int(v) for k, v in zip(self.WS_SECTIONS, o)}
        assert offs["total"] == self.workspace.numel()
        return offs, R * (S // 32)

    def n_tile_records(self):
        """Backward tile records written by the last nof_field_step (device counters in the workspace:
        colour-backward tiles at the list's front, count[0], sigma-only tiles at its back, count[2])."""
        off = self._ws_offsets()[0]["n_tiles"]
        c = self.workspace[off:off + 12].view(torch.int32).tolist()
        return int(c[0] + c[2])

    def tile_lists(self):
        """The last field pass's tile lists (k_compact): (backward entries, colour entries) as sorted
        int32 tensors — the order inside a list depends on the blocks' atomic order, the set does not.
        Backward entries are first sample id | sigma-only bit (bit 31), colour entries first sample ids."""
        offs, nt = self._ws_offsets()
        cnt = self.workspace[offs["n_tiles"]:offs["n_tiles"] + 12].view(torch.int32).tolist()
        full = self.workspace[offs["tile_sid"]:offs["tile_sid"] + 4 * nt].view(torch.int32)
        # colour-backward entries at the front (count[0]), sigma-only ones at the back (count[2])
        bl = torch.cat([full[:cnt[0]], full[nt - cnt[2]:]])
        assert bool((full[:cnt[0]] >= 0).all()) and bool((full[nt - cnt[2]:] < 0).all()), "tile list halves mixed"
        cl = self.workspace[offs["ctile"]:offs["ctile"] + 4 * nt].view(torch.int32)[:cnt[1]]
        return torch.sort(bl)[0], torch.sort(cl)[0]

    def field_kernel_ms(self):
        """Durations (ms) of the timed nof_field_step launches (HIP events on the launch stream)."""
        torch.cuda.synchronize()
        out = [a.elapsed_time(b) for a, b in self.kernel_ms]
        self.kernel_ms = []
        return out

    def split(self, flat):
        """Flat [emb | mlp | features | pose] vector -> dict keyed like oracle.nerf_step params."""
        d = {"embeddings": flat[:self.n_emb].view(-1, self.C)}
        o = self.mlp_off
        for k in ML.MLP_KEYS:
            n = int(np.prod(ML.shapes(self.n_in, self.n_ff)[k]))
            d[k] = flat[o:o + n].view(ML.shapes(self.n_in, self.n_ff)[k])
            o += n
        if self.n_ff:
            d["features"] = flat[self.feat_off:self.pose_off].view(self.F, self.n_ff)
        d["pose"] = flat[self.pose_off:].view(self.F, 6)
        return d
