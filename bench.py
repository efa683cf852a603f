"""Benchmark: NeRF training rays/s + ms/iter (BASELINE.json metric) on the
fused MI355X step.

Workload (BASELINE config 2, per GPU): a 16-frame 640x480 synthetic RGB-D
memory pool (bundlesdf_amd/synthetic.py), 2048 rays per frame per step
(32,768 rays/step/GPU, throughput mode), 128 octree + 64 around-depth samples
per ray, L=16 hash grid (finest 128, 2^22 rows, C=2), NeRFSmall 2x64 SDF MLP
+ 3-layer colour MLP, amp on (fp16 table mirror + f16 MFMA, fp32 accumulate,
GradScaler) as config.yml ships. One step = sampling + forward + losses +
full backward + (N>1) RCCL all-reduce of the flat gradient bucket + Adam.

N>1 (torch.distributed.run, one rank per GPU): frames are sharded — rank r
owns frames [16r, 16r+16) of a 16N-frame ring — so per-GPU work is fixed
(weak scaling) and value = N * 32768 rays / max-over-ranks step time.

Prints ONE JSON line (rank 0). The cpu_baseline leg times the CPU oracle
(oracle/nerf_step.py: the reference's step restated; pinned to the
reference's own train_loop by tests/golden/train_step.npz) on a bounded
sample of the same workload on this host.
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
ENC_FWD_B = 12 + 16 * (8 * 2 * 2 + 2 * 2)      # SURVEY §8d encode fwd, fp16 table: 588 B/sample
GRID_BWD_B = 12 + 16 * (2 * 2 + 2 * 8 * 2 * 2)  # §8d grid bwd, fp16 table + fp16 gradient RMW: 1100 B/sample
DW_TILE_B = (28 + 2) * 64 * 8 * 2               # k_dw: one backward tile record (28 fragments) + 2 feature fragments
MFMA_F16_PEAK_TFLOPS = 2500.0  # MI355X dense FP16/BF16 MFMA (MI355X_MICROARCH.md; no sparsity)
MLP_FWD_FLOP = 2 * (32 * 64 + 64 * 16 + 24 * 64 + 64 * 64 + 64 * 3)  # 17,792 FLOP/sample (A14)
MLP_KERNELS = ("k_mlp_fwd", "k_mlp_bwd", "k_dw")


def pmc_traffic(kernel):
    """Per-launch HBM bytes of `kernel` from the newest committed PMC summary
    (profiles/<round>/pmc_traffic.json, scripts/pmc_traffic.py). PMC counters
    need their own rocprofv3 passes, so bench.py reports the committed
    measurement of the same command and names it."""
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
    if not os.path.isdir(root):
        return None, None
    for d in sorted(os.listdir(root), reverse=True):
        p = os.path.join(root, d, "pmc_traffic.json")
        if os.path.exists(p):
            e = json.load(open(p)).get(kernel)
            if e:
                return e["traffic_bytes"], os.path.relpath(p, os.path.dirname(root))
    return None, None


def pmc_mfma():
    """Newest committed MFMA-busy PMC summary (profiles/<round>/pmc_mfma.json,
    scripts/pmc_mfma.py) — hardware MFMA utilisation of the MLP kernels."""
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
    if not os.path.isdir(root):
        return None
    for d in sorted(os.listdir(root), reverse=True):
        p = os.path.join(root, d, "pmc_mfma.json")
        if os.path.exists(p):
            e = json.load(open(p))
            e["source"] = os.path.relpath(p, os.path.dirname(root))
            return e
    return None


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def rank_frames(rank, world, frames_per_gpu, cfg_over):
    """Host side of a rank's shard: cfg, this rank's rendered frames (global ids
    lo..hi-1), all poses (normalised) and the octree cloud."""
    from bundlesdf_amd import synthetic as SY
    F_total = frames_per_gpu * world
    sc, trans = SY.normalization()
    poses_all = SY.camera_poses(F_total, seed=0)
    cfg = SY.default_cfg(sc_factor=sc, translation=trans, **cfg_over)
    # render only this rank's frames
    lo, hi = rank * frames_per_gpu, (rank + 1) * frames_per_gpu
    rgbs, depths, masks = [], [], []
    for T in poses_all[lo:hi]:
        rgb, depth, mask = SY.render_frame(T)
        rgbs.append(rgb)
        depths.append(depth)
        masks.append(mask)
    rgbs = np.stack(rgbs).astype(np.float64)
    depths, masks = np.stack(depths), np.stack(masks)
    depths[depths < 0.1] = 99
    rgbs[masks == 0] = 128
    depths[masks == 0] = 99
    poses_n = poses_all.copy()
    poses_n[:, :3, 3] = (poses_n[:, :3, 3] + trans) * sc
    seq_local = dict(rgbs=(rgbs / 255.0).astype(np.float32), depths=(depths * sc)[..., None].astype(np.float32),
                     masks=masks[..., None], poses=poses_n[lo:hi], K=SY.K_CAM.copy())
    pts = (SY.object_surface_points(seed=0) + trans) * sc
    return cfg, seq_local, poses_n, pts, lo, hi


def build_rank_scene(rank, world, frames_per_gpu, cfg_over, dev):
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.octree import build_occupancy, coarsen
    from bundlesdf_amd.ray_pool import PointGrid, make_pool_rays
    cfg, seq_local, poses_n, pts, lo, hi = rank_frames(rank, world, frames_per_gpu, cfg_over)
    sc = cfg["sc_factor"]
    max_level = int(np.ceil(np.log2(2.0 / (cfg["octree_smallest_voxel_size"] * sc))))
    level = int(np.floor(np.log2(2.0 / (cfg["octree_raytracing_voxel_size"] * sc))))
    dil = max(1, int(np.ceil(cfg["octree_dilate_size"] / cfg["octree_smallest_voxel_size"])))
    occ_f = build_occupancy(torch.from_numpy(pts).float().to(dev), max_level, dil)
    occ = coarsen(occ_f, 2 ** (max_level - level)).contiguous()
    # ray pool on the device, as NerfRunner builds it (nerf_runner.py:170-194,244-314):
    # dilation, box + octree filters, octree-cloud denoise; global frame ids
    pool_args = (range(lo, hi), seq_local["rgbs"], seq_local["depths"], seq_local["masks"], seq_local["poses"],
                 seq_local["K"], cfg)
    grid = PointGrid(pts, 0.02 * sc, dev)
    pool_kw = dict(occ=occ, point_grid=grid, device=dev, index_base=lo)
    pool = make_pool_rays(*pool_args, **pool_kw)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(3):
        pool = make_pool_rays(*pool_args, **pool_kw)
    torch.cuda.synchronize(dev)
    pool_ms = (time.perf_counter() - t0) / 3 * 1e3
    pool_info = {"frames": hi - lo, "pixels": int((hi - lo) * SY.H_IMG * SY.W_IMG), "rays": int(len(pool)),
                 "ms": round(pool_ms, 2), "Mpixel_per_s": round((hi - lo) * SY.H_IMG * SY.W_IMG / pool_ms / 1e3, 1),
                 "includes": "H2D upload of the frames + 5 HIP launches + n_out readback (make_pool_rays)"}
    counts = torch.bincount(pool[:, 8].long() - lo, minlength=hi - lo).cpu().numpy()
    frame_start = np.cumsum(np.concatenate([[0], counts]))
    return cfg, pool, frame_start, poses_n.astype(np.float32), occ, pool_info, (pool_args, pts, level)


def make_models(cfg, F_total, dev, with_features=False):
    from bundlesdf_amd.grid import GridEncoder
    from bundlesdf_amd.nerf_helpers import FeatureArray, NeRFSmall, PoseArray
    torch.manual_seed(0)
    enc = GridEncoder(3, cfg["num_levels"], cfg["feature_grid_dim"], cfg["base_res"], cfg["log2_hashmap_size"],
                      cfg["finest_res"]).to(dev)
    n_ff = cfg.get("frame_features", 0)
    net = NeRFSmall(2, 64, 15, 3, 64, input_ch=enc.out_dim, input_ch_views=9 + n_ff).to(dev)
    pa = PoseArray(F_total, cfg["max_trans"] * cfg["sc_factor"], cfg["max_rot"]).to(dev)
    if with_features:
        return enc, net, pa, (FeatureArray(F_total, n_ff).to(dev) if n_ff > 0 else None)
    return enc, net, pa


# BASELINE config 5 (global refine) overrides, run_custom.py:122-133; bench --workload global_refine
GLOBAL_REFINE = dict(N_samples=64, N_samples_around_depth=256, first_frame_weight=1, finest_res=256, num_levels=16,
                     fs_sdf=0.1, frame_features=2, rgb_weight=100)


def cpu_baseline(cfg, pool, c2w, occ, rays=128, steps=2, threads=1):
    """CPU oracle (reference step restated) on `rays` rays x `steps` steps, fp32."""
    from bundlesdf_amd.grid import level_layout
    from oracle import nerf_step as NS
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    pls, offs = level_layout(3, cfg["num_levels"], 2, cfg["base_res"], cfg["log2_hashmap_size"], cfg["finest_res"])
    torch.manual_seed(0)
    from bundlesdf_amd.nerf_helpers import NeRFSmall
    net = NeRFSmall(2, 64, 15, 3, 64, input_ch=2 * cfg["num_levels"], input_ch_views=9)
    params = {k: v.detach().clone() for k, v in net.state_dict().items()}
    params["embeddings"] = torch.empty(int(offs[-1]), 2).uniform_(-1e-4, 1e-4)
    params["pose"] = torch.zeros(c2w.shape[0], 6)
    meta = (offs, float(np.log2(pls)), cfg["base_res"])
    ccfg = dict(cfg, amp=False)
    S = cfg["N_samples"] + cfg["N_samples_around_depth"]
    times = []
    state = None
    for it in range(steps + 1):
        ids = rng.choice(len(pool), rays, replace=False)
        batch = torch.from_numpy(pool[ids])
        t_rand = torch.from_numpy(rng.uniform(size=(rays, S)).astype(np.float32))
        t0 = time.perf_counter()
        out = NS.train_step(params, batch, torch.from_numpy(c2w), occ, ccfg, t_rand, meta, step=it,
                            lr=cfg["lrate"], adam_state=state)
        params, state = out["params"], out["adam_state"]
        if it > 0:                                  # first step = warm-up
            times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return dict(value=rays / t, unit="rays/s", cores=threads, kind="port",
                sample=f"{rays} rays/step x {steps} timed steps (+1 warm-up) of the same workload "
                       f"(S={S}, L={cfg['num_levels']}, 2^{cfg['log2_hashmap_size']} table), fp32, "
                       f"oracle/nerf_step.py on {threads} host core(s); median {t:.2f} s/step")


def cpu_pool_baseline(pool_src, occ, threads, frames=2):
    """The reference's host ray-pool path (oracle/ray_pool.py: numpy make_frame_rays +
    octree filter + cKDTree denoise) on the first `frames` frames; ms per frame."""
    from oracle import ray_pool as RP
    (_, rgbs, depths, masks, poses, K, cfg), pts, _ = pool_src
    torch.set_num_threads(threads)
    t0 = time.perf_counter()
    RP.build_pool(range(frames), rgbs, depths, masks, poses, K, cfg, occ=occ, cloud=pts)
    return round((time.perf_counter() - t0) / frames * 1e3, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: a 120-step slice of a 500-step training round (config.yml n_step); the
    # first ~20 steps (free space not yet learned: every empty-space sample carries a
    # gradient) run ~15 % slower and are reported separately as warmup_ms_per_step
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    # config2 (default, the headline metric's workload) or global_refine (BASELINE config 5 shape per GPU:
    # 500 frames / 8 GPUs -> 63 frames/GPU, 4096 rays/frame, S = 64 + 256, finest 256, frame_features 2)
    ap.add_argument("--workload", choices=["config2", "global_refine"], default="config2")
    ap.add_argument("--frames-per-gpu", type=int, default=None)
    ap.add_argument("--rays-per-frame", type=int, default=None)
    ap.add_argument("--blocks-per-cu", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-rays", type=int, default=2048)
    args = ap.parse_args()
    gr = args.workload == "global_refine"
    if args.frames_per_gpu is None:
        args.frames_per_gpu = 63 if gr else 16
    if args.rays_per_frame is None:
        args.rays_per_frame = 4096 if gr else 2048
    if gr:
        args.no_cpu_baseline = True   # the CPU port of a 258k-ray x 320-sample step would run for hours

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # NOF_BENCH_BACKEND=gloo + NOF_BENCH_SHARE_GPU=1: rehearsal of the N-rank path on
    # a single GPU (ranks share cuda:0). The real multi-GPU run uses RCCL ("nccl").
    backend = os.environ.get("NOF_BENCH_BACKEND", "nccl")
    if os.environ.get("NOF_BENCH_SHARE_GPU") == "1":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        if backend == "nccl":
            torch.distributed.init_process_group("nccl", device_id=dev)
        else:
            torch.distributed.init_process_group(backend)
        pg = torch.distributed.group.WORLD
    from bundlesdf_amd.fused import FusedStep
    t_setup = time.time()
    cfg, pool, frame_start, c2w, occ, pool_info, pool_src = build_rank_scene(rank, world, args.frames_per_gpu,
                                                                             dict(amp=True, **(GLOBAL_REFINE if gr else {})),
                                                                             dev)
    F_total = args.frames_per_gpu * world
    enc, net, pa, fa = make_models(cfg, F_total, dev, with_features=True)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True,
                   frame_start=frame_start, blocks_per_cu=args.blocks_per_cu, process_group=pg, world_size=world,
                   feature_array=fa)
    log(f"setup {time.time() - t_setup:.1f}s: pool {pool.shape[0]} rays, occupancy {tuple(occ.shape)}")
    R_local = args.frames_per_gpu * args.rays_per_frame

    def one(it):
        ids = fs.sample_ids(args.rays_per_frame, seed=1000 * rank + it)
        return fs.step(ids=ids)

    torch.cuda.synchronize()
    t_w = time.perf_counter()
    for it in range(args.warmup):
        one(it)
    torch.cuda.synchronize()
    t_w = time.perf_counter() - t_w
    if world > 1:
        torch.distributed.barrier()
    # ---- timed region: K plain steps (no instrumentation: HIP timing events slow
    # the host enqueue path on ROCm and would perturb the wall clock)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for it in range(args.steps):
        out = one(args.warmup + it)
    t_enq = time.perf_counter() - t0            # host time to enqueue the K steps
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    dt = float(t.item())
    ms = dt / args.steps * 1e3
    value = world * R_local * args.steps / dt
    loss = float(out["loss_terms"][:4].sum().item())
    # ---- kernel-timing pass: the next K steps of the same workload with HIP
    # events recorded between the field kernels on their stream
    fs.time_kernels = True
    n_valid = torch.zeros(1, device=dev)
    n_bwd = torch.zeros(1, device=dev)
    n_atom = torch.zeros(2, device=dev)
    for it in range(args.steps):
        out = one(args.warmup + args.steps + it)
        n_valid += out["loss_terms"][4]
        n_bwd += out["loss_terms"][5]
        n_atom += fs.scatter_atomic_counts()
    torch.cuda.synchronize()
    kms = fs.field_kernel_ms()
    k_ms = float(np.mean(kms))
    br, n_calls = fs.field_kernel_breakdown()
    nv = float(n_valid.item()) / args.steps
    nb = float(n_bwd.item()) / args.steps
    n_rec = float(fs.n_tile_records())
    # algorithmic bytes per launch of each kernel (SURVEY §8d per-unit figures x units of one launch)
    alg = {"k_encode": nv * ENC_FWD_B, "k_scatter": nb * GRID_BWD_B, "k_dw": n_rec * DW_TILE_B}
    kernels = {}
    for name, kms_k in br.items():
        e = {"ms": round(kms_k, 4)}
        if name in alg and kms_k > 0:
            e["achieved_GBs"] = round(alg[name] / (kms_k * 1e-3) / 1e9, 1)
        kernels[name] = e
    dom = max((k for k in alg), key=lambda k: br[k])
    achieved = alg[dom] / (br[dom] * 1e-3) / 1e9
    per_unit = {"k_encode": f"{ENC_FWD_B} B/in-box sample (§8d encode fwd, fp16 table)",
                "k_scatter": f"{GRID_BWD_B} B/backward sample (§8d grid bwd, fp16 table + fp16 gradient RMW)",
                "k_dw": f"{DW_TILE_B} B/backward tile record"}[dom]
    traffic, traffic_src = pmc_traffic(dom) if not gr else (None, "no PMC pass committed for this workload")
    # MLP on MFMA (north_star: MFMA utilisation against the gfx950 peak). Algorithmic
    # FLOPs are the reference's: every in-box sample runs the forward and the full
    # backward (3 x 17,792 FLOP, §8d), whatever this implementation skips.
    mlp_ms = sum(br.get(k, 0.0) for k in MLP_KERNELS)
    mlp_tf = nv * 3 * MLP_FWD_FLOP / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else 0.0
    mlp = {"kernels": list(MLP_KERNELS), "ms": round(mlp_ms, 4), "alg_flop_per_sample": 3 * MLP_FWD_FLOP,
           "achieved": round(mlp_tf, 1), "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s",
           "frac": round(mlp_tf / MFMA_F16_PEAK_TFLOPS, 4), "pmc_mfma_busy": None if gr else pmc_mfma()}
    result = {
        "metric": "NeRF training rays/sec + ms/iter, 64-frame pool, 2048 rays/frame",
        "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp16 table+MLP (MFMA) / fp32 accumulate+Adam (amp)", "data": "synthetic",
        "config": {"workload": ("BASELINE config 5 (global refine) per-GPU shape: 63-frame pool/GPU, 4096 rays/frame, "
                                "320 samples/ray (64 + 256 around depth), L=16 hash grid (finest 256, 2^22, top levels "
                                "hashed), frame_features 2, NeRFSmall 2x64 SDF + 3x64 colour, amp, one pass (no "
                                "micro-batches)") if gr else
                               ("BASELINE config 2: 16-frame pool/GPU, 2048 rays/frame, 192 samples/ray, L=16 hash "
                                "grid (finest 128, 2^22), NeRFSmall 2x64 SDF + 3x64 colour, amp"),
                   "rays_per_step_per_gpu": R_local, "frames_per_gpu": args.frames_per_gpu,
                   "parallelism": (f"dp{world} (frame-sharded, {'RCCL' if backend == 'nccl' else backend} all-reduce)"
                                   if world > 1 else "single GPU")},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src, "alg_bytes": int(alg[dom]),
                     "kernel_ms": round(br[dom], 4), "per_unit": per_unit,
                     "units_per_launch": int({"k_encode": nv, "k_scatter": nb, "k_dw": n_rec}[dom]),
                     "timed_calls": n_calls,
                     "timing": "HIP events between the field kernels over a second pass of K steps right after the "
                               "timed region (same workload); value/ms_per_step come from the uninstrumented pass"},
        "warmup_ms_per_step": round(t_w / max(args.warmup, 1) * 1e3, 3),
        "field_step_ms": round(k_ms, 3),
        "host_enqueue_ms_per_step": round(t_enq / args.steps * 1e3, 3),
        "kernels": kernels,
        "mlp_mfma": mlp,
        "samples_in_box": int(nv), "samples_backward": int(nb), "tile_records": int(n_rec),
        "scatter_hbm_atomics": {"table_flush": int(n_atom[0].item() / args.steps),
                                "probe_overflow": int(n_atom[1].item() / args.steps)},
        "loss": round(loss, 5),
        "ray_pool": pool_info,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        result["cpu_baseline"] = cpu_baseline(cfg, pool.cpu().numpy(), c2w, occ.cpu().numpy(), rays=args.cpu_rays,
                                              steps=3, threads=threads)
        result["ray_pool"]["cpu_oracle_ms_per_frame"] = cpu_pool_baseline(pool_src, occ.cpu().numpy(), threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
