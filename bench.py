"""Benchmark: NeRF training rays/s + ms/iter (BASELINE.json metric) on the
fused MI355X step.

Headline workload (default; BASELINE.json `metric`, config 4's pool): a
64-frame 640x480 synthetic RGB-D memory pool (bundlesdf_amd/synthetic.py),
2048 rays per frame per optimiser step (131,072 rays/step), 128 octree + 64
around-depth samples per ray, L=16 hash grid (finest 128, 2^22 rows, C=2),
NeRFSmall 2x64 SDF MLP + 3-layer colour MLP, amp on (fp16 table mirror + f16
MFMA, fp32 accumulate, GradScaler) as config.yml ships. One step = sampling +
forward + losses + full backward + (N>1) the RCCL gradient exchange (amp: reduce-scatter
of the table gradient, Adam on the rank's shard, all-gather of the fp16 table mirror,
all-reduce of the MLP / feature / pose bucket; bundlesdf_amd/exchange.py) + Adam.

N>1 (torch.distributed.run, one rank per GPU): the 64 frames are sharded
64/N per rank (rank r owns frames [r*64/N, (r+1)*64/N)), so the global batch
stays 131,072 rays per step (strong scaling) and value =
131,072 rays / max-over-ranks step time.

At N=1 the same JSON line also carries the other BASELINE configurations,
each on a fresh scene and fresh models with the same protocol: `config2`
(16-frame pool, 32,768 rays/step), `parity_mode` (NerfRunner.train()'s
N_rand=2048 rays per step drawn by the epoch randperm over the 64-frame pool)
and `config1` (1 frame, 512 rays, L=4, fp32) next to the CPU oracle on the
same config-1 shape. `cpu_baseline` times the CPU oracle (oracle/nerf_step.py:
the reference's step restated; pinned to the reference's own train_loop by
tests/golden/train_step.npz) on a bounded sample of the headline workload.
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
L2_SHARED_GATHER_GBS = 16800.0                  # MI355X_MICROARCH.md cache-tier gather ceiling (L2-shared rows)
GRID_BWD_B = 12 + 16 * (2 * 2 + 2 * 8 * 2 * 2)  # §8d grid bwd, fp16 table + fp16 gradient RMW: 1100 B/sample
MFMA_F16_PEAK_TFLOPS = 2500.0  # MI355X dense FP16/BF16 MFMA (MI355X_MICROARCH.md; no sparsity)
MLP_FWD_FLOP = 2 * (32 * 64 + 64 * 16 + 24 * 64 + 64 * 64 + 64 * 3)  # 17,792 FLOP/sample (A14)
MLP_KERNELS = ("k_colour", "k_mlp_bwd")   # the colour forward bucket (compaction + k_colour + k_ray_final), the backward


def _pmc_files(root, prefix):
    """Committed PMC summaries, newest round first; inside a round the measurement of the current
    build named in profiles/<round>/PMC_LATEST (its tag) first, then the others by name."""
    for d in sorted(os.listdir(root), reverse=True):
        dd = os.path.join(root, d)
        if not os.path.isdir(dd):
            continue
        names = sorted((fn for fn in os.listdir(dd) if fn.startswith(prefix) and fn.endswith(".json")), reverse=True)
        lp = os.path.join(dd, "PMC_LATEST")
        tag = open(lp).read().strip() if os.path.exists(lp) else None
        if tag:
            names.sort(key=lambda fn: fn != f"{prefix}_{tag}.json")
        for fn in names:
            yield os.path.join(dd, fn)


def pmc_traffic(kernel, workload="headline", frames=64):
    """Per-launch HBM bytes of `kernel` from the newest committed PMC summary of
    the same workload (profiles/<round>/pmc_traffic*.json with a matching
    "_workload" key, scripts/pmc_traffic.py). PMC counters need their own
    rocprofv3 passes, so bench.py reports the committed measurement of the same
    command and names it."""
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
    if not os.path.isdir(root):
        return None, None
    want = f"{workload}:{frames}"
    for p in _pmc_files(root, "pmc_traffic"):
        js = json.load(open(p))
        if js.get("_workload", "config2:16") != want:
            continue
        e = js.get(kernel)
        if e:
            return e["traffic_bytes"], os.path.relpath(p, os.path.dirname(root))
    return None, f"no PMC pass committed for workload {want}"


def executed_mlp_flops(fs, mlp_ms):
    """Useful MLP FLOPs the MLP kernels actually executed in the last step (tile counters:
    every 32-sample tile with a sample in the box runs the sigma net, weighted tiles the
    colour net; backward records run dX + dW for the layers they touch), over the MLP
    kernels' time. The sigma net runs inside the encode kernel, so its forward FLOPs run in
    k_encode's time: they are reported apart and left out of the MLP kernels' rate."""
    c = fs.tile_counters()
    n_in, cin = fs.n_in, 24 + fs.n_ff
    sig = 2 * (n_in * 64 + 64 * 16)
    col = 2 * (cin * 64 + 64 * 64 + 64 * 3)
    sig_fwd = 32 * c["tiles_sigma"] * sig
    fl = 32 * (c["tiles_colour"] * col + 2 * (c["records_colour"] * (sig + col) + c["records_sigma"] * sig))
    tf = fl / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else 0.0
    return dict(c, flop=int(fl), achieved=round(tf, 1), frac=round(tf / MFMA_F16_PEAK_TFLOPS, 4),
                sigma_forward_in_k_encode_flop=int(sig_fwd),
                note="useful (unpadded) FLOPs of the tiles the MLP kernels executed in the last timed step "
                     "(the sigma-net forward inside k_encode is counted apart)")


def pmc_mfma(workload="headline", frames=64):
    """Newest committed MFMA-busy PMC summary of the same workload
    (profiles/<round>/pmc_mfma*.json, scripts/pmc_mfma.py) — hardware MFMA utilisation of
    the MLP kernels."""
    root = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles")
    if not os.path.isdir(root):
        return None
    want = f"{workload}:{frames}"
    for p in _pmc_files(root, "pmc_mfma"):
        e = json.load(open(p))
        if e.get("_workload", "headline:64") != want:
            continue
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


def rounds_for(steps_req, n_iters):
    """The timed region is whole training rounds: bundlesdf.py re-creates the model for
    every online round (add_new_frames(reuse_weights=False) -> create_nerf, bundlesdf.py:223,
    nerf_runner.py:379-380) and trains n_step + 1 steps (nerf_runner.py:854-862). The step
    cost depends on the training state (work with exactly zero gradient is skipped), so the
    representative figure is the mean over a whole round from initialisation."""
    n = max(1, -(-int(steps_req) // n_iters)) if steps_req else 1
    return n, n * n_iters


def run_steps(step_fn, fs, P0, warmup, n_rounds, n_iters, world, dev, phases=()):
    """W untimed warm-up steps (graph capture, caches), then the model is re-initialised
    and EXACTLY n_rounds x n_iters steps are timed between barrier + synchronize on both
    sides, each round from the initial parameters (fs.reset_state). Returns (max-over-ranks
    seconds, warm-up s, host enqueue s, last output, phase ms/step over `phases` — step
    boundaries of the first round, from HIP events on the step stream)."""
    torch.cuda.synchronize()
    t_w = time.perf_counter()
    for it in range(warmup):
        step_fn(it)
    torch.cuda.synchronize()
    t_w = time.perf_counter() - t_w
    fs.reset_state(P0)
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    bounds = sorted(set([0] + [b for b in phases if 0 < b < n_iters] + [n_iters]))
    evs = {}
    t0 = time.perf_counter()
    out = None
    it = 0
    for rd in range(n_rounds):
        if rd:
            fs.reset_state(P0)
        for k in range(n_iters):
            if rd == 0 and k in bounds:
                evs[k] = torch.cuda.Event(enable_timing=True)
                evs[k].record()
            out = step_fn(it)
            it += 1
            if k % 100 == 99:
                log(f"  round {rd} step {k + 1}/{n_iters}")   # progress (no device sync)
        if rd == 0:
            evs[n_iters] = torch.cuda.Event(enable_timing=True)
            evs[n_iters].record()
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        dt = float(t.item())
    prof = {f"steps_{a}_{b}": round(evs[a].elapsed_time(evs[b]) / (b - a), 4) for a, b in zip(bounds[:-1], bounds[1:])}
    return dt, t_w, t_enq, out, prof


def host_cpu():
    """CPU model and physical core count of this host (lscpu's fields, from /proc/cpuinfo),
    and the threads the CPU baseline may use: the box grants one GPU job a share of 16
    threads (OMP_NUM_THREADS), so the baseline runs min(physical cores, that share)."""
    model, cores = "unknown", set()
    try:
        phys = core = None
        for line in open("/proc/cpuinfo"):
            k, _, v = line.partition(":")
            k, v = k.strip(), v.strip()
            if k == "model name":
                model = v
            elif k == "physical id":
                phys = v
            elif k == "core id":
                core = v
                cores.add((phys, core))
    except OSError:
        pass
    n_phys = len(cores) or (os.cpu_count() or 1)
    share = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return {"cpu_model": model, "host_physical_cores": n_phys, "threads": max(1, min(n_phys, share)),
            "thread_share": share}


def side_line(cfg_over, frames, rays_per_frame, dev, warmup, n_rounds, parity=False, amp=True, graph=True):
    """A single-GPU measurement of another BASELINE configuration (fresh scene,
    fresh models, same protocol): config 2 (16-frame pool), parity mode
    (NerfRunner.train()'s N_rand rays drawn uniformly over the pool), config 1."""
    from bundlesdf_amd.fused import FusedStep
    from bundlesdf_amd.nerf_runner import DataLoader
    cfg, pool, frame_start, c2w, occ, _, _ = build_rank_scene(0, 1, frames, dict(amp=amp, **cfg_over), dev)
    enc, net, pa, fa = make_models(cfg, frames, dev, with_features=True)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=amp, frame_start=frame_start,
                   feature_array=fa)
    if parity:
        torch.manual_seed(0)                      # NerfRunner: set_seed(0); the epoch randperm is a CPU draw
        dl = DataLoader(pool, cfg["N_rand"])
        R = cfg["N_rand"]
        if graph:   # NerfRunner.train() replays one captured graph per DataLoader batch
            step_fn = lambda it: fs.graph_step_epoch(*dl.next_slice(), R)  # noqa: E731
        else:
            step_fn = lambda it: fs.step(ids=dl.next_ids())  # noqa: E731
    else:
        R = frames * rays_per_frame
        if graph:
            step_fn = lambda it: fs.graph_step(rays_per_frame, batch_seed_base=7000)  # noqa: E731
        else:
            step_fn = lambda it: fs.step(ids=fs.sample_ids(rays_per_frame, seed=7000 + it))  # noqa: E731
    n_iters = cfg["n_step"] + 1
    P0 = fs.P.detach().clone()
    dt, t_w, _, out, prof = run_steps(step_fn, fs, P0, warmup, n_rounds, n_iters, 1, dev, phases=(20, 100))
    steps = n_rounds * n_iters
    ms = dt / steps * 1e3
    e = {"value": round(R * steps / dt, 1), "unit": "rays/s", "ms_per_step": round(ms, 4), "rays_per_step": R,
         "steps": steps, "execution": "hipGraph replay" if graph else "eager launches",
         "frames": frames, "round_phases_ms_per_step": prof,
         "loss": round(float(out["loss_terms"][:4].sum().item()), 5)}
    del fs
    torch.cuda.empty_cache()
    return e, (cfg, pool, c2w, occ)


def _free_port():
    import socket
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv):
    """`python bench.py --gpus N` with no launcher around it (WORLD_SIZE unset): start the N
    ranks as ONE child process, `python -m torch.distributed.run --nproc-per-node N ... bench.py
    <same arguments>` (a child, never an exec: this process has not touched the GPU and stays
    the parent), forward the children's output, and print rank 0's JSON line. Returns the
    child's exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + list(argv)
    log(f"launching {n} ranks: {' '.join(cmd[1:])}")
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, text=True, bufsize=1)
    line = None
    for ln in proc.stdout:
        if ln.lstrip().startswith("{"):
            line = ln.strip()            # rank 0's result line
        else:
            sys.stderr.write(ln)
            sys.stderr.flush()
    rc = proc.wait()
    if line is not None:
        print(line, flush=True)
    elif rc == 0:
        log("no result line from rank 0")
        rc = 1
    return rc


def init_distributed(backend, dev=None):
    """The process group with bounded waits: every collective (and the rendezvous) gives up after
    exchange.COLLECTIVE_TIMEOUT_S; on RCCL the async error handling turns a stuck or failed
    collective into an error on every rank instead of a silent hang (set before the group exists)."""
    import datetime
    from bundlesdf_amd import exchange as EX
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    kw = dict(timeout=datetime.timedelta(seconds=EX.COLLECTIVE_TIMEOUT_S))
    if backend == "nccl":
        kw["device_id"] = dev
    torch.distributed.init_process_group(backend, **kw)


def dry_run(world, rank):
    """--dry-run (CPU test of the launch plumbing): the process group over gloo with the bench's
    timeout, three 'steps' of one collective each through exchange.collective (as the training
    exchange issues them), rank 0 prints a JSON line with the world size; nothing touches the GPU.
    NOF_DRY_RUN_STALL_RANK=r makes rank r stall before its second collective (the failure
    rehearsal: its peers must time out and every rank exit non-zero)."""
    from bundlesdf_amd import exchange as EX
    if world > 1:
        init_distributed("gloo")
        stall = int(os.environ.get("NOF_DRY_RUN_STALL_RANK", "-1"))
        for step in range(3):
            if step == 1 and rank == stall:
                time.sleep(4 * EX.COLLECTIVE_TIMEOUT_S)
            t = torch.ones(1)
            EX.collective("all_reduce", lambda: torch.distributed.all_reduce(t), step)
            assert int(t.item()) == world
    if rank == 0:
        print(json.dumps({"metric": "dry-run", "n_gpus": world, "dry_run": True}), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--dry-run", action="store_true", help="launch plumbing only (no GPU): CPU tests")
    # the timed region is whole training rounds of n_step + 1 = 501 steps (config.yml n_step),
    # each from a freshly initialised model (rounds_for): --steps K times ceil(K / 501) rounds
    # (default one); W warm-up steps run before and the model is re-initialised after them
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=20)
    # headline (default): BASELINE.json's metric — the 64-frame pool at 2048 rays/frame
    # (131,072 rays per optimiser step), sharded 64/N frames per rank (config 4's strong
    # scaling at fixed R_global); config2: 16 frames per GPU (weak); global_refine: the
    # BASELINE config 5 per-GPU shape (63 frames/GPU, 4096 rays/frame, S = 64 + 256)
    ap.add_argument("--workload", choices=["headline", "config2", "global_refine"], default="headline")
    ap.add_argument("--pool-frames", type=int, default=64)
    ap.add_argument("--frames-per-gpu", type=int, default=None)
    ap.add_argument("--rays-per-frame", type=int, default=None)
    ap.add_argument("--blocks-per-cu", type=int, default=0, help="reserved (the removed per-ray forward kernel's grid)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip the config-2 / parity-mode / config-1 lines")
    ap.add_argument("--cpu-rays", type=int, default=2048)
    ap.add_argument("--no-graph", action="store_true",
                    help="time eager launches instead of the captured hipGraph step (the eager rate is reported "
                         "beside the graph rate either way)")
    args = ap.parse_args()
    gr = args.workload == "global_refine"
    if args.gpus < 1:
        raise SystemExit(f"--gpus {args.gpus}: need at least 1")
    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            # no launcher: this process becomes the parent of the N ranks (it never touches the GPU)
            sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but the launcher started WORLD_SIZE={os.environ['WORLD_SIZE']} ranks")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.dry_run:
        dry_run(world, rank)
        return
    local = int(os.environ.get("LOCAL_RANK", "0"))
    strong = args.workload == "headline" and args.frames_per_gpu is None
    if args.frames_per_gpu is None:
        if args.workload == "headline":
            if args.pool_frames % world:
                raise SystemExit(f"--pool-frames {args.pool_frames} is not divisible by {world} ranks")
            args.frames_per_gpu = args.pool_frames // world
        else:
            args.frames_per_gpu = 63 if gr else 16
    if args.rays_per_frame is None:
        args.rays_per_frame = 4096 if gr else 2048
    if gr:
        args.no_cpu_baseline = True   # the CPU port of a 258k-ray x 320-sample step would run for hours
        args.no_extras = True

    # NOF_BENCH_BACKEND=gloo + NOF_BENCH_SHARE_GPU=1: rehearsal of the N-rank path on
    # a single GPU (ranks share cuda:0). The real multi-GPU run uses RCCL ("nccl").
    backend = os.environ.get("NOF_BENCH_BACKEND", "nccl")
    if os.environ.get("NOF_BENCH_SHARE_GPU") == "1":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    if world > 1:
        init_distributed(backend, dev)
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

    def ids_fn(it):
        return fs.sample_ids(args.rays_per_frame, seed=1000 * rank + it)

    def eager_fn(it):
        return fs.step(ids=ids_fn(it))

    def graph_fn(it):
        # the captured step draws its batch with seed 1000 * rank + global step (device schedule)
        return fs.graph_step(args.rays_per_frame, batch_seed_base=1000 * rank)

    n_iters = cfg["n_step"] + 1
    n_rounds, steps = rounds_for(args.steps, n_iters)
    P0 = fs.P.detach().clone()            # the round's initial parameters (create_nerf)
    use_graph = not args.no_graph
    dt, t_w, t_enq, out, phases = run_steps(graph_fn if use_graph else eager_fn, fs, P0, args.warmup, n_rounds,
                                            n_iters, world, dev, phases=(20, 100))
    ms = dt / steps * 1e3
    value = world * R_local * steps / dt
    loss = float(out["loss_terms"][:4].sum().item())
    # the other execution mode over one more whole round from initialisation
    dt_o, _, t_enq_o, _, _ = run_steps(eager_fn if use_graph else graph_fn, fs, P0, 0, 1, n_iters, world, dev)
    other = {"execution": "eager launches" if use_graph else "hipGraph replay",
             "ms_per_step": round(dt_o / n_iters * 1e3, 3), "steps": n_iters,
             "value": round(world * R_local * n_iters / dt_o, 1),
             "host_enqueue_ms_per_step": round(t_enq_o / n_iters * 1e3, 3)}
    # ---- kernel-timing pass: one more whole round (eager launches from initialisation) with
    # HIP events recorded between the field kernels on their stream
    fs.reset_state(P0)
    fs.time_kernels = True
    n_valid = torch.zeros(1, device=dev)
    n_bwd = torch.zeros(1, device=dev)
    n_atom = torch.zeros(2, device=dev)
    for it in range(n_iters):
        out = fs.step(ids=ids_fn(it))
        if it % 100 == 99:
            log(f"  kernel-timing round step {it + 1}/{n_iters}")
        n_valid += out["loss_terms"][4]
        n_bwd += out["loss_terms"][5]
        n_atom += fs.scatter_atomic_counts()
    torch.cuda.synchronize()
    kms = fs.field_kernel_ms()
    k_ms = float(np.mean(kms))
    br, n_calls = fs.field_kernel_breakdown()
    fs.time_kernels = False
    nv = float(n_valid.item()) / n_iters
    nb = float(n_bwd.item()) / n_iters
    n_rec = float(fs.n_tile_records())
    # algorithmic bytes per launch of each kernel (SURVEY §8d per-unit figures x units of one launch)
    alg = {"k_encode": nv * ENC_FWD_B, "k_scatter": nb * GRID_BWD_B}
    kernels = {}
    for name, kms_k in br.items():
        e = {"ms": round(kms_k, 4)}
        if name in alg and kms_k > 0:
            e["achieved_GBs"] = round(alg[name] / (kms_k * 1e-3) / 1e9, 1)
        kernels[name] = e
    if "achieved_GBs" in kernels.get("k_encode", {}):
        # the encode's corner gathers are served from L2 / Infinity Cache, not HBM (its PMC traffic is
        # far below the algorithmic bytes): its ceiling is the cache tier's (MI355X_MICROARCH.md, gathers
        # of L2-shared rows), not the HBM peak
        ke = kernels["k_encode"]
        ke["cache_tier"] = {"ceiling_GBs": L2_SHARED_GATHER_GBS, "frac": round(ke["achieved_GBs"] / L2_SHARED_GATHER_GBS, 4),
                            "note": "algorithmic bytes / duration vs the L2-shared-row gather ceiling (16.8 TB/s; "
                                    "random Infinity-Cache gathers: 8.6 TB/s)"}
    dom = max((k for k in alg), key=lambda k: br[k])
    achieved = alg[dom] / (br[dom] * 1e-3) / 1e9
    per_unit = {"k_encode": f"{ENC_FWD_B} B/in-box sample (§8d encode fwd, fp16 table)",
                "k_scatter": f"{GRID_BWD_B} B/backward sample (§8d grid bwd, fp16 table + fp16 gradient RMW)"}[dom]
    traffic, traffic_src = pmc_traffic(dom, args.workload, args.frames_per_gpu) if not gr else \
        (None, "no PMC pass committed for this workload")
    # MLP on MFMA (north_star: MFMA utilisation against the gfx950 peak): the headline figure
    # counts the FLOPs the kernels executed (tile counters, unpadded); the reference-FLOP
    # figure (every in-box sample runs forward + full backward, 3 x 17,792 FLOP, §8d) beside it
    mlp_ms = sum(br.get(k, 0.0) for k in MLP_KERNELS)
    mlp_tf = nv * 3 * MLP_FWD_FLOP / (mlp_ms * 1e-3) / 1e12 if mlp_ms > 0 else 0.0
    ex = executed_mlp_flops(fs, mlp_ms)
    mlp = {"kernels": list(MLP_KERNELS), "ms": round(mlp_ms, 4), "achieved": ex["achieved"],
           "peak": MFMA_F16_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": ex["frac"], "executed": ex,
           "reference_flops": {"alg_flop_per_sample": 3 * MLP_FWD_FLOP, "achieved": round(mlp_tf, 1),
                               "frac": round(mlp_tf / MFMA_F16_PEAK_TFLOPS, 4),
                               "note": "reference FLOPs of every in-box sample, including tiles this "
                                       "implementation skips (zero gradient)"},
           "pmc_mfma_busy": None if gr else pmc_mfma(args.workload, args.frames_per_gpu)}
    if gr:
        workload = ("BASELINE config 5 (global refine) per-GPU shape: 63-frame pool/GPU, 4096 rays/frame, "
                    "320 samples/ray (64 + 256 around depth), L=16 hash grid (finest 256, 2^22, top levels "
                    "hashed), frame_features 2, NeRFSmall 2x64 SDF + 3x64 colour, amp, one pass (no micro-batches)")
    elif strong:
        workload = (f"BASELINE metric: {F_total}-frame pool, {args.rays_per_frame} rays/frame = "
                    f"{F_total * args.rays_per_frame} rays per optimiser step ({args.frames_per_gpu} frames on each "
                    f"of {world} GPU(s): config 4's frame sharding at fixed R_global), 192 samples/ray, L=16 hash "
                    "grid (finest 128, 2^22), NeRFSmall 2x64 SDF + 3x64 colour, amp")
    else:
        workload = (f"{args.frames_per_gpu}-frame pool/GPU (BASELINE config 2 at 16), {args.rays_per_frame} "
                    "rays/frame, 192 samples/ray, L=16 hash grid (finest 128, 2^22), NeRFSmall 2x64 SDF + 3x64 "
                    "colour, amp")
    result = {
        "metric": "NeRF training rays/sec + ms/iter, 64-frame pool, 2048 rays/frame",
        "value": round(value, 1), "unit": "rays/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "fp16 table+MLP (MFMA) / fp32 accumulate+Adam (amp)", "data": "synthetic",
        "config": {"workload": workload, "rays_per_step": world * R_local, "rays_per_step_per_gpu": R_local,
                   "pool_frames": F_total, "frames_per_gpu": args.frames_per_gpu,
                   "rays_per_frame": args.rays_per_frame,
                   "parallelism": (f"dp{world} (frame-sharded, {'RCCL' if backend == 'nccl' else backend}: "
                                   + ("reduce-scatter of the fp16 table gradient + sharded Adam + all-gather of the "
                                      "fp16 table mirror, all-reduce of the MLP/feature/pose bucket)"
                                      if fs.exchange == "sharded" else "fp32 gradient all-reduce)")
                                   if world > 1 else "single GPU")},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1),
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": traffic_src, "alg_bytes": int(alg[dom]),
                     "kernel_ms": round(br[dom], 4), "per_unit": per_unit,
                     "units_per_launch": int({"k_encode": nv, "k_scatter": nb}[dom]),
                     "timed_calls": n_calls,
                     "timing": "HIP events between the field kernels over one whole round (501 eager steps from "
                               "initialisation, same workload) after the timed region; value/ms_per_step come "
                               "from the uninstrumented pass"},
        "timed_region": (f"{n_rounds} whole training round(s) of n_step + 1 = {n_iters} steps, each from a freshly "
                         "initialised model (bundlesdf.py:223 re-creates it every online round); the W warm-up "
                         "steps run before and are followed by a re-initialisation"),
        "steps_requested": args.steps,
        "steps_policy": (f"whole training rounds: steps = ceil(steps_requested / {n_iters}) x {n_iters} (one round "
                         "when --steps is not given), never fewer than requested. A round starts from a freshly "
                         "initialised model, as bundlesdf.py re-creates it every online round, and its per-step "
                         "cost changes over the round (round_phases_ms_per_step), so a partial round would not "
                         "measure the reference's training step"),
        "round_phases_ms_per_step": phases,
        "execution": "hipGraph replay (one captured graph per step: schedule, batch draw, field pass, "
                     "optimiser)" if use_graph else "eager launches",
        "other_execution": other,
        "warmup_ms_per_step": round(t_w / max(args.warmup, 1) * 1e3, 3) if args.warmup else None,
        "field_step_ms": round(k_ms, 3),
        # graph mode: the host waits for the replay GRAPH_INFLIGHT steps back, so its loop time
        # tracks the GPU; the eager pass's enqueue time is in other_execution
        "host_enqueue_ms_per_step": None if use_graph else round(t_enq / steps * 1e3, 3),
        "kernels": kernels,
        "mlp_mfma": mlp,
        "samples_in_box": int(nv), "samples_backward": int(nb), "tile_records": int(n_rec),
        "scatter_hbm_atomics": {"table_flush": int(n_atom[0].item() / n_iters),
                                "probe_overflow": int(n_atom[1].item() / n_iters)},
        "loss": round(loss, 5),
        "ray_pool": pool_info,
    }
    del fs
    torch.cuda.empty_cache()
    if rank == 0 and world == 1 and not args.no_extras:
        # other BASELINE configurations, same protocol (fresh scene + models each)
        result["config2"], _ = side_line({}, 16, 2048, dev, args.warmup, 1)
        result["config2"]["workload"] = "BASELINE config 2: 16-frame pool, 2048 rays/frame (32,768 rays/step), amp"
        result["parity_mode"], _ = side_line({}, args.pool_frames, 2048, dev, args.warmup, 1, parity=True)
        result["parity_mode"]["workload"] = (f"NerfRunner.train() semantics: N_rand=2048 rays per step drawn by the "
                                             f"epoch randperm over the whole {args.pool_frames}-frame pool, amp")
        pe, _ = side_line({}, args.pool_frames, 2048, dev, args.warmup, 1, parity=True, graph=False)
        result["parity_mode"]["eager"] = {k: pe[k] for k in ("value", "ms_per_step", "execution")}
        c1, (cfg1, pool1, c2w1, occ1) = side_line(dict(num_levels=4), 1, 512, dev, args.warmup, 1,
                                                  amp=False)
        c1["workload"] = "BASELINE config 1: 1 frame, 512 rays/step, 192 samples/ray, L=4 (config.yml), fp32"
        if not args.no_cpu_baseline:
            hc = host_cpu()
            c1["cpu_oracle"] = cpu_baseline(cfg1, pool1.cpu().numpy(), c2w1, occ1.cpu().numpy(), rays=512, steps=5,
                                            threads=hc["threads"])
            c1["cpu_oracle"].update(hc)
            c1["gpu_over_cpu"] = round(c1["value"] / c1["cpu_oracle"]["value"], 1)
        result["config1"] = c1
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        hc = host_cpu()
        threads = hc["threads"]
        result["cpu_baseline"] = cpu_baseline(cfg, pool.cpu().numpy(), c2w, occ.cpu().numpy(), rays=args.cpu_rays,
                                              steps=3, threads=threads)
        result["cpu_baseline"].update(hc)
        result["gpu_over_cpu"] = round(value / result["cpu_baseline"]["value"], 1)
        result["ray_pool"]["cpu_oracle_ms_per_frame"] = cpu_pool_baseline(pool_src, occ.cpu().numpy(), threads)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    try:
        main()
    except Exception as exc:          # noqa: BLE001
        if int(os.environ.get("WORLD_SIZE", "1")) > 1:
            # a rank whose collective failed or timed out (exchange.CollectiveError names rank / step /
            # phase) ends at once with a non-zero status: no retry, no wait in the group's teardown
            log_all = f"[rank {os.environ.get('RANK', '?')}] bench.py failed: {type(exc).__name__}: {exc}"
            print(log_all, file=sys.stderr, flush=True)
            os._exit(3)
        raise
