"""NerfRunner.train()-sized steps (2048 rays over the 64-frame pool, graph replay) for a rocprofv3
kernel-stats profile of the small-batch shapes: python scripts/small_batch_prof.py [steps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda", 0)
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(0, 1, 64, dict(amp=True), dev)
    enc, net, pa = bench.make_models(cfg, 64, dev)
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True, frame_start=frame_start)
    if os.environ.get("ABLATE"):   # timing-build ablation bits (NOF_LIB = libnof_ablate.so)
        fs.ablate = int(os.environ["ABLATE"])
    if os.environ.get("LPW"):   # k_scatter levels per wave (0: the library's choice by batch size)
        fs.scatter_levels_per_wave = int(os.environ["LPW"])
    if os.environ.get("SK"):   # scatter kernel: 0 / 2 run-scan (other values: NOF_EINVAL)
        fs.scatter_kernel = int(os.environ["SK"])
    if os.environ.get("BWDF"):   # MLP backward weight-gradient flush: 1 per wave, 2 block-reduced (0: by batch size)
        fs.bwd_flush = int(os.environ["BWDF"])
    if os.environ.get("SLOTS"):   # k_scatter LDS row-table slots per wave (0: the library's choice)
        fs.scatter_slots = int(os.environ["SLOTS"])
    if os.environ.get("EG"):   # k_encode levels in flight per lane (0: the library's choice by batch size)
        fs.encode_group = int(os.environ["EG"])
    if os.environ.get("PER_FRAME") == "1":
        step = lambda: fs.graph_step(32)   # noqa: E731  64 frames x 32 rays = 2048 rays per step
    else:   # NerfRunner.train(): N_rand = 2048 ids of the epoch randperm over the pool (bench parity_mode)
        from bundlesdf_amd.nerf_runner import DataLoader
        torch.manual_seed(0)
        dl = DataLoader(pool, cfg["N_rand"])
        step = lambda: fs.graph_step_epoch(*dl.next_slice(), cfg["N_rand"])   # noqa: E731
    P0 = fs.P.detach().clone()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    fs.reset_state(P0)     # the timed steps: a round from initialisation, as bench.py
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for _ in range(n):
        step()
    t1.record()
    torch.cuda.synchronize()
    print(f"small batch: {t0.elapsed_time(t1) / n:.4f} ms/step (2048 rays, graph replay), "
          f"scatter levels per wave {os.environ.get('LPW', 'default')}, slots {os.environ.get('SLOTS', 'default')}, "
          f"ablate {os.environ.get('ABLATE', '0')}, bwd_flush {os.environ.get('BWDF', 'default')}, scatter_kernel {os.environ.get('SK', 'default')}, "
          f"encode_group {os.environ.get('EG', 'default')}")


if __name__ == "__main__":
    main()
