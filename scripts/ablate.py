"""Timing ablation of nof_field_step on the bench workload (diagnostic only:
ablated runs compute wrong results). Prints one JSON line per variant with the
median field-kernel time (HIP events) over interleaved rounds."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402

ONLY = os.environ.get("ONLY")
# timing-build ablation bits (field_step.hip ABL(); results invalid when set)
MASKS = {"full": 0, "no_scatter_table": 1, "esig_no_rec": 2, "no_encode_gather": 8, "esig_sync_staging": 16,
         "no_backward_level": 32, "esig_no_barrier": 64, "flush_no_hbm": 128, "esig_no_sigma_mfma": 256,
         "esig_no_barrier_no_mfma": 64 | 256, "enc_no_quads": 512, "f32_scan": 4096, "no_counters": 16384,
         "esig_no_handoff": 32768, "esig_no_rec_no_handoff": 2 | 32768, "sc_ret0": 65536, "sc_ret_flags": 131072,
         "sc_ret_init": 262144, "no_dw_atomics": 1 << 21, "no_flush": 1 << 22, "util_probe": 1 << 25,
         "dpp_no_claims": 1 << 26, "head_probe": 1 << 27, "dpp_no_claims_no_flush": (1 << 26) | (1 << 22),
         # the scatter's per-level-group split: levels 4q .. 4q+3 skipped (ABL_SKIPQ)
         "skip_lv0_3": 1 << 23, "skip_lv4_7": 1 << 24, "skip_lv8_11": 1 << 29, "skip_lv12_15": 1 << 30,
         "skip_all_levels": (1 << 23) | (1 << 24) | (1 << 29) | (1 << 30),
         # the encode's fixed costs: launch + staging only, the sampler only, the sampler's walk twice
         "enc_ret_start": 1 << 19, "enc_ret_sampler": 8192, "enc_double_walk": 4}


def main():
    dev = torch.device("cuda", 0)
    frames = int(os.environ.get("FRAMES", "16"))   # 16: config 2; 64: the headline pool
    # OPT_POSES=0: cfg optimize_poses = 0 (frozen poses: no input gradient)
    cfg, pool, frame_start, c2w, occ, _, _ = bench.build_rank_scene(
        0, 1, frames, dict(amp=True, optimize_poses=int(os.environ.get("OPT_POSES", "1"))), dev)
    enc, net, pa = bench.make_models(cfg, frames, dev)
    bpc = int(os.environ.get("BPC", "0"))
    fs = FusedStep(cfg, pool, torch.from_numpy(c2w), occ, enc, net, pa, amp=True,
                   frame_start=frame_start, blocks_per_cu=bpc, time_kernels=True)
    if os.environ.get("USE_QUADS"):   # 0: the encode's pair loads instead of the xy-quad mirror
        fs.use_quads = os.environ["USE_QUADS"] != "0"
    if os.environ.get("LPW"):   # k_scatter levels per wave (0: the library's choice by batch size)
        fs.scatter_levels_per_wave = int(os.environ["LPW"])
    if os.environ.get("SK"):   # scatter kernel: 0 / 2 run-scan (other values: NOF_EINVAL)
        fs.scatter_kernel = int(os.environ["SK"])
    if os.environ.get("BWDF"):   # MLP backward weight-gradient flush: 1 per wave, 2 block-reduced
        fs.bwd_flush = int(os.environ["BWDF"])
    if "XCD" in os.environ:   # xcd_order bits (bit 0: k_encode, bit 1: k_scatter)
        fs.xcd_order = int(os.environ["XCD"])
    for it in range(int(os.environ.get("WARM", "40"))):
        fs.step(ids=fs.sample_ids(2048, it))
    torch.cuda.synchronize()
    fs.field_kernel_breakdown()
    fs.wait_exchange()   # emb16 may be an all-gather target still in flight (N > 1)
    P0, M0, V0, E0 = fs.P.clone(), fs.M.clone(), fs.V.clone(), fs.emb16.clone()
    if ONLY:
        for k in list(MASKS):
            if k not in ONLY.split(","):
                del MASKS[k]
    res = {k: [] for k in MASKS}
    per = {k: [] for k in MASKS}
    for rnd in range(3):
        for name, m in MASKS.items():
            fs.wait_exchange()
            fs.P.copy_(P0); fs.M.copy_(M0); fs.V.copy_(V0); fs.emb16.copy_(E0)
            fs.ablate = m
            fs.scatter_slots = int(os.environ.get("SLOTS", "0"))
            for it in range(3):
                fs.step(ids=fs.sample_ids(2048, 100 + it))
            torch.cuda.synchronize()
            bd, _ = fs.field_kernel_breakdown()
            if name == "head_probe":
                bd = dict(bd, representatives=float(fs.scatter_atomic_counts()[1]))
            if name == "util_probe":   # flushed rows + active lanes / 64 x busy (level, chunk) iterations
                c = fs.scatter_atomic_counts()
                bd = dict(bd, flush_plus_active_lanes=float(c[0]), busy_iterations=float(c[1]) / 64)
            if name == "full":   # table-flush HBM atomics (distinct rows per ray and level) / probe overflow
                c = fs.scatter_atomic_counts()
                bd = dict(bd, flush_atomics=float(c[0]), overflow_atomics=float(c[1]))
            if name == "grad_probe":   # last step: samples of backward tiles with a non-zero gradient / in the box
                bd = dict(bd, nonzero_grad_samples=float(fs.loss_acc[141].item()),
                          inbox_bwd_tile_samples=float(fs.loss_acc[142].item()))
            per[name].append(bd)
            res[name].append(sum(v for k, v in bd.items() if k.startswith("k_")))
    for name in MASKS:
        print(json.dumps({"variant": name, "mask": MASKS[name], "bpc": bpc, "frames": frames, "lpw": os.environ.get("LPW", "0"), "sk": os.environ.get("SK", "0"), "bwdf": os.environ.get("BWDF", "0"), "quads": os.environ.get("USE_QUADS", "1"),
                          "optimize_poses": int(cfg["optimize_poses"]),
                          "lib": os.path.basename(os.environ.get("NOF_LIB", "libnof.so")), "slots": os.environ.get("SLOTS", "0"),
                          "field_ms_median": round(float(np.median([sum(v for k, v in b.items() if k.startswith("k_")) for b in per[name]])), 3),
                          "field_ms_min": round(float(np.min(res[name])), 3),
                          "kernels": {k: round(float(np.median([b[k] for b in per[name]])), 4) for k in per[name][0]}}),
              flush=True)


if __name__ == "__main__":
    main()
