"""Host-side profile of FusedStep.step (diagnostic): wall time of each libnof /
torch call on the host, no synchronisation, to find calls that block."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bundlesdf_amd import _lib  # noqa: E402
from bundlesdf_amd.fused import FusedStep  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    cfg, pool, frame_start, c2w, occ = bench.build_rank_scene(0, 1, 16, dict(amp=True))
    enc, net, pa = bench.make_models(cfg, 16, dev)
    fs = FusedStep(cfg, torch.from_numpy(pool).to(dev), torch.from_numpy(c2w), occ.to(dev), enc, net, pa, amp=True,
                   frame_start=frame_start)
    L = _lib.lib()
    times = {}
    orig = {}
    for name in ["nof_pose_forward", "nof_trace_rays", "nof_pack_mlp", "nof_field_step", "nof_pose_backward",
                 "nof_unscale_check", "nof_adam_step", "nof_scaler_update", "nof_sample_batch"]:
        f = getattr(L, name)
        orig[name] = f

        def wrap(*a, _f=f, _n=name):
            t = time.perf_counter()
            r = _f(*a)
            times.setdefault(_n, []).append(time.perf_counter() - t)
            return r
        setattr(L, name, wrap)
    for it in range(5):
        fs.step(ids=fs.sample_ids(2048, it))
    torch.cuda.synchronize()
    times.clear()
    t0 = time.perf_counter()
    steps = []
    for it in range(20):
        ts = time.perf_counter()
        fs.step(ids=fs.sample_ids(2048, 100 + it))
        steps.append(time.perf_counter() - ts)
    t_enq = time.perf_counter() - t0
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"enqueue {t_enq / 20 * 1e3:.3f} ms/step, total {dt / 20 * 1e3:.3f} ms/step, "
          f"step host median {np.median(steps) * 1e3:.3f} max {np.max(steps) * 1e3:.3f}")
    for k, v in times.items():
        print(f"  {k:26s} median {np.median(v) * 1e3:8.3f} ms  max {np.max(v) * 1e3:8.3f} ms")


if __name__ == "__main__":
    main()
