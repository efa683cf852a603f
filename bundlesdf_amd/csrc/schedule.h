// Per-step schedule (nof_step_schedule, include/nof.h): the step block of the device step counter
// *step (get_truncation nerf_runner.py:661-674, schedule_lr :577-581 applied every 10 steps
// :761-762, the sampling seeds), then *step advances. One thread; shared by k_step_schedule
// (optim.hip) and the merged step prologue (pose.hip).
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

#include "nof_device.h"

namespace nof {
__device__ __forceinline__ void step_schedule_one(const nof_schedule_desc &d, int32_t *step, nof_step_params *out) {
    const int32_t gs = *step;
    nof_step_params p;
    const double n_iters = (double)d.n_step + 1.0;
    if (gs <= 10) {
        p.lr0 = d.lrate;
        p.lr1 = d.lrate_pose;
    } else {
        const double last = 10.0 * (double)((gs - 1) / 10);
        const double f = pow(d.decay_rate, last / n_iters);
        p.lr0 = d.lrate * f;
        p.lr1 = d.lrate_pose * f;
    }
    double t = d.trunc;
    if (d.trunc_decay == 1) {
        t = d.trunc_start - (d.trunc_start - d.trunc) * (double)gs / (double)d.n_step;
    } else if (d.trunc_decay == 2) {
        const double lamb = log(d.trunc / d.trunc_start) / ((double)d.n_step / 4.0);
        t = fmax(d.trunc_start * exp((double)gs * lamb), d.trunc);
    }
    p.trunc = (float)(t * d.sc_factor);
    p.seed = (uint32_t)gs * 0x9E3779B1u + d.seed_base;
    p.batch_seed = d.batch_seed_base + (uint32_t)gs;
    p.step = gs;
    *out = p;
    *step = gs + 1;
}
}  // namespace nof
