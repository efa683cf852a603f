// Optimiser step over the flat parameter buffer [hash table | MLP | pose]:
// torch.cuda.amp.GradScaler (unscale_, inf check, update: nerf_runner.py:159,
// :757-760) and torch.optim.Adam(betas=(0.9,0.999), eps=1e-15, wd=0) with two
// param groups ('basic', 'pose_array': nerf_runner.py:490-502). One pass
// reads p, g, m, v and writes p, m, v (28 B/param: the dense-Adam roofline),
// zeroes g for the next step and refreshes the fp16 mirror of the table used
// by the amp forward.
#include "nof_device.h"
#include "schedule.h"

#pragma clang fp contract(off)

namespace nof {

// g[f16_lo, f16_hi) are gradients the reference holds in fp16 (under autocast the
// nn.Linear weight / bias gradients are fp16 GEMM results, cast to the fp32 .grad):
// a scaled value beyond the fp16 range (|g| >= 65520 rounds to inf) is an overflow
// there, so the step is skipped exactly when the reference's GradScaler skips it.
__global__ __launch_bounds__(256) void k_unscale_check(float *__restrict__ g, int64_t n,
                                                       const float *__restrict__ scale,
                                                       int32_t *__restrict__ found_inf,
                                                       const __half *__restrict__ g16, int64_t n16, int64_t f16_lo,
                                                       int64_t f16_hi) {
    const float inv = 1.0f / *scale;
    bool bad = false;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        const float raw = g[i];
        const float v = raw * inv;
        g[i] = v;
        bad |= !isfinite(v) || (i >= f16_lo && i < f16_hi && fabsf(raw) >= 65520.0f);
    }
    // the fp16 gradient 8 values (16 B) per lane; a half is inf / nan iff its exponent bits are all set
    const int64_t n8 = (reinterpret_cast<uintptr_t>(g16) & 15) ? 0 : n16 / 8;
    const uint4 *g8 = reinterpret_cast<const uint4 *>(g16);
    uint32_t ex = 0;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
        const uint4 v = g8[i];
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            ex |= ((w[k] & 0x7C00u) == 0x7C00u) ? 1u : 0u;
            ex |= ((w[k] & 0x7C000000u) == 0x7C000000u) ? 1u : 0u;
        }
    }
    bad |= ex != 0;
    const __half *g1 = g16;
    for (int64_t i = 8 * n8 + (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (int64_t)gridDim.x * blockDim.x)
        bad |= !isfinite(__half2float(g1[i]));
    if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(found_inf, 1);
}

// torch.optim.Adam single-tensor update (torch/optim/adam.py _single_tensor_adam):
//   m.lerp_(g, 1-b1); v.mul_(b2).addcmul_(g, g, value=1-b2)
//   denom = sqrt(v) / sqrt(bc2) + eps; p.addcdiv_(m, denom, value=-lr/bc1)
//
// `active` (nullable): one byte per group of ADAM_GROUP consecutive parameters (one wave's
// 64 lanes x 4), set once the group has had a non-zero gradient. A group that never had one
// holds m = v = 0, and Adam then leaves it exactly unchanged (m' = 0, v' = 0, p' = p +
// (-lr) (0 / (0 + eps)) = p; its fp16 mirror already holds half(p)), so its p / m / v are
// neither read nor written — the dense update the reference runs (nerf_runner.py:490-502,
// every table entry every step) at the cost of the gradient read for the untouched part of
// the table (most of the fine levels early in a round, and at small batches all round).
constexpr int ADAM_GROUP = 256;
__global__ __launch_bounds__(256) void k_adam(float *__restrict__ p, float *__restrict__ g, float *__restrict__ m,
                                              float *__restrict__ v, int64_t n, int64_t group1_start, double lr0,
                                              double lr1, float b1, float b2, float eps,
                                              const int32_t *__restrict__ step_count,
                                              const int32_t *__restrict__ found_inf, __half *__restrict__ mirror,
                                              int64_t mirror_n, __half *__restrict__ g16,
                                              const float *__restrict__ scale, const nof_step_params *__restrict__ sp,
                                              uint8_t *__restrict__ active) {
    if (sp) { lr0 = sp->lr0; lr1 = sp->lr1; }
    const float inv = scale ? 1.0f / *scale : 1.0f;
    const bool skip = found_inf && *found_inf;
    // bias corrections exactly as torch computes them on the host (python doubles)
    const double t = (double)(*step_count + 1);
    const double bc1 = 1.0 - pow((double)b1, t), bc2 = 1.0 - pow((double)b2, t);
    const float step0 = (float)(lr0 / bc1), step1 = (float)(lr1 / bc1), bc2s = (float)sqrt(bc2);
    const float w = 1.0f - b1, c2 = 1.0f - b2;
    // one element: torch.optim.Adam single-tensor update (lerp form of exp_avg as torch's _single_tensor_adam)
    auto upd = [&](int64_t i, float gi, float &pi, float &mi, float &vi) {
        mi = (w < 0.5f) ? mi + w * (gi - mi) : gi - (gi - mi) * (1.0f - w);
        vi = vi * b2 + c2 * gi * gi;
        const float denom = sqrtf(vi) / bc2s + eps;
        const float ss = (i < group1_start) ? step0 : step1;
        pi = pi + (-ss) * (mi / denom);
    };
    auto grad_at = [&](int64_t i) {
        float gi;
        if (g16 && i < mirror_n) {
            const __half hv = g16[i];
            gi = __half2float(hv) * inv;
            if (__half_as_ushort(hv) != 0) g16[i] = __float2half_rn(0.f);
        } else {
            gi = g[i];
            g[i] = 0.f;
        }
        return gi;
    };
    // 4 consecutive parameters per lane (16-B loads / stores of p, m, v; 8-B of the fp16
    // gradient and mirror) — the update is HBM-bound at ~30 B/parameter
    const int64_t n4 = n >> 2, tid = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t q = tid; q < n4; q += stride) {
        const int64_t i0 = 4 * q;
        float gi[4];
        if (g16 && i0 + 3 < mirror_n) {
            const uint2 raw = reinterpret_cast<const uint2 *>(g16)[q];
            // cleared for the next step only where it holds something: most table rows get no gradient
            // in a step, and rewriting their zeros was 26 MB of the kernel's HBM writes
            if ((raw.x | raw.y) != 0u) reinterpret_cast<uint2 *>(g16)[q] = make_uint2(0u, 0u);
            const __half2 h0 = *reinterpret_cast<const __half2 *>(&raw.x), h1 = *reinterpret_cast<const __half2 *>(&raw.y);
            gi[0] = __low2float(h0) * inv; gi[1] = __high2float(h0) * inv;
            gi[2] = __low2float(h1) * inv; gi[3] = __high2float(h1) * inv;
        } else if (!g16 || i0 >= mirror_n) {
            const float4 gv = reinterpret_cast<const float4 *>(g)[q];
            reinterpret_cast<float4 *>(g)[q] = make_float4(0.f, 0.f, 0.f, 0.f);
            gi[0] = gv.x; gi[1] = gv.y; gi[2] = gv.z; gi[3] = gv.w;
        } else {
#pragma unroll
            for (int j = 0; j < 4; ++j) gi[j] = grad_at(i0 + j);
        }
        if (skip) continue;
        if (active) {   // a wave's 64 lanes hold one group (q = 64 grp + lane: the stride is a multiple of 64)
            const bool nz = gi[0] != 0.f || gi[1] != 0.f || gi[2] != 0.f || gi[3] != 0.f;
            const int64_t grp = q >> 6;
            const bool any_nz = __any(nz);
            if (!active[grp]) {
                if (!any_nz) continue;          // never touched: exactly unchanged
                if ((threadIdx.x & 63) == 0) active[grp] = 1;
            }
        }
        float4 pv = reinterpret_cast<const float4 *>(p)[q], mv = reinterpret_cast<const float4 *>(m)[q],
               vv = reinterpret_cast<const float4 *>(v)[q];
        upd(i0, gi[0], pv.x, mv.x, vv.x);
        upd(i0 + 1, gi[1], pv.y, mv.y, vv.y);
        upd(i0 + 2, gi[2], pv.z, mv.z, vv.z);
        upd(i0 + 3, gi[3], pv.w, mv.w, vv.w);
        reinterpret_cast<float4 *>(m)[q] = mv;
        reinterpret_cast<float4 *>(v)[q] = vv;
        reinterpret_cast<float4 *>(p)[q] = pv;
        if (mirror && i0 + 3 < mirror_n) {
            const __half2 h0 = __floats2half2_rn(pv.x, pv.y), h1 = __floats2half2_rn(pv.z, pv.w);
            uint2 raw;
            raw.x = *reinterpret_cast<const uint32_t *>(&h0);
            raw.y = *reinterpret_cast<const uint32_t *>(&h1);
            reinterpret_cast<uint2 *>(mirror)[q] = raw;
        } else if (mirror) {
            const float pj[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
            for (int j = 0; j < 4; ++j)
                if (i0 + j < mirror_n) mirror[i0 + j] = __float2half_rn(pj[j]);
        }
    }
    // tail (n not a multiple of 4)
    for (int64_t i = 4 * n4 + tid; i < n; i += stride) {
        const float gi = grad_at(i);
        if (skip) continue;
        float pi = p[i], mi = m[i], vi = v[i];
        upd(i, gi, pi, mi, vi);
        m[i] = mi;
        v[i] = vi;
        p[i] = pi;
        if (mirror && i < mirror_n) mirror[i] = __float2half_rn(pi);
    }
}

// GradScaler.update(): backoff on inf, growth every `interval` clean steps;
// advances Adam's step count unless the step was skipped.
__global__ void k_scaler_update(float *scale, int32_t *tracker, int32_t *found_inf, int32_t *step_count, float growth,
                                float backoff, int32_t interval, int enabled) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    if (!*found_inf) *step_count = *step_count + 1;
    if (!enabled) { *found_inf = 0; return; }
    if (*found_inf) {
        *scale = *scale * backoff;
        *tracker = 0;
    } else {
        const int t = *tracker + 1;
        if (t == interval) { *scale = *scale * growth; *tracker = 0; }
        else *tracker = t;
    }
    *found_inf = 0;
}

__global__ __launch_bounds__(256) void k_to_half(const float *__restrict__ src, __half *__restrict__ dst, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
        dst[i] = __float2half_rn(src[i]);
}

// fp16 table gradient -> fp32 (and cleared) ahead of the data-parallel
// all-reduce, which sums one flat fp32 bucket.
__global__ __launch_bounds__(256) void k_grad16_to_f32(__half *__restrict__ g16, float *__restrict__ g, int64_t n) {
    const int64_t n2 = n >> 1;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2; i += (int64_t)gridDim.x * blockDim.x) {
        const __half2 v = reinterpret_cast<const __half2 *>(g16)[i];
        reinterpret_cast<float2 *>(g)[i] = make_float2(__low2float(v), __high2float(v));
        reinterpret_cast<__half2 *>(g16)[i] = __floats2half2_rn(0.f, 0.f);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0 && (n & 1)) {
        g[n - 1] = __half2float(g16[n - 1]);
        g16[n - 1] = __float2half_rn(0.f);
    }
}

static int grid_for(int64_t n) {
    const int64_t b = (n + 255) / 256;
    return (int)(b < 8192 ? (b > 0 ? b : 1) : 8192);
}

}  // namespace nof

extern "C" int nof_unscale_check(float *grads, int64_t n, const float *scale, int32_t *found_inf, const void *grads16,
                                 int64_t n16, int64_t f16_lo, int64_t f16_hi, void *stream) {
    if (n <= 0 && n16 <= 0) return NOF_OK;
    // at most 4096 blocks: 7.0 / 6.4 / 6.5 / 7.1 us at 6.3 K (one item per lane) / 4096 / 2048 / 1024
    // blocks at the headline (profiles/r4/small_grid_sweep.txt)
    hipLaunchKernelGGL(nof::k_unscale_check, dim3((int)std::min<int64_t>(4096, nof::grid_for(n > n16 / 8 ? n : n16 / 8))), dim3(256), 0,
                       (hipStream_t)stream, grads, n, scale, found_inf, (const __half *)grads16, n16, f16_lo, f16_hi);
    return nof::check_launch("unscale_check");
}

extern "C" size_t nof_adam_active_bytes(int64_t n) { return (size_t)((n / 4 + 63) / 64); }

extern "C" int nof_adam_step(float *params, float *grads, float *exp_avg, float *exp_avg_sq, int64_t n,
                             int64_t group1_start, double lr0, double lr1, float beta1, float beta2, float eps,
                             const int32_t *step_count, const int32_t *found_inf, void *mirror_f16, int64_t mirror_n,
                             void *grads16, const float *scale, const nof_step_params *sp, uint8_t *active,
                             void *stream) {
    if (n <= 0) return NOF_OK;
    auto misaligned = [](const void *q, uintptr_t a) { return q && ((uintptr_t)q & (a - 1)); };
    if (misaligned(params, 16) || misaligned(grads, 16) || misaligned(exp_avg, 16) || misaligned(exp_avg_sq, 16) ||
        misaligned(mirror_f16, 8) || misaligned(grads16, 8))
        return nof::set_error(NOF_EINVAL, "adam_step: params/grads/exp_avg/exp_avg_sq need 16-B and the fp16 "
                                          "buffers 8-B alignment (4 parameters per lane)");
    // at most 4096 blocks (~3 items per lane at the headline's 13 M parameters): the median k_adam
    // time over the headline steps was 44.6 / 38.6 / 41.9 / 41.3 us at 8192 / 4096 / 2048 / 1024
    // blocks (scripts/adam_blocks_sweep.sh, profiles/r4/adam_blocks_sweep.txt)
    const int64_t nb = std::max<int64_t>(1, std::min<int64_t>(((n + 3) / 4 + 255) / 256, 4096));
    hipLaunchKernelGGL(nof::k_adam, dim3((unsigned)nb), dim3(256), 0, (hipStream_t)stream, params, grads, exp_avg,
                       exp_avg_sq, n, group1_start, lr0, lr1, beta1, beta2, eps, step_count, found_inf,
                       (__half *)mirror_f16, mirror_n, (__half *)grads16, scale, sp, active);
    return nof::check_launch("adam_step");
}

extern "C" int nof_scaler_update(float *scale, int32_t *growth_tracker, int32_t *found_inf, int32_t *step_count,
                                 float growth_factor, float backoff_factor, int32_t growth_interval, int enabled,
                                 void *stream) {
    hipLaunchKernelGGL(nof::k_scaler_update, dim3(1), dim3(64), 0, (hipStream_t)stream, scale, growth_tracker,
                       found_inf, step_count, growth_factor, backoff_factor, growth_interval, enabled);
    return nof::check_launch("scaler_update");
}

extern "C" int nof_grad16_to_f32(void *grads16, float *grads, int64_t n, void *stream) {
    if (n <= 0) return NOF_OK;
    if (((uintptr_t)grads16 & 3) || ((uintptr_t)grads & 7))
        return nof::set_error(NOF_EINVAL, "grad16_to_f32: needs 4-B (fp16) / 8-B (fp32) aligned buffers");
    hipLaunchKernelGGL(nof::k_grad16_to_f32, dim3(nof::grid_for((n + 1) / 2)), dim3(256), 0, (hipStream_t)stream,
                       (__half *)grads16, grads, n);
    return nof::check_launch("grad16_to_f32");
}

extern "C" int nof_to_half(const float *src, void *dst, int64_t n, void *stream) {
    if (n <= 0) return NOF_OK;
    hipLaunchKernelGGL(nof::k_to_half, dim3(nof::grid_for(n)), dim3(256), 0, (hipStream_t)stream, src, (__half *)dst, n);
    return nof::check_launch("to_half");
}

// ---------------------------------------------------------- step schedule
// One thread: the step block of *step (host formulas of fused.lr_at / fused.truncation,
// the reference's get_truncation / schedule_lr, in double), then *step += 1.
__global__ void k_step_schedule(nof_schedule_desc d, int32_t *step, nof_step_params *out) {
    if (threadIdx.x == 0) nof::step_schedule_one(d, step, out);
}

extern "C" int nof_step_schedule(const nof_schedule_desc *d, int32_t *step, nof_step_params *out, void *stream) {
    if (!d || !step || !out) return nof::set_error(NOF_EINVAL, "step_schedule: null argument");
    if (d->trunc_decay < 0 || d->trunc_decay > 2 || d->n_step <= 0)
        return nof::set_error(NOF_EINVAL, "step_schedule: trunc_decay %d / n_step %d", d->trunc_decay, d->n_step);
    hipLaunchKernelGGL(k_step_schedule, dim3(1), dim3(64), 0, (hipStream_t)stream, *d, step, out);
    return nof::check_launch("step_schedule");
}
