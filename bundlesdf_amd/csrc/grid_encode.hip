// Multires dense/hash grid encoder — drop-in kernels behind
// gridencoder.grid_encode_forward / grid_encode_backward
// (reference: mycuda/torch_ngp_grid_encoder/gridencoder.cu:106-502).
//
// Layout contract (kept from the reference so grid.py's permutes still work):
//   inputs [B,D] f32 in [0,1], embeddings [sO,C], offsets [L+1] i32,
//   outputs [L,B,C] (level-major: one level's table is hot in L2 at a time),
//   dy_dx [B, L*D*C], grad [L,B,C], grad_inputs [B,D].
//
// CDNA4 notes: one lane per (sample, level); blockIdx.y = level so all waves
// of a dispatch window hit one level table (the L=16 table is 26-52 MB and
// stays resident in the 256 MB Infinity Cache; the per-level slab is what the
// 4 MB per-XCD L2 sees). Corner rows (C channels) are fetched as one vector
// load. Float32 arithmetic reproduces nvcc's contraction of the reference
// expressions with explicit fmaf, and everything else with contraction OFF,
// so the fp32 forward is bit-identical to oracle/grid_oracle.c.
#include "nof_device.h"

#pragma clang fp contract(off)

namespace nof {

template <typename T, uint32_t C> struct Row;
template <uint32_t C> struct Row<float, C> {
    __device__ static void load(const float *p, float (&v)[C]) {
        if constexpr (C == 2) { float2 t = *reinterpret_cast<const float2 *>(p); v[0] = t.x; v[1] = t.y; }
        else if constexpr (C == 4) { float4 t = *reinterpret_cast<const float4 *>(p); v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w; }
        else {
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) v[c] = p[c];
        }
    }
};
template <uint32_t C> struct Row<__half, C> {
    __device__ static void load(const __half *p, float (&v)[C]) {
        if constexpr (C % 2 == 0) {
#pragma unroll
            for (uint32_t c = 0; c < C; c += 2) {
                __half2 t = *reinterpret_cast<const __half2 *>(p + c);
                v[c] = __low2float(t); v[c + 1] = __high2float(t);
            }
        } else {
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) v[c] = __half2float(p[c]);
        }
    }
};

// kernel_grid (gridencoder.cu:106-246).
template <typename T, uint32_t D, uint32_t C>
__global__ __launch_bounds__(256) void k_grid_fwd(const float *__restrict__ inputs, const T *__restrict__ grid,
                                                  const int32_t *__restrict__ offsets, T *__restrict__ outputs,
                                                  uint32_t B, uint32_t L, LevelParams lp, int calc_grad_inputs,
                                                  T *__restrict__ dy_dx, uint32_t gridtype, int align_corners) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint32_t level = blockIdx.y;
    const uint32_t off = (uint32_t)offsets[level];
    const uint32_t hashmap_size = (uint32_t)offsets[level + 1] - off;
    grid += (size_t)off * C;
    T *out = outputs + (size_t)level * B * C + (size_t)b * C;

    float x[D];
    bool oob = false;
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        x[d] = inputs[(size_t)b * D + d];
        if (x[d] < 0 || x[d] > 1) oob = true;
    }
    if (oob) {
#pragma unroll
        for (uint32_t ch = 0; ch < C; ch++) Scalar<T>::store(out + ch, 0.f);
        if (calc_grad_inputs) {
            T *dd = dy_dx + (size_t)b * D * L * C + (size_t)level * D * C;
#pragma unroll
            for (uint32_t k = 0; k < D * C; k++) Scalar<T>::store(dd + k, 0.f);
        }
        return;
    }

    const float scale = lp.scale[level];
    const uint32_t resolution = lp.res[level];
    float pos[D];
    uint32_t pg[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        pos[d] = __builtin_fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
    }

    float acc[C];
#pragma unroll
    for (uint32_t c = 0; c < C; ++c) acc[c] = 0.f;
#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); idx++) {
        float w = 1.f;
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; d++) {
            if ((idx & (1u << d)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
            else { w *= pos[d]; pl[d] = pg[d] + 1; }
        }
        const uint32_t row = grid_row<D>(gridtype, align_corners, hashmap_size, resolution, pl);
        float v[C];
        Row<T, C>::load(grid + (size_t)row * C, v);
#pragma unroll
        for (uint32_t ch = 0; ch < C; ch++) {
            if constexpr (sizeof(T) == 2) acc[ch] = hround(acc[ch] + hround(w * v[ch]));  // c10::Half +=
            else acc[ch] = __builtin_fmaf(w, v[ch], acc[ch]);
        }
    }
#pragma unroll
    for (uint32_t ch = 0; ch < C; ch++) Scalar<T>::store(out + ch, acc[ch]);

    if (calc_grad_inputs) {
        T *dd = dy_dx + (size_t)b * D * L * C + (size_t)level * D * C;
#pragma unroll
        for (uint32_t gd = 0; gd < D; gd++) {
            float rg[C];
#pragma unroll
            for (uint32_t c = 0; c < C; ++c) rg[c] = 0.f;
#pragma unroll
            for (uint32_t idx = 0; idx < (1u << (D - 1)); idx++) {
                float w = scale;
                uint32_t pl[D];
#pragma unroll
                for (uint32_t nd = 0; nd < D - 1; nd++) {
                    const uint32_t d = (nd >= gd) ? (nd + 1) : nd;
                    if ((idx & (1u << nd)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
                    else { w *= pos[d]; pl[d] = pg[d] + 1; }
                }
                pl[gd] = pg[gd];
                const uint32_t rl = grid_row<D>(gridtype, align_corners, hashmap_size, resolution, pl);
                pl[gd] = pg[gd] + 1;
                const uint32_t rr = grid_row<D>(gridtype, align_corners, hashmap_size, resolution, pl);
                float vl[C], vr[C];
                Row<T, C>::load(grid + (size_t)rl * C, vl);
                Row<T, C>::load(grid + (size_t)rr * C, vr);
#pragma unroll
                for (uint32_t ch = 0; ch < C; ch++) {
                    if constexpr (sizeof(T) == 2) rg[ch] = hround(rg[ch] + hround(w * hround(vr[ch] - vl[ch])));
                    else rg[ch] = __builtin_fmaf(w, vr[ch] - vl[ch], rg[ch]);
                }
            }
#pragma unroll
            for (uint32_t ch = 0; ch < C; ch++) Scalar<T>::store(dd + gd * C + ch, rg[ch]);
        }
    }
}

// kernel_grid_backward (gridencoder.cu:249-336): one lane per (sample, level)
// scatters w * grad into the 2^D corners. fp32 -> global_atomic_add_f32;
// fp16 -> global_atomic_pk_add_f16 on channel pairs (the reference's __half2
// path, :319-327). Lanes of one wave hold consecutive samples, which along a
// ray share corners; the memory-side atomic unit merges each instruction's
// lanes per 64-B line.
template <typename T, uint32_t D, uint32_t C>
__global__ __launch_bounds__(256) void k_grid_bwd(const T *__restrict__ grad, const float *__restrict__ inputs,
                                                  const int32_t *__restrict__ offsets, T *__restrict__ grad_grid,
                                                  uint32_t B, LevelParams lp, uint32_t gridtype, int align_corners) {
    const uint32_t b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    const uint32_t level = blockIdx.y;
    const uint32_t off = (uint32_t)offsets[level];
    const uint32_t hashmap_size = (uint32_t)offsets[level + 1] - off;
    grad_grid += (size_t)off * C;

    float x[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        x[d] = inputs[(size_t)b * D + d];
        if (x[d] < 0 || x[d] > 1) return;  // grad is zero-initialised (:276-281)
    }
    const float scale = lp.scale[level];
    const uint32_t resolution = lp.res[level];
    float pos[D];
    uint32_t pg[D];
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        pos[d] = __builtin_fmaf(x[d], scale, align_corners ? 0.0f : 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
    }
    float g[C];
#pragma unroll
    for (uint32_t c = 0; c < C; c++) g[c] = Scalar<T>::load(grad + (size_t)level * B * C + (size_t)b * C + c);

#pragma unroll
    for (uint32_t idx = 0; idx < (1u << D); idx++) {
        float w = 1.f;
        uint32_t pl[D];
#pragma unroll
        for (uint32_t d = 0; d < D; d++) {
            if ((idx & (1u << d)) == 0) { w *= 1 - pos[d]; pl[d] = pg[d]; }
            else { w *= pos[d]; pl[d] = pg[d] + 1; }
        }
        const uint32_t row = grid_row<D>(gridtype, align_corners, hashmap_size, resolution, pl);
        T *dst = grad_grid + (size_t)row * C;
        if constexpr (sizeof(T) == 2) {
            if constexpr (C % 2 == 0) {
#pragma unroll
                for (uint32_t c = 0; c < C; c += 2) atomic_add_h2(dst + c, w * g[c], w * g[c + 1]);
            } else {
                unsafeAtomicAdd(dst, __float2half_rn(w * g[0]));
            }
        } else {
#pragma unroll
            for (uint32_t c = 0; c < C; c++) atomic_add_f32(dst + c, w * g[c]);
        }
    }
}

// kernel_input_backward (gridencoder.cu:339-365).
template <typename T, uint32_t D, uint32_t C>
__global__ __launch_bounds__(256) void k_input_bwd(const T *__restrict__ grad, const T *__restrict__ dy_dx,
                                                   T *__restrict__ grad_inputs, uint32_t B, uint32_t L) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= B * D) return;
    const uint32_t b = t / D, d = t - b * D;
    const T *dd = dy_dx + (size_t)b * L * D * C;
    float r = 0.f;
    for (uint32_t l = 0; l < L; l++) {
#pragma unroll
        for (uint32_t ch = 0; ch < C; ch++) {
            const float gv = Scalar<T>::load(grad + (size_t)l * B * C + (size_t)b * C + ch);
            const float dv = Scalar<T>::load(dd + l * D * C + d * C + ch);
            if constexpr (sizeof(T) == 2) r = hround(r + hround(gv * dv));
            else r = __builtin_fmaf(gv, dv, r);
        }
    }
    Scalar<T>::store(grad_inputs + t, r);
}

template <typename T, uint32_t D, uint32_t C>
static int launch_fwd(const float *inputs, const void *emb, const int32_t *offsets, void *outputs, uint32_t B,
                      uint32_t L, const LevelParams &lp, int cgi, void *dy_dx, uint32_t gridtype, int ac,
                      hipStream_t st) {
    dim3 grid(div_up(B, 256), L);
    hipLaunchKernelGGL((k_grid_fwd<T, D, C>), grid, dim3(256), 0, st, inputs, (const T *)emb, offsets, (T *)outputs,
                       B, L, lp, cgi, (T *)dy_dx, gridtype, ac);
    return check_launch("grid_encode_forward");
}

template <typename T, uint32_t D, uint32_t C>
static int launch_bwd(const void *grad, const float *inputs, const int32_t *offsets, void *gemb, uint32_t B,
                      uint32_t L, const LevelParams &lp, int cgi, const void *dy_dx, void *gin, uint32_t gridtype,
                      int ac, hipStream_t st) {
    dim3 grid(div_up(B, 256), L);
    hipLaunchKernelGGL((k_grid_bwd<T, D, C>), grid, dim3(256), 0, st, (const T *)grad, inputs, offsets, (T *)gemb, B,
                       lp, gridtype, ac);
    int rc = check_launch("grid_encode_backward");
    if (rc || !cgi) return rc;
    hipLaunchKernelGGL((k_input_bwd<T, D, C>), dim3(div_up((uint64_t)B * D, 256)), dim3(256), 0, st,
                       (const T *)grad, (const T *)dy_dx, (T *)gin, B, L);
    return check_launch("grid_encode_backward(input)");
}

template <typename T, uint32_t D>
static int dispatch_c_fwd(uint32_t C, const float *in, const void *e, const int32_t *o, void *out, uint32_t B,
                          uint32_t L, const LevelParams &lp, int cgi, void *dd, uint32_t gt, int ac, hipStream_t st) {
    switch (C) {
        case 1: return launch_fwd<T, D, 1>(in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
        case 2: return launch_fwd<T, D, 2>(in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
        case 4: return launch_fwd<T, D, 4>(in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
        case 8: return launch_fwd<T, D, 8>(in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
    }
    return set_error(NOF_EINVAL, "GridEncoding: C must be 1, 2, 4, or 8.");
}

template <typename T, uint32_t D>
static int dispatch_c_bwd(uint32_t C, const void *g, const float *in, const int32_t *o, void *ge, uint32_t B,
                          uint32_t L, const LevelParams &lp, int cgi, const void *dd, void *gi, uint32_t gt, int ac,
                          hipStream_t st) {
    switch (C) {
        case 1: return launch_bwd<T, D, 1>(g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
        case 2: return launch_bwd<T, D, 2>(g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
        case 4: return launch_bwd<T, D, 4>(g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
        case 8: return launch_bwd<T, D, 8>(g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
    }
    return set_error(NOF_EINVAL, "GridEncoding: C must be 1, 2, 4, or 8.");
}

template <typename T>
static int dispatch_fwd(uint32_t D, uint32_t C, const float *in, const void *e, const int32_t *o, void *out,
                        uint32_t B, uint32_t L, const LevelParams &lp, int cgi, void *dd, uint32_t gt, int ac,
                        hipStream_t st) {
    switch (D) {
        case 1: return dispatch_c_fwd<T, 1>(C, in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
        case 2: return dispatch_c_fwd<T, 2>(C, in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
        case 3: return dispatch_c_fwd<T, 3>(C, in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
        case 4: return dispatch_c_fwd<T, 4>(C, in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
        case 5: return dispatch_c_fwd<T, 5>(C, in, e, o, out, B, L, lp, cgi, dd, gt, ac, st);
    }
    return set_error(NOF_EINVAL, "GridEncoding: D must be 1, 2, 3, 4, or 5.");
}

template <typename T>
static int dispatch_bwd(uint32_t D, uint32_t C, const void *g, const float *in, const int32_t *o, void *ge,
                        uint32_t B, uint32_t L, const LevelParams &lp, int cgi, const void *dd, void *gi, uint32_t gt,
                        int ac, hipStream_t st) {
    switch (D) {
        case 1: return dispatch_c_bwd<T, 1>(C, g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
        case 2: return dispatch_c_bwd<T, 2>(C, g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
        case 3: return dispatch_c_bwd<T, 3>(C, g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
        case 4: return dispatch_c_bwd<T, 4>(C, g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
        case 5: return dispatch_c_bwd<T, 5>(C, g, in, o, ge, B, L, lp, cgi, dd, gi, gt, ac, st);
    }
    return set_error(NOF_EINVAL, "GridEncoding: D must be 1, 2, 3, 4, or 5.");
}

}  // namespace nof

extern "C" int nof_grid_encode_forward(const float *inputs, const void *embeddings, const int32_t *offsets,
                                       void *outputs, uint32_t B, uint32_t D, uint32_t C, uint32_t L, float S,
                                       uint32_t H, int calc_grad_inputs, void *dy_dx, uint32_t gridtype,
                                       int align_corners, int dtype, void *stream) {
    if (L == 0 || L > NOF_MAX_LEVELS) return nof::set_error(NOF_EINVAL, "grid_encode_forward: L=%u out of range", L);
    if (B == 0) return NOF_OK;
    nof::LevelParams lp;
    nof::level_params(L, S, H, lp);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == NOF_F32)
        return nof::dispatch_fwd<float>(D, C, inputs, embeddings, offsets, outputs, B, L, lp, calc_grad_inputs, dy_dx,
                                        gridtype, align_corners, st);
    if (dtype == NOF_F16)
        return nof::dispatch_fwd<__half>(D, C, inputs, embeddings, offsets, outputs, B, L, lp, calc_grad_inputs, dy_dx,
                                         gridtype, align_corners, st);
    return nof::set_error(NOF_EINVAL, "grid_encode_forward: unsupported dtype %d", dtype);
}

extern "C" int nof_grid_encode_backward(const void *grad, const float *inputs, const void *embeddings,
                                        const int32_t *offsets, void *grad_embeddings, uint32_t B, uint32_t D,
                                        uint32_t C, uint32_t L, float S, uint32_t H, int calc_grad_inputs,
                                        const void *dy_dx, void *grad_inputs, uint32_t gridtype, int align_corners,
                                        int dtype, void *stream) {
    (void)embeddings;  // the reference passes it but only reads positions (gridencoder.cu:249-336)
    if (L == 0 || L > NOF_MAX_LEVELS) return nof::set_error(NOF_EINVAL, "grid_encode_backward: L=%u out of range", L);
    if (B == 0) return NOF_OK;
    nof::LevelParams lp;
    nof::level_params(L, S, H, lp);
    hipStream_t st = (hipStream_t)stream;
    if (dtype == NOF_F32)
        return nof::dispatch_bwd<float>(D, C, grad, inputs, offsets, grad_embeddings, B, L, lp, calc_grad_inputs,
                                        dy_dx, grad_inputs, gridtype, align_corners, st);
    if (dtype == NOF_F16)
        return nof::dispatch_bwd<__half>(D, C, grad, inputs, offsets, grad_embeddings, B, L, lp, calc_grad_inputs,
                                         dy_dx, grad_inputs, gridtype, align_corners, st);
    return nof::set_error(NOF_EINVAL, "grid_encode_backward: unsupported dtype %d", dtype);
}
