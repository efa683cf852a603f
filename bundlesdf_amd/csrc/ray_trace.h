// Dense-occupancy 3-D DDA ray trace shared by the boundary kernel
// (nof_octree_ray_trace) and the fused training step (field_step.hip).
// Replaces kaolin's SPC unbatched_raytrace (Utils.py:457) + the packing of
// common.cu:128-149.
#pragma once
#include "nof_device.h"

#pragma clang fp contract(off)

namespace nof {

// --- dense-occupancy ray trace (replaces kaolin unbatched_raytrace) --------
__device__ __forceinline__ void slab(float o, float inv, bool par, float lo, float hi, float &tn, float &tf) {
    if (par) {
        const bool in = (o >= lo && o <= hi);
        tn = in ? -INFINITY : INFINITY;
        tf = in ? INFINITY : -INFINITY;
        return;
    }
    const float a = (lo - o) * inv, b = (hi - o) * inv;
    tn = a < b ? a : b;
    tf = a < b ? b : a;
}

// One lane per ray: 3-D DDA over the N^3 grid on [-1,1]^3; for each occupied
// voxel the per-voxel slab test gives [t_in, t_out] (distance along the unit
// world direction), filtered like common.cu:140-142. Same float operation
// order as oracle/ray_oracle.c (contraction off) -> identical intervals.
// emit(k, tin, tout) receives each kept interval (k = its index < Kmax).
template <typename Emit>
__device__ __forceinline__ int trace_ray_emit(const uint8_t *__restrict__ occ, int N, const float o[3], const float d[3],
                                              int Kmax, Emit emit) {
    const float vs = 2.0f / (float)N;
    float inv[3];
    bool par[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) { par[a] = (d[a] == 0.0f); inv[a] = par[a] ? 0.0f : 1.0f / d[a]; }
    float t0 = -INFINITY, t1 = INFINITY;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        float tn, tf;
        slab(o[a], inv[a], par[a], -1.0f, 1.0f, tn, tf);
        t0 = tn > t0 ? tn : t0;
        t1 = tf < t1 ? tf : t1;
    }
    if (t0 < 0.0f) t0 = 0.0f;
    int k = 0;
    if (!(t1 > t0)) return 0;
    int idx[3], step[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float p = o[a] + d[a] * t0;
        int i = (int)floorf((p + 1.0f) / vs);
        i = i < 0 ? 0 : (i > N - 1 ? N - 1 : i);
        idx[a] = i;
        step[a] = par[a] ? 0 : (d[a] > 0 ? 1 : -1);
    }
    for (int it = 0; it < 3 * N + 3; ++it) {
        float tin = -INFINITY, tout = INFINITY, nextt = INFINITY;
        int nexta = -1;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            const float lo = -1.0f + (float)idx[a] * vs, hi = -1.0f + (float)(idx[a] + 1) * vs;
            float tn, tf;
            slab(o[a], inv[a], par[a], lo, hi, tn, tf);
            tin = tn > tin ? tn : tin;
            tout = tf < tout ? tf : tout;
            if (!par[a] && tf < nextt) { nextt = tf; nexta = a; }
        }
        if (occ[((size_t)idx[2] * N + idx[1]) * N + idx[0]]) {
            if (tin == 0.0f || tout == 0.0f) break;
            if (!(tin > tout) && !(fabsf(tout - tin) < 1e-4f) && k < Kmax) {
                emit(k, tin, tout);
                k++;
            }
        }
        if (nexta < 0) break;
        idx[nexta] += step[nexta];
        if (idx[nexta] < 0 || idx[nexta] >= N) break;
    }
    return k;
}

__device__ __forceinline__ int trace_ray(const uint8_t *__restrict__ occ, int N, const float o[3], const float d[3], int Kmax,
                                         float *__restrict__ out) {
    return trace_ray_emit(occ, N, o, d, Kmax, [&](int k, float tin, float tout) {
        out[k * 2] = tin;
        out[k * 2 + 1] = tout;
    });
}

}  // namespace nof
