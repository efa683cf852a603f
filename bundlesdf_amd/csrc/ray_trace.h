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
    // The voxel walk is pure arithmetic; only the occupancy test reads memory. Voxels are walked in
    // batches of TB: the batch's indices and slab intervals first, then its TB occupancy loads
    // issued together, then the batch's voxels in order (the same tests, breaks and emissions as
    // a one-voxel-at-a-time loop, so the intervals are identical): one dependent load latency per
    // batch instead of per voxel (the trace of a small batch is latency-bound: NerfRunner.train's
    // 2048 rays put 32 waves on the chip)
    constexpr int TB = 8;
    const int n_it = 3 * N + 3;
    int it = 0;
    bool walk = true;
    while (walk) {
        int vi[TB];
        float vin[TB], vout[TB];
        int nv = 0;
#pragma unroll
        for (int b = 0; b < TB; ++b) {
            vi[b] = 0;
            vin[b] = 0.f;
            vout[b] = 0.f;
            if (walk && it < n_it) {
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
                vi[b] = (idx[2] * N + idx[1]) * N + idx[0];
                vin[b] = tin;
                vout[b] = tout;
                nv = b + 1;
                ++it;
                if (nexta < 0) {
                    walk = false;
                } else {
                    const int na = nexta == 0 ? idx[0] + step[0] : (nexta == 1 ? idx[1] + step[1] : idx[2] + step[2]);
                    if (nexta == 0) idx[0] = na;
                    else if (nexta == 1) idx[1] = na;
                    else idx[2] = na;
                    if (na < 0 || na >= N) walk = false;
                }
            }
        }
        if (it >= n_it) walk = false;
        uint8_t oc[TB];
#pragma unroll
        for (int b = 0; b < TB; ++b) oc[b] = b < nv ? occ[(size_t)vi[b]] : (uint8_t)0;
#pragma unroll
        for (int b = 0; b < TB; ++b) {
            if (oc[b]) {
                if (vin[b] == 0.0f || vout[b] == 0.0f) return k;
                if (!(vin[b] > vout[b]) && !(fabsf(vout[b] - vin[b]) < 1e-4f) && k < Kmax) {
                    emit(k, vin[b], vout[b]);
                    k++;
                }
            }
        }
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
