/*
 * ORACLE — test infrastructure only. CPU restatement of the reference's ray
 * sampling kernels (mycuda/common.cu) and of the kaolin-SPC ray trace that
 * Utils.py:443-475 wraps. Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library.
 *
 * Parity status:
 *  - sampler / postprocess: restated from common.cu:40-105 / :128-149; pinned by
 *    the known-answer vectors recorded in SURVEY.md §8c (G2) and by the golden
 *    fixtures in tests/golden/ (CUDA source itself is unbuildable here).
 *  - octree ray trace: kaolin is not vendored (third-party, unpinned master at
 *    docker/dockerfile:84,94-96) and not installed -> PARITY UNPINNED. The
 *    restatement enumerates occupied voxels of a dense occupancy grid at `level`
 *    front-to-back (3-D DDA) and emits per-voxel slab-test [t_in, t_out], then
 *    applies the common.cu:140-142 filters — the semantics Utils.py:457-470
 *    documents.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>

/* sample_rays_uniform_occupied_voxels_kernel, common.cu:40-105. The reference
 * prints and spins forever on malformed input (:66-71, :87-92); this
 * restatement leaves z unchanged and counts the error instead. */
int oracle_sample_occupied(const float *z_in_out, const float *z_sampled, float *z_vals,
                           int N_rays, int K, int S) {
    int errors = 0;
    const float eps = 1e-4f;
    for (int r = 0; r < N_rays; ++r) {
        const float *box = z_in_out + (size_t)r * K * 2;
        for (int s = 0; s < S; ++s) {
            float z_remain = z_sampled[(size_t)r * S + s];
            float *out = z_vals + (size_t)r * S + s;
            if (box[0] == 0) continue;                                   /* :54 */
            int i = 0;
            for (;;) {
                if (i >= K) {                                            /* :58-76 */
                    if (z_remain <= eps) *out = box[(K - 1) * 2 + 1]; else errors++;
                    break;
                }
                if (box[i * 2] == 0) {                                   /* :78-94 */
                    if (z_remain <= eps && i >= 1) *out = box[(i - 1) * 2 + 1]; else errors++;
                    break;
                }
                float len = box[i * 2 + 1] - box[i * 2];                 /* :96-103 */
                if (z_remain <= len) { *out = box[i * 2] + z_remain; break; }
                z_remain -= len;
                i++;
            }
        }
    }
    return errors;
}

/* postprocessOctreeRayTracingKernel, common.cu:128-149 (+ host :151-167).
 * `out` is [N_rays, max_int, 2], zero-initialised by the caller (:158). */
void oracle_postprocess_octree(const int64_t *ray_index, const float *depth_in_out,
                               const int64_t *unique_ids, const int64_t *start_poss,
                               int64_t M, int64_t U, int max_int, float *out) {
    for (int64_t u = 0; u < U; ++u) {
        const int64_t r = unique_ids[u];
        int k = 0;
        for (int64_t i = start_poss[u]; i < M; i++) {
            if (ray_index[i] != r) break;
            float a = depth_in_out[i * 2], b = depth_in_out[i * 2 + 1];
            if (a == 0 || b == 0) break;
            if (a > b) continue;
            if (fabsf(b - a) < 1e-4f) continue;
            out[((size_t)r * max_int + k) * 2] = a;
            out[((size_t)r * max_int + k) * 2 + 1] = b;
            k++;
        }
    }
}

/* Slab test of the axis-aligned box [lo, hi] (one axis). Parallel rays (d==0)
 * get (-inf, +inf) when inside the slab and an empty span otherwise. */
static void slab(float o, float inv, int parallel, float lo, float hi, float *tn, float *tf) {
    if (parallel) {
        if (o >= lo && o <= hi) { *tn = -INFINITY; *tf = INFINITY; }
        else { *tn = INFINITY; *tf = -INFINITY; }
        return;
    }
    float a = (lo - o) * inv, b = (hi - o) * inv;
    *tn = a < b ? a : b;
    *tf = a < b ? b : a;
}

/* Dense-grid restatement of kaolin.render.spc.unbatched_raytrace(level,
 * return_depth, with_exit) followed by postprocessOctreeRayTracing: returns,
 * per ray, the front-to-back [t_in, t_out] of occupied voxels of the N^3 grid
 * over [-1,1]^3, dropping reversed or < 1e-4 intervals. `out` [R, Kmax, 2]
 * must be zeroed by the caller; `counts` [R] receives the hit count. */
void oracle_octree_ray_trace(const uint8_t *occ, int N, const float *rays_o, const float *rays_d,
                             int R, int Kmax, float *out, int *counts) {
    const float vs = 2.0f / (float)N;
    for (int r = 0; r < R; ++r) {
        const float *o = rays_o + (size_t)r * 3, *d = rays_d + (size_t)r * 3;
        float inv[3]; int par[3];
        for (int a = 0; a < 3; ++a) { par[a] = (d[a] == 0.0f); inv[a] = par[a] ? 0.0f : 1.0f / d[a]; }
        float t0 = -INFINITY, t1 = INFINITY;
        for (int a = 0; a < 3; ++a) {
            float tn, tf; slab(o[a], inv[a], par[a], -1.0f, 1.0f, &tn, &tf);
            if (tn > t0) t0 = tn;
            if (tf < t1) t1 = tf;
        }
        int k = 0;
        if (t0 < 0.0f) t0 = 0.0f;
        if (t1 > t0) {
            const float tm = t0;                          /* entry point */
            int idx[3], step[3];
            for (int a = 0; a < 3; ++a) {
                float p = o[a] + d[a] * tm;
                int i = (int)floorf((p + 1.0f) / vs);
                if (i < 0) i = 0;
                if (i > N - 1) i = N - 1;
                idx[a] = i;
                step[a] = par[a] ? 0 : (d[a] > 0 ? 1 : -1);
            }
            for (int it = 0; it < 3 * N + 3; ++it) {
                float tin = -INFINITY, tout = INFINITY;
                int nexta = -1; float nextt = INFINITY;
                for (int a = 0; a < 3; ++a) {
                    float lo = -1.0f + (float)idx[a] * vs, hi = -1.0f + (float)(idx[a] + 1) * vs;
                    float tn, tf; slab(o[a], inv[a], par[a], lo, hi, &tn, &tf);
                    if (tn > tin) tin = tn;
                    if (tf < tout) tout = tf;
                    if (!par[a] && tf < nextt) { nextt = tf; nexta = a; }
                }
                if (occ[((size_t)idx[2] * N + idx[1]) * N + idx[0]]) {
                    if (tin == 0.0f || tout == 0.0f) break;
                    if (!(tin > tout) && !(fabsf(tout - tin) < 1e-4f) && k < Kmax) {
                        out[((size_t)r * Kmax + k) * 2] = tin;
                        out[((size_t)r * Kmax + k) * 2 + 1] = tout;
                        k++;
                    }
                }
                if (nexta < 0) break;
                idx[nexta] += step[nexta];
                if (idx[nexta] < 0 || idx[nexta] >= N) break;
            }
        }
        counts[r] = k;
    }
}
