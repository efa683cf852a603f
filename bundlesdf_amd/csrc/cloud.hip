// Point-cloud operators of the NeRF hand-off: the device
// replacements of open3d's remove_statistical_outlier statistic and
// sklearn's DBSCAN, as used by compute_scene_bounds_worker (tool.py:42-63),
// find_biggest_cluster (tool.py:18-24) and the continual-mode cloud update
// (bundlesdf.py:160-169).
//
//  k_knn_mean_dist   one wave per query point: exact k-th smallest squared
//                    distance by a 63-step radix select over the f64 bit
//                    pattern (each step one coalesced pass over the cloud),
//                    then the mean of the k smallest distances.
//  k_core_count      per point, neighbours within eps from the 27 grid cells
//                    around it (cell edge = eps) -> core flag.
//  k_hook / k_jump   union-find over core-core eps edges: hook the larger
//                    root under the smaller (atomicMin), then full path
//                    compression; the host repeats until no hook happened.
//  k_label           core -> root (= the cluster's lowest core index, where
//                    sklearn starts it); border -> root of its lowest-index
//                    core neighbour; noise -> -1.
#include "nof_device.h"

#pragma clang fp contract(off)

namespace nof {

__global__ __launch_bounds__(256) void k_knn_mean_dist(const double *__restrict__ pts, int32_t n, int32_t k,
                                                       double *__restrict__ out) {
    const int lane = threadIdx.x & 63;
    const int q = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * 4 + (threadIdx.x >> 6)));
    if (q >= n) return;
    const double qx = pts[(size_t)q * 3], qy = pts[(size_t)q * 3 + 1], qz = pts[(size_t)q * 3 + 2];
    auto d2bits = [&](int j) -> uint64_t {
        const double dx = pts[(size_t)j * 3] - qx, dy = pts[(size_t)j * 3 + 1] - qy, dz = pts[(size_t)j * 3 + 2] - qz;
        return __double_as_longlong((dx * dx + dy * dy) + dz * dz);
    };
    const int ke = k < n ? k : n;
    // radix select of the ke-th smallest squared distance (non-negative doubles
    // order like their bit patterns): bit b of the answer is 0 iff at least ke
    // values are <= (prefix with bit b clear and all lower bits set)
    uint64_t prefix = 0;
    for (int b = 62; b >= 0; --b) {
        const uint64_t trial = prefix | ((1ull << b) - 1ull);
        int c = 0;
        for (int j = lane; j < n; j += 64) c += d2bits(j) <= trial;
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) c += __shfl_xor(c, o, 64);
        if (c < ke) prefix |= 1ull << b;
    }
    const double t = __longlong_as_double(prefix);
    int below = 0;
    double s = 0.0;
    for (int j = lane; j < n; j += 64) {
        const uint64_t v = d2bits(j);
        if (v < prefix) { ++below; s += sqrt(__longlong_as_double(v)); }
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        below += __shfl_xor(below, o, 64);
        s += __shfl_xor(s, o, 64);
    }
    if (lane == 0) out[q] = (s + (double)(ke - below) * sqrt(t)) / (double)ke;
}

struct Grid {
    double org[3], eps, eps2;
    int32_t dims[3];
    const int32_t *start;
    const double *cpts;
    const int32_t *ids;
};

__device__ __forceinline__ void cell_of(const Grid &g, const double *p, int c[3]) {
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double x = floor((p[a] - g.org[a]) / g.eps);
        c[a] = x < 0 ? 0 : (x > g.dims[a] - 1 ? g.dims[a] - 1 : (int)x);
    }
}

// Visit every grid point j with |p_j - p| <= eps (p itself included): f(j).
template <typename F>
__device__ __forceinline__ void for_neighbours(const Grid &g, const double *p, F f) {
    int c[3];
    cell_of(g, p, c);
    for (int z = c[2] - 1; z <= c[2] + 1; ++z) {
        if (z < 0 || z >= g.dims[2]) continue;
        for (int y = c[1] - 1; y <= c[1] + 1; ++y) {
            if (y < 0 || y >= g.dims[1]) continue;
            for (int x = c[0] - 1; x <= c[0] + 1; ++x) {
                if (x < 0 || x >= g.dims[0]) continue;
                const int64_t cell = ((int64_t)z * g.dims[1] + y) * g.dims[0] + x;
                for (int32_t i = g.start[cell]; i < g.start[cell + 1]; ++i) {
                    const double *q = g.cpts + (size_t)i * 3;
                    const double dx = q[0] - p[0], dy = q[1] - p[1], dz = q[2] - p[2];
                    if (sqrt((dx * dx + dy * dy) + dz * dz) <= g.eps) f(g.ids[i]);
                }
            }
        }
    }
}

__global__ __launch_bounds__(256) void k_core_count(Grid g, const double *__restrict__ pts, int32_t n,
                                                    int32_t min_samples, uint8_t *__restrict__ core,
                                                    int32_t *__restrict__ parent) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    int cnt = 0;
    for_neighbours(g, pts + (size_t)i * 3, [&](int) { ++cnt; });
    core[i] = cnt >= min_samples;
    parent[i] = i;
}

__device__ __forceinline__ int find_root(const int32_t *parent, int i) {
    int p = parent[i];
    while (p != i) {
        i = p;
        p = parent[i];
    }
    return i;
}

__global__ __launch_bounds__(256) void k_hook(Grid g, const double *__restrict__ pts, int32_t n,
                                              const uint8_t *__restrict__ core, int32_t *parent,
                                              int32_t *__restrict__ changed) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n || !core[i]) return;
    int hooked = 0;
    for_neighbours(g, pts + (size_t)i * 3, [&](int j) {
        if (j == i || !core[j]) return;
        const int ri = find_root(parent, i), rj = find_root(parent, j);
        if (ri == rj) return;
        const int hi = ri > rj ? ri : rj, lo = ri > rj ? rj : ri;
        atomicMin(&parent[hi], lo);
        hooked = 1;
    });
    if (hooked) atomicOr(changed, 1);
}

__global__ __launch_bounds__(256) void k_jump(int32_t n, int32_t *parent) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    parent[i] = find_root(parent, i);
}

__global__ __launch_bounds__(256) void k_label(Grid g, const double *__restrict__ pts, int32_t n,
                                               const uint8_t *__restrict__ core, const int32_t *__restrict__ parent,
                                               int32_t *__restrict__ labels) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    if (core[i]) { labels[i] = parent[i]; return; }
    int best = 0x7fffffff;
    for_neighbours(g, pts + (size_t)i * 3, [&](int j) {
        if (core[j] && j < best) best = j;
    });
    labels[i] = best == 0x7fffffff ? -1 : parent[best];
}

static size_t align256c(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace nof

using namespace nof;

extern "C" {

int nof_knn_mean_dist(const double *points, int32_t n, int32_t k, double *mean_dist, void *stream) {
    if (n < 0 || k <= 0 || (n > 0 && (!points || !mean_dist)))
        return set_error(NOF_EINVAL, "knn_mean_dist: bad arguments (n=%d, k=%d)", n, k);
    if (n == 0) return 0;
    hipLaunchKernelGGL(k_knn_mean_dist, dim3(div_up(n, 4)), dim3(256), 0, (hipStream_t)stream, points, n, k,
                       mean_dist);
    return check_launch("knn_mean_dist");
}

size_t nof_dbscan_workspace_bytes(int32_t n, int64_t n_cells) {
    return align256c((size_t)(n_cells + 1) * 4) + align256c((size_t)n * 24) + align256c((size_t)n * 4) * 2 +
           align256c((size_t)n) + 256 + nof_point_grid_workspace_bytes(n_cells);
}

int nof_dbscan(const double *points, int32_t n, double eps, int32_t min_samples, const double *origin,
               const int32_t *dims, int32_t *labels, void *workspace, void *stream) {
    if (n < 0 || !(eps > 0) || min_samples < 1 || !origin || !dims || (n > 0 && (!points || !labels)) || !workspace)
        return set_error(NOF_EINVAL, "dbscan: bad arguments");
    if (dims[0] <= 0 || dims[1] <= 0 || dims[2] <= 0) return set_error(NOF_EINVAL, "dbscan: bad grid dims");
    const int64_t nc = (int64_t)dims[0] * dims[1] * dims[2];
    if (nc > (1ll << 26)) return set_error(NOF_EINVAL, "dbscan: %lld grid cells (max 2^26)", (long long)nc);
    if (n == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    char *ws = (char *)workspace;
    Grid g;
    g.start = (int32_t *)ws;
    ws += align256c((size_t)(nc + 1) * 4);
    g.cpts = (double *)ws;
    ws += align256c((size_t)n * 24);
    g.ids = (int32_t *)ws;
    ws += align256c((size_t)n * 4);
    int32_t *parent = (int32_t *)ws;
    ws += align256c((size_t)n * 4);
    uint8_t *core = (uint8_t *)ws;
    ws += align256c((size_t)n);
    int32_t *changed = (int32_t *)ws;
    ws += 256;
    for (int a = 0; a < 3; ++a) { g.org[a] = origin[a]; g.dims[a] = dims[a]; }
    g.eps = eps;
    g.eps2 = eps * eps;
    int rc = nof_point_grid_build(points, n, origin, dims, eps, (int32_t *)g.start, (double *)g.cpts,
                                  (int32_t *)g.ids, ws, stream);
    if (rc) return rc;
    const unsigned nb = div_up(n, 256);
    hipLaunchKernelGGL(k_core_count, dim3(nb), dim3(256), 0, s, g, points, n, min_samples, core, parent);
    for (int round = 0; round < 64; ++round) {
        int32_t h = 0;
        if (hipMemsetAsync(changed, 0, 4, s) != hipSuccess) return set_error(NOF_ELAUNCH, "dbscan: memset failed");
        hipLaunchKernelGGL(k_hook, dim3(nb), dim3(256), 0, s, g, points, n, core, parent, changed);
        hipLaunchKernelGGL(k_jump, dim3(nb), dim3(256), 0, s, n, parent);
        if (hipMemcpyAsync(&h, changed, 4, hipMemcpyDeviceToHost, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)
            return set_error(NOF_ELAUNCH, "dbscan: flag read-back failed");
        if (!h) break;
        if (round == 63) return set_error(NOF_ELAUNCH, "dbscan: union-find did not converge in 64 rounds");
    }
    hipLaunchKernelGGL(k_label, dim3(nb), dim3(256), 0, s, g, points, n, core, parent, labels);
    return check_launch("dbscan");
}

}  // extern "C"

namespace nof {
// Per-segment mean of rows gathered through a permutation, summed in
// permutation order (open3d's AccumulatedPoint: sum in insertion order, then
// / count): one thread per segment.
__global__ __launch_bounds__(256) void k_segment_mean(const double *__restrict__ vals, int32_t C,
                                                      const int64_t *__restrict__ perm,
                                                      const int64_t *__restrict__ seg_start, int32_t S,
                                                      double *__restrict__ out) {
    const int sidx = blockIdx.x * 256 + threadIdx.x;
    if (sidx >= S) return;
    const int64_t b = seg_start[sidx], e = seg_start[sidx + 1];
    for (int c = 0; c < C; ++c) {
        double acc = 0.0;
        for (int64_t i = b; i < e; ++i) acc += vals[(size_t)perm[i] * C + c];
        out[(size_t)sidx * C + c] = acc / (double)(e - b);
    }
}
}  // namespace nof

extern "C" int nof_segment_mean(const double *vals, int32_t C, const int64_t *perm, const int64_t *seg_start,
                                int32_t S, double *out, void *stream) {
    if (C <= 0 || S < 0 || (S > 0 && (!vals || !perm || !seg_start || !out)))
        return set_error(NOF_EINVAL, "segment_mean: bad arguments");
    if (S == 0) return 0;
    hipLaunchKernelGGL(k_segment_mean, dim3(div_up(S, 256)), dim3(256), 0, (hipStream_t)stream, vals, C, perm,
                       seg_start, S, out);
    return check_launch("segment_mean");
}
