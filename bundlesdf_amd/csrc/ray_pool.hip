// Ray-pool construction on the device: replaces the host
// loop of NerfRunner.make_frame_rays (nerf_runner.py:244-314) with
// compute_near_far_and_filter_rays (:39-65) / ray_box_intersection_batch
// (nerf_helpers.py:403-446), the octree filter (:300-312, kaolin trace ->
// dense DDA of ray_trace.h) and the octree-cloud denoise (:175-194, :408-423;
// cKDTree nearest neighbour -> uniform-grid radius test).
//
// One pass over all pixels of a batch of frames:
//   k_dilate_rows / k_dilate_cols  cv2.dilate with a k x k ones kernel as two
//                                  separable window counts (prefix sums in LDS)
//   k_select                       per-pixel predicate + near/far, block counts
//   k_scan_counts                  exclusive offsets of the block counts
//   k_emit                         order-preserving compaction of the selected
//                                  pixels into [n,12] reference-layout rays
// The output order is frame-major, then row-major pixel order — the order of
// np.where(mask) + np.concatenate of the reference — so the pool equals the
// reference's row for row. Geometry runs in f64 like the reference (its rays
// are float64 numpy arrays) with sums in the reference's order and no FMA
// contraction; only the stored near/far are rounded to f32, as torch.tensor(
// rays, dtype=float) does.
#include "nof_device.h"
#include "ray_trace.h"

#pragma clang fp contract(off)

namespace nof {

constexpr int POOL_BLOCK = 256;
constexpr int POOL_MAX_W = 4096;
constexpr int POOL_MAX_H = 1024;

// Block-wide (256 threads) exclusive scan of one int per thread.
__device__ __forceinline__ int block_excl_scan(int v, int &total, int *wsum) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int off = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < POOL_BLOCK / 64; ++w) {
        const int t = wsum[w];
        off += (w < wave) ? t : 0;
        tot += t;
    }
    __syncthreads();
    total = tot;
    return off + x - v;
}

__device__ __forceinline__ int dilate_size(const nof_ray_pool_desc &d, int f) {
    // nerf_runner.py:275-286: 100x100 for frame 0 (its mask is assumed perfect),
    // (60 // down_scale_ratio)^2 for the others; cv2 uses 3x3 for an empty kernel
    int k = (d.first_frame_id + f == 0) ? d.dilate_first : d.dilate_other;
    return k <= 0 ? 3 : k;
}

// Horizontal pass: out[f,v,u] = any(mask[f,v,u-lo .. u+hi] > 0), lo = k/2,
// hi = k-1-lo (cv2.dilate's default anchor = kernel centre; scipy's
// maximum_filter window is the same, borders never add pixels).
__global__ __launch_bounds__(POOL_BLOCK) void k_dilate_rows(nof_ray_pool_desc d, uint8_t *__restrict__ out) {
    __shared__ int pre[POOL_MAX_W + 1];
    __shared__ int wsum[POOL_BLOCK / 64];
    const int f = blockIdx.y, v = blockIdx.x, W = d.W;
    const uint8_t *row = d.mask + ((size_t)f * d.H + v) * W;
    const int ipt = (W + POOL_BLOCK - 1) / POOL_BLOCK, u0 = threadIdx.x * ipt;
    int s = 0;
    for (int i = 0; i < ipt; ++i) {
        const int u = u0 + i;
        if (u < W) s += row[u] > 0;
    }
    int tot;
    int run = block_excl_scan(s, tot, wsum);
    for (int i = 0; i < ipt; ++i) {
        const int u = u0 + i;
        if (u < W) { run += row[u] > 0; pre[u + 1] = run; }
    }
    if (threadIdx.x == 0) pre[0] = 0;
    __syncthreads();
    const int k = dilate_size(d, f), lo = k / 2, hi = k - 1 - lo;
    uint8_t *o = out + ((size_t)f * d.H + v) * W;
    for (int u = threadIdx.x; u < W; u += POOL_BLOCK) {
        const int a = u - lo < 0 ? 0 : u - lo, b = u + hi + 1 > W ? W : u + hi + 1;
        o[u] = (pre[b] - pre[a]) > 0;
    }
}

// Vertical pass over the horizontal result: 64 columns per block (one per
// lane, coalesced row reads), column prefix counts in LDS (u16: H <= 1024).
__global__ __launch_bounds__(POOL_BLOCK) void k_dilate_cols(nof_ray_pool_desc d, const uint8_t *__restrict__ hrow,
                                                            uint8_t *__restrict__ out) {
    __shared__ uint16_t pre[(POOL_MAX_H + 1) * 64];
    __shared__ int wtot[POOL_BLOCK];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int f = blockIdx.y, c = blockIdx.x * 64 + lane, H = d.H, W = d.W;
    const bool ok = c < W;
    const uint8_t *src = hrow + (size_t)f * H * W;
    const int rpw = (H + 3) / 4, r0 = wave * rpw, r1 = (r0 + rpw < H) ? r0 + rpw : H;
    int run = 0;
    for (int v = r0; v < r1; ++v) {
        run += ok ? src[(size_t)v * W + c] : 0;
        pre[(v + 1) * 64 + lane] = (uint16_t)run;
    }
    wtot[wave * 64 + lane] = run;
    __syncthreads();
    int add = 0;
    for (int w = 0; w < wave; ++w) add += wtot[w * 64 + lane];
    for (int v = r0; v < r1; ++v) pre[(v + 1) * 64 + lane] = (uint16_t)(pre[(v + 1) * 64 + lane] + add);
    if (wave == 0) pre[lane] = 0;
    __syncthreads();
    if (!ok) return;
    const int k = dilate_size(d, f), lo = k / 2, hi = k - 1 - lo;
    uint8_t *o = out + (size_t)f * H * W;
    for (int v = wave; v < H; v += 4) {
        const int a = v - lo < 0 ? 0 : v - lo, b = v + hi + 1 > H ? H : v + hi + 1;
        o[(size_t)v * W + c] = (pre[b * 64 + lane] - pre[a * 64 + lane]) > 0;
    }
}

// Camera ray of pixel (u, v), get_camera_rays_np (nerf_helpers.py:358-363):
// float32 arithmetic on float32 pixel coordinates and intrinsics.
__device__ __forceinline__ void camera_dir(const nof_ray_pool_desc &d, int u, int v, float dir[3]) {
    dir[0] = ((float)u - d.cx) / d.fx;
    dir[1] = -(((float)v - d.cy) / d.fy);
    dir[2] = -1.0f;
}

// ray_box_intersection_batch (nerf_helpers.py:403-446) for one ray, f64,
// same comparisons and clamps; returns tmin (-1 on a miss) and tmax.
__device__ __forceinline__ void ray_box(const double o[3], const double dir_in[3], const double *bmin,
                                        const double *bmax, double &tmin_out, double &tmax_out) {
    const double n = sqrt((dir_in[0] * dir_in[0] + dir_in[1] * dir_in[1]) + dir_in[2] * dir_in[2]) + 1e-10;
    double inv[3], lo[3], hi[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        inv[a] = 1.0 / (dir_in[a] / n);
        const bool neg = inv[a] < 0;
        lo[a] = ((neg ? bmax[a] : bmin[a]) - o[a]) * inv[a];
        hi[a] = ((neg ? bmin[a] : bmax[a]) - o[a]) * inv[a];
    }
    double tmin = lo[0], tmax = hi[0];
    if (tmin < 0) tmin = 0;
    double tymin = lo[1];
    const double tymax = hi[1];
    if (tymin < 0) tymin = 0;
    bool hit = !((tmin > tymax) || (tymin > tmax));
    if (tymin > tmin) tmin = tymin;
    if (tymax < tmax) tmax = tymax;
    double tzmin = lo[2];
    const double tzmax = hi[2];
    if (tzmin < 0) tzmin = 0;
    if ((tmin > tzmax) || (tzmin > tmax)) hit = false;
    if (tzmin > tmin) tmin = tzmin;
    if (tzmax < tmax) tmax = tzmax;
    tmin_out = hit ? tmin : -1.0;
    tmax_out = hit ? tmax : -1.0;
}

// Octree-cloud denoise (nerf_runner.py:175-194): true when some cloud point
// lies within r of the back-projected depth point pw (cKDTree distance,
// sqrt of the ordered sum of squares, compared like dists > r).
__device__ __forceinline__ bool near_cloud(const nof_ray_pool_desc &d, const double pw[3]) {
    int lo[3], hi[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double c = floor((pw[a] - d.grid_origin[a]) / d.grid_cell);
        const double l = fmin(fmax(c - 1, 0.0), (double)d.grid_dims[a]);
        const double h = fmax(fmin(c + 1, (double)(d.grid_dims[a] - 1)), -1.0);
        lo[a] = (int)l;
        hi[a] = (int)h;
    }
    for (int z = lo[2]; z <= hi[2]; ++z)
        for (int y = lo[1]; y <= hi[1]; ++y)
            for (int x = lo[0]; x <= hi[0]; ++x) {
                const int64_t cell = ((int64_t)z * d.grid_dims[1] + y) * d.grid_dims[0] + x;
                for (int32_t i = d.cell_start[cell]; i < d.cell_start[cell + 1]; ++i) {
                    const double *q = d.cell_points + (size_t)i * 3;
                    const double dx = pw[0] - q[0], dy = pw[1] - q[1], dz = pw[2] - q[2];
                    if (!(sqrt((dx * dx + dy * dy) + dz * dz) > d.grid_radius)) return true;
                }
            }
    return false;
}

// Per-pixel predicate (make_frame_rays :254-312 + denoise): flag, near/far
// (f32) and the block's count.
__global__ __launch_bounds__(POOL_BLOCK) void k_select(nof_ray_pool_desc d, const uint8_t *__restrict__ dil,
                                                       uint8_t *__restrict__ flag, float *__restrict__ nearfar,
                                                       int32_t *__restrict__ blk_count) {
    const int64_t P = (int64_t)d.F * d.H * d.W;
    const int64_t p = (int64_t)blockIdx.x * POOL_BLOCK + threadIdx.x;
    bool sel = false;
    float nr = 0.f, fr = 0.f;
    if (p < P) {
        const int64_t hw = (int64_t)d.H * d.W;
        const int f = (int)(p / hw), v = (int)((p % hw) / d.W), u = (int)(p % d.W);
        const bool m = d.mask[p] > 0;
        const float depth = d.depth[p];
        // type 1 (invalid depth inside the mask) never enters the pool (:264-266, :290)
        const bool invalid = (depth < d.near_sc || depth > d.far_sc) && m;
        sel = dil[p] && !invalid && !(d.occ_mask && d.occ_mask[p] > 0);
        if (sel) {
            const double *T = d.cam_in_world + (size_t)f * 16;
            float dirf[3];
            camera_dir(d, u, v, dirf);
            const double dc[3] = {dirf[0], dirf[1], dirf[2]};
            double dw[3];
#pragma unroll
            for (int a = 0; a < 3; ++a) dw[a] = (T[a * 4 + 0] * dc[0] + T[a * 4 + 1] * dc[1]) + T[a * 4 + 2] * dc[2];
            const double o[3] = {T[3], T[7], T[11]};
            double tmin, tmax;
            ray_box(o, dw, d.bbox, d.bbox + 3, tmin, tmax);
            sel = tmin >= 0;
            const double nrm = sqrt((dc[0] * dc[0] + dc[1] * dc[1]) + dc[2] * dc[2]);
            const double uz = dc[2] / nrm;
            nr = (float)fabs(uz * tmin);
            fr = (float)fabs(uz * tmax);
            if (sel && d.occ) {
                // octree filter (:300-312): unit camera dir rotated to world, f32 trace
                const double ux = dc[0] / nrm, uy = dc[1] / nrm;
                float of[3], df[3];
#pragma unroll
                for (int a = 0; a < 3; ++a) {
                    of[a] = (float)o[a];
                    df[a] = (float)((T[a * 4 + 0] * ux + T[a * 4 + 1] * uy) + T[a * 4 + 2] * uz);
                }
                float hit[2] = {0.f, 0.f};
                const int k = trace_ray(d.occ, d.occ_n, of, df, 1, hit);
                sel = k > 0 && hit[0] > 0.f;
            }
            if (sel && d.cell_start && m && (double)depth <= d.far_sc64) {
                const double pc[3] = {dc[0] * (double)depth, dc[1] * (double)depth, dc[2] * (double)depth};
                double pw[3];
#pragma unroll
                for (int a = 0; a < 3; ++a)
                    pw[a] = ((T[a * 4 + 0] * pc[0] + T[a * 4 + 1] * pc[1]) + T[a * 4 + 2] * pc[2]) + T[a * 4 + 3];
                sel = near_cloud(d, pw);
            }
        }
        flag[p] = sel;
        nearfar[p * 2] = nr;
        nearfar[p * 2 + 1] = fr;
    }
    const int c = __syncthreads_count(sel);
    if (threadIdx.x == 0) blk_count[blockIdx.x] = c;
}

// Exclusive offsets of n counts (one block of 1024 threads, contiguous chunk
// per thread); off[n] = total.
__global__ __launch_bounds__(1024) void k_scan_counts(const int32_t *__restrict__ cnt, int64_t n,
                                                      int64_t *__restrict__ off) {
    __shared__ int64_t wsum[16];
    const int64_t chunk = (n + 1023) / 1024, b = threadIdx.x * chunk;
    const int64_t e = b + chunk < n ? b + chunk : n;
    int64_t s = 0;
    for (int64_t i = b; i < e; ++i) s += cnt[i];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    int64_t x = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int64_t y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    int64_t base = 0, tot = 0;
    for (int w = 0; w < 16; ++w) {
        base += w < wave ? wsum[w] : 0;
        tot += wsum[w];
    }
    int64_t run = base + x - s;
    for (int64_t i = b; i < e; ++i) {
        off[i] = run;
        run += cnt[i];
    }
    if (threadIdx.x == 0) off[n] = tot;
}

// Order-preserving compaction: selected pixel -> row blk_off[b] + rank in block.
// Row layout (reference column order, 12 columns): dir(0-2, unnormalised GL
// camera frame), rgb(3-5), depth(6), mask>0 (7), frame id (8), type 0 (9),
// near (10), far (11).
__global__ __launch_bounds__(POOL_BLOCK) void k_emit(nof_ray_pool_desc d, const uint8_t *__restrict__ flag,
                                                     const float *__restrict__ nearfar,
                                                     const int64_t *__restrict__ blk_off, int64_t nblk,
                                                     float *__restrict__ rays, int64_t *__restrict__ n_out) {
    __shared__ int wsum[POOL_BLOCK / 64];
    const int64_t P = (int64_t)d.F * d.H * d.W;
    const int64_t p = (int64_t)blockIdx.x * POOL_BLOCK + threadIdx.x;
    const int sel = (p < P) ? flag[p] : 0;
    int tot;
    const int rank = block_excl_scan(sel, tot, wsum);
    if (blockIdx.x == 0 && threadIdx.x == 0) n_out[0] = blk_off[nblk];
    if (!sel) return;
    const int64_t hw = (int64_t)d.H * d.W;
    const int f = (int)(p / hw), v = (int)((p % hw) / d.W), u = (int)(p % d.W);
    float dir[3];
    camera_dir(d, u, v, dir);
    float *r = rays + (blk_off[blockIdx.x] + rank) * 12;
    r[0] = dir[0];
    r[1] = dir[1];
    r[2] = dir[2];
    r[3] = d.rgb[p * 3];
    r[4] = d.rgb[p * 3 + 1];
    r[5] = d.rgb[p * 3 + 2];
    r[6] = d.depth[p];
    r[7] = d.mask[p] > 0 ? 1.f : 0.f;
    r[8] = (float)(d.first_frame_id + f);
    r[9] = 0.f;
    r[10] = nearfar[p * 2];
    r[11] = nearfar[p * 2 + 1];
}

// --- uniform point grid for the denoise radius test ----------------------
__device__ __forceinline__ int64_t point_cell(const double *p, const double *org, const int32_t *dims, double cell) {
    int c[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const double x = floor((p[a] - org[a]) / cell);
        c[a] = x < 0 ? 0 : (x > dims[a] - 1 ? dims[a] - 1 : (int)x);
    }
    return ((int64_t)c[2] * dims[1] + c[1]) * dims[0] + c[0];
}

struct GridArgs {
    double org[3];
    int32_t dims[3];
    double cell;
};

__global__ __launch_bounds__(256) void k_grid_count(const double *__restrict__ pts, int32_t M, GridArgs g,
                                                    int32_t *__restrict__ count) {
    const int32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= M) return;
    atomicAdd(&count[point_cell(pts + (size_t)i * 3, g.org, g.dims, g.cell)], 1);
}

__global__ __launch_bounds__(256) void k_grid_fill(const double *__restrict__ pts, int32_t M, GridArgs g,
                                                   const int64_t *__restrict__ start, int32_t *__restrict__ cursor,
                                                   int32_t *__restrict__ cell_start, int64_t n_cells,
                                                   double *__restrict__ out, int32_t *__restrict__ ids) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x, stride = (int64_t)gridDim.x * 256;
    for (int64_t c = i; c <= n_cells; c += stride) cell_start[c] = (int32_t)start[c];
    for (int64_t j = i; j < M; j += stride) {
        const int64_t c = point_cell(pts + j * 3, g.org, g.dims, g.cell);
        const int64_t slot = start[c] + atomicAdd(&cursor[c], 1);
        out[slot * 3] = pts[j * 3];
        out[slot * 3 + 1] = pts[j * 3 + 1];
        out[slot * 3 + 2] = pts[j * 3 + 2];
        if (ids) ids[slot] = (int32_t)j;
    }
}

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

}  // namespace nof

using namespace nof;

extern "C" {

size_t nof_ray_pool_workspace_bytes(int32_t F, int32_t H, int32_t W) {
    const size_t P = (size_t)F * H * W, nblk = (P + POOL_BLOCK - 1) / POOL_BLOCK;
    return align256(P) * 3 + align256(P * 8) + align256(nblk * 4) + align256((nblk + 1) * 8);
}

int nof_make_frame_rays(const nof_ray_pool_desc *desc, void *stream) {
    if (!desc) return set_error(NOF_EINVAL, "make_frame_rays: NULL desc");
    const nof_ray_pool_desc d = *desc;
    if (d.F <= 0 || d.H <= 0 || d.W <= 0) return set_error(NOF_EINVAL, "make_frame_rays: empty frame batch");
    if (d.W > POOL_MAX_W || d.H > POOL_MAX_H)
        return set_error(NOF_EINVAL, "make_frame_rays: frames up to %dx%d (got %dx%d)", POOL_MAX_W, POOL_MAX_H, d.W,
                         d.H);
    if (!d.rgb || !d.depth || !d.mask || !d.cam_in_world || !d.rays || !d.n_out || !d.workspace)
        return set_error(NOF_EINVAL, "make_frame_rays: NULL input/output pointer");
    if (d.occ && d.occ_n <= 0) return set_error(NOF_EINVAL, "make_frame_rays: occ_n must be > 0");
    if (d.cell_start && (!d.cell_points || d.grid_cell <= 0 || d.grid_dims[0] <= 0 || d.grid_dims[1] <= 0 ||
                         d.grid_dims[2] <= 0))
        return set_error(NOF_EINVAL, "make_frame_rays: bad denoise point grid");
    hipStream_t s = (hipStream_t)stream;
    const size_t P = (size_t)d.F * d.H * d.W;
    const int64_t nblk = (int64_t)((P + POOL_BLOCK - 1) / POOL_BLOCK);
    char *ws = (char *)d.workspace;
    uint8_t *hrow = (uint8_t *)ws;
    uint8_t *dil = hrow + align256(P);
    uint8_t *flag = dil + align256(P);
    float *nearfar = (float *)(flag + align256(P));
    int32_t *blk_count = (int32_t *)((char *)nearfar + align256(P * 8));
    int64_t *blk_off = (int64_t *)((char *)blk_count + align256(nblk * 4));
    hipLaunchKernelGGL(k_dilate_rows, dim3(d.H, d.F), dim3(POOL_BLOCK), 0, s, d, hrow);
    hipLaunchKernelGGL(k_dilate_cols, dim3((d.W + 63) / 64, d.F), dim3(POOL_BLOCK), 0, s, d, hrow, dil);
    hipLaunchKernelGGL(k_select, dim3((unsigned)nblk), dim3(POOL_BLOCK), 0, s, d, dil, flag, nearfar, blk_count);
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, blk_count, nblk, blk_off);
    hipLaunchKernelGGL(k_emit, dim3((unsigned)nblk), dim3(POOL_BLOCK), 0, s, d, flag, nearfar, blk_off, nblk, d.rays,
                       d.n_out);
    return check_launch("make_frame_rays");
}

size_t nof_point_grid_workspace_bytes(int64_t n_cells) {
    return align256((size_t)n_cells * 4) * 2 + align256((size_t)(n_cells + 1) * 8);
}

int nof_point_grid_build(const double *points, int32_t M, const double *origin, const int32_t *dims, double cell,
                         int32_t *cell_start, double *cell_points, int32_t *cell_ids, void *workspace, void *stream) {
    if (M < 0 || !origin || !dims || cell <= 0 || !cell_start || (M > 0 && (!points || !cell_points)) || !workspace)
        return set_error(NOF_EINVAL, "point_grid_build: bad arguments");
    if (dims[0] <= 0 || dims[1] <= 0 || dims[2] <= 0) return set_error(NOF_EINVAL, "point_grid_build: bad dims");
    const int64_t nc = (int64_t)dims[0] * dims[1] * dims[2];
    if (nc > (1ll << 28)) return set_error(NOF_EINVAL, "point_grid_build: %lld cells (max 2^28)", (long long)nc);
    hipStream_t s = (hipStream_t)stream;
    GridArgs g;
    for (int a = 0; a < 3; ++a) {
        g.org[a] = origin[a];
        g.dims[a] = dims[a];
    }
    g.cell = cell;
    int32_t *count = (int32_t *)workspace;
    int32_t *cursor = (int32_t *)((char *)workspace + align256((size_t)nc * 4));
    int64_t *start = (int64_t *)((char *)cursor + align256((size_t)nc * 4));
    if (hipMemsetAsync(count, 0, (size_t)nc * 4, s) != hipSuccess || hipMemsetAsync(cursor, 0, (size_t)nc * 4, s) != hipSuccess)
        return set_error(NOF_ELAUNCH, "point_grid_build: memset failed");
    if (M > 0) hipLaunchKernelGGL(k_grid_count, dim3(div_up(M, 256)), dim3(256), 0, s, points, M, g, count);
    hipLaunchKernelGGL(k_scan_counts, dim3(1), dim3(1024), 0, s, count, nc, start);
    const unsigned nb = div_up((uint64_t)(M > nc + 1 ? M : nc + 1), 256);
    hipLaunchKernelGGL(k_grid_fill, dim3(nb < 65535u ? nb : 65535u), dim3(256), 0, s, points, M, g, start, cursor,
                       cell_start, nc, cell_points, cell_ids);
    return check_launch("point_grid_build");
}

}  // extern "C"
