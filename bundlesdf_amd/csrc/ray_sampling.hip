// Ray-sampling kernels: drop-in replacements for the reference's `common`
// extension (mycuda/common.cu) plus the dense-occupancy ray trace that
// replaces kaolin's SPC unbatched_raytrace (Utils.py:443-475).
#include "nof_device.h"
#include "ray_trace.h"

#pragma clang fp contract(off)

namespace nof {

// sample_rays_uniform_occupied_voxels_kernel (common.cu:40-105). One lane per
// (ray, sample), ray-major so a wave's lanes share one ray's box list (a
// broadcast read) and its z_sampled / z_vals rows are coalesced. The walk is
// the reference's sequential subtraction, so results are bit-identical. On
// malformed input the reference prints and spins forever (:66-71, :87-92);
// here the sample is left untouched and an error counter is bumped.
__global__ __launch_bounds__(256) void k_sample_occupied(const float *__restrict__ z_in_out,
                                                         const float *__restrict__ z_sampled,
                                                         float *__restrict__ z_vals, int32_t n_rays, int32_t K,
                                                         int32_t S, int32_t *__restrict__ err) {
    const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= (int64_t)n_rays * S) return;
    const int64_t r = t / S;
    const float *box = z_in_out + r * K * 2;
    float z_remain = z_sampled[t];
    const float eps = 1e-4f;
    if (box[0] == 0) return;
    for (int i = 0;; ++i) {
        if (i >= K) {
            if (z_remain <= eps) z_vals[t] = box[(K - 1) * 2 + 1];
            else if (err) atomicAdd(err, 1);
            return;
        }
        const float zin = box[i * 2], zout = box[i * 2 + 1];
        if (zin == 0) {
            if (z_remain <= eps && i >= 1) z_vals[t] = box[(i - 1) * 2 + 1];
            else if (err) atomicAdd(err, 1);
            return;
        }
        const float len = zout - zin;
        if (z_remain <= len) { z_vals[t] = zin + z_remain; return; }
        z_remain -= len;
    }
}

// postprocessOctreeRayTracingKernel (common.cu:128-149).
__global__ __launch_bounds__(256) void k_postprocess_octree(const int64_t *__restrict__ ray_index,
                                                            const float *__restrict__ depth_in_out,
                                                            const int64_t *__restrict__ unique_ids,
                                                            const int64_t *__restrict__ start_poss, int64_t M,
                                                            int64_t U, int32_t max_int, float *__restrict__ out) {
    const int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (u >= U) return;
    const int64_t r = unique_ids[u];
    float *dst = out + r * max_int * 2;
    int k = 0;
    for (int64_t i = start_poss[u]; i < M; i++) {
        if (ray_index[i] != r) break;
        const float a = depth_in_out[i * 2], b = depth_in_out[i * 2 + 1];
        if (a == 0 || b == 0) break;
        if (a > b) continue;
        if (fabsf(b - a) < 1e-4f) continue;
        if (k < max_int) { dst[k * 2] = a; dst[k * 2 + 1] = b; }
        k++;
    }
}

// rayColorToTextureImageKernel (common.cu:171-219): barycentric UV of each hit.
__global__ __launch_bounds__(256) void k_texture_uv(const int64_t *__restrict__ F, const float *__restrict__ V,
                                                    const float *__restrict__ hit, const int64_t *__restrict__ fid,
                                                    const float *__restrict__ uvs_tex, float *__restrict__ uvs,
                                                    int64_t M) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= M) return;
    const int64_t *f = F + fid[i] * 3;
    float v[3][3];
#pragma unroll
    for (int r = 0; r < 3; r++)
#pragma unroll
        for (int c = 0; c < 3; c++) v[r][c] = V[f[r] * 3 + c];
    const float p[3] = {hit[i * 3], hit[i * 3 + 1], hit[i * 3 + 2]};
    auto cross = [](const float *a, const float *b, float *o) {
        o[0] = a[1] * b[2] - a[2] * b[1];
        o[1] = a[2] * b[0] - a[0] * b[2];
        o[2] = a[0] * b[1] - a[1] * b[0];
    };
    auto dot = [](const float *a, const float *b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; };
    float A[3], Bv[3], n[3], e1[3], e2[3], c[3], q1[3], q2[3], q0[3];
    for (int k = 0; k < 3; k++) {
        A[k] = v[1][k] - v[2][k]; Bv[k] = v[1][k] - v[0][k];
        e1[k] = v[1][k] - v[0][k]; e2[k] = v[2][k] - v[0][k];
        q1[k] = v[1][k] - p[k]; q2[k] = v[2][k] - p[k]; q0[k] = v[0][k] - p[k];
    }
    cross(A, Bv, n);
    cross(e1, e2, c);
    const float abc = dot(n, c);
    cross(q1, q2, c);
    const float pbc = dot(n, c);
    cross(q2, q0, c);
    const float pca = dot(n, c);
    const float w0 = pbc / abc, w1 = pca / abc, w2 = 1 - w0 - w1;
    for (int j = 0; j < 2; j++)
        uvs[i * 2 + j] = uvs_tex[f[0] * 2 + j] * w0 + uvs_tex[f[1] * 2 + j] * w1 + uvs_tex[f[2] * 2 + j] * w2;
}

__global__ __launch_bounds__(256) void k_octree_ray_trace(const uint8_t *__restrict__ occ, int N,
                                                          const float *__restrict__ rays_o,
                                                          const float *__restrict__ rays_d, int R, int Kmax,
                                                          float *__restrict__ out, int32_t *__restrict__ counts) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    const float o[3] = {rays_o[r * 3], rays_o[r * 3 + 1], rays_o[r * 3 + 2]};
    const float d[3] = {rays_d[r * 3], rays_d[r * 3 + 1], rays_d[r * 3 + 2]};
    float *dst = out + (size_t)r * Kmax * 2;
    const int k = trace_ray(occ, N, o, d, Kmax, dst);
    for (int j = k; j < Kmax; ++j) { dst[j * 2] = 0.f; dst[j * 2 + 1] = 0.f; }
    if (counts) counts[r] = k;
}

}  // namespace nof

extern "C" int nof_sample_rays_uniform_occupied_voxels(const float *z_in_out, const float *z_sampled, float *z_vals,
                                                       int32_t n_rays, int32_t n_intersect, int32_t n_samples,
                                                       int32_t *error_count, void *stream) {
    if (n_rays < 0 || n_intersect < 1 || n_samples < 0)
        return nof::set_error(NOF_EINVAL, "sampleRaysUniformOccupiedVoxels: bad shape (%d,%d,%d)", n_rays,
                              n_intersect, n_samples);
    const int64_t n = (int64_t)n_rays * n_samples;
    if (n == 0) return NOF_OK;
    hipLaunchKernelGGL(nof::k_sample_occupied, dim3(nof::div_up(n, 256)), dim3(256), 0, (hipStream_t)stream, z_in_out,
                       z_sampled, z_vals, n_rays, n_intersect, n_samples, error_count);
    return nof::check_launch("sampleRaysUniformOccupiedVoxels");
}

extern "C" int nof_postprocess_octree_ray_tracing(const int64_t *ray_index, const float *depth_in_out,
                                                  const int64_t *unique_ids, const int64_t *start_poss,
                                                  int64_t n_hits, int64_t n_unique, int32_t max_intersections,
                                                  float *out, void *stream) {
    if (n_unique <= 0) return NOF_OK;
    hipLaunchKernelGGL(nof::k_postprocess_octree, dim3(nof::div_up(n_unique, 256)), dim3(256), 0, (hipStream_t)stream,
                       ray_index, depth_in_out, unique_ids, start_poss, n_hits, n_unique, max_intersections, out);
    return nof::check_launch("postprocessOctreeRayTracing");
}

extern "C" int nof_ray_color_to_texture_uv(const int64_t *F, const float *V, const float *hit_locations,
                                           const int64_t *hit_face_ids, const float *uvs_tex, float *uvs,
                                           int64_t n_hits, void *stream) {
    if (n_hits <= 0) return NOF_OK;
    hipLaunchKernelGGL(nof::k_texture_uv, dim3(nof::div_up(n_hits, 256)), dim3(256), 0, (hipStream_t)stream, F, V,
                       hit_locations, hit_face_ids, uvs_tex, uvs, n_hits);
    return nof::check_launch("rayColorToTextureImageCUDA");
}

extern "C" int nof_octree_ray_trace(const uint8_t *occ, int32_t N, const float *rays_o, const float *rays_d,
                                    int32_t R, int32_t Kmax, float *out, int32_t *counts, void *stream) {
    if (N <= 0 || Kmax <= 0) return nof::set_error(NOF_EINVAL, "octree_ray_trace: bad N=%d Kmax=%d", N, Kmax);
    if (R <= 0) return NOF_OK;
    hipLaunchKernelGGL(nof::k_octree_ray_trace, dim3(nof::div_up(R, 256)), dim3(256), 0, (hipStream_t)stream, occ, N,
                       rays_o, rays_d, R, Kmax, out, counts);
    return nof::check_launch("octree_ray_trace");
}
