// Texture baking from the training images: the device path
// of NerfRunner.mesh_texture_from_train_images (nerf_runner.py:1467-1541).
// The reference renders each camera's depth with pyrender, back-projects it,
// snaps the points to the mesh with trimesh.proximity.closest_point, turns
// them into texel coordinates with common.rayColorToTextureImageCUDA and
// accumulates the first colour per texel with torch.unique + scatter. Here:
//
//  k_raster        one thread per face: project (OpenCV pinhole, f64), walk
//                  the integer pixel centres of the bbox, edge-function
//                  coverage (either orientation, edges inclusive),
//                  perspective-correct depth, atomicMin of (depth bits << 32 |
//                  face) into a 64-bit z-buffer -> depth and face id at once.
//  k_hits          per pixel: depth >= min_depth and the object mask ->
//                  back-projection (depth2xyzmap arithmetic), camera->object
//                  transform, closest point on the rasterised face (the
//                  reference's closest_point, restricted to the face the pixel
//                  sees) -> hit location + face id (dense, -1 = none).
//  k_tex_first /   texel = round-half-even(uv) flattened with the reference's
//  k_tex_add       row stride (W-1) (nerf_runner.py:1524-1531); the first
//                  hit (pixel order) of each texel adds its colour and weight 1.
#include "nof_device.h"

#pragma clang fp contract(off)

namespace nof {

struct Cam {
    double R[9], t[3];        // ob -> cam (OpenCV)
    double fx, fy, cx, cy;
};

__global__ __launch_bounds__(256) void k_raster(const float *__restrict__ V, const int64_t *__restrict__ F,
                                                int64_t nF, Cam c, int H, int W, double znear, double zfar,
                                                unsigned long long *__restrict__ zbuf) {
    const int64_t f = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (f >= nF) return;
    double u[3], v[3], z[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        const float *p = V + F[f * 3 + k] * 3;
        const double x = p[0], y = p[1], w = p[2];
        const double X = ((c.R[0] * x + c.R[1] * y) + c.R[2] * w) + c.t[0];
        const double Y = ((c.R[3] * x + c.R[4] * y) + c.R[5] * w) + c.t[1];
        const double Z = ((c.R[6] * x + c.R[7] * y) + c.R[8] * w) + c.t[2];
        if (!(Z > znear)) return;            // no near-plane clipping: faces crossing it are dropped
        z[k] = Z;
        u[k] = c.fx * X / Z + c.cx;
        v[k] = c.fy * Y / Z + c.cy;
    }
    const double area = (u[1] - u[0]) * (v[2] - v[0]) - (u[2] - u[0]) * (v[1] - v[0]);
    if (area == 0.0) return;
    int u0 = (int)ceil(fmin(fmin(u[0], u[1]), u[2])), u1 = (int)floor(fmax(fmax(u[0], u[1]), u[2]));
    int v0 = (int)ceil(fmin(fmin(v[0], v[1]), v[2])), v1 = (int)floor(fmax(fmax(v[0], v[1]), v[2]));
    u0 = u0 < 0 ? 0 : u0;
    v0 = v0 < 0 ? 0 : v0;
    u1 = u1 > W - 1 ? W - 1 : u1;
    v1 = v1 > H - 1 ? H - 1 : v1;
    for (int py = v0; py <= v1; ++py)
        for (int px = u0; px <= u1; ++px) {
            const double X = px, Y = py;
            // barycentric weights of vertex k = edge function of the opposite edge / area
            const double e0 = ((u[2] - u[1]) * (Y - v[1]) - (v[2] - v[1]) * (X - u[1])) / area;
            const double e1 = ((u[0] - u[2]) * (Y - v[2]) - (v[0] - v[2]) * (X - u[2])) / area;
            const double e2 = ((u[1] - u[0]) * (Y - v[0]) - (v[1] - v[0]) * (X - u[0])) / area;
            if (e0 < 0.0 || e1 < 0.0 || e2 < 0.0) continue;
            const double zi = 1.0 / ((e0 / z[0] + e1 / z[1]) + e2 / z[2]);
            if (!(zi <= zfar)) continue;
            const float zf = (float)zi;
            const unsigned long long key = ((unsigned long long)__float_as_uint(zf) << 32) | (unsigned long long)f;
            atomicMin(&zbuf[(size_t)py * W + px], key);
        }
}

// Closest point of triangle (a, b, c) to p (Voronoi-region walk, f64).
__device__ __forceinline__ void closest_on_tri(const double p[3], const double a[3], const double b[3],
                                               const double c[3], double out[3]) {
    double ab[3], ac[3], ap[3];
    for (int k = 0; k < 3; ++k) { ab[k] = b[k] - a[k]; ac[k] = c[k] - a[k]; ap[k] = p[k] - a[k]; }
    auto dot = [](const double *x, const double *y) { return (x[0] * y[0] + x[1] * y[1]) + x[2] * y[2]; };
    const double d1 = dot(ab, ap), d2 = dot(ac, ap);
    if (d1 <= 0 && d2 <= 0) { for (int k = 0; k < 3; ++k) out[k] = a[k]; return; }
    double bp[3];
    for (int k = 0; k < 3; ++k) bp[k] = p[k] - b[k];
    const double d3 = dot(ab, bp), d4 = dot(ac, bp);
    if (d3 >= 0 && d4 <= d3) { for (int k = 0; k < 3; ++k) out[k] = b[k]; return; }
    const double vc = d1 * d4 - d3 * d2;
    if (vc <= 0 && d1 >= 0 && d3 <= 0) {
        const double t = d1 / (d1 - d3);
        for (int k = 0; k < 3; ++k) out[k] = a[k] + t * ab[k];
        return;
    }
    double cp[3];
    for (int k = 0; k < 3; ++k) cp[k] = p[k] - c[k];
    const double d5 = dot(ab, cp), d6 = dot(ac, cp);
    if (d6 >= 0 && d5 <= d6) { for (int k = 0; k < 3; ++k) out[k] = c[k]; return; }
    const double vb = d5 * d2 - d1 * d6;
    if (vb <= 0 && d2 >= 0 && d6 <= 0) {
        const double t = d2 / (d2 - d6);
        for (int k = 0; k < 3; ++k) out[k] = a[k] + t * ac[k];
        return;
    }
    const double va = d3 * d6 - d5 * d4;
    if (va <= 0 && (d4 - d3) >= 0 && (d5 - d6) >= 0) {
        const double t = (d4 - d3) / ((d4 - d3) + (d5 - d6));
        for (int k = 0; k < 3; ++k) out[k] = b[k] + t * (c[k] - b[k]);
        return;
    }
    const double den = 1.0 / ((va + vb) + vc);
    const double s = vb * den, t = vc * den;
    for (int k = 0; k < 3; ++k) out[k] = (a[k] + ab[k] * s) + ac[k] * t;
}

__global__ __launch_bounds__(256) void k_hits(const unsigned long long *__restrict__ zbuf, int H, int W,
                                              const uint8_t *__restrict__ mask, float min_depth,
                                              const float *__restrict__ V, const int64_t *__restrict__ F,
                                              Cam inv, float *__restrict__ loc, int64_t *__restrict__ face) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= H * W) return;
    const unsigned long long key = zbuf[i];
    face[i] = -1;
    if (key == ~0ull || !mask[i]) return;
    const float z = __uint_as_float((uint32_t)(key >> 32));
    if (!(z >= min_depth)) return;
    const int64_t f = (int64_t)(key & 0xffffffffull);
    const int py = i / W, px = i - py * W;
    // depth2xyzmap (Utils.py:219-231): f64 arithmetic, f32 result
    const float xc = (float)(((double)px - inv.cx) * (double)z / inv.fx);
    const float yc = (float)(((double)py - inv.cy) * (double)z / inv.fy);
    const double pc[3] = {xc, yc, (double)z};
    double p[3];
    for (int k = 0; k < 3; ++k) p[k] = ((inv.R[3 * k] * pc[0] + inv.R[3 * k + 1] * pc[1]) + inv.R[3 * k + 2] * pc[2]) + inv.t[k];
    double a[3], b[3], c[3], q[3];
    for (int k = 0; k < 3; ++k) {
        a[k] = V[F[f * 3] * 3 + k];
        b[k] = V[F[f * 3 + 1] * 3 + k];
        c[k] = V[F[f * 3 + 2] * 3 + k];
    }
    closest_on_tri(p, a, b, c, q);
    for (int k = 0; k < 3; ++k) loc[(size_t)i * 3 + k] = (float)q[k];
    face[i] = f;
}

__device__ __forceinline__ int64_t texel_flat(const float *uv, int TW) {
    const int64_t x = (int64_t)rint(uv[0]), y = (int64_t)rint(uv[1]);   // torch.round: half to even
    return y * (TW - 1) + x;
}

__global__ __launch_bounds__(256) void k_tex_first(const float *__restrict__ uvs, int64_t M, int TW,
                                                   int64_t n_first, int32_t *__restrict__ first) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= M) return;
    const int64_t fl = texel_flat(uvs + k * 2, TW);
    if (fl >= 0 && fl < n_first) atomicMin(&first[fl], (int32_t)k);
}

__global__ __launch_bounds__(256) void k_tex_add(const float *__restrict__ uvs, const int32_t *__restrict__ pix,
                                                 int64_t M, const float *__restrict__ img, int TH, int TW,
                                                 int64_t n_first, int32_t *__restrict__ first,
                                                 float *__restrict__ tex, float *__restrict__ wtex) {
    const int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (k >= M) return;
    const int64_t fl = texel_flat(uvs + k * 2, TW);
    if (fl < 0 || fl >= n_first || first[fl] != (int32_t)k) return;
    first[fl] = 0x7fffffff;                 // reset for the next frame (only the winner writes)
    const int64_t ux = fl % (TW - 1), uy = fl / (TW - 1);
    if (uy >= TH) return;                   // (W-1)-stride alias of the last texel: outside the image
    const float *col = img + (size_t)pix[k] * 3;
    float *t = tex + ((size_t)uy * TW + ux) * 3;
    t[0] += col[0];
    t[1] += col[1];
    t[2] += col[2];
    wtex[(size_t)uy * TW + ux] += 1.f;
}

static Cam make_cam(const double *T, const double *K) {
    Cam c;
    for (int r = 0; r < 3; ++r) {
        for (int k = 0; k < 3; ++k) c.R[3 * r + k] = T[4 * r + k];
        c.t[r] = T[4 * r + 3];
    }
    c.fx = K[0]; c.fy = K[4]; c.cx = K[2]; c.cy = K[5];
    return c;
}

}  // namespace nof

using namespace nof;

extern "C" {

int nof_raster_faces(const float *V, const int64_t *F, int64_t n_faces, const double *ob_in_cam, const double *K,
                     int32_t H, int32_t W, double znear, double zfar, uint64_t *zbuf, void *stream) {
    if (n_faces < 0 || H <= 0 || W <= 0 || !ob_in_cam || !K || !zbuf || (n_faces > 0 && (!V || !F)))
        return set_error(NOF_EINVAL, "raster_faces: bad arguments");
    if (n_faces >= (1ll << 32)) return set_error(NOF_EINVAL, "raster_faces: more than 2^32 faces");
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(zbuf, 0xff, (size_t)H * W * 8, s) != hipSuccess)
        return set_error(NOF_ELAUNCH, "raster_faces: memset failed");
    if (n_faces == 0) return 0;
    hipLaunchKernelGGL(k_raster, dim3(div_up(n_faces, 256)), dim3(256), 0, s, V, F, n_faces, make_cam(ob_in_cam, K),
                       H, W, znear, zfar, (unsigned long long *)zbuf);
    return check_launch("raster_faces");
}

int nof_texture_hits(const uint64_t *zbuf, int32_t H, int32_t W, const uint8_t *mask, float min_depth, const float *V,
                     const int64_t *F, const double *cam_in_ob, const double *K, float *hit_locations,
                     int64_t *hit_face_ids, void *stream) {
    if (H <= 0 || W <= 0 || !zbuf || !mask || !V || !F || !cam_in_ob || !K || !hit_locations || !hit_face_ids)
        return set_error(NOF_EINVAL, "texture_hits: bad arguments");
    hipLaunchKernelGGL(k_hits, dim3(div_up((uint64_t)H * W, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const unsigned long long *)zbuf, H, W, mask, min_depth, V, F, make_cam(cam_in_ob, K),
                       hit_locations, hit_face_ids);
    return check_launch("texture_hits");
}

int nof_texture_accumulate(const float *uvs, const int32_t *pix, int64_t n_hits, const float *colors, int32_t tex_h,
                           int32_t tex_w, int32_t *first, float *tex, float *weight, void *stream) {
    if (n_hits < 0 || tex_h <= 0 || tex_w <= 1 || !first || !tex || !weight || (n_hits > 0 && (!uvs || !pix || !colors)))
        return set_error(NOF_EINVAL, "texture_accumulate: bad arguments");
    if (n_hits >= (1ll << 31)) return set_error(NOF_EINVAL, "texture_accumulate: too many hits");
    if (n_hits == 0) return 0;
    hipStream_t s = (hipStream_t)stream;
    const int64_t n_first = (int64_t)tex_h * (tex_w - 1) + tex_w;
    hipLaunchKernelGGL(k_tex_first, dim3(div_up(n_hits, 256)), dim3(256), 0, s, uvs, n_hits, tex_w, n_first, first);
    hipLaunchKernelGGL(k_tex_add, dim3(div_up(n_hits, 256)), dim3(256), 0, s, uvs, pix, n_hits, colors, tex_h, tex_w,
                       n_first, first, tex, weight);
    return check_launch("texture_accumulate");
}

}  // extern "C"
