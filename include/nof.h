/*
 * nof.h — C ABI of the MI355X-native neural-object-field (NOF) trainer.
 *
 * Every entry point takes plain device pointers, sizes and a HIP stream
 * (hipStream_t passed as void*; NULL = legacy default stream), launches
 * asynchronously on that stream, keeps no state between calls and returns a
 * nof_status. Callers pre-allocate every output (the reference's ownership
 * convention, grid.py:54-59,86-91 / nerf_runner.py:1006). On failure the call
 * returns non-zero and nof_last_error() describes it (the reference raises
 * c10::Error / std::runtime_error -> Python RuntimeError; the Python shims in
 * bundlesdf_amd/ convert a non-zero status into RuntimeError).
 *
 * Group 1 (B1 in SURVEY.md §8b) replaces the reference's torch-extension
 * entry points one-for-one; group 2 is the fused training step the trainer
 * (bundlesdf_amd/nerf_runner.py) drives.
 */
#ifndef NOF_H
#define NOF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    NOF_OK = 0,
    NOF_EINVAL = 1,   /* bad argument (shape / dtype / unsupported C or D) */
    NOF_ELAUNCH = 2,  /* kernel launch failed */
    NOF_EDEVICE = 3   /* device-side error flag raised */
} nof_status;

typedef enum { NOF_F32 = 0, NOF_F16 = 1 } nof_dtype;

#define NOF_MAX_LEVELS 32

/* Thread-local description of the last failure (static storage). */
const char *nof_last_error(void);
/* Library build identification string (arch, build flags). */
const char *nof_version(void);

/* ------------------------------------------------------------------ group 1
 * Drop-in replacements of the reference extension entry points.
 */

/* Replaces gridencoder.grid_encode_forward
 *   (mycuda/torch_ngp_grid_encoder/gridencoder.h:23, gridencoder.cu:447-470).
 * inputs [B,D] f32 in [0,1]; embeddings [sO,C] (dtype); offsets [L+1] i32;
 * outputs [L,B,C] (dtype); dy_dx [B,L*D*C] (dtype) when calc_grad_inputs.
 * C in {1,2,4,8}, D in {1..5}; gridtype 0 = hash, 1 = tiled. */
int nof_grid_encode_forward(const float *inputs, const void *embeddings, const int32_t *offsets, void *outputs,
                            uint32_t B, uint32_t D, uint32_t C, uint32_t L, float S, uint32_t H,
                            int calc_grad_inputs, void *dy_dx, uint32_t gridtype, int align_corners,
                            int dtype, void *stream);

/* Replaces gridencoder.grid_encode_backward
 *   (gridencoder.h:24, gridencoder.cu:472-502).
 * grad [L,B,C]; grad_embeddings [sO,C] zero-initialised by the caller;
 * grad_inputs [B,D] (dtype) when calc_grad_inputs. Accumulation into
 * grad_embeddings uses device atomics (order-dependent low bits, as in the
 * reference). */
int nof_grid_encode_backward(const void *grad, const float *inputs, const void *embeddings,
                             const int32_t *offsets, void *grad_embeddings, uint32_t B, uint32_t D, uint32_t C,
                             uint32_t L, float S, uint32_t H, int calc_grad_inputs, const void *dy_dx,
                             void *grad_inputs, uint32_t gridtype, int align_corners, int dtype, void *stream);

/* Replaces common.sampleRaysUniformOccupiedVoxels (mycuda/common.h:28,
 * common.cu:107-125). z_in_out [N,K,2], z_sampled [N,S], z_vals [N,S] f32.
 * Malformed rays (the reference prints and spins forever, common.cu:66-71,
 * 87-92) leave z unchanged and increment *error_count (device int, may be
 * NULL). */
int nof_sample_rays_uniform_occupied_voxels(const float *z_in_out, const float *z_sampled, float *z_vals,
                                            int32_t n_rays, int32_t n_intersect, int32_t n_samples,
                                            int32_t *error_count, void *stream);

/* Replaces common.postprocessOctreeRayTracing (common.h:29, common.cu:151-167).
 * out [n_rays, max_intersections, 2] f32 must be zeroed by the caller (the
 * reference allocates it itself, on cuda:0 — common.cu:158; the Python shim
 * allocates on the input's device). */
int nof_postprocess_octree_ray_tracing(const int64_t *ray_index, const float *depth_in_out,
                                       const int64_t *unique_intersect_ray_ids, const int64_t *start_poss,
                                       int64_t n_hits, int64_t n_unique, int32_t max_intersections,
                                       float *out, void *stream);

/* Replaces common.rayColorToTextureImageCUDA (common.h:30, common.cu:188-238):
 * barycentric UV of each hit point. F [Fc,3] i64, V [Nv,3] f32,
 * hit_locations [M,3] f32, hit_face_ids [M] i64, uvs_tex [Nv,2] f32,
 * uvs [M,2] f32 (output). */
int nof_ray_color_to_texture_uv(const int64_t *F, const float *V, const float *hit_locations,
                                const int64_t *hit_face_ids, const float *uvs_tex, float *uvs, int64_t n_hits,
                                void *stream);

/* ------------------------------------------------------------------ group 2
 * Fused training step (bundlesdf_amd/nerf_runner.py). Replaces the per-step
 * work of NerfRunner.train_loop (nerf_runner.py:677-762): kaolin ray trace
 * (Utils.py:443-475), the two samplers (nerf_runner.py:979-1080), run_network
 * (:1226-1303), raw2outputs (:1131-1168), the losses (nerf_helpers.py:367-399)
 * and their backward, and Adam.
 */

/* Per-level float32 scale and resolution exactly as gridencoder.cu:155-156
 * computes them (host function, no device work). */
void nof_level_params(uint32_t L, float S, uint32_t H, float *scales, uint32_t *resolutions);

/* Dense-occupancy ray trace at grid resolution N over [-1,1]^3 (replaces
 * kaolin unbatched_raytrace + postprocessOctreeRayTracing, Utils.py:457-470).
 * occ [N^3] u8 (x fastest); rays_o/rays_d [R,3] f32 world (unit d);
 * out [R,Kmax,2] f32 (zero-padded), counts [R] i32 (may be NULL). */
int nof_octree_ray_trace(const uint8_t *occ, int32_t N, const float *rays_o, const float *rays_d, int32_t R,
                         int32_t Kmax, float *out, int32_t *counts, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NOF_H */
