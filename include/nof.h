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

#include <stddef.h>
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

/* Per-step schedule on the device (hipGraph replay). The step's scalars — the
 * truncation band of get_truncation (nerf_runner.py:661-674), the learning rates
 * of schedule_lr (:577-581, applied every 10 steps, :761-762) and the sampling
 * seeds — are functions of the global step. nof_step_schedule reads the device
 * step counter *step, writes the block for that step into *out and advances
 * *step, all on `stream`; the consumers below take the block by device pointer
 * (nullable: NULL = use their scalar arguments), so one captured graph replays
 * every step with the schedule of the step it runs as. */
typedef struct {
    double lr0, lr1;          /* Adam learning rates of group 0 (table + MLP + features) / group 1 (poses) */
    float trunc;              /* truncation * sc_factor */
    uint32_t seed;            /* field-pass sampling seed: step * 0x9E3779B1 + seed_base */
    uint32_t batch_seed;      /* nof_sample_batch seed: batch_seed_base + step */
    int32_t step;             /* the global step this block belongs to */
} nof_step_params;

typedef struct {
    double lrate, lrate_pose, decay_rate;   /* cfg lrate, lrate_pose, decay_rate */
    double trunc, trunc_start, sc_factor;   /* cfg trunc, trunc_start, sc_factor */
    int32_t trunc_decay;      /* 0: constant, 1: 'linear', 2: 'exp' (cfg trunc_decay_type) */
    int32_t n_step;           /* cfg n_step */
    uint32_t seed_base, batch_seed_base;
} nof_schedule_desc;

int nof_step_schedule(const nof_schedule_desc *d, int32_t *step, nof_step_params *out, void *stream);

/* Step 1 — batch gather + ray setup + ray trace + interval clipping
 * (render_rays :1043-1059, Utils.py:443-475, sample_rays_uniform_occupied_voxels
 * :984-1001). pool [N_pool,12] f32 ray table (reference column order); ids [R]
 * (NULL: the first R rows of pool are the batch); tf [F,16] world_from_cam per
 * frame (pose correction applied); rays_out [R,12] (written when ids != NULL);
 * intervals [R,Kmax,2] f32 in z units: the ray's counts[r] intervals, then (when counts[r] <
 * Kmax) one zero entry ending the list — the entries after it are not written; totals [R];
 * counts [R] (nullable). */
int nof_trace_rays(const float *pool, const int32_t *ids, int32_t R, const float *tf, const uint8_t *occ, int32_t N,
                   int32_t Kmax, float near_sc, float far_sc, float trunc, float *rays_out, float *intervals,
                   float *totals, int32_t *counts, const nof_step_params *sp, void *stream);

/* nof_trace_rays on the step's batch of an epoch permutation (NerfRunner's DataLoader,
 * nerf_runner.py:90-107: consecutive R-id slices of one randperm): ids = perm + (sp->step -
 * *epoch_step0) * R, where *epoch_step0 (device int) is the global step that drew the epoch's first
 * slice. Both are read on the device, so one captured graph replays every step of an epoch with no
 * per-step id copy; the caller rewrites perm (same buffer) and *epoch_step0 only when a new epoch
 * starts. sp and epoch_step0 must not be NULL. The caller keeps (step - *epoch_step0 + 1) R <= the
 * permutation's length. */
int nof_trace_rays_epoch(const float *pool, const int32_t *perm, const int32_t *epoch_step0, int32_t R,
                         const float *tf, const uint8_t *occ, int32_t N, int32_t Kmax, float near_sc, float far_sc,
                         float trunc, float *rays_out, float *intervals, float *totals, int32_t *counts,
                         const nof_step_params *sp, void *stream);

/* Throughput-mode ray selection: rays_per_frame uniform draws (with replacement)
 * inside each frame's contiguous pool segment [frame_start[f], frame_start[f+1]),
 * written per frame in ascending pool order (rays_per_frame <= 4096). */
int nof_sample_batch(const int64_t *frame_start, int32_t F, int32_t rays_per_frame, uint32_t seed, int32_t *ids,
                     const nof_step_params *sp, void *stream);

/* Packs the NeRFSmall parameters (flat, MLP_KEYS order, 9107 f32) into MFMA
 * A-operand fragments (frags, mlp_dtype) and a [5][64] bias image using the
 * index table of bundlesdf_amd/mlp_layout.py. */
int nof_pack_mlp(const float *mlp, const int32_t *idx, int32_t n_frag_elems, int32_t n_bias, void *frags,
                 float *bias, int mlp_dtype, void *stream);

/* Step 2 — the fused field pass: sampling, encode, MLP (MFMA), compositing,
 * losses and the full backward. Accumulates (does not zero) grad_table and
 * grad_mlp; zeroes loss_acc [144] and then writes it; writes ray_grad [R,12] =
 * dL/d tf[frame][0:3,0:4] per ray. All gradients are multiplied by *loss_scale
 * (GradScaler). */
typedef struct {
    const float *rays;        /* [R,12] */
    const float *tf;          /* [F,16] */
    const float *intervals;   /* [R,Kmax,2] */
    const float *totals;      /* [R] */
    const float *t_rand;      /* [R,S] stratification draws, or NULL (counter RNG from seed) */
    uint32_t seed;
    int32_t R, Kmax, N_oct, N_dep, S, perturb;
    float near_sc, far_sc, trunc, neg_trunc_ratio, sdf_lambda, fs_sdf, first_frame_weight;
    float rgb_weight, fs_weight, empty_weight, trunc_weight;
    const float *loss_scale;  /* device scalar */
    const void *table;        /* [T,2] table_dtype (the fp16 mirror under amp) */
    const float *levels;      /* [L,4] from nof_level_table: scale, res, row offset, rows (int bits) */
    uint32_t L, C, D;
    int32_t table_dtype, mlp_dtype;
    const void *frags;        /* nof_pack_mlp output */
    const float *bias;
    float *grad_table;        /* [T,2] f32 (fp32 mode) */
    void *grad_table16;       /* [T,2] f16 (amp mode: packed fp16x2 atomics, as the reference's __half2 path) */
    float *grad_mlp;          /* [9107 + 64*n_ff] f32 (mlp_layout.offsets) */
    float *ray_grad;          /* [R,12] f32 */
    float *loss_acc;          /* [144] f32: rgb, fs (free space), empty, sdf — normalised, unscaled;
                                 [4] samples inside the box, [5] samples through the backward, [6..7] not written
                                 (FusedStep puts reg_features in [6] when frame_features > 0,
                                 pose_reg in [7] when pose_reg_weight > 0);
                                 [8 + 2i], [9 + 2i] (i < 64): HBM scatter atomics (table flush,
                                 probe overflow), spread over 64 counters — sum them (count_atomics);
                                 [136..139] executed tiles: sigma net, colour net, colour / sigma-only
                                 backward records; [140] fs_rgb loss (the reference's unweighted metric,
                                 train_loop :730; the loss adds fs_rgb_weight times it); [141..143] not written */
    float *dbg_z;             /* optional [R,S] */
    float *dbg_raw;           /* optional [R,S,4] (rgb logits, sdf) */
    uint8_t *dbg_valid;       /* optional [R,S] */
    float *dbg_rgb;           /* optional [R,3] */
    int32_t blocks_per_cu;    /* reserved (the removed per-ray forward kernel's grid); ignored */
    int32_t ablate;           /* timing-only ablation bits; must be 0 (results are wrong otherwise) */
    void *workspace;          /* nof_field_workspace_bytes(R, S, mlp_dtype) bytes, caller-owned */
    int32_t scatter_slots;    /* LDS hash slots per wave for the table-gradient scatter (0 -> 512; power of two, 64..2048) */
    int32_t n_ff;             /* cfg frame_features (0..3): FeatureArray channels fed to the colour net
                                 (nerf_runner.py:221,234-235,1268-1277); 0 = none */
    const float *ff;          /* [F, n_ff] f32 FeatureArray.data, or NULL */
    float *grad_ff;           /* [F, n_ff] f32 gradient (accumulated, scaled by *loss_scale), or NULL */
    float fs_rgb_weight;      /* cfg fs_rgb_weight (train_loop :728-731): 0 = off; > 0 adds
                                 fs_rgb_weight * mean(((sigmoid(rgb logits) - 1) * front)^2 * sample_weights),
                                 the unweighted mean in loss_acc[140] */
    int32_t xcd_order;        /* bit 0: k_encode, bit 1: k_scatter take their blocks in XCD-contiguous order
                                 (each XCD's L2 serves a contiguous range of the batch); 0: dispatch order */
    const nof_step_params *step_params;   /* device, nullable: trunc and seed from the block (graph replay) */
    int32_t skip_pose_grad;   /* 1: poses frozen (cfg optimize_poses = 0): no dL/dtf — the reference's grid
                                 backward then skips dy_dx (inputs need no grad), so k_scatter skips the
                                 corner re-gather and ray_grad is not written */
    int32_t scatter_levels_per_wave; /* 0: by batch size (a wave per ray from 192 K rays, 8 levels
                                        per wave from 48 K, 4 from 8 K, else 2); n: scatter waves take
                                        n levels of a ray */
    void *table_quads;        /* amp, optional (NULL: unused): 16 B per table row (n_rows = the last level's
                                 offset + size), rebuilt from `table` at the start of every field pass with
                                 R >= quads_min_rays; row r of a dense level holds the fp16 pairs of rows
                                 {r, r+1, r+rs, r+rs+1} (rs = res + 1), so k_encode reads a cell's 8
                                 corners in two 16-B loads (z, z+1) instead of four 8-B pair loads */
    int64_t table_rows;       /* rows of `table` (= table_quads' length in 16-B records) */
    int32_t quads_min_rays;   /* batch size from which table_quads is used (0 -> 32768, the measured break-even
                                 of its per-step rebuild); tests lower it to run the headline's quad encode on
                                 oracle-sized batches */
    int32_t scatter_kernel;   /* table-gradient scatter: 0 / 2 the run-scan k_scatter (lanes over samples, DPP
                                 segmented scan; scatter_levels_per_wave). 1 (level-serial), 3 (hybrid) and 4
                                 (paired run-scan) were measured slower and removed: NOF_EINVAL */
    int32_t scatter_waves_per_ray; /* reserved (the removed level-serial scatter); ignored */
    int32_t scatter_ls_levels; /* reserved (the removed hybrid scatter); ignored */
    int32_t encode_sigma;     /* 0 / 1: the sigma net (layers 1-2) runs inside the encode kernel on the tile it
                                 just encoded (sdf, sdf-loss terms, flags, colour-net input; features stored only
                                 for backward tiles), the colour net runs tile-parallel over the colour tiles
                                 (k_colour) and a thread per ray composites and finishes the losses
                                 (k_ray_final). 2 and 3 (per-ray forward layouts) were removed: NOF_EINVAL */
    int32_t bwd_flush;        /* amp MLP backward weight-gradient flush: 0 / 2 (default) summed over the 8-wave
                                 block first (one atomic per element per block), 1 one atomic per element per wave */
    int32_t count_atomics;    /* 1: the scatter kernels count their HBM atomics (table flush, probe overflow) into
                                 loss_acc[8..135] (diagnostics); 0: those words stay zero */
    int32_t scatter_flat;     /* reserved, must be 0 (the removed item-list scatter) */
    int32_t compact_per_block; /* k_compact flags per block: 0 by batch size (4096 from 262,144 tiles, where each
                                  thread reads 16 flags with one 16-B load; else 512), or a multiple of 256 in
                                  [256, 4096] — the tests force 4096 on small batches to run the 16-flag path */
    int32_t encode_group;     /* k_encode levels whose corner gathers a lane keeps in flight together: 0 by batch
                                 size (1 from 8,192 rays, where 8 waves per SIMD hide the gathers; more below,
                                 where the grid is too small to), or 1, 2, 4 */
    int32_t quads_prebuilt;   /* 1: the caller rebuilt table_quads for this step with nof_quad_mirror (same
                                 descriptor), ordered before this call (e.g. on a side stream joined by an
                                 event, overlapping the prologue and trace); 0: nof_field_step rebuilds it */
    int32_t mlp_pass1_tiles;  /* reserved, 0 or 1 (one tile per wave): several tiles per wave iteration (k_mlp_bwd_s1)
                                 were measured slower and removed — other values: NOF_EINVAL */
    int32_t scatter_fuse_levels; /* reserved, 0 or 1: level-fused scatter chunks (a level's partial last chunk
                                    continued with the next level's samples) were measured slower and removed */
    int32_t encode_wpb;       /* reserved, 0 or 8: 16-wave encode blocks were measured slower and removed */
} nof_field_desc;

/* Launches on `stream`: k_ray_ctx (one 128-B context record per ray: direction,
 * target, pose rows, view direction, depth, interval total, frame), [k_quad_mirror
 * (amp, large batches)], k_encode (one wave per 32-sample tile: sampling +
 * multires encode + sigma net on MFMA, sdf-loss terms; flags the tiles whose
 * backward is non-zero and hands them per-sample loss terms through the
 * workspace), k_compact (lists of the backward and colour tiles), k_colour
 * (persistent waves over the colour tiles: colour net on MFMA), k_ray_final (a
 * thread per ray: compositing, losses), k_mlp_bwd (two persistent passes over
 * the backward list: MFMA MLP backward with the weight / bias gradients
 * accumulated in registers, and dL/dfeature; amp takes the weight gradients'
 * K = samples operands from LDS transposes), k_scatter (a wave per (ray, level
 * group): table-gradient scatter + input gradient). */
int nof_field_step(const nof_field_desc *desc, void *stream);

/* The xy-quad mirror rebuild of nof_field_step (table -> table_quads), as its own launch: reads
 * table, levels, L, C, R, table_quads, table_rows, quads_min_rays and the dtypes of desc; a no-op
 * when the step would not use the mirror. Lets the caller overlap it with the work before the
 * field pass (the step then runs with quads_prebuilt = 1). No reference counterpart: the quad
 * mirror is this library's layout for the encode's corner gathers (gridencoder.cu:145-205). */
int nof_quad_mirror(const nof_field_desc *desc, void *stream);

/* SDF query (replaces run_network_density, nerf_runner.py:1306-1346, as used
 * by extract_mesh :1349-1382): clip to [-1,1], multires encode, sigma net.
 * Point mode: points [n,3] f32. Grid mode (points NULL): the nx*ny*nz points
 * (gx[i], gy[j], gz[k]) in meshgrid 'ij' order. occ [occ_n^3] u8 (x fastest,
 * nullable): points in empty voxels read 1.0, as extract_mesh fills them.
 * table / level_table / frags / bias as for nof_field_step (amp: fp16 table
 * mirror + fp16 fragments). sdf [n] f32 output. */
int nof_query_sdf(const void *table, int32_t table_dtype, const float *level_table, uint32_t L, const void *frags,
                  const float *bias, int32_t mlp_dtype, int32_t mlp_in, const float *points, int64_t n,
                  const float *gx, const float *gy, const float *gz, int32_t nx, int32_t ny, int32_t nz,
                  const uint8_t *occ, int32_t occ_n, float *sdf, void *stream);

/* Pose corrections on the device (replaces PoseArray.get_matrices,
 * nerf_helpers.py:127-154, and tf = T @ c2w, nerf_runner.py:1050-1052, with
 * their autograd). data [F,6] f32 (PoseArray.data); c2w [F,4,4] f32;
 * max_rot_rad = max_rot * pi / 180. Writes tf_out [F,4,4] and the Jacobian
 * jac [F,12,6] of tf[:3,:4] w.r.t. data (frame 0 is the identity, zero
 * Jacobian). */
int nof_pose_forward(const float *data, const float *c2w, int32_t F, float max_trans, float max_rot_rad,
                     float *tf_out, float *jac, void *stream);

/* The step prologue in one launch: nof_step_schedule (sched nullable: skipped), nof_pose_forward
 * and nof_pack_mlp with the same arguments and results (graph replay: one kernel node instead of
 * three). */
int nof_step_prologue(const nof_schedule_desc *sched, int32_t *step, nof_step_params *sp_out, const float *data,
                      const float *c2w, int32_t F, float max_trans, float max_rot_rad, float *tf_out, float *jac,
                      const float *mlp, const int32_t *idx, int32_t n_frag_elems, int32_t n_bias, void *frags,
                      float *bias, int mlp_dtype, void *stream);

/* Pose gradient: fg[F,12] (scratch: zero on entry, left zero) = per-frame sum of
 * ray_grad [R,12] over the rays' frame ids (rays [R,12], column 8); grad_pose [F,6]
 * += jac^T fg. F <= 1024. */
int nof_pose_backward(const float *ray_grad, const float *rays, int32_t R, const float *jac, int32_t F, float *fg,
                      float *grad_pose, void *stream);

/* Workspace bytes nof_field_step needs (features, feature gradients, z, tile
 * flags, the backward tile list, per-ray / per-tile hand-off records, per-ray
 * context records). */
size_t nof_field_workspace_bytes(int32_t R, int32_t S, int32_t mlp_dtype);

/* Byte offsets of the workspace sections, in this order: feat, dfeat, zbuf, tile_bwd (tile
 * flags), tile_sid (backward tile list), n_tiles (list counters + loss rows), ray_aux, tile_aux,
 * rctx, gmask, rrec, ctile (colour tile list), and the total (= nof_field_workspace_bytes) —
 * NOF_WS_SECTIONS values into offsets[n]. For host readers of the tile lists / counters. */
#define NOF_WS_SECTIONS 13
int nof_field_workspace_offsets(int32_t R, int32_t S, int32_t mlp_dtype, uint64_t *offsets, int32_t n);

/* Per-kernel timing of nof_field_step: when enabled, every call records HIP
 * events on its stream around its 4 kernels (encode, mlp, scatter, dw).
 * collect synchronises, writes the summed milliseconds per kernel over the
 * recorded calls (n >= 4) and the number of calls, and resets. */
int nof_field_timing(int32_t enable);
int nof_field_timing_collect(float *ms_sum, int32_t n, int32_t *calls);

/* Host helper: fills the [L,4] level table nof_field_step reads (float32
 * scale/resolution of gridencoder.cu:155-156; offsets from the host copy of
 * the GridEncoder offsets buffer). */
void nof_level_table(uint32_t L, float S, uint32_t H, const int32_t *offsets_host, float *table_host);

/* GradScaler.unscale_ + found-inf check over grads [n] (in place); also
 * checks (without modifying) the fp16 table gradient grads16 [n16]. Entries
 * [f16_lo, f16_hi) of grads are gradients the reference holds in fp16 under
 * autocast (nn.Linear weights / biases): a scaled value beyond the fp16 range
 * (|g| >= 65520) counts as an overflow there, as it would in the reference. */
int nof_unscale_check(float *grads, int64_t n, const float *scale, int32_t *found_inf, const void *grads16,
                      int64_t n16, int64_t f16_lo, int64_t f16_hi, void *stream);

/* Adam over the flat buffer; elements >= group1_start use lr1 (pose group),
 * the rest lr0. t = *step_count + 1 (device counter: steps the GradScaler
 * skipped do not count, as in torch). Zeroes grads; the update is skipped
 * (the zeroing is not) when *found_inf. When mirror_f16 != NULL the first
 * mirror_n updated params are also written as fp16 (amp table mirror) and
 * their gradients are read from grads16 (fp16, still scaled: multiplied by
 * 1 / *scale here) instead of grads. sp (nullable): lr0 / lr1 from the step block.
 * active (nullable, nof_adam_active_bytes(n) bytes, zeroed with the moments): one flag per
 * group of 256 consecutive parameters, set once the group had a non-zero gradient; a group
 * that never had one (m = v = 0) is left exactly as dense Adam leaves it — unchanged —
 * without reading or writing its params / moments. Flags must be 1 for any group whose
 * moments were set from outside (0 only where exp_avg = exp_avg_sq = 0). */
size_t nof_adam_active_bytes(int64_t n);
int nof_adam_step(float *params, float *grads, float *exp_avg, float *exp_avg_sq, int64_t n, int64_t group1_start,
                  double lr0, double lr1, float beta1, float beta2, float eps, const int32_t *step_count,
                  const int32_t *found_inf, void *mirror_f16, int64_t mirror_n, void *grads16, const float *scale,
                  const nof_step_params *sp, uint8_t *active, void *stream);

/* GradScaler.update (growth_factor 2, backoff 0.5, interval 2000 in the
 * reference) when enabled; always advances *step_count unless *found_inf,
 * then clears *found_inf. */
int nof_scaler_update(float *scale, int32_t *growth_tracker, int32_t *found_inf, int32_t *step_count,
                      float growth_factor, float backoff_factor, int32_t growth_interval, int enabled, void *stream);

/* Data-parallel exchange (amp): grads[i] = (float)grads16[i], grads16[i] = 0
 * for i < n, so the table gradient joins the flat fp32 all-reduce bucket
 *  instead of being summed in fp16. */
int nof_grad16_to_f32(void *grads16, float *grads, int64_t n, void *stream);

/* fp32 -> fp16 copy (table mirror initialisation). */
int nof_to_half(const float *src, void *dst, int64_t n, void *stream);

/* ------------------------------------------------------------------ group 3
 * Ray-pool construction. Replaces the host loop of
 * NerfRunner.make_frame_rays (nerf_runner.py:244-314) + compute_near_far_and_
 * filter_rays (:39-65) + ray_box_intersection_batch (nerf_helpers.py:403-446)
 * + the octree filter (:300-312) + the octree-cloud denoise (:175-194 in
 * __init__, :408-423 in add_new_frames) for a batch of consecutive frames.
 */
typedef struct {
    const float *rgb;           /* [F,H,W,3] f32 in [0,1] */
    const float *depth;         /* [F,H,W] f32 (sc-scaled; BAD_DEPTH*sc where invalid) */
    const uint8_t *mask;        /* [F,H,W] u8 (object mask, > 0 = object) */
    const uint8_t *occ_mask;    /* [F,H,W] u8 or NULL (> 0 = occluded: removed after dilation) */
    const double *cam_in_world; /* [F,4,4] f64 row-major, normalised GL camera-to-object poses */
    int32_t F, H, W;
    int32_t first_frame_id;     /* global id of frame 0 of the batch (column 8 = first_frame_id + f) */
    int32_t dilate_first;       /* mask dilation kernel of global frame 0 (100) */
    int32_t dilate_other;       /* of the other frames (60 // down_scale_ratio) */
    float fx, fy, cx, cy;       /* intrinsics (of the down-scaled frames), rounded to f32 */
    float near_sc, far_sc;      /* cfg near*sc_factor, far*sc_factor rounded to f32 (invalid-depth test) */
    double far_sc64;            /* far*sc_factor in f64 (denoise candidate test, on float64 rays) */
    double bbox[6];             /* cfg bounding_box: xyz min, xyz max */
    const uint8_t *occ;         /* [n^3] u8 occupancy at the ray-tracing level (x fastest), NULL = no octree filter */
    int32_t occ_n;
    /* denoise point grid from nof_point_grid_build, cell_start NULL = no denoise */
    const int32_t *cell_start;  /* [cells+1] */
    const double *cell_points;  /* [M,3] f64, grouped by cell */
    double grid_origin[3];
    int32_t grid_dims[3];
    double grid_cell;           /* cell edge; must be >= grid_radius */
    double grid_radius;         /* 0.02 * sc_factor: rays whose depth point is farther from every cloud point are dropped */
    void *workspace;            /* nof_ray_pool_workspace_bytes(F, H, W) bytes */
    float *rays;                /* [F*H*W, 12] f32 output (reference column order), first *n_out rows valid */
    int64_t *n_out;             /* device int64: number of rays written */
} nof_ray_pool_desc;

size_t nof_ray_pool_workspace_bytes(int32_t F, int32_t H, int32_t W);

/* Five launches: row / column mask dilation, per-pixel selection (+ near/far,
 * octree trace, denoise radius test), block-offset scan, ordered compaction.
 * Output rows are in the reference's order (frame-major, then row-major
 * pixels). W <= 4096, H <= 1024. */
int nof_make_frame_rays(const nof_ray_pool_desc *desc, void *stream);

/* Uniform grid of the octree point cloud for the denoise radius test:
 * points [M,3] f64 -> cell_start [cells+1] i32, cell_points [M,3] f64 grouped
 * by cell (cell = clamp(floor((p - origin) / cell), 0, dims-1), x fastest),
 * cell_ids [M] i32 (nullable): input index of each grouped point (the order
 * within a cell is unspecified). workspace: nof_point_grid_workspace_bytes(cells). */
size_t nof_point_grid_workspace_bytes(int64_t n_cells);
int nof_point_grid_build(const double *points, int32_t M, const double *origin, const int32_t *dims, double cell,
                         int32_t *cell_start, double *cell_points, int32_t *cell_ids, void *workspace, void *stream);

/* ------------------------------------------------------------------ group 4
 * Scene-bounds / hand-off point-cloud operators, the
 * device replacements of the open3d / sklearn calls in tool.py:18-39,42-63
 * (compute_scene_bounds_worker, find_biggest_cluster) and bundlesdf.py:160-169.
 */

/* remove_statistical_outlier's per-point statistic (open3d PointCloud::
 * RemoveStatisticalOutliers): mean Euclidean distance to the min(k, n)
 * nearest points, the point itself included (exact selection, f64). */
int nof_knn_mean_dist(const double *points, int32_t n, int32_t k, double *mean_dist, void *stream);

/* DBSCAN (sklearn.cluster.DBSCAN, euclidean, neighbourhoods |p - q| <= eps
 * including p; core = neighbourhood size >= min_samples). labels [n] i32:
 * for points of a cluster the lowest core-point index of the cluster (the
 * point sklearn starts that cluster from), -1 for noise; a border point takes
 * the cluster of its lowest-index core neighbour. Uniform grid of cell eps
 * over the points' bounds (origin, dims: cells per axis, <= 2^26 in total).
 * Synchronises `stream` once per union-find round (few rounds). */
size_t nof_dbscan_workspace_bytes(int32_t n, int64_t n_cells);
/* Voxel down-sampling's averaging (open3d VoxelDownSample, AccumulatedPoint):
 * out[s, :] = mean of vals[perm[i], :] for i in [seg_start[s], seg_start[s+1]),
 * summed in that order in f64. vals [M,C], perm [M] i64 (points sorted by
 * voxel, stable), seg_start [S+1] i64, out [S,C]. */
int nof_segment_mean(const double *vals, int32_t C, const int64_t *perm, const int64_t *seg_start, int32_t S,
                     double *out, void *stream);
int nof_dbscan(const double *points, int32_t n, double eps, int32_t min_samples, const double *origin,
               const int32_t *dims, int32_t *labels, void *workspace, void *stream);

/* ------------------------------------------------------------------ group 5
 * Texture baking from the training images, the device
 * path of NerfRunner.mesh_texture_from_train_images (nerf_runner.py:1467-1541).
 */

/* Depth + face-id z-buffer of a mesh seen by an OpenCV pinhole camera (the
 * reference's pyrender depth pass): zbuf [H*W] u64 = (f32 depth bits << 32 |
 * face), all ones where empty (this call fills it). Pixel centres at integer
 * (u, v); coverage edges inclusive, either winding; faces with a vertex at
 * z <= znear are skipped; depths beyond zfar are dropped. V [Nv,3] f32,
 * F [Fc,3] i64, ob_in_cam [4,4] f64 row-major, K [3,3] f64 row-major. */
int nof_raster_faces(const float *V, const int64_t *F, int64_t n_faces, const double *ob_in_cam, const double *K,
                     int32_t H, int32_t W, double znear, double zfar, uint64_t *zbuf, void *stream);

/* Per pixel of a z-buffer: where depth >= min_depth and mask [H*W] u8 is set,
 * the back-projected point (depth2xyzmap, Utils.py:219-231) moved to the
 * object frame by cam_in_ob [4,4] f64 and snapped to the closest point of the
 * rasterised face (trimesh.proximity.closest_point of the reference, on the
 * face the pixel sees): hit_locations [H*W,3] f32, hit_face_ids [H*W] i64
 * (-1 = no hit). */
int nof_texture_hits(const uint64_t *zbuf, int32_t H, int32_t W, const uint8_t *mask, float min_depth, const float *V,
                     const int64_t *F, const double *cam_in_ob, const double *K, float *hit_locations,
                     int64_t *hit_face_ids, void *stream);

/* nerf_runner.py:1524-1535 for one frame: texel = round-half-even(uvs[k])
 * flattened as y*(tex_w-1)+x (the reference's stride), the first hit k of
 * each texel adds colors[pix[k]] (f32 [*,3]) to tex [tex_h,tex_w,3] and 1 to
 * weight [tex_h,tex_w]. first: i32 [tex_h*(tex_w-1)+tex_w], all 0x7fffffff
 * on entry and on return. */
int nof_texture_accumulate(const float *uvs, const int32_t *pix, int64_t n_hits, const float *colors, int32_t tex_h,
                           int32_t tex_w, int32_t *first, float *tex, float *weight, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NOF_H */
