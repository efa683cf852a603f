// Fused NeRF training step for gfx950 (CDNA4): ray setup + octree ray trace,
// stratified/around-depth sampling, multires grid encode, tiny MLP on MFMA,
// depth-guided compositing, SDF/free-space/colour losses and the complete
// backward pass (MLP weights, hash-table scatter, input gradient -> per-ray
// pose gradient). Replaces the per-step body of NerfRunner.train_loop
// (nerf_runner.py:677-762) — render_rays :1013-1128, the samplers
// :979-1010/:67-87, run_network :1226-1303, raw2outputs :1131-1168,
// get_sdf_loss nerf_helpers.py:382-399 and autograd.
//
// Work decomposition, one stream, no host synchronisation:
//  * k_trace: one lane per ray — DDA through the occupancy grid, intervals
//    converted to z, clipped at depth+trunc, summed.
//  * k_encode: one wave per (ray, 32-sample tile): z, validity, multires
//    encode; lane (sample n = l & 31, half h = l >> 5) handles levels
//    {8s + 4(q>>1) + 2h + (q&1)} — the row set of its MFMA accumulator
//    registers, so the encoding is the layer-1 B operand in place: the sigma
//    net runs on the tile, then the sdf-loss terms, the backward / colour flags
//    and the per-sample loss terms of backward tiles (tile aux).
//  * k_compact: lists of the flagged tiles (backward, colour).
//  * k_colour: persistent waves over the colour tiles (colour net on MFMA);
//    k_ray_final: a thread per ray — compositing and losses.
//  * k_mlp_bwd: two persistent passes over the list: the tile's forward is
//    recomputed, the MFMA backward runs, every weight / bias gradient is
//    accumulated in registers over the wave's tiles (one atomic per element at
//    the end); dL/dfeature, the SH part of the pose gradient. amp:
//    k_mlp_bwd_tr takes the weight gradients' K = samples operands from LDS
//    transposes (mlp_lds.h) instead of swapped-operand recomputes. Both live in
//    field_mlp_bwd.h, included in place below (same translation unit).
//  * k_scatter: one wave per ray: the ray's backward samples compacted, corner
//    re-gather, input gradient, table gradient reduced in registers (DPP) and
//    LDS before one HBM atomic per distinct row; the point part of the pose
//    gradient.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <array>
#include <type_traits>
#include <vector>

#include "nof_device.h"
#include "ray_trace.h"
#include "mlp_lds.h"

#pragma clang fp contract(off)

// Timing-only ablation switches (scripts/ablate.py) exist only in a build with
// -DNOF_ABLATE=1; in the product library every ABL() test is a compile-time false.
#ifndef NOF_ABLATE
#define NOF_ABLATE 0
#endif
#define ABL(bits) (NOF_ABLATE && (a.ablate & (bits)))
#define ABL_HOST(d, bits) (NOF_ABLATE && ((d)->ablate & (bits)))
// level quarter q (levels 4q .. 4q+3) skipped by the scatter (timing build)
#define ABL_SKIPQ(q) ((q) < 2 ? (1 << (23 + (q))) : (1 << (27 + (q))))

namespace nof {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int MLP_N_MAX = 9107 + 64 * 3;   // NeRFSmall(2x64, geo 15, colour 3x64), input <= 32, views 9 (+ <= 3 frame features)
// flat-parameter offsets (MLP_KEYS order, bundlesdf_amd/mlp_layout.py) for input width IN
struct MlpOff {
    int w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, n, in, cin;
    // FF = frame_features: color_net.0 input = [frame features (FF), SH (9), geo (15)] (nerf_runner.py:221,1277)
    __host__ __device__ MlpOff(int IN, int FF = 0) : in(IN), cin(24 + FF) {
        w1 = 0; b1 = 64 * IN; w2 = b1 + 64; b2 = w2 + 16 * 64; w3 = b2 + 16; b3 = w3 + 64 * cin; w4 = b3 + 64;
        b4 = w4 + 64 * 64; w5 = b4 + 64; b5 = w5 + 3 * 64; n = b5 + 3;
    }
};
// fragment ids (bundlesdf_amd/mlp_layout.py)
constexpr int FR_L1 = 0, FR_L2 = 4, FR_L3 = 8, FR_L4 = 12, FR_L5 = 20, FR_B5 = 24, FR_B4 = 26, FR_B3 = 34,
              FR_B2 = 38, FR_B1 = 42, N_FRAGS = 46;
// Cin row k -> column of color_net.0.weight for ff frame features: rows 1..15 geo,
// 16..24 SH, 25..25+ff-1 the ray's frame features (mlp_layout.cin_to_w3_col).
__device__ __forceinline__ int cin_col(int i, int ff) {
    return (i >= 1 && i <= 15) ? ff + 9 + i - 1
                               : ((i >= 16 && i <= 24) ? ff + i - 16 : ((i >= 25 && i < 25 + ff) ? i - 25 : -1));
}
constexpr float SH_C0 = 0.28209479177387814f, SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f, SH_C2_2 = 0.31539156525252005f,
                SH_C2_3 = -1.0925484305920792f, SH_C2_4 = 0.5462742152960396f;

struct FieldArgs {
    const float *rays;        // [R,12] batch (dir3 rgb3 depth mask frame type near far)
    const float *tf;          // [F,16] world_from_cam (pose correction applied), row-major
    const float *intervals;   // [R,Kmax,2] z units
    const float *totals;      // [R]
    float *rctx;              // [R][RCTX] per-ray context records (k_ray_ctx, workspace)
    const float *t_rand;      // [R,S] or null (counter RNG)
    uint32_t seed;
    int R, Kmax, N_oct, N_dep, S;
    int perturb;
    float near_sc, far_sc, trunc, ntr, lambda, fs_sdf, ffw, rgb_w, fs_w, empty_w, trunc_w;
    float fs_rgb_w;           // cfg fs_rgb_weight: colour of front (free-space) samples pulled to white (train_loop :728-731)
    float inv_3R, inv_RS, inv_3RS;
    const float *loss_scale;  // device scalar (GradScaler scale; 1 in fp32 mode)
    const void *table;        // [T,2] (float or half)
    const float4 *levels;     // [L]: scale, res (bits), row offset (bits), rows (bits)
    uint32_t L;
    int mlp_in;               // L*C
    int n_ff;                 // frame_features (0..3): per-frame latent code fed to the colour net
    const float *ff;          // [F, n_ff] f32 (FeatureArray.data)
    float *grad_ff;           // [F, n_ff] f32 (scaled like grad_mlp)
    const void *frags;        // [46][64][8] TM
    const float *bias;        // [5][64]
    float *grad_table;        // [T,2] f32 (fp32 mode)
    __half *grad_table16;     // [T,2] f16 (amp mode: the reference's __half2 gradient, gridencoder.cu:319-327)
    float *grad_mlp;          // [9107] f32
    float *ray_grad;          // [R,12]
    uint32_t *tile_gmask;     // [R*S/32] k_encode -> k_scatter: bit n = sample n of the tile carries a loss gradient
    const uint4 *quads;       // amp, R >= 32 K: xy-quad mirror of the fp16 table (k_quad_mirror), or null
    uint32_t n_rows;          // table rows (the quad mirror's length)
    bool quads_ready;         // the caller rebuilt `quads` for this step (nof_quad_mirror on a side stream)
    float *loss_part;         // [LOSS_COPIES][16] per-wave loss / counter partials (workspace), folded into loss_acc
    float *loss_acc;          // [8 + 128 + 8]: rgb, fs, empty, sdf (normalised), n_valid, n_bwd, -, -; [8 + 2i + {0,1}] HBM scatter atomics (flush, direct), spread; [136..139] work counters
    float *dbg_z;             // [R,S]
    float *dbg_raw;           // [R,S,4]
    uint8_t *dbg_valid;       // [R,S]
    float *dbg_rgb;           // [R,3]
    void *feat;               // [R*S*32] TM features, fragment order (workspace)
    void *dfeat;              // [16][R*S][2] TM dL/dfeature (scaled), level-major (store_dfeat; workspace)
    float *zbuf;              // [R*S] sample z (workspace)
    uint8_t *tile_bwd;        // [R*S/32] tile ran the backward (workspace)
    uint32_t slot_mask;       // scatter LDS hash slots per wave - 1 (power of two)
    int *tile_sid;            // [R*S/32] list of flagged tiles: first sample id | sigma-only bit (k_compact; workspace)
    int *n_tiles;             // device counter of records (workspace)
    float *ray_aux;           // [R][RAY_AUX] k_ray_final -> k_mlp_bwd / k_scatter (workspace)
    float4 *tile_aux;         // [R*S/32][TILE_AUX] per-record masks + loss terms (workspace)
    int ablate;               // timing-only ablation bits (builds with -DNOF_ABLATE=1 only; results invalid otherwise)
    int xcd_order;            // bit 0: k_encode, bit 1: k_scatter blocks in XCD-contiguous order (xcd_block)
    const nof_step_params *sp;   // device step block (graph replay) or null: trunc / seed from it
    int no_dx;                // poses frozen: no input gradient (no corner re-gather, no dL/dtf)
    int scatter_lpw;          // k_scatter levels per wave (L: wave per ray; fewer: waves per (ray, level group))
    float *rrec;              // [R*S/32][TREC] per-tile partial sums (k_encode SIG / k_colour -> k_ray_final; workspace)
    int *ctile_list;          // [R*S/32] colour tiles (flag 1 or 3) as first sample id (k_compact; workspace)
    int bwd_flush;            // k_mlp_bwd_tr weight-gradient flush: 0 by batch size, 1 per wave, 2 block-reduced
    int count_atomics;        // the scatter kernels count their HBM atomics into loss_acc[8..135] (diagnostics)
    int compact_per;          // k_compact flags per block (0: by batch size; tests force the 16-flags-per-thread path)
    int encode_group;         // k_encode levels per lane with gathers in flight together (resolved: 1, 2 or 4)
};

constexpr int LOSS_ACC_COUNTERS = 136;
constexpr int LOSS_ACC_WORDS = 144;   // loss_acc's length (include/nof.h)
// per tile (tile-parallel forward): the tile's partial sums, stored (not added) by k_encode SIG
// (weight sum, valid count, sdf terms, work-counter bits: every in-range tile) and k_colour
// (composited colour, fs_rgb term: colour tiles only); k_ray_final sums a ray's tiles in tile
// order, so the ray's sums are deterministic (raw2outputs' fixed-order sum) — no float atomics
constexpr int TREC = 12;
enum { TR_WSUM = 0, TR_NVALID, TR_LFS, TR_LEM, TR_LSDF, TR_CNT, TR_RACC = 8, TR_LFSR = 11 };
enum { TC_SIG = 1, TC_COL = 2, TC_CRCOL = 4, TC_CRSIG = 8 };   // TR_CNT bits (as an int)
constexpr int LOSS_COPIES = 64, LOSS_SLOTS = 16, LOSS_FOLD_N = 13;
// workspace words zeroed per step: the record counter (+ padding to 16 words) and the loss rows
constexpr uint64_t LOSS_ZERO_WORDS = 16 + (uint64_t)LOSS_COPIES * LOSS_SLOTS;

// The kernels' view of the step's scalars: the device step block when given (one
// captured graph replays every step), else the values the host put in the descriptor.
__device__ __forceinline__ FieldArgs step_args(const FieldArgs &a0) {
    FieldArgs a = a0;
    if (a0.sp) {
        a.trunc = a0.sp->trunc;
        a.seed = a0.sp->seed;
    }
    return a;
}

// The field kernels' FieldArgs (their only kernel argument, at offset 0 of the kernarg segment)
// through a pointer the compiler cannot see through (laundered in the constant address space, so the
// reads stay scalar loads): the reads after it are issued there, not hoisted to the kernel's start
// and held in SGPRs across its gathers
__device__ __forceinline__ const FieldArgs &late_args() {
    auto k = __builtin_amdgcn_kernarg_segment_ptr();   // constant address space: scalar loads
    asm volatile("" : "+s"(k));
    return *(const FieldArgs *)k;
}

// ----------------------------------------------------------------- helpers
__device__ __forceinline__ int acc_row(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }

// Wave reductions on DPP (no LDS traffic): inclusive prefix sums inside each 16-lane
// row (row_shr 1, 2, 4, 8), then row_bcast:15 carries row totals into rows 1 / 3 and
// row_bcast:31 the first half's total into the second half. Must be called with the
// whole wave active (every call site is wave-uniform).
template <int CTRL, int ROWS = 0xf>
__device__ __forceinline__ float dpp_add(float v) {
    return v + __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, ROWS, 0xf, true));
}
__device__ __forceinline__ float row_prefix(float v) {
    v = dpp_add<0x111>(v);   // row_shr:1
    v = dpp_add<0x112>(v);   // row_shr:2
    v = dpp_add<0x114>(v);   // row_shr:4
    return dpp_add<0x118>(v);   // row_shr:8
}
__device__ __forceinline__ float lane_value(float v, int l) {
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), l));
}
__device__ __forceinline__ float wave_sum(float v) {
    v = row_prefix(v);
    v = dpp_add<0x142, 0xa>(v);   // row_bcast:15 -> rows 1, 3
    v = dpp_add<0x143, 0xc>(v);   // row_bcast:31 -> rows 2, 3
    return lane_value(v, 63);
}
// sums of the two 32-lane halves, both returned wave-uniform
__device__ __forceinline__ void half_sums(float v, float &s0, float &s1) {
    v = row_prefix(v);
    v = dpp_add<0x142, 0xa>(v);
    s0 = lane_value(v, 31);
    s1 = lane_value(v, 63);
}

// v_rcp_f32 (1 ulp) instead of an IEEE division: ~10 instructions fewer per call
__device__ __forceinline__ float sigmoidf(float x) { return __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// The dispatcher hands block b to XCD b % 8. xcd_block maps it to a logical
// block so each XCD (own 4 MB L2) works a contiguous range of blocks: with
// frame-major ray batches an XCD then gathers the table rows of ~2 views.
__device__ __forceinline__ int xcd_block(int b, int nb) {
    const int per = nb >> 3, rem = nb & 7, x = b & 7, i = b >> 3;
    return (x < rem ? x * (per + 1) : rem * (per + 1) + (x - rem) * per) + i;
}

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ float rng_uniform(uint32_t seed, uint32_t ray, uint32_t s) {
    uint32_t h = hash32(seed ^ hash32(ray * 0x9E3779B1U + hash32(s + 0x632BE5ABU)));
    return (float)(h >> 8) * (1.0f / 16777216.0f);
}

// torch.linspace(0, 1, n)[i] (two-sided FMA formula of ATen's range factory)
__device__ __forceinline__ float linspace01(int i, int n) {
    if (n == 1) return 0.0f;
    const float step = 1.0f / (float)(n - 1);
    return (i < n / 2) ? __builtin_fmaf(step, (float)i, 0.0f) : __builtin_fmaf(-step, (float)(n - 1 - i), 1.0f);
}

// Fragment types: 8 elements per lane per 16-wide K step.
template <typename TM> struct FragT;
template <> struct FragT<_Float16> { typedef h8v T; };
template <> struct FragT<float> { struct T { float v[8]; }; };

template <typename TM> __device__ __forceinline__ void frag_set(typename FragT<TM>::T &f, int j, float x);
template <> __device__ __forceinline__ void frag_set<_Float16>(h8v &f, int j, float x) { f[j] = (_Float16)x; }
template <> __device__ __forceinline__ void frag_set<float>(FragT<float>::T &f, int j, float x) { f.v[j] = x; }
template <typename TM> __device__ __forceinline__ float frag_get(const typename FragT<TM>::T &f, int j);
template <> __device__ __forceinline__ float frag_get<_Float16>(const h8v &f, int j) { return (float)f[j]; }
template <> __device__ __forceinline__ float frag_get<float>(const FragT<float>::T &f, int j) { return f.v[j]; }
template <typename TM> __device__ __forceinline__ void frag_zero(typename FragT<TM>::T &f) {
#pragma unroll
    for (int j = 0; j < 8; ++j) frag_set<TM>(f, j, 0.f);
}

__device__ __forceinline__ void mma(f16v &acc, const h8v &a, const h8v &b) {
    acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, acc, 0, 0, 0);
}
__device__ __forceinline__ void mma(f16v &acc, const FragT<float>::T &a, const FragT<float>::T &b) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a.v[j], b.v[j], acc, 0, 0, 0);
}

template <typename TM>
__device__ __forceinline__ typename FragT<TM>::T load_frag(const void *frags, int id, int lane) {
    typename FragT<TM>::T f;
    // Opaque per use: keeps the compiler from hoisting all 46 weight
    // fragments out of the ray loop into registers (that costs occupancy).
    asm volatile("" : "+s"(id));
    const TM *p = reinterpret_cast<const TM *>(frags) + ((size_t)id * 64 + lane) * 8;
    if constexpr (sizeof(TM) == 2) {
        f = *reinterpret_cast<const h8v *>(p);
    } else {
        const float4 a = *reinterpret_cast<const float4 *>(p), b = *reinterpret_cast<const float4 *>(p + 4);
        f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w; f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
    }
    return f;
}

__device__ __forceinline__ void acc_init_bias(f16v &acc, const float *bias_row64, int mt, int h) {
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = bias_row64[32 * mt + acc_row(q, h)];
}
__device__ __forceinline__ void acc_zero(f16v &acc) {
#pragma unroll
    for (int q = 0; q < 16; ++q) acc[q] = 0.f;
}
// fp16 pair helpers (packed instructions: one v_cvt_pk_f16_f32 / v_pk_max_f16 /
// v_and_b32 per two elements instead of per-element convert / max / select)
typedef _Float16 h2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ h2v pk_round(float a, float b) { return h2v{(_Float16)a, (_Float16)b}; }
__device__ __forceinline__ void frag_put2(h8v &f, int p, h2v u) { f[2 * p] = u[0]; f[2 * p + 1] = u[1]; }
// fp16 ReLU of a packed pair as a signed 16-bit max with 0: every negative half (sign bit set,
// -0 included) becomes +0, the others stay — max(u, 0) for every non-NaN u, and the result's sign
// bits are always clear (pair_bits relies on it)
__device__ __forceinline__ h2v relu_pk(h2v u) {
    uint32_t r;
    asm("v_pk_max_i16 %0, %1, 0" : "=v"(r) : "v"(__builtin_bit_cast(uint32_t, u)));
    return __builtin_bit_cast(h2v, r);
}
// fp16 ReLU masks are kept per pair: pair P's low half at bit P, its high half at bit
// P + 16 (so a pair's two 0/1 halves, from one v_pk_min_u16, enter with one shift-or).
// the pair's ReLU-derivative bits (u > 0 per half; u is a relu_pk output: +0 or positive)
__device__ __forceinline__ uint32_t pair_bits(h2v u, int P) {
    const uint32_t x = __builtin_bit_cast(uint32_t, u);
    uint32_t y;
    // one packed unsigned min per pair (written as asm: the compiler expands min(x, 1) into
    // per-half compares and selects)
    asm("v_pk_min_u16 %0, %1, %2" : "=v"(y) : "v"(x), "s"(0x00010001u));
    return y << P;
}
constexpr uint32_t MASK_ALL = 0xffffffffu;
// the pair u with the halves whose mask bits (P, P + 16) are clear zeroed: the two bits moved to bits 0
// and 16 (a 0 / 1 factor per half) times the halves' bit patterns by one packed 16-bit integer multiply
// — three instructions where expanding the bits into 0xffff masks and and-ing took four
__device__ __forceinline__ h2v pk_keep(h2v u, uint32_t m, int P) {
    const uint32_t f = (m >> P) & 0x00010001u;
    uint32_t r;
    asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(__builtin_bit_cast(uint32_t, u)), "v"(f));
    return __builtin_bit_cast(h2v, r);
}

// acc registers 8s..8s+7 -> fragment of K step s (optionally ReLU; fp16: rounded, then
// max(., 0) on the packed pair, the same values as rounding max(v, 0))
template <typename TM>
__device__ __forceinline__ void acc_to_frag(const f16v &acc, int s, bool relu, typename FragT<TM>::T &f) {
    if constexpr (sizeof(TM) == 2) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            h2v u = pk_round(acc[8 * s + 2 * p], acc[8 * s + 2 * p + 1]);
            if (relu) u = relu_pk(u);
            frag_put2(f, p, u);
        }
    } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            float v = acc[8 * s + j];
            frag_set<TM>(f, j, relu ? fmaxf(v, 0.f) : v);
        }
    }
}


// wave-uniform data read through the constant address space: scalar loads
typedef const __attribute__((address_space(4))) uint32_t *ConstU32;

// ------------------------------------------------------------- the sampler
// z of sample s of ray r (render_rays :1060-1080 / sample_rays_uniform :67-87
// / sampleRaysUniformOccupiedVoxels common.cu:40-105).
__device__ __forceinline__ float sample_z(const FieldArgs &a, int r, int s, float depth, bool vdepth, float total,
                                          const float *__restrict__ box) {
    int idx, n;
    float near, far;
    bool walk;
    if (s < a.N_oct) { idx = s; n = a.N_oct; near = 0.f; far = total; walk = true; }
    else {
        idx = s - a.N_oct; n = a.N_dep;
        if (vdepth) { near = depth - a.trunc; far = depth + a.trunc * a.ntr; walk = false; }
        else { near = 0.f; far = total; walk = true; }
    }
    auto zlin = [&](int i) {
        const float t = linspace01(i, n);
        return near * (1.f - t) + far * t;
    };
    float z = zlin(idx);
    if (a.perturb) {
        const float zc = z;
        const float lower = (idx == 0) ? zc : .5f * (zc + zlin(idx - 1));
        const float upper = (idx == n - 1) ? zc : .5f * (zlin(idx + 1) + zc);
        const float u = a.t_rand ? a.t_rand[(size_t)r * a.S + s] : rng_uniform(a.seed, (uint32_t)r, (uint32_t)s);
        z = lower + (upper - lower) * u;
        z = fminf(fmaxf(z, near), far);
    }
    // common.cu:40-105 walk (sequential subtraction; exact reference rounding), over the ray's
    // interval list in batches of WB intervals read by one scalar load (box is wave-uniform:
    // every caller passes its wave's ray): each lane runs the same per-interval steps as the
    // reference's loop — rem -= len until rem <= len — as selects on the batch's scalar registers,
    // and the wave leaves once every lane has its interval. (A loop of one dependent scalar load
    // per interval cost 0.28 ms of the headline encode.) Lanes that do not walk are done at once.
    if (!__any(walk)) return z;   // a tile of around-depth samples only
    const ConstU32 bq = (ConstU32)(size_t)box;
    if (__uint_as_float(bq[0]) == 0.f) return walk ? 0.f : z;
    const float eps = 1e-4f;
    float rem = z, res = z, prev_out = 0.f;
    bool done = !walk;
    const int Kmax = a.Kmax;
    constexpr int WB = 8;   // intervals per batch: one 64-B scalar load
    int i = 0;
    for (; i + WB <= Kmax; i += WB) {
        float b[2 * WB];
#pragma unroll
        for (int k = 0; k < 2 * WB; ++k) b[k] = __uint_as_float(bq[2 * i + k]);
#pragma unroll
        for (int j = 0; j < WB; ++j) {
            const float zin = b[2 * j], zout = b[2 * j + 1];
            if (zin == 0.f) return done ? res : ((rem <= eps && i + j >= 1) ? prev_out : 0.f);
            const float len = zout - zin;
            const bool hit = !done && rem <= len;
            res = hit ? zin + rem : res;
            rem = done || hit ? rem : rem - len;
            done = done || hit;
            prev_out = zout;
        }
        if (!__any(!done)) return res;
    }
    for (; i < Kmax; ++i) {   // the last Kmax mod WB intervals, one at a time
        const float zin = __uint_as_float(bq[2 * i]), zout = __uint_as_float(bq[2 * i + 1]);
        if (zin == 0.f) return done ? res : ((rem <= eps && i >= 1) ? prev_out : 0.f);
        const float len = zout - zin;
        const bool hit = !done && rem <= len;
        res = hit ? zin + rem : res;
        rem = done || hit ? rem : rem - len;
        done = done || hit;
        prev_out = zout;
    }
    return done ? res : (rem <= eps ? __uint_as_float(bq[(Kmax - 1) * 2 + 1]) : 0.f);
}

// raw2outputs sdf2weights numerator (nerf_runner.py:1151-1158)
__device__ __forceinline__ float bell_weight(const FieldArgs &a, float depth, float z) {
    if (depth > a.far_sc) return 0.f;
    const float u = (depth - z) / a.trunc;
    float w = sigmoidf(u * a.lambda) * sigmoidf(-u * a.lambda);
    const float dz = z - depth;
    const bool m = (dz <= a.trunc * a.ntr) && (dz >= -a.trunc);
    return m ? w : 0.f;
}

// --------------------------------------------------------------- encoding
// One level of kernel_grid (gridencoder.cu:106-246) for this lane's sample:
// features (C=2) and, when want_d, d feature / d x01 (3 x 2).
struct LevelInfo { float scale; uint32_t res, off, hs; };
__device__ __forceinline__ LevelInfo level_info(const FieldArgs &a, int lv) {
    const float4 v = a.levels[lv];
    return {v.x, __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)};
}
// the same record read through the constant address space (lv wave-uniform): a scalar load
__device__ __forceinline__ LevelInfo level_info_uniform(const FieldArgs &a, int lv) {
    const ConstU32 p = (ConstU32)(size_t)(a.levels + lv);
    return {__uint_as_float(p[0]), p[1], p[2], p[3]};
}

// The fp16 table as a buffer resource: corner-pair loads take a 32-bit byte offset (one shift)
// instead of a 64-bit address per load (the table is < 2 GB)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t table_rsrc(const void *table) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void *>(table), (short)0, 0x7fffffff, 0x00020000);
}
typedef uint32_t u2v __attribute__((ext_vector_type(2)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint2 table_pair16(__amdgpu_buffer_rsrc_t rsrc, uint32_t row) {
    const u2v v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, row * 4u, 0, 0);
    return make_uint2(v.x, v.y);
}

// Dense-level test (res+1)^3 <= rows and the dense row index. _v: in full-rate 24-bit integer
// multiplies (v_mul_u32_u24; v_mul_lo_u32 / 64-bit multiplies issue at quarter rate): rs <=
// 1625 keeps rs^3 < 2^32, and every operand stays below 2^24
// (written as instructions: the compiler otherwise widens them back to v_mul_lo_u32). Per-lane
// level values (k_encode's lane halves); a wave-uniform level keeps scalar arithmetic.
__device__ __forceinline__ uint32_t mul24(uint32_t a, uint32_t b) {
    uint32_t d;
    asm("v_mul_u32_u24 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
    return d;
}
__device__ __forceinline__ uint32_t mad24(uint32_t a, uint32_t b, uint32_t c) {
    uint32_t d;
    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ bool level_dense_v(uint32_t rs, uint32_t hs) {
    return rs <= 1625u && mul24(mul24(rs, rs), rs) <= hs;
}
__device__ __forceinline__ uint32_t dense_base_v(uint32_t off, const uint32_t pg[3], uint32_t rs) {
    return off + pg[0] + mul24(mad24(pg[2], rs, pg[1]), rs);
}
__device__ __forceinline__ bool level_dense(uint32_t rs, uint32_t hs) { return (uint64_t)rs * rs * rs <= hs; }

// Rows of the 8 corners of cell pg (bit d of idx = +1 along d), as
// get_grid_index (gridencoder.cu:65-83). Dense levels ((res+1)^3 <= rows:
// every level at config 2) need one index plus constant offsets; hashed
// levels use grid_row per corner.
__device__ __forceinline__ void corner_rows(const LevelInfo &li, const uint32_t pg[3], uint32_t rows[8]) {
    const uint32_t rs = li.res + 1;
    if (level_dense(rs, li.hs)) {
        // dense: rs^3 <= rows < 2^32, so rs <= 1625 and the 24-bit multiplies are exact
        const uint32_t base = dense_base_v(li.off, pg, rs), rs2 = rs * rs;
#pragma unroll
        for (int idx = 0; idx < 8; ++idx)
            rows[idx] = base + (idx & 1) + ((idx >> 1) & 1 ? rs : 0u) + ((idx >> 2) & 1 ? rs2 : 0u);
    } else {
#pragma unroll
        for (int idx = 0; idx < 8; ++idx) {
            uint32_t pl[3];
#pragma unroll
            for (int d = 0; d < 3; ++d) pl[d] = pg[d] + ((idx >> d) & 1);
            rows[idx] = li.off + grid_row<3>(0, false, li.hs, li.res, pl);
        }
    }
}

// Corner values of one level for this lane's sample (kernel_grid index math).
template <typename TT, bool PAIRED = false>
__device__ __forceinline__ void gather_level(const FieldArgs &a, const LevelInfo &li, const float x01[3], float pos[3],
                                             float e[8][2], uint32_t rows[8]) {
    const TT *tab = reinterpret_cast<const TT *>(a.table);
    uint32_t pg[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        pos[d] = __builtin_fmaf(x01[d], li.scale, 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
    }
    corner_rows(li, pg, rows);
    const uint32_t rs = li.res + 1;
    if (PAIRED && level_dense(rs, li.hs)) {
        // dense level: corners idx and idx+1 (x, x+1) are adjacent rows -> one
        // 2-row load per pair (dword-aligned multi-dword global loads are legal)
#pragma unroll
        for (int idx = 0; idx < 8; idx += 2) {
            const TT *p = tab + (size_t)rows[idx] * 2;
            if constexpr (sizeof(TT) == 4) {
                typedef float f4a __attribute__((ext_vector_type(4), aligned(8)));
                const f4a v = *reinterpret_cast<const f4a *>(p);
                e[idx][0] = v.x; e[idx][1] = v.y; e[idx + 1][0] = v.z; e[idx + 1][1] = v.w;
            } else {
                uint2 v;
                __builtin_memcpy(&v, p, 8);
                const __half2 h0 = __builtin_bit_cast(__half2, v.x), h1 = __builtin_bit_cast(__half2, v.y);
                e[idx][0] = __low2float(h0); e[idx][1] = __high2float(h0);
                e[idx + 1][0] = __low2float(h1); e[idx + 1][1] = __high2float(h1);
            }
        }
    } else {
#pragma unroll
        for (int idx = 0; idx < 8; ++idx) {
            const TT *p = tab + (size_t)rows[idx] * 2;
            if constexpr (sizeof(TT) == 4) {
                const float2 v = *reinterpret_cast<const float2 *>(p);
                e[idx][0] = v.x; e[idx][1] = v.y;
            } else {
                const __half2 v = *reinterpret_cast<const __half2 *>(p);
                e[idx][0] = __low2float(v); e[idx][1] = __high2float(v);
            }
        }
    }
}

template <typename TT>
__device__ __forceinline__ void encode_level(const FieldArgs &a, const LevelInfo &li, const float x01[3], float f[2]) {
    float pos[3], e[8][2];
    uint32_t rows[8];
    gather_level<TT, true>(a, li, x01, pos, e, rows);
    f[0] = 0.f; f[1] = 0.f;
#pragma unroll
    for (int idx = 0; idx < 8; ++idx) {
        float w = 1.f;
#pragma unroll
        for (int d = 0; d < 3; ++d) w *= ((idx >> d) & 1) ? pos[d] : 1 - pos[d];
        f[0] = __builtin_fmaf(w, e[idx][0], f[0]);
        f[1] = __builtin_fmaf(w, e[idx][1], f[1]);
    }
}

// DPP helpers: value of lane n+d (row_shl) / n-d (row_shr) inside the 16-lane
// row, 0 outside it.
template <int CTRL> __device__ __forceinline__ int dpp_i(int v) {
    return __builtin_amdgcn_update_dpp(0, v, CTRL, 0xf, 0xf, true);
}
#define DPP_ROW_SHL(n) (0x100 + (n))
#define DPP_ROW_SHR(n) (0x110 + (n))

// Backward of one level (kernel_grid_backward + kernel_input_backward,
// gridencoder.cu:249-365) for this lane's sample: adds d<g, feature>/d x01
// (the reference's dy_dx, re-gathered, never materialised) to gx and
// accumulates w*g of the 8 corners into the wave's LDS hash table.
//
// MI355X: device float atomics cost one memory-side request per active lane
// (~20 G lane-ops/s chip-wide, same-address lanes are NOT merged), so the
// scatter is reduced twice before it reaches HBM: (1) the lanes hold
// consecutive samples of one ray, so equal cells form contiguous runs — a
// segmented suffix sum over each 16-lane DPP row folds a run into its head;
// (2) heads insert into a per-wave open-addressing table in LDS keyed by the
// global table row, which dedupes across rows, chunks and corner slots for
// the whole ray at this level. flush_table then issues one HBM atomic per
// distinct row. MUST be called by all lanes of the wave (DPP).
constexpr uint32_t SLOT_EMPTY = 0xffffffffu;

// relaxed, wave-local LDS CAS: lets the 8 corner claims of a lane stay in flight together
__device__ __forceinline__ uint32_t lds_cas(uint32_t *p, uint32_t key) {
    uint32_t e = SLOT_EMPTY;
    __hip_atomic_compare_exchange_strong(p, &e, key, __ATOMIC_RELAXED, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return e;   // previous content
}

// LDS row table of one scatter wave. amp (F16V): interleaved slots [key | packed fp16x2 value]
// (8 B; the claim and the add use one address), fp32: keys[mask + 1] then float2 values.
template <bool F16V> __device__ __forceinline__ uint32_t *slot_key(uint32_t *keys, uint32_t s) {
    return keys + (F16V ? 2 * s : s);
}
__device__ __forceinline__ void lds_add_h2(void *vals, uint32_t s, uint32_t packed) {
    // one packed fp16x2 LDS add (the reference's __half2 accumulation class); vals = keys + 1
    __builtin_amdgcn_ds_atomic_fadd_v2f16(
        (__attribute__((address_space(3))) h2v *)(reinterpret_cast<uint32_t *>(vals) + 2 * s),
        __builtin_bit_cast(h2v, packed));
}
template <bool F16V>
__device__ __forceinline__ void lds_add(void *vals, uint32_t s, float v0, float v1) {
    if constexpr (F16V) {
        lds_add_h2(vals, s, __builtin_bit_cast(uint32_t, h2v{(_Float16)v0, (_Float16)v1}));
    } else {
        float *f = reinterpret_cast<float *>(vals) + 2 * s;
        __hip_atomic_fetch_add(f, v0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        __hip_atomic_fetch_add(f + 1, v1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

// Slow path of a claim whose home slot holds another row: linear probing from
// the next slot; a full probe chain goes straight to HBM (returns false).
template <bool F16V>
__device__ __forceinline__ bool lds_probe(uint32_t *keys, void *vals, uint32_t mask, uint32_t key, float v0, float v1,
                                          float *g32, __half *g16) {
    uint32_t s = key;
#pragma unroll 1
    for (int p = 1; p < 16; ++p) {
        s = (s + 1) & mask;
        const uint32_t old = lds_cas(slot_key<F16V>(keys, s), key);
        if (old == SLOT_EMPTY || old == key) {
            lds_add<F16V>(vals, s, v0, v1);
            return true;
        }
    }
    if (g16) atomic_add_h2(g16 + (size_t)key * 2, v0, v1);
    else { atomic_add_f32(g32 + (size_t)key * 2, v0); atomic_add_f32(g32 + (size_t)key * 2 + 1, v1); }
    return false;
}

// amp form of gather_level for the input gradient: the corner pairs stay fp16x2 and are
// contracted with g = (g0, g1) by one v_dot2_f32_f16 each (fp32 accumulation of the exact
// fp16 products): t[k] = g0 e[k][0] + g1 e[k][1], without converting the 16 corner values
__device__ __forceinline__ void gather_level_t16(const FieldArgs &a, const LevelInfo &li, h2v g01, float t[8],
                                                 const uint32_t rows[8]) {
    const __half *tab = reinterpret_cast<const __half *>(a.table);
    const uint32_t rs = li.res + 1;
    if (level_dense(rs, li.hs)) {
#pragma unroll
        for (int idx = 0; idx < 8; idx += 2) {   // dense: corners idx, idx+1 are adjacent rows
            uint2 v;
            __builtin_memcpy(&v, tab + (size_t)rows[idx] * 2, 8);
            t[idx] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, v.x), g01, 0.f, false);
            t[idx + 1] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, v.y), g01, 0.f, false);
        }
    } else {
#pragma unroll
        for (int idx = 0; idx < 8; ++idx) {
            const uint32_t v = *reinterpret_cast<const uint32_t *>(tab + (size_t)rows[idx] * 2);
            t[idx] = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2v, v), g01, 0.f, false);
        }
    }
}

// member: the lane holds one of the ray's compacted backward samples (its cell takes part in the runs);
// active: its dL/dfeature at this level is non-zero (its terms are non-zero). part: 1 for the
// around-depth samples, 0 for the octree samples (see the run keys below)
template <typename TT, bool F16V>
__device__ __forceinline__ void backward_level(const FieldArgs &a, const LevelInfo &li, bool member, bool active,
                                               uint32_t part, const float x01[3], float g0, float g1, h2v g01,
                                               float gx[3], int lane, uint32_t *keys, void *vals, uint32_t mask,
                                               float *g32, __half *g16, int &n_direct) {
    // every lane's cell, weights and rows, unconditionally (a member's sample is in the box: pos >= 0.5,
    // truncation = floor; a non-member lane computes finite values it never uses — a branch here only
    // made the compiler materialise zeros for the skipped lanes)
    float pos[3];
    uint32_t pg[3], crow[8];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        pos[d] = __builtin_fmaf(x01[d], li.scale, 0.5f);
        pg[d] = (uint32_t)pos[d];
        pos[d] = __builtin_amdgcn_fractf(pos[d]);
    }
    corner_rows(li, pg, crow);
    if (active && !a.no_dx) {   // frozen poses: no corner values
        // d<g, feature>/d x01 of the trilinear interpolant (the reference's dy_dx contracted
        // with g): one scalar field t = g0 e[.][0] + g1 e[.][1] over the 8 corners, then its
        // x / y / z slopes by successive lerps (bit d of the corner index = +1 along d)
        float t[8];
        if constexpr (sizeof(TT) == 2) {
            gather_level_t16(a, li, g01, t, crow);
        } else {
            float e[8][2], pos_unused[3];
            uint32_t rows_unused[8];
            gather_level<TT, true>(a, li, x01, pos_unused, e, rows_unused);
#pragma unroll
            for (int k = 0; k < 8; ++k) t[k] = __builtin_fmaf(g1, e[k][1], g0 * e[k][0]);
        }
        float dx[4], ax[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {            // j = y + 2 z
            dx[j] = t[2 * j + 1] - t[2 * j];
            ax[j] = __builtin_fmaf(pos[0], dx[j], t[2 * j]);
        }
        float dy[2], by[2], ux[2];
#pragma unroll
        for (int z = 0; z < 2; ++z) {
            dy[z] = ax[2 * z + 1] - ax[2 * z];
            by[z] = __builtin_fmaf(pos[1], dy[z], ax[2 * z]);
            ux[z] = __builtin_fmaf(pos[1], dx[2 * z + 1] - dx[2 * z], dx[2 * z]);
        }
        gx[0] = __builtin_fmaf(li.scale, __builtin_fmaf(pos[2], ux[1] - ux[0], ux[0]), gx[0]);
        gx[1] = __builtin_fmaf(li.scale, __builtin_fmaf(pos[2], dy[1] - dy[0], dy[0]), gx[1]);
        gx[2] = __builtin_fmaf(li.scale, by[1] - by[0], gx[2]);
    }
    if ABL(1) return;
    // run keys: exact cell coordinates (10 bits each; res <= 1023) and the sample part in bit 31;
    // lanes past the ray's list unique. Within a part the samples are in ascending z, so a straight ray
    // visits each cell in one contiguous stretch: equal keys are always one run (the around-depth part
    // revisits the octree part's cells, hence the part bit), and a member whose dL/dfeature is zero
    // keeps its cell's key with zero terms, so it never splits a run
    const int key = member ? (int)((1u + (pg[0] | (pg[1] << 10) | (pg[2] << 20))) | (part << 31))
                           : (0x40000000 + lane + 1);
    // One representative per run of the whole wave: the run's TAIL (last lane), after a
    // segmented inclusive prefix sum across the wave (row_shr 1..8 inside each 16-lane row,
    // then row_bcast:15 / row_bcast:31 carry row totals into the next rows for runs that
    // cross a row boundary). Heads-per-row (a suffix scan inside rows) made a run that
    // crosses rows claim the same 8 slots once per row, in the same LDS instruction.
    // wave_shr:1 / wave_shl:1 (GFX9 DPP): the neighbour lanes' keys across row boundaries;
    // lanes 0 / 63 read 0, which is never a key
    const bool tail = member && (dpp_i<0x130>(key) != key);
    if (ABL(1 << 27)) {   // timing-build probe: representatives (tails)
        n_direct += tail ? 1 : 0;
    }
    // s_d: the lane's run continues d lanes back inside its row (in-row sources before the row start
    // read 0, never a key); equal keys are one run, so no run ids are needed
    const bool s1 = dpp_i<DPP_ROW_SHR(1)>(key) == key, s2 = dpp_i<DPP_ROW_SHR(2)>(key) == key;
    const bool s4 = dpp_i<DPP_ROW_SHR(4)>(key) == key, s8 = dpp_i<DPP_ROW_SHR(8)>(key) == key;
    // cross-row steps: the lane's run includes the row_bcast:15 source (lane 15 / 47, rows 1 / 3) or
    // the row_bcast:31 source (lane 31, rows 2 / 3)
    const bool sb15 = __builtin_amdgcn_update_dpp(0, key, 0x142, 0xa, 0xf, false) == key;
    const bool sb31 = __builtin_amdgcn_update_dpp(0, key, 0x143, 0xc, 0xf, false) == key;
    // wave-uniform: the scan steps some run actually needs (s_d: run continues d lanes back)
    const bool any1 = __any(s1), any2 = __any(s2);
    const bool any4 = __any(s4), any8 = __any(s8);
    const bool anyb15 = __any(sb15), anyb31 = __any(sb31);
    // corner weights times g (inactive lanes: g = 0 and pos = 0, so every value is 0)
    const float h0 = active ? g0 : 0.f, h1 = active ? g1 : 0.f;
    float wxy[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) wxy[j] = ((j & 1) ? pos[0] : 1 - pos[0]) * ((j & 2) ? pos[1] : 1 - pos[1]);
    const float wz0[2] = {(1 - pos[2]) * h0, pos[2] * h0}, wz1[2] = {(1 - pos[2]) * h1, pos[2] * h1};
    float v0[8], v1[8];
#pragma unroll
    for (int idx = 0; idx < 8; ++idx) {
        v0[idx] = wxy[idx & 3] * wz0[idx >> 2];
        v1[idx] = wxy[idx & 3] * wz1[idx >> 2];
    }
    // segmented prefix sum (runs are contiguous): one wave-uniform branch per scan step and
    // one v_fmac_f32_dpp per value: v += v[src] * m with m in {0, 1} (exactly v + x or v;
    // in-row sources before the row start read 0). Written as asm because the compiler
    // splits the DPP read from the FMA.
    // amp (F16V): the 16 values are packed into 8 fp16 pairs first (the LDS table holds fp16
    // pairs anyway) and scanned by v_pk_fmac_f16 with DPP — half the scan instructions. A run's
    // terms are then summed in fp16 (a tree of log2(run) roundings), the rounding class of the
    // reference, which adds every sample-corner term into the fp16 gradient one by one
    // (gridencoder.cu:319-327). Timing build: ABL 4096 keeps the fp32 scan.
    uint32_t pk[8];
    const bool pscan = F16V && !ABL(4096);
    if (pscan) {
#pragma unroll
        for (int idx = 0; idx < 8; ++idx) pk[idx] = __builtin_bit_cast(uint32_t, h2v{(_Float16)v0[idx], (_Float16)v1[idx]});
#define PFMAC_DPP(I, CTRL) "v_pk_fmac_f16_dpp %" #I ", %" #I ", %8 " CTRL "\n"
#define PSCAN_STEP(SK, CTRL)                                                                                      \
        if (any##SK) {                                                                                            \
            const uint32_t m = s##SK ? 0x3C003C00u : 0u;                                                          \
            asm("s_nop 1\n" PFMAC_DPP(0, CTRL) PFMAC_DPP(1, CTRL) PFMAC_DPP(2, CTRL) PFMAC_DPP(3, CTRL)          \
                PFMAC_DPP(4, CTRL) PFMAC_DPP(5, CTRL) PFMAC_DPP(6, CTRL) PFMAC_DPP(7, CTRL)                      \
                : "+v"(pk[0]), "+v"(pk[1]), "+v"(pk[2]), "+v"(pk[3]), "+v"(pk[4]), "+v"(pk[5]), "+v"(pk[6]),     \
                  "+v"(pk[7])                                                                                     \
                : "v"(m));                                                                                        \
        }
        PSCAN_STEP(1, "row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        PSCAN_STEP(2, "row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        PSCAN_STEP(4, "row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        PSCAN_STEP(8, "row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1")
        PSCAN_STEP(b15, "row_bcast:15 row_mask:0xa bank_mask:0xf")
        PSCAN_STEP(b31, "row_bcast:31 row_mask:0xc bank_mask:0xf")
#undef PFMAC_DPP
#undef PSCAN_STEP
    }
#define FMAC_DPP(I, CTRL) "v_fmac_f32_dpp %" #I ", %" #I ", %16 " CTRL "\n"
#define SCAN_STEP(SK, CTRL)                                                                                       \
    if (!pscan && any##SK) {                                                                                      \
        const float m = s##SK ? 1.f : 0.f;                                                                        \
        asm("s_nop 1\n" FMAC_DPP(0, CTRL) FMAC_DPP(1, CTRL) FMAC_DPP(2, CTRL) FMAC_DPP(3, CTRL)                  \
            FMAC_DPP(4, CTRL) FMAC_DPP(5, CTRL) FMAC_DPP(6, CTRL) FMAC_DPP(7, CTRL) FMAC_DPP(8, CTRL)            \
            FMAC_DPP(9, CTRL) FMAC_DPP(10, CTRL) FMAC_DPP(11, CTRL) FMAC_DPP(12, CTRL) FMAC_DPP(13, CTRL)        \
            FMAC_DPP(14, CTRL) FMAC_DPP(15, CTRL)                                                                \
            : "+v"(v0[0]), "+v"(v0[1]), "+v"(v0[2]), "+v"(v0[3]), "+v"(v0[4]), "+v"(v0[5]), "+v"(v0[6]),         \
              "+v"(v0[7]), "+v"(v1[0]), "+v"(v1[1]), "+v"(v1[2]), "+v"(v1[3]), "+v"(v1[4]), "+v"(v1[5]),         \
              "+v"(v1[6]), "+v"(v1[7])                                                                            \
            : "v"(m));                                                                                            \
    }
    SCAN_STEP(1, "row_shr:1 row_mask:0xf bank_mask:0xf bound_ctrl:1")
    SCAN_STEP(2, "row_shr:2 row_mask:0xf bank_mask:0xf bound_ctrl:1")
    SCAN_STEP(4, "row_shr:4 row_mask:0xf bank_mask:0xf bound_ctrl:1")
    SCAN_STEP(8, "row_shr:8 row_mask:0xf bank_mask:0xf bound_ctrl:1")
    SCAN_STEP(b15, "row_bcast:15 row_mask:0xa bank_mask:0xf")
    SCAN_STEP(b31, "row_bcast:31 row_mask:0xc bank_mask:0xf")
#undef FMAC_DPP
#undef SCAN_STEP
    if (!tail) return;
    if (ABL(1 << 26)) {   // timing build: the DPP scan without the table claims / adds
        n_direct += (v0[0] + v1[7] == 12345.f || (pscan && pk[3] == 12345u)) ? 1 : 0;
        return;
    }
    if constexpr (F16V) {
        if (!pscan) {   // the fp32 scan's sums, packed once (v_cvt_pk_f16_f32)
#pragma unroll
            for (int idx = 0; idx < 8; ++idx)
                pk[idx] = __builtin_bit_cast(uint32_t, h2v{(_Float16)v0[idx], (_Float16)v1[idx]});
        }
    }
    // claim the 8 home slots (home = the row itself mod the table size: the x-runs of
    // corner rows stay in consecutive slots, so the in-order flush issues few 64-B
    // segments per instruction) with all 8 CASes in flight, then add
    uint32_t old[8];
#pragma unroll
    for (int idx = 0; idx < 8; ++idx) old[idx] = lds_cas(slot_key<F16V>(keys, crow[idx] & mask), crow[idx]);
    // adds without branches: a claim that lost its home slot adds 0 there (harmless) and
    // takes the probe path afterwards, in one wave-uniform branch that is rarely entered
    // (which claims lost is recomputed there from old[])
    bool all_ok = true;
#pragma unroll
    for (int idx = 0; idx < 8; ++idx) {
        const bool ok = old[idx] == SLOT_EMPTY || old[idx] == crow[idx];
        all_ok = all_ok && ok;
        if constexpr (F16V) {   // the packed sums, selected once
            lds_add_h2(vals, crow[idx] & mask, ok ? pk[idx] : 0u);
        } else {
            lds_add<F16V>(vals, crow[idx] & mask, ok ? v0[idx] : 0.f, ok ? v1[idx] : 0.f);
        }
    }
    if (__builtin_expect(__any(!all_ok), 0)) {
#pragma unroll
        for (int idx = 0; idx < 8; ++idx)
            if (!(old[idx] == SLOT_EMPTY || old[idx] == crow[idx])) {
                float u0 = v0[idx], u1 = v1[idx];
                if constexpr (F16V) {   // the scanned fp16 pair (exact in fp32)
                    const h2v q = __builtin_bit_cast(h2v, pk[idx]);
                    u0 = (float)q[0];
                    u1 = (float)q[1];
                }
                n_direct += lds_probe<F16V>(keys, vals, mask, crow[idx], u0, u1, g32, g16) ? 0 : 1;
            }
    }
}

// One HBM atomic per occupied slot, then the slot is emptied for the next level.
// Lane l takes slots l + 64 j (consecutive lanes -> consecutive home slots -> rows
// in few 64-B segments per atomic instruction); four slots per lane are read
// together, every slot is reset unconditionally, so each group of 256 slots costs
// one LDS round trip instead of one per occupied slot.
// NJ (compile-time) slots per lane of one group of 64 NJ slots: the reads are issued together (a
// run-time slot count per group made the compiler wait after each read), the resets, then the adds
template <bool F16V, int NJ>
__device__ __forceinline__ int flush_group(uint32_t *keys, void *vals, uint32_t s0, int lane, float *g32, __half *g16,
                                           bool no_hbm) {
    uint32_t k[NJ];
    uint32_t vb[NJ];          // F16V: packed fp16x2
    float va[NJ], vc[NJ];     // fp32 pairs
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const uint32_t sl = s0 + 64 * j + lane;
        if constexpr (F16V) {   // [key | value] in one 8-B read
            const uint2 kv = reinterpret_cast<const uint2 *>(keys)[sl];
            k[j] = kv.x;
            vb[j] = kv.y;
        } else {
            k[j] = keys[sl];
            const float2 v = reinterpret_cast<float2 *>(vals)[sl];
            va[j] = v.x; vc[j] = v.y;
        }
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        const uint32_t sl = s0 + 64 * j + lane;
        if constexpr (F16V) {
            reinterpret_cast<uint2 *>(keys)[sl] = make_uint2(0xffffffffu, 0u);
        } else {
            keys[sl] = 0xffffffffu;
            reinterpret_cast<float2 *>(vals)[sl] = make_float2(0.f, 0.f);
        }
    }
    int n = 0;
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
        n += (int)__popcll(__ballot(k[j] != 0xffffffffu));   // wave-uniform count (scalar register)
        if (k[j] != 0xffffffffu && !no_hbm) {
            if constexpr (F16V) {
                typedef _Float16 h2v __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2v *)(g16 + (size_t)k[j] * 2),
                                                          __builtin_bit_cast(h2v, vb[j]));
            } else if (g16) {
                atomic_add_h2(g16 + (size_t)k[j] * 2, va[j], vc[j]);
            } else {
                atomic_add_f32(g32 + (size_t)k[j] * 2, va[j]);
                atomic_add_f32(g32 + (size_t)k[j] * 2 + 1, vc[j]);
            }
        }
    }
    return n;
}
template <bool F16V>
__device__ __forceinline__ int flush_table(uint32_t *keys, void *vals, uint32_t mask, int lane, float *g32,
                                           __half *g16, bool no_hbm) {
    int n = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    if (mask + 1 >= 256) {   // 256 .. 2048 slots: groups of four slots per lane
        for (uint32_t s0 = 0; s0 <= mask; s0 += 256) n += flush_group<F16V, 4>(keys, vals, s0, lane, g32, g16, no_hbm);
    } else if (mask + 1 == 128) {
        n = flush_group<F16V, 2>(keys, vals, 0, lane, g32, g16, no_hbm);
    } else {
        n = flush_group<F16V, 1>(keys, vals, 0, lane, g32, g16, no_hbm);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    return n;
}

__device__ __forceinline__ int lane_level(int s, int q, int h) { return 8 * s + 4 * (q >> 1) + 2 * h + (q & 1); }

// --------------------------------------------------------- MLP forward
// MFMA A-operand (weight fragment) sources: LDS-staged fragments (whole or partial staging).
template <typename TM> struct LdsW {
    const TM *p;
    __device__ __forceinline__ typename FragT<TM>::T get(int id, int lane) const { return load_frag<TM>(p, id, lane); }
};
// LDS fragments read from one per-lane base address made opaque once per tile (fence() at the top of each
// tile of a loop), so every read is that base + a constant (the ds_read offset field): load_frag's per-read
// opaque index costs an s_mov and a v_lshl_add per read. The per-tile fence still keeps the reads inside the
// tile loop (hoisted, the fragments would take the registers). Fragment `id` sits at slot id - base.
template <typename TM> struct LdsWt {
    typedef __attribute__((address_space(3))) const char *LdsPtr;
    LdsPtr q;   // this lane's byte address of slot 0 minus base slots
    __device__ __forceinline__ LdsWt(const TM *p, int lane, int base = 0)
        : q((LdsPtr)(reinterpret_cast<const char *>(p) + ((int64_t)lane - (int64_t)base * 64) * 8 * (int64_t)sizeof(TM))) {}
    __device__ __forceinline__ void fence() { asm volatile("" : "+v"(q)); }
    __device__ __forceinline__ typename FragT<TM>::T get(int id, int) const {
        const LdsPtr a = q + id * 64 * 8 * (int)sizeof(TM);
        typename FragT<TM>::T f;
        if constexpr (sizeof(TM) == 2) {
            f = *reinterpret_cast<__attribute__((address_space(3))) const h8v *>(a);
        } else {
            typedef float f4e __attribute__((ext_vector_type(4)));
            typedef __attribute__((address_space(3))) const f4e *L4;
            const f4e x = *reinterpret_cast<L4>(a), y = *reinterpret_cast<L4>(a + 16);
            f.v[0] = x.x; f.v[1] = x.y; f.v[2] = x.z; f.v[3] = x.w; f.v[4] = y.x; f.v[5] = y.y; f.v[6] = y.z; f.v[7] = y.w;
        }
        return f;
    }
};

template <typename TM> struct Acts {
    typename FragT<TM>::T X[2], H1[2][2], Cin[2], H3[2][2], H4[2][2];
};

template <typename TM, typename W>
__device__ __forceinline__ void mlp_sdf_net(const W &wfr, const float *wb, Acts<TM> &A, int lane, float &sdf,
                                            f16v &l2) {
    const int h = lane >> 5;
    f16v acc[2];
    // L1: 32 -> 64, ReLU
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        acc_init_bias(acc[mt], wb + 0 * 64, mt, h);
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[mt], wfr.get(FR_L1 + mt * 2 + s, lane), A.X[s]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H1[t][s]);
    // L2: 64 -> 16 (sdf, geo[15])
    acc_init_bias(acc[0], wb + 1 * 64, 0, h);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[0], wfr.get(FR_L2 + 2 * t + s, lane), A.H1[t][s]);
    float sdf_v = acc[0][0];
    if constexpr (sizeof(TM) == 2) sdf_v = (float)(_Float16)sdf_v;   // fp16 Linear output under autocast
    sdf = __shfl(sdf_v, lane & 31, 64);                                 // row 0 lives in half 0
    l2 = acc[0];
}

// Colour net on [geo, SH(view dir)] from the sigma net's L2 accumulator:
// fills A.Cin, A.H3, A.H4 and returns the 3 logits (all lanes, sample lane & 31).
template <typename TM, typename W>
__device__ __forceinline__ void mlp_colour_net(const W &wfr, const float *wb, Acts<TM> &A, const f16v &l2,
                                               const typename FragT<TM>::T &shf, int lane, float logit[3], bool masks,
                                               uint32_t &m3, uint32_t &m4);
template <typename TM>
__device__ __forceinline__ uint32_t relu_mask(const typename FragT<TM>::T (&H)[2][2]);
template <typename TM, typename W>
__device__ __forceinline__ void mlp_colour_net_cin(const W &wfr, const float *wb, Acts<TM> &A,
                                                   const typename FragT<TM>::T &cin,
                                                   const typename FragT<TM>::T &shf, int lane, float logit[3]);

// ...and, when `masks`, the ReLU masks of H3 / H4 to m3 / m4.
template <typename TM, typename W>
__device__ __forceinline__ void mlp_colour_net(const W &wfr, const float *wb, Acts<TM> &A, const f16v &l2,
                                               const typename FragT<TM>::T &shf, int lane, float logit[3], bool masks,
                                               uint32_t &m3, uint32_t &m4) {
    const int h = lane >> 5;
    f16v acc[2];
    // colour input: rows 0..15 = [sdf (zero weight), geo], rows 16..24 = SH (sh_frag)
    acc_to_frag<TM>(l2, 0, false, A.Cin[0]);
    A.Cin[1] = shf;
    // L3: 24 -> 64, ReLU
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        acc_init_bias(acc[mt], wb + 2 * 64, mt, h);
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[mt], wfr.get(FR_L3 + mt * 2 + s, lane), A.Cin[s]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H3[t][s]);
    if (masks) m3 = relu_mask<TM>(A.H3);
    // L4: 64 -> 64, ReLU
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        acc_init_bias(acc[mt], wb + 3 * 64, mt, h);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) mma(acc[mt], wfr.get(FR_L4 + mt * 4 + 2 * t + s, lane), A.H3[t][s]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H4[t][s]);
    if (masks) m4 = relu_mask<TM>(A.H4);
    // L5: 64 -> 3
    acc_init_bias(acc[0], wb + 4 * 64, 0, h);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[0], wfr.get(FR_L5 + 2 * t + s, lane), A.H4[t][s]);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float v = acc[0][c];
        if constexpr (sizeof(TM) == 2) v = (float)(_Float16)v;
        logit[c] = __shfl(v, lane & 31, 64);
    }
}

// The colour net from a stored colour-net input fragment (k_encode SIG: the sigma net's L2 output
// rows 0..15 as fp16, exactly acc_to_frag(l2, 0) of mlp_colour_net)
template <typename TM, typename W>
__device__ __forceinline__ void mlp_colour_net_cin(const W &wfr, const float *wb, Acts<TM> &A,
                                                   const typename FragT<TM>::T &cin,
                                                   const typename FragT<TM>::T &shf, int lane, float logit[3]) {
    const int h = lane >> 5;
    f16v acc[2];
    A.Cin[0] = cin;
    A.Cin[1] = shf;
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        acc_init_bias(acc[mt], wb + 2 * 64, mt, h);
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[mt], wfr.get(FR_L3 + mt * 2 + s, lane), A.Cin[s]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H3[t][s]);
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        acc_init_bias(acc[mt], wb + 3 * 64, mt, h);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) mma(acc[mt], wfr.get(FR_L4 + mt * 4 + 2 * t + s, lane), A.H3[t][s]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H4[t][s]);
    acc_init_bias(acc[0], wb + 4 * 64, 0, h);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[0], wfr.get(FR_L5 + 2 * t + s, lane), A.H4[t][s]);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float v = acc[0][c];
        if constexpr (sizeof(TM) == 2) v = (float)(_Float16)v;
        logit[c] = __shfl(v, lane & 31, 64);
    }
}

// ------------------------------------------------------ per-ray context
struct RayCtx {
    float dir[3], tgt[3], Rm[3][3], tv[3], vd[3];
    float depth, total;
    int frame, rtype;
    bool vdepth;
    const float *box;
    float ff[3];   // the frame's latent code (frame_features, n_ff <= 3 words; 0 past n_ff)
};
// Per-ray context record (k_ray_ctx, once per step): the fields of RayCtx in one 128-B row
// so the kernels' per-ray prologue is one batch of independent scalar loads instead of the
// dependent chain ray row -> frame -> pose row
constexpr int RCTX = 32;
__device__ __forceinline__ RayCtx build_ray(const FieldArgs &a, int r) {
    RayCtx c;
    const float *ray = a.rays + (size_t)r * 12;
#pragma unroll
    for (int i = 0; i < 3; ++i) { c.dir[i] = ray[i]; c.tgt[i] = ray[3 + i]; }
    c.depth = ray[6];
    c.frame = (int)ray[8];
    c.rtype = (int)ray[9];
    const float *T = a.tf + (size_t)c.frame * 16;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
#pragma unroll
        for (int j = 0; j < 3; ++j) c.Rm[i][j] = T[i * 4 + j];
        c.tv[i] = T[i * 4 + 3];
    }
    const float nrm = sqrtf((c.dir[0] * c.dir[0] + c.dir[1] * c.dir[1]) + c.dir[2] * c.dir[2]);
#pragma unroll
    for (int i = 0; i < 3; ++i) c.vd[i] = c.dir[i] / nrm;
    c.vdepth = (c.depth >= a.near_sc) && (c.depth <= a.far_sc);
    c.total = a.totals[r];
    c.box = a.intervals + (size_t)r * a.Kmax * 2;
#pragma unroll
    for (int i = 0; i < 3; ++i) c.ff[i] = i < a.n_ff ? a.ff[(size_t)c.frame * a.n_ff + i] : 0.f;
    return c;
}
__global__ __launch_bounds__(256) void k_ray_ctx(FieldArgs a_) {
    const FieldArgs a = step_args(a_);
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    // the step's counters, loss rows and loss_acc are zeroed here (one launch fewer per step; the
    // step is a captured graph of kernel nodes only)
    for (int i = r; i < (int)LOSS_ZERO_WORDS; i += gridDim.x * blockDim.x) a.n_tiles[i] = 0;
    for (int i = r; i < LOSS_ACC_WORDS; i += gridDim.x * blockDim.x) a.loss_acc[i] = 0.f;
    if (r >= a.R) return;
    const RayCtx c = build_ray(a, r);
    float4 *o = reinterpret_cast<float4 *>(a.rctx + (size_t)r * RCTX);
    o[0] = make_float4(c.dir[0], c.dir[1], c.dir[2], c.tgt[0]);
    o[1] = make_float4(c.tgt[1], c.tgt[2], c.Rm[0][0], c.Rm[0][1]);
    o[2] = make_float4(c.Rm[0][2], c.Rm[1][0], c.Rm[1][1], c.Rm[1][2]);
    o[3] = make_float4(c.Rm[2][0], c.Rm[2][1], c.Rm[2][2], c.tv[0]);
    o[4] = make_float4(c.tv[1], c.tv[2], c.vd[0], c.vd[1]);
    o[5] = make_float4(c.vd[2], c.depth, c.total, __int_as_float(c.frame));
    o[6] = make_float4(__int_as_float(c.rtype), c.ff[0], c.ff[1], c.ff[2]);
    o[7] = make_float4(0.f, 0.f, 0.f, 0.f);
}
// every caller passes a wave-uniform ray: the record is read through the constant address
// space (scalar loads, the context stays in scalar registers)
// LATE: the record's address laundered by an empty asm, so a call inside a loop reloads the record
// (scalar-cache hits) instead of the compiler holding its fields in SGPRs across the loop
template <bool LATE = false>
__device__ __forceinline__ RayCtx load_ray(const FieldArgs &a, int r) {
    size_t addr = (size_t)(a.rctx + (size_t)r * RCTX);
    if (LATE) asm volatile("" : "+s"(addr));
    const ConstU32 q = (ConstU32)addr;
    auto f = [&](int i) { return __uint_as_float(q[i]); };
    RayCtx c;
#pragma unroll
    for (int i = 0; i < 3; ++i) { c.dir[i] = f(i); c.tgt[i] = f(3 + i); c.tv[i] = f(15 + i); c.vd[i] = f(18 + i); }
#pragma unroll
    for (int i = 0; i < 3; ++i)
#pragma unroll
        for (int j = 0; j < 3; ++j) c.Rm[i][j] = f(6 + 3 * i + j);
    c.depth = f(21);
    c.total = f(22);
    c.frame = (int)q[23];
    c.rtype = (int)q[24];
#pragma unroll
    for (int i = 0; i < 3; ++i) c.ff[i] = f(25 + i);
    c.vdepth = (c.depth >= a.near_sc) && (c.depth <= a.far_sc);
    c.box = a.intervals + (size_t)r * a.Kmax * 2;
    return c;
}
// transform_pts (Utils.py:253-257) of p = dir * z; validity = inside [-1,1]^3 (run_network :1244)
__device__ __forceinline__ bool sample_point(const RayCtx &c, float z, float p[3], float x[3]) {
#pragma unroll
    for (int i = 0; i < 3; ++i) p[i] = c.dir[i] * z;
#pragma unroll
    for (int i = 0; i < 3; ++i) x[i] = ((c.Rm[i][0] * p[0] + c.Rm[i][1] * p[1]) + c.Rm[i][2] * p[2]) + c.tv[i];
    return fabsf(x[0]) <= 1.f && fabsf(x[1]) <= 1.f && fabsf(x[2]) <= 1.f;
}

// Feature / feature-gradient rows are stored per sample in MFMA-fragment
// order: 4 chunks of 8 elements, chunk (s*2 + h) = the B-operand fragment of
// K step s for lane half h. One lane's chunk = 16 B (fp16) / 32 B (fp32).
template <typename TM>
__device__ __forceinline__ void store_chunk(void *buf, size_t sample0, int n, int s, int h, const typename FragT<TM>::T &f) {
    // sample0 (the tile's first sample) is wave-uniform: a scalar 64-bit base plus a 32-bit lane offset
    TM *p = reinterpret_cast<TM *>(buf) + sample0 * 32 + (uint32_t)(n * 32 + (s * 2 + h) * 8);
    if constexpr (sizeof(TM) == 2) {
        *reinterpret_cast<h8v *>(p) = f;
    } else {
        *reinterpret_cast<float4 *>(p) = make_float4(f.v[0], f.v[1], f.v[2], f.v[3]);
        *reinterpret_cast<float4 *>(p + 4) = make_float4(f.v[4], f.v[5], f.v[6], f.v[7]);
    }
}
// dL/dfeature, level-major: plane lv holds the (feature 0, feature 1) pair of every
// sample ([L][R*S][2] TM), so k_scatter's per-level read is one coalesced 256-B (fp16)
// row per wave instead of 64 lanes each touching their own 64-B sample row. The
// fragment chunk (ss, h) holds levels lane_level(ss, q, h), q = 0..3 (2 values each).
template <typename TM>
__device__ __forceinline__ void store_dfeat(void *buf, size_t RS, size_t sample0, int n, int ss, int h,
                                            const typename FragT<TM>::T &f) {
    // the plane bases of the lane half's levels are wave-uniform (sample0 = the tile's first sample; h
    // selects between two uniform bases): scalar 64-bit arithmetic, a 32-bit lane offset
    TM *p = reinterpret_cast<TM *>(buf) + sample0 * 2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const int l0 = 8 * ss + 4 * (q >> 1) + (q & 1);
        TM *d0 = p + (size_t)l0 * RS * 2, *d1 = p + (size_t)(l0 + 2) * RS * 2;
        TM *d = (h ? d1 : d0) + (uint32_t)(n * 2);
        if constexpr (sizeof(TM) == 2) {
            typedef _Float16 h2v __attribute__((ext_vector_type(2)));
            h2v v = {f[2 * q], f[2 * q + 1]};
            *reinterpret_cast<h2v *>(d) = v;
        } else {
            *reinterpret_cast<float2 *>(d) = make_float2(f.v[2 * q], f.v[2 * q + 1]);
        }
    }
}
template <typename TM>
__device__ __forceinline__ typename FragT<TM>::T load_chunk(const void *buf, size_t sample0, int n, int s, int h) {
    const TM *p = reinterpret_cast<const TM *>(buf) + sample0 * 32 + (uint32_t)(n * 32 + (s * 2 + h) * 8);
    typename FragT<TM>::T f;
    if constexpr (sizeof(TM) == 2) {
        f = *reinterpret_cast<const h8v *>(p);
    } else {
        const float4 u = *reinterpret_cast<const float4 *>(p), v = *reinterpret_cast<const float4 *>(p + 4);
        f.v[0] = u.x; f.v[1] = u.y; f.v[2] = u.z; f.v[3] = u.w; f.v[4] = v.x; f.v[5] = v.y; f.v[6] = v.z; f.v[7] = v.w;
    }
    return f;
}

// per ray: [0..2] dL/drgb (x rgb_weight, ray weight, 1/3R), [3] wtot, [4] ray weight
constexpr int RAY_AUX = 8;

// per flagged tile (float4): [lane] (fp32 k_mlp_bwd pass 0 -> pass 1) ReLU masks of H3, H3^t, H4;
// [64 + n] (sdf-loss gradient without the ray weight, depth-guided weight if valid, valid, fs_rgb
// front) of sample n; [96 + n] (fp32 pass 0 -> pass 1) dO of sample n; [128 ..] (k_encode -> k_colour /
// pass 0) the colour-net input fragment Cin[0] of the tile (16 B per lane fp16 at [128 + lane], 32 B
// fp32 at [128 + 2 lane]), overwritten by amp pass 0 with the sigma-net output gradient for pass 1
// (fp16, [128 + lane]); amp only (k_colour -> k_mlp_bwd_tr pass 0): the SH fragment Cin[1] at
// [192 + lane], the ray's view directions in .zw of [0..2] (vd0 vd1 | vd2 R vd.x | R vd.y R vd.z)
constexpr int TILE_AUX = 256;
template <typename TM>
__device__ __forceinline__ void store_cin(float4 *aux, int lane, const typename FragT<TM>::T &f) {
    if constexpr (sizeof(TM) == 2) {
        reinterpret_cast<h8v *>(aux + 128)[lane] = f;
    } else {
        aux[128 + 2 * lane] = make_float4(f.v[0], f.v[1], f.v[2], f.v[3]);
        aux[129 + 2 * lane] = make_float4(f.v[4], f.v[5], f.v[6], f.v[7]);
    }
}
template <typename TM>
__device__ __forceinline__ typename FragT<TM>::T load_cin(const float4 *aux, int lane) {
    typename FragT<TM>::T f;
    if constexpr (sizeof(TM) == 2) {
        f = reinterpret_cast<const h8v *>(aux + 128)[lane];
    } else {
        const float4 u = aux[128 + 2 * lane], v = aux[129 + 2 * lane];
        f.v[0] = u.x; f.v[1] = u.y; f.v[2] = u.z; f.v[3] = u.w; f.v[4] = v.x; f.v[5] = v.y; f.v[6] = v.z; f.v[7] = v.w;
    }
    return f;
}
// loss_acc layout: [0..7] loss terms / counts, [8..135] spread scatter atomic counters,
// [136..139] forward executed-work counters (sigma tiles, colour tiles, colour records, sigma records),
// [140] fs_rgb loss (normalised, unscaled; cfg fs_rgb_weight > 0)

// The kernels' per-wave loss terms and work counters go to LOSS_COPIES copies of a 16-slot row
// (copy = wave id mod LOSS_COPIES) and loss_fold (first wave of the scatter kernel) adds the copies into loss_acc at the end of the
// field pass: one HBM atomic per wave and slot on a single address serialises at the memory side
// (the former per-ray forward's 13 per-wave loss atomics from 4096 persistent waves cost 0.09 ms per step).
// Slots: 0..4 loss rgb / fs / empty / sdf / n_valid, 5 n_bwd, 6..9 work counters, 10 fs_rgb loss,
// 11..12 timing-build probes; LOSS_FOLD_DST = their loss_acc indices.

__device__ __forceinline__ float *loss_row(const FieldArgs &a, int wave_id) {
    return a.loss_part + (size_t)(wave_id & (LOSS_COPIES - 1)) * LOSS_SLOTS;
}
// ReLU derivative of a 64-row activation as 32 bits (bit 16t + 8s + j)
template <typename TM>
__device__ __forceinline__ uint32_t relu_mask(const typename FragT<TM>::T (&H)[2][2]) {
    uint32_t m = 0;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if constexpr (sizeof(TM) == 2) {   // pair layout (pair_bits)
#pragma unroll
                for (int p = 0; p < 4; ++p) m |= pair_bits(h2v{H[t][s][2 * p], H[t][s][2 * p + 1]}, 8 * t + 4 * s + p);
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) m |= (frag_get<TM>(H[t][s], j) > 0 ? 1u : 0u) << (16 * t + 8 * s + j);
            }
        }
    return m;
}
template <typename TM>
__device__ __forceinline__ void masked_frags(const f16v (&acc)[2], uint32_t m, typename FragT<TM>::T (&d)[2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            if constexpr (sizeof(TM) == 2) {
#pragma unroll
                for (int p = 0; p < 4; ++p)
                    frag_put2(d[t][s], p, pk_keep(pk_round(acc[t][8 * s + 2 * p], acc[t][8 * s + 2 * p + 1]), m,
                                                  8 * t + 4 * s + p));
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j)
                    frag_set<TM>(d[t][s], j, ((m >> (16 * t + 8 * s + j)) & 1u) ? acc[t][8 * s + j] : 0.f);
            }
        }
}

// amp: the ReLU-derivative factors of a 64-row activation kept per pair (0 / 1 per half, the v_pk_min_u16
// result relu_mask packs into bits) for a mask consumed within the same tile, and its packed bits
__device__ __forceinline__ uint32_t relu_factors(const h8v (&H)[2][2], uint32_t (&r)[16]) {
    uint32_t m = 0;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const int P = 8 * t + 4 * s + p;
                r[P] = pair_bits(h2v{H[t][s][2 * p], H[t][s][2 * p + 1]}, 0);
                m |= r[P] << P;
            }
    return m;
}
// masked_frags with the factors of relu_factors: one packed multiply per pair
__device__ __forceinline__ void masked_frags_r(const f16v (&acc)[2], const uint32_t (&r)[16], h8v (&d)[2][2]) {
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const uint32_t u = __builtin_bit_cast(uint32_t, pk_round(acc[t][8 * s + 2 * p], acc[t][8 * s + 2 * p + 1]));
                uint32_t v;
                asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(v) : "v"(u), "v"(r[8 * t + 4 * s + p]));
                frag_put2(d[t][s], p, __builtin_bit_cast(h2v, v));
            }
}

// G levels of one lane's sample encoded together: the base row and the 4 paired
// (x, x+1) loads of every level in the group are issued before any is consumed, then
// the trilinear sums run in encode_level's order (same results). Dense levels only
// take the paired loads; a hashed level falls back to encode_level.
// HALVES: the lane's level is lvs[k] of lane 0 in the wave's first half and that + 2 in the second
// (lane_level): the level record is then read by two wave-uniform (scalar) loads instead of a
// per-lane vector load ahead of the corner gathers
// LREC: the level records come from the wave's LDS table (level_table: per level {scale, res, off,
// hs} and {rs, rs^2, dense, 0}), one ds_read per record per lane — each lane half reads its own
// level's record (no per-half selects of scalar values, no dense test per lane, no SGPR pressure)
struct LevelRec { LevelInfo li; uint32_t rs, rs2, dense; };
__device__ __forceinline__ LevelRec level_rec(const uint4 *lvt, int lv) {
    const uint4 r0 = lvt[2 * lv], r1 = lvt[2 * lv + 1];
    return {{__uint_as_float(r0.x), r0.y, r0.z, r0.w}, r1.x, r1.y, r1.z};
}
// fill the wave's level table (lanes 0..15: one level each; levels past L read as hashed / not dense)
__device__ __forceinline__ void level_table(const FieldArgs &a, uint4 *lvt, int lane) {
    if (lane < 16) {
        LevelInfo li = {1.f, 0u, 0u, 0u};
        if (lane < (int)a.L) li = level_info(a, lane);
        const uint32_t rs = li.res + 1;
        const bool dn = lane < (int)a.L && level_dense(rs, li.hs);
        lvt[2 * lane] = make_uint4(__float_as_uint(li.scale), li.res, li.off, li.hs);
        lvt[2 * lane + 1] = make_uint4(rs, rs * rs, dn ? 1u : 0u, 0u);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
}
template <typename TT, int G, bool HALVES = false, bool LREC = false>
__device__ __forceinline__ void encode_levels(const FieldArgs &a, const int (&lvs)[G], bool on, const float x01[3],
                                              float (&out)[G][2], const uint4 *lvt = nullptr) {
    const TT *tab = reinterpret_cast<const TT *>(a.table);
    float pos[G][3];
    uint32_t base[G], rs[G], rs2[G];
    bool dense[G];
    LevelInfo lis[G];
#pragma unroll
    for (int k = 0; k < G; ++k) {
        LevelInfo &li = lis[k];
        if constexpr (LREC) {
            const LevelRec rec = level_rec(lvt, lvs[k]);
            li = rec.li;
            rs[k] = rec.rs;
            rs2[k] = rec.rs2;
            dense[k] = on && rec.dense != 0u;
        } else {
            if constexpr (HALVES) {
                const int l0 = __builtin_amdgcn_readfirstlane(lvs[k]);
                const LevelInfo i0 = level_info_uniform(a, l0), i1 = level_info_uniform(a, l0 + 2);
                const bool hi = lvs[k] != l0;
                li = {hi ? i1.scale : i0.scale, hi ? i1.res : i0.res, hi ? i1.off : i0.off, hi ? i1.hs : i0.hs};
            } else {
                li = level_info(a, lvs[k]);
            }
            rs[k] = li.res + 1;
            rs2[k] = mul24(rs[k], rs[k]);
            dense[k] = on && lvs[k] < (int)a.L && level_dense_v(rs[k], li.hs);
        }
        uint32_t pg[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            // pos >= 0.5 for every in-box sample: truncation is the floor and v_fract_f32 the
            // exact pos - floor(pos) (off-box lanes' values are never used)
            pos[k][d] = __builtin_fmaf(x01[d], li.scale, 0.5f);
            pg[d] = (uint32_t)pos[k][d];
            pos[k][d] = __builtin_amdgcn_fractf(pos[k][d]);
        }
        base[k] = dense_base_v(li.off, pg, rs[k]);
    }
    typedef typename std::conditional<sizeof(TT) == 4, float4, uint2>::type Raw;
    Raw raw[G][4];
    const __amdgpu_buffer_rsrc_t trs = table_rsrc(a.table);
    if constexpr (sizeof(TT) == 2) {
        if (a.quads) {   // xy-quad mirror: the z and z+1 quads of the cell, two 16-B loads
            // unconditional, a lane whose level is not dense (or whose sample is off the box) reading quad 0:
            // its values are never used (the sums below skip it), and no zero-fill or exec mask per level
            const __amdgpu_buffer_rsrc_t qrs = table_rsrc(a.quads);
#pragma unroll
            for (int k = 0; k < G; ++k) {
                const uint32_t b0 = dense[k] ? base[k] : 0u, b1 = dense[k] ? base[k] + rs2[k] : 0u;
                const u4v q0 = __builtin_amdgcn_raw_buffer_load_b128(qrs, b0 * 16u, 0, 0);
                const u4v q1 = __builtin_amdgcn_raw_buffer_load_b128(qrs, b1 * 16u, 0, 0);
                raw[k][0] = make_uint2(q0.x, q0.y);
                raw[k][1] = make_uint2(q0.z, q0.w);
                raw[k][2] = make_uint2(q1.x, q1.y);
                raw[k][3] = make_uint2(q1.z, q1.w);
            }
            goto sums;
        }
    }
#pragma unroll
    for (int k = 0; k < G; ++k)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            raw[k][i] = Raw{};
            if (dense[k]) {
                const uint32_t row = base[k] + ((i & 1) ? rs[k] : 0u) + ((i & 2) ? rs2[k] : 0u);
                if constexpr (sizeof(TT) == 4) {
                    const TT *ptr = tab + (size_t)row * 2;
                    typedef float f4a __attribute__((ext_vector_type(4), aligned(8)));
                    const f4a v = *reinterpret_cast<const f4a *>(ptr);
                    raw[k][i] = make_float4(v.x, v.y, v.z, v.w);
                } else {
                    raw[k][i] = table_pair16(trs, row);
                }
            }
        }
sums:
#pragma unroll
    for (int k = 0; k < G; ++k) {
        out[k][0] = 0.f;
        out[k][1] = 0.f;
        if (!(on && lvs[k] < (int)a.L)) continue;
        if (!dense[k]) {
            encode_level<TT>(a, lis[k], x01, out[k]);
            continue;
        }
        if constexpr (sizeof(TT) == 2) {
            // fp16 corners: v_fma_mix_f32 takes each fp16 half straight from the loaded pair (the
            // exact f16 -> f32 widening inside the fma: the same result as convert + fma, without
            // the 16 conversions)
            float o0 = 0.f, o1 = 0.f;
#pragma unroll
            for (int idx = 0; idx < 8; ++idx) {
                float w = 1.f;
#pragma unroll
                for (int d = 0; d < 3; ++d) w *= ((idx >> d) & 1) ? pos[k][d] : 1 - pos[k][d];
                const uint32_t pr = (idx & 1) ? raw[k][idx >> 1].y : raw[k][idx >> 1].x;
                asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[0,1,0]" : "+v"(o0) : "v"(w), "v"(pr));
                asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "+v"(o1) : "v"(w), "v"(pr));
            }
            out[k][0] = o0;
            out[k][1] = o1;
        } else {
            float e[8][2];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                e[2 * i][0] = raw[k][i].x; e[2 * i][1] = raw[k][i].y;
                e[2 * i + 1][0] = raw[k][i].z; e[2 * i + 1][1] = raw[k][i].w;
            }
#pragma unroll
            for (int idx = 0; idx < 8; ++idx) {
                float w = 1.f;
#pragma unroll
                for (int d = 0; d < 3; ++d) w *= ((idx >> d) & 1) ? pos[k][d] : 1 - pos[k][d];
                out[k][0] = __builtin_fmaf(w, e[idx][0], out[k][0]);
                out[k][1] = __builtin_fmaf(w, e[idx][1], out[k][1]);
            }
        }
    }
}

// ------------------------------------------------------ kernel 1: encode + sigma net
// One wave per (ray, 32-sample tile): stratified/around-depth z
// (render_rays :1060-1080), world point, validity, and the multires
// encoding of the lane's 8 levels (kernel_grid, gridencoder.cu:106-246) —
// the lane layout is the layer-1 MFMA B operand, so the sigma net runs on the
// tile in place. Low register count -> high occupancy for the latency-bound
// gathers. SGPRs capped at 80: on gfx950 a wave's SGPR block (count rounded up to 16, + 16) comes
// out of an 800-entry budget per SIMD, so the 95 the compiler wanted admitted 7 waves per SIMD —
// 3 of these 8-wave blocks per CU, 6 waves per SIMD — where 80 admit 8 (MI355X_MICROARCH.md,
// residency); amp: 64 VGPRs (8 waves per SIMD), the uniform values spill to VGPR lanes
// DBG: the debug outputs (dbg_z / dbg_valid / dbg_raw) are written; the production instance compiles
// them out (their pointers and branches took SGPRs the 80-SGPR cap then spilled to VGPR lanes)
template <typename TM, typename TT, int G, bool DBG>
__global__ __launch_bounds__(512) __attribute__((amdgpu_num_sgpr(80),
                                                 amdgpu_waves_per_eu(sizeof(TM) == 2 ? (G == 1 ? 8 : G == 2 ? 6 : 4) : (G == 4 ? 4 : 5), 8)))
void k_encode(FieldArgs a_) {
    const FieldArgs a = step_args(a_);
    const int lane = threadIdx.x & 63, n = lane & 31, h = lane >> 5;
    const int ntiles = a.S / 32;
    constexpr int WPB = 8;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    {
        // layer 1 / 2 weight fragments (FR_L1, FR_L2: 8 x 1 KB fp16) and their biases, copied global -> LDS
        // by LDS-DMA (global_load_lds: no registers, no wait here): one 16-B piece per lane and fp16 KB,
        // the biases by the first two waves; the block's barrier comes after the gathers
        typedef __attribute__((address_space(1))) void *GPtr;
        typedef __attribute__((address_space(3))) void *LPtr;
        const int wv = threadIdx.x >> 6;
        if (ABL(16)) {   // timing build: synchronous staging through registers, barrier before the gathers
            const uint4 *src = reinterpret_cast<const uint4 *>(a.frags);
            uint4 *dst = reinterpret_cast<uint4 *>(smem);
            for (int i = threadIdx.x; i < 8 * 64 * 8 * (int)sizeof(TM) / 16; i += blockDim.x) dst[i] = src[i];
            float *s_b = reinterpret_cast<float *>(smem + 8 * 64 * 8 * sizeof(TM));
            for (int i = threadIdx.x; i < 2 * 64; i += blockDim.x) s_b[i] = a.bias[i];
            __syncthreads();
        } else {
#pragma unroll
            for (int i = 0; i < (int)sizeof(TM) / 2; ++i) {
                const size_t off = (size_t)i * 8192 + (size_t)wv * 1024;
                __builtin_amdgcn_global_load_lds((GPtr)((const char *)a.frags + off + lane * 16), (LPtr)(smem + off), 16,
                                                 0, 0);
            }
            if (wv < 2)
                __builtin_amdgcn_global_load_lds((GPtr)(a.bias + wv * 64 + lane),
                                                 (LPtr)(smem + 8 * 64 * 8 * sizeof(TM) + wv * 256), 4, 0, 0);
        }
    }
    // the wave's level table (after the weights and biases): the encode reads each lane's level record from it
    uint4 *lvt = reinterpret_cast<uint4 *>(smem + 8 * 64 * 8 * sizeof(TM) + 2 * 64 * sizeof(float)) + (threadIdx.x >> 6) * 32;
    level_table(a, lvt, lane);
    const int bx = (a.xcd_order & 1) ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int gw0 = __builtin_amdgcn_readfirstlane(bx * WPB + (int)(threadIdx.x >> 6));
    const bool in_range = gw0 < a.R * ntiles;
    // every wave reaches the block barrier; a wave past the last tile encodes the last tile
    // again (no stores) and leaves after it
    const int gw = in_range ? gw0 : a.R * ntiles - 1;
    const int r = gw / ntiles, t = gw - r * ntiles;
    if (ABL(1 << 19)) return;   // timing build: the waves' launch, staging and nothing else
    const RayCtx c = load_ray(a, r);
    const int s = 32 * t + n;
    const size_t sid = (size_t)r * a.S + s;
    float z = sample_z(a, r, s, c.depth, c.vdepth, c.total, c.box);
    if (ABL(4)) {   // timing build: the sampler's interval walk twice (its cost = the difference)
        const float z2 = sample_z(a, r, s, c.depth * 0.999f, c.vdepth, c.total * 0.999f, c.box);
        z = z2 == 12345.f ? z2 : z;
    }
    float p[3], x[3];
    const bool valid = sample_point(c, z, p, x);
    if (h == 0 && in_range) {
        a.zbuf[sid] = z;
        if (DBG && a.dbg_z) a.dbg_z[sid] = z;
        if (DBG && a.dbg_valid) a.dbg_valid[sid] = valid;
    }
    if (ABL(8192)) return;   // timing build: the sampler and the z store only
    const float x01[3] = {(x[0] + 1) / 2, (x[1] + 1) / 2, (x[2] + 1) / 2};
    typename FragT<TM>::T f[2];
#pragma unroll
    for (int g0 = 0; g0 < 8; g0 += G) {
        int lvs[G];
#pragma unroll
        for (int k = 0; k < G; ++k) lvs[k] = lane_level((g0 + k) >> 2, (g0 + k) & 3, h);
        float v[G][2];
        encode_levels<TT, G, true, true>(a, lvs, valid && !ABL(8), x01, v, lvt);
#pragma unroll
        for (int k = 0; k < G; ++k) {
            frag_set<TM>(f[(g0 + k) >> 2], 2 * ((g0 + k) & 3), v[k][0]);
            frag_set<TM>(f[(g0 + k) >> 2], 2 * ((g0 + k) & 3) + 1, v[k][1]);
        }
    }
    {
        // the sigma net on the tile just encoded (the features are the layer-1 B operand as they
        // stand), and everything of the forward tile pass that needs only the sdf: loss terms, the
        // backward / colour flags, the per-sample loss terms and gradient mask of backward tiles,
        // the colour-net input of colour tiles; features are stored only for backward tiles
        if (!ABL(64)) __syncthreads();   // the staged fragments (timing build: ABL 64 skips the barrier)
        if (!in_range) return;
        // the tail's arguments (loss weights, output pointers) re-read from the kernel arguments here,
        // after the gathers, instead of held in SGPRs across them (the 80-SGPR cap spilled them)
        const FieldArgs a = step_args(late_args());
        const bool tvalid = __any(valid);
        uint8_t *flag = a.tile_bwd + (size_t)r * ntiles + t;
        float4 *trec = reinterpret_cast<float4 *>(a.rrec + ((size_t)r * ntiles + t) * TREC);
        // the tile's share of the ray's weight sum (every sample, raw2outputs) and valid count in ONE
        // reduction: both lane halves hold the tile's 32 samples, the lower half carries the weight,
        // the upper half the valid flag (timing build: ABL 2 skips the per-tile record's reductions)
        float ws = 0.f, nv = 0.f;
        if (!ABL(2)) half_sums(h == 0 ? bell_weight(a, c.depth, z) : (valid ? 1.f : 0.f), ws, nv);
        if (!tvalid && !(DBG && a.dbg_raw)) {
            if (lane == 0) {
                *flag = 0;
                if (trec) {
                    trec[0] = make_float4(ws, nv, 0.f, 0.f);
                    trec[1] = make_float4(0.f, 0.f, 0.f, 0.f);
                }
            }
            return;
        }
        const TM *s_fr = reinterpret_cast<const TM *>(smem);
        const float *s_b = reinterpret_cast<const float *>(smem + 8 * 64 * 8 * sizeof(TM));
        Acts<TM> A;
        A.X[0] = f[0];
        A.X[1] = f[1];
        float sdf = 0.f;
        f16v l2;
        if (ABL(256)) {   // timing build: no sigma-net MFMAs
#pragma unroll
            for (int q = 0; q < 16; ++q) l2[q] = 0.f;
            sdf = z * 1e-3f;
        } else {
            mlp_sdf_net<TM>(LdsWt<TM>(s_fr, lane), s_b, A, lane, sdf, l2);   // one tile per wave: no fence needed
        }
        const float w = bell_weight(a, c.depth, z);
        const bool front = z < c.depth - a.trunc;
        const bool fsr = a.fs_rgb_w > 0.f && front && valid && c.rtype == 0;
        const bool colour = __any(w > 0.f && valid) || __any(fsr) || (DBG && a.dbg_raw != nullptr);
        const float sv = valid ? 1.f : 0.f;
        const bool back = z > c.depth + a.trunc * a.ntr;
        const float sdfm = (!front && !back && c.vdepth) ? 1.f : 0.f;
        const bool fsm = (c.depth > a.far_sc) && (sdf < a.fs_sdf);
        const bool em = front && (c.depth <= a.far_sc) && (sdf < 1.f);
        const float efs = fsm ? (sdf - a.fs_sdf) : 0.f;
        const float esdf = (z + sdf * a.trunc) * sdfm - c.depth * sdfm;
        float dsdf = a.fs_w * 0.5f * 2.f * efs * sv * a.inv_RS;
        dsdf += em ? a.fs_w * a.empty_w * (sdf > 1.f ? 1.f : (sdf < 1.f ? -1.f : 0.f)) * sv * a.inv_RS : 0.f;
        dsdf += a.trunc_w * 0.5f * 2.f * esdf * sdfm * a.trunc * sv * a.inv_RS;
        const bool cand = tvalid && c.rtype == 0 && (__any(w > 0.f && valid) || __any(dsdf != 0.f) || __any(fsr));
        // 1: backward with the colour net, 2: sigma-only backward, 3: colour net in the forward only
        if (lane == 0) *flag = cand ? (colour ? 1 : 2) : (colour ? 3 : 0);
        if (trec && !ABL(2)) {   // the tile's sdf-loss terms (ray weight applied by k_ray_final) and work-counter bits
            // a sample's fs / empty / sdf terms are mutually exclusive (depth > far / front / the band),
            // so a tile whose every loss gradient dsdf is zero has zero loss values too: no reductions.
            // Otherwise two reductions: fs (lower half) with empty (upper half), then sdf
            float lfs = 0.f, lem = 0.f, lsd = 0.f;
            if (__any(dsdf != 0.f)) {
                half_sums(h == 0 ? a.fs_w * 0.5f * efs * efs * sv * a.inv_RS
                                 : (em ? a.fs_w * a.empty_w * fabsf(sdf - 1.f) * sv * a.inv_RS : 0.f),
                          lfs, lem);
                float unused;
                half_sums(h == 0 ? a.trunc_w * 0.5f * esdf * esdf * sv * a.inv_RS : 0.f, lsd, unused);
            }
            if (lane == 0) {
                const int cnt = TC_SIG | (colour ? TC_COL : 0) | (cand ? (colour ? TC_CRCOL : TC_CRSIG) : 0);
                trec[0] = make_float4(ws, nv, lfs, lem);
                trec[1] = make_float4(lsd, __int_as_float(cnt), 0.f, 0.f);
            }
            // (the sample id re-derived from the tile's scalar slot: keeping the 64-bit sid live across the
            // gathers spilled it to scratch, one 8-B store per lane and tile)
            if (DBG && a.dbg_raw && h == 0) a.dbg_raw[(((size_t)r * ntiles + t) * 32 + n) * 4 + 3] = sdf;
        }
        const size_t slot = (size_t)r * ntiles + t;
        if (ABL(32768)) return;   // timing build: no backward / colour hand-off stores
        if (cand) {
            store_chunk<TM>(a.feat, (size_t)r * a.S + 32 * t, n, 0, h, f[0]);
            store_chunk<TM>(a.feat, (size_t)r * a.S + 32 * t, n, 1, h, f[1]);
            if (h == 0) a.tile_aux[slot * TILE_AUX + 64 + n] = make_float4(dsdf, valid ? w : 0.f, sv, fsr ? 1.f : 0.f);
            const uint32_t gmask = (uint32_t)__ballot(h == 0 && valid && (w > 0.f || dsdf != 0.f || fsr));
            if (lane == 0) a.tile_gmask[slot] = gmask;
        }
        if (colour) {
            typename FragT<TM>::T cin;
            acc_to_frag<TM>(l2, 0, false, cin);
            store_cin<TM>(a.tile_aux + slot * TILE_AUX, lane, cin);
        }
    }
}

// ------------------------------------------ kernel 2: MLP forward + losses
// Weight fragments + biases staged once per block in LDS (47 KB fp16).
template <typename TM>
__device__ __forceinline__ void stage_mlp(const FieldArgs &a, char *smem) {
    TM *s_fr = reinterpret_cast<TM *>(smem);
    float *s_b = reinterpret_cast<float *>(smem + N_FRAGS * 64 * 8 * sizeof(TM));
    const uint4 *src = reinterpret_cast<const uint4 *>(a.frags);
    uint4 *dst = reinterpret_cast<uint4 *>(s_fr);
    for (int i = threadIdx.x; i < N_FRAGS * 64 * 8 * (int)sizeof(TM) / 16; i += blockDim.x) dst[i] = src[i];
    for (int i = threadIdx.x; i < 5 * 64; i += blockDim.x) s_b[i] = a.bias[i];
    __syncthreads();
}

// The colour net's fragments only (FR_L3 .. FR_B5 - 1: 16 of the 46, 16 KB in fp16) and the bias
// image: k_colour needs nothing else, and a third of the LDS lets more of its blocks share a CU
constexpr int COL_FR0 = FR_L3, COL_NFR = FR_B5 - FR_L3;
template <typename TM> __host__ __device__ constexpr size_t colour_lds_bytes() {
    return (size_t)COL_NFR * 64 * 8 * sizeof(TM) + 5 * 64 * sizeof(float);
}
template <typename TM>
__device__ __forceinline__ void stage_colour(const FieldArgs &a, char *smem) {
    float *s_b = reinterpret_cast<float *>(smem + COL_NFR * 64 * 8 * sizeof(TM));
    const uint4 *src = reinterpret_cast<const uint4 *>(reinterpret_cast<const TM *>(a.frags) + (size_t)COL_FR0 * 64 * 8);
    uint4 *dst = reinterpret_cast<uint4 *>(smem);
    for (int i = threadIdx.x; i < COL_NFR * 64 * 8 * (int)sizeof(TM) / 16; i += blockDim.x) dst[i] = src[i];
    for (int i = threadIdx.x; i < 5 * 64; i += blockDim.x) s_b[i] = a.bias[i];
    __syncthreads();
}

// SH(view direction) rows 16..24 of the colour-net input as the second K-step
// B fragment (h0: SH0..3, SH8; h1: SH4..7) — one per ray.
// the view direction in the object frame (the SH input, run_network :1281)
__device__ __forceinline__ void view_dir(const RayCtx &c, float &x, float &y, float &z) {
    x = (c.Rm[0][0] * c.vd[0] + c.Rm[0][1] * c.vd[1]) + c.Rm[0][2] * c.vd[2];
    y = (c.Rm[1][0] * c.vd[0] + c.Rm[1][1] * c.vd[1]) + c.Rm[1][2] * c.vd[2];
    z = (c.Rm[2][0] * c.vd[0] + c.Rm[2][1] * c.vd[1]) + c.Rm[2][2] * c.vd[2];
}
__device__ __forceinline__ void sh_values(const RayCtx &c, float sh[9]) {
    float x, y, z;
    view_dir(c, x, y, z);
    const float xx = x * x, yy = y * y, zz = z * z;
    sh[0] = SH_C0; sh[1] = -SH_C1 * y; sh[2] = SH_C1 * z; sh[3] = -SH_C1 * x;
    sh[4] = SH_C2_0 * (x * y); sh[5] = SH_C2_1 * (y * z); sh[6] = SH_C2_2 * ((2.0f * zz - xx) - yy);
    sh[7] = SH_C2_3 * (x * z); sh[8] = SH_C2_4 * (xx - yy);
}
template <typename TM>
__device__ __forceinline__ typename FragT<TM>::T sh_frag(const RayCtx &c, int h, int n_ff = 0) {
    float sh[9];
    sh_values(c, sh);
    typename FragT<TM>::T f;
    frag_zero<TM>(f);
    if (h == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) frag_set<TM>(f, j, sh[j]);
        frag_set<TM>(f, 4, sh[8]);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) frag_set<TM>(f, j, sh[4 + j]);
    }
    if (h == 0 && n_ff > 0) {   // frame features: Cin rows 25.. (from the ray's context record: scalar registers)
#pragma unroll
        for (int j = 0; j < 3; ++j) frag_set<TM>(f, 5 + j, c.ff[j]);
    }
    return f;
}

// ---------------------------- kernel 2 (tile-parallel forward): colour net + ray finalisation
// k_encode SIG ran the sigma net, the sdf-loss terms and the flags; what is left of the forward's
// per-ray pass is the colour net on the colour tiles (flag 1 or 3, k_compact's colour list) and the
// per-ray compositing / losses. k_colour: persistent waves over the colour-tile list — a wave per
// TILE, not per ray, so independent tiles fill the SIMDs (a per-ray forward wave walked its ray's six
// tiles one after another) — colour net from the stored colour-net input, the tile's composited
// colour and fs_rgb term stored in the tile's record (rrec), and the SH fragment / view directions the
// backward reads. k_ray_final: a thread per ray — rgb_map, dL/drgb, the ray weight and the losses
// (raw2outputs + train_loop :687-751), the backward's per-ray hand-off (ray_aux), the loss rows.
template <typename TM, int WPB, int WAVES, bool DBG>
__global__ __launch_bounds__(WPB * 64) __attribute__((amdgpu_waves_per_eu(WAVES, WAVES))) void k_colour(FieldArgs a_) {
    const FieldArgs a = step_args(a_);
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = lane & 31, h = lane >> 5;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    stage_colour<TM>(a, smem);
    const float *s_b = reinterpret_cast<const float *>(smem + COL_NFR * 64 * 8 * sizeof(TM));
    LdsWt<TM> W(reinterpret_cast<const TM *>(smem), lane, COL_FR0);
    const int n_col = __builtin_amdgcn_readfirstlane(a.n_tiles[1]);
    const int wg = __builtin_amdgcn_readfirstlane((int)blockIdx.x * WPB + wave);
    const int stride = gridDim.x * WPB;
    // the tile's vector loads (colour-net input, depths, flag) are issued one tile ahead, the list
    // entry two tiles ahead: a tile starts with its inputs in flight or landed instead of one
    // memory latency (k_encode wrote them; they come from L2 / HBM) at 4 waves per SIMD
    typedef typename FragT<TM>::T Frag;
    int cur = wg < n_col ? a.ctile_list[wg] : 0;
    int nxt = a.ctile_list[min(wg + stride, max(n_col - 1, 0))];
    Frag cin_n;
    frag_zero<TM>(cin_n);
    float z_n = 0.f;
    auto fetch = [&](int sid_first) {
        z_n = a.zbuf[(size_t)sid_first + n];
        cin_n = load_cin<TM>(a.tile_aux + (size_t)(sid_first >> 5) * TILE_AUX, lane);
    };
    if (wg < n_col) fetch(__builtin_amdgcn_readfirstlane(cur));
    // the first prefetch has landed before the loop (a builtin wait the compiler tracks), so the
    // loop header's merged state does not make every tile wait on the previous tile's stores
    __builtin_amdgcn_s_waitcnt(0x0f70);
    // The loop body is straight-line in its memory operations (no store or load under a branch:
    // the per-lane stores are made wave-wide with duplicate lanes writing identical data, the debug
    // dump is a template instance): the compiler's wait counts then name exactly the load a value
    // needs. Each prefetched register is consumed where it landed before its reload is issued (no
    // loop-carried copy of an in-flight load): z at the tile's top, the colour-net input by the
    // net, after which the next tile's loads go out (the last tile re-fetches itself, clamped); the
    // list entry two tiles ahead is loaded at the top and copied at the tile's end.
    for (int li = wg; li < n_col; li += stride) {
        const int sid0 = __builtin_amdgcn_readfirstlane(cur);
        const int nn = a.ctile_list[min(li + 2 * stride, n_col - 1)];
        const int r = sid0 / a.S;
        const size_t slot = (size_t)(sid0 >> 5);
        const size_t sid = (size_t)sid0 + n;
        const RayCtx c = load_ray(a, r);
        const float z = z_n;
        const float w = bell_weight(a, c.depth, z);
        float p[3], x[3];
        const bool valid = sample_point(c, z, p, x);
        const bool front = z < c.depth - a.trunc;
        // the sample's weights, computed here (pinned: not sunk past the reload of z_n)
        float wc = valid && w > 0.f ? w : 0.f;
        float wf = a.fs_rgb_w > 0.f && front && valid && c.rtype == 0 ? a.inv_3RS : 0.f;
        asm volatile("" : "+v"(wc), "+v"(wf));
        const Frag shf = sh_frag<TM>(c, h, a.n_ff);
        Acts<TM> A;
        float logit[3];
        W.fence();   // the fragment reads stay in this tile
        mlp_colour_net_cin<TM>(W, s_b, A, cin_n, shf, lane, logit);
        fetch(__builtin_amdgcn_readfirstlane(li + stride < n_col ? nxt : sid0));
        // both lane halves hold the tile's 32 samples (the logits are broadcast): the lower half carries
        // the composited colour's r and b, the upper half g and the fs_rgb term — two half-wave sums
        // fs_rgb: mean over R x S x 3 of ((sigmoid - 1) front)^2 sw; the ray weight in k_ray_final
        float rc[3], lf = 0.f;
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            const float sg = sigmoidf(logit[cc]);
            rc[cc] = wc * sg;
            lf += (sg - 1.f) * (sg - 1.f) * wf;
        }
        if constexpr (DBG) {
            if (h == 0) {
                float *o = a.dbg_raw + sid * 4;
                o[0] = logit[0]; o[1] = logit[1]; o[2] = logit[2];
            }
        }
        if constexpr (sizeof(TM) == 2) {
            // the SH fragment and the ray's view directions for k_mlp_bwd_tr (read for backward tiles,
            // flag 1; written for every colour tile, whose aux rows hold nothing else there). The view
            // directions are three float2 words: lanes 2..63 all write word 2's identical data
            reinterpret_cast<h8v *>(a.tile_aux + slot * TILE_AUX + 192)[lane] = shf;
            float vx, vy, vz;
            view_dir(c, vx, vy, vz);
            const float2 d = lane == 0 ? make_float2(c.vd[0], c.vd[1])
                                       : (lane == 1 ? make_float2(c.vd[2], vx) : make_float2(vy, vz));
            reinterpret_cast<float2 *>(a.tile_aux + slot * TILE_AUX + min(lane, 2))[1] = d;
        }
        float s0, s1, s2, sf;
        half_sums(h == 0 ? rc[0] : rc[1], s0, s1);
        half_sums(h == 0 ? rc[2] : lf, s2, sf);
        // wave-uniform sums: every lane writes the same 16 B (no lane-0 branch)
        reinterpret_cast<float4 *>(a.rrec + slot * TREC)[2] = make_float4(s0, s1, s2, sf);
        cur = nxt;
        nxt = nn;
    }
}

__global__ __launch_bounds__(256) void k_ray_final(FieldArgs a_) {
    const FieldArgs a = step_args(a_);
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // loss rgb, fs, empty, sdf, n_valid, fs_rgb, and the four work counters
    float v[10];
#pragma unroll
    for (int k = 0; k < 10; ++k) v[k] = 0.f;
    if (r < a.R) {
        // the ray's tiles in order: every tile's sdf record, the colour record of the colour tiles
        const int ntiles = a.S / 32;
        float wtot = 0.f, nvalid = 0.f, lfs = 0.f, lem = 0.f, lsdf = 0.f, lfsr = 0.f;
        float racc[3] = {0.f, 0.f, 0.f};
        int csig = 0, ccol = 0, crcol = 0, crsig = 0;
        // every load of a tile issued together (the colour record is read whatever the flag and
        // selected after: a flag-dependent load was a second round trip per tile)
#pragma unroll 4
        for (int t = 0; t < ntiles; ++t) {
            const size_t slot = (size_t)r * ntiles + t;
            const float4 *q = reinterpret_cast<const float4 *>(a.rrec + slot * TREC);
            const float4 q0 = q[0], q1 = q[1], q2 = q[2];
            const uint8_t fl = a.tile_bwd[slot];
            wtot += q0.x; nvalid += q0.y; lfs += q0.z; lem += q0.w; lsdf += q1.x;
            const int cnt = __float_as_int(q1.y);
            csig += cnt & TC_SIG; ccol += (cnt >> 1) & 1; crcol += (cnt >> 2) & 1; crsig += (cnt >> 3) & 1;
            if (fl == 1 || fl == 3) {
                racc[0] += q2.x; racc[1] += q2.y; racc[2] += q2.z; lfsr += q2.w;
            }
        }
        const float *cx = a.rctx + (size_t)r * RCTX;
        const float tgt[3] = {cx[3], cx[4], cx[5]};
        const int frame = __float_as_int(cx[23]), rtype = __float_as_int(cx[24]);
        const bool vray = nvalid > 0.f && rtype == 0;
        const float rw = vray ? (frame == 0 ? a.ffw : 1.f) : 0.f;
        float drgb[3], lr = 0.f, rgb[3];
#pragma unroll
        for (int cc = 0; cc < 3; ++cc) {
            rgb[cc] = racc[cc] / (wtot + 1e-10f);
            const float e = rgb[cc] - tgt[cc];
            drgb[cc] = a.rgb_w * 2.f * e * rw * a.inv_3R;
            lr += e * e * rw;
        }
        v[0] = a.rgb_w * lr * a.inv_3R;
        v[1] = lfs * rw;
        v[2] = lem * rw;
        v[3] = lsdf * rw;
        v[4] = nvalid;
        v[5] = lfsr * rw;
        v[6] = (float)csig; v[7] = (float)ccol; v[8] = (float)crcol; v[9] = (float)crsig;
        if (a.dbg_rgb) {
            a.dbg_rgb[r * 3] = rgb[0]; a.dbg_rgb[r * 3 + 1] = rgb[1]; a.dbg_rgb[r * 3 + 2] = rgb[2];
        }
        // per-ray hand-off: dL/drgb, wtot, ray weight; the pose gradient starts at zero
        float4 *ra = reinterpret_cast<float4 *>(a.ray_aux + (size_t)r * RAY_AUX);
        ra[0] = make_float4(drgb[0], drgb[1], drgb[2], wtot);
        ra[1] = make_float4(rw, 0.f, 0.f, 0.f);
        float4 *rg = reinterpret_cast<float4 *>(a.ray_grad + (size_t)r * 12);
        rg[0] = make_float4(0.f, 0.f, 0.f, 0.f);
        rg[1] = make_float4(0.f, 0.f, 0.f, 0.f);
        rg[2] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    __shared__ float s_v[4][10];
#pragma unroll
    for (int k = 0; k < 10; ++k) {
        const float t = wave_sum(v[k]);
        if (lane == 0) s_v[wave][k] = t;
    }
    __syncthreads();
    if (threadIdx.x < 10) {
        const int k = threadIdx.x;
        const float t = s_v[0][k] + s_v[1][k] + s_v[2][k] + s_v[3][k];
        constexpr int slot[10] = {0, 1, 2, 3, 4, 10, 6, 7, 8, 9};
        if (t != 0.f && (k != 5 || a.fs_rgb_w > 0.f)) atomic_add_f32(loss_row(a, (int)blockIdx.x) + slot[k], t);
    }
}

// k_encode levels in flight per lane below 8,192 rays (FieldArgs::encode_group 0: by batch size)
constexpr int ENCODE_GROUP_SMALL = 2;

// Lists of the tiles k_encode flagged (the order inside a list is free: the MLP backward only
// sums over it). Backward tiles: those with the colour net (tile_bwd 1) from the list's FRONT,
// counted at count[0], as first sample ids; the sigma-only ones (2) from its BACK (entry j at
// n - 1 - j), counted at count[2], as first sample id | bit 31 — so the MLP backward walks the two
// kinds in separate loops with straight-line bodies (no merge of the colour path's loads with the
// other path in the loop, whose conservative wait would hold every tile on its own loads). With
// clist, in the same pass: the colour tiles (flag 1 or 3: the colour net runs in the forward,
// k_colour) as first sample ids, counted at count[1]. One returning atomic per list and block of
// 4096 flags.
constexpr int COMPACT_PER_BLOCK = 4096;   // flags per block at the headline sizes
__global__ __launch_bounds__(256) void k_compact(const uint8_t *__restrict__ flags, int n, int *__restrict__ list,
                                                 int *__restrict__ count, int per_block, int *__restrict__ clist) {
    // a thread's flags are per_block / 256 consecutive bytes (16 at 4096 per block: one 16-B
    // load), so one block-wide scan of the per-thread counts places every entry (in index order)
    __shared__ int s_wave[3][4];
    __shared__ int s_base[3];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int fpt = per_block >> 8;   // 16 or 2
    const int b0 = blockIdx.x * per_block + threadIdx.x * fpt;
    uint8_t fl[16];
    if (fpt == 16 && b0 + 16 <= n) {
        const uint4 v = *reinterpret_cast<const uint4 *>(flags + b0);
        const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 16; ++k) fl[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
    } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) fl[k] = (k < fpt && b0 + k < n) ? flags[b0 + k] : 0;
    }
    // per thread: colour-backward (1), sigma-only backward (2), colour (1 or 3) counts
    int mine[3] = {0, 0, 0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        mine[0] += fl[k] == 1;
        mine[1] += fl[k] == 2;
        mine[2] += (fl[k] == 1 || fl[k] == 3);
    }
    int pm[3] = {mine[0], mine[1], mine[2]};   // inclusive wave scans
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
#pragma unroll
        for (int q = 0; q < 3; ++q) {
            const int u = __shfl_up(pm[q], o, 64);
            if (lane >= o) pm[q] += u;
        }
    }
    if (lane == 63) {
#pragma unroll
        for (int q = 0; q < 3; ++q) s_wave[q][wave] = pm[q];
    }
    __syncthreads();
    if (threadIdx.x < 3) {
        const int q = threadIdx.x;
        const int tot = s_wave[q][0] + s_wave[q][1] + s_wave[q][2] + s_wave[q][3];
        int *cnt = count + (q == 0 ? 0 : (q == 1 ? 2 : 1));
        s_base[q] = (tot && (q < 2 || clist)) ? atomicAdd(cnt, tot) : 0;
    }
    __syncthreads();
    int off[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) {
        off[q] = s_base[q] + pm[q] - mine[q];
        for (int w = 0; w < wave; ++w) off[q] += s_wave[q][w];
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
        const int i = b0 + k;
        if (fl[k] == 1) list[off[0]++] = i << 5;
        if (fl[k] == 2) list[n - 1 - off[1]++] = (i << 5) | (int)0x80000000;
        if (clist && (fl[k] == 1 || fl[k] == 3)) clist[off[2]++] = i << 5;
    }
}

// entry li of the backward list walked as one sequence: the colour-backward tiles [0, n_c) at the
// front, then the sigma-only tiles from the back (k_compact)
__device__ __forceinline__ int bwd_entry(const FieldArgs &a, int li, int n_c, int cap) {
    return a.tile_sid[li < n_c ? li : cap - 1 - (li - n_c)];
}

#include "field_mlp_bwd.h"   // kernel 3: the MLP backward (k_mlp_bwd, k_mlp_bwd_tr)

// The loss rows (64 copies, written by k_ray_final and k_mlp_bwd pass 1) summed into
// loss_acc: run by the first wave of the scatter kernel's first block (the scatter launches after
// every loss-row writer and writes none of these words: one launch fewer per step)
__device__ __forceinline__ void loss_fold(const float *__restrict__ part, float *__restrict__ loss_acc, int k);

// --------------------------------------------------- kernel 3: scatter
// LDS words of one scatter wave: the row table (keys, VW value words per slot) and the
// compacted list of the ray's backward samples (uint16, up to 320)
__host__ __device__ constexpr uint32_t scatter_wave_words(uint32_t mask, int VW) {
    return (1 + VW) * (mask + 1) + 160;
}
// One wave per ray with any tile marked by kernel 2. Levels outer, 64-sample
// chunks inner: re-gathers the corners to form d<g,feature>/dx (the
// reference's dy_dx), reduces the table gradient of the whole ray at this
// level in the wave's LDS hash table (backward_level) and flushes it with one
// HBM atomic per distinct row, and adds the transform_pts part of dL/dtf
// (sum over samples of 0.5 dL/dx01 (x) [p, 1]) to the ray's 3x4 gradient.
// SGPRs capped at 80 as k_encode's, so the hardware admits 8 waves per SIMD instead of 7 (a wave's SGPR
// block, count rounded up to 16 + 16, out of 800 per SIMD). Round 5 measured the cap neutral with 94
// SGPRs wanted (2.00 / 2.03 vs 2.02 / 2.03 ms); with the ray's pose rows re-read per iteration (92
// wanted, no spill uncapped) it measured 1.959 vs 2.001 ms uncapped and 2.033 for round 5's kernel
// (medians of 5, alternating builds, profiles/r6/ab_r6_scatter_ctx_reload_sgpr_cap.jsonl)
template <typename TM, typename TT, bool F16V, int WAVES>
__global__ __launch_bounds__(256) __attribute__((amdgpu_num_sgpr(80), amdgpu_waves_per_eu(WAVES, 8))) void k_scatter(FieldArgs a_) {
    const FieldArgs a = step_args(a_);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    if (blockIdx.x == 0 && wave == 0) loss_fold(a.loss_part, a.loss_acc, lane);
    const int bx = (a.xcd_order & 2) ? xcd_block(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    // small batches (NerfRunner.train's 2048 rays) split each ray's levels over several waves
    // so the chip has enough of them; large batches keep one wave per ray (lpw = L)
    const int lpw = a.scatter_lpw, ngrp = ((int)a.L + lpw - 1) / lpw;
    const int gw = __builtin_amdgcn_readfirstlane(bx * 4 + wave);
    const int r = __builtin_amdgcn_readfirstlane(gw / ngrp);
    if (r >= a.R || ABL(65536)) return;
    const int lv0 = __builtin_amdgcn_readfirstlane((gw - r * ngrp) * lpw);
    const int nlev = min(lpw, (int)a.L - lv0);
    const int ntiles = a.S / 32;
    const uint8_t *flags = a.tile_bwd + (size_t)r * ntiles;
    // the tiles' flags and gradient masks are loaded together (lane t: tile t; one memory latency, not two
    // dependent ones); a mask counts only for a backward tile (flag 1 / 2; 3: forward-only colour tile)
    const uint8_t fl = lane < ntiles ? flags[lane] : (uint8_t)0;
    uint32_t gm = lane < ntiles ? a.tile_gmask[(size_t)r * ntiles + lane] : 0u;
    const bool tf = fl == 1 || fl == 2;
    if (!__any(tf) || ABL(131072)) return;
    gm = tf ? gm : 0u;
    const uint32_t mask = a.slot_mask;
    constexpr int VW = F16V ? 1 : 2;   // value words per slot
    uint32_t *keys = reinterpret_cast<uint32_t *>(smem) + (size_t)wave * scatter_wave_words(mask, VW);
    // amp: interleaved [key | value] slots (vals = keys + 1, stride 2 words); fp32: keys, then values
    uint32_t *vals = F16V ? keys + 1 : keys + mask + 1;
    uint16_t *slist = reinterpret_cast<uint16_t *>(keys + (1 + VW) * (mask + 1));
    if constexpr (F16V) {
        for (uint32_t s = lane; s <= mask; s += 64) reinterpret_cast<uint2 *>(keys)[s] = make_uint2(0xffffffffu, 0u);
    } else {
        for (uint32_t s = lane; s <= mask; s += 64) keys[s] = 0xffffffffu;
        for (uint32_t s = lane; s < VW * (mask + 1); s += 64) vals[s] = 0u;
    }
    if ABL(262144) return;
    float *g32 = (sizeof(TM) == 2) ? nullptr : a.grad_table;
    __half *g16 = (sizeof(TM) == 2) ? a.grad_table16 : nullptr;
    const RayCtx c = load_ray(a, r);
    // The ray's backward samples — in a flagged tile, inside the box, and carrying a loss
    // gradient (k_encode's per-sample loss terms in the tile aux: a depth-guided weight, an
    // sdf-loss term or the fs_rgb term; every other sample's dL/dfeature is exactly zero, since
    // the rendering weights do not depend on the network) — compacted in sample order into
    // the wave's LDS list, so the (level, chunk) iterations run over full 64-lane chunks.
    // Sample order is kept, so runs of equal cells stay contiguous (two runs of one cell
    // separated by skipped samples merge: same sum).
    int n_act = 0;
    for (int ch = 0; ch * 64 < a.S; ++ch) {
        const int s = 64 * ch + lane;
        // this chunk's two tiles' masks (lanes 0-31: tile 2 ch, 32-63: tile 2 ch + 1), read from lanes 2 ch, 2 ch + 1
        const uint32_t m0 = (uint32_t)__builtin_amdgcn_readlane((int)gm, 2 * ch);
        const uint32_t m1 = 2 * ch + 1 < 64 ? (uint32_t)__builtin_amdgcn_readlane((int)gm, 2 * ch + 1) : 0u;
        const bool cand = s < a.S && (((lane < 32 ? m0 : m1) >> (s & 31)) & 1u);
        const uint64_t b = __ballot(cand);
        if (cand) slist[n_act + (int)__popcll(b & ((1ull << lane) - 1ull))] = (uint16_t)s;
        n_act += (int)__popcll(b);
    }
    n_act = __builtin_amdgcn_readfirstlane(n_act);
    if (n_act == 0) return;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const int nch = (n_act + 63) / 64;
    // dL/dtf of the ray (transform_pts part): sum over samples of 0.5 gx (x) [p, 1] with
    // p = dir z, i.e. 0.5 (sum gx z) (x) dir and 0.5 sum gx: six per-lane sums
    float sgz[3] = {0.f, 0.f, 0.f}, sg[3] = {0.f, 0.f, 0.f};
    int n_flush = 0, n_direct = 0;   // HBM atomics issued: table flushes / probe-chain overflow
    if (!ABL(32)) {
        // (level, chunk) iterations, levels outer; the depth and the dL/dfeature pair of the
        // next iteration are loaded one iteration ahead (independent of this iteration's
        // gathers), so each iteration waits on one dependent round trip (the corner gather)
        typedef typename std::conditional<sizeof(TM) == 2, uint32_t, float2>::type GPair;
        const size_t RS = (size_t)a.R * a.S;
        const int n_it = nlev * nch;
        // unconditional loads (a lane past the list reads the ray's sample 0; the last iteration
        // re-reads a valid level): a branch around them made the compiler's wait counts conservative
        auto issue = [&](int lv, int ch, float &z, GPair &g, uint32_t &prt) {
            const int j = 64 * ch + lane;   // < 64 ceil(S / 64) <= 320: inside the list's LDS words
            const int sj_raw = (int)slist[j];
            const int sj = j < n_act ? sj_raw : 0;
            const size_t sid = (size_t)r * a.S + sj;
            prt = sj >= a.N_oct ? 1u : 0u;   // the around-depth part of the ray's samples
            z = a.zbuf[sid];
            g = reinterpret_cast<const GPair *>(a.dfeat)[(size_t)lv * RS + sid];
        };
        float z_nx = 0.f;
        GPair g_nx{};
        uint32_t prt_nx = 0u;
        issue(lv0, 0, z_nx, g_nx, prt_nx);
        // (level, chunk) of this iteration and of the next one, stepped without divisions
        int lv = lv0, ch = 0, lv_n = lv0, ch_n = 0;
        for (int it = 0; it < n_it; ++it) {
            const float z = z_nx;
            const GPair gq = g_nx;
            const uint32_t part = prt_nx;
            if (++ch_n == nch) { ch_n = 0; ++lv_n; }
            issue(min(lv_n, (int)a.L - 1), ch_n, z_nx, g_nx, prt_nx);
            const bool member = 64 * ch + lane < n_act;
            // unconditionally (a non-member lane's z, g are zero: finite values it never uses)
            float p[3], x[3], g0, g1;
            h2v g01;
            // the ray's pose rows re-read per iteration (scalar-cache hits): held across the loop they
            // took 15 SGPRs, which kept the kernel above the 80 that admit 8 waves per SIMD
            sample_point(load_ray<true>(a, r), z, p, x);   // a member's sample is inside the box (compaction)
            if constexpr (sizeof(TM) == 2) {
                g01 = __builtin_bit_cast(h2v, gq);
                g0 = (float)g01[0];
                g1 = (float)g01[1];
            } else {
                g01 = h2v{(_Float16)0.f, (_Float16)0.f};
                g0 = gq.x;
                g1 = gq.y;
            }
            const bool act = member && (g0 != 0.f || g1 != 0.f);
            if (ABL(1 << 25)) {   // utilisation probe (timing build): active lanes / busy-iteration lanes
                n_flush += __any(act) ? (int)__popcll(__ballot(act)) : 0;
                n_direct += (__any(act) && lane == 0) ? 64 : 0;
            }
            // timing build: ABL_SKIPQ skips a quarter of the levels (their gathers, scan, claims and
            // flush; the loads of the iteration stay) — the per-level-group split of the kernel time
            const bool skipq = ABL(ABL_SKIPQ(lv >> 2));
            if (__any(act) && !skipq) {
                const LevelInfo li = level_info_uniform(a, lv);   // lv is wave-uniform: a scalar load
                const float x01[3] = {(x[0] + 1) / 2, (x[1] + 1) / 2, (x[2] + 1) / 2};
                float gx[3] = {0.f, 0.f, 0.f};
                backward_level<TT, F16V>(a, li, member, act, part, x01, g0, g1, g01, gx, lane, keys, vals, mask, g32, g16,
                                         n_direct);
                // dL/dx_world = 0.5 dL/dx01 (grid.py:160)
#pragma unroll
                for (int i = 0; i < 3; ++i) {
                    sgz[i] = __builtin_fmaf(gx[i], z, sgz[i]);
                    sg[i] += gx[i];
                }
            }
            if (ch == nch - 1 && !ABL(1) && !ABL(1 << 22) && !skipq) {
                const int nfl = flush_table<F16V>(keys, vals, mask, lane, g32, g16, ABL(128));
                n_flush += nfl;
            }
            if (++ch == nch) { ch = 0; ++lv; }
        }
    }
    if (!a.no_dx) {
        float tz[3], t1[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) {
            tz[i] = 0.5f * wave_sum(sgz[i]);
            t1[i] = 0.5f * wave_sum(sg[i]);
        }
        if (lane < 12) {
            const int i = lane >> 2, j = lane & 3;
            const float gzi = i == 0 ? tz[0] : (i == 1 ? tz[1] : tz[2]);
            const float g1i = i == 0 ? t1[0] : (i == 1 ? t1[1] : t1[2]);
            const float dj = j == 0 ? c.dir[0] : (j == 1 ? c.dir[1] : c.dir[2]);
            const float v = j < 3 ? gzi * dj : g1i;
            if (ngrp == 1) a.ray_grad[(size_t)r * 12 + lane] += v;
            else atomic_add_f32(a.ray_grad + (size_t)r * 12 + lane, v);
        }
    }
    // HBM atomic counters (diagnostics, count_atomics only: 9 us of NerfRunner.train's 0.31 ms step
    // otherwise), spread over 64 slot pairs: one hot address taking an atomic from every wave
    // serialises at the memory side (~0.45 ms per step)
    // n_flush is wave-uniform (ballot counts in flush_table), n_direct per lane
    if (!a.count_atomics || ABL(16384)) return;
    const float nf = (float)__builtin_amdgcn_readfirstlane(n_flush), nd = wave_sum((float)n_direct);
    float *cnt = a.loss_acc + 8 + 2 * (r & 63);
    if (lane == 0 && nf != 0.f) atomic_add_f32(cnt, nf);
    if (lane == 0 && nd != 0.f) atomic_add_f32(cnt + 1, nd);
}

// ------------------------------------------- SDF query (mesh extraction)
// run_network_density (nerf_runner.py:1306-1346) on a dense grid or a point
// list: clip to [-1,1], multires encode, sigma net (L1, ReLU, L2) -> sdf.
// Grid mode follows extract_mesh (:1349-1382): point (i,j,k) = (gx[i], gy[j],
// gz[k]) in meshgrid 'ij' order; points whose octree voxel at the ray-tracing
// level is empty are not queried and read 1.0. One wave per 32 points; the
// encode is spread over both lane halves exactly as in k_encode and the MLP
// runs on MFMA with the weights staged in LDS.
struct QueryArgs {
    const float *pts;                  // [n,3] (point mode) or null
    const float *gx, *gy, *gz;         // grid axes (grid mode)
    int nx, ny, nz;
    int64_t n;
    const uint8_t *occ;                // [N^3] occupancy at the ray-tracing level (x fastest) or null
    int occ_n;
    float *sdf;                        // [n]
};

template <typename TM, typename TT>
__global__ __launch_bounds__(256) void k_query_sdf(FieldArgs a, QueryArgs q) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    TM *s_fr = reinterpret_cast<TM *>(smem);
    float *s_b = reinterpret_cast<float *>(smem + N_FRAGS * 64 * 8 * sizeof(TM));
    {
        const uint4 *src = reinterpret_cast<const uint4 *>(a.frags);
        uint4 *dst = reinterpret_cast<uint4 *>(s_fr);
        for (int i = threadIdx.x; i < N_FRAGS * 64 * 8 * (int)sizeof(TM) / 16; i += blockDim.x) dst[i] = src[i];
        for (int i = threadIdx.x; i < 5 * 64; i += blockDim.x) s_b[i] = a.bias[i];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, n = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t ntile = (q.n + 31) / 32;
    for (int64_t t = (int64_t)blockIdx.x * 4 + wave; t < ntile; t += (int64_t)gridDim.x * 4) {
        const int64_t idx = t * 32 + n;
        const bool inb = idx < q.n;
        float x[3] = {0.f, 0.f, 0.f};
        if (inb) {
            if (q.pts) {
#pragma unroll
                for (int d = 0; d < 3; ++d) x[d] = q.pts[idx * 3 + d];
            } else {
                const int64_t k = idx % q.nz, ij = idx / q.nz;
                const int64_t j = ij % q.ny, i = ij / q.ny;
                x[0] = q.gx[i]; x[1] = q.gy[j]; x[2] = q.gz[k];
            }
        }
        bool valid = inb;
        if (inb && q.occ) {   // OctreeManager.get_center_ids >= 0 (Utils.py:392-394)
            const float N = (float)q.occ_n;
            uint32_t c[3];
            bool inside = true;
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                inside = inside && fabsf(x[d]) <= 1.f;
                const float f = floorf((x[d] + 1.f) * 0.5f * N);
                c[d] = (uint32_t)fminf(fmaxf(f, 0.f), N - 1.f);
            }
            valid = inside && q.occ[((size_t)c[2] * q.occ_n + c[1]) * q.occ_n + c[0]] != 0;
        }
        if (!__any(valid)) {
            if (inb && h == 0) q.sdf[idx] = 1.f;
            continue;
        }
#pragma unroll
        for (int d = 0; d < 3; ++d) x[d] = fminf(fmaxf(x[d], -1.f), 1.f);   // torch.clip(inputs, -1, 1)
        const float x01[3] = {(x[0] + 1) / 2, (x[1] + 1) / 2, (x[2] + 1) / 2};
        Acts<TM> A;
#pragma unroll
        for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
            for (int qq = 0; qq < 4; ++qq) {
                const int lv = lane_level(ss, qq, h);
                float v[2] = {0.f, 0.f};
                if (inb && lv < (int)a.L) encode_level<TT>(a, level_info(a, lv), x01, v);
                frag_set<TM>(A.X[ss], 2 * qq, v[0]);
                frag_set<TM>(A.X[ss], 2 * qq + 1, v[1]);
            }
        }
        float sdf;
        f16v l2;
        mlp_sdf_net<TM>(LdsW<TM>{s_fr}, s_b, A, lane, sdf, l2);
        if (inb && h == 0) q.sdf[idx] = valid ? sdf : 1.f;
    }
}

// end of the field pass: loss_acc[LOSS_FOLD_DST[k]] += sum of the LOSS_COPIES copies of slot k
__device__ __forceinline__ void loss_fold(const float *__restrict__ part, float *__restrict__ loss_acc, int k) {
    if (k >= LOSS_FOLD_N) return;
    constexpr int dst[LOSS_FOLD_N] = {0, 1, 2, 3, 4, 5, LOSS_ACC_COUNTERS, LOSS_ACC_COUNTERS + 1, LOSS_ACC_COUNTERS + 2,
                                      LOSS_ACC_COUNTERS + 3, LOSS_ACC_COUNTERS + 4, LOSS_ACC_COUNTERS + 5,
                                      LOSS_ACC_COUNTERS + 6};
    float s = 0.f;
    for (int c = 0; c < LOSS_COPIES; ++c) s += part[c * LOSS_SLOTS + k];
    loss_acc[dst[k]] += s;
}

// xy-quad mirror of the fp16 table for k_encode (amp, dense levels): quad r = the fp16 pairs of
// rows {r, r+1, r+rs, r+rs+1} of r's level (rs = res + 1), i.e. the corners (x, y), (x+1, y),
// (x, y+1), (x+1, y+1) of the cell whose (x, y, z) corner is row r. A cell's 8 corners are then
// the quads at its base row and base + rs^2: two 16-B loads instead of four 8-B pair loads
// (k_encode's corner gathers are bound by L1 line accesses: 26 per sample with pairs). Rebuilt
// from the mirror at the start of every field pass (the optimiser / all-gather update the
// pairs); rows whose quad would leave the level (never a cell corner) and hashed levels are
// not written. One row per thread (16-B stores of consecutive lanes are contiguous; four rows per
// thread with one 16-B load each measured 49 vs 29 us at the headline).
__global__ __launch_bounds__(256) void k_quad_mirror(FieldArgs a) {
    // persistent grid over the dense levels' rows (a prefix of the table: levels are stored
    // coarse to fine and a level is dense up to its first hashed one); the level records in LDS,
    // each thread's level advanced as its rows grow (a per-block scalar walk from level 0 was a
    // dependent load chain per 256 rows)
    __shared__ uint32_t s_off[16], s_rs[16], s_end[16];
    if (threadIdx.x < a.L) {
        const LevelInfo li = level_info(a, threadIdx.x);
        s_off[threadIdx.x] = li.off;
        s_rs[threadIdx.x] = li.res + 1;
        s_end[threadIdx.x] = level_dense(li.res + 1, li.hs) ? li.off + li.hs : 0u;
    }
    __syncthreads();
    uint32_t end = 0;
    for (int l = 0; l < (int)a.L && s_end[l]; ++l) end = s_end[l];
    const uint32_t *t = reinterpret_cast<const uint32_t *>(a.table);
    uint4 *quads = const_cast<uint4 *>(a.quads);
    int lv = 0;
    for (uint32_t i = blockIdx.x * 256u + threadIdx.x; i < end; i += gridDim.x * 256u) {
        while (lv + 1 < (int)a.L && s_off[lv + 1] <= i) ++lv;
        const uint32_t rs = s_rs[lv], hi = i + rs + 1;
        if (hi >= s_end[lv]) continue;   // the quad would leave the level: never a cell corner
        quads[i] = make_uint4(t[i], t[i + 1], t[i + rs], t[hi]);
    }
}

__global__ void k_zero_i32(int *__restrict__ p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0;
}

// ---------------------------------------------------- ray setup + trace
__global__ __launch_bounds__(256) void k_trace(const float *__restrict__ pool, const int32_t *__restrict__ ids, int R,
                                               const float *__restrict__ tf, const uint8_t *__restrict__ occ, int N,
                                               int Kmax, float near_sc, float far_sc, float trunc,
                                               float *__restrict__ rays_out, float *__restrict__ intervals,
                                               float *__restrict__ totals, int32_t *__restrict__ counts,
                                               const nof_step_params *__restrict__ sp,
                                               const int32_t *__restrict__ epoch_step0) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
    if (sp) trunc = sp->trunc;
    // epoch permutation (nof_trace_rays_epoch): this step's slice, from the device step block
    if (epoch_step0) ids += (size_t)(sp->step - *epoch_step0) * (size_t)R;
    const float *src = pool + (size_t)(ids ? ids[r] : r) * 12;
    float ray[12];
#pragma unroll
    for (int k = 0; k < 12; ++k) ray[k] = src[k];
    if (ids) {
#pragma unroll
        for (int k = 0; k < 12; ++k) rays_out[(size_t)r * 12 + k] = ray[k];
    }
    const float nrm = sqrtf((ray[0] * ray[0] + ray[1] * ray[1]) + ray[2] * ray[2]);
    const float vd[3] = {ray[0] / nrm, ray[1] / nrm, ray[2] / nrm};
    const float *T = tf + (size_t)((int)ray[8]) * 16;
    const float o[3] = {T[3], T[7], T[11]};
    float d[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) d[i] = (T[i * 4] * vd[0] + T[i * 4 + 1] * vd[1]) + T[i * 4 + 2] * vd[2];
    float *dst = intervals + (size_t)r * Kmax * 2;
    // depths_in_out -> z (sample_rays_uniform_occupied_voxels :986-998; note the second normalisation),
    // applied to each interval as the trace emits it (no read-back of the written intervals)
    const float n2 = sqrtf((vd[0] * vd[0] + vd[1] * vd[1]) + vd[2] * vd[2]);
    const float vz = fabsf(vd[2] / n2);
    const float depth = ray[6];
    const bool vdepth = (depth >= near_sc) && (depth <= far_sc);
    const float hi = depth + trunc;
    float total = 0.f;
    const int k = trace_ray_emit(occ, N, o, d, Kmax, [&](int j, float tin, float tout) {
        float zi = tin * vz, zo = tout * vz;
        if (vdepth && zi > 0.f && zo > 0.f) {
            zi = fminf(fmaxf(zi, 0.f), hi);
            zo = fminf(fmaxf(zo, 0.f), hi);
        }
        *reinterpret_cast<float2 *>(dst + j * 2) = make_float2(zi, zo);
        total += zo - zi;
    });
    // one zero entry ends the list (sample_z's walk stops at the first zero z_in, as the reference's
    // common.cu walk over its zero-padded depths_in_out): the rest of the row is never read, and
    // zero-padding all Kmax entries was most of this kernel's HBM writes
    if (k < Kmax) *reinterpret_cast<float2 *>(dst + k * 2) = make_float2(0.f, 0.f);
    totals[r] = total;
    if (counts) counts[r] = k;
}

// ------------------------------------------------------------ MLP pack
template <typename TM>
__global__ __launch_bounds__(256) void k_pack_mlp(const float *__restrict__ mlp, const int32_t *__restrict__ idx,
                                                  int n_frag_elems, int n_bias, TM *__restrict__ frags,
                                                  float *__restrict__ bias) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n_frag_elems) {
        const int k = idx[i];
        frags[i] = (TM)(k >= 0 ? mlp[k] : 0.f);
    } else if (i < n_frag_elems + n_bias) {
        const int k = idx[i];
        bias[i - n_frag_elems] = k >= 0 ? mlp[k] : 0.f;
    }
}

// -------------------------------------------------------------- batch
// Throughput-mode ray selection: rays_per_frame uniform draws (with replacement)
// inside each frame's contiguous pool segment (frame_start [F+1]), one block per frame,
// produced already in ascending pool (raster) order, so neighbouring waves trace neighbouring
// pixels and share their table rows in L2. The k sorted draws are generated directly as the
// order statistics of k uniforms: U_(j) = S_j / S_k with S_j = E_0 + ... + E_j the prefix sums
// of k + 1 exponential variates (E = -log u, counter-hash u) — one block-wide prefix sum
// instead of a bitonic sort of the draws (66 barrier stages for 2048: ~26 us per step on the
// 64 frames' blocks); id_j = lo + floor(cnt U_(j)) has the distribution of k sorted iid
// uniform draws from the frame's rays.
constexpr int SAMPLE_BATCH_MAX = 4096;
__global__ __launch_bounds__(1024) void k_sample_batch(const int64_t *__restrict__ frame_start, int F,
                                                      int rays_per_frame, uint32_t seed, int32_t *__restrict__ ids,
                                                      const nof_step_params *__restrict__ sp) {
    if (sp) seed = sp->batch_seed;
    __shared__ float s_t[1024];
    const int f = blockIdx.x, t = threadIdx.x;
    const int k = rays_per_frame, m = k + 1;
    const int chunk = (m + 1023) / 1024;   // <= 5 (rays_per_frame <= 4096)
    const int j0 = t * chunk, j1 = min(m, j0 + chunk);
    const int64_t lo = frame_start[f], cnt = frame_start[f + 1] - lo;
    // this thread's exponential variates, their running sum
    float e[5];
    float run = 0.f;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        e[q] = 0.f;
        const int j = j0 + q;
        if (q < chunk && j < j1) {
            const uint32_t i = (uint32_t)(f * m + j);
            const uint32_t u = hash32(seed ^ hash32(i * 0x85EBCA6BU + 0x27D4EB2FU));
            e[q] = -__logf(((float)u + 0.5f) * 2.3283064e-10f);   // u in (0, 1)
            run += e[q];
        }
    }
    // block-wide inclusive scan of the threads' sums (Hillis-Steele in LDS)
    s_t[t] = run;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        const float x = s_t[t] + (t >= off ? s_t[t - off] : 0.f);
        __syncthreads();
        s_t[t] = x;
        __syncthreads();
    }
    const float total = s_t[1023];
    float acc = t > 0 ? s_t[t - 1] : 0.f;
    const float scale = (float)cnt / total;
#pragma unroll
    for (int q = 0; q < 5; ++q) {
        const int j = j0 + q;
        if (q < chunk && j < min(j1, k)) {   // S_j for j < k (S_k = total, the normaliser)
            acc += e[q];
            int64_t id = (int64_t)(acc * scale);
            id = (id < 0 || cnt <= 0) ? 0 : (id >= cnt ? cnt - 1 : id);
            ids[(size_t)f * k + j] = (int32_t)(lo + id);
        }
    }
}

}  // namespace nof

extern "C" int nof_trace_rays(const float *pool, const int32_t *ids, int32_t R, const float *tf, const uint8_t *occ,
                              int32_t N, int32_t Kmax, float near_sc, float far_sc, float trunc, float *rays_out,
                              float *intervals, float *totals, int32_t *counts, const nof_step_params *sp,
                              void *stream) {
    if (R <= 0) return NOF_OK;
    if (N <= 0 || Kmax <= 0) return nof::set_error(NOF_EINVAL, "trace_rays: bad N=%d Kmax=%d", N, Kmax);
    // one lane per ray: small batches (NerfRunner.train's 2048 rays) in 64-lane blocks, so the rays'
    // serial DDA chains spread over 32 CUs instead of 8
    const int tb = R >= 65536 ? 256 : 64;
    hipLaunchKernelGGL(nof::k_trace, dim3(nof::div_up(R, tb)), dim3(tb), 0, (hipStream_t)stream, pool, ids, R, tf,
                       occ, N, Kmax, near_sc, far_sc, trunc, rays_out, intervals, totals, counts, sp,
                       (const int32_t *)nullptr);
    return nof::check_launch("trace_rays");
}

extern "C" int nof_trace_rays_epoch(const float *pool, const int32_t *perm, const int32_t *epoch_step0, int32_t R,
                                    const float *tf, const uint8_t *occ, int32_t N, int32_t Kmax, float near_sc,
                                    float far_sc, float trunc, float *rays_out, float *intervals, float *totals,
                                    int32_t *counts, const nof_step_params *sp, void *stream) {
    if (R <= 0) return NOF_OK;
    if (!perm || !epoch_step0 || !sp)
        return nof::set_error(NOF_EINVAL, "trace_rays_epoch: perm, epoch_step0 and the step block are required");
    if (N <= 0 || Kmax <= 0) return nof::set_error(NOF_EINVAL, "trace_rays_epoch: bad N=%d Kmax=%d", N, Kmax);
    const int tb = R >= 65536 ? 256 : 64;
    hipLaunchKernelGGL(nof::k_trace, dim3(nof::div_up(R, tb)), dim3(tb), 0, (hipStream_t)stream, pool, perm, R, tf,
                       occ, N, Kmax, near_sc, far_sc, trunc, rays_out, intervals, totals, counts, sp, epoch_step0);
    return nof::check_launch("trace_rays_epoch");
}

extern "C" int nof_pack_mlp(const float *mlp, const int32_t *idx, int32_t n_frag_elems, int32_t n_bias, void *frags,
                            float *bias, int mlp_dtype, void *stream) {
    const int n = n_frag_elems + n_bias;
    if (mlp_dtype == NOF_F16)
        hipLaunchKernelGGL(nof::k_pack_mlp<_Float16>, dim3(nof::div_up(n, 256)), dim3(256), 0, (hipStream_t)stream,
                           mlp, idx, n_frag_elems, n_bias, (_Float16 *)frags, bias);
    else
        hipLaunchKernelGGL(nof::k_pack_mlp<float>, dim3(nof::div_up(n, 256)), dim3(256), 0, (hipStream_t)stream, mlp,
                           idx, n_frag_elems, n_bias, (float *)frags, bias);
    return nof::check_launch("pack_mlp");
}

extern "C" int nof_sample_batch(const int64_t *frame_start, int32_t F, int32_t rays_per_frame, uint32_t seed,
                                int32_t *ids, const nof_step_params *sp, void *stream) {
    const int n = F * rays_per_frame;
    if (n <= 0) return NOF_OK;
    if (rays_per_frame > nof::SAMPLE_BATCH_MAX)
        return nof::set_error(NOF_EINVAL, "sample_batch: rays_per_frame %d > %d", rays_per_frame,
                              nof::SAMPLE_BATCH_MAX);
    // one block of 1024 threads per frame: the bitonic stages run 2 compare-swaps per thread
    // (256 threads took 8 per stage, ~60 us per 64-frame batch)
    hipLaunchKernelGGL(nof::k_sample_batch, dim3(F), dim3(1024), 0, (hipStream_t)stream, frame_start,
                       F, rays_per_frame, seed, ids, sp);
    return nof::check_launch("sample_batch");
}

namespace {
// Optional per-kernel timing (nof_field_timing): one set of events per call,
// recorded on the launch stream between the kernels.
constexpr int N_FIELD_KERNELS = 4;   // encode, mlp_fwd (+ compact), mlp_bwd (2 passes), scatter
struct FieldTiming {
    bool on = false;
    std::vector<std::array<hipEvent_t, N_FIELD_KERNELS + 1>> sets;
    size_t used = 0;
};
FieldTiming g_timing;
hipEvent_t *timing_set() {
    if (!g_timing.on) return nullptr;
    if (g_timing.used == g_timing.sets.size()) {
        std::array<hipEvent_t, N_FIELD_KERNELS + 1> e{};
        for (auto &x : e)
            if (hipEventCreate(&x) != hipSuccess) return nullptr;
        g_timing.sets.push_back(e);
    }
    return g_timing.sets[g_timing.used++].data();
}
inline void mark(hipEvent_t *ev, int i, hipStream_t st) {
    if (ev) (void)hipEventRecord(ev[i], st);
}

template <typename TM, typename TT, int WPB>
int launch_field(const nof::FieldArgs &a, int n_cu, hipStream_t st) {
    const int ntiles = a.S / 32;
    // the record counter and the loss rows (contiguous in the workspace) are reset by a kernel, not
    // a memset: the step is captured into a hipGraph, and kernel nodes are the only node kind it holds
    hipLaunchKernelGGL(nof::k_ray_ctx, dim3(nof::div_up(a.R, 256)), dim3(256), 0, st, a);
    hipEvent_t *ev = timing_set();
    mark(ev, 0, st);
    if (a.quads && !a.quads_ready)   // amp, large batches: the encode's xy-quad mirror (timed with k_encode)
        hipLaunchKernelGGL(nof::k_quad_mirror, dim3((int)std::min<int64_t>((int64_t)n_cu * 8, nof::div_up(a.n_rows, 256))), dim3(256), 0, st, a);
    // encode + sigma net: 8-wave blocks (the layer-1 / 2 fragments staged once per 8 tiles)
    // weights + biases + 8 waves' level tables (16 levels x 32 B)
    const size_t elds = (size_t)8 * 64 * 8 * sizeof(TM) + 2 * 64 * sizeof(float) + 8 * 16 * 32;
    {
        const dim3 eg(nof::div_up((uint64_t)a.R * ntiles, 8));
        if (a.dbg_z || a.dbg_valid || a.dbg_raw) {
            if (a.encode_group == 4) hipLaunchKernelGGL((nof::k_encode<TM, TT, 4, true>), eg, dim3(512), elds, st, a);
            else if (a.encode_group == 2) hipLaunchKernelGGL((nof::k_encode<TM, TT, 2, true>), eg, dim3(512), elds, st, a);
            else hipLaunchKernelGGL((nof::k_encode<TM, TT, 1, true>), eg, dim3(512), elds, st, a);
        } else {
            if (a.encode_group == 4) hipLaunchKernelGGL((nof::k_encode<TM, TT, 4, false>), eg, dim3(512), elds, st, a);
            else if (a.encode_group == 2) hipLaunchKernelGGL((nof::k_encode<TM, TT, 2, false>), eg, dim3(512), elds, st, a);
            else hipLaunchKernelGGL((nof::k_encode<TM, TT, 1, false>), eg, dim3(512), elds, st, a);
        }
    }
    int rc = nof::check_launch("field_step(encode)");
    if (rc) return rc;
    mark(ev, 1, st);
    // tile-parallel colour forward: the colour-tile list comes from the same compaction pass as
    // the backward list (the flags are final after k_encode)
    {
        const int nflags = a.R * ntiles;
        const int per = a.compact_per > 0 ? a.compact_per : (nflags >= 262144 ? nof::COMPACT_PER_BLOCK : 512);
        hipLaunchKernelGGL(nof::k_compact, dim3(nof::div_up((uint64_t)nflags, per)), dim3(256), 0, st, a.tile_bwd,
                           nflags, a.tile_sid, a.n_tiles, per, a.ctile_list);
        rc = nof::check_launch("field_step(compact)");
        if (rc) return rc;
        // 4-wave blocks, 6 per CU (6 waves per SIMD at 80 registers; 17 KB of colour-net fragments per block):
        // 5 per CU measured 0.249 / 0.247 ms, 6 0.237 / 0.234, 8 (64 registers, spilling) 0.394 (profiles/r5/ab_r5m_*)
        constexpr int WPB_C = 4;
        const int nbc = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)n_cu * 6, ((int64_t)nflags + 7) / 8));
        const size_t clds = nof::colour_lds_bytes<TM>();
        if (a.dbg_raw)
            hipLaunchKernelGGL((nof::k_colour<TM, WPB_C, 6, true>), dim3(nbc), dim3(WPB_C * 64), clds, st, a);
        else
            hipLaunchKernelGGL((nof::k_colour<TM, WPB_C, 6, false>), dim3(nbc), dim3(WPB_C * 64), clds, st, a);
        rc = nof::check_launch("field_step(colour)");
        if (rc) return rc;
        hipLaunchKernelGGL(nof::k_ray_final, dim3(nof::div_up(a.R, 256)), dim3(256), 0, st, a);
        rc = nof::check_launch("field_step(ray_final)");
        if (rc) return rc;
    }
    mark(ev, 2, st);
    // + 16 floats: k_mlp_bwd's per-wave frame-feature gradient sums
    const size_t mlds = (size_t)nof::N_FRAGS * 64 * 8 * sizeof(TM) + 5 * 64 * sizeof(float) + 16 * sizeof(float);
    if constexpr (sizeof(TM) == 2) {
        // amp: the weight gradients take their K = samples operands from LDS transposes
        // (k_mlp_bwd_tr): 8-wave blocks (12 KB of images per wave), one per CU
        // the weight gradients summed over the 8-wave block before the atomics (8 x fewer; bwd_flush 0 / 2,
        // the default; 1: one atomic per element per wave), the grid widened to every CU. Measured
        // against the per-wave flush (round 4, same box): 2048 rays 0.351 ->
        // 0.306 ms per step, 16 K rays 0.255 -> 0.161 ms, 32 K 0.372 -> 0.309, 64 K 0.603 -> 0.576,
        // the 131 K-ray headline 1.109 -> 1.086 and 1.123 -> 1.107 ms
        const int64_t nt_all = (int64_t)a.R * ntiles;
        const bool blk = a.bwd_flush != 1;
        const int nbt = (int)std::max<int64_t>(1, std::min<int64_t>(n_cu, (nt_all + (blk ? 47 : 127)) / (blk ? 48 : 128)));
        const size_t tl0 = nof::bwd_tr_lds(0, 8), tl1 = nof::bwd_tr_lds(1, 8);
        if (a.n_ff > 0) {
            if (blk) hipLaunchKernelGGL((nof::k_mlp_bwd_tr<8, 0, true, true>), dim3(nbt), dim3(8 * 64), tl0, st, a);
            else hipLaunchKernelGGL((nof::k_mlp_bwd_tr<8, 0, true>), dim3(nbt), dim3(8 * 64), tl0, st, a);
        } else {
            if (blk) hipLaunchKernelGGL((nof::k_mlp_bwd_tr<8, 0, false, true>), dim3(nbt), dim3(8 * 64), tl0, st, a);
            else hipLaunchKernelGGL((nof::k_mlp_bwd_tr<8, 0>), dim3(nbt), dim3(8 * 64), tl0, st, a);
        }
        rc = nof::check_launch("field_step(mlp_bwd_tr0)");
        if (rc) return rc;
        if (blk) hipLaunchKernelGGL((nof::k_mlp_bwd_tr<8, 1, false, true>), dim3(nbt), dim3(8 * 64), tl1, st, a);
        else hipLaunchKernelGGL((nof::k_mlp_bwd_tr<8, 1>), dim3(nbt), dim3(8 * 64), tl1, st, a);
        rc = nof::check_launch("field_step(mlp_bwd_tr1)");
        if (rc) return rc;
    } else {
        // fp32 (parity mode): two persistent passes of 4-wave blocks; small batches get fewer persistent
        // waves (~16 tiles of the batch per wave), so the per-wave weight-gradient atomics at the end do
        // not outweigh the tiles. Pass 1 would spill at 2 waves per SIMD in fp32 and keeps one.
        const int nbb = (int)std::max<int64_t>(1, std::min<int64_t>(n_cu * 2, ((int64_t)a.R * ntiles + 63) / 64));
        hipLaunchKernelGGL((nof::k_mlp_bwd<TM, 4, 2, 0>), dim3(nbb), dim3(4 * 64), mlds, st, a);
        rc = nof::check_launch("field_step(mlp_bwd0)");
        if (rc) return rc;
        const int nb1 = std::min(nbb, n_cu);
        if (a.n_ff > 0) hipLaunchKernelGGL((nof::k_mlp_bwd<TM, 4, 1, 1, true>), dim3(nb1), dim3(4 * 64), mlds, st, a);
        else hipLaunchKernelGGL((nof::k_mlp_bwd<TM, 4, 1, 1>), dim3(nb1), dim3(4 * 64), mlds, st, a);
        rc = nof::check_launch("field_step(mlp_bwd)");
        if (rc) return rc;
    }
    mark(ev, 3, st);
    const int n_grp = ((int)a.L + a.scatter_lpw - 1) / a.scatter_lpw;
    const dim3 sg(nof::div_up((uint64_t)a.R * n_grp, 4));
    // per-ray table accumulation in LDS: amp adds packed fp16x2 (the reference's __half2
    // atomicAdd per sample and corner, gridencoder.cu:319-327, rounds once per sample; here
    // once per DPP run of samples — 0.16 ms less per config-2 step than fp32 pairs), fp32
    // mode adds fp32 pairs
    if constexpr (sizeof(TM) == 2) {
        const size_t lds = (size_t)4 * 4 * nof::scatter_wave_words(a.slot_mask, 1);
        hipLaunchKernelGGL((nof::k_scatter<TM, TT, true, 7>), sg, dim3(256), lds, st, a);
    } else {
        hipLaunchKernelGGL((nof::k_scatter<TM, TT, false, 1>), sg, dim3(256),
                           (size_t)4 * 4 * nof::scatter_wave_words(a.slot_mask, 2), st, a);
    }
    rc = nof::check_launch("field_step(scatter)");
    if (rc) return rc;
    mark(ev, 4, st);
    return NOF_OK;
}
}  // namespace

namespace {
struct FieldWorkspace {
    size_t feat, dfeat, zbuf, tile_bwd, tile_sid, n_tiles, ray_aux, tile_aux, rctx, gmask, rrec, ctile, total;
    FieldWorkspace(int R, int S, int mlp_dtype) {
        auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
        const size_t el = mlp_dtype == NOF_F16 ? 2 : 4, n = (size_t)R * S, nt = (size_t)R * (S / 32);
        size_t o = 0;
        feat = o; o += al(n * 32 * el);
        dfeat = o; o += al(n * 32 * el);
        zbuf = o; o += al(n * 4);
        tile_bwd = o; o += al(nt);
        tile_sid = o; o += al(nt * 4);
        n_tiles = o; o += al(4 * nof::LOSS_ZERO_WORDS);   // + the loss rows (folded by the scatter kernel)
        ray_aux = o; o += al((size_t)R * nof::RAY_AUX * 4);
        tile_aux = o; o += al(nt * nof::TILE_AUX * 16);
        rctx = o; o += al((size_t)R * nof::RCTX * 4);
        gmask = o; o += al(nt * 4);
        rrec = o; o += al(nt * nof::TREC * 4);
        ctile = o; o += al(nt * 4);
        total = o;
    }
};
}  // namespace

extern "C" size_t nof_field_workspace_bytes(int32_t R, int32_t S, int32_t mlp_dtype) {
    return FieldWorkspace(R, S, mlp_dtype).total;
}

extern "C" int nof_field_workspace_offsets(int32_t R, int32_t S, int32_t mlp_dtype, uint64_t *offsets, int32_t n) {
    if (R < 0 || S <= 0 || !offsets || n < NOF_WS_SECTIONS)
        return nof::set_error(NOF_EINVAL, "field_workspace_offsets: bad R=%d S=%d or n=%d < %d", R, S, n,
                              NOF_WS_SECTIONS);
    const FieldWorkspace w(R, S, mlp_dtype);
    const size_t o[NOF_WS_SECTIONS] = {w.feat, w.dfeat, w.zbuf, w.tile_bwd, w.tile_sid, w.n_tiles, w.ray_aux,
                                       w.tile_aux, w.rctx, w.gmask, w.rrec, w.ctile, w.total};
    for (int i = 0; i < NOF_WS_SECTIONS; ++i) offsets[i] = o[i];
    return NOF_OK;
}

namespace {
// the encode's xy-quad mirror: amp, batches large enough to repay its per-step rebuild (~25 us)
bool quads_on(const nof_field_desc *d) {
    return d->table_quads && d->table_rows > 0 && d->mlp_dtype == NOF_F16 && d->table_dtype == NOF_F16 &&
           d->R >= (d->quads_min_rays > 0 ? d->quads_min_rays : 32768) && !ABL_HOST(d, 512);
}
}  // namespace

extern "C" int nof_quad_mirror(const nof_field_desc *d, void *stream) {
    if (d->L > 16 || d->C != 2)
        return nof::set_error(NOF_EINVAL, "quad_mirror: needs C=2, L<=16 (got %u,%u)", d->C, d->L);
    if (d->R <= 0 || !quads_on(d)) return NOF_OK;   // the step would not read the mirror
    nof::FieldArgs a{};
    a.table = d->table; a.levels = (const float4 *)d->levels; a.L = d->L;
    a.quads = (const uint4 *)d->table_quads; a.n_rows = (uint32_t)d->table_rows;
    int dev = 0, n_cu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n_cu = 256;
    hipLaunchKernelGGL(nof::k_quad_mirror, dim3((int)std::min<int64_t>((int64_t)n_cu * 8, nof::div_up(a.n_rows, 256))),
                       dim3(256), 0, (hipStream_t)stream, a);
    return nof::check_launch("quad_mirror");
}

extern "C" int nof_field_step(const nof_field_desc *d, void *stream) {
    if (d->S % 32 != 0 || d->S > 320 || d->N_oct + d->N_dep != d->S)
        return nof::set_error(NOF_EINVAL, "field_step: S=%d must be N_oct+N_dep, a multiple of 32, <= 320", d->S);
    if (d->L > 16 || d->C != 2 || d->D != 3)
        return nof::set_error(NOF_EINVAL, "field_step: needs D=3, C=2, L<=16 (got %u,%u,%u)", d->D, d->C, d->L);
    if (d->R <= 0) return NOF_OK;
    nof::FieldArgs a;
    a.rays = d->rays; a.tf = d->tf; a.intervals = d->intervals; a.totals = d->totals; a.t_rand = d->t_rand;
    a.seed = d->seed; a.R = d->R; a.Kmax = d->Kmax; a.N_oct = d->N_oct; a.N_dep = d->N_dep; a.S = d->S;
    a.perturb = d->perturb; a.near_sc = d->near_sc; a.far_sc = d->far_sc; a.trunc = d->trunc;
    a.ntr = d->neg_trunc_ratio; a.lambda = d->sdf_lambda; a.fs_sdf = d->fs_sdf; a.ffw = d->first_frame_weight;
    a.rgb_w = d->rgb_weight; a.fs_w = d->fs_weight; a.empty_w = d->empty_weight; a.trunc_w = d->trunc_weight;
    a.inv_3R = 1.0f / (3.0f * (float)d->R);
    a.inv_RS = 1.0f / ((float)d->R * (float)d->S);
    a.inv_3RS = 1.0f / (3.0f * (float)d->R * (float)d->S);
    a.xcd_order = d->xcd_order;
    a.no_dx = d->skip_pose_grad != 0;
    a.quads = quads_on(d) ? (const uint4 *)d->table_quads : nullptr;
    a.n_rows = (uint32_t)d->table_rows;
    a.quads_ready = d->quads_prebuilt != 0;
    {   // k_scatter: a wave per (ray, level group). Measured optimum (scripts/ablate.py LPW sweep,
        // DESIGN §4): a wave per ray from 192 K rays (config 5's 258 K: 13.2 vs 13.7 ms with 8),
        // 8 levels per wave from 32 K (the headline: 2.36 -> 2.29 ms vs a wave per ray; at 8 waves per
        // SIMD, round 6: 1.879 vs 1.917 ms, and config 2's 32 K rays 0.495 vs 0.512 ms with 4), 4 from
        // 8 K (16 K rays: 0.37 -> 0.33 ms vs 8; round 6: 0.294 vs 0.306), 2 below (NerfRunner.train's
        // 2048 rays: 0.418 -> 0.395 ms per step vs 1)
        const int L = std::max(1, (int)d->L);
        const int want = d->R >= 196608 ? 16 : (d->R >= 32768 ? 8 : (d->R >= 8192 ? 4 : 2));
        a.scatter_lpw = std::min(L, d->scatter_levels_per_wave > 0 ? (int)d->scatter_levels_per_wave : want);
        // the scatter_kernel values 1 (level-serial) and 3 (hybrid) and scatter_flat 1 were measured slower
        // at every batch size and removed: only the run-scan k_scatter remains
        // scatter_kernel 1 (level-serial), 3 (hybrid) and 4 (paired: two list entries per lane, two levels per
        // iteration) were measured slower and removed: only the run-scan k_scatter remains
        if (d->scatter_kernel != 0 && d->scatter_kernel != 2)
            return nof::set_error(NOF_EINVAL, "field_step: scatter_kernel %d (0 / 2: the run-scan scatter; 1, 3 and 4 "
                                  "were removed)", d->scatter_kernel);
        if (d->scatter_flat != 0)
            return nof::set_error(NOF_EINVAL, "field_step: scatter_flat was removed (must be 0)");
        a.scatter_lpw = std::max(1, a.scatter_lpw);
    }
    // encode_sigma 2 (sigma net in a per-ray forward kernel) and 3 (per-ray colour forward) were measured no
    // faster than the default and removed: the sigma net runs in k_encode, the colour net tile-parallel
    if (d->encode_sigma != 0 && d->encode_sigma != 1)
        return nof::set_error(NOF_EINVAL, "field_step: encode_sigma %d (0 / 1; 2 and 3 were removed)", d->encode_sigma);
    if (d->bwd_flush < 0 || d->bwd_flush > 2)
        return nof::set_error(NOF_EINVAL, "field_step: bwd_flush %d (0 by batch size, 1 per wave, 2 block)", d->bwd_flush);
    a.bwd_flush = d->bwd_flush;
    a.count_atomics = d->count_atomics != 0;
    if (d->compact_per_block != 0 && (d->compact_per_block < 256 || d->compact_per_block > nof::COMPACT_PER_BLOCK ||
                                      d->compact_per_block % 256 != 0))
        return nof::set_error(NOF_EINVAL, "field_step: compact_per_block %d (0 by batch size, else a multiple of 256 "
                              "in [256, %d])", d->compact_per_block, nof::COMPACT_PER_BLOCK);
    a.compact_per = d->compact_per_block;
    if (d->encode_group != 0 && d->encode_group != 1 && d->encode_group != 2 && d->encode_group != 4)
        return nof::set_error(NOF_EINVAL, "field_step: encode_group %d (0 by batch size, or 1, 2, 4)", d->encode_group);
    a.encode_group = d->encode_group ? d->encode_group : (d->R >= 8192 ? 1 : nof::ENCODE_GROUP_SMALL);
    if (d->mlp_pass1_tiles != 0 && d->mlp_pass1_tiles != 1)
        return nof::set_error(NOF_EINVAL, "field_step: mlp_pass1_tiles %d (0 / 1; several tiles per wave were "
                                          "measured slower and removed)", d->mlp_pass1_tiles);
    if (d->scatter_fuse_levels != 0 && d->scatter_fuse_levels != 1)
        return nof::set_error(NOF_EINVAL, "field_step: scatter_fuse_levels %d (0 / 1; level-fused scatter chunks "
                                          "were measured slower and removed)", d->scatter_fuse_levels);
    if (d->encode_wpb != 0 && d->encode_wpb != 8)
        return nof::set_error(NOF_EINVAL, "field_step: encode_wpb %d (0 / 8; 16-wave encode blocks were measured "
                                          "slower and removed)", d->encode_wpb);
    a.sp = d->step_params;
    a.fs_rgb_w = d->fs_rgb_weight;
    a.loss_scale = d->loss_scale; a.table = d->table; a.levels = (const float4 *)d->levels; a.L = d->L;
    a.mlp_in = (int)(d->L * d->C);
    if (d->n_ff < 0 || d->n_ff > 3 || (d->n_ff > 0 && (!d->ff || !d->grad_ff)))
        return nof::set_error(NOF_EINVAL, "field_step: frame_features must be 0..3 with ff and grad_ff set (got %d)",
                              d->n_ff);
    a.n_ff = d->n_ff; a.ff = d->ff; a.grad_ff = d->grad_ff;
    a.frags = d->frags; a.bias = d->bias; a.grad_table = d->grad_table; a.grad_mlp = d->grad_mlp;
    a.grad_table16 = (__half *)d->grad_table16;
    if (d->mlp_dtype == NOF_F16 && !d->grad_table16)
        return nof::set_error(NOF_EINVAL, "field_step: amp mode needs grad_table16 (fp16 table gradient)");
    a.ray_grad = d->ray_grad; a.loss_acc = d->loss_acc; a.dbg_z = d->dbg_z; a.dbg_raw = d->dbg_raw;
    a.dbg_valid = d->dbg_valid; a.dbg_rgb = d->dbg_rgb; a.ablate = d->ablate;
    if (d->ablate && !NOF_ABLATE)
        return nof::set_error(NOF_EINVAL, "field_step: ablate bits need a -DNOF_ABLATE=1 build (timing experiments only)");
    {
        char *w = (char *)d->workspace;
        if (!w) return nof::set_error(NOF_EINVAL, "field_step: workspace is NULL (nof_field_workspace_bytes)");
        const FieldWorkspace ws(d->R, d->S, d->mlp_dtype);
        a.feat = w + ws.feat;
        a.dfeat = w + ws.dfeat;
        a.zbuf = (float *)(w + ws.zbuf);
        a.tile_bwd = (uint8_t *)(w + ws.tile_bwd);
        a.tile_sid = (int *)(w + ws.tile_sid);
        a.n_tiles = (int *)(w + ws.n_tiles);
        a.loss_part = (float *)(w + ws.n_tiles) + 16;
        a.ray_aux = (float *)(w + ws.ray_aux);
        a.tile_aux = (float4 *)(w + ws.tile_aux);
        a.rctx = (float *)(w + ws.rctx);
        a.tile_gmask = (uint32_t *)(w + ws.gmask);
        a.rrec = (float *)(w + ws.rrec);
        a.ctile_list = (int *)(w + ws.ctile);
        const int slots = d->scatter_slots ? d->scatter_slots : 512;
        if (slots < 64 || slots > 2048 || (slots & (slots - 1)))
            return nof::set_error(NOF_EINVAL, "field_step: scatter_slots must be a power of two in [64, 2048]");
        a.slot_mask = (uint32_t)slots - 1;
    }
    hipStream_t st = (hipStream_t)stream;
    int dev = 0, n_cu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n_cu = 256;
    if (d->mlp_dtype == NOF_F16 && d->table_dtype == NOF_F16)
        return launch_field<_Float16, __half, 4>(a, n_cu, st);
    if (d->mlp_dtype == NOF_F32 && d->table_dtype == NOF_F32)
        return launch_field<float, float, 4>(a, n_cu, st);
    return nof::set_error(NOF_EINVAL, "field_step: mlp/table dtype must both be f16 (amp) or both f32");
}

extern "C" int nof_field_timing(int32_t enable) {
    g_timing.on = enable != 0;
    g_timing.used = 0;
    return NOF_OK;
}

extern "C" int nof_field_timing_collect(float *ms_sum, int32_t n, int32_t *calls) {
    if (!ms_sum || n < N_FIELD_KERNELS) return nof::set_error(NOF_EINVAL, "field_timing_collect: need 4 floats");
    for (int k = 0; k < n; ++k) ms_sum[k] = 0.f;
    for (size_t i = 0; i < g_timing.used; ++i) {
        auto &e = g_timing.sets[i];
        if (hipEventSynchronize(e[N_FIELD_KERNELS]) != hipSuccess)
            return nof::set_error(NOF_ELAUNCH, "field_timing_collect: event sync failed");
        for (int k = 0; k < N_FIELD_KERNELS; ++k) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, e[k], e[k + 1]) != hipSuccess)
                return nof::set_error(NOF_ELAUNCH, "field_timing_collect: elapsed time failed");
            ms_sum[k] += ms;
        }
    }
    if (calls) *calls = (int32_t)g_timing.used;
    g_timing.used = 0;
    return NOF_OK;
}

extern "C" int nof_query_sdf(const void *table, int32_t table_dtype, const float *level_table, uint32_t L,
                             const void *frags, const float *bias, int32_t mlp_dtype, int32_t mlp_in,
                             const float *points, int64_t n, const float *gx, const float *gy, const float *gz,
                             int32_t nx, int32_t ny, int32_t nz, const uint8_t *occ, int32_t occ_n, float *sdf,
                             void *stream) {
    if (!table || !level_table || !frags || !bias || !sdf || L == 0 || L > 16 || mlp_in != (int)L * 2)
        return nof::set_error(NOF_EINVAL, "query_sdf: bad table / MLP arguments (C = 2, L <= 16)");
    if (table_dtype != mlp_dtype) return nof::set_error(NOF_EINVAL, "query_sdf: table and MLP dtypes must match");
    if (!points && (!gx || !gy || !gz || nx <= 0 || ny <= 0 || nz <= 0))
        return nof::set_error(NOF_EINVAL, "query_sdf: need points or three grid axes");
    if (!points) n = (int64_t)nx * ny * nz;
    if (n <= 0) return NOF_OK;
    nof::FieldArgs a{};
    a.table = table;
    a.levels = reinterpret_cast<const float4 *>(level_table);
    a.L = L;
    a.mlp_in = mlp_in;
    a.frags = frags;
    a.bias = bias;
    nof::QueryArgs q{points, gx, gy, gz, nx, ny, nz, n, occ, occ_n, sdf};
    hipStream_t st = (hipStream_t)stream;
    int dev = 0, n_cu = 256;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        n_cu = 256;
    const int64_t ntile = (n + 31) / 32;
    const int blocks = (int)std::min<int64_t>((ntile + 3) / 4, (int64_t)n_cu * 2);
    if (mlp_dtype == NOF_F16) {
        const size_t lds = (size_t)nof::N_FRAGS * 64 * 8 * 2 + 5 * 64 * 4;
        hipLaunchKernelGGL((nof::k_query_sdf<_Float16, __half>), dim3(blocks), dim3(256), lds, st, a, q);
    } else {
        const size_t lds = (size_t)nof::N_FRAGS * 64 * 8 * 4 + 5 * 64 * 4;
        hipLaunchKernelGGL((nof::k_query_sdf<float, float>), dim3(blocks), dim3(256), lds, st, a, q);
    }
    return nof::check_launch("query_sdf");
}
