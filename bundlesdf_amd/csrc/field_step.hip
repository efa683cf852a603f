// Fused NeRF training step for gfx950 (CDNA4): ray setup + octree ray trace,
// stratified/around-depth sampling, multires grid encode, tiny MLP on MFMA,
// depth-guided compositing, SDF/free-space/colour losses and the complete
// backward pass (MLP weights, hash-table scatter, input gradient -> per-ray
// pose gradient). Replaces the per-step body of NerfRunner.train_loop
// (nerf_runner.py:677-762) — render_rays :1013-1128, the samplers
// :979-1010/:67-87, run_network :1226-1303, raw2outputs :1131-1168,
// get_sdf_loss nerf_helpers.py:382-399 and autograd.
//
// Work decomposition:
//  * k_trace: one lane per ray — DDA through the occupancy grid, intervals
//    converted to z, clipped at depth+trunc, summed.
//  * k_field: persistent; ONE WAVE PER RAY. A wave holds 32 samples x 2
//    halves (lane l: sample n = l & 31, half h = l >> 5). Pass A computes z,
//    the depth-guided weights and (only for tiles with non-zero weight) the
//    MLP colour to get rgb_map — a purely in-wave reduction, no barriers.
//    Pass B recomputes each tile's forward with the encode derivative,
//    evaluates the loss gradient in registers, runs the MLP backward on MFMA
//    (activations stay in VGPRs as B operands; weight gradients go through a
//    per-wave LDS transpose and a block-shared LDS fp32 accumulator), and
//    scatters the table gradient with device atomics. Per-ray pose gradients
//    (dL/dtf, 3x4) are written once per ray.
//  * Lane h handles levels {8s + 4(q>>1) + 2h + (q&1)}, s in 0..1, q in 0..3 —
//    the row set of its MFMA accumulator registers, so the encode output is
//    the layer-1 B operand in place and the layer-1 backward accumulator is
//    the scatter input in place.
#include <algorithm>

#include "nof_device.h"
#include "ray_trace.h"

#pragma clang fp contract(off)

namespace nof {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef float f16v __attribute__((ext_vector_type(16)));

constexpr int MLP_N_MAX = 9107;   // NeRFSmall(2x64, geo 15, colour 3x64), input <= 32, views 9
// flat-parameter offsets (MLP_KEYS order, bundlesdf_amd/mlp_layout.py) for input width IN
struct MlpOff {
    int w1, b1, w2, b2, w3, b3, w4, b4, w5, b5, n, in;
    __host__ __device__ MlpOff(int IN) : in(IN) {
        w1 = 0; b1 = 64 * IN; w2 = b1 + 64; b2 = w2 + 16 * 64; w3 = b2 + 16; b3 = w3 + 64 * 24; w4 = b3 + 64;
        b4 = w4 + 64 * 64; w5 = b4 + 64; b5 = w5 + 3 * 64; n = b5 + 3;
    }
};
// fragment ids (bundlesdf_amd/mlp_layout.py)
constexpr int FR_L1 = 0, FR_L2 = 4, FR_L3 = 8, FR_L4 = 12, FR_L5 = 20, FR_B5 = 24, FR_B4 = 26, FR_B3 = 34,
              FR_B2 = 38, FR_B1 = 42, N_FRAGS = 46;
constexpr float SH_C0 = 0.28209479177387814f, SH_C1 = 0.4886025119029199f;
constexpr float SH_C2_0 = 1.0925484305920792f, SH_C2_1 = -1.0925484305920792f, SH_C2_2 = 0.31539156525252005f,
                SH_C2_3 = -1.0925484305920792f, SH_C2_4 = 0.5462742152960396f;

struct FieldArgs {
    const float *rays;        // [R,12] batch (dir3 rgb3 depth mask frame type near far)
    const float *tf;          // [F,16] world_from_cam (pose correction applied), row-major
    const float *intervals;   // [R,Kmax,2] z units
    const float *totals;      // [R]
    const float *t_rand;      // [R,S] or null (counter RNG)
    uint32_t seed;
    int R, Kmax, N_oct, N_dep, S;
    int perturb;
    float near_sc, far_sc, trunc, ntr, lambda, fs_sdf, ffw, rgb_w, fs_w, empty_w, trunc_w;
    float inv_3R, inv_RS;
    const float *loss_scale;  // device scalar (GradScaler scale; 1 in fp32 mode)
    const void *table;        // [T,2] (float or half)
    const float4 *levels;     // [L]: scale, res (bits), row offset (bits), rows (bits)
    uint32_t L;
    int mlp_in;               // L*C
    const void *frags;        // [46][64][8] TM
    const float *bias;        // [5][64]
    float *grad_table;        // [T,2] f32 (fp32 mode)
    __half *grad_table16;     // [T,2] f16 (amp mode: the reference's __half2 gradient, gridencoder.cu:319-327)
    float *grad_mlp;          // [9107] f32
    float *ray_grad;          // [R,12]
    float *loss_acc;          // [4]: rgb, fs, empty, sdf (already normalised)
    float *dbg_z;             // [R,S]
    float *dbg_raw;           // [R,S,4]
    uint8_t *dbg_valid;       // [R,S]
    float *dbg_rgb;           // [R,3]
    int ablate;               // timing-only ablation bits (0 in every real run; results invalid otherwise)
};

// ----------------------------------------------------------------- helpers
__device__ __forceinline__ int acc_row(int q, int h) { return (q & 3) + 8 * (q >> 2) + 4 * h; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ __forceinline__ float half_sum(float v) {   // sum within each 32-lane half
#pragma unroll
    for (int o = 16; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.0f / (1.0f + __expf(-x)); }

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
// acc registers 8s..8s+7 -> fragment of K step s (optionally ReLU)
template <typename TM>
__device__ __forceinline__ void acc_to_frag(const f16v &acc, int s, bool relu, typename FragT<TM>::T &f) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        float v = acc[8 * s + j];
        frag_set<TM>(f, j, relu ? fmaxf(v, 0.f) : v);
    }
}

// -------------------------------------------------- per-wave LDS transposes
// image[row][sample] of TM with padded rows; filled from accumulator-layout
// values (row(q,h), column = sample n), read as 8 consecutive samples.
template <typename TM> struct Img {
    static constexpr int STRIDE = (sizeof(TM) == 2) ? 40 : 36;   // elements per row (pads 16 B)
    static constexpr int ROWS = 32;
    static constexpr int BYTES = ROWS * STRIDE * (int)sizeof(TM);
};

template <typename TM>
__device__ __forceinline__ void img_put_frag(TM *img, const typename FragT<TM>::T &f, int s, int h, int n) {
#pragma unroll
    for (int j = 0; j < 8; ++j) img[acc_row(8 * s + j, h) * Img<TM>::STRIDE + n] = (TM)frag_get<TM>(f, j);
}
template <typename TM>
__device__ __forceinline__ typename FragT<TM>::T img_get(const TM *img, int row, int col0) {
    typename FragT<TM>::T f;
    const TM *p = img + row * Img<TM>::STRIDE + col0;
    if constexpr (sizeof(TM) == 2) {
        f = *reinterpret_cast<const h8v *>(p);
    } else {
        const float4 a = *reinterpret_cast<const float4 *>(p), b = *reinterpret_cast<const float4 *>(p + 4);
        f.v[0] = a.x; f.v[1] = a.y; f.v[2] = a.z; f.v[3] = a.w; f.v[4] = b.x; f.v[5] = b.y; f.v[6] = b.z; f.v[7] = b.w;
    }
    return f;
}

// dW[o][i] += sum_n Y[o][n] X[i][n] for one 32x32 (mo, mi) tile; rows beyond
// (O, I) and the Cin columns without a weight are dropped. cin_map selects the
// layer-3 column remap (Cin row k -> color_net.0 column).
template <typename TM>
__device__ __forceinline__ void dw_tile(const TM *imgY, const TM *imgX, float *s_dw, int woff, int O, int I_torch,
                                        int obase, int ibase, bool cin_map, int lane, int ablate = 0) {
    if (ablate & 2) return;
    const int m = lane & 31, h = lane >> 5;
    f16v acc;
    acc_zero(acc);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        typename FragT<TM>::T a = img_get<TM>(imgY, m, 16 * s + 8 * h);
        typename FragT<TM>::T b = img_get<TM>(imgX, m, 16 * s + 8 * h);
        mma(acc, a, b);
    }
    const int i = ibase + m;
    int col = i;
    if (cin_map) col = (i >= 1 && i <= 15) ? 9 + i - 1 : ((i >= 16 && i <= 24) ? i - 16 : -1);
    if (col < 0 || col >= I_torch) return;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
        const int o = obase + acc_row(q, h);
        if (o < O && acc[q] != 0.f)
            __hip_atomic_fetch_add(&s_dw[woff + o * I_torch + col], acc[q], __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}
// bias gradient: row sums of the Y image (rows < O)
template <typename TM>
__device__ __forceinline__ void db_rows(const TM *imgY, float *s_dw, int boff, int O, int obase, int lane,
                                        int ablate = 0) {
    if (ablate & 2) return;
    if (lane < 32 && obase + lane < O) {
        float sum = 0.f;
#pragma unroll
        for (int c = 0; c < 32; c += 8) {
            typename FragT<TM>::T f = img_get<TM>(imgY, lane, c);
#pragma unroll
            for (int j = 0; j < 8; ++j) sum += frag_get<TM>(f, j);
        }
        if (sum != 0.f)
            __hip_atomic_fetch_add(&s_dw[boff + obase + lane], sum, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
}

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
    if (!walk) return z;
    // common.cu:40-105 walk (sequential subtraction; exact reference rounding)
    if (box[0] == 0.f) return 0.f;
    float rem = z;
    const float eps = 1e-4f;
    for (int i = 0;; ++i) {
        if (i >= a.Kmax) return rem <= eps ? box[(a.Kmax - 1) * 2 + 1] : 0.f;
        const float zin = box[i * 2], zout = box[i * 2 + 1];
        if (zin == 0.f) return (rem <= eps && i >= 1) ? box[(i - 1) * 2 + 1] : 0.f;
        const float len = zout - zin;
        if (rem <= len) return zin + rem;
        rem -= len;
    }
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

// Corner rows of one level for this lane's sample (kernel_grid index math).
template <typename TT>
__device__ __forceinline__ void gather_level(const FieldArgs &a, const LevelInfo &li, const float x01[3], float pos[3],
                                             float e[8][2]) {
    const TT *tab = reinterpret_cast<const TT *>(a.table);
    uint32_t pg[3];
#pragma unroll
    for (int d = 0; d < 3; ++d) {
        pos[d] = __builtin_fmaf(x01[d], li.scale, 0.5f);
        pg[d] = (uint32_t)floorf(pos[d]);
        pos[d] -= (float)pg[d];
    }
#pragma unroll
    for (int idx = 0; idx < 8; ++idx) {
        uint32_t pl[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) pl[d] = pg[d] + ((idx >> d) & 1);
        const uint32_t row = grid_row<3>(0, false, li.hs, li.res, pl);
        const TT *p = tab + ((size_t)li.off + row) * 2;
        if constexpr (sizeof(TT) == 4) {
            const float2 v = *reinterpret_cast<const float2 *>(p);
            e[idx][0] = v.x; e[idx][1] = v.y;
        } else {
            const __half2 v = *reinterpret_cast<const __half2 *>(p);
            e[idx][0] = __low2float(v); e[idx][1] = __high2float(v);
        }
    }
}

template <typename TT>
__device__ __forceinline__ void encode_level(const FieldArgs &a, int lv, const float x01[3], float f[2]) {
    const LevelInfo li = level_info(a, lv);
    float pos[3], e[8][2];
    gather_level<TT>(a, li, x01, pos, e);
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
template <int CTRL> __device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, true));
}
#define DPP_ROW_SHL(n) (0x100 + (n))
#define DPP_ROW_SHR(n) (0x110 + (n))

// Backward of one level (kernel_grid_backward + kernel_input_backward,
// gridencoder.cu:249-365) for this lane's sample: returns d<g, feature>/d x01
// from re-gathered corners (the reference's dy_dx, never materialised) and
// scatters w*g into the 8 corner rows.
//
// MI355X: device float atomics cost one memory-side request per active lane
// (~20 G lane-ops/s chip-wide, same-address lanes are NOT merged). Samples of a
// tile are consecutive along one ray, so equal cells form contiguous runs of
// lanes: a segmented suffix sum over each 16-lane DPP row (4 VALU steps, no
// LDS) folds every run into its first lane, and only run heads issue atomics —
// packed fp16x2 (one lane-op for both channels; the reference's amp __half2
// path) or 2 x fp32. MUST be called by all lanes of the wave (DPP).
template <typename TT, bool HALF_GRAD>
__device__ __forceinline__ void backward_level(const FieldArgs &a, int lv, bool active, const float x01[3], float g0,
                                               float g1, float gx[3], int lane) {
    const LevelInfo li = level_info(a, lv < (int)a.L ? lv : 0);
    float pos[3] = {0.f, 0.f, 0.f}, e[8][2];
    uint32_t pg[3] = {0u, 0u, 0u};
    if (active) {
        gather_level<TT>(a, li, x01, pos, e);
#pragma unroll
        for (int d = 0; d < 3; ++d) pg[d] = (uint32_t)floorf(__builtin_fmaf(x01[d], li.scale, 0.5f));
#pragma unroll
        for (int gd = 0; gd < 3; ++gd) {
            float r0 = 0.f, r1 = 0.f;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                float w = li.scale;
                int idx = 0, nd = 0;
#pragma unroll
                for (int d = 0; d < 3; ++d) {
                    if (d == gd) continue;
                    const int bit = (k >> nd) & 1;
                    w *= bit ? pos[d] : 1 - pos[d];
                    idx |= bit << d;
                    ++nd;
                }
                const int ir = idx | (1 << gd);
                r0 = __builtin_fmaf(w, e[ir][0] - e[idx][0], r0);
                r1 = __builtin_fmaf(w, e[ir][1] - e[idx][1], r1);
            }
            gx[gd] += g0 * r0 + g1 * r1;
        }
    }
    if (a.ablate & 1) return;
    // run keys: exact cell coordinates (10 bits each; res <= 1023); inactive lanes unique
    const int key = active ? (int)(1u + (pg[0] | (pg[1] << 10) | (pg[2] << 20))) : (0x40000000 + lane + 1);
    const bool s1 = dpp_i<DPP_ROW_SHL(1)>(key) == key, s2 = dpp_i<DPP_ROW_SHL(2)>(key) == key;
    const bool s4 = dpp_i<DPP_ROW_SHL(4)>(key) == key, s8 = dpp_i<DPP_ROW_SHL(8)>(key) == key;
    const bool head = active && (dpp_i<DPP_ROW_SHR(1)>(key) != key);
#pragma unroll
    for (int idx = 0; idx < 8; ++idx) {
        float w = 1.f;
        uint32_t pl[3];
#pragma unroll
        for (int d = 0; d < 3; ++d) {
            const int bit = (idx >> d) & 1;
            w *= bit ? pos[d] : 1 - pos[d];
            pl[d] = pg[d] + bit;
        }
        float v0 = active ? w * g0 : 0.f, v1 = active ? w * g1 : 0.f;
        // segmented suffix sum within the row (runs are contiguous)
        { const float t0 = dpp_f<DPP_ROW_SHL(1)>(v0), t1 = dpp_f<DPP_ROW_SHL(1)>(v1); if (s1) { v0 += t0; v1 += t1; } }
        { const float t0 = dpp_f<DPP_ROW_SHL(2)>(v0), t1 = dpp_f<DPP_ROW_SHL(2)>(v1); if (s2) { v0 += t0; v1 += t1; } }
        { const float t0 = dpp_f<DPP_ROW_SHL(4)>(v0), t1 = dpp_f<DPP_ROW_SHL(4)>(v1); if (s4) { v0 += t0; v1 += t1; } }
        { const float t0 = dpp_f<DPP_ROW_SHL(8)>(v0), t1 = dpp_f<DPP_ROW_SHL(8)>(v1); if (s8) { v0 += t0; v1 += t1; } }
        if (head) {
            const uint32_t row = grid_row<3>(0, false, li.hs, li.res, pl);
            const size_t o = ((size_t)li.off + row) * 2;
            if constexpr (HALF_GRAD) atomic_add_h2(a.grad_table16 + o, v0, v1);
            else { atomic_add_f32(a.grad_table + o, v0); atomic_add_f32(a.grad_table + o + 1, v1); }
        }
    }
}

__device__ __forceinline__ int lane_level(int s, int q, int h) { return 8 * s + 4 * (q >> 1) + 2 * h + (q & 1); }

// --------------------------------------------------------- MLP forward
template <typename TM> struct Acts {
    typename FragT<TM>::T X[2], H1[2][2], Cin[2], H3[2][2], H4[2][2];
};

template <typename TM>
__device__ __forceinline__ void mlp_forward(const FieldArgs &a, Acts<TM> &A, const float sh[9], int lane, float &sdf,
                                            float logit[3]) {
    const int h = lane >> 5;
    f16v acc[2];
    // L1: 32 -> 64, ReLU
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        acc_init_bias(acc[mt], a.bias + 0 * 64, mt, h);
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[mt], load_frag<TM>(a.frags, FR_L1 + mt * 2 + s, lane), A.X[s]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H1[t][s]);
    // L2: 64 -> 16 (sdf, geo[15])
    acc_init_bias(acc[0], a.bias + 1 * 64, 0, h);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[0], load_frag<TM>(a.frags, FR_L2 + 2 * t + s, lane), A.H1[t][s]);
    float sdf_v = acc[0][0];
    if constexpr (sizeof(TM) == 2) sdf_v = (float)(_Float16)sdf_v;   // fp16 Linear output under autocast
    sdf = __shfl(sdf_v, lane & 31, 64);                                 // row 0 lives in half 0
    // colour input: rows 0..15 = [sdf (zero weight), geo], rows 16..24 = SH
    acc_to_frag<TM>(acc[0], 0, false, A.Cin[0]);
    frag_zero<TM>(A.Cin[1]);
    if (h == 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j) frag_set<TM>(A.Cin[1], j, sh[j]);
        frag_set<TM>(A.Cin[1], 4, sh[8]);
    } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) frag_set<TM>(A.Cin[1], j, sh[4 + j]);
    }
    // L3: 24 -> 64, ReLU
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        acc_init_bias(acc[mt], a.bias + 2 * 64, mt, h);
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[mt], load_frag<TM>(a.frags, FR_L3 + mt * 2 + s, lane), A.Cin[s]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H3[t][s]);
    // L4: 64 -> 64, ReLU
#pragma unroll
    for (int mt = 0; mt < 2; ++mt) {
        acc_init_bias(acc[mt], a.bias + 3 * 64, mt, h);
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int s = 0; s < 2; ++s) mma(acc[mt], load_frag<TM>(a.frags, FR_L4 + mt * 4 + 2 * t + s, lane), A.H3[t][s]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) acc_to_frag<TM>(acc[t], s, true, A.H4[t][s]);
    // L5: 64 -> 3
    acc_init_bias(acc[0], a.bias + 4 * 64, 0, h);
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) mma(acc[0], load_frag<TM>(a.frags, FR_L5 + 2 * t + s, lane), A.H4[t][s]);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float v = acc[0][c];
        if constexpr (sizeof(TM) == 2) v = (float)(_Float16)v;
        logit[c] = __shfl(v, lane & 31, 64);
    }
}

// -------------------------------------------------------- field kernel
template <typename TM, typename TT, int WPB>
__global__ __launch_bounds__(WPB * 64) void k_field(FieldArgs a) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    float *s_dw = reinterpret_cast<float *>(smem);                         // [MLP_N] (padded to 9216)
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int n = lane & 31, h = lane >> 5;
    char *wbase = smem + 9216 * 4 + wave * (2 * Img<TM>::BYTES + 320 * 4);
    TM *imgY = reinterpret_cast<TM *>(wbase);
    TM *imgX = reinterpret_cast<TM *>(wbase + Img<TM>::BYTES);
    float *s_z = reinterpret_cast<float *>(wbase + 2 * Img<TM>::BYTES);    // [S <= 320]

    for (int i = threadIdx.x; i < 9216; i += blockDim.x) s_dw[i] = 0.f;
    __syncthreads();

    const float lscale = *a.loss_scale;
    const MlpOff mof(a.mlp_in);
    float loss_rgb = 0.f, loss_fs = 0.f, loss_empty = 0.f, loss_sdf = 0.f, n_valid = 0.f, n_bwd = 0.f;
    const int ntiles = a.S / 32;

    const int wave_u = __builtin_amdgcn_readfirstlane(wave);
    for (int r = blockIdx.x * WPB + wave_u; r < a.R; r += gridDim.x * WPB) {
        const float *ray = a.rays + (size_t)r * 12;
        const float dir[3] = {ray[0], ray[1], ray[2]};
        const float tgt[3] = {ray[3], ray[4], ray[5]};
        const float depth = ray[6];
        const int frame = (int)ray[8];
        const int rtype = (int)ray[9];
        const float *T = a.tf + (size_t)frame * 16;
        const float Rm[3][3] = {{T[0], T[1], T[2]}, {T[4], T[5], T[6]}, {T[8], T[9], T[10]}};
        const float tv[3] = {T[3], T[7], T[11]};
        const float nrm = sqrtf((dir[0] * dir[0] + dir[1] * dir[1]) + dir[2] * dir[2]);
        const float vd[3] = {dir[0] / nrm, dir[1] / nrm, dir[2] / nrm};
        const bool vdepth = (depth >= a.near_sc) && (depth <= a.far_sc);
        const float total = a.totals[r];
        const float *box = a.intervals + (size_t)r * a.Kmax * 2;
        // SH(degree 3) of the world view direction (run_network :1280-1285)
        const float idir[3] = {(Rm[0][0] * vd[0] + Rm[0][1] * vd[1]) + Rm[0][2] * vd[2],
                               (Rm[1][0] * vd[0] + Rm[1][1] * vd[1]) + Rm[1][2] * vd[2],
                               (Rm[2][0] * vd[0] + Rm[2][1] * vd[1]) + Rm[2][2] * vd[2]};
        float sh[9];
        {
            const float x = idir[0], y = idir[1], z = idir[2];
            const float xx = x * x, yy = y * y, zz = z * z;
            sh[0] = SH_C0; sh[1] = -SH_C1 * y; sh[2] = SH_C1 * z; sh[3] = -SH_C1 * x;
            sh[4] = SH_C2_0 * (x * y); sh[5] = SH_C2_1 * (y * z); sh[6] = SH_C2_2 * ((2.0f * zz - xx) - yy);
            sh[7] = SH_C2_3 * (x * z); sh[8] = SH_C2_4 * (xx - yy);
        }

        // ------------------------------------------------------ pass A
        float wsum = 0.f, racc[3] = {0.f, 0.f, 0.f};
        bool anyv = false;
        for (int t = 0; t < ntiles; ++t) {
            const int s = 32 * t + n;
            const float z = sample_z(a, r, s, depth, vdepth, total, box);
            if (h == 0) s_z[s] = z;
            const float w = bell_weight(a, depth, z);
            const float p[3] = {dir[0] * z, dir[1] * z, dir[2] * z};
            float x[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) x[i] = ((Rm[i][0] * p[0] + Rm[i][1] * p[1]) + Rm[i][2] * p[2]) + tv[i];
            const bool valid = fabsf(x[0]) <= 1.f && fabsf(x[1]) <= 1.f && fabsf(x[2]) <= 1.f;
            if (h == 0) { wsum += w; n_valid += valid ? 1.f : 0.f; }
            anyv |= valid;
            if (a.dbg_z && h == 0) a.dbg_z[(size_t)r * a.S + s] = z;
            if (a.dbg_valid && h == 0) a.dbg_valid[(size_t)r * a.S + s] = valid;
            const bool need = __any((w > 0.f && valid) || (a.dbg_raw != nullptr)) && !(a.ablate & 16);
            if (!need) continue;
            Acts<TM> A;
            const float x01[3] = {(x[0] + 1) / 2, (x[1] + 1) / 2, (x[2] + 1) / 2};
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int lv = lane_level(ss, q, h);
                    float f[2] = {0.f, 0.f};
                    if (valid && lv < (int)a.L) encode_level<TT>(a, lv, x01, f);
                    frag_set<TM>(A.X[ss], 2 * q, f[0]);
                    frag_set<TM>(A.X[ss], 2 * q + 1, f[1]);
                    if (q & 1) __builtin_amdgcn_sched_barrier(0);   // bound gathers in flight (2 levels)
                }
            }
            float sdf, logit[3];
            mlp_forward<TM>(a, A, sh, lane, sdf, logit);
            if (h == 0 && valid && w > 0.f) {
#pragma unroll
                for (int c = 0; c < 3; ++c) racc[c] += w * sigmoidf(logit[c]);
            }
            if (a.dbg_raw && h == 0) {
                float *o = a.dbg_raw + ((size_t)r * a.S + s) * 4;
                o[0] = logit[0]; o[1] = logit[1]; o[2] = logit[2]; o[3] = sdf;
            }
        }
        const float wtot = wave_sum(wsum);
        float rgb[3];
#pragma unroll
        for (int c = 0; c < 3; ++c) rgb[c] = wave_sum(racc[c]) / (wtot + 1e-10f);
        const bool vray = __any(anyv) && rtype == 0;
        const float rw = vray ? (frame == 0 ? a.ffw : 1.f) : 0.f;
        float drgb[3];
        float lr = 0.f;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            const float e = rgb[c] - tgt[c];
            drgb[c] = a.rgb_w * 2.f * e * rw * a.inv_3R;
            lr += e * e * rw;
        }
        if (lane == 0) loss_rgb += a.rgb_w * lr * a.inv_3R;
        if (a.dbg_rgb && lane == 0) {
            a.dbg_rgb[r * 3] = rgb[0]; a.dbg_rgb[r * 3 + 1] = rgb[1]; a.dbg_rgb[r * 3 + 2] = rgb[2];
        }
        if (rw == 0.f) {          // no loss term of this ray has a non-zero weight
            if (lane < 12) a.ray_grad[(size_t)r * 12 + lane] = 0.f;
            continue;
        }

        // ------------------------------------------------------ pass B
        float gtf[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) gtf[k] = 0.f;
        float dsh[5] = {0.f, 0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < ntiles; ++t) {
            const int s = 32 * t + n;
            const float z = s_z[s];
            const float p[3] = {dir[0] * z, dir[1] * z, dir[2] * z};
            float x[3];
#pragma unroll
            for (int i = 0; i < 3; ++i) x[i] = ((Rm[i][0] * p[0] + Rm[i][1] * p[1]) + Rm[i][2] * p[2]) + tv[i];
            const bool valid = fabsf(x[0]) <= 1.f && fabsf(x[1]) <= 1.f && fabsf(x[2]) <= 1.f;
            if (!__any(valid)) continue;
            const float x01[3] = {(x[0] + 1) / 2, (x[1] + 1) / 2, (x[2] + 1) / 2};
            Acts<TM> A;
#pragma unroll
            for (int ss = 0; ss < 2; ++ss) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const int lv = lane_level(ss, q, h);
                    float f[2] = {0.f, 0.f};
                    if (valid && lv < (int)a.L && !(a.ablate & 8)) encode_level<TT>(a, lv, x01, f);
                    frag_set<TM>(A.X[ss], 2 * q, f[0]);
                    frag_set<TM>(A.X[ss], 2 * q + 1, f[1]);
                    if (q & 1) __builtin_amdgcn_sched_barrier(0);   // bound gathers in flight (2 levels)
                }
            }
            float sdf, logit[3];
            mlp_forward<TM>(a, A, sh, lane, sdf, logit);
            // ---- loss gradient for this sample (train_loop :687-751, get_sdf_loss)
            const float sw = valid ? rw : 0.f;
            const float w = bell_weight(a, depth, z);
            const float wn = valid ? w / (wtot + 1e-10f) : 0.f;
            float dlogit[3];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float sg = sigmoidf(logit[c]);
                dlogit[c] = drgb[c] * wn * sg * (1.f - sg);
            }
            const bool front = z < depth - a.trunc;
            const bool back = z > depth + a.trunc * a.ntr;
            const float sdfm = (!front && !back && vdepth) ? 1.f : 0.f;
            const bool fsm = (depth > a.far_sc) && (sdf < a.fs_sdf);
            const bool em = front && (depth <= a.far_sc) && (sdf < 1.f);
            const float efs = fsm ? (sdf - a.fs_sdf) : 0.f;
            const float esdf = (z + sdf * a.trunc) * sdfm - depth * sdfm;
            float dsdf = a.fs_w * 0.5f * 2.f * efs * sw * a.inv_RS;
            dsdf += em ? a.fs_w * a.empty_w * (sdf > 1.f ? 1.f : (sdf < 1.f ? -1.f : 0.f)) * sw * a.inv_RS : 0.f;
            dsdf += a.trunc_w * 0.5f * 2.f * esdf * sdfm * a.trunc * sw * a.inv_RS;
            if (h == 0) {
                loss_fs += a.fs_w * 0.5f * efs * efs * sw * a.inv_RS;
                loss_empty += em ? a.fs_w * a.empty_w * fabsf(sdf - 1.f) * sw * a.inv_RS : 0.f;
                loss_sdf += a.trunc_w * 0.5f * esdf * esdf * sw * a.inv_RS;
            }
            const bool nz = (dsdf != 0.f) || (dlogit[0] != 0.f) || (dlogit[1] != 0.f) || (dlogit[2] != 0.f);
            if (!__any(nz)) continue;
            if (h == 0) n_bwd += valid ? 1.f : 0.f;
            if (a.ablate & 4) continue;
            dsdf *= lscale;
#pragma unroll
            for (int c = 0; c < 3; ++c) dlogit[c] *= lscale;

            // ---- MLP backward (activations in A; weight grads via LDS)
            typename FragT<TM>::T dO, fb[2][2];
            frag_zero<TM>(dO);
            if (h == 0) {
#pragma unroll
                for (int c = 0; c < 3; ++c) frag_set<TM>(dO, c, dlogit[c]);
            }
            f16v acc[2];
            // dW5 / db5 : Y = dlogit rows 0..2 (natural order), X = H4
            {
#pragma unroll
                for (int j = 0; j < 8; ++j)   // natural-order fragment: row 8h + j
                    imgY[(8 * h + j) * Img<TM>::STRIDE + n] = (TM)frag_get<TM>(dO, j);
#pragma unroll
                for (int j = 0; j < 8; ++j) imgY[(16 + 8 * h + j) * Img<TM>::STRIDE + n] = (TM)0.f;
                db_rows<TM>(imgY, s_dw, mof.b5, 3, 0, lane, a.ablate);
#pragma unroll
                for (int mi = 0; mi < 2; ++mi) {
                    img_put_frag<TM>(imgX, A.H4[mi][0], 0, h, n);
                    img_put_frag<TM>(imgX, A.H4[mi][1], 1, h, n);
                    dw_tile<TM>(imgY, imgX, s_dw, mof.w5, 3, 64, 0, 32 * mi, false, lane, a.ablate);
                }
            }
            // B5: dH4 = W5^T dO, ReLU mask
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_zero(acc[mt]);
                mma(acc[mt], load_frag<TM>(a.frags, FR_B5 + mt, lane), dO);
            }
            typename FragT<TM>::T dH[2][2];
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        frag_set<TM>(dH[t2][s2], j, frag_get<TM>(A.H4[t2][s2], j) > 0 ? acc[t2][8 * s2 + j] : 0.f);
            // dW4 / db4 : Y = dH4, X = H3
#pragma unroll
            for (int mo = 0; mo < 2; ++mo) {
                img_put_frag<TM>(imgY, dH[mo][0], 0, h, n);
                img_put_frag<TM>(imgY, dH[mo][1], 1, h, n);
                db_rows<TM>(imgY, s_dw, mof.b4, 64, 32 * mo, lane, a.ablate);
#pragma unroll
                for (int mi = 0; mi < 2; ++mi) {
                    img_put_frag<TM>(imgX, A.H3[mi][0], 0, h, n);
                    img_put_frag<TM>(imgX, A.H3[mi][1], 1, h, n);
                    dw_tile<TM>(imgY, imgX, s_dw, mof.w4, 64, 64, 32 * mo, 32 * mi, false, lane, a.ablate);
                }
            }
            // B4: dH3 = W4^T dH4, ReLU mask
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_zero(acc[mt]);
#pragma unroll
                for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2)
                        mma(acc[mt], load_frag<TM>(a.frags, FR_B4 + mt * 4 + 2 * t2 + s2, lane), dH[t2][s2]);
            }
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        frag_set<TM>(dH[t2][s2], j, frag_get<TM>(A.H3[t2][s2], j) > 0 ? acc[t2][8 * s2 + j] : 0.f);
            // dW3 / db3 : Y = dH3, X = Cin (remapped columns)
            img_put_frag<TM>(imgX, A.Cin[0], 0, h, n);
            img_put_frag<TM>(imgX, A.Cin[1], 1, h, n);
#pragma unroll
            for (int mo = 0; mo < 2; ++mo) {
                img_put_frag<TM>(imgY, dH[mo][0], 0, h, n);
                img_put_frag<TM>(imgY, dH[mo][1], 1, h, n);
                db_rows<TM>(imgY, s_dw, mof.b3, 64, 32 * mo, lane, a.ablate);
                dw_tile<TM>(imgY, imgX, s_dw, mof.w3, 64, 24, 32 * mo, 0, true, lane, a.ablate);
            }
            // B3: dCin = W3'^T dH3  (rows 1..15 = dgeo, 16..24 = dSH)
            acc_zero(acc[0]);
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) mma(acc[0], load_frag<TM>(a.frags, FR_B3 + 2 * t2 + s2, lane), dH[t2][s2]);
            // dSH rows: h0 regs 8..11 -> SH0..3, reg 12 -> SH8; h1 regs 8..11 -> SH4..7
#pragma unroll
            for (int j = 0; j < 5; ++j) dsh[j] += acc[0][8 + j];
            // dH2 = [dsdf, dgeo] in rows 0..15
            typename FragT<TM>::T dH2[2];
            acc_to_frag<TM>(acc[0], 0, false, dH2[0]);
            if (h == 0) frag_set<TM>(dH2[0], 0, dsdf);
            frag_zero<TM>(dH2[1]);
            // dW2 / db2 : Y = dH2 (16 rows), X = H1
            img_put_frag<TM>(imgY, dH2[0], 0, h, n);
            img_put_frag<TM>(imgY, dH2[1], 1, h, n);
            db_rows<TM>(imgY, s_dw, mof.b2, 16, 0, lane, a.ablate);
#pragma unroll
            for (int mi = 0; mi < 2; ++mi) {
                img_put_frag<TM>(imgX, A.H1[mi][0], 0, h, n);
                img_put_frag<TM>(imgX, A.H1[mi][1], 1, h, n);
                dw_tile<TM>(imgY, imgX, s_dw, mof.w2, 16, 64, 0, 32 * mi, false, lane, a.ablate);
            }
            // B2: dH1 = W2^T dH2, ReLU mask
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                acc_zero(acc[mt]);
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) mma(acc[mt], load_frag<TM>(a.frags, FR_B2 + mt * 2 + s2, lane), dH2[s2]);
            }
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
                    for (int j = 0; j < 8; ++j)
                        frag_set<TM>(dH[t2][s2], j, frag_get<TM>(A.H1[t2][s2], j) > 0 ? acc[t2][8 * s2 + j] : 0.f);
            // dW1 / db1 : Y = dH1, X = encoded features
            img_put_frag<TM>(imgX, A.X[0], 0, h, n);
            img_put_frag<TM>(imgX, A.X[1], 1, h, n);
#pragma unroll
            for (int mo = 0; mo < 2; ++mo) {
                img_put_frag<TM>(imgY, dH[mo][0], 0, h, n);
                img_put_frag<TM>(imgY, dH[mo][1], 1, h, n);
                db_rows<TM>(imgY, s_dw, mof.b1, 64, 32 * mo, lane, a.ablate);
                dw_tile<TM>(imgY, imgX, s_dw, mof.w1, 64, a.mlp_in, 32 * mo, 0, false, lane, a.ablate);
            }
            // B1: dX = W1^T dH1 -> per-level feature gradients (this lane's levels)
            acc_zero(acc[0]);
#pragma unroll
            for (int t2 = 0; t2 < 2; ++t2)
#pragma unroll
                for (int s2 = 0; s2 < 2; ++s2) mma(acc[0], load_frag<TM>(a.frags, FR_B1 + 2 * t2 + s2, lane), dH[t2][s2]);

            // ---- table scatter + input gradient
            float gx[3] = {0.f, 0.f, 0.f};
            if (!(a.ablate & 32)) {
#pragma unroll
                for (int ss = 0; ss < 2; ++ss)
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        const int lv = lane_level(ss, q, h);
                        const float g0 = acc[0][8 * ss + 2 * q], g1 = acc[0][8 * ss + 2 * q + 1];
                        const bool act = valid && lv < (int)a.L && (g0 != 0.f || g1 != 0.f);
                        backward_level<TT, (sizeof(TM) == 2)>(a, lv, act, x01, g0, g1, gx, lane);
                        __builtin_amdgcn_sched_barrier(0);
                    }
            }
            // dL/dx_world = 0.5 dL/dx01 (grid.py:160), both halves' levels
#pragma unroll
            for (int d = 0; d < 3; ++d) {
                gx[d] *= 0.5f;
                gx[d] += __shfl_xor(gx[d], 32, 64);
            }
            if (h == 0) {
#pragma unroll
                for (int i = 0; i < 3; ++i) {
#pragma unroll
                    for (int j = 0; j < 3; ++j) gtf[i * 4 + j] += gx[i] * p[j];
                    gtf[i * 4 + 3] += gx[i];
                }
            }
        }
        // ---- per-ray pose gradient: transform_pts + SH(view) paths
        float gsh[9];
        {
            const float d0 = wave_sum(h == 0 ? dsh[0] : 0.f), d1 = wave_sum(h == 0 ? dsh[1] : 0.f);
            const float d2 = wave_sum(h == 0 ? dsh[2] : 0.f), d3 = wave_sum(h == 0 ? dsh[3] : 0.f);
            const float d8 = wave_sum(h == 0 ? dsh[4] : 0.f);
            const float d4 = wave_sum(h == 1 ? dsh[0] : 0.f), d5 = wave_sum(h == 1 ? dsh[1] : 0.f);
            const float d6 = wave_sum(h == 1 ? dsh[2] : 0.f), d7 = wave_sum(h == 1 ? dsh[3] : 0.f);
            gsh[0] = d0; gsh[1] = d1; gsh[2] = d2; gsh[3] = d3; gsh[4] = d4; gsh[5] = d5; gsh[6] = d6; gsh[7] = d7;
            gsh[8] = d8;
        }
        const float x = idir[0], y = idir[1], zz = idir[2];
        const float gdir[3] = {
            -SH_C1 * gsh[3] + SH_C2_0 * y * gsh[4] + SH_C2_2 * (-2.f * x) * gsh[6] + SH_C2_3 * zz * gsh[7] +
                SH_C2_4 * 2.f * x * gsh[8],
            -SH_C1 * gsh[1] + SH_C2_0 * x * gsh[4] + SH_C2_1 * zz * gsh[5] + SH_C2_2 * (-2.f * y) * gsh[6] -
                SH_C2_4 * 2.f * y * gsh[8],
            SH_C1 * gsh[2] + SH_C2_1 * y * gsh[5] + SH_C2_2 * 4.f * zz * gsh[6] + SH_C2_3 * x * gsh[7]};
        float out = 0.f;
#pragma unroll
        for (int k = 0; k < 12; ++k) {
            float v = wave_sum(gtf[k]);
            const int i = k >> 2, j = k & 3;
            if (j < 3) v += gdir[i] * vd[j];
            if (lane == k) out = v;
        }
        if (lane < 12) a.ray_grad[(size_t)r * 12 + lane] = out;
    }

    // flush: losses and the block's MLP-gradient accumulator
    loss_rgb = wave_sum(loss_rgb);
    loss_fs = wave_sum(loss_fs);
    loss_empty = wave_sum(loss_empty);
    loss_sdf = wave_sum(loss_sdf);
    n_valid = wave_sum(n_valid);
    n_bwd = wave_sum(n_bwd);
    if (lane == 0) {
        atomic_add_f32(a.loss_acc + 4, n_valid);
        atomic_add_f32(a.loss_acc + 5, n_bwd);
        atomic_add_f32(a.loss_acc + 0, loss_rgb);
        atomic_add_f32(a.loss_acc + 1, loss_fs);
        atomic_add_f32(a.loss_acc + 2, loss_empty);
        atomic_add_f32(a.loss_acc + 3, loss_sdf);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < mof.n; i += blockDim.x)
        if (s_dw[i] != 0.f) atomic_add_f32(a.grad_mlp + i, s_dw[i]);
}

// ---------------------------------------------------- ray setup + trace
__global__ __launch_bounds__(256) void k_trace(const float *__restrict__ pool, const int32_t *__restrict__ ids, int R,
                                               const float *__restrict__ tf, const uint8_t *__restrict__ occ, int N,
                                               int Kmax, float near_sc, float far_sc, float trunc,
                                               float *__restrict__ rays_out, float *__restrict__ intervals,
                                               float *__restrict__ totals, int32_t *__restrict__ counts) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= R) return;
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
    const int k = trace_ray(occ, N, o, d, Kmax, dst);
    // depths_in_out -> z (sample_rays_uniform_occupied_voxels :986-998; note the second normalisation)
    const float n2 = sqrtf((vd[0] * vd[0] + vd[1] * vd[1]) + vd[2] * vd[2]);
    const float vz = fabsf(vd[2] / n2);
    const float depth = ray[6];
    const bool vdepth = (depth >= near_sc) && (depth <= far_sc);
    const float hi = depth + trunc;
    float total = 0.f;
    for (int j = 0; j < k; ++j) {
        float zi = dst[j * 2] * vz, zo = dst[j * 2 + 1] * vz;
        if (vdepth && zi > 0.f && zo > 0.f) {
            zi = fminf(fmaxf(zi, 0.f), hi);
            zo = fminf(fmaxf(zo, 0.f), hi);
        }
        dst[j * 2] = zi;
        dst[j * 2 + 1] = zo;
        total += zo - zi;
    }
    for (int j = k; j < Kmax; ++j) { dst[j * 2] = 0.f; dst[j * 2 + 1] = 0.f; }
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
// Throughput-mode ray selection: rays_per_frame uniform draws inside each
// frame's contiguous pool segment (frame_start [F+1]).
__global__ __launch_bounds__(256) void k_sample_batch(const int64_t *__restrict__ frame_start, int F,
                                                      int rays_per_frame, uint32_t seed, int32_t *__restrict__ ids) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= F * rays_per_frame) return;
    const int f = i / rays_per_frame;
    const int64_t lo = frame_start[f], cnt = frame_start[f + 1] - lo;
    const uint32_t u = hash32(seed ^ hash32((uint32_t)i * 0x85EBCA6BU + 0x27D4EB2FU));
    ids[i] = (int32_t)(lo + (int64_t)(((uint64_t)u * (uint64_t)cnt) >> 32));
}

}  // namespace nof

extern "C" int nof_trace_rays(const float *pool, const int32_t *ids, int32_t R, const float *tf, const uint8_t *occ,
                              int32_t N, int32_t Kmax, float near_sc, float far_sc, float trunc, float *rays_out,
                              float *intervals, float *totals, int32_t *counts, void *stream) {
    if (R <= 0) return NOF_OK;
    if (N <= 0 || Kmax <= 0) return nof::set_error(NOF_EINVAL, "trace_rays: bad N=%d Kmax=%d", N, Kmax);
    hipLaunchKernelGGL(nof::k_trace, dim3(nof::div_up(R, 256)), dim3(256), 0, (hipStream_t)stream, pool, ids, R, tf,
                       occ, N, Kmax, near_sc, far_sc, trunc, rays_out, intervals, totals, counts);
    return nof::check_launch("trace_rays");
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
                                int32_t *ids, void *stream) {
    const int n = F * rays_per_frame;
    if (n <= 0) return NOF_OK;
    hipLaunchKernelGGL(nof::k_sample_batch, dim3(nof::div_up(n, 256)), dim3(256), 0, (hipStream_t)stream, frame_start,
                       F, rays_per_frame, seed, ids);
    return nof::check_launch("sample_batch");
}

namespace {
template <typename TM, typename TT, int WPB>
int launch_field(const nof::FieldArgs &a, int n_blocks, hipStream_t st) {
    const size_t lds = 9216 * 4 + (size_t)WPB * (2 * nof::Img<TM>::BYTES + 320 * 4);
    hipLaunchKernelGGL((nof::k_field<TM, TT, WPB>), dim3(n_blocks), dim3(WPB * 64), lds, st, a);
    return nof::check_launch("field_step");
}
}  // namespace

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
    a.loss_scale = d->loss_scale; a.table = d->table; a.levels = (const float4 *)d->levels; a.L = d->L;
    a.mlp_in = (int)(d->L * d->C);
    a.frags = d->frags; a.bias = d->bias; a.grad_table = d->grad_table; a.grad_mlp = d->grad_mlp;
    a.grad_table16 = (__half *)d->grad_table16;
    if (d->mlp_dtype == NOF_F16 && !d->grad_table16)
        return nof::set_error(NOF_EINVAL, "field_step: amp mode needs grad_table16 (fp16 table gradient)");
    a.ray_grad = d->ray_grad; a.loss_acc = d->loss_acc; a.dbg_z = d->dbg_z; a.dbg_raw = d->dbg_raw;
    a.dbg_valid = d->dbg_valid; a.dbg_rgb = d->dbg_rgb; a.ablate = d->ablate;
    hipStream_t st = (hipStream_t)stream;
    int dev = 0, n_cu = 256;
    if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, dev);
    if (d->mlp_dtype == NOF_F16 && d->table_dtype == NOF_F16) {
        constexpr int WPB = 4;
        const int nb = (int)std::min<int64_t>((d->R + WPB - 1) / WPB, (int64_t)n_cu * d->blocks_per_cu);
        return launch_field<_Float16, __half, WPB>(a, nb, st);
    }
    if (d->mlp_dtype == NOF_F32 && d->table_dtype == NOF_F32) {
        constexpr int WPB = 4;
        const int nb = (int)std::min<int64_t>((d->R + WPB - 1) / WPB, (int64_t)n_cu * d->blocks_per_cu);
        return launch_field<float, float, WPB>(a, nb, st);
    }
    return nof::set_error(NOF_EINVAL, "field_step: mlp/table dtype must both be f16 (amp) or both f32");
}
