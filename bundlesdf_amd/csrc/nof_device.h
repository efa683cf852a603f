// Shared device helpers for the NOF HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>

#include "../../include/nof.h"

#define NOF_WAVE 64

namespace nof {

// Host-side error plumbing (defined in nof_runtime.cpp).
int set_error(int code, const char *fmt, ...);
int check_launch(const char *what);

// Per-level float32 scale / resolution (host-computed, bit-identical to the
// reference's in-kernel float32 math, gridencoder.cu:155-156).
struct LevelParams {
    float scale[NOF_MAX_LEVELS];
    uint32_t res[NOF_MAX_LEVELS];
};
void level_params(uint32_t L, float S, uint32_t H, LevelParams &lp);

// --- hashing / indexing (semantics of gridencoder.cu:46-83) ---------------
template <uint32_t D>
__device__ __forceinline__ uint32_t fast_hash(const uint32_t (&p)[D]) {
    constexpr uint32_t primes[7] = {1u, 2654435761u, 805459861u, 3674653429u,
                                    2097192037u, 1434869437u, 2165219737u};
    uint32_t r = 0;
#pragma unroll
    for (uint32_t i = 0; i < D; ++i) r ^= p[i] * primes[i];
    return r;
}

// Row index (not yet multiplied by C) of grid point p in a level table of
// `hashmap_size` rows. Equivalent to get_grid_index(): the modulo is a no-op
// whenever the dense stride fits, so it is only evaluated otherwise.
template <uint32_t D>
__device__ __forceinline__ uint32_t grid_row(uint32_t gridtype, bool align_corners, uint32_t hashmap_size,
                                             uint32_t resolution, const uint32_t (&p)[D]) {
    uint32_t stride = 1, index = 0;
    const uint32_t rs = align_corners ? resolution : resolution + 1;
#pragma unroll
    for (uint32_t d = 0; d < D; d++) {
        if (stride <= hashmap_size) {
            index += p[d] * stride;
            stride *= rs;
        }
    }
    if (stride > hashmap_size) {
        if (gridtype == 0) index = fast_hash<D>(p);
        index %= hashmap_size;
    }
    return index;
}

__device__ __forceinline__ float h2f(__half h) { return __half2float(h); }
__device__ __forceinline__ __half f2h(float f) { return __float2half_rn(f); }
__device__ __forceinline__ float hround(float f) { return __half2float(__float2half_rn(f)); }

template <typename T> struct Scalar;
template <> struct Scalar<float> {
    __device__ static float load(const float *p) { return *p; }
    __device__ static void store(float *p, float v) { *p = v; }
};
template <> struct Scalar<__half> {
    __device__ static float load(const __half *p) { return __half2float(*p); }
    __device__ static void store(__half *p, float v) { *p = __float2half_rn(v); }
};

// No-return packed-f16 global atomic add (global_atomic_pk_add_f16).
__device__ __forceinline__ void atomic_add_h2(__half *addr, float a, float b) {
    typedef _Float16 __attribute__((ext_vector_type(2))) h2v;
    h2v v = {(_Float16)__float2half_rn(a), (_Float16)__float2half_rn(b)};
    __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2v *)addr, v);
}
__device__ __forceinline__ void atomic_add_f32(float *addr, float v) {
    __hip_atomic_fetch_add(addr, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

inline uint32_t div_up(uint64_t a, uint64_t b) { return (uint32_t)((a + b - 1) / b); }

}  // namespace nof
