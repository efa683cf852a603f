// LDS transposes of MFMA activation fragments for k_mlp_bwd (gfx950 ds_read_b64_tr_b16).
//
// A 32x32x16 f16 MFMA operand fragment in the "normal" layout of the MLP chain holds, in lane
// n + 32 h (n = sample of the tile), element j of K step s = unit 16 s + 8 (j >> 2) + 4 h +
// (j & 3) of a 32-unit block (the accumulator row order, field_step.hip acc_row). The weight
// gradients need the same values with the samples as K: lane = unit, element j = sample
// 16 ks + 8 h + j. Instead of recomputing every activation / gradient a second time with the
// MFMA operands swapped (and converting it again), the normal fragment is written once into
// a per-wave LDS image [32 samples][32 units] and read back transposed by ds_read_b64_tr_b16,
// which delivers, per group of 16 lanes, a 4-row x 16-column block column-major
// (cdna_hip_programming.md T10).
//
// Image: 64-B rows (one sample), 8 chunks of 4 units; chunk c of row n lives in slot
// c ^ ((n >> 1) & 7). The writes (two 8-B chunks per lane and K step) are 2-way (the minimum
// for 64 dwords on 32 banks); the transposed reads are conflict-free: a 32-lane half reads
// rows r0 .. r0 + 3 x both 16-unit groups, i.e. 4 rows x 8 slots = all 64 banks, whatever the
// XOR. The read needs the whole wave active (EXEC all ones: the gather crosses lanes).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace nof {

typedef _Float16 h8v __attribute__((ext_vector_type(8)));
typedef short s4v __attribute__((ext_vector_type(4)));
typedef _Float16 h4v __attribute__((ext_vector_type(4)));
typedef uint32_t u4v __attribute__((ext_vector_type(4)));
constexpr int IMG_BYTES = 32 * 64;   // one [32 samples][32 units] fp16 block

__device__ __forceinline__ uint32_t img_off(int n, int c) { return (uint32_t)(n * 64 + ((c ^ ((n >> 1) & 7)) << 3)); }

// the two normal K-step fragments f[0], f[1] of one 32-unit block -> image
__device__ __forceinline__ void img_write(char *img, const h8v (&f)[2], int lane) {
    const int n = lane & 31, h = lane >> 5;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
        const u4v w = __builtin_bit_cast(u4v, f[s]);   // elements 0..3: units 16s + 4h + 0..3; 4..7: + 8
        *reinterpret_cast<uint2 *>(img + img_off(n, 4 * s + h)) = make_uint2(w.x, w.y);
        *reinterpret_cast<uint2 *>(img + img_off(n, 4 * s + 2 + h)) = make_uint2(w.z, w.w);
    }
}
// one normal fragment (K step s only: 16 units) -> image (the other half of the block untouched)
__device__ __forceinline__ void img_write1(char *img, const h8v &f, int s, int lane) {
    const int n = lane & 31, h = lane >> 5;
    const u4v w = __builtin_bit_cast(u4v, f);
    *reinterpret_cast<uint2 *>(img + img_off(n, 4 * s + h)) = make_uint2(w.x, w.y);
    *reinterpret_cast<uint2 *>(img + img_off(n, 4 * s + 2 + h)) = make_uint2(w.z, w.w);
}

__device__ __forceinline__ s4v tr16(const char *p) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s4v *)(const_cast<char *>(p)));
}

// K = samples operand of K step ks (samples 16 ks .. 16 ks + 15): lane = unit (lane & 31),
// element j = sample 16 ks + 8 h + j
__device__ __forceinline__ h8v img_read_tr(const char *img, int ks, int lane) {
    const int g = (lane >> 4) & 1, h = lane >> 5, q = (lane >> 2) & 3, p = lane & 3;
    const int r0 = 16 * ks + 8 * h + q;
    const h4v a = __builtin_bit_cast(h4v, tr16(img + img_off(r0, 4 * g + p)));
    const h4v b = __builtin_bit_cast(h4v, tr16(img + img_off(r0 + 4, 4 * g + p)));
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

// K = samples operand of a 16x16x32 MFMA over the tile's 32 samples: lane = unit 16 half + (lane & 15)
// of the image's 32, element j = sample 8 (lane >> 4) + j. Conflict-free as img_read_tr: a 32-lane
// half reads rows q and 8 + q (q < 4), whose XOR slots fall in opposite 4-slot quads
__device__ __forceinline__ h8v img_read_tr_k32(const char *img, int half, int lane) {
    const int G = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const int r0 = 8 * G + q;
    const h4v a = __builtin_bit_cast(h4v, tr16(img + img_off(r0, 4 * half + p)));
    const h4v b = __builtin_bit_cast(h4v, tr16(img + img_off(r0 + 4, 4 * half + p)));
    return __builtin_shufflevector(a, b, 0, 1, 2, 3, 4, 5, 6, 7);
}

}  // namespace nof
