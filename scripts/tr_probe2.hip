// Raw semantics probe of ds_read_b64_tr_b16: LDS holds M[row][col] = 64 row + col (16-bit,
// 32 rows x 64 cols, 128-B rows, no swizzle); lane l supplies the address of
// M[l >> 2 & 3 (+ 4 * (l >> 4))][4 (l & 3)] and the 4 returned elements are dumped.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef short s4v __attribute__((ext_vector_type(4)));
__global__ void k(short *out) {
    __shared__ __attribute__((aligned(16))) short img[32 * 64];
    for (int i = threadIdx.x; i < 32 * 64; i += 64) img[i] = (short)i;
    __syncthreads();
    const int l = threadIdx.x;
    const int row = ((l >> 2) & 3) + 4 * (l >> 4), col = 4 * (l & 3);
    const s4v v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s4v *)(img + row * 64 + col));
    for (int e = 0; e < 4; ++e) out[l * 4 + e] = v[e];
}
int main() {
    short *d, h[256];
    (void)hipMalloc(&d, 512);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(h, d, 512, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; ++l) {
        printf("lane %2d:", l);
        for (int e = 0; e < 4; ++e) printf(" (r%d,c%d)", h[l * 4 + e] / 64, h[l * 4 + e] % 64);
        printf("\n");
    }
    return 0;
}
