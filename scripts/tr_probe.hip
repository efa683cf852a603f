// Layout probe for k_mlp_bwd's LDS transposes (ds_read_b64_tr_b16): a normal activation
// fragment (lane = sample n + 32 h, element j = unit 16 s + 8 (j >> 2) + 4 h + (j & 3) of a
// 32-unit block) written with the swizzled image of field_step.hip (img_write) must read back
// (img_read_tr) as the K = samples operand: lane = unit (lane & 31), element j = sample
// 16 ks + 8 h + j. Asymmetric exact data (value = 64 unit + sample, fp16-exact). Prints the
// mismatch count. Build: hipcc --offload-arch=gfx950 -O3 scripts/tr_probe.hip -o scripts/tr_probe.bin
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../bundlesdf_amd/csrc/mlp_lds.h"

__global__ void k_probe(int *bad) {
    __shared__ __attribute__((aligned(16))) char img[nof::IMG_BYTES];
    const int lane = threadIdx.x, n = lane & 31, h = lane >> 5;
    nof::h8v f[2];
    for (int s = 0; s < 2; ++s)
        for (int j = 0; j < 8; ++j) {
            const int u = 16 * s + 8 * (j >> 2) + 4 * h + (j & 3);
            f[s][j] = (_Float16)(64 * u + n);
        }
    nof::img_write(img, f, lane);
    __syncthreads();
    int nb = 0;
    for (int ks = 0; ks < 2; ++ks) {
        const nof::h8v t = nof::img_read_tr(img, ks, lane);
        for (int j = 0; j < 8; ++j) {
            const int u = lane & 31, smp = 16 * ks + 8 * h + j;
            if ((float)t[j] != (float)(64 * u + smp)) ++nb;
        }
    }
    atomicAdd(bad, nb);
}

int main() {
    int *d, hbad = -1;
    (void)hipMalloc(&d, 4);
    (void)hipMemset(d, 0, 4);
    hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, d);
    (void)hipMemcpy(&hbad, d, 4, hipMemcpyDeviceToHost);
    printf("{\"tr_probe_mismatches\": %d}\n", hbad);
    return hbad != 0;
}
