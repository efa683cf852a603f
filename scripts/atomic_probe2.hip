// Diagnostic microbenchmark (not part of libnof): packed fp16x2 atomic
// throughput on MI355X vs the address pattern of one wave instruction.
//   pattern 0: 64 random rows per instruction (the unsorted scatter flush)
//   pattern 1: 64 consecutive rows (one 256-B span) per instruction
//   pattern 2: 64 rows spread over 8 random 8-row clusters (sorted flush of a ray's rows)
//   pattern 3: stride-2 rows over a 512-B span
// Checks the sum of all adds (lost updates -> mismatch).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdio.h>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
typedef _Float16 h2v __attribute__((ext_vector_type(2)));

__global__ void k_scatter(float *tab, uint32_t rows, int apt, int pattern) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    for (int i = 0; i < apt; ++i) {
        const uint32_t w = hash32(wave * 7919u + i * 104729u);
        uint32_t row;
        if (pattern == 0) row = hash32(w ^ (lane * 2654435761u)) % rows;
        else if (pattern == 1) row = (w % (rows / 64)) * 64 + lane;
        else if (pattern == 2) row = (hash32(w + (lane >> 3)) % (rows / 8)) * 8 + (lane & 7);
        else row = (w % (rows / 128)) * 128 + 2 * lane;
        h2v v = {(_Float16)1.0f, (_Float16)1.0f};
        __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2v *)(tab + row), v);
    }
}
__global__ void k_reduce(const float *tab, uint32_t rows, double *out) {
    double s = 0;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < rows; i += gridDim.x * blockDim.x) {
        const __half2 v = *reinterpret_cast<const __half2 *>(tab + i);
        s += (double)__low2float(v) + (double)__high2float(v);
    }
    atomicAdd(out, s);
}

int main() {
    const uint32_t rows = 6512256;
    const int threads = 256, blocks = 8192, apt = 8;
    float *tab; double *sum;
    hipMalloc(&tab, (size_t)rows * 4); hipMalloc(&sum, 8);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    const double n_ops = (double)threads * blocks * apt;
    for (int pattern = 0; pattern < 4; ++pattern) {
        float best = 1e30f; double total = 0;
        for (int rep = 0; rep < 3; ++rep) {
            hipMemset(tab, 0, (size_t)rows * 4); hipMemset(sum, 0, 8);
            hipEventRecord(e0);
            hipLaunchKernelGGL(k_scatter, dim3(blocks), dim3(threads), 0, 0, tab, rows, apt, pattern);
            hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); if (ms < best) best = ms;
            hipLaunchKernelGGL(k_reduce, dim3(1024), dim3(256), 0, 0, tab, rows, sum);
            hipMemcpy(&total, sum, 8, hipMemcpyDeviceToHost);
        }
        printf("{\"pattern\": %d, \"ms\": %.3f, \"G_lane_ops_per_s\": %.2f, \"sum\": %.0f, \"expected\": %.0f}\n",
               pattern, best, n_ops / (best * 1e-3) / 1e9, total, 2 * n_ops);
        fflush(stdout);
    }
    return 0;
}
