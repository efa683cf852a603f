// Diagnostic microbenchmark (not part of libnof): scatter-add throughput of
// fp32 atomics on MI355X for the hash-table gradient pattern.
//   mode 0: device (agent) scope atomics into one table
//   mode 1: workgroup-scope atomics into a per-XCD private copy (HW_REG_XCC_ID)
//   mode 2: like 1, packed fp16x2 atomics (one dword per row)
// Every lane adds 1.0 to pseudo-random rows (clustered like ray samples:
// runs of `run` consecutive lanes hit the same row); the copies are summed
// and the total checked against the number of adds (lost updates -> error).
#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdio.h>
#include <stdlib.h>
#include <vector>

__device__ __forceinline__ uint32_t hash32(uint32_t x) {
    x ^= x >> 16; x *= 0x7feb352dU; x ^= x >> 15; x *= 0x846ca68bU; x ^= x >> 16;
    return x;
}
__device__ __forceinline__ int xcc_id() {
    int v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    return v & 0xf;
}

__global__ void k_scatter(float *tab, int rows, int adds_per_thread, int run, int mode, int *xcc_seen) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    float *t = tab;
    if (mode >= 1) {
        const int x = xcc_id();
        if (threadIdx.x == 0) atomicOr(xcc_seen, 1 << x);
        t = tab + (size_t)x * rows * 2;
    }
    for (int i = 0; i < adds_per_thread; ++i) {
        const uint32_t key = (tid / run) * 1315423911u + i * 2654435761u;
        const uint32_t row = hash32(key) % rows;
        if (mode == 0) {
            __hip_atomic_fetch_add(t + row * 2, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(t + row * 2 + 1, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else if (mode == 1) {
            __hip_atomic_fetch_add(t + row * 2, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            __hip_atomic_fetch_add(t + row * 2 + 1, 1.0f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else {
            typedef _Float16 h2v __attribute__((ext_vector_type(2)));
            h2v v = {(_Float16)1.0f, (_Float16)1.0f};
            __builtin_amdgcn_global_atomic_fadd_v2f16((__attribute__((address_space(1))) h2v *)(t + row), v);
        }
    }
}

__global__ void k_reduce(const float *tab, int rows, int copies, double *out) {
    double s = 0;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)rows * 2; i += gridDim.x * blockDim.x)
        for (int c = 0; c < copies; ++c) s += tab[(size_t)c * rows * 2 + i];
    atomicAdd(out, s);
}
__global__ void k_reduce_h(const float *tab, int rows, int copies, double *out) {
    double s = 0;
    for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < (size_t)rows; i += gridDim.x * blockDim.x)
        for (int c = 0; c < copies; ++c) {
            const __half2 v = *reinterpret_cast<const __half2 *>(tab + (size_t)c * rows * 2 + i);
            s += (double)__low2float(v) + (double)__high2float(v);
        }
    atomicAdd(out, s);
}

int main(int argc, char **argv) {
    const int rows = 6512256;
    const int threads = 256, blocks = 8192, apt = 16;
    float *tab;
    double *sum;
    int *xs;
    hipMalloc(&tab, (size_t)8 * rows * 2 * 4);
    hipMalloc(&sum, 8);
    hipMalloc(&xs, 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const double n_adds = (double)threads * blocks * apt * 2;
    for (int run : {1, 4, 16}) {
        for (int mode = 0; mode < 3; ++mode) {
            const int copies = mode == 0 ? 1 : 8;
            float best = 1e30f;
            double total = 0;
            int seen = 0;
            for (int rep = 0; rep < 3; ++rep) {
                hipMemset(tab, 0, (size_t)copies * rows * 2 * 4);
                hipMemset(sum, 0, 8);
                hipMemset(xs, 0, 4);
                hipEventRecord(e0);
                hipLaunchKernelGGL(k_scatter, dim3(blocks), dim3(threads), 0, 0, tab, rows, apt, run, mode, xs);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
                float ms;
                hipEventElapsedTime(&ms, e0, e1);
                if (ms < best) best = ms;
                if (mode == 2) hipLaunchKernelGGL(k_reduce_h, dim3(1024), dim3(256), 0, 0, tab, rows, copies, sum);
                else hipLaunchKernelGGL(k_reduce, dim3(1024), dim3(256), 0, 0, tab, rows, copies, sum);
                hipMemcpy(&total, sum, 8, hipMemcpyDeviceToHost);
                hipMemcpy(&seen, xs, 4, hipMemcpyDeviceToHost);
            }
            printf("{\"run\": %d, \"mode\": %d, \"ms\": %.3f, \"Gadds_per_s\": %.2f, \"sum\": %.0f, \"expected\": %.0f, "
                   "\"xcc_mask\": %d}\n", run, mode, best, n_adds / (best * 1e-3) / 1e9, total, n_adds, seen);
            fflush(stdout);
        }
    }
    return 0;
}
