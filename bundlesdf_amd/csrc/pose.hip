// Per-frame pose correction of the training step on the device:
//   forward  — PoseArray.get_matrices (nerf_helpers.py:127-154: tanh bound,
//              pytorch3d se3_exp_map, transpose, frame 0 = identity) fused with
//              tf = T @ c2w (nerf_runner.py:1050-1052), plus the exact Jacobian
//              d tf[:3,:4] / d data (forward-mode dual numbers through the same
//              op sequence, 6 tangents per scalar);
//   backward — dL/dtf per ray (written by the field kernels) reduced per frame
//              and contracted with the Jacobian into the pose gradient.
// Replaces ~40 small torch kernels (and their autograd graph) per step with
// three launches.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "nof_device.h"
#include "schedule.h"

namespace nof {
namespace {

struct Dual {
    float v;
    float d[6];
};
__device__ __forceinline__ Dual dconst(float v) {
    Dual r;
    r.v = v;
#pragma unroll
    for (int i = 0; i < 6; ++i) r.d[i] = 0.f;
    return r;
}
__device__ __forceinline__ Dual operator+(const Dual &a, const Dual &b) {
    Dual r;
    r.v = a.v + b.v;
#pragma unroll
    for (int i = 0; i < 6; ++i) r.d[i] = a.d[i] + b.d[i];
    return r;
}
__device__ __forceinline__ Dual operator-(const Dual &a, const Dual &b) {
    Dual r;
    r.v = a.v - b.v;
#pragma unroll
    for (int i = 0; i < 6; ++i) r.d[i] = a.d[i] - b.d[i];
    return r;
}
__device__ __forceinline__ Dual operator*(const Dual &a, const Dual &b) {
    Dual r;
    r.v = a.v * b.v;
#pragma unroll
    for (int i = 0; i < 6; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
    return r;
}
__device__ __forceinline__ Dual scale(const Dual &a, float s) {
    Dual r;
    r.v = a.v * s;
#pragma unroll
    for (int i = 0; i < 6; ++i) r.d[i] = a.d[i] * s;
    return r;
}
__device__ __forceinline__ Dual dapply(const Dual &a, float v, float dv) {   // f(a) with f' = dv
    Dual r;
    r.v = v;
#pragma unroll
    for (int i = 0; i < 6; ++i) r.d[i] = a.d[i] * dv;
    return r;
}
__device__ __forceinline__ Dual dsin(const Dual &a) { return dapply(a, sinf(a.v), cosf(a.v)); }
__device__ __forceinline__ Dual dcos(const Dual &a) { return dapply(a, cosf(a.v), -sinf(a.v)); }
__device__ __forceinline__ Dual dsqrt(const Dual &a) {
    const float s = sqrtf(a.v);
    return dapply(a, s, 0.5f / s);
}
__device__ __forceinline__ Dual drecip(const Dual &a) { return dapply(a, 1.0f / a.v, -1.0f / (a.v * a.v)); }
// torch.clamp(x, min): gradient passes where x >= min
__device__ __forceinline__ Dual dclamp_min(const Dual &a, float lo) {
    return a.v >= lo ? a : dconst(lo);
}

// Pose of frame f: tf = T(data_f) @ c2w_f; tf_out [16] row-major 4x4, jac [12][6].
__device__ __forceinline__ void pose_forward_one(int f, const float *__restrict__ data, const float *__restrict__ c2w,
                                                 float max_trans, float max_rot_rad, float *__restrict__ tf_out,
                                                 float *__restrict__ jac) {
    Dual T[4][4];
    if (f == 0) {
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) T[i][j] = dconst(i == j ? 1.f : 0.f);
    } else {
        Dual lg[6];
#pragma unroll
        for (int p = 0; p < 6; ++p) {
            const float x = data[f * 6 + p];
            const float th = tanhf(x);
            Dual d = dconst(th);
            d.d[p] = 1.f - th * th;
            lg[p] = scale(d, p < 3 ? max_trans : max_rot_rad);
        }
        const Dual *t = lg, *w = lg + 3;
        const Dual nrms = (w[0] * w[0] + w[1] * w[1]) + w[2] * w[2];
        const Dual ang = dsqrt(dclamp_min(nrms, 1e-4f));
        const Dual ang_inv = drecip(ang);
        const Dual sn = dsin(ang), cs = dcos(ang);
        const Dual fac1 = ang_inv * sn;
        const Dual one = dconst(1.f);
        const Dual fac2 = (ang_inv * ang_inv) * (one - cs);
        // K = hat(w), K2 = K @ K
        const Dual zero = dconst(0.f);
        Dual K[3][3] = {{zero, dconst(0.f) - w[2], w[1]}, {w[2], zero, dconst(0.f) - w[0]}, {dconst(0.f) - w[1], w[0], zero}};
        Dual K2[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) K2[i][j] = (K[i][0] * K[0][j] + K[i][1] * K[1][j]) + K[i][2] * K[2][j];
        const Dual ang2 = ang * ang;
        const Dual cV1 = (one - cs) * drecip(ang2);
        const Dual cV2 = (ang - sn) * drecip(ang2 * ang);
        Dual R[3][3], V[3][3];
#pragma unroll
        for (int i = 0; i < 3; ++i)
#pragma unroll
            for (int j = 0; j < 3; ++j) {
                const Dual e = dconst(i == j ? 1.f : 0.f);
                R[i][j] = (fac1 * K[i][j] + fac2 * K2[i][j]) + e;
                V[i][j] = (e + K[i][j] * cV1) + K2[i][j] * cV2;
            }
        Dual Tv[3];
#pragma unroll
        for (int i = 0; i < 3; ++i) Tv[i] = (V[i][0] * t[0] + V[i][1] * t[1]) + V[i][2] * t[2];
        // se3_exp_map is row-vector form [R 0; T 1]; PoseArray transposes it
#pragma unroll
        for (int i = 0; i < 3; ++i) {
#pragma unroll
            for (int j = 0; j < 3; ++j) T[i][j] = R[j][i];
            T[i][3] = Tv[i];
            T[3][i] = dconst(0.f);
        }
        T[3][3] = dconst(1.f);
    }
    const float *C = c2w + (size_t)f * 16;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            Dual acc = T[i][0] * dconst(C[0 * 4 + j]);
#pragma unroll
            for (int k = 1; k < 4; ++k) acc = acc + T[i][k] * dconst(C[k * 4 + j]);
            tf_out[(size_t)f * 16 + i * 4 + j] = acc.v;
            if (i < 3) {
#pragma unroll
                for (int p = 0; p < 6; ++p) jac[((size_t)f * 12 + i * 4 + j) * 6 + p] = acc.d[p];
            }
        }
}
__global__ __launch_bounds__(64) void k_pose_forward(const float *__restrict__ data, const float *__restrict__ c2w,
                                                     int F, float max_trans, float max_rot_rad,
                                                     float *__restrict__ tf_out, float *__restrict__ jac) {
    const int f = blockIdx.x * blockDim.x + threadIdx.x;
    if (f < F) pose_forward_one(f, data, c2w, max_trans, max_rot_rad, tf_out, jac);
}

// The step prologue in one launch (graph replay: three dependent-free pieces that each took a
// ~5 us launch of their own): block 0 the step schedule (k_step_schedule), the next
// div_up(F, 256) blocks the pose forward (k_pose_forward), the rest the MLP fragment packing
// (k_pack_mlp, field_step.hip: fragment element i <- mlp[idx[i]], then the bias image).
template <typename TM>
__global__ __launch_bounds__(256) void k_prologue(nof_schedule_desc sd, int32_t *step, nof_step_params *sp_out,
                                                  const float *__restrict__ data, const float *__restrict__ c2w, int F,
                                                  float max_trans, float max_rot_rad, float *__restrict__ tf_out,
                                                  float *__restrict__ jac, const float *__restrict__ mlp,
                                                  const int32_t *__restrict__ idx, int n_frag_elems, int n_bias,
                                                  TM *__restrict__ frags, float *__restrict__ bias, int sched) {
    const int nbp = (F + 255) / 256;
    if (blockIdx.x == 0) {
        if (sched && threadIdx.x == 0) step_schedule_one(sd, step, sp_out);
        return;
    }
    if ((int)blockIdx.x <= nbp) {
        const int f = ((int)blockIdx.x - 1) * 256 + (int)threadIdx.x;
        if (f < F) pose_forward_one(f, data, c2w, max_trans, max_rot_rad, tf_out, jac);
        return;
    }
    const int i = ((int)blockIdx.x - 1 - nbp) * 256 + (int)threadIdx.x;
    if (i < n_frag_elems) {
        const int k = idx[i];
        frags[i] = (TM)(k >= 0 ? mlp[k] : 0.f);
    } else if (i < n_frag_elems + n_bias) {
        const int k = idx[i];
        bias[i - n_frag_elems] = k >= 0 ? mlp[k] : 0.f;
    }
}

// fg[F][12] += sum over rays of frame f of ray_grad[r][12] (block-level LDS
// accumulation, then one atomic per (frame, entry) the block touched). Each block takes a
// contiguous run of rays: the batches are drawn per frame in ascending order, so a block touches
// one or two frames (a grid-stride split had every block touch every frame: 512 same-address
// atomics on each of the F x 12 sums).
__global__ __launch_bounds__(256) void k_pose_reduce(const float *__restrict__ ray_grad, const float *__restrict__ rays,
                                                     int R, int F, float *__restrict__ fg) {
    extern __shared__ float s_fg[];   // [F][12]
    for (int i = threadIdx.x; i < F * 12; i += blockDim.x) s_fg[i] = 0.f;
    __syncthreads();
    const int64_t per = ((int64_t)R + gridDim.x - 1) / gridDim.x;
    const int64_t e0 = (int64_t)blockIdx.x * per * 12, e1 = std::min<int64_t>((int64_t)R * 12, e0 + per * 12);
    for (int64_t e = e0 + threadIdx.x; e < e1; e += blockDim.x) {
        const int r = (int)(e / 12), k = (int)(e % 12);
        const int f = (int)rays[(size_t)r * 12 + 8];
        const float g = ray_grad[e];
        if (g != 0.f && f >= 0 && f < F) atomicAdd(&s_fg[f * 12 + k], g);
    }
    __syncthreads();
    for (int i = threadIdx.x; i < F * 12; i += blockDim.x)
        if (s_fg[i] != 0.f) atomic_add_f32(fg + i, s_fg[i]);
}

// grad_pose[f][p] += sum_k fg[f][k] * jac[f][k][p]; then fg is cleared for the next call (a block
// per frame: its 6 threads read the frame's 12 sums before a barrier, one thread clears them)
__global__ __launch_bounds__(64) void k_pose_grad(float *__restrict__ fg, const float *__restrict__ jac, int F,
                                                  float *__restrict__ grad_pose) {
    const int f = blockIdx.x, p = threadIdx.x;
    float s = 0.f;
    if (p < 6) {
#pragma unroll
        for (int k = 0; k < 12; ++k) s = __builtin_fmaf(fg[f * 12 + k], jac[((size_t)f * 12 + k) * 6 + p], s);
    }
    __syncthreads();
    if (p < 6) grad_pose[f * 6 + p] += s;
    if (p < 12) fg[f * 12 + p] = 0.f;
}

}  // namespace
}  // namespace nof

extern "C" int nof_pose_forward(const float *data, const float *c2w, int32_t F, float max_trans, float max_rot_rad,
                                float *tf_out, float *jac, void *stream) {
    if (!data || !c2w || !tf_out || !jac || F <= 0) return nof::set_error(NOF_EINVAL, "pose_forward: bad arguments");
    hipLaunchKernelGGL(nof::k_pose_forward, dim3(nof::div_up(F, 64)), dim3(64), 0, (hipStream_t)stream, data, c2w, F,
                       max_trans, max_rot_rad, tf_out, jac);
    return nof::check_launch("pose_forward");
}

extern "C" int nof_step_prologue(const nof_schedule_desc *sched, int32_t *step, nof_step_params *sp_out,
                                 const float *data, const float *c2w, int32_t F, float max_trans, float max_rot_rad,
                                 float *tf_out, float *jac, const float *mlp, const int32_t *idx, int32_t n_frag_elems,
                                 int32_t n_bias, void *frags, float *bias, int mlp_dtype, void *stream) {
    if (!data || !c2w || !tf_out || !jac || F <= 0 || !mlp || !idx || !frags || !bias || n_frag_elems < 0 ||
        n_bias < 0 || (sched && (!step || !sp_out)))
        return nof::set_error(NOF_EINVAL, "step_prologue: bad arguments");
    if (mlp_dtype != NOF_F16 && mlp_dtype != NOF_F32)
        return nof::set_error(NOF_EINVAL, "step_prologue: mlp_dtype %d", mlp_dtype);
    nof_schedule_desc sd{};
    if (sched) {
        if (sched->trunc_decay < 0 || sched->trunc_decay > 2 || sched->n_step <= 0)
            return nof::set_error(NOF_EINVAL, "step_prologue: trunc_decay %d / n_step %d", sched->trunc_decay,
                                  sched->n_step);
        sd = *sched;
    }
    const int nbp = nof::div_up(F, 256), nbk = nof::div_up(n_frag_elems + n_bias, 256);
    const dim3 grid(1 + nbp + nbk);
    if (mlp_dtype == NOF_F16)
        hipLaunchKernelGGL(nof::k_prologue<_Float16>, grid, dim3(256), 0, (hipStream_t)stream, sd, step, sp_out, data,
                           c2w, F, max_trans, max_rot_rad, tf_out, jac, mlp, idx, n_frag_elems, n_bias,
                           (_Float16 *)frags, bias, sched ? 1 : 0);
    else
        hipLaunchKernelGGL(nof::k_prologue<float>, grid, dim3(256), 0, (hipStream_t)stream, sd, step, sp_out, data,
                           c2w, F, max_trans, max_rot_rad, tf_out, jac, mlp, idx, n_frag_elems, n_bias,
                           (float *)frags, bias, sched ? 1 : 0);
    return nof::check_launch("step_prologue");
}

namespace nof {
__global__ void k_zero_f32(float *__restrict__ p, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) p[i] = 0.f;
}
}  // namespace nof

extern "C" int nof_pose_backward(const float *ray_grad, const float *rays, int32_t R, const float *jac, int32_t F,
                                 float *fg, float *grad_pose, void *stream) {
    if (!ray_grad || !rays || !jac || !fg || !grad_pose || R < 0 || F <= 0 || F > 1024)
        return nof::set_error(NOF_EINVAL, "pose_backward: bad arguments (F <= 1024)");
    hipStream_t st = (hipStream_t)stream;
    // fg is zero on entry and left zero (k_pose_grad clears what it consumed): no zeroing launch
    if (R > 0) {
        const int blocks = (int)std::min<int64_t>(nof::div_up((uint64_t)R * 12, 256), 512);
        hipLaunchKernelGGL(nof::k_pose_reduce, dim3(blocks), dim3(256), (size_t)F * 12 * sizeof(float), st, ray_grad,
                           rays, R, F, fg);
        const int rc = nof::check_launch("pose_backward(reduce)");
        if (rc) return rc;
    }
    hipLaunchKernelGGL(nof::k_pose_grad, dim3(F), dim3(64), 0, st, fg, jac, F, grad_pose);
    return nof::check_launch("pose_backward(grad)");
}
