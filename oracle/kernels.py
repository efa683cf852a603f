"""ORACLE — test infrastructure only (tests/, __graft_entry__.smoke(),
bench.py cpu_baseline). numpy front-end over liboracle.so, the C restatement
of the reference kernels (see grid_oracle.c / ray_oracle.c headers for the
reference lines and the pinning status of each function)."""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None
_p = ctypes.c_void_p
_u32 = ctypes.c_uint32
_int = ctypes.c_int
_f32 = ctypes.c_float
_i64 = ctypes.c_int64


def build():
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return os.path.join(_HERE, "liboracle.so")


def lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, "liboracle.so")
        if not os.path.exists(path):
            build()
        L = ctypes.CDLL(path)
        L.oracle_level_params.argtypes = [_u32, _f32, _u32, _p, _p]
        fw = [_p, _p, _p, _p, _u32, _u32, _u32, _u32, _f32, _u32, _int, _p, _u32, _int]
        bw = [_p, _p, _p, _p, _u32, _u32, _u32, _u32, _f32, _u32, _int, _p, _p, _u32, _int]
        for n in ("oracle_grid_encode_forward_f32", "oracle_grid_encode_forward_f16"):
            getattr(L, n).argtypes = fw
        for n in ("oracle_grid_encode_backward_f32", "oracle_grid_encode_backward_f16"):
            getattr(L, n).argtypes = bw
        L.oracle_sample_occupied.argtypes = [_p, _p, _p, _int, _int, _int]
        L.oracle_sample_occupied.restype = _int
        L.oracle_postprocess_octree.argtypes = [_p, _p, _p, _p, _i64, _i64, _int, _p]
        L.oracle_octree_ray_trace.argtypes = [_p, _int, _p, _p, _int, _int, _p, _p]
        _LIB = L
    return _LIB


def _ptr(a):
    return ctypes.c_void_p(a.ctypes.data) if a is not None else ctypes.c_void_p(0)


def level_params(L, S, H):
    sc = np.zeros(L, np.float32)
    res = np.zeros(L, np.uint32)
    lib().oracle_level_params(L, np.float32(S), H, _ptr(sc), _ptr(res))
    return sc, res


def grid_encode_forward(inputs, embeddings, offsets, S, H, calc_grad_inputs=False, gridtype=0, align_corners=False):
    """gridencoder.cu:106-246 restated. Returns (outputs [L,B,C], dy_dx [B,L*D*C] or None), dtype of embeddings."""
    inputs = np.ascontiguousarray(inputs, np.float32)
    offsets = np.ascontiguousarray(offsets, np.int32)
    half = embeddings.dtype == np.float16
    emb = np.ascontiguousarray(embeddings)
    B, D = inputs.shape
    L = offsets.shape[0] - 1
    C = emb.shape[1]
    out = np.zeros((L, B, C), emb.dtype)
    dydx = np.zeros((B, L * D * C), emb.dtype) if calc_grad_inputs else None
    fn = lib().oracle_grid_encode_forward_f16 if half else lib().oracle_grid_encode_forward_f32
    fn(_ptr(inputs), _ptr(emb), _ptr(offsets), _ptr(out), B, D, C, L, np.float32(S), int(H), int(calc_grad_inputs),
       _ptr(dydx), int(gridtype), int(align_corners))
    return out, dydx


def grid_encode_backward(grad, inputs, offsets, n_rows, S, H, calc_grad_inputs=False, dy_dx=None, gridtype=0,
                         align_corners=False):
    """gridencoder.cu:249-365 restated (serial accumulation order). grad [L,B,C]."""
    grad = np.ascontiguousarray(grad)
    inputs = np.ascontiguousarray(inputs, np.float32)
    offsets = np.ascontiguousarray(offsets, np.int32)
    half = grad.dtype == np.float16
    L, B, C = grad.shape
    D = inputs.shape[1]
    gemb = np.zeros((n_rows, C), grad.dtype)
    gin = np.zeros((B, D), grad.dtype) if calc_grad_inputs else None
    dd = np.ascontiguousarray(dy_dx) if calc_grad_inputs else None
    fn = lib().oracle_grid_encode_backward_f16 if half else lib().oracle_grid_encode_backward_f32
    fn(_ptr(grad), _ptr(inputs), _ptr(offsets), _ptr(gemb), B, D, C, L, np.float32(S), int(H), int(calc_grad_inputs),
       _ptr(dd), _ptr(gin), int(gridtype), int(align_corners))
    return gemb, gin


def sample_occupied(z_in_out, z_sampled, z_vals=None):
    """common.cu:40-105 restated; returns (z_vals, n_errors)."""
    z_in_out = np.ascontiguousarray(z_in_out, np.float32)
    z_sampled = np.ascontiguousarray(z_sampled, np.float32)
    z = np.zeros_like(z_sampled) if z_vals is None else np.ascontiguousarray(z_vals, np.float32).copy()
    n, k, _ = z_in_out.shape
    err = lib().oracle_sample_occupied(_ptr(z_in_out), _ptr(z_sampled), _ptr(z), n, k, z_sampled.shape[1])
    return z, err


def postprocess_octree(ray_index, depth_in_out, unique_ids, start_poss, max_int, n_rays):
    """common.cu:128-167 restated."""
    ray_index = np.ascontiguousarray(ray_index, np.int64)
    depth_in_out = np.ascontiguousarray(depth_in_out, np.float32)
    unique_ids = np.ascontiguousarray(unique_ids, np.int64)
    start_poss = np.ascontiguousarray(start_poss, np.int64)
    out = np.zeros((n_rays, max_int, 2), np.float32)
    lib().oracle_postprocess_octree(_ptr(ray_index), _ptr(depth_in_out), _ptr(unique_ids), _ptr(start_poss),
                                    ray_index.shape[0], unique_ids.shape[0], int(max_int), _ptr(out))
    return out


def octree_ray_trace(occ, rays_o, rays_d, kmax):
    """Dense-grid restatement of kaolin unbatched_raytrace + postprocess (PARITY UNPINNED)."""
    occ = np.ascontiguousarray(occ, np.uint8)
    N = occ.shape[0]
    rays_o = np.ascontiguousarray(rays_o, np.float32)
    rays_d = np.ascontiguousarray(rays_d, np.float32)
    R = rays_o.shape[0]
    out = np.zeros((R, kmax, 2), np.float32)
    counts = np.zeros(R, np.int32)
    lib().oracle_octree_ray_trace(_ptr(occ), N, _ptr(rays_o), _ptr(rays_d), R, kmax, _ptr(out), _ptr(counts))
    return out, counts
