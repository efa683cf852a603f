"""ctypes binding of libnof.so (the C ABI declared in include/nof.h).

torch is imported first so that its bundled HIP runtime (soname
libamdhip64.so.7) is the one libnof.so binds to: one runtime, one set of
streams. There is no CPU fallback anywhere behind this module — a missing or
unloadable library raises immediately.
"""
import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL load, see module doc)

_HERE = os.path.dirname(os.path.abspath(__file__))
# NOF_LIB: the timing-ablation build (scripts/ablate.py) only
LIB_PATH = os.environ.get("NOF_LIB") or os.path.join(_HERE, "libnof.so")
_LIB = None

_p = ctypes.c_void_p
_u32 = ctypes.c_uint32
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_f32 = ctypes.c_float
_int = ctypes.c_int

_SIGNATURES = {
    "nof_last_error": ([], ctypes.c_char_p),
    "nof_version": ([], ctypes.c_char_p),
    "nof_level_params": ([_u32, _f32, _u32, _p, _p], None),
    "nof_grid_encode_forward": ([_p, _p, _p, _p, _u32, _u32, _u32, _u32, _f32, _u32, _int, _p, _u32, _int, _int, _p],
                                _int),
    "nof_grid_encode_backward": ([_p, _p, _p, _p, _p, _u32, _u32, _u32, _u32, _f32, _u32, _int, _p, _p, _u32, _int,
                                  _int, _p], _int),
    "nof_sample_rays_uniform_occupied_voxels": ([_p, _p, _p, _i32, _i32, _i32, _p, _p], _int),
    "nof_postprocess_octree_ray_tracing": ([_p, _p, _p, _p, _i64, _i64, _i32, _p, _p], _int),
    "nof_ray_color_to_texture_uv": ([_p, _p, _p, _p, _p, _p, _i64, _p], _int),
    "nof_octree_ray_trace": ([_p, _i32, _p, _p, _i32, _i32, _p, _p, _p], _int),
    "nof_step_schedule": ([_p, _p, _p, _p], _int),
    "nof_trace_rays": ([_p, _p, _i32, _p, _p, _i32, _i32, _f32, _f32, _f32, _p, _p, _p, _p, _p, _p], _int),
    "nof_trace_rays_epoch": ([_p, _p, _p, _i32, _p, _p, _i32, _i32, _f32, _f32, _f32, _p, _p, _p, _p, _p, _p], _int),
    "nof_sample_batch": ([_p, _i32, _i32, _u32, _p, _p, _p], _int),
    "nof_pack_mlp": ([_p, _p, _i32, _i32, _p, _p, _int, _p], _int),
    "nof_field_step": ([_p, _p], _int),
    "nof_quad_mirror": ([_p, _p], _int),
    "nof_field_workspace_bytes": ([_i32, _i32, _i32], ctypes.c_size_t),
    "nof_field_workspace_offsets": ([_i32, _i32, _i32, _p, _i32], _int),
    "nof_field_timing": ([_i32], _int),
    "nof_pose_forward": ([_p, _p, _i32, _f32, _f32, _p, _p, _p], _int),
    "nof_step_prologue": ([_p, _p, _p, _p, _p, _i32, _f32, _f32, _p, _p, _p, _p, _i32, _i32, _p, _p, _int, _p], _int),
    "nof_query_sdf": ([_p, _i32, _p, ctypes.c_uint32, _p, _p, _i32, _i32, _p, ctypes.c_int64, _p, _p, _p, _i32, _i32,
                       _i32, _p, _i32, _p, _p], _int),
    "nof_pose_backward": ([_p, _p, _i32, _p, _i32, _p, _p, _p], _int),
    "nof_field_timing_collect": ([_p, _i32, _p], _int),
    "nof_level_table": ([_u32, _f32, _u32, _p, _p], None),
    "nof_unscale_check": ([_p, _i64, _p, _p, _p, _i64, _i64, _i64, _p], _int),
    "nof_adam_active_bytes": ([_i64], ctypes.c_size_t),
    "nof_adam_step": ([_p, _p, _p, _p, _i64, _i64, ctypes.c_double, ctypes.c_double, _f32, _f32, _f32, _p, _p, _p,
                       _i64, _p, _p, _p, _p, _p], _int),
    "nof_scaler_update": ([_p, _p, _p, _p, _f32, _f32, _i32, _int, _p], _int),
    "nof_to_half": ([_p, _p, _i64, _p], _int),
    "nof_grad16_to_f32": ([_p, _p, _i64, _p], _int),
    "nof_ray_pool_workspace_bytes": ([_i32, _i32, _i32], ctypes.c_size_t),
    "nof_make_frame_rays": ([_p, _p], _int),
    "nof_point_grid_workspace_bytes": ([_i64], ctypes.c_size_t),
    "nof_point_grid_build": ([_p, _i32, _p, _p, ctypes.c_double, _p, _p, _p, _p, _p], _int),
    "nof_knn_mean_dist": ([_p, _i32, _i32, _p, _p], _int),
    "nof_dbscan_workspace_bytes": ([_i32, _i64], ctypes.c_size_t),
    "nof_raster_faces": ([_p, _p, _i64, _p, _p, _i32, _i32, ctypes.c_double, ctypes.c_double, _p, _p], _int),
    "nof_texture_hits": ([_p, _i32, _i32, _p, _f32, _p, _p, _p, _p, _p, _p, _p], _int),
    "nof_texture_accumulate": ([_p, _p, _i64, _p, _i32, _i32, _p, _p, _p, _p], _int),
    "nof_segment_mean": ([_p, _i32, _p, _p, _i32, _p, _p], _int),
    "nof_dbscan": ([_p, _i32, ctypes.c_double, _i32, _p, _p, _p, _p, _p], _int),
}


class FieldDesc(ctypes.Structure):
    """Mirror of nof_field_desc (include/nof.h)."""
    _fields_ = [("rays", _p), ("tf", _p), ("intervals", _p), ("totals", _p), ("t_rand", _p), ("seed", _u32),
                ("R", _i32), ("Kmax", _i32), ("N_oct", _i32), ("N_dep", _i32), ("S", _i32), ("perturb", _i32),
                ("near_sc", _f32), ("far_sc", _f32), ("trunc", _f32), ("neg_trunc_ratio", _f32), ("sdf_lambda", _f32),
                ("fs_sdf", _f32), ("first_frame_weight", _f32), ("rgb_weight", _f32), ("fs_weight", _f32),
                ("empty_weight", _f32), ("trunc_weight", _f32), ("loss_scale", _p), ("table", _p), ("levels", _p),
                ("L", _u32), ("C", _u32), ("D", _u32), ("table_dtype", _i32), ("mlp_dtype", _i32), ("frags", _p),
                ("bias", _p), ("grad_table", _p), ("grad_table16", _p), ("grad_mlp", _p), ("ray_grad", _p), ("loss_acc", _p), ("dbg_z", _p),
                ("dbg_raw", _p), ("dbg_valid", _p), ("dbg_rgb", _p), ("blocks_per_cu", _i32), ("ablate", _i32),
                ("workspace", _p), ("scatter_slots", _i32),
                ("n_ff", _i32), ("ff", _p), ("grad_ff", _p), ("fs_rgb_weight", _f32),
                ("xcd_order", _i32), ("step_params", _p), ("skip_pose_grad", _i32),
                ("scatter_levels_per_wave", _i32), ("table_quads", _p),
                ("table_rows", ctypes.c_int64), ("quads_min_rays", _i32), ("scatter_kernel", _i32),
                ("scatter_waves_per_ray", _i32), ("scatter_ls_levels", _i32), ("encode_sigma", _i32),
                ("bwd_flush", _i32), ("count_atomics", _i32),
                ("scatter_flat", _i32), ("compact_per_block", _i32),
                ("encode_group", _i32), ("quads_prebuilt", _i32), ("mlp_pass1_tiles", _i32),
                ("scatter_fuse_levels", _i32), ("encode_wpb", _i32)]


class StepParams(ctypes.Structure):
    """Mirror of nof_step_params (include/nof.h): the device step block."""
    _fields_ = [("lr0", ctypes.c_double), ("lr1", ctypes.c_double), ("trunc", _f32), ("seed", _u32),
                ("batch_seed", _u32), ("step", _i32)]


class ScheduleDesc(ctypes.Structure):
    """Mirror of nof_schedule_desc (include/nof.h)."""
    _d = ctypes.c_double
    _fields_ = [("lrate", _d), ("lrate_pose", _d), ("decay_rate", _d), ("trunc", _d), ("trunc_start", _d),
                ("sc_factor", _d), ("trunc_decay", _i32), ("n_step", _i32), ("seed_base", _u32),
                ("batch_seed_base", _u32)]


class RayPoolDesc(ctypes.Structure):
    """Mirror of nof_ray_pool_desc (include/nof.h)."""
    _d = ctypes.c_double
    _fields_ = [("rgb", _p), ("depth", _p), ("mask", _p), ("occ_mask", _p), ("cam_in_world", _p), ("F", _i32),
                ("H", _i32), ("W", _i32), ("first_frame_id", _i32), ("dilate_first", _i32), ("dilate_other", _i32),
                ("fx", _f32), ("fy", _f32), ("cx", _f32), ("cy", _f32), ("near_sc", _f32), ("far_sc", _f32),
                ("far_sc64", _d), ("bbox", _d * 6), ("occ", _p), ("occ_n", _i32), ("cell_start", _p),
                ("cell_points", _p), ("grid_origin", _d * 3), ("grid_dims", _i32 * 3), ("grid_cell", _d),
                ("grid_radius", _d), ("workspace", _p), ("rays", _p), ("n_out", _p)]


def declared_symbols():
    return list(_SIGNATURES)


def lib():
    """Load libnof.so once; raise if it is missing (no fallback)."""
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} is missing: build it with `python -m bundlesdf_amd.build` "
                               "(the HIP path has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        for name, (args, res) in _SIGNATURES.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _LIB = L
    return _LIB


def check(rc, what=""):
    if rc != 0:
        msg = lib().nof_last_error().decode(errors="replace")
        raise RuntimeError(f"{what}: {msg}" if what else msg)


def ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


def stream_of(t):
    """Current HIP stream of tensor t's device (graph-capture safe)."""
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(t, name):
    if not (t.is_cuda):
        raise RuntimeError(f"{name} must be a CUDA tensor")


def require_contiguous(t, name):
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be a contiguous tensor")
