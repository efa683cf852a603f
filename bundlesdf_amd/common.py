"""Module `common` — drop-in for the reference's pybind extension
(mycuda/bindings.cpp:14-18), backed by libnof.

Deviation from the reference, on purpose: malformed sampler input does not
hang the GPU (common.cu:66-71,87-92 spin forever); the sample is left as is
and a per-device error counter is bumped. `sampler_error_count()` reads it
(a host sync — call it off the critical path).
"""
import torch

from . import _lib

_ERR = {}


def _err_counter(device):
    key = (device.type, device.index)
    if key not in _ERR:
        _ERR[key] = torch.zeros(1, dtype=torch.int32, device=device)
    return _ERR[key]


def sampler_error_count(device=None):
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    return int(_err_counter(device).item())


def reset_sampler_errors(device=None):
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    _err_counter(device).zero_()


def _check_input(t, name):
    if not t.is_cuda:
        raise RuntimeError(f"{name} must be a CUDA tensor")
    if not t.is_contiguous():
        raise RuntimeError(f"{name} must be contiguous")


def sampleRaysUniformOccupiedVoxels(z_in_out, z_sampled, z_vals):
    """common.cu:107-125: map stratified u in [0, sum(len)] to z through the ray's packed boxes."""
    for n, t in (("z_in_out", z_in_out), ("z_sampled", z_sampled), ("z_vals", z_vals)):
        _check_input(t, n)
    if z_vals.shape != z_sampled.shape:
        raise RuntimeError("z_vals.sizes()==z_sampled.sizes()")
    for n, t in (("z_in_out", z_in_out), ("z_sampled", z_sampled), ("z_vals", z_vals)):
        if t.dtype != torch.float32:
            raise RuntimeError(f"{n}: expected scalar type Float but found {t.dtype}")
    n_rays, n_samples = z_sampled.shape
    rc = _lib.lib().nof_sample_rays_uniform_occupied_voxels(
        _lib.ptr(z_in_out), _lib.ptr(z_sampled), _lib.ptr(z_vals), int(n_rays), int(z_in_out.shape[1]),
        int(n_samples), _lib.ptr(_err_counter(z_vals.device)), _lib.stream_of(z_vals))
    _lib.check(rc, "sampleRaysUniformOccupiedVoxels")
    return z_vals


def postprocessOctreeRayTracing(ray_index, depth_in_out, unique_intersect_ray_ids, start_poss, max_intersections,
                                N_rays):
    """common.cu:151-167. Returns [N_rays, max_intersections, 2] f32 on the *input's* device
    (the reference hard-codes cuda:0, common.cu:158)."""
    for n, t in (("ray_index", ray_index), ("depth_in_out", depth_in_out), ("start_poss", start_poss)):
        _check_input(t, n)
    _check_input(unique_intersect_ray_ids, "unique_intersect_ray_ids")
    for n, t in (("ray_index", ray_index), ("unique_intersect_ray_ids", unique_intersect_ray_ids),
                 ("start_poss", start_poss)):
        if t.dtype != torch.int64:
            raise RuntimeError(f"{n}: expected scalar type Long but found {t.dtype}")
    if depth_in_out.dtype != torch.float32:
        raise RuntimeError(f"depth_in_out: expected scalar type Float but found {depth_in_out.dtype}")
    out = torch.zeros((int(N_rays), int(max_intersections), 2), dtype=torch.float32, device=depth_in_out.device)
    rc = _lib.lib().nof_postprocess_octree_ray_tracing(
        _lib.ptr(ray_index), _lib.ptr(depth_in_out), _lib.ptr(unique_intersect_ray_ids), _lib.ptr(start_poss),
        int(ray_index.shape[0]), int(unique_intersect_ray_ids.shape[0]), int(max_intersections), _lib.ptr(out),
        _lib.stream_of(out))
    _lib.check(rc, "postprocessOctreeRayTracing")
    return out


def rayColorToTextureImageCUDA(F, V, hit_locations, hit_face_ids, uvs_tex, uvs):
    """common.cu:223-238: barycentric UV per hit, written into uvs [M,2]."""
    for n, t in (("F", F), ("V", V), ("hit_locations", hit_locations), ("hit_face_ids", hit_face_ids),
                 ("uvs_tex", uvs_tex), ("uvs", uvs)):
        _check_input(t, n)
    if F.dtype != torch.int64 or hit_face_ids.dtype != torch.int64:
        raise RuntimeError("F / hit_face_ids: expected scalar type Long")
    for n, t in (("V", V), ("hit_locations", hit_locations), ("uvs_tex", uvs_tex), ("uvs", uvs)):
        if t.dtype != torch.float32:
            raise RuntimeError(f"{n}: expected scalar type Float but found {t.dtype}")
    rc = _lib.lib().nof_ray_color_to_texture_uv(
        _lib.ptr(F), _lib.ptr(V), _lib.ptr(hit_locations), _lib.ptr(hit_face_ids), _lib.ptr(uvs_tex), _lib.ptr(uvs),
        int(hit_locations.shape[0]), _lib.stream_of(uvs))
    _lib.check(rc, "rayColorToTextureImageCUDA")
