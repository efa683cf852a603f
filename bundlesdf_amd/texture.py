"""Texture baking from the training images:
NerfRunner.mesh_texture_from_train_images (nerf_runner.py:1467-1541) on the
device.

Per training frame the reference renders the mesh's depth with pyrender,
back-projects the masked pixels, snaps them to the mesh
(trimesh.proximity.closest_point), converts the hits to texel coordinates with
common.rayColorToTextureImageCUDA and adds each texel's first colour. Here the
frame loop is four launches on one stream: nof_raster_faces (depth + face-id
z-buffer), nof_texture_hits (back-projection + closest point on the seen
face), nof_ray_color_to_texture_uv (the B1 boundary op, barycentric UV) and
nof_texture_accumulate (first hit per texel, the reference's (W-1) row
stride); the texture and weights stay in HBM until the final divide.

UV atlas: the reference calls mesh.unwrap() (xatlas, not installed). unwrap()
below is a deterministic per-face atlas — faces in pairs, each pair a grid
cell split along its diagonal, an inset of about one texel — so parity with
xatlas' charts is out of reach (PARITY UNPINNED for the atlas); everything
after the UVs is checked against oracle/texture.py on identical UVs.
"""
import numpy as np
import torch

from . import _lib
from .handoff import GLCAM_IN_CVCAM
from .mesh import Mesh


def unwrap(mesh, tex_res=1024):
    """Per-face atlas -> new Mesh (3 vertices per face, faces = arange) with .uv [3F,2] in [0,1]."""
    F = np.asarray(mesh.faces, np.int64)
    nF = len(F)
    cells = max(1, (nF + 1) // 2)
    g = int(np.ceil(np.sqrt(cells)))
    texel = g / max(tex_res - 1, 1)                    # one texel in cell-local units
    e = min(0.2, 1.0 * texel)
    d = min(0.2, 2.0 * texel)
    lower = np.array([[e, e], [1 - e - d, e], [e, 1 - e - d]])
    upper = np.array([[1 - e, 1 - e], [e + d, 1 - e], [1 - e, e + d]])
    f = np.arange(nF)
    c = f // 2
    org = np.stack([c % g, c // g], -1).astype(np.float64)
    local = np.where((f % 2 == 0)[:, None, None], lower[None], upper[None])
    uv = ((org[:, None, :] + local) / g).reshape(-1, 2)
    out = Mesh(np.asarray(mesh.vertices, np.float64)[F].reshape(-1, 3), np.arange(3 * nF).reshape(nF, 3))
    out.uv = uv
    return out


def bake_texture(mesh, rgbs_raw, masks, cvcam_in_obs, K, H, W, min_depth, zfar, tex_res=1024, device=None):
    """Texture of `mesh` (with .uv) from the frames: rgbs_raw [N,H,W,3] (raw colour
    values), masks [N,H,W(,1)], cvcam_in_obs [N,4,4] (OpenCV camera in object),
    K [3,3]. Returns the uint8 image [tex_res, tex_res, 3] (rows flipped, as the
    reference stores it)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    L = _lib.lib()
    V = torch.as_tensor(np.asarray(mesh.vertices, np.float32), device=dev).contiguous()
    Fc = torch.as_tensor(np.asarray(mesh.faces, np.int64), device=dev).contiguous()
    uvs_tex = torch.as_tensor((np.asarray(mesh.uv) * np.array([tex_res - 1, tex_res - 1]).reshape(1, 2))
                              .astype(np.float32), device=dev).contiguous()
    Kd = np.ascontiguousarray(np.asarray(K, np.float64))
    tex = torch.zeros((tex_res, tex_res, 3), dtype=torch.float32, device=dev)
    wtex = torch.zeros((tex_res, tex_res), dtype=torch.float32, device=dev)
    first = torch.full((tex_res * (tex_res - 1) + tex_res,), 0x7fffffff, dtype=torch.int32, device=dev)
    zbuf = torch.empty(H * W, dtype=torch.int64, device=dev)
    loc = torch.empty((H * W, 3), dtype=torch.float32, device=dev)
    fid = torch.empty(H * W, dtype=torch.int64, device=dev)
    st = _lib.stream_of(V)
    for i in range(len(rgbs_raw)):
        cam_in_ob = np.ascontiguousarray(np.asarray(cvcam_in_obs[i], np.float64))
        ob_in_cam = np.ascontiguousarray(np.linalg.inv(cam_in_ob))
        _lib.check(L.nof_raster_faces(_lib.ptr(V), _lib.ptr(Fc), len(Fc), ob_in_cam.ctypes.data_as(_lib._p),
                                      Kd.ctypes.data_as(_lib._p), H, W, 0.1, float(zfar), _lib.ptr(zbuf), st),
                   "raster_faces")
        m = torch.as_tensor(np.asarray(masks[i]).reshape(H, W).astype(bool).astype(np.uint8), device=dev)
        _lib.check(L.nof_texture_hits(_lib.ptr(zbuf), H, W, _lib.ptr(m), float(min_depth), _lib.ptr(V), _lib.ptr(Fc),
                                      cam_in_ob.ctypes.data_as(_lib._p), Kd.ctypes.data_as(_lib._p), _lib.ptr(loc),
                                      _lib.ptr(fid), st), "texture_hits")
        pix = torch.nonzero(fid >= 0).reshape(-1)
        M = len(pix)
        if M == 0:
            continue
        hl = loc[pix].contiguous()
        hf = fid[pix].contiguous()
        uvs = torch.empty((M, 2), dtype=torch.float32, device=dev)
        _lib.check(L.nof_ray_color_to_texture_uv(_lib.ptr(Fc), _lib.ptr(V), _lib.ptr(hl), _lib.ptr(hf),
                                                 _lib.ptr(uvs_tex), _lib.ptr(uvs), M, st), "ray_color_to_texture_uv")
        img = torch.as_tensor(np.asarray(rgbs_raw[i], np.float32).reshape(H * W, 3), device=dev).contiguous()
        pix32 = pix.to(torch.int32).contiguous()
        _lib.check(L.nof_texture_accumulate(_lib.ptr(uvs), _lib.ptr(pix32), M, _lib.ptr(img), tex_res, tex_res,
                                            _lib.ptr(first), _lib.ptr(tex), _lib.ptr(wtex), st), "texture_accumulate")
    out = tex / wtex[..., None]
    out = torch.nan_to_num(out, nan=0.0).clamp(0, 255).to(torch.uint8)   # 0/0 texels: 0
    return out.flip(0).cpu().numpy()


def mesh_texture_from_train_images(runner, mesh, rgbs_raw, train_texture=False, tex_res=1024):
    """nerf_runner.py:1467-1541 for a NerfRunner: poses with the learned corrections,
    merge/dedupe, unwrap, bake; returns the unwrapped mesh with .uv and .texture."""
    if train_texture:
        raise NotImplementedError("mesh_texture_from_train_images: train_texture=True is not implemented")
    assert len(runner.images) == len(rgbs_raw)
    dev = runner.device
    ids = torch.arange(len(runner.images), device=dev)
    with torch.no_grad():
        tf = runner.c2w_array[ids]
        if runner.models["pose_array"] is not None:
            tf = runner.models["pose_array"].get_matrices(ids) @ tf
    tf = tf.cpu().numpy()
    cvcam_in_obs = np.stack([tf[i] @ np.linalg.inv(GLCAM_IN_CVCAM) for i in range(len(tf))])
    mesh.merge_vertices()
    mesh.remove_duplicate_faces()
    mesh = unwrap(mesh, tex_res)
    sc = runner.cfg["sc_factor"]
    mesh.texture = bake_texture(mesh, rgbs_raw, runner.masks, cvcam_in_obs, runner.K, runner.H, runner.W,
                                0.1 * sc, runner.cfg["far"] * sc, tex_res, dev)
    return mesh
