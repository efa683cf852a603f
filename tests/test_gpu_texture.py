"""GPU: texture-baking kernels (nof_raster_faces, nof_texture_hits,
nof_ray_color_to_texture_uv, nof_texture_accumulate) against oracle/texture.py
on identical inputs: z-buffer keys, hit faces / locations and the accumulated
texture exact; barycentric UVs within 1e-5 (the reference kernel's nvcc FMA
contraction is not reproduced)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _sphere_mesh():
    from bundlesdf_amd.mesh import Mesh, marching_cubes
    n = 20
    ax = np.linspace(-0.5, 0.5, n)
    X, Y, Z = np.meshgrid(ax, ax, ax, indexing="ij")
    v, f = marching_cubes(np.sqrt(X ** 2 + Y ** 2 + Z ** 2) - 0.35, 0.0)
    v = v / (n - 1) - 0.5
    return Mesh(v, f)


def _cam(eye):
    from bundlesdf_amd import synthetic as SY
    from bundlesdf_amd.handoff import GLCAM_IN_CVCAM
    return SY.look_at(np.asarray(eye, np.float64)) @ GLCAM_IN_CVCAM   # cvcam_in_ob


def test_raster_hits_accumulate_exact(cuda_device):
    from bundlesdf_amd import _lib
    from bundlesdf_amd.texture import unwrap
    from oracle import texture as TX
    mesh = unwrap(_sphere_mesh(), 256)
    H, W = 48, 64
    K = np.array([[60.0, 0, 31.5], [0, 60.0, 23.5], [0, 0, 1]])
    L = _lib.lib()
    V = torch.as_tensor(mesh.vertices.astype(np.float32), device=cuda_device)
    F = torch.as_tensor(mesh.faces, device=cuda_device)
    st = _lib.stream_of(V)
    tex_res = 256
    uvs_tex = (mesh.uv * (tex_res - 1)).astype(np.float32)
    tex_o = np.zeros((tex_res, tex_res, 3), np.float32)
    w_o = np.zeros((tex_res, tex_res), np.float32)
    tex = torch.zeros((tex_res, tex_res, 3), device=cuda_device)
    wt = torch.zeros((tex_res, tex_res), device=cuda_device)
    first = torch.full((tex_res * (tex_res - 1) + tex_res,), 0x7fffffff, dtype=torch.int32, device=cuda_device)
    rng = np.random.default_rng(0)
    for eye in ([1.2, 0.3, 0.4], [-0.4, 1.1, -0.3]):
        cam_in_ob = _cam(eye)
        ob_in_cam = np.ascontiguousarray(np.linalg.inv(cam_in_ob))
        zb = torch.empty(H * W, dtype=torch.int64, device=cuda_device)
        _lib.check(L.nof_raster_faces(_lib.ptr(V), _lib.ptr(F), len(F), ob_in_cam.ctypes.data_as(_lib._p),
                                      K.ctypes.data_as(_lib._p), H, W, 0.1, 3.0, _lib.ptr(zb), st))
        zref = TX.raster(mesh.vertices, mesh.faces, ob_in_cam, K, H, W, 0.1, 3.0)
        np.testing.assert_array_equal(zb.cpu().numpy().view(np.uint64), zref)
        assert (zref != np.iinfo(np.uint64).max).sum() > 300
        mask = (rng.uniform(size=(H, W)) > 0.1).astype(np.uint8)
        m = torch.as_tensor(mask, device=cuda_device)
        loc = torch.empty((H * W, 3), device=cuda_device)
        fid = torch.empty(H * W, dtype=torch.int64, device=cuda_device)
        c = np.ascontiguousarray(cam_in_ob)
        _lib.check(L.nof_texture_hits(_lib.ptr(zb), H, W, _lib.ptr(m), 0.1, _lib.ptr(V), _lib.ptr(F),
                                      c.ctypes.data_as(_lib._p), K.ctypes.data_as(_lib._p), _lib.ptr(loc),
                                      _lib.ptr(fid), st))
        lref, fref = TX.hits(zref, H, W, mask, 0.1, mesh.vertices, mesh.faces, cam_in_ob, K)
        np.testing.assert_array_equal(fid.cpu().numpy(), fref)
        np.testing.assert_array_equal(loc.cpu().numpy()[fref >= 0], lref[fref >= 0])
        pix = np.nonzero(fref >= 0)[0]
        ut = torch.as_tensor(uvs_tex, device=cuda_device)
        hl = loc[torch.as_tensor(pix, device=cuda_device)].contiguous()
        hf = fid[torch.as_tensor(pix, device=cuda_device)].contiguous()
        uvs = torch.empty((len(pix), 2), device=cuda_device)
        _lib.check(L.nof_ray_color_to_texture_uv(_lib.ptr(F), _lib.ptr(V), _lib.ptr(hl), _lib.ptr(hf), _lib.ptr(ut),
                                                 _lib.ptr(uvs), len(pix), st))
        uref = TX.texture_uv(mesh.faces, mesh.vertices.astype(np.float32), lref[pix], fref[pix], uvs_tex)
        np.testing.assert_allclose(uvs.cpu().numpy(), uref, rtol=1e-5, atol=1e-4)
        colors = rng.uniform(0, 255, (H * W, 3)).astype(np.float32)
        col = torch.as_tensor(colors, device=cuda_device)
        p32 = torch.as_tensor(pix.astype(np.int32), device=cuda_device)
        _lib.check(L.nof_texture_accumulate(_lib.ptr(uvs), _lib.ptr(p32), len(pix), _lib.ptr(col), tex_res, tex_res,
                                            _lib.ptr(first), _lib.ptr(tex), _lib.ptr(wt), st))
        TX.accumulate(uvs.cpu().numpy(), pix, colors, tex_o, w_o)
    np.testing.assert_array_equal(tex.cpu().numpy(), tex_o)
    np.testing.assert_array_equal(wt.cpu().numpy(), w_o)
    assert (first.cpu().numpy() == 0x7fffffff).all()
    assert w_o.sum() > 300


def test_unwrap_atlas():
    from bundlesdf_amd.texture import unwrap
    mesh = unwrap(_sphere_mesh(), 512)
    assert mesh.uv.min() >= 0 and mesh.uv.max() <= 1
    # every face's UV triangle is non-degenerate and faces do not share texels' centres
    t = mesh.uv[mesh.faces]
    area = (t[:, 1, 0] - t[:, 0, 0]) * (t[:, 2, 1] - t[:, 0, 1]) - (t[:, 2, 0] - t[:, 0, 0]) * (t[:, 1, 1] - t[:, 0, 1])
    assert (np.abs(area) > 0).all()
