"""ORACLE — test infrastructure only (tests/). CPU restatement of the texture
baking path (checker for bundlesdf_amd.texture):

  texture_uv     rayColorToTextureImageKernel + calculateBarycentricCoordinate3D
                 (common.cu:168-219), float32, no contraction (nvcc's default FMA
                 contraction of the reference is not reproduced: PARITY UNPINNED
                 at the last bit; tests compare with a tolerance)
  raster         the depth pass the reference gets from pyrender
                 (offscreen_renderer.py:39-45, nerf_runner.py:1502-1505) as a
                 z-buffer over integer pixel centres, f64, ties to the smaller
                 (depth, face) — PARITY UNPINNED (pyrender is not installed)
  hits           depth2xyzmap (Utils.py:219-231) + cam->object + closest point
                 on the seen face (trimesh.proximity.closest_point, :1510)
  accumulate     nerf_runner.py:1524-1535 (round-half-even texel, (W-1) row
                 stride, first hit per texel adds colour and weight 1)
Written to mirror the device arithmetic operation by operation so the
z-buffer, faces and texture compare exactly on identical inputs.
"""
import numpy as np


def texture_uv(F, V, hits, face_ids, uvs_tex):
    F = np.asarray(F, np.int64)
    V = np.asarray(V, np.float32)
    out = np.zeros((len(hits), 2), np.float32)
    f32 = np.float32
    for i in range(len(hits)):
        f = F[face_ids[i]]
        v = V[f]
        p = np.asarray(hits[i], np.float32)

        def cross(a, b):
            return np.array([a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]],
                            np.float32)

        def dot(a, b):
            return f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2])
        n = cross(v[1] - v[2], v[1] - v[0])
        abc = dot(n, cross(v[1] - v[0], v[2] - v[0]))
        pbc = dot(n, cross(v[1] - p, v[2] - p))
        pca = dot(n, cross(v[2] - p, v[0] - p))
        w0, w1 = f32(pbc / abc), f32(pca / abc)
        w2 = f32(f32(f32(1) - w0) - w1)
        for j in range(2):
            t = uvs_tex[f, j].astype(np.float32)
            out[i, j] = f32(f32(f32(t[0] * w0) + f32(t[1] * w1)) + f32(t[2] * w2))
    return out


def raster(V, F, ob_in_cam, K, H, W, znear, zfar):
    """-> uint64 keys [H*W] (f32 depth bits << 32 | face), all ones where empty."""
    zbuf = np.full(H * W, np.iinfo(np.uint64).max, np.uint64)
    R, t = np.asarray(ob_in_cam, np.float64)[:3, :3], np.asarray(ob_in_cam, np.float64)[:3, 3]
    fx, fy, cx, cy = K[0, 0], K[1, 1], K[0, 2], K[1, 2]
    V = np.asarray(V, np.float32).astype(np.float64)
    for f in range(len(F)):
        u, v, z = np.zeros(3), np.zeros(3), np.zeros(3)
        ok = True
        for k in range(3):
            x, y, w = V[F[f, k]]
            X = ((R[0, 0] * x + R[0, 1] * y) + R[0, 2] * w) + t[0]
            Y = ((R[1, 0] * x + R[1, 1] * y) + R[1, 2] * w) + t[1]
            Z = ((R[2, 0] * x + R[2, 1] * y) + R[2, 2] * w) + t[2]
            if not Z > znear:
                ok = False
                break
            z[k], u[k], v[k] = Z, fx * X / Z + cx, fy * Y / Z + cy
        if not ok:
            continue
        area = (u[1] - u[0]) * (v[2] - v[0]) - (u[2] - u[0]) * (v[1] - v[0])
        if area == 0.0:
            continue
        u0, u1 = max(0, int(np.ceil(u.min()))), min(W - 1, int(np.floor(u.max())))
        v0, v1 = max(0, int(np.ceil(v.min()))), min(H - 1, int(np.floor(v.max())))
        for py in range(v0, v1 + 1):
            for px in range(u0, u1 + 1):
                X, Y = float(px), float(py)
                e0 = ((u[2] - u[1]) * (Y - v[1]) - (v[2] - v[1]) * (X - u[1])) / area
                e1 = ((u[0] - u[2]) * (Y - v[2]) - (v[0] - v[2]) * (X - u[2])) / area
                e2 = ((u[1] - u[0]) * (Y - v[0]) - (v[1] - v[0]) * (X - u[0])) / area
                if e0 < 0 or e1 < 0 or e2 < 0:
                    continue
                zi = 1.0 / ((e0 / z[0] + e1 / z[1]) + e2 / z[2])
                if not zi <= zfar:
                    continue
                key = (np.uint64(np.float32(zi).view(np.uint32)) << np.uint64(32)) | np.uint64(f)
                i = py * W + px
                if key < zbuf[i]:
                    zbuf[i] = key
    return zbuf


def _closest_on_tri(p, a, b, c):
    ab, ac, ap = b - a, c - a, p - a

    def dot(x, y):
        return (x[0] * y[0] + x[1] * y[1]) + x[2] * y[2]
    d1, d2 = dot(ab, ap), dot(ac, ap)
    if d1 <= 0 and d2 <= 0:
        return a.copy()
    bp = p - b
    d3, d4 = dot(ab, bp), dot(ac, bp)
    if d3 >= 0 and d4 <= d3:
        return b.copy()
    vc = d1 * d4 - d3 * d2
    if vc <= 0 and d1 >= 0 and d3 <= 0:
        return a + (d1 / (d1 - d3)) * ab
    cp = p - c
    d5, d6 = dot(ab, cp), dot(ac, cp)
    if d6 >= 0 and d5 <= d6:
        return c.copy()
    vb = d5 * d2 - d1 * d6
    if vb <= 0 and d2 >= 0 and d6 <= 0:
        return a + (d2 / (d2 - d6)) * ac
    va = d3 * d6 - d5 * d4
    if va <= 0 and (d4 - d3) >= 0 and (d5 - d6) >= 0:
        return b + ((d4 - d3) / ((d4 - d3) + (d5 - d6))) * (c - b)
    den = 1.0 / ((va + vb) + vc)
    return (a + ab * (vb * den)) + ac * (vc * den)


def hits(zbuf, H, W, mask, min_depth, V, F, cam_in_ob, K):
    """-> (locations [H*W,3] f32, face ids [H*W] i64, -1 = none)."""
    loc = np.zeros((H * W, 3), np.float32)
    face = np.full(H * W, -1, np.int64)
    T = np.asarray(cam_in_ob, np.float64)
    V = np.asarray(V, np.float32).astype(np.float64)
    mask = np.asarray(mask).reshape(-1)
    for i in np.nonzero(zbuf != np.iinfo(np.uint64).max)[0]:
        if not mask[i]:
            continue
        key = int(zbuf[i])
        z = np.uint32(key >> 32).view(np.float32)
        if not z >= np.float32(min_depth):
            continue
        f = key & 0xffffffff
        py, px = divmod(int(i), W)
        xc = np.float32((float(px) - K[0, 2]) * float(z) / K[0, 0])
        yc = np.float32((float(py) - K[1, 2]) * float(z) / K[1, 1])
        pc = np.array([xc, yc, z], np.float64)
        p = np.array([((T[k, 0] * pc[0] + T[k, 1] * pc[1]) + T[k, 2] * pc[2]) + T[k, 3] for k in range(3)])
        q = _closest_on_tri(p, V[F[f, 0]], V[F[f, 1]], V[F[f, 2]])
        loc[i] = q.astype(np.float32)
        face[i] = f
    return loc, face


def accumulate(uvs, pix, colors, tex, wtex):
    """In place: first hit per texel (pixel order) adds its colour and weight 1."""
    TH, TW = wtex.shape
    x = np.rint(uvs[:, 0]).astype(np.int64)
    y = np.rint(uvs[:, 1]).astype(np.int64)
    flat = y * (TW - 1) + x
    seen = set()
    for k in range(len(flat)):
        fl = int(flat[k])
        if fl in seen or fl < 0 or fl >= TH * (TW - 1) + TW:
            continue
        seen.add(fl)
        ux, uy = fl % (TW - 1), fl // (TW - 1)
        if uy >= TH:
            continue
        tex[uy, ux] += colors[pix[k]]
        wtex[uy, ux] += 1.0
