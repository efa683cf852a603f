"""Synthetic RGB-D sequence for the benchmark and tests.

Object = union of a sphere (r = 0.08 m) and a box (half extents
0.05/0.03/0.04 m, centred 0.06 m along x); procedural albedo
0.5 + 0.5 sin(20 p); cameras on a ring of radius 0.45 m looking at the
origin (azimuth 2 pi i / F, elevation 30 deg * sin(2 pi i / 16)) with a
2 mm / 1 deg jitter. Depth is the exact analytic first hit (float64).

The ray pool follows NerfRunner.make_frame_rays (nerf_runner.py:244-314)
and the scene normalisation of tool.py:28-39 + bundlesdf.py:151-153:
  sc_factor = 2 / max_extent * 0.9 * 0.7, translation = -centre.
"""
import numpy as np

H_IMG, W_IMG = 480, 640
K_CAM = np.array([[600.0, 0, 319.5], [0, 600.0, 239.5], [0, 0, 1]])
SPHERE_R = 0.08
BOX_C = np.array([0.06, 0.0, 0.0])
BOX_H = np.array([0.05, 0.03, 0.04])
GLCAM_IN_CVCAM = np.diag([1.0, -1.0, -1.0, 1.0])


def look_at(eye, target=np.zeros(3), up=np.array([0.0, 0.0, 1.0])):
    """GL camera-in-world pose (camera looks down -z)."""
    f = target - eye
    f = f / np.linalg.norm(f)
    r = np.cross(f, up)
    if np.linalg.norm(r) < 1e-8:
        r = np.cross(f, np.array([0.0, 1.0, 0.0]))
    r = r / np.linalg.norm(r)
    u = np.cross(r, f)
    T = np.eye(4)
    T[:3, 0], T[:3, 1], T[:3, 2], T[:3, 3] = r, u, -f, eye
    return T


def _rot(axis, ang):
    axis = axis / np.linalg.norm(axis)
    Kx = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    return np.eye(3) + np.sin(ang) * Kx + (1 - np.cos(ang)) * Kx @ Kx


def camera_poses(n_frames, radius=0.45, seed=0):
    rng = np.random.default_rng(seed)
    poses = []
    for i in range(n_frames):
        az = 2 * np.pi * i / n_frames
        el = np.deg2rad(30.0) * np.sin(2 * np.pi * i / 16)
        eye = radius * np.array([np.cos(az) * np.cos(el), np.sin(az) * np.cos(el), np.sin(el)])
        T = look_at(eye)
        if i > 0:
            T[:3, 3] += rng.normal(0, 0.002, 3)
            T[:3, :3] = _rot(rng.normal(size=3), np.deg2rad(rng.normal(0, 1.0))) @ T[:3, :3]
        poses.append(T)
    return np.stack(poses)


def _hit_sphere(o, d):
    b = (o * d).sum(-1)
    c = (o * o).sum(-1) - SPHERE_R ** 2
    disc = b * b - c
    t = -b - np.sqrt(np.maximum(disc, 0))
    return np.where((disc >= 0) & (t > 0), t, np.inf)


def _hit_box(o, d):
    lo, hi = BOX_C - BOX_H, BOX_C + BOX_H
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
        t1, t2 = (lo - o) * inv, (hi - o) * inv
    tn = np.nanmax(np.minimum(t1, t2), -1)
    tf = np.nanmin(np.maximum(t1, t2), -1)
    return np.where((tf >= tn) & (tn > 0), tn, np.inf)


def render_frame(glcam_in_world):
    """Returns rgb uint8 [H,W,3], depth float [H,W] (metres, 0 = no hit), mask uint8 [H,W]."""
    i, j = np.meshgrid(np.arange(W_IMG, dtype=np.float64), np.arange(H_IMG, dtype=np.float64), indexing="xy")
    dirs_cam = np.stack([(i - K_CAM[0, 2]) / K_CAM[0, 0], -(j - K_CAM[1, 2]) / K_CAM[1, 1], -np.ones_like(i)], -1)
    R, t = glcam_in_world[:3, :3], glcam_in_world[:3, 3]
    d = dirs_cam.reshape(-1, 3) @ R.T
    dn = d / np.linalg.norm(d, axis=-1, keepdims=True)
    o = np.broadcast_to(t, dn.shape)
    th = np.minimum(_hit_sphere(o, dn), _hit_box(o, dn))
    hit = np.isfinite(th)
    p = o + dn * np.where(hit, th, 0)[:, None]
    albedo = 0.5 + 0.5 * np.sin(20 * p)
    # depth along the camera axis (z-depth): t * |unit dir_cam . z|
    zc = np.abs(dirs_cam.reshape(-1, 3)[:, 2] / np.linalg.norm(dirs_cam.reshape(-1, 3), axis=-1))
    depth = np.where(hit, th * zc, 0.0).reshape(H_IMG, W_IMG)
    rgb = (np.where(hit[:, None], albedo, 0.0) * 255).round().astype(np.uint8).reshape(H_IMG, W_IMG, 3)
    return rgb, depth, hit.reshape(H_IMG, W_IMG).astype(np.uint8) * 255


def normalization():
    lo = np.minimum(-SPHERE_R * np.ones(3), BOX_C - BOX_H)
    hi = np.maximum(SPHERE_R * np.ones(3), BOX_C + BOX_H)
    center = (lo + hi) / 2
    sc = 2.0 / (hi - lo).max() * 0.9 * 0.7
    return sc, -center


def object_surface_points(n=20000, seed=0):
    """Points on the object surface (world), used as the octree build cloud."""
    rng = np.random.default_rng(seed)
    v = rng.normal(size=(n, 3))
    sph = v / np.linalg.norm(v, axis=1, keepdims=True) * SPHERE_R
    face = rng.integers(0, 6, n)
    u = rng.uniform(-1, 1, (n, 3))
    ax = face // 2
    u[np.arange(n), ax] = np.where(face % 2 == 0, -1.0, 1.0)
    box = BOX_C + u * BOX_H
    return np.concatenate([sph, box])


def make_sequence(n_frames, seed=0):
    """Frames, normalised per preprocess_data (nerf_helpers.py:218-240)."""
    sc, trans = normalization()
    poses = camera_poses(n_frames, seed=seed)
    rgbs, depths, masks = [], [], []
    for T in poses:
        rgb, depth, mask = render_frame(T)
        rgbs.append(rgb)
        depths.append(depth)
        masks.append(mask)
    rgbs = np.stack(rgbs).astype(np.float64)
    depths = np.stack(depths)
    masks = np.stack(masks)
    # preprocess_data
    depths[depths < 0.1] = 99
    rgbs[masks == 0] = 128
    depths[masks == 0] = 99
    rgbs = (rgbs / 255.0).astype(np.float32)
    depths = depths * sc
    poses_n = poses.copy()
    poses_n[:, :3, 3] += trans
    poses_n[:, :3, 3] *= sc
    pts = (object_surface_points(seed=seed) + trans) * sc
    return dict(rgbs=rgbs, depths=depths[..., None].astype(np.float32), masks=masks[..., None], poses=poses_n,
                K=K_CAM.copy(), sc_factor=float(sc), translation=trans, octree_pts=pts)


def default_cfg(**over):
    """config.yml keys used by the trainer (BASELINE config 2 overrides: L=16)."""
    cfg = dict(n_step=500, N_rand=2048, lrate=0.01, lrate_pose=0.01, decay_rate=0.1, amp=True, N_samples=128,
               N_samples_around_depth=64, N_importance=0, perturb=1, use_viewdirs=1, i_embed=1, i_embed_views=2,
               multires=8, multires_views=3, feature_grid_dim=2, finest_res=128, base_res=16, num_levels=16,
               log2_hashmap_size=22, use_octree=1, first_frame_weight=10, octree_embed_base_voxel_size=0.02,
               octree_smallest_voxel_size=0.02, octree_raytracing_voxel_size=0.02, octree_dilate_size=0.02,
               bounding_box=[[-1, -1, -1], [1, 1, 1]], use_mask=1, dilate_mask_size=0, rays_valid_depth_only=True,
               near=0.1, far=2.0, rgb_weight=10, depth_weight=0, trunc=0.01, trunc_start=0.01, sdf_lambda=5,
               neg_trunc_ratio=1, trunc_decay_type="", fs_weight=100, empty_weight=0.01, fs_rgb_weight=0,
               trunc_weight=6000, frame_features=0, optimize_poses=1, pose_reg_weight=0, eikonal_weight=0,
               feature_reg_weight=0.1, fs_sdf=0.001, max_trans=0.02, max_rot=20, down_scale_ratio=1,
               denoise_depth_use_octree_cloud=True, chunk=99999999999, netchunk=6553600, tv_loss_weight=0,
               i_print=999999, i_img=999999, i_weights=999999, i_mesh=999999, i_pose=999999,
               save_octree_clouds=False, raw_noise_std=0, white_bkgd=0, gradient_max_norm=0.1,
               gradient_pose_max_norm=0.1, N_importance_iter=1, share_coarse_fine=1, mode="sdf",
               sparse_loss_weight=0, point_cloud_loss_weight=0, point_cloud_loss_normal_weight=0,
               normal_loss_weight=0, first_frame_ray_in_batch=0, pose_optimize_start=0, no_batching=0,
               continual=True)
    cfg.update(over)
    return cfg


def frame_rays(seq, frame_id, cfg):
    """make_frame_rays (nerf_runner.py:244-314) minus the octree filter, on the
    device (ray_pool.make_pool_rays): [n,12] f32 numpy rays (dir3, rgb3, depth,
    mask, frame_id, type, near, far)."""
    from .nerf_runner import make_frame_rays
    return make_frame_rays(frame_id, seq["rgbs"], seq["depths"], seq["masks"], seq["poses"], seq["K"], cfg)


def build_pool(seq, cfg, frames=None):
    """Pool of `frames` (default all) without octree filter / denoise, built on the device."""
    from .ray_pool import make_pool_rays
    frames = range(len(seq["rgbs"])) if frames is None else frames
    return make_pool_rays(frames, seq["rgbs"], seq["depths"], seq["masks"], seq["poses"], seq["K"],
                          cfg).cpu().numpy()
