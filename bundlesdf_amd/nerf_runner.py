"""Drop-in for the reference trainer API used by bundlesdf.py:
NerfRunner(cfg, images, depths, masks, normal_maps, poses, K, ...) with
add_new_frames / train / models / cfg, plus the module-level helpers that
`from nerf_runner import *` brings into bundlesdf.py (preprocess_data & co.).

Behaviour follows nerf_runner.py:110-233 (constructor), :244-314
(make_frame_rays), :350-431 (add_new_frames), :434-487 (build_octree),
:490-502 (optimiser), :854-862 (train). The training step itself is the
MI355X fused path (bundlesdf_amd.fused.FusedStep: HIP trace + sampling +
encode + MFMA MLP + losses + backward + Adam/GradScaler), which replaces
train_loop (:577-762) on identical batches.

MI355X-first differences (documented in DESIGN.md):
  * the ray pool is built on the device (ray_pool.make_pool_rays: dilation,
    box/octree filters and the denoise radius test in HIP kernels, reference
    row order) and stays resident in HBM; DataLoader draws each epoch's
    torch.randperm on the CPU generator exactly as the reference does (index
    parity, :90-107) and hands the trainer device ids (the reference gathers
    the rows on the host and copies them);
  * the octree is the dense occupancy grid of bundlesdf_amd.octree;
  * normal maps are kept (self.normal_maps) but, as in the reference's
    default config (normal_loss_weight 0), not used by the loss; the pool is
    always stored in the 12-column layout the kernels read.
Configurations the fused path does not implement raise NotImplementedError
(frame_features > 3, N_importance > 0, i_embed != 1, non-SH view encoding,
and the loss branches that are dead in the reference: depth_weight > 0,
eikonal_weight > 0). fs_rgb_weight and the trunc_decay_type schedules run on
the device.
extract_mesh runs the fused SDF query kernel + device marching cubes
(bundlesdf_amd/mesh.py); mesh_texture_from_train_images bakes on the device
(bundlesdf_amd/texture.py)."""
import logging
import random

import numpy as np
import torch

from .fused import FusedStep, truncation
from .nerf_helpers import (BAD_COLOR, FeatureArray, NeRFSmall, PoseArray, SHEncoder,  # noqa: F401
                           get_camera_rays_np, get_embedder, preprocess_data, to8b)
from .octree import OctreeManager
from .ray_pool import PointGrid, make_pool_rays

BAD_DEPTH = 99

__all__ = ["NerfRunner", "DataLoader", "make_frame_rays", "compute_near_far_and_filter_rays", "BAD_DEPTH",
           "BAD_COLOR", "preprocess_data", "get_camera_rays_np", "get_embedder", "NeRFSmall", "PoseArray",
           "FeatureArray", "SHEncoder", "to8b"]


def set_seed(seed):
    """Utils.py:71-78: python, numpy and torch (CPU + every device) generators."""
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)


def _box_entry_exit(origins, dirs, bounds):
    """Slab test of rays against the axis-aligned box bounds [2,3] in float64 with
    the reference's conventions (ray_box_intersection_batch, nerf_helpers.py:403-446):
    unit directions (+1e-10), each axis' entry parameter clamped at 0 before it is
    combined, misses reported as (-1, -1)."""
    d = dirs / (np.linalg.norm(dirs, axis=-1, keepdims=True) + 1e-10)
    with np.errstate(divide="ignore", invalid="ignore"):
        inv = 1.0 / d
    neg = inv < 0
    t_in = np.where(neg, bounds[1], bounds[0]) - origins
    t_out = np.where(neg, bounds[0], bounds[1]) - origins
    with np.errstate(invalid="ignore"):
        t_in, t_out = t_in * inv, t_out * inv
    t_in = np.where(t_in < 0, 0.0, t_in)
    lo, hi = t_in[:, 0].copy(), t_out[:, 0].copy()
    hit = np.ones(len(d), bool)
    for ax in (1, 2):
        a_in, a_out = t_in[:, ax], t_out[:, ax]
        hit &= ~((lo > a_out) | (a_in > hi))
        lo = np.where(a_in > lo, a_in, lo)
        hi = np.where(a_out < hi, a_out, hi)
    lo[~hit] = -1
    hi[~hit] = -1
    return lo, hi


def compute_near_far_and_filter_rays(cam_in_world, rays, cfg):
    """nerf_runner.py:39-65 (host utility, re-exported for bundlesdf.py): rays in the
    camera frame [..., D] hit-tested against cfg['bounding_box'] from the camera
    centre; the hits come back as [n, D+2] with |near|, |far| in camera-z units.
    The training pool does not use this function: it is built on the device by
    ray_pool.make_pool_rays."""
    rays = np.asarray(rays)
    rays = rays.reshape(-1, rays.shape[-1])
    T = np.asarray(cam_in_world, np.float64)
    du = rays[:, :3] / np.linalg.norm(rays[:, :3], axis=-1, keepdims=True)
    dirs = rays[:, :3].astype(np.float64) @ T[:3, :3].T
    origins = np.broadcast_to(T[:3, 3], dirs.shape)
    bounds = np.asarray(cfg.get("bounding_box", [[-1, -1, -1], [1, 1, 1]]), np.float64).reshape(2, 3)
    tmin, tmax = _box_entry_exit(origins, dirs, bounds)
    hit = tmin >= 0
    near = np.abs(du[:, 2] * tmin)[hit]
    far = np.abs(du[:, 2] * tmax)[hit]
    return np.concatenate([rays[hit], near[:, None], far[:, None]], -1)


def make_frame_rays(frame_id, images, depths, masks, poses, K, cfg, occ_masks=None, octree_m=None):
    """nerf_runner.py:244-314 for one frame -> [n,12] f32 numpy rays: dir(0-2, GL
    camera frame, unnormalised), rgb(3-5), depth(6), mask(7), frame_id(8), type(9),
    near(10), far(11). Runs the device pool builder (ray_pool.make_pool_rays):
    mask dilation (100 px for frame 0, 60/down_scale otherwise), occluded pixels
    removed, type-0 rays only, box near/far filter, octree filter when octree_m
    is given (trace at octree_raytracing_voxel_size must hit something)."""
    occ = None
    if octree_m is not None:
        sc = cfg["sc_factor"]
        occ = octree_m.occupancy(int(np.floor(np.log2(2.0 / (cfg["octree_raytracing_voxel_size"] * sc)))))
    dev = occ.device if occ is not None else None
    r = make_pool_rays([frame_id], images, depths, masks, poses, K, cfg, occ_masks=occ_masks, occ=occ, device=dev)
    return r.cpu().numpy()


class DataLoader:
    """nerf_runner.py:90-107: epoch permutation over the pool, consecutive slices of
    batch_size ids, reshuffle when a slice would run past the end. The permutation is
    the reference's own draw — torch.randperm on the CPU default generator, which
    set_seed seeds (so the batches are the reference's, index for index) — copied to
    the device once per epoch as int32 ids; the pool stays resident in HBM and only
    ids are produced (no host gather, no per-step H2D copy)."""

    def __init__(self, rays, batch_size):
        self.rays = rays
        self.batch_size = batch_size
        self.pos = 0
        self._pinned = None
        self._dev_perm = None
        self.ids = self._perm()

    def _perm(self):
        """The epoch's draw (the reference's randperm on the CPU generator), narrowed to int32 on
        the host and copied through a persistent pinned buffer without blocking the host: the
        copy is ordered on the current stream before every later step's use of the ids, and the
        buffer is rewritten only at the next epoch wrap (a whole epoch of steps later; the host
        waits for the previous copy first)."""
        perm = torch.randperm(len(self.rays)).to(torch.int32)
        dev = self.rays.device
        if dev.type != "cuda":
            return perm.to(dev)
        if self._pinned is None or self._pinned.numel() != perm.numel():
            self._pinned = torch.empty(perm.numel(), dtype=torch.int32).pin_memory()
            self._copied = None
        if self._copied is not None:
            self._copied.synchronize()
        self._pinned.copy_(perm)
        # one device buffer for every epoch (stream order puts the rewrite after every step already
        # enqueued on the old permutation): a captured step can read its slice from it by address
        if self._dev_perm is None or self._dev_perm.numel() != perm.numel():
            self._dev_perm = torch.empty(perm.numel(), dtype=torch.int32, device=dev)
        self._dev_perm.copy_(self._pinned, non_blocking=True)
        self._copied = torch.cuda.Event()
        self._copied.record()
        return self._dev_perm

    def next_ids(self):
        if self.pos + self.batch_size < len(self.ids):
            out = self.ids[self.pos:self.pos + self.batch_size]
            self.pos += self.batch_size
            return out
        self.ids = self._perm()
        self.pos = self.batch_size
        return self.ids[:self.batch_size]

    def next_slice(self):
        """next_ids() for a captured step that reads its slice on the device
        (FusedStep.graph_step_epoch): returns (the epoch permutation buffer, the slice's index k);
        the slice itself is ids[k batch_size : (k + 1) batch_size]."""
        self.next_ids()
        return self.ids, self.pos // self.batch_size - 1

    def __next__(self):
        self.batch_ray_ids = self.next_ids().long()
        return self.rays[self.batch_ray_ids]


def _check_supported(cfg):
    if cfg.get("frame_features", 0) > 3:
        raise NotImplementedError("fused MI355X path: frame_features <= 3 (global refine uses 2)")
    if cfg.get("N_importance", 0) > 0:
        raise NotImplementedError("fused MI355X path: N_importance > 0 (fine network) is not implemented")
    if cfg.get("i_embed", 1) != 1 or cfg.get("i_embed_views", 2) != 2 or not cfg.get("use_viewdirs", 1):
        raise NotImplementedError("fused MI355X path: hash-grid positions + SH view directions only")
    if cfg.get("feature_grid_dim", 2) != 2 or cfg.get("num_levels", 16) > 16:
        raise NotImplementedError("fused MI355X path: level_dim 2 and at most 16 levels")
    if not cfg.get("use_octree", 1):
        raise NotImplementedError("fused MI355X path: octree-guided sampling only (use_octree=1)")
    if cfg.get("finest_res", 512) > 1023:
        # k_scatter's run keys hold 10 bits per cell coordinate (field_step.hip; FusedStep checks the
        # level table itself too): the reference's configs stop at 512
        raise NotImplementedError("fused MI355X path: finest_res <= 1023")
    # loss branches of train_loop (:687-751) that are dead in the reference itself
    if cfg.get("depth_weight", 0) > 0:
        raise NotImplementedError("depth_weight > 0: train_loop :711-719 reads an undefined `depth` in the reference "
                                  "(NameError there); not implemented")
    if cfg.get("eikonal_weight", 0) > 0:
        raise NotImplementedError("eikonal_weight > 0: train_loop renders with get_normals=False (:685), so "
                                  "extras['normals'] (:733-737) does not exist in the reference; not implemented")
    if (cfg.get("trunc_decay_type", "") or "") not in ("", "linear", "exp"):
        raise NotImplementedError(f"trunc_decay_type {cfg['trunc_decay_type']!r}")
    if cfg.get("mode", "sdf") != "sdf":
        raise NotImplementedError("fused MI355X path: mode 'sdf' only")


class NerfRunner:
    def __init__(self, cfg, images, depths, masks, normal_maps, poses, K, _run=None, occ_masks=None,
                 build_octree_pcd=None, device=None):
        set_seed(0)
        _check_supported(cfg)
        self.cfg = cfg
        self.cfg["tv_loss_weight"] = float(eval(str(self.cfg.get("tv_loss_weight", 0)), {}, {}))
        self._run = _run
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.K = np.asarray(K, np.float64).copy()
        self.images, self.depths, self.masks = images, depths, masks
        self.normal_maps, self.occ_masks = normal_maps, occ_masks
        self.poses = np.asarray(poses)
        self.mesh = None
        self.train_pose = False
        self.N_iters = self.cfg["n_step"] + 1
        pts = build_octree_pcd.points if hasattr(build_octree_pcd, "points") else build_octree_pcd
        self.build_octree_pts = np.asarray(pts, np.float64).copy()
        r = int(cfg["down_scale_ratio"])
        self.down_scale = np.ones(2, dtype=np.float32)
        if r != 1:
            H, W = images[0].shape[:2]
            self.images, self.depths, self.masks = images[:, ::r, ::r], depths[:, ::r, ::r], masks[:, ::r, ::r]
            if normal_maps is not None:
                self.normal_maps = normal_maps[:, ::r, ::r]
            if occ_masks is not None:
                self.occ_masks = occ_masks[:, ::r, ::r]
            h, w = self.images.shape[1:3]
            self.cfg["dilate_mask_size"] = int(self.cfg.get("dilate_mask_size", 0) // r)
            self.K[0] *= float(w) / W
            self.K[1] *= float(h) / H
            self.down_scale = np.array([float(w) / W, float(h) / H])
        self.H, self.W = self.images[0].shape[:2]
        self.octree_m = None
        if self.cfg["use_octree"]:
            self.build_octree()
        self.create_nerf()
        self.global_step = 0
        self.c2w_array = torch.as_tensor(self.poses, dtype=torch.float32, device=self.device)
        self.best_models, self.best_loss = None, np.inf
        self.rays = self._pool_rays(range(len(self.masks)))
        logging.info(f"rays {tuple(self.rays.shape)}")
        self._new_trainer()

    # ------------------------------------------------------------ pieces
    def _pool_rays(self, frames):
        """make_frame_rays over `frames` + the octree-cloud denoise (nerf_runner.py:
        170-194, :401-423), built on the device: [n,12] f32 rays in HBM."""
        frames = list(frames)
        if not frames:
            return torch.empty((0, 12), dtype=torch.float32, device=self.device)
        occ = self._occ_trace_level() if self.octree_m is not None else None
        grid = None
        if self.cfg["denoise_depth_use_octree_cloud"]:
            grid = PointGrid(self.build_octree_pts, 0.02 * self.cfg["sc_factor"], self.device)
        rays = make_pool_rays(frames, self.images, self.depths, self.masks, self.poses, self.K, self.cfg,
                              occ_masks=self.occ_masks, occ=occ, point_grid=grid, device=self.device)
        logging.info(f"pool rays of frames {frames[0]}..{frames[-1]}: {len(rays)}")
        return rays

    def make_frame_rays(self, frame_id):
        """Reference method form (nerf_runner.py:244): numpy rays of one frame."""
        return make_frame_rays(frame_id, self.images, self.depths, self.masks, self.poses, self.K, self.cfg,
                               self.occ_masks, self.octree_m)

    def build_octree(self):
        """nerf_runner.py:434-474: finest level from octree_smallest_voxel_size,
        dilation radius ceil(octree_dilate_size / smallest voxel)."""
        sc = self.cfg["sc_factor"]
        max_level = int(np.ceil(np.log2(2.0 / (self.cfg["octree_smallest_voxel_size"] * sc))))
        dil = max(1, int(np.ceil(self.cfg["octree_dilate_size"] / self.cfg["octree_smallest_voxel_size"])))
        pts = torch.as_tensor(self.build_octree_pts, dtype=torch.float32, device=self.device)
        self.octree_m = OctreeManager(pts, max_level, dilate_radius=dil)

    def create_nerf(self):
        """nerf_runner.py:204-242. The modules are initialised on the CPU default generator
        in the reference's order (GridEncoder table, NeRFSmall layers, FeatureArray) and then
        moved to the device, so under set_seed(0) the initial parameters are the reference's
        bit for bit (tests/golden/runner_seed.npz)."""
        cfg = self.cfg
        models = {}
        embed_fn, input_ch = get_embedder(cfg["multires"], cfg, i=cfg["i_embed"], octree_m=self.octree_m)
        models["embed_fn"] = embed_fn.to(self.device)
        embeddirs_fn, input_ch_views = get_embedder(cfg["multires_views"], cfg, i=cfg["i_embed_views"],
                                                    octree_m=self.octree_m)
        models["embeddirs_fn"] = embeddirs_fn
        models["model"] = NeRFSmall(num_layers=2, hidden_dim=64, geo_feat_dim=15, num_layers_color=3,
                                    hidden_dim_color=64, input_ch=input_ch,
                                    input_ch_views=input_ch_views + cfg.get("frame_features", 0)).to(self.device)
        models["model_fine"] = None
        models["feature_array"] = (FeatureArray(len(self.images), cfg["frame_features"]).to(self.device)
                                   if cfg.get("frame_features", 0) > 0 else None)
        models["pose_array"] = PoseArray(len(self.images), max_trans=cfg["max_trans"] * cfg["sc_factor"],
                                         max_rot=cfg["max_rot"]).to(self.device) if cfg["optimize_poses"] else None
        self.models = models

    def _occ_trace_level(self):
        sc = self.cfg["sc_factor"]
        level = int(np.floor(np.log2(2.0 / (self.cfg["octree_raytracing_voxel_size"] * sc))))
        return self.octree_m.occupancy(level)

    def _new_trainer(self):
        """create_optimizer (:490-502) + GradScaler (:159): the fused trainer owns the
        flat parameter / Adam / scaler state; module parameters become views of it."""
        if self.models["pose_array"] is None:
            # frozen poses: a PoseArray at zero with lrate_pose 0 is the identity correction
            self.models["pose_array"] = PoseArray(len(self.images), self.cfg["max_trans"] * self.cfg["sc_factor"],
                                                  self.cfg["max_rot"]).to(self.device)
            self.cfg["lrate_pose"] = 0.0
        self.trainer = FusedStep(self.cfg, self.rays, self.c2w_array, self._occ_trace_level(),
                                 self.models["embed_fn"], self.models["model"], self.models["pose_array"],
                                 amp=bool(self.cfg["amp"]), feature_array=self.models["feature_array"])
        self.data_loader = DataLoader(self.rays, self.cfg["N_rand"])
        self.optimizer = self.trainer          # step/state owner (Adam + GradScaler on device)
        self.amp_scaler = self.trainer

    # ------------------------------------------------------------ API
    def add_new_frames(self, images, depths, masks, normal_maps, poses, occ_masks=None, new_pcd=None,
                       reuse_weights=False):
        """nerf_runner.py:350-431: append frames, reset poses for all frames,
        rebuild the octree from the new cloud, recreate (or keep) the networks,
        new optimiser state, add the new frames' rays to the pool."""
        prev = len(self.images)
        r = int(self.cfg["down_scale_ratio"])
        images, depths, masks = images[:, ::r, ::r], depths[:, ::r, ::r], masks[:, ::r, ::r]
        if normal_maps is not None and self.normal_maps is not None:
            self.normal_maps = np.concatenate((self.normal_maps, normal_maps[:, ::r, ::r]), 0)
        if occ_masks is not None:
            occ = occ_masks[:, ::r, ::r]
            self.occ_masks = occ if self.occ_masks is None else np.concatenate((self.occ_masks, occ), 0)
        self.images = np.concatenate((self.images, images), 0)
        self.depths = np.concatenate((self.depths, depths), 0)
        self.masks = np.concatenate((self.masks, masks), 0)
        self.poses = np.asarray(poses).copy()
        self.c2w_array = torch.as_tensor(self.poses, dtype=torch.float32, device=self.device)
        if self.cfg["use_octree"] and new_pcd is not None:
            # pcd.voxel_down_sample(0.005) (nerf_runner.py:373) on the device (handoff.PointCloud)
            from .handoff import PointCloud
            pc = new_pcd if isinstance(new_pcd, PointCloud) else PointCloud(
                np.asarray(new_pcd.points if hasattr(new_pcd, "points") else new_pcd, np.float64), device=self.device)
            self.build_octree_pts = pc.voxel_down_sample(0.005).points.copy()
            self.build_octree()
        if not reuse_weights:
            self.create_nerf()
        else:
            if self.cfg.get("frame_features", 0) > 0:
                # nerf_runner.py:380-386: new codes for every frame, the trained rows of the
                # previous frames copied over
                fa = FeatureArray(len(self.images), self.cfg["frame_features"]).to(self.device)
                old = self.models["feature_array"]
                if old is not None:
                    with torch.no_grad():
                        fa.data.data[:prev] = old.data.detach()[:prev].to(self.device)
                self.models["feature_array"] = fa
            # pose corrections are new for every frame (:388-391); with optimize_poses = 0 the
            # trainer rebuilds its frozen identity stand-in at the new frame count
            self.models["pose_array"] = (PoseArray(len(self.images), self.cfg["max_trans"] * self.cfg["sc_factor"],
                                                   self.cfg["max_rot"]).to(self.device)
                                         if self.cfg["optimize_poses"] else None)
        self.global_step = 0
        self.best_models, self.best_loss = None, np.inf
        if not self.cfg["no_batching"]:
            new = self._pool_rays(range(prev, len(self.masks)))
            self.rays = torch.cat((self.rays, new), 0)
        self._new_trainer()

    def train(self):
        """nerf_runner.py:854-862: N_iters = n_step + 1 fused steps on DataLoader batches."""
        set_seed(0)
        out = None
        for it in range(self.N_iters):
            if self.N_iters >= 10 and it % (self.N_iters // 10) == 0:
                logging.info(f"train progress {it}/{self.N_iters}")
            # one captured graph per step (schedule, batch slice, field pass, optimiser read the device
            # step block: no per-step id copy); eager launches when kernel timing is on (events are not
            # capturable)
            if self.trainer.time_kernels:
                out = self.trainer.step(ids=self.data_loader.next_ids())
            else:
                perm, k = self.data_loader.next_slice()
                out = self.trainer.graph_step_epoch(perm, k, self.data_loader.batch_size)
            self.global_step += 1
        return out

    def get_truncation(self):
        """nerf_runner.py:661-674: the truncation band of the current step (linear / exp
        annealing from trunc_start when trunc_decay_type is set), times sc_factor."""
        return truncation(self.cfg, self.global_step)

    def save_weights(self, out_file, models=None):
        models = self.models if models is None else models
        data = {"global_step": self.global_step, "model": models["model"].state_dict(),
                "embed_fn": models["embed_fn"].state_dict(),
                "octree": self.octree_m.octree if self.octree_m is not None else None}
        if models.get("pose_array") is not None and self.cfg["optimize_poses"]:
            data["pose_array"] = models["pose_array"].state_dict()
        if models.get("feature_array") is not None:
            data["feature_array"] = models["feature_array"].state_dict()
        torch.save(data, out_file)

    def load_weights(self, ckpt_path):
        """nerf_runner.py:527-541: network, embedder, frame features and pose
        corrections (each when both the checkpoint and the runner have it), copied in
        place into the trainer's flat parameter buffer (the module parameters are
        views of it). The Adam state starts fresh, as after create_optimizer."""
        ckpt = torch.load(ckpt_path, weights_only=True, map_location=self.device)
        with torch.no_grad():
            for k in ("model", "embed_fn", "feature_array", "pose_array"):
                if self.models.get(k) is None or ckpt.get(k) is None:
                    continue
                for name, v in ckpt[k].items():
                    t = dict(self.models[k].named_parameters()).get(name)
                    if t is None:
                        t = dict(self.models[k].named_buffers())[name]
                    t.copy_(v)
        if self.trainer.amp:
            self.trainer.refresh_half_table()

    def run_network_density(self, inputs, get_normals=False):
        """nerf_runner.py:1306-1346: sdf of points already in normalised space ([-1,1]
        clip), as [N,1] plus the all-true valid mask (hash-grid embedder)."""
        if get_normals:
            raise NotImplementedError("run_network_density(get_normals=True) is not implemented on the fused path")
        flat = torch.as_tensor(inputs, dtype=torch.float32).reshape(-1, 3)
        sdf = self.trainer.query_sdf(points=flat)
        valid = torch.ones(flat.shape[0], dtype=torch.bool, device=sdf.device)
        return sdf.reshape(*inputs.shape[:-1], 1), valid

    @torch.no_grad()
    def extract_mesh(self, level=None, voxel_size=0.003, isolevel=0.0, return_sigma=False):
        """nerf_runner.py:1349-1408: sdf on the dense grid of voxel centres over
        cfg['bounding_box'] (voxel_size in metres, scaled by sc_factor), points in
        empty octree voxels at the ray-tracing level read 1.0, marching cubes at
        `isolevel`, vertices mapped back to network space. Returns a Mesh
        (.vertices, .faces, .export) — trimesh is not available here."""
        from .mesh import Mesh, grid_axes, marching_cubes
        voxel_size *= self.cfg["sc_factor"]
        tx, ty, tz = grid_axes(self.cfg["bounding_box"], voxel_size)
        occ = self._occ_trace_level() if self.octree_m is not None else None
        sdf = self.trainer.query_sdf(axes=(tx, ty, tz), occ=occ).reshape(len(tx), len(ty), len(tz))
        try:
            vertices, faces = marching_cubes(sdf, isolevel)
        except Exception as e:   # the reference logs and returns None
            logging.info(f"ERROR Marching Cubes {e}")
            return None
        voxel_size_ndc = np.array([tx[-1] - tx[0], ty[-1] - ty[0], tz[-1] - tz[0]]) / np.array(
            [len(tx) - 1, len(ty) - 1, len(tz) - 1])
        offset = np.array([tx[0], ty[0], tz[0]])
        vertices = voxel_size_ndc.reshape(1, 3) * vertices + offset.reshape(1, 3)
        mesh = Mesh(vertices, faces)
        if return_sigma:
            q = np.stack(np.meshgrid(tx, ty, tz, indexing="ij"), -1).astype(np.float32).reshape(-1, 3)
            return mesh, sdf.cpu().numpy(), torch.from_numpy(q).to(sdf.device)
        return mesh

    def mesh_texture_from_train_images(self, mesh, rgbs_raw, train_texture=False, tex_res=1024):
        """nerf_runner.py:1467-1541: bake a texture for `mesh` (normalised space) from
        the training frames on the device (bundlesdf_amd.texture); returns the
        unwrapped mesh with .uv and .texture (Mesh.export writes obj + mtl + png)."""
        from .texture import mesh_texture_from_train_images
        return mesh_texture_from_train_images(self, mesh, rgbs_raw, train_texture=train_texture, tex_res=tex_res)
