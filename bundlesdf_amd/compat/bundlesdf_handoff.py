"""Hand-off shim. bundlesdf.py takes the scene-bounds / pose
helpers from `from Utils import *` and `from tool import *` (bundlesdf.py:10-13),
modules that also carry the tracker's code, so they are not replaced wholesale:
after importing bundlesdf, call

    import bundlesdf
    from bundlesdf_amd.compat.bundlesdf_handoff import install
    install(bundlesdf)

which rebinds, in that module's namespace only, toOpen3dCloud, depth2xyzmap,
compute_scene_bounds(_worker), compute_translation_scales, find_biggest_cluster,
get_optimized_poses_in_real_world and mesh_to_real_world to the device
implementations of bundlesdf_amd.handoff (open3d / sklearn calls -> HIP)."""
from bundlesdf_amd import handoff as _H

NAMES = ["toOpen3dCloud", "depth2xyzmap", "compute_scene_bounds_worker", "compute_scene_bounds",
         "compute_translation_scales", "find_biggest_cluster", "get_optimized_poses_in_real_world",
         "mesh_to_real_world"]


def install(module):
    for n in NAMES:
        setattr(module, n, getattr(_H, n))
    return module
