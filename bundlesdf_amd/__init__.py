"""bundlesdf_amd — MI355X-native neural-object-field trainer.

Drop-in for the per-step SDF/colour rendering + online optimisation loop of
BundleSDF's nerf_runner.py. Kernels live in libnof.so (HIP,
gfx950) behind the C ABI in include/nof.h; the Python modules mirror the
reference's operator/module interfaces:

  bundlesdf_amd.gridencoder   <- mycuda/torch_ngp_grid_encoder (pybind `gridencoder`)
  bundlesdf_amd.common        <- mycuda (pybind `common`)
  bundlesdf_amd.grid          <- mycuda/torch_ngp_grid_encoder/grid.py
  bundlesdf_amd.nerf_helpers  <- nerf_helpers.py
  bundlesdf_amd.nerf_runner   <- nerf_runner.py (NerfRunner)
"""
__version__ = "0.1.0"
