"""`mycuda.torch_ngp_grid_encoder.grid` shim (GridEncoder, grid.py:107)."""
from bundlesdf_amd.grid import GridEncoder, _grid_encode  # noqa: F401

grid_encode = _grid_encode.apply
