"""`import gridencoder` shim (mycuda/torch_ngp_grid_encoder/grid.py:23)."""
from bundlesdf_amd.gridencoder import grid_encode_backward, grid_encode_forward  # noqa: F401
