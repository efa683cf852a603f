"""`from nerf_runner import *` shim (bundlesdf.py:11)."""
from bundlesdf_amd.nerf_runner import *  # noqa: F401,F403
from bundlesdf_amd.nerf_runner import __all__  # noqa: F401
