"""`mycuda.common` shim (mycuda/common.h:28-30 entry points)."""
from bundlesdf_amd.common import (postprocessOctreeRayTracing, rayColorToTextureImageCUDA,  # noqa: F401
                                  sampleRaysUniformOccupiedVoxels)
