"""CPU: the module-name shims resolve the reference's import statements to
this package."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_reference_imports_resolve():
    code = (
        "import gridencoder\n"
        "from mycuda import common\n"
        "from mycuda.torch_ngp_grid_encoder.grid import GridEncoder\n"
        "from nerf_runner import *\n"
        "import bundlesdf_amd.gridencoder as g, bundlesdf_amd.common as c, bundlesdf_amd.grid as gr\n"
        "assert gridencoder.grid_encode_forward is g.grid_encode_forward\n"
        "assert gridencoder.grid_encode_backward is g.grid_encode_backward\n"
        "assert common.sampleRaysUniformOccupiedVoxels is c.sampleRaysUniformOccupiedVoxels\n"
        "assert common.postprocessOctreeRayTracing is c.postprocessOctreeRayTracing\n"
        "assert common.rayColorToTextureImageCUDA is c.rayColorToTextureImageCUDA\n"
        "assert GridEncoder is gr.GridEncoder\n"
        "assert NerfRunner.__module__ == 'bundlesdf_amd.nerf_runner'\n"
        "assert callable(preprocess_data)\n"
        "e = GridEncoder(3, 16, 2, 16, 19, desired_resolution=128)\n"
        "assert e.n_params == e.embeddings.numel() and e.out_dim == 32\n"
        "assert set(e.state_dict()) == {'embeddings', 'offsets'}\n"
    )
    env = dict(os.environ, PYTHONPATH=os.pathsep.join([os.path.join(ROOT, "bundlesdf_amd", "compat"), ROOT]))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
