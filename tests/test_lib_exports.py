"""CPU: libnof.so (the C-ABI drop-in) loads and exports every entry point
include/nof.h declares, and the Python binding declares exactly those. No
compute calls are made here (no GPU in the build container)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_symbols():
    src = open(os.path.join(ROOT, "include", "nof.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(nof_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def libnof():
    from bundlesdf_amd import build
    build.build()
    from bundlesdf_amd import _lib
    return _lib.lib()


def test_header_symbols_exported(libnof):
    syms = _header_symbols()
    assert len(syms) >= 8
    for s in syms:
        assert hasattr(libnof, s), f"{s} declared in include/nof.h but not exported"


def test_binding_matches_header():
    from bundlesdf_amd import _lib
    assert sorted(_lib.declared_symbols()) == _header_symbols()


def test_host_only_entry_points(libnof):
    import numpy as np
    from oracle import kernels as K
    sc = np.zeros(16, np.float32)
    res = np.zeros(16, np.uint32)
    libnof.nof_level_params(16, np.float32(0.2), 16, sc.ctypes.data_as(ctypes.c_void_p),
                            res.ctypes.data_as(ctypes.c_void_p))
    osc, ores = K.level_params(16, np.float32(0.2), 16)
    np.testing.assert_array_equal(sc, osc)
    np.testing.assert_array_equal(res, ores)
    assert b"gfx950" in libnof.nof_version()


@pytest.mark.parametrize("cname,pyname", [("nof_field_desc", "FieldDesc"), ("nof_ray_pool_desc", "RayPoolDesc"),
                                          ("nof_step_params", "StepParams"), ("nof_schedule_desc", "ScheduleDesc")])
def test_descriptor_layout_matches_header(tmp_path, cname, pyname):
    """The ctypes mirrors in _lib.py have the C header's field offsets and size
    (gcc compiles include/nof.h and prints offsetof of every field)."""
    import subprocess
    from bundlesdf_amd import _lib
    S = getattr(_lib, pyname)
    fields = [f[0] for f in S._fields_]
    src = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{os.path.join(ROOT, "include", "nof.h")}"',
           'int main(void) {', f'  printf("%zu\\n", sizeof({cname}));']
    src += [f'  printf("%zu\\n", offsetof({cname}, {f}));' for f in fields]
    src += ['  return 0;', '}']
    c = tmp_path / "layout.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(c)], check=True)
    vals = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == ctypes.sizeof(S)
    for f, off in zip(fields, vals[1:]):
        assert getattr(S, f).offset == off, f
