"""Timing-build library of field_step.hip at a git revision (default HEAD) linked with the
current timing-build objects of the other sources -> bundlesdf_amd/libnof_prev.so, for
scripts/gpu_ab.sh A/B runs against libnof_ablate.so (PROD=1: production builds, against libnof.so).
Usage: [PROD=1] python scripts/build_prev.py [REV]"""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
# PROD=1: production builds (ablation bits compiled out) of both, for A/B against libnof.so
os.environ["NOF_ABLATE"] = "0" if os.environ.get("PROD") == "1" else "1"
from bundlesdf_amd import build as B  # noqa: E402

rev = sys.argv[1] if len(sys.argv) > 1 else "HEAD"
B.build()
# FILES: the csrc sources taken from REV (default field_step.hip); the rest from the working tree
files = os.environ.get("FILES", "field_step.hip").split(",")
prev_objs = []
for fn in files:
    src = f"/tmp/nof_prev_{fn}"
    with open(src, "w") as f:
        f.write(subprocess.run(["git", "-C", ROOT, "show", f"{rev}:bundlesdf_amd/csrc/{fn}"], check=True,
                               capture_output=True, text=True).stdout)
    obj = src + ".o"
    r = subprocess.run([B.HIPCC] + B.CFLAGS + ["-I" + B.CSRC, "-c", src, "-o", obj], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    prev_objs.append(obj)
keep = open(B.OUT + ".objs").read().split()
objs = [os.path.join(B.OBJDIR, o) for o in keep if not any(o.startswith(fn) for fn in files)]
r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o",
                    os.path.join(B.HERE, "libnof_prev.so")] + prev_objs + objs, capture_output=True, text=True)
assert r.returncode == 0, r.stderr[-3000:]
print("built libnof_prev.so from", rev)
