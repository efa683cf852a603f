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
# FILES: the csrc sources taken from REV (default field_step.hip); HEADERS: csrc headers taken from REV
# as well (default field_mlp_bwd.h, the MLP backward kernels field_step.hip includes in place; skipped
# when REV predates them) — placed first on the include path; the rest from the working tree
files = os.environ.get("FILES", "field_step.hip").split(",")
headers = os.environ.get("HEADERS", "field_mlp_bwd.h").split(",")
inc = "/tmp/nof_prev_inc"
os.makedirs(inc, exist_ok=True)
for fn in os.listdir(inc):
    os.remove(os.path.join(inc, fn))


def git_show(fn):
    r = subprocess.run(["git", "-C", ROOT, "show", f"{rev}:bundlesdf_amd/csrc/{fn}"], capture_output=True, text=True)
    return r.stdout if r.returncode == 0 else None


for fn in headers:
    text = git_show(fn)
    if text is not None:
        with open(os.path.join(inc, fn), "w") as f:
            f.write(text)
prev_objs = []
for fn in files:
    src = os.path.join(inc, fn)
    text = git_show(fn)
    assert text is not None, f"{fn} not in {rev}"
    with open(src, "w") as f:
        f.write(text)
    obj = f"/tmp/nof_prev_{fn}.o"
    r = subprocess.run([B.HIPCC] + B.CFLAGS + ["-I" + inc, "-I" + B.CSRC, "-c", src, "-o", obj], capture_output=True,
                       text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    prev_objs.append(obj)
keep = open(B.OUT + ".objs").read().split()
objs = [os.path.join(B.OBJDIR, o) for o in keep if not any(o.startswith(fn) for fn in files)]
r = subprocess.run([B.HIPCC, f"--offload-arch={B.ARCH}", "-shared", "-fPIC", "-o",
                    os.path.join(B.HERE, "libnof_prev.so")] + prev_objs + objs, capture_output=True, text=True)
assert r.returncode == 0, r.stderr[-3000:]
print("built libnof_prev.so from", rev)
