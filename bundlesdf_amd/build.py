"""Build libnof.so (the C-ABI HIP library) in-tree for gfx950.

Every kernel source under csrc/ is compiled by hipcc for --offload-arch=gfx950
(no hipify, no CUDA), objects are cached by content hash, and the library is
linked at bundlesdf_amd/libnof.so so it travels with the repo snapshot.
"""
import concurrent.futures as cf
import hashlib
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
# NOF_ABLATE=1 builds the timing-experiment variant (ABL() bits live) as libnof_ablate.so;
# only scripts/ablate.py loads it (NOF_LIB), the product library is always libnof.so
ABLATE = os.environ.get("NOF_ABLATE", "0") == "1"
OUT = os.path.join(HERE, "libnof_ablate.so" if ABLATE else "libnof.so")
OBJDIR = os.path.join(HERE, "build", "obj_ablate" if ABLATE else "obj")
ARCH = os.environ.get("NOF_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

CFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function",
          "-Wno-unused-variable", "-munsafe-fp-atomics", "-fno-strict-aliasing"] + (["-DNOF_ABLATE=1"] if ABLATE else [])


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp")))


def _digest(path):
    h = hashlib.sha1()
    h.update(" ".join(CFLAGS).encode())
    with open(path, "rb") as f:
        h.update(f.read())
    for hdr in sorted(os.listdir(CSRC)):
        if hdr.endswith(".h"):
            with open(os.path.join(CSRC, hdr), "rb") as f:
                h.update(f.read())
    with open(os.path.join(HERE, "..", "include", "nof.h"), "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def _compile(src):
    obj = os.path.join(OBJDIR, os.path.basename(src) + "." + _digest(src) + ".o")
    if os.path.exists(obj):
        return obj
    cmd = [HIPCC] + CFLAGS + ["-c", src, "-o", obj + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stderr}")
    os.replace(obj + ".tmp", obj)
    return obj


def build(verbose=False, jobs=None):
    os.makedirs(OBJDIR, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), int(os.environ.get("MAX_JOBS", "8")))
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(_compile, srcs))
    # relink whenever the object set differs from the one the library was linked from
    manifest = OUT + ".objs"
    want = "\n".join(os.path.basename(o) for o in objs)
    if os.path.exists(OUT) and os.path.exists(manifest):
        with open(manifest) as f:
            if f.read() == want:
                return OUT
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", OUT + ".tmp"] + objs
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stderr}")
    os.replace(OUT + ".tmp", OUT)
    with open(manifest, "w") as f:
        f.write(want)
    if verbose:
        print(f"built {OUT}")
    return OUT


if __name__ == "__main__":
    build(verbose=True)
    sys.exit(0)
