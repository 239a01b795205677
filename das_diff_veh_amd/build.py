"""Builds libdvh.so (HIP kernels + C-ABI) in-tree for gfx950 with hipcc.

The library lands in ``das_diff_veh_amd/lib/libdvh.so`` so that it travels with the repository
snapshot to the GPU box (git-ignored, not gpurun-ignored).  Objects are rebuilt only when a
source or header is newer than the object.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG, "csrc")
OUT_DIR = os.path.join(PKG, "lib")
LIB = os.path.join(OUT_DIR, "libdvh.so")
OBJ_DIR = os.path.join(OUT_DIR, "obj")
ARCH = os.environ.get("DVH_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics", "-fno-slp-vectorize",
          "-fvisibility=hidden", "-Wall", "-Wno-unused-function"]


def _sources():
    return sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.cpp")))


def _newest_header():
    hs = glob.glob(os.path.join(CSRC, "*.h")) + glob.glob(os.path.join(os.path.dirname(PKG), "include", "*.h"))
    return max((os.path.getmtime(h) for h in hs), default=0.0)


def _compile(src, verbose=False):
    obj = os.path.join(OBJ_DIR, os.path.basename(src) + ".o")
    if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), _newest_header()):
        return obj
    cmd = [HIPCC, *CFLAGS, "-I", CSRC, "-I", os.path.join(os.path.dirname(PKG), "include"), "-c", src, "-o", obj]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {src}:\n{r.stdout}\n{r.stderr}")
    return obj


def build(verbose=False, jobs=None, out=None, defines=(), flags=()):
    """Build libdvh.so (or, with out/defines/flags, a variant library for A/B timing)."""
    global LIB, OBJ_DIR, CFLAGS
    if out is not None:
        saved = LIB, OBJ_DIR, CFLAGS
        LIB, OBJ_DIR = out, out + ".obj"
        CFLAGS = CFLAGS + [f"-D{d}" for d in defines] + list(flags)
        try:
            return build(verbose, jobs)
        finally:
            LIB, OBJ_DIR, CFLAGS = saved
    os.makedirs(OBJ_DIR, exist_ok=True)
    srcs = _sources()
    jobs = jobs or min(len(srcs), 8)
    with cf.ThreadPoolExecutor(jobs) as ex:
        objs = list(ex.map(lambda s: _compile(s, verbose), srcs))
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= max(os.path.getmtime(o) for o in objs):
        return LIB
    tmp = LIB + ".tmp"  # linked aside and renamed: a reader never sees a partly written library
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp, *objs]
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed:\n{r.stdout}\n{r.stderr}")
    os.replace(tmp, LIB)
    return LIB


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if a != "-v"]
    if args:  # python -m das_diff_veh_amd.build OUT.so DEFINE=1 ...
        print(build(verbose="-v" in sys.argv, out=os.path.abspath(args[0]), defines=args[1:]))
    else:
        print(build(verbose="-v" in sys.argv))
