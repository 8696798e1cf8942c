"""Build librtamd.so (host C++ + gfx950 HIP kernels) in-tree with hipcc.

The library is the product: a C-ABI shared object whose entry points are declared in
include/rt_amd.h.  It is built for gfx950 only, in place, so the .so travels with the
repository snapshot to the GPU box.
"""
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
LIB = os.path.join(PKG, "librtamd.so")
# the kernels are compiled twice (core / extension builds of rt_kernels.inc), in parallel
SOURCES = ["rt_host.cpp", "rt_device.hip", "rt_kern_core.hip", "rt_kern_ext.hip", "rt_multi.cpp", "rt_sbvh.cpp"]
HEADERS = ["rt_math.h", "rt_internal.h", "rt_libm.h", "rt_dev_types.h", "rt_kernels.inc",
           os.path.join("..", "..", "include", "rt_amd.h")]

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
# -ffp-contract=off + IEEE div/sqrt (hipcc's default) keep the kernels' float results
# bit-identical to the reference's evaluation order.
# -fno-slp-vectorize: plain -O3 packs adjacent f32 adds/multiplies into v_pk_*_f32 plus the
# v_mov shuffles feeding them; scalar f32 issues faster on gfx950 and the frame kernel drops
# from 91 to 68 VGPRs (5 -> 7 waves/SIMD): TEAPOT-F 1080p 0.120 -> 0.106 ms, CFG5-sub 10.4 ->
# 9.4 ms, bit-identical (profiles/r01/ab_nslp_*.json).
LIBS = ["-lz", "-ldl"]   # zlib: PNG textures (rt_image_load); dl: RCCL is resolved at run time (rt_multi.cpp)
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-slp-vectorize", "-fPIC",
         "-shared",
         "-Wall", "-Wno-unused-function"]


def _source_hash():
    """sha256 over the sources, headers, flags and this script: the library is rebuilt when any
    of them differs from what it was built from (content, not file times, which a copied tree
    -- e.g. a gpurun snapshot -- does not preserve)."""
    import hashlib
    h = hashlib.sha256()
    for f in [os.path.join(CSRC, x) for x in SOURCES + HEADERS] + [os.path.abspath(__file__)]:
        with open(f, "rb") as fh:
            h.update(os.path.basename(f).encode() + b"\0" + fh.read())
    h.update(" ".join(FLAGS + LIBS).encode())
    return h.hexdigest()


STAMP = LIB + ".srchash"


def _stale():
    if not os.path.exists(LIB) or not os.path.exists(STAMP):
        return True
    with open(STAMP) as f:
        return f.read().strip() != _source_hash()


def build(force=False, verbose=False):
    if not force and not _stale():
        return LIB
    objdir = os.path.join(PKG, "_obj")
    os.makedirs(objdir, exist_ok=True)
    compile_flags = [f for f in FLAGS if f != "-shared"]
    procs = []
    objs = []
    for f in SOURCES:   # one hipcc per translation unit, concurrently
        obj = os.path.join(objdir, os.path.splitext(f)[0] + ".o")
        lang = ["-x", "hip"]
        cmd = [HIPCC] + compile_flags + lang + ["-c", os.path.join(CSRC, f), "-o", obj]
        if verbose:
            print(" ".join(cmd), file=sys.stderr)
        procs.append((f, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)))
        objs.append(obj)
    for f, p in procs:
        out, err = p.communicate()
        if p.returncode != 0:
            raise RuntimeError(f"hipcc failed on {f} ({p.returncode}):\n{out}\n{err}")
    cmd = [HIPCC, "--offload-arch=gfx950", "-fPIC", "-shared", "--hip-link", "-o", LIB + ".tmp"] + objs + LIBS
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"link failed ({r.returncode}):\n{r.stdout}\n{r.stderr}")
    os.replace(LIB + ".tmp", LIB)
    with open(STAMP, "w") as f:
        f.write(_source_hash() + "\n")
    return LIB


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True))
