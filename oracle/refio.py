"""Test infrastructure: ctypes face of oracle/_ref/libref_io.so -- the reference's vendored
tinyobjloader (template/tiny_obj_loader.h) and stb_image (lib/stb_image.h), compiled
unmodified from /root/reference by `make -C oracle ref` (oracle/ref_io.cpp is the driver).
Used only by tests/ and tests/golden/make_ref_fixtures.py, never by the product."""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REFERENCE = "/root/reference"
LIB = os.path.join(HERE, "_ref", "libref_io.so")
_lib = None


def available():
    """The reference tree is here (this container; the GPU box has none)."""
    return os.path.isfile(os.path.join(REFERENCE, "template", "tiny_obj_loader.h"))


def build():
    subprocess.run(["make", "-s", "-C", HERE, "ref"], check=True)


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB)
        L.ref_load_model.argtypes = [C.c_char_p, C.POINTER(C.POINTER(C.c_float)), C.POINTER(C.c_uint32),
                                     C.POINTER(C.POINTER(C.c_int32)), C.POINTER(C.c_uint32)]
        L.ref_load_image.argtypes = [C.c_char_p, C.POINTER(C.POINTER(C.c_uint32)), C.POINTER(C.c_int),
                                     C.POINTER(C.c_int), C.POINTER(C.c_int)]
        L.ref_free.argtypes = [C.c_void_p]
        _lib = L
    return _lib


def load_model(path):
    """Scene::LoadModel's view of an OBJ through tinyobj::LoadObj (template/scene.h:156-201):
    (attrib.vertices as float32 [nv, 3], triangle corners as vertex indices [nt, 3])."""
    L = lib()
    v, f = C.POINTER(C.c_float)(), C.POINTER(C.c_int32)()
    nv, nt = C.c_uint32(), C.c_uint32()
    if L.ref_load_model(path.encode(), C.byref(v), C.byref(nv), C.byref(f), C.byref(nt)) != 0:
        raise IOError(f"tinyobj::LoadObj failed on {path}")
    try:
        V = np.ctypeslib.as_array(v, (nv.value * 3,)).copy().reshape(-1, 3) if nv.value else np.zeros((0, 3), np.float32)
        F = np.ctypeslib.as_array(f, (nt.value * 3,)).copy().reshape(-1, 3) if nt.value else np.zeros((0, 3), np.int32)
    finally:
        L.ref_free(v)
        L.ref_free(f)
    return V, F


def load_image(path):
    """Surface::LoadImage through stbi_load (template/template.cpp:1579-1601): (texels as
    uint32 0x00RRGGBB [h, w], stb's channel count)."""
    L = lib()
    p, w, h, n = C.POINTER(C.c_uint32)(), C.c_int(), C.c_int(), C.c_int()
    if L.ref_load_image(path.encode(), C.byref(p), C.byref(w), C.byref(h), C.byref(n)) != 0:
        raise IOError(f"stbi_load failed on {path}")
    try:
        px = np.ctypeslib.as_array(p, (w.value * h.value,)).copy().reshape(h.value, w.value)
    finally:
        L.ref_free(p)
    return px, n.value
