"""ctypes binding of liboracle.so -- TEST INFRASTRUCTURE ONLY.

The oracle is the CPU restatement of the reference hot path (see rt_oracle.h for
the parity-pin statement).  Only tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg may import this module; the product never does.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liboracle.so")


class Stats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in
                ("coverage", "shadow", "isect", "occl", "bf_tested", "bf_mismatch", "aabb_tests", "prim_tests",
                 "aabb_occl", "prim_occl")]

    def as_dict(self):
        return {n: int(getattr(self, n)) for n, _ in self._fields_}


class Camera(C.Structure):
    _fields_ = [("pos", C.c_float * 3), ("tl", C.c_float * 3), ("tr", C.c_float * 3), ("bl", C.c_float * 3),
                ("lens_radius", C.c_float), ("rwidth", C.c_float), ("rheight", C.c_float)]


PROBE_PRIMARY, PROBE_PS, PROBE_PT = 0, 1, 2
DIFFUSE, MIRROR, DIELECTRIC, CHECKER, LIGHT = 0, 1, 2, 3, 4

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = C.CDLL(LIB_PATH)
        vp, ip, fp = C.c_void_p, C.POINTER(C.c_int32), C.POINTER(C.c_float)
        L.or_scene_recipe.restype = vp
        L.or_scene_recipe.argtypes = [C.c_char_p, C.c_char_p]
        L.or_scene_new.restype = vp
        L.or_scene_free.argtypes = [vp]
        for n in ("or_scene_num_prims", "or_scene_nodes_used", "or_scene_depth", "or_scene_build_bvh"):
            getattr(L, n).argtypes = [vp]
            getattr(L, n).restype = C.c_int
        L.or_scene_nodes.restype = vp
        L.or_scene_nodes.argtypes = [vp]
        L.or_scene_set_bvh.argtypes = [vp, vp, C.c_int, C.POINTER(C.c_uint32), C.c_int]
        L.or_scene_set_bvh.restype = C.c_int
        L.or_scene_indices.restype = C.POINTER(C.c_uint32)
        L.or_scene_indices.argtypes = [vp]
        L.or_scene_add_material.argtypes = [vp, C.c_int, fp, fp, C.c_float, C.c_float]
        L.or_scene_add_sphere.argtypes = [vp, fp, C.c_float, C.c_int]
        L.or_scene_add_plane.argtypes = [vp, fp, C.c_float, C.c_int]
        L.or_scene_add_triangle.argtypes = [vp, fp, fp, fp, C.c_int]
        L.or_scene_add_material_tex.argtypes = [vp, C.c_int, fp, fp, C.c_float, C.c_float, C.c_int]
        L.or_scene_add_texture.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_uint32)]
        L.or_scene_add_cube.argtypes = [vp, fp, fp, fp, C.c_int]
        L.or_scene_add_quad.argtypes = [vp, C.c_float, fp, C.c_int]
        L.or_scene_set_integrator.argtypes = [vp, C.c_int]
        L.or_scene_set_sky.argtypes = [vp, C.c_int, C.c_int, C.POINTER(C.c_uint32)]
        L.or_camera_default.argtypes = [C.POINTER(Camera), C.c_int, C.c_int]
        L.or_probe.argtypes = [vp, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(Stats)]
        L.or_primary_hits.argtypes = [vp, C.POINTER(Camera), C.c_int, C.c_int, C.c_int, ip, C.c_int, fp, ip, fp, fp]
        L.or_trace_pixels.argtypes = [vp, C.POINTER(Camera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, ip, C.c_int,
                                      fp, C.POINTER(Stats)]
        L.or_tick.argtypes = [vp, C.POINTER(Camera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                              fp, C.POINTER(C.c_uint32), C.POINTER(Stats), C.c_int]
        L.or_trace_rays.argtypes = [vp, fp, C.c_int, C.POINTER(C.c_uint8), C.c_int, C.POINTER(C.c_uint32), fp,
                                    C.POINTER(Stats)]
        L.or_camera_rays.argtypes = [C.POINTER(Camera), C.c_int, C.c_int, C.c_int, ip, C.c_int, fp]
        L.or_pixel_work.argtypes = [vp, C.POINTER(Camera), C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, ip, C.c_int,
                                    C.POINTER(C.c_uint32)]
        L.or_walk_need.argtypes = [vp, C.POINTER(Camera), C.c_int, C.c_int, C.c_int, ip, C.c_int, C.c_int, fp, ip]
        L.or_intersect.argtypes = [vp, fp, C.c_int, fp, ip, fp, fp, C.c_int]
        L.or_intersect_packets.argtypes = [vp, fp, C.c_int, fp, ip, fp, fp]
        L.or_occluded.argtypes = [vp, fp, C.c_int, C.POINTER(C.c_uint8)]
        L.or_obj_parse.argtypes = [C.c_char_p, C.POINTER(fp), ip, C.POINTER(ip), ip]
        L.or_obj_parse.restype = C.c_int
        L.or_free.argtypes = [vp]
        L.or_init_seed.argtypes = [C.c_uint32]
        L.or_init_seed.restype = C.c_uint32
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


def obj_parse(path):
    L = lib()
    vp, tp = C.POINTER(C.c_float)(), C.POINTER(C.c_int32)()
    nv, nt = C.c_int32(), C.c_int32()
    rc = L.or_obj_parse(path.encode(), C.byref(vp), C.byref(nv), C.byref(tp), C.byref(nt))
    if rc != 0:
        raise IOError(f"or_obj_parse({path}) -> {rc}")
    V = np.ctypeslib.as_array(vp, shape=(nv.value, 3)).copy()
    T = np.ctypeslib.as_array(tp, shape=(nt.value, 3)).copy()
    L.or_free(C.cast(vp, C.c_void_p))
    L.or_free(C.cast(tp, C.c_void_p))
    return V, T


class Scene:
    """Oracle scene: one of the SURVEY 8(d) recipes built from RTMESH1 files."""

    def __init__(self, recipe, mesh_dir):
        self.L = lib()
        self.h = self.L.or_scene_recipe(recipe.encode(), mesh_dir.encode())
        if not self.h:
            raise RuntimeError(f"oracle recipe {recipe!r} failed (mesh dir {mesh_dir})")

    def __del__(self):
        if getattr(self, "h", None):
            self.L.or_scene_free(self.h)
            self.h = None

    def set_integrator(self, mode):
        """0 = Renderer::Trace (path tracer), 1 = Renderer::WhittedTrace, 2 = packet mode."""
        self.L.or_scene_set_integrator(self.h, mode)

    @property
    def num_prims(self):
        return self.L.or_scene_num_prims(self.h)

    @property
    def nodes_used(self):
        return self.L.or_scene_nodes_used(self.h)

    @property
    def depth(self):
        return self.L.or_scene_depth(self.h)

    def nodes(self):
        n = self.nodes_used
        buf = (C.c_uint8 * (32 * n)).from_address(self.L.or_scene_nodes(self.h))
        return np.frombuffer(bytes(buf), dtype=np.uint8).reshape(n, 32)

    def indices(self):
        p = self.L.or_scene_indices(self.h)
        return np.ctypeslib.as_array(p, shape=(self.num_prims,)).copy()

    def probe(self, W, H, mode, depth=10, spp=1, brute=True):
        st = Stats()
        self.L.or_probe(self.h, W, H, mode, depth, spp, int(brute), C.byref(st))
        return st.as_dict()

    @staticmethod
    def camera(W, H):
        cam = Camera()
        lib().or_camera_default(C.byref(cam), W, H)
        return cam

    def camera_rays(self, W, H, pixels, frame=0):
        pixels = np.ascontiguousarray(pixels, dtype=np.int32)
        rays = np.empty((len(pixels), 7), np.float32)
        cam = self.camera(W, H)
        self.L.or_camera_rays(C.byref(cam), W, H, frame, _p(pixels, C.c_int32), len(pixels), _p(rays, C.c_float))
        return rays

    def primary_hits(self, W, H, pixels, frame=0):
        pixels = np.ascontiguousarray(pixels, dtype=np.int32)
        n = len(pixels)
        t = np.empty(n, np.float32); o = np.empty(n, np.int32); u = np.empty(n, np.float32); v = np.empty(n, np.float32)
        cam = self.camera(W, H)
        self.L.or_primary_hits(self.h, C.byref(cam), W, H, frame, _p(pixels, C.c_int32), n,
                               _p(t, C.c_float), _p(o, C.c_int32), _p(u, C.c_float), _p(v, C.c_float))
        return t, o, u, v

    def trace_pixels(self, W, H, pixels, spp=1, depth=10, frame=0):
        pixels = np.ascontiguousarray(pixels, dtype=np.int32)
        rgb = np.empty((len(pixels), 3), np.float32)
        st = Stats()
        cam = self.camera(W, H)
        self.L.or_trace_pixels(self.h, C.byref(cam), W, H, spp, depth, frame, _p(pixels, C.c_int32), len(pixels),
                               _p(rgb, C.c_float), C.byref(st))
        return rgb, st.as_dict()

    def pixel_work(self, W, H, pixels, spp=1, depth=10, frame=0):
        """Traversal counters per pixel [n, 8]: closest-hit nodes / prims, any-hit nodes / prims,
        closest-hit pops of interior / leaf entries already beyond the ray's t, 0, 0."""
        pixels = np.ascontiguousarray(pixels, dtype=np.int32)
        out = np.zeros((len(pixels), 8), np.uint32)
        cam = self.camera(W, H)
        self.L.or_pixel_work(self.h, C.byref(cam), W, H, spp, depth, frame, _p(pixels, C.c_int32), len(pixels),
                             _p(out, C.c_uint32))
        return out

    def walk_need(self, W, H, pixels=None, frame=0, cam=None, all_hits=False, with_obj=False):
        """Per camera ray (sample 0 of `frame`): the cull margin the wave camera walk needs to return
        IntersectBVH's answer R -- (entry of R's leaf box - t_R) / t_R, 0 if R lies at or past it
        (or_walk_need); all_hits: the max of that over every primitive the ray hits; with_obj: also
        R's primitive id per ray."""
        pixels = np.arange(W * H, dtype=np.int32) if pixels is None else np.ascontiguousarray(pixels, np.int32)
        out = np.zeros(len(pixels), np.float32)
        obj = np.full(len(pixels), -1, np.int32)
        c = self.camera(W, H) if cam is None else self.camera_from(W, H, cam)
        self.L.or_walk_need(self.h, C.byref(c), W, H, frame, _p(pixels, C.c_int32), len(pixels), int(all_hits),
                            _p(out, C.c_float), _p(obj, C.c_int32) if with_obj and not all_hits else None)
        return (out, obj) if with_obj else out

    def trace_rays(self, rays, seeds, depth=10, flags=None):
        """Renderer::Trace / WhittedTrace (set_integrator) on (n, 7) rays with per-ray RNG states;
        returns (radiance [n, 3], seeds after the call, stats)."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 7)
        seeds = np.array(seeds, np.uint32).copy()
        rgb = np.empty((len(rays), 3), np.float32)
        fl = None if flags is None else np.ascontiguousarray(flags, np.uint8)
        st = Stats()
        self.L.or_trace_rays(self.h, _p(rays, C.c_float), len(rays), None if fl is None else _p(fl, C.c_uint8), depth,
                             _p(seeds, C.c_uint32), _p(rgb, C.c_float), C.byref(st))
        return rgb, seeds, st.as_dict()

    @classmethod
    def camera_from(cls, W, H, cam):
        """The default camera of a W x H frame with the position / screen corners / lens radius of
        `cam` (an object with pos, top_left, top_right, bottom_left, lens_radius: the library's
        rt.Camera) -- a moved camera as Camera::AdjustCamera leaves it (camera.h:54-86)."""
        c = cls.camera(W, H)
        for a, b in (("pos", "pos"), ("tl", "top_left"), ("tr", "top_right"), ("bl", "bottom_left")):
            getattr(c, a)[:] = list(getattr(cam, b))
        c.lens_radius = cam.lens_radius
        return c

    def tick(self, W, H, acc, spp=1, depth=10, frame=0, y0=0, y1=None, threads=0, cam=None):
        """One Renderer::Tick over rows [y0, y1): updates acc (H*W*4 f32) in place, returns RGB8.
        cam: a moved camera (camera_from), else the default one."""
        y1 = H if y1 is None else y1
        out = np.zeros(W * H, np.uint32)
        st = Stats()
        cam = self.camera(W, H) if cam is None else self.camera_from(W, H, cam)
        self.L.or_tick(self.h, C.byref(cam), W, H, spp, depth, frame, y0, y1, _p(acc, C.c_float),
                       _p(out, C.c_uint32), C.byref(st), threads)
        return out, st.as_dict()

    def intersect(self, rays, brute=False):
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        n = len(rays)
        t = np.empty(n, np.float32); o = np.empty(n, np.int32); u = np.empty(n, np.float32); v = np.empty(n, np.float32)
        self.L.or_intersect(self.h, _p(rays, C.c_float), n, _p(t, C.c_float), _p(o, C.c_int32), _p(u, C.c_float),
                            _p(v, C.c_float), int(brute))
        return t, o, u, v

    def intersect_packets(self, rays):
        """Scene::IntersectBVHPacket over packets of 64 consecutive rays."""
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        n = len(rays)
        t = np.empty(n, np.float32); o = np.empty(n, np.int32); u = np.empty(n, np.float32); v = np.empty(n, np.float32)
        self.L.or_intersect_packets(self.h, _p(rays, C.c_float), n, _p(t, C.c_float), _p(o, C.c_int32),
                                    _p(u, C.c_float), _p(v, C.c_float))
        return t, o, u, v

    def occluded(self, rays):
        rays = np.ascontiguousarray(rays, dtype=np.float32)
        out = np.empty(len(rays), np.uint8)
        self.L.or_occluded(self.h, _p(rays, C.c_float), len(rays), _p(out, C.c_uint8))
        return out
