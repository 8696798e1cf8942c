"""MI355X-native ray-tracing hot path of pmichels19/AdvancedGraphicsRayTracer.

Python face of librtamd.so (C-ABI in include/rt_amd.h).  The classes mirror the
reference's C++ surface for this path:

    Scene.IntersectBVH / Scene.IsOccluded   <- Scene::IntersectBVH / IsOccluded (template/scene.h:285, 452)
    Renderer.Tick                            <- Renderer::Tick (renderer.cpp:200-309)
    Camera                                   <- Camera (camera.h:28-52)

Everything computes on the GPU through librtamd.so; there is no CPU fallback.  A
missing library or device raises RTError.  Device buffers are torch tensors (torch is
plumbing here: memory, streams, torch.distributed).
"""
import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.abspath(os.environ.get("RTAMD_LIB", os.path.join(PKG_DIR, "librtamd.so")))   # RTAMD_LIB: A/B builds (tools/)
DATA_DIR = os.path.join(PKG_DIR, "data")
HEADER = os.path.join(os.path.dirname(PKG_DIR), "include", "rt_amd.h")

ABI_VERSION = 4   # include/rt_amd.h RT_ABI_VERSION
RT_OK, RT_ERR_INVALID, RT_ERR_NO_DEVICE, RT_ERR_HIP, RT_ERR_IO, RT_ERR_UNSUPPORTED, RT_ERR_COMM = 0, -1, -2, -3, -4, -5, -6
RT_COMM_ID_BYTES = 128
MULTI_PIPELINED, MULTI_TIMING, MULTI_BALANCED = 1, 2, 4
SPHERE, PLANE, CUBE, QUAD, TRIANGLE = 0, 1, 2, 3, 4
DIFFUSE, MIRROR, DIELECTRIC, CHECKERBOARD, LIGHT, DSMIX, TEXTURE = 0, 1, 2, 3, 4, 5, 6
MODE_PATH = 0
MODE_WHITTED = 1
MODE_PACKET = 2
WALK_LANE, WALK_WAVE, WALK_AUTO = 0, 1, 2
WALK_CHECK_OFF, WALK_CHECK_COUNT, WALK_CHECK_VERIFY = 0, 1, 2
BVH_PLAIN, BVH_SBVH = 0, 1
# renderer.h:9, renderer.h:13, renderer.cpp:105 (TracePacket's bounces: Trace's default depth)
DEFAULT_DEPTH = {MODE_PATH: 10, MODE_WHITTED: 20, MODE_PACKET: 10}
RECIPES = ("teapotF", "teapot", "mig16", "cfg3", "cfg5", "default")


class RTError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"[{code}] {msg}")
        self.code = code


class Prim(C.Structure):
    _fields_ = [("type", C.c_int32), ("material", C.c_int32), ("v", C.c_float * 9)]


class Material(C.Structure):
    _fields_ = [("kind", C.c_int32), ("color", C.c_float * 3), ("color2", C.c_float * 3), ("ior", C.c_float),
                ("diffuse", C.c_float), ("texture", C.c_int32)]


class Texture(C.Structure):
    _fields_ = [("pixels", C.POINTER(C.c_uint32)), ("width", C.c_uint32), ("height", C.c_uint32)]


class SceneDesc(C.Structure):
    _fields_ = [("prims", C.POINTER(Prim)), ("num_prims", C.c_uint32),
                ("materials", C.POINTER(Material)), ("num_materials", C.c_uint32),
                ("sky_pixels", C.POINTER(C.c_uint32)), ("sky_width", C.c_uint32), ("sky_height", C.c_uint32),
                ("bvh_nodes", C.c_void_p), ("bvh_num_nodes", C.c_uint32), ("bvh_indices", C.POINTER(C.c_uint32)),
                ("device", C.c_int32), ("transforms", C.POINTER(C.c_float)),
                ("textures", C.POINTER(Texture)), ("num_textures", C.c_uint32), ("bvh_kind", C.c_int32)]


class SceneInfo(C.Structure):
    _fields_ = [("num_prims", C.c_uint32), ("nodes_used", C.c_uint32), ("depth", C.c_uint32), ("max_leaf", C.c_uint32),
                ("num_refs", C.c_uint32)]


class Camera(C.Structure):
    """Camera state (camera.h:93-100)."""
    _fields_ = [("pos", C.c_float * 3), ("top_left", C.c_float * 3), ("top_right", C.c_float * 3),
                ("bottom_left", C.c_float * 3), ("lens_radius", C.c_float)]

    @classmethod
    def default(cls, width, height):
        cam = cls()
        _check(lib().rt_camera_default(width, height, C.byref(cam)))
        return cam


class FrameParams(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in ("width", "height", "spp", "depth", "frame", "mode", "reset")]


class Counters(C.Structure):
    _fields_ = [(n, C.c_uint64) for n in ("primary", "shadow", "bounce", "frames")]


RAY_DTYPE = np.dtype([("o", "<f4", 3), ("d", "<f4", 3), ("tmax", "<f4")])
HIT_DTYPE = np.dtype([("t", "<f4"), ("obj", "<i4"), ("u", "<f4"), ("v", "<f4")])

_lib = None


def lib():
    """Load librtamd.so.  Raises RTError when the native library is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RTError(RT_ERR_NO_DEVICE, f"{LIB_PATH} not built (run __graft_entry__.build()); no CPU fallback exists")
    L = C.CDLL(LIB_PATH)
    vp, u32, i32, f = C.c_void_p, C.c_uint32, C.c_int32, C.c_float
    fp = C.POINTER(C.c_float)
    sigs = {
        "rt_abi_version": ([], C.c_int),
        "rt_last_error": ([], C.c_char_p),
        "rt_device_count": ([C.POINTER(C.c_int)], C.c_int),
        "rt_free": ([vp], None),
        "rt_obj_load": ([C.c_char_p, C.POINTER(fp), C.POINTER(u32), C.POINTER(C.POINTER(i32)), C.POINTER(u32)], C.c_int),
        "rt_mesh_load": ([C.c_char_p, C.POINTER(fp), C.POINTER(u32), C.POINTER(C.POINTER(i32)), C.POINTER(u32)], C.c_int),
        "rt_mesh_save": ([C.c_char_p, fp, u32, C.POINTER(i32), u32], C.c_int),
        "rt_mat4_translate": ([f, f, f, fp], C.c_int),
        "rt_mat4_scale": ([f, fp], C.c_int),
        "rt_mat4_rotate": ([C.c_int, f, fp], C.c_int),
        "rt_mat4_mul": ([fp, fp, fp], C.c_int),
        "rt_mesh_to_prims": ([fp, u32, C.POINTER(i32), u32, fp, i32, C.POINTER(Prim)], C.c_int),
        "rt_recipe_describe": ([C.c_char_p, C.c_char_p, C.POINTER(Prim), C.POINTER(u32), C.POINTER(Material),
                                C.POINTER(u32)], C.c_int),
        "rt_bvh_build_host": ([C.POINTER(Prim), C.POINTER(C.c_float), u32, vp, C.POINTER(u32), C.POINTER(SceneInfo)],
                              C.c_int),
        "rt_sbvh_build_host": ([C.POINTER(Prim), C.POINTER(C.c_float), u32, C.POINTER(vp), C.POINTER(C.POINTER(u32)),
                                C.POINTER(SceneInfo)], C.c_int),
        "rt_image_load": ([C.c_char_p, C.POINTER(C.POINTER(u32)), C.POINTER(u32), C.POINTER(u32)], C.c_int),
        "rt_scene_create": ([C.POINTER(SceneDesc), C.POINTER(vp)], C.c_int),
        "rt_scene_create_recipe": ([C.c_char_p, C.c_char_p, i32, C.POINTER(vp)], C.c_int),
        "rt_scene_create_recipe_ex": ([C.c_char_p, C.c_char_p, i32, i32, C.POINTER(vp)], C.c_int),
        "rt_scene_destroy": ([vp], C.c_int),
        "rt_scene_get_info": ([vp, C.POINTER(SceneInfo)], C.c_int),
        "rt_scene_set_camera_walk": ([vp, C.c_int], C.c_int),
        "rt_scene_copy_bvh": ([vp, vp, C.POINTER(u32)], C.c_int),
        "rt_intersect": ([vp, vp, vp, u32, vp], C.c_int),
        "rt_occluded": ([vp, vp, vp, u32, vp], C.c_int),
        "rt_intersect_host": ([vp, vp, vp, u32], C.c_int),
        "rt_occluded_host": ([vp, vp, vp, u32], C.c_int),
        "rt_intersect_packets": ([vp, vp, vp, u32, vp], C.c_int),
        "rt_intersect_packets_host": ([vp, vp, vp, u32], C.c_int),
        "rt_trace": ([vp, C.c_int, vp, vp, vp, u32, vp, vp, vp, u32, vp], C.c_int),
        "rt_trace_host": ([vp, C.c_int, vp, vp, vp, u32, vp, vp, vp, u32], C.c_int),
        "rt_comm_unique_id": ([vp], C.c_int),
        "rt_comm_create": ([vp, C.c_int, C.c_int, C.c_int, C.POINTER(vp)], C.c_int),
        "rt_comm_wrap": ([vp, C.c_int, C.POINTER(vp)], C.c_int),
        "rt_comm_info": ([vp, C.POINTER(C.c_int), C.POINTER(C.c_int)], C.c_int),
        "rt_comm_destroy": ([vp], C.c_int),
        "rt_render_frame_multi": ([vp, vp, C.POINTER(Camera), C.POINTER(FrameParams), vp, u32, vp], C.c_int),
        "rt_multi_flush": ([vp, vp, vp, vp], C.c_int),
        "rt_comm_timing": ([vp, C.POINTER(C.c_double), C.POINTER(C.c_double), C.POINTER(C.c_uint64)], C.c_int),
        "rt_comm_deal_info": ([vp, C.POINTER(C.c_int), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                               C.POINTER(C.c_uint64)], C.c_int),
        "rt_comm_deal_hash": ([vp, C.POINTER(C.c_uint64)], C.c_int),
        "rt_camera_default": ([u32, u32, C.POINTER(Camera)], C.c_int),
        "rt_renderer_create": ([vp, u32, u32, C.POINTER(vp)], C.c_int),
        "rt_renderer_destroy": ([vp], C.c_int),
        "rt_render_frame": ([vp, C.POINTER(Camera), C.POINTER(FrameParams), vp, vp], C.c_int),
        "rt_render_frame_host": ([vp, C.POINTER(Camera), C.POINTER(FrameParams), vp], C.c_int),
        "rt_shard_capacity": ([u32, u32, u32, C.POINTER(u32)], C.c_int),
        "rt_render_shard": ([vp, C.POINTER(Camera), C.POINTER(FrameParams), u32, u32, vp, vp], C.c_int),
        "rt_assemble_shards": ([vp, vp, u32, vp, vp], C.c_int),
        "rt_tile_deal": ([u32, u32, C.POINTER(u32), u32, C.POINTER(u32), C.POINTER(u32)], C.c_int),
        "rt_render_shard_tiles": ([vp, C.POINTER(Camera), C.POINTER(FrameParams), C.POINTER(u32), u32, vp, vp], C.c_int),
        "rt_assemble_tiles": ([vp, vp, u32, C.POINTER(u32), C.POINTER(u32), u32, vp, vp], C.c_int),
        "rt_renderer_counters": ([vp, C.POINTER(Counters)], C.c_int),
        "rt_renderer_read_accumulator": ([vp, fp], C.c_int),
        "rt_renderer_overlap": ([vp, C.POINTER(C.c_int), fp], C.c_int),
        "rt_renderer_overlap_depth": ([vp, C.POINTER(C.c_int), fp], C.c_int),
        "rt_renderer_device_bytes": ([vp, C.POINTER(C.c_uint64), C.POINTER(C.c_uint32)], C.c_int),
        "rt_renderer_tile_costs": ([vp, C.POINTER(u32), u32, C.POINTER(u32)], C.c_int),
        "rt_renderer_tile_work": ([vp, C.POINTER(Camera), C.POINTER(FrameParams), C.POINTER(u32), u32, vp, vp], C.c_int),
        "rt_renderer_choices": ([vp, C.POINTER(C.c_int), C.POINTER(C.c_int), fp, fp], C.c_int),
        "rt_renderer_set_walk_check": ([vp, C.c_int], C.c_int),
        "rt_renderer_walk_stats": ([vp, C.POINTER(C.c_uint64)], C.c_int),
        "rt_renderer_stream": ([vp, C.POINTER(vp)], C.c_int),
        "rt_frame_kernel_name": ([vp, C.POINTER(FrameParams)], C.c_char_p),
        "rt_synchronize": ([vp], C.c_int),
    }
    for name, (args, res) in sigs.items():
        fn = getattr(L, name)
        fn.argtypes = args
        fn.restype = res
    if L.rt_abi_version() != ABI_VERSION:
        raise RTError(RT_ERR_INVALID, "librtamd.so ABI mismatch")
    _lib = L
    return L


def _check(rc):
    if rc != RT_OK:
        raise RTError(rc, lib().rt_last_error().decode(errors="replace"))
    return rc


def device_count():
    n = C.c_int(0)
    rc = lib().rt_device_count(C.byref(n))
    return n.value if rc == RT_OK else 0


def _fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


# ---------------------------------------------------------------- host-side scene preparation
def load_obj(path):
    """tinyobj-compatible OBJ read (Scene::LoadModel's input): (verts[nv,3] f32, faces[nt,3] i32)."""
    return _take_mesh(lib().rt_obj_load, path)


def load_mesh(path):
    """RTMESH1 container read."""
    return _take_mesh(lib().rt_mesh_load, path)


def _take_mesh(fn, path):
    L = lib()
    vp, fp = C.POINTER(C.c_float)(), C.POINTER(C.c_int32)()
    nv, nt = C.c_uint32(), C.c_uint32()
    _check(fn(os.fsencode(path), C.byref(vp), C.byref(nv), C.byref(fp), C.byref(nt)))
    try:
        V = np.ctypeslib.as_array(vp, shape=(nv.value, 3)).copy() if nv.value else np.zeros((0, 3), np.float32)
        F = np.ctypeslib.as_array(fp, shape=(nt.value, 3)).copy() if nt.value else np.zeros((0, 3), np.int32)
    finally:
        L.rt_free(C.cast(vp, C.c_void_p))
        L.rt_free(C.cast(fp, C.c_void_p))
    return V, F


def save_mesh(path, verts, faces):
    V = np.ascontiguousarray(verts, np.float32)
    F = np.ascontiguousarray(faces, np.int32)
    _check(lib().rt_mesh_save(os.fsencode(path), _fptr(V), len(V), F.ctypes.data_as(C.POINTER(C.c_int32)), len(F)))


def mat4_translate(x, y, z):
    m = np.zeros(16, np.float32)
    _check(lib().rt_mat4_translate(x, y, z, _fptr(m)))
    return m


def mat4_scale(s):
    m = np.zeros(16, np.float32)
    _check(lib().rt_mat4_scale(s, _fptr(m)))
    return m


def mat4_rotate(axis, angle):
    m = np.zeros(16, np.float32)
    _check(lib().rt_mat4_rotate(axis, angle, _fptr(m)))
    return m


def mat4_mul(*ms):
    acc = np.ascontiguousarray(ms[0], np.float32).copy()
    for m in ms[1:]:
        m = np.ascontiguousarray(m, np.float32)
        out = np.zeros(16, np.float32)
        _check(lib().rt_mat4_mul(_fptr(acc), _fptr(m), _fptr(out)))
        acc = out
    return acc


def mesh_to_prims(verts, faces, M, material):
    """Scene::LoadModel's face loop: one triangle per face, vertices TransformPosition'ed by M."""
    V = np.ascontiguousarray(verts, np.float32)
    F = np.ascontiguousarray(faces, np.int32)
    Mm = np.ascontiguousarray(M, np.float32)
    out = (Prim * len(F))()
    _check(lib().rt_mesh_to_prims(_fptr(V), len(V), F.ctypes.data_as(C.POINTER(C.c_int32)), len(F), _fptr(Mm),
                                  material, out))
    return list(out)


def recipe_describe(name, mesh_dir=DATA_DIR):
    """The SURVEY.md 8(d) scene as (prims, materials) lists, without touching a device."""
    L = lib()
    n, m = C.c_uint32(), C.c_uint32()
    _check(L.rt_recipe_describe(name.encode(), os.fsencode(mesh_dir), None, C.byref(n), None, C.byref(m)))
    pa, ma = (Prim * n.value)(), (Material * m.value)()
    _check(L.rt_recipe_describe(name.encode(), os.fsencode(mesh_dir), pa, C.byref(n), ma, C.byref(m)))
    return list(pa), list(ma)


def _transforms(prims):
    """per-primitive mat4 array for cubes / quads (None if the scene has none)"""
    if not any(getattr(p, "T", None) is not None for p in prims):
        return None
    T = np.tile(np.eye(4, dtype=np.float32).reshape(16), (len(prims), 1))
    for i, p in enumerate(prims):
        if getattr(p, "T", None) is not None:
            T[i] = np.asarray(p.T, np.float32).reshape(16)
    return T


def build_bvh_host(prims):
    """Plain binned-SAH BVH on the host (template/scene.h:845-976): (nodes[n,32] u8, indices, info)."""
    arr = (Prim * len(prims))(*prims)
    T = _transforms(prims)
    nodes = np.zeros((2 * len(prims) + 2, 32), np.uint8)
    idx = np.zeros(len(prims), np.uint32)
    info = SceneInfo()
    _check(lib().rt_bvh_build_host(arr, None if T is None else T.ctypes.data_as(C.POINTER(C.c_float)), len(prims),
                                   nodes.ctypes.data_as(C.c_void_p),
                                   idx.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(info)))
    return nodes[:info.nodes_used], idx, _info_dict(info)


def build_sbvh_host(prims):
    """The opt-in spatial-split BVH on the host: (nodes [n, 32] uint8, reference indices, info)."""
    L = lib()
    pa = (Prim * len(prims))(*prims)
    T = _transforms(prims)
    nodes, idx, info = C.c_void_p(), C.POINTER(C.c_uint32)(), SceneInfo()
    _check(L.rt_sbvh_build_host(pa, T.ctypes.data_as(C.POINTER(C.c_float)) if T is not None else None, len(prims),
                                C.byref(nodes), C.byref(idx), C.byref(info)))
    try:
        out_nodes = np.frombuffer(C.string_at(nodes, 32 * info.nodes_used), np.uint8).reshape(-1, 32).copy()
        out_idx = np.ctypeslib.as_array(idx, shape=(info.num_refs,)).copy()
    finally:
        L.rt_free(nodes)
        L.rt_free(C.cast(idx, C.c_void_p))
    return out_nodes, out_idx, _info_dict(info)


def _info_dict(info):
    return {"num_prims": info.num_prims, "nodes_used": info.nodes_used, "depth": info.depth, "max_leaf": info.max_leaf,
            "num_refs": info.num_refs}


def sphere(center, radius, material):
    p = Prim(SPHERE, material)
    p.v[0], p.v[1], p.v[2], p.v[3] = center[0], center[1], center[2], radius
    return p


def plane(normal, distance, material):
    p = Prim(PLANE, material)
    p.v[0], p.v[1], p.v[2], p.v[3] = normal[0], normal[1], normal[2], distance
    return p


def triangle(a, b, c, material):
    p = Prim(TRIANGLE, material)
    for k, q in enumerate((a, b, c)):
        p.v[3 * k], p.v[3 * k + 1], p.v[3 * k + 2] = q
    return p


def material(kind, color=(0, 0, 0), color2=(0, 0, 0), ior=0.0, diffuse=-1.0, texture=-1):
    m = Material(kind)
    m.color[:] = color
    m.color2[:] = color2
    m.ior = ior
    m.diffuse = diffuse
    m.texture = texture
    return m


def cube(pos, size, material, T=None):
    """Primitive::createCube(pos, size, material, T) (Primitive.h:717-728)"""
    p = Prim(CUBE, material)
    p.v[0], p.v[1], p.v[2] = pos
    p.v[3], p.v[4], p.v[5] = (size, size, size) if np.isscalar(size) else size
    p.T = None if T is None else np.asarray(T, np.float32).reshape(16)
    return p


def quad(size, material, T=None):
    """Primitive::createQuad(size, material, T) (Primitive.h:735-739)"""
    p = Prim(QUAD, material)
    p.v[0] = size
    p.T = None if T is None else np.asarray(T, np.float32).reshape(16)
    return p


def tile_deal(width, height, num_shards, cost=None):
    """rt_tile_deal: (deal_tiles[ntiles], deal_off[num_shards + 1]) -- the Morton-ordered 8x8
    tiles cut into runs of equal summed cost (cost[t] per global tile; None = equal)."""
    n = ((width + 7) // 8) * ((height + 7) // 8)
    tiles, off = np.zeros(n, np.uint32), np.zeros(num_shards + 1, np.uint32)
    cp = None
    if cost is not None:
        c = np.ascontiguousarray(cost, np.uint32)
        assert len(c) == n
        cp = c.ctypes.data_as(C.POINTER(C.c_uint32))
    _check(lib().rt_tile_deal(width, height, cp, num_shards, tiles.ctypes.data_as(C.POINTER(C.c_uint32)),
                              off.ctypes.data_as(C.POINTER(C.c_uint32))))
    return tiles, off


def load_image(path):
    """Surface(file) / Surface::LoadImage (template/template.cpp:1571-1601): uint32 [h, w] 0x00RRGGBB."""
    L = lib()
    px = C.POINTER(C.c_uint32)()
    w, h = C.c_uint32(), C.c_uint32()
    _check(L.rt_image_load(os.fsencode(path), C.byref(px), C.byref(w), C.byref(h)))
    try:
        return np.ctypeslib.as_array(px, shape=(h.value, w.value)).copy()
    finally:
        L.rt_free(px)


# ---------------------------------------------------------------- device objects
def _torch():
    import torch
    return torch


def _as_device_rays(rays, device):
    torch = _torch()
    if isinstance(rays, torch.Tensor):
        t = rays
    else:
        t = torch.from_numpy(np.ascontiguousarray(rays, np.float32).reshape(-1, 7))
    return t.to(device=f"cuda:{device}", dtype=torch.float32).contiguous().reshape(-1, 7)


class Scene:
    """Scene (template/scene.h:37): primitives + materials + plain BVH, resident in HBM."""

    def __init__(self, prims=None, materials=None, sky=None, bvh=None, device=0, textures=(), _handle=None,
                 bvh_kind=BVH_PLAIN):
        """prims: Prim records (cube()/quad() carry their mat4 in .T); textures: uint32 [h, w]
        arrays of 0x00RRGGBB referenced by texture_material(index)."""
        self.L = lib()
        self.device = device
        self.h = C.c_void_p()
        if _handle is not None:
            self.h = _handle
            return
        pa = (Prim * len(prims))(*prims)
        ma = (Material * len(materials))(*materials)
        d = SceneDesc()
        d.prims, d.num_prims = pa, len(prims)
        d.materials, d.num_materials = ma, len(materials)
        d.device = device
        d.bvh_kind = bvh_kind
        keep = []
        if sky is not None:
            sky = np.ascontiguousarray(sky, np.uint32)
            d.sky_pixels = sky.ctypes.data_as(C.POINTER(C.c_uint32))
            d.sky_height, d.sky_width = sky.shape
            keep.append(sky)
        T = _transforms(prims)
        if T is not None:
            d.transforms = T.ctypes.data_as(C.POINTER(C.c_float))
            keep.append(T)
        if len(textures):
            texs = [np.ascontiguousarray(t, np.uint32) for t in textures]
            ta = (Texture * len(texs))()
            for k, t in enumerate(texs):
                ta[k].pixels = t.ctypes.data_as(C.POINTER(C.c_uint32))
                ta[k].height, ta[k].width = t.shape
            d.textures, d.num_textures = ta, len(texs)
            keep += texs + [ta]
        if bvh is not None:
            nodes, idx = np.ascontiguousarray(bvh[0], np.uint8), np.ascontiguousarray(bvh[1], np.uint32)
            d.bvh_nodes = nodes.ctypes.data_as(C.c_void_p)
            d.bvh_num_nodes = len(nodes)
            d.bvh_indices = idx.ctypes.data_as(C.POINTER(C.c_uint32))
            keep += [nodes, idx]
        _check(self.L.rt_scene_create(C.byref(d), C.byref(self.h)))

    @classmethod
    def recipe(cls, name, mesh_dir=DATA_DIR, device=0, bvh_kind=BVH_PLAIN):
        """One of the SURVEY.md 8(d) benchmark scenes ("teapotF", "teapot", "mig16", "cfg3", "cfg5");
        bvh_kind BVH_SBVH builds the opt-in spatial-split tree."""
        h = C.c_void_p()
        _check(lib().rt_scene_create_recipe_ex(name.encode(), os.fsencode(mesh_dir), device, bvh_kind, C.byref(h)))
        return cls(device=device, _handle=h)

    def close(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.L.rt_scene_destroy(h)
            self.h = None

    __del__ = close

    @property
    def info(self):
        i = SceneInfo()
        _check(self.L.rt_scene_get_info(self.h, C.byref(i)))
        return _info_dict(i)

    def bvh(self):
        info = self.info
        nodes = np.zeros((info["nodes_used"], 32), np.uint8)
        idx = np.zeros(info["num_refs"], np.uint32)
        _check(self.L.rt_scene_copy_bvh(self.h, nodes.ctypes.data_as(C.c_void_p),
                                        idx.ctypes.data_as(C.POINTER(C.c_uint32))))
        return nodes, idx

    def IntersectBVH(self, rays, stream=None):
        """Batched Scene::IntersectBVH.  rays: (n,7) [O, D, tmax] numpy or torch.
        Returns (t f32, obj i32, u f32, v f32) torch tensors on the scene's device."""
        torch = _torch()
        r = _as_device_rays(rays, self.device)
        n = r.shape[0]
        hits = torch.empty((n, 4), dtype=torch.float32, device=r.device)
        if n:
            s = stream if stream is not None else torch.cuda.current_stream(r.device).cuda_stream
            _check(self.L.rt_intersect(self.h, C.c_void_p(r.data_ptr()), C.c_void_p(hits.data_ptr()), n, C.c_void_p(s)))
        return hits[:, 0], hits.view(torch.int32)[:, 1], hits[:, 2], hits[:, 3]

    def set_camera_walk(self, walk):
        """WALK_LANE, WALK_WAVE or WALK_AUTO (default): how camera rays walk the BVH (same results)."""
        _check(self.L.rt_scene_set_camera_walk(self.h, walk))

    def IntersectBVHPacket(self, rays, stream=None):
        """Batched Scene::IntersectBVHPacket: rays [64k, 64k+64) form packet k."""
        torch = _torch()
        r = _as_device_rays(rays, self.device)
        n = r.shape[0]
        hits = torch.empty((n, 4), dtype=torch.float32, device=r.device)
        if n:
            s = stream if stream is not None else torch.cuda.current_stream(r.device).cuda_stream
            _check(self.L.rt_intersect_packets(self.h, C.c_void_p(r.data_ptr()), C.c_void_p(hits.data_ptr()), n,
                                               C.c_void_p(s)))
        return hits[:, 0], hits.view(torch.int32)[:, 1], hits[:, 2], hits[:, 3]

    def IsOccluded(self, rays, stream=None):
        """Batched Scene::IsOccluded: bool tensor."""
        torch = _torch()
        r = _as_device_rays(rays, self.device)
        n = r.shape[0]
        out = torch.empty(n, dtype=torch.uint8, device=r.device)
        if n:
            s = stream if stream is not None else torch.cuda.current_stream(r.device).cuda_stream
            _check(self.L.rt_occluded(self.h, C.c_void_p(r.data_ptr()), C.c_void_p(out.data_ptr()), n, C.c_void_p(s)))
        return out.bool()

    def trace(self, rays, seeds, depth=10, last_specular=True, inside=False, mode=MODE_PATH, hits=False,
              stream=None):
        """Batched Renderer::Trace(ray, lastSpecular, depth) (renderer.cpp:17-72), or WhittedTrace
        (renderer.cpp:138-195) with mode=MODE_WHITTED.  rays: (n, 7); seeds: n uint32 RNG states.
        last_specular / inside: bool or per-ray arrays.  Returns (radiance [n, 3] f32, seeds after
        the call [n] int32 holding the uint32 bits, ray counts {"shadow", "bounce"}[, hits as in
        IntersectBVH]) as torch tensors on the scene's device."""
        torch = _torch()
        r = _as_device_rays(rays, self.device)
        n = r.shape[0]
        dev = r.device
        sd = torch.as_tensor(np.asarray(seeds, np.uint32).view(np.int32) if not isinstance(seeds, torch.Tensor)
                             else seeds, dtype=torch.int32).to(dev).clone().reshape(-1)
        if sd.numel() != n:
            raise RTError(RT_ERR_INVALID, "one seed per ray")
        ls = np.broadcast_to(np.asarray(last_specular, bool), (n,))
        ins = np.broadcast_to(np.asarray(inside, bool), (n,))
        flags = torch.from_numpy((ls.astype(np.uint8) | (ins.astype(np.uint8) << 1)).copy()).to(dev)
        rad = torch.empty((n, 3), dtype=torch.float32, device=dev)
        counts = torch.zeros(2, dtype=torch.int64, device=dev)
        hit = torch.empty((n, 4), dtype=torch.float32, device=dev) if hits else None
        if n:
            s = stream if stream is not None else torch.cuda.current_stream(dev).cuda_stream
            _check(self.L.rt_trace(self.h, mode, C.c_void_p(r.data_ptr()), C.c_void_p(sd.data_ptr()),
                                   C.c_void_p(flags.data_ptr()), depth, C.c_void_p(rad.data_ptr()),
                                   C.c_void_p(hit.data_ptr()) if hits else None, C.c_void_p(counts.data_ptr()), n,
                                   C.c_void_p(s)))
        out = (rad, sd, counts)
        if hits:
            out += ((hit[:, 0], hit.view(torch.int32)[:, 1], hit[:, 2], hit[:, 3]),)
        return out

    def intersect_host(self, rays):
        """Host-array variant (copies through the library's staging buffer)."""
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 7)
        hits = np.zeros(len(rays), HIT_DTYPE)
        _check(self.L.rt_intersect_host(self.h, rays.ctypes.data_as(C.c_void_p), hits.ctypes.data_as(C.c_void_p),
                                        len(rays)))
        return hits

    def intersect_packets_host(self, rays):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 7)
        hits = np.zeros(len(rays), HIT_DTYPE)
        _check(self.L.rt_intersect_packets_host(self.h, rays.ctypes.data_as(C.c_void_p),
                                                hits.ctypes.data_as(C.c_void_p), len(rays)))
        return hits

    def occluded_host(self, rays):
        rays = np.ascontiguousarray(rays, np.float32).reshape(-1, 7)
        out = np.zeros(len(rays), np.uint8)
        _check(self.L.rt_occluded_host(self.h, rays.ctypes.data_as(C.c_void_p), out.ctypes.data_as(C.c_void_p),
                                       len(rays)))
        return out.astype(bool)


class Renderer:
    """Renderer (renderer.h:5-160): owns the float4 accumulator; Tick = one frame."""

    def __init__(self, scene, width, height):
        self.L = lib()
        self.scene = scene
        self.width, self.height = width, height
        self.camera = Camera.default(width, height)
        self.h = C.c_void_p()
        _check(self.L.rt_renderer_create(scene.h, width, height, C.byref(self.h)))
        self.frame = 0
        self.mode = MODE_PATH     # MODE_PATH / MODE_WHITTED / MODE_PACKET (the PACKET_TRAVERSAL build)

    @property
    def useWhitted(self):       # renderer.h:158; toggled by the K key (renderer.h:138)
        return self.mode == MODE_WHITTED

    @useWhitted.setter
    def useWhitted(self, on):
        self.mode = MODE_WHITTED if on else MODE_PATH

    def Trace(self, rays, seeds, lastSpecular=True, depth=10, stream=None):
        """Renderer::Trace (renderer.h:9) on a batch of rays with per-ray RNG states; returns
        (radiance [n, 3], seeds after the call) on the device (Scene.trace)."""
        rad, sd, _ = self.scene.trace(rays, seeds, depth=depth, last_specular=lastSpecular, stream=stream)
        return rad, sd

    def WhittedTrace(self, rays, seeds, depth=20, stream=None):
        """Renderer::WhittedTrace (renderer.h:13) on a batch of rays."""
        rad, sd, _ = self.scene.trace(rays, seeds, depth=depth, mode=MODE_WHITTED, stream=stream)
        return rad, sd

    def close(self):
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.L.rt_renderer_destroy(h)
            self.h = None

    __del__ = close

    def params(self, spp=1, depth=None, frame=None, reset=False):
        mode = self.mode
        depth = DEFAULT_DEPTH[mode] if depth is None else depth
        return FrameParams(self.width, self.height, spp, depth, self.frame if frame is None else frame, mode,
                           int(reset))

    def Tick(self, out=None, spp=1, depth=None, frame=None, reset=False, stream=None):
        """Renderer::Tick: trace, accumulate, pack RGB8 into out (torch uint32/int32 [H*W] on device)."""
        torch = _torch()
        if out is None:
            out = torch.empty(self.width * self.height, dtype=torch.int32, device=f"cuda:{self.scene.device}")
        p = self.params(spp, depth, frame, reset)
        s = stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream
        _check(self.L.rt_render_frame(self.h, C.byref(self.camera), C.byref(p), C.c_void_p(out.data_ptr()),
                                      C.c_void_p(s)))
        if frame is None:
            self.frame += 1
        return out

    def tick_host(self, spp=1, depth=None, frame=None, reset=False):
        """Renderer::Tick with the RGB8 frame returned in host memory (numpy uint32 [H*W])."""
        out = np.zeros(self.width * self.height, np.uint32)
        p = self.params(spp, depth, frame, reset)
        _check(self.L.rt_render_frame_host(self.h, C.byref(self.camera), C.byref(p), out.ctypes.data_as(C.c_void_p)))
        if frame is None:
            self.frame += 1
        return out

    def shard_capacity(self, num_shards):
        n = C.c_uint32()
        _check(self.L.rt_shard_capacity(self.width, self.height, num_shards, C.byref(n)))
        return n.value

    def render_shard(self, out, shard, num_shards, spp=1, depth=None, frame=None, reset=False, stream=None):
        torch = _torch()
        p = self.params(spp, depth, frame, reset)
        s = stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream
        _check(self.L.rt_render_shard(self.h, C.byref(self.camera), C.byref(p), shard, num_shards,
                                      C.c_void_p(out.data_ptr()), C.c_void_p(s)))
        if frame is None:
            self.frame += 1
        return out

    def render_shard_tiles(self, out, tiles, spp=1, depth=None, frame=None, reset=False, stream=None):
        """rt_render_shard_tiles: the listed global tiles (an explicit deal's share), packed [i][64]."""
        torch = _torch()
        p = self.params(spp, depth, frame, reset)
        t = np.ascontiguousarray(tiles, np.uint32)
        s = stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream
        _check(self.L.rt_render_shard_tiles(self.h, C.byref(self.camera), C.byref(p), t.ctypes.data_as(C.POINTER(C.c_uint32)),
                                            len(t), C.c_void_p(out.data_ptr()), C.c_void_p(s)))
        if frame is None:
            self.frame += 1
        return out

    def assemble_tiles(self, gathered, stride_px, deal_tiles, deal_off, out, stream=None):
        """rt_assemble_tiles: shard k's packed tiles at gathered[k * stride_px:] -> out (row-major)."""
        torch = _torch()
        dt = np.ascontiguousarray(deal_tiles, np.uint32)
        do = np.ascontiguousarray(deal_off, np.uint32)
        s = stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream
        _check(self.L.rt_assemble_tiles(self.h, C.c_void_p(gathered.data_ptr()), stride_px,
                                        dt.ctypes.data_as(C.POINTER(C.c_uint32)), do.ctypes.data_as(C.POINTER(C.c_uint32)),
                                        len(do) - 1, C.c_void_p(out.data_ptr()), C.c_void_p(s)))
        return out

    def assemble(self, gathered, num_shards, out, stream=None):
        torch = _torch()
        s = stream if stream is not None else torch.cuda.current_stream(out.device).cuda_stream
        _check(self.L.rt_assemble_shards(self.h, C.c_void_p(gathered.data_ptr()), num_shards,
                                         C.c_void_p(out.data_ptr()), C.c_void_p(s)))
        return out

    def kernel_name(self, spp=1, depth=None):
        """The frame kernel Tick launches for these params (rocprofv3 name, abbreviated)."""
        name = self.L.rt_frame_kernel_name(self.h, C.byref(self.params(spp, depth)))
        if name is None:
            raise RTError(-1, self.L.rt_last_error().decode())
        return name.decode()

    def counters(self):
        c = Counters()
        _check(self.L.rt_renderer_counters(self.h, C.byref(c)))
        return {n: int(getattr(c, n)) for n, _ in Counters._fields_}

    def overlap(self):
        """Overlapped primary+shadow frames: (state, group ms) -- state 1 overlapped, 0 serial,
        -1 not decided yet; ms = the timed groups (serial, overlapped, overlapped, serial)."""
        st = C.c_int()
        ms = np.zeros(4, np.float32)
        _check(self.L.rt_renderer_overlap(self.h, C.byref(st), _fptr(ms)))
        return st.value, [round(float(x), 4) for x in ms]

    def overlap_depth(self):
        """Primary+shadow frames in flight: (depth, group ms) -- 1 serial, 2..6 overlapped, -1 not
        decided yet; ms = the timed groups (serial, 2, 4, 6, 6, 4, 2, serial or serial, 2, 2, serial)."""
        d = C.c_int()
        ms = np.zeros(8, np.float32)
        _check(self.L.rt_renderer_overlap_depth(self.h, C.byref(d), _fptr(ms)))
        return d.value, [round(float(x), 4) for x in ms]

    def device_bytes(self):
        """(bytes of device memory the renderer holds, overlapped-frame result buffers allocated)."""
        b, n = C.c_uint64(), C.c_uint32()
        _check(self.L.rt_renderer_device_bytes(self.h, C.byref(b), C.byref(n)))
        return b.value, n.value

    def choices(self):
        """Timed choices of the current parameter set: {walk: 0 lane / 1 wave / -1, split: 1 / 0 / -1,
        walk_ms, split_ms} (groups A, B, B, A)."""
        w, sp = C.c_int(), C.c_int()
        wm, sm = np.zeros(4, np.float32), np.zeros(4, np.float32)
        _check(self.L.rt_renderer_choices(self.h, C.byref(w), C.byref(sp), _fptr(wm), _fptr(sm)))
        return {"walk": w.value, "split": sp.value, "walk_ms": [round(float(x), 4) for x in wm],
                "split_ms": [round(float(x), 4) for x in sm]}

    def set_walk_check(self, level):
        """WALK_CHECK_OFF (default) / WALK_CHECK_COUNT / WALK_CHECK_VERIFY (rt_renderer_set_walk_check)."""
        _check(self.L.rt_renderer_set_walk_check(self.h, level))

    def walk_stats(self):
        """The wave camera walk's cumulative counters: {walked, margin_boxes, retraced, verify_mismatch}."""
        out = (C.c_uint64 * 4)()
        _check(self.L.rt_renderer_walk_stats(self.h, out))
        return {"walked": int(out[0]), "margin_boxes": int(out[1]), "retraced": int(out[2]), "verify_mismatch": int(out[3])}

    def tile_costs(self):
        """Per-local-tile wave cycles behind the measured tile order (empty until recorded)."""
        n = C.c_uint32()
        _check(self.L.rt_renderer_tile_costs(self.h, None, 0, C.byref(n)))
        out = np.zeros(n.value, np.uint32)
        if n.value:
            _check(self.L.rt_renderer_tile_costs(self.h, out.ctypes.data_as(C.POINTER(C.c_uint32)), n.value, C.byref(n)))
        return out

    def tile_work(self, spp=1, depth=None, frame=None, pixels=False, stream=None):
        """Deterministic work map of one frame (rt_renderer_tile_work, a dry run: nothing rendered):
        per row-major tile, node visits + primitive tests of its rays.  pixels=True also returns the
        per-pixel counters [H*W, 8] (closest-hit nodes, closest-hit prims, any-hit nodes, any-hit prims,
        closest-hit pops of interior / leaf entries already beyond the ray's t, 0, 0)."""
        tx, ty = (self.width + 7) // 8, (self.height + 7) // 8
        work = np.zeros(tx * ty, np.uint32)
        p = self.params(spp, depth, frame)
        buf = None
        if pixels:
            torch = _torch()
            buf = torch.zeros(self.width * self.height * 8, dtype=torch.int32, device=f"cuda:{self.scene.device}")
        _check(self.L.rt_renderer_tile_work(self.h, C.byref(self.camera), C.byref(p),
                                            work.ctypes.data_as(C.POINTER(C.c_uint32)), len(work),
                                            None if buf is None else C.c_void_p(buf.data_ptr()),
                                            None if stream is None else C.c_void_p(stream)))
        if buf is None:
            return work
        return work, buf.view(-1, 8).cpu().numpy().view(np.uint32)

    def accumulator(self):
        acc = np.zeros((self.height * self.width, 4), np.float32)
        _check(self.L.rt_renderer_read_accumulator(self.h, _fptr(acc)))
        return acc
