"""Host-side checks of librtamd.so that need no GPU: exports, OBJ/mesh reading, mat4,
camera, BVH build (vs the oracle's restatement of template/scene.h:845-976), errors."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

from conftest import ROOT


def header_functions():
    text = open(os.path.join(ROOT, "include", "rt_amd.h")).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(rt_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_header_symbol(rt):
    names = header_functions()
    assert len(names) >= 30
    out = subprocess.run(["nm", "-D", "--defined-only", rt.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (rt_\w+)$", out, flags=re.M))
    missing = [n for n in names if n not in exported]
    assert not missing, missing
    lib = ctypes.CDLL(rt.LIB_PATH)
    for n in names:
        assert getattr(lib, n)


def test_library_is_gfx950_code_object(rt, tmp_path):
    # --offloading extracts the bundled code objects next to its input: run it on a copy
    import shutil
    lib = shutil.copy(rt.LIB_PATH, tmp_path / "librtamd.so")
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                         capture_output=True, text=True, cwd=tmp_path)
    text = out.stdout + out.stderr
    assert "gfx950" in text


def build_compat_host(rt, tmp_path):
    exe = tmp_path / "compat_host"
    # plain g++ host (hipMalloc for the device frame of rt_render_frame_multi: HIP host API only)
    subprocess.run(["g++", "-std=c++17", "-Wall", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"),
                    "-I", "/opt/rocm/include", os.path.join(ROOT, "tests", "cpp", "compat_host.cpp"), "-o", str(exe),
                    rt.LIB_PATH, "-L/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{os.path.dirname(rt.LIB_PATH)}",
                    "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return str(exe)


def test_compat_header_compiles(rt, tmp_path):
    """The reference-shaped C++ host builds against the header and links the library;
    without a GPU it must fail loudly with RT_ERR_NO_DEVICE (exit 3), never fall back."""
    exe = build_compat_host(rt, tmp_path)
    r = subprocess.run([exe, rt.DATA_DIR], capture_output=True, text=True)
    if rt.device_count() == 0:
        assert r.returncode == 3, r.stdout
    else:
        assert r.returncode == 0, r.stdout


def test_reference_shaped_host(rt):
    """tests/cpp/reference_main.cpp: the reference's main (template/template.cpp:133-139, 269-287)
    and float3 math with only `#include "precomp.h"` swapped for rt_compat.hpp -- Surface,
    `new Renderer()`, Init, Tick(float), the K key, Shutdown; the default scene from the bundled
    meshes.  Without a GPU it must stop with RT_ERR_NO_DEVICE (exit 3) after the host-side
    checks passed; with one, frames come back (exit 0)."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "cpp"), "reference_main"], check=True)
    env = dict(os.environ, RT_MESH_DIR=rt.DATA_DIR)
    r = subprocess.run([os.path.join(ROOT, "tests", "cpp", "reference_main")], capture_output=True, text=True, env=env)
    assert r.returncode == (3 if rt.device_count() == 0 else 0), r.stdout + r.stderr


def test_default_recipe_from_reference_assets(rt, oracle, reference_assets):
    """Recipe "default" = the reference's as-shipped Scene() (template/scene.h:40-128): read from
    the reference's own assets/*.obj (the recipe loader falls back to OBJ files) it equals the
    bundled-mesh recipe bit for bit, and its plain BVH equals the oracle's."""
    pa, ma = rt.recipe_describe("default")
    pb, mb = rt.recipe_describe("default", mesh_dir=reference_assets)
    raw = lambda xs: b"".join(bytes(x) for x in xs)
    assert len(pa) == 1 + 21364 + 6546 and raw(pa) == raw(pb) and raw(ma) == raw(mb)
    nodes, idx, info = rt.build_bvh_host(pa)
    o = oracle.Scene("default", rt.DATA_DIR)
    on = o.nodes().copy()
    nodes = nodes.copy()
    on[1] = 0
    nodes[1] = 0
    assert info["nodes_used"] == o.nodes_used and np.array_equal(nodes, on) and np.array_equal(idx, o.indices())


def test_abi_version_and_device_count(rt):
    assert rt.lib().rt_abi_version() == rt.ABI_VERSION == 4
    assert rt.device_count() >= 0


@pytest.mark.parametrize("name", ["teapot", "mig29", "Shiba", "glider"])
def test_obj_loader_matches_oracle_and_bundled_mesh(rt, oracle, reference_assets, name):
    path = os.path.join(reference_assets, name + ".obj")
    V, F = rt.load_obj(path)
    V2, F2 = oracle.obj_parse(path)
    assert np.array_equal(V.view(np.uint32), V2.view(np.uint32))
    assert np.array_equal(F, F2)
    Vb, Fb = rt.load_mesh(os.path.join(rt.DATA_DIR, name + ".rtmesh"))
    assert np.array_equal(V.view(np.uint32), Vb.view(np.uint32)) and np.array_equal(F, Fb)


def test_bundled_mesh_sizes(rt):
    # teapot 1,024 tris; mig29 6,546; Shiba 15,252; glider 21,364
    want = {"teapot": 1024, "mig29": 6546, "Shiba": 15252, "glider": 21364}
    for n, nt in want.items():
        V, F = rt.load_mesh(os.path.join(rt.DATA_DIR, n + ".rtmesh"))
        assert len(F) == nt and F.min() >= 0 and F.max() < len(V)


def test_obj_parser_edge_cases(rt, oracle, tmp_path):
    p = tmp_path / "edge.obj"
    p.write_text("# comment\r\n"
                 "v 1 2 3\r\n"
                 "v  -0.5e+1 .25 -.125\n"
                 "v 4.90876e-009 1E2 +7\n"
                 "v 1.12345678901 2 3\n"
                 "\n"
                 "vn 0 0 1\n"
                 "f 1 2 3\n"
                 "f -4/1/1 -3//1 -2 -1\n"
                 "f 1 2\n")
    V, F = rt.load_obj(str(p))
    V2, F2 = oracle.obj_parse(str(p))
    assert np.array_equal(V.view(np.uint32), V2.view(np.uint32)) and np.array_equal(F, F2)
    assert V.shape == (4, 3) and F.shape == (3, 3)   # triangle + split quad; the 2-vertex face is dropped
    assert V[1, 0] == np.float32(-5.0) and V[2, 1] == np.float32(100.0)


def test_obj_errors(rt, tmp_path):
    with pytest.raises(rt.RTError) as e:
        rt.load_obj(str(tmp_path / "missing.obj"))
    assert e.value.code == rt.RT_ERR_IO
    bad = tmp_path / "bad.obj"
    bad.write_text("v 0 0 0\nf 0 1 2\n")
    with pytest.raises(rt.RTError):
        rt.load_obj(str(bad))


def test_mat4_matches_oracle(rt, oracle):
    import ctypes as C
    L = oracle.lib()
    fp = C.POINTER(C.c_float)
    for axis, fn in enumerate(("or_mat4_rotate_x", "or_mat4_rotate_y", "or_mat4_rotate_z")):
        for a in (0.3, -0.55 * np.pi, 1.1 * np.pi):
            ref = np.zeros(16, np.float32)
            getattr(L, fn).argtypes = [fp, C.c_float]
            getattr(L, fn)(ref.ctypes.data_as(fp), a)
            got = rt.mat4_rotate(axis, a)
            assert np.array_equal(ref.view(np.uint32), got.view(np.uint32))
    T, R, S = rt.mat4_translate(0, 0, 2), rt.mat4_rotate(1, np.float32(0.5) * np.float32(np.pi)), rt.mat4_scale(2.5)
    M = rt.mat4_mul(T, R, S)
    assert M[3] == np.float32(0) and M[11] == np.float32(2) and M[15] == 1


def test_camera_default_matches_oracle(rt, oracle):
    for W, H in ((1280, 720), (1920, 1080), (100, 75)):
        c = rt.Camera.default(W, H)
        o = oracle.Scene.camera(W, H)
        for f in ("pos", "tl", "tr", "bl"):
            g = {"tl": "top_left", "tr": "top_right", "bl": "bottom_left"}.get(f, f)
            assert list(getattr(c, g)) == list(getattr(o, f))
        assert np.float32(c.lens_radius) == np.float32(o.lens_radius)


@pytest.mark.parametrize("name", ["teapotF", "teapot", "mig16", "cfg3", "cfg5"])
def test_bvh_identical_to_oracle(rt, oracle, name):
    prims, mats = rt.recipe_describe(name)
    nodes, idx, info = rt.build_bvh_host(prims)
    o = oracle.Scene(name, rt.DATA_DIR)
    on = o.nodes().copy()
    nodes = nodes.copy()
    on[1] = 0
    nodes[1] = 0          # node 1 is the unused alignment slot (template/scene.h:849)
    assert info["nodes_used"] == o.nodes_used and info["depth"] == o.depth
    assert np.array_equal(nodes, on)
    assert np.array_equal(idx, o.indices())


def test_parallel_bvh_build_matches_oracle_on_soups(rt, oracle):
    """The thread-pool builder renumbers to the recursion's order: identical trees on
    large random soups (clustered + uniform), with cubes / quads / spheres mixed in."""
    import ctypes as C
    rng = np.random.default_rng(3)
    n = 60000
    centers = np.concatenate([rng.normal(0, 0.3, (n // 2, 3)), rng.uniform(-5, 5, (n - n // 2, 3))]).astype(np.float32)
    V = (centers[:, None, :] + rng.normal(0, 0.02, (n, 3, 3))).astype(np.float32)
    prims = [rt.sphere((0, 4, -2), 0.5, 0)] + [rt.triangle(*map(tuple, V[i]), 0) for i in range(n)]
    prims += [rt.cube((0.5, 0, 0), (0.3, 0.2, 0.4), 0, rt.mat4_rotate(1, 0.4)), rt.quad(0.7, 0, rt.mat4_translate(1, 1, 1)),
              rt.sphere((1, 2, 3), 0.25, 0)]
    nodes, idx, info = rt.build_bvh_host(prims)
    L = oracle.lib()
    h = L.or_scene_new()
    f3 = lambda *v: (C.c_float * 3)(*v)
    f16 = lambda T: (C.c_float * 16)(*(np.eye(4, dtype=np.float32).reshape(16) if T is None else T))
    L.or_scene_add_material(h, 0, f3(1, 1, 1), f3(0, 0, 0), 0.0, -1.0)
    for p in prims:
        v = list(p.v)
        if p.type == rt.SPHERE:
            L.or_scene_add_sphere(h, f3(*v[:3]), v[3], 0)
        elif p.type == rt.CUBE:
            L.or_scene_add_cube(h, f3(*v[:3]), f3(*v[3:6]), f16(p.T), 0)
        elif p.type == rt.QUAD:
            L.or_scene_add_quad(h, v[0], f16(p.T), 0)
        else:
            L.or_scene_add_triangle(h, f3(*v[:3]), f3(*v[3:6]), f3(*v[6:9]), 0)
    L.or_scene_build_bvh(h)
    o = oracle.Scene.__new__(oracle.Scene)
    o.L, o.h = L, h
    on = o.nodes().copy()
    nodes = nodes.copy()
    on[1] = 0
    nodes[1] = 0
    assert info["nodes_used"] == o.nodes_used and info["depth"] == o.depth
    assert np.array_equal(nodes, on)
    assert np.array_equal(idx, o.indices())


def test_bvh_small_and_degenerate_inputs(rt):
    light = rt.sphere((0, 4, -2), 0.5, 0)
    # a single primitive: the root is a leaf (maxDepthBVH returns 1)
    nodes, idx, info = rt.build_bvh_host([light])
    assert info["nodes_used"] == 2 and info["depth"] == 1 and list(idx) == [0]
    # coincident centroids cannot be split: one leaf holding all of them
    tris = [light] + [rt.triangle((0, 0, 1), (1, 0, 1), (0, 1, 1), 0) for _ in range(5)]
    nodes, idx, info = rt.build_bvh_host(tris)
    assert info["max_leaf"] >= 5


def test_scene_creation_without_device_fails_loudly(rt):
    if rt.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises(rt.RTError) as e:
        rt.Scene.recipe("teapotF")
    assert e.value.code == rt.RT_ERR_NO_DEVICE


def test_unknown_recipe(rt):
    with pytest.raises(rt.RTError) as e:
        rt.recipe_describe("nope")
    assert e.value.code == rt.RT_ERR_INVALID


def test_prebuilt_bvh_above_24bit_node_index_is_refused(rt):
    """The device node word packs leftFirst << 8 | count: interior child indices are 24 bits
    wide, so a tree with more than 2^24 nodes must be refused (before any device call), not
    silently truncated.  The count is checked before the node array is read."""
    import ctypes as C
    light = rt.sphere((0, 4, -2), 0.5, 0)
    pa = (rt.Prim * 1)(light)
    ma = (rt.Material * 1)(rt.material(rt.LIGHT, (1, 1, 1)))
    nodes = np.zeros((4, 32), np.uint8)
    idx = np.zeros(1, np.uint32)
    d = rt.SceneDesc()
    d.prims, d.num_prims = pa, 1
    d.materials, d.num_materials = ma, 1
    d.bvh_nodes = nodes.ctypes.data_as(C.c_void_p)
    d.bvh_num_nodes = (1 << 24) + 2
    d.bvh_indices = idx.ctypes.data_as(C.POINTER(C.c_uint32))
    h = C.c_void_p()
    rc = rt.lib().rt_scene_create(C.byref(d), C.byref(h))
    assert rc == rt.RT_ERR_UNSUPPORTED, rt.lib().rt_last_error()
    assert b"2^24" in rt.lib().rt_last_error()


def test_renderer_overlap_query_rejects_null_arguments(rt):
    """rt_renderer_overlap (overlapped primary+shadow frames' state) checks its arguments on
    the host before touching the renderer: no GPU needed."""
    import ctypes as C
    L = rt.lib()
    st = C.c_int(7)
    assert L.rt_renderer_overlap(None, C.byref(st), None) == rt.RT_ERR_INVALID
    assert st.value == 7
    assert b"rt_renderer_overlap" in L.rt_last_error()
