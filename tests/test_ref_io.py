"""The OBJ and PNG readers pinned to the reference's OWN code: tinyobjloader
(template/tiny_obj_loader.h) and stb_image (lib/stb_image.h), vendored by the reference and
compiled unmodified from /root/reference into oracle/_ref/libref_io.so (oracle/ref_io.cpp,
`make -C oracle ref`).  They decide every triangle's vertex bits and primitive id
(Scene::LoadModel, template/scene.h:156-201) and every texel (Surface::LoadImage,
template/template.cpp:1579-1601).

In this container the reference itself is the checker; on the GPU box (no /root/reference)
the committed tinyobj / stb digests of tests/golden/ref_meshes.json pin the bundled meshes."""
import hashlib
import json
import os

import numpy as np
import pytest

import pngref
from conftest import ROOT

GOLDEN = os.path.join(ROOT, "tests", "golden", "ref_meshes.json")
MESHES = ["teapot", "mig29", "Shiba", "glider"]
IMAGES = ["earth", "logo", "font"]


@pytest.fixture(scope="module")
def refio():
    import refio as m
    if not m.available():
        pytest.skip("reference sources not present (GPU box): tests/golden/ref_meshes.json pins the meshes there")
    m.build()
    return m


def tri_digest(V, F):
    """sha256 of the triangles' float32 vertex bits in primitive-id order (what LoadModel feeds
    Primitive::createTriangle, before TransformPosition)."""
    return hashlib.sha256(np.ascontiguousarray(V[F], np.float32).tobytes()).hexdigest()


@pytest.mark.parametrize("name", MESHES)
def test_obj_load_equals_tinyobj(rt, oracle, refio, reference_assets, name):
    """rt_obj_load (and the oracle's parser, and the bundled .rtmesh) give tinyobj's vertex
    bits and LoadModel's triangle order, bit for bit."""
    path = os.path.join(reference_assets, name + ".obj")
    Vr, Fr = refio.load_model(path)
    V, F = rt.load_obj(path)
    assert np.array_equal(V.view(np.uint32), Vr.view(np.uint32))
    assert np.array_equal(F, Fr)
    Vo, Fo = oracle.obj_parse(path)
    assert np.array_equal(Vo.view(np.uint32), Vr.view(np.uint32)) and np.array_equal(Fo, Fr)
    Vb, Fb = rt.load_mesh(os.path.join(rt.DATA_DIR, name + ".rtmesh"))
    assert np.array_equal(Vb.view(np.uint32), Vr.view(np.uint32)) and np.array_equal(Fb, Fr)


def test_bundled_meshes_match_tinyobj_digests(rt):
    """Runs everywhere (GPU box included): the bundled meshes the scene recipes load hash to
    the digests tinyobj produced from the reference's assets (tests/golden/make_ref_fixtures.py)."""
    with open(GOLDEN) as f:
        g = json.load(f)
    for name in MESHES:
        V, F = rt.load_mesh(os.path.join(rt.DATA_DIR, name + ".rtmesh"))
        want = g["meshes"][name]
        assert (len(V), len(F)) == (want["vertices"], want["triangles"])
        assert tri_digest(V, F) == want["triangles_sha256"], name


def _fmt_float(rng, x):
    k = rng.integers(0, 9)
    if k == 0:
        return f"{x:.6f}"
    if k == 1:
        return f"{x:.9e}"
    if k == 2:
        return f"{x:.3E}"
    if k == 3:
        return repr(float(np.float32(x)))
    if k == 4:
        return f"{x:+.4f}"
    if k == 5:   # leading dot / minus dot
        s = f"{x:.5f}"
        return s.replace("0.", ".", 1) if s.startswith(("0.", "-0.")) else s
    if k == 6:
        return str(int(round(x)))
    if k == 7:
        return f"{x:.12f}"
    return f"{x:.8g}"


def random_obj(rng, n_faces=40):
    """An OBJ exercising the parser: number formats, comments, CRLF, tabs, vn / vt / o / g / s /
    usemtl lines, v / v/vt / v//vn / v/vt/vn corners, negative (relative) indices, and faces of
    3 to 8 corners (convex, concave and collinear polygons) -- all indices in range."""
    lines, nv = [], 0
    nl = "\r\n" if rng.random() < 0.3 else "\n"
    for f in range(n_faces):
        if rng.random() < 0.15:
            lines.append(rng.choice(["# comment", "", "s off", "s 1", "o part%d" % f, "g grp%d" % f,
                                     "usemtl m%d" % (f % 3), "vn 0 0 1", "vt 0.5 0.5", "\t# indented"]))
        k = int(rng.choice([3, 3, 3, 4, 4, 4, 5, 6, 7, 8]))
        # a polygon in a random plane: star-shaped (concave) or convex, sometimes collinear points
        ang = np.sort(rng.uniform(0, 2 * np.pi, k))
        rad = rng.uniform(0.5, 2.0, k) if rng.random() < 0.5 else np.ones(k)
        pts2 = np.stack([rad * np.cos(ang), rad * np.sin(ang)], 1)
        if rng.random() < 0.1:
            pts2[1] = 0.5 * (pts2[0] + pts2[2])
        basis = np.linalg.qr(rng.normal(size=(3, 3)))[0]
        if rng.random() < 0.3:      # axis-aligned planes exercise the projection-axis choice
            basis = np.eye(3)[rng.permutation(3)]
        P = pts2[:, :1] * basis[0] + pts2[:, 1:2] * basis[1] + rng.normal(size=3)
        P = P * rng.choice([1.0, 100.0, 1e-3])
        first = nv
        for p in P:
            sep = "\t" if rng.random() < 0.1 else " "
            extra = " 1.0" if rng.random() < 0.05 else ""
            lines.append("v" + sep + sep.join(_fmt_float(rng, c) for c in p) + extra + ("  " if rng.random() < 0.1 else ""))
            nv += 1
        corners = []
        style = rng.integers(0, 4)
        for j in range(k):
            idx = first + j + 1
            if rng.random() < 0.3:
                idx = idx - nv - 1           # relative: -1 is the last vertex read
            corners.append([f"{idx}", f"{idx}/1", f"{idx}//1", f"{idx}/1/1"][style])
        lines.append("f " + " ".join(corners))
    return nl.join(lines) + (nl if rng.random() < 0.7 else "")


@pytest.mark.parametrize("seed", range(12))
def test_obj_parser_fuzz_against_tinyobj(rt, refio, tmp_path, seed):
    """Random OBJ text (formats, separators, relative indices, polygons up to 8 corners): the
    library's reader equals tinyobj::LoadObj + LoadModel's triangle loop -- vertex bits, the
    quad's shorter-diagonal split (tiny_obj_loader.h:1484-1580) and the ear clipping of larger
    polygons (1705-1928)."""
    rng = np.random.default_rng(1000 + seed)
    p = tmp_path / f"fuzz{seed}.obj"
    p.write_bytes(random_obj(rng).encode())
    Vr, Fr = refio.load_model(str(p))
    V, F = rt.load_obj(str(p))
    assert np.array_equal(V.view(np.uint32), Vr.view(np.uint32))
    assert F.shape == Fr.shape and np.array_equal(F, Fr)


def test_obj_edge_cases_against_tinyobj(rt, refio, tmp_path):
    p = tmp_path / "edge.obj"
    p.write_text("# comment\r\n"
                 "v 1 2 3\r\n"
                 "v  -0.5e+1 .25 -.125\n"
                 "v 4.90876e-009 1E2 +7\n"
                 "v 1.12345678901 2 3\n"
                 "v 0.1000000000000000055511151231257827 1e-45 3.4028235e38\n"
                 "\n"
                 "vn 0 0 1\n"
                 "f 1 2 3\n"
                 "f -4/1/1 -3//1 -2 -1\n"
                 "f 1 2\n"
                 "f 1 2 3 4 5\n")
    Vr, Fr = refio.load_model(str(p))
    V, F = rt.load_obj(str(p))
    assert np.array_equal(V.view(np.uint32), Vr.view(np.uint32)) and np.array_equal(F, Fr)
    assert len(F) == 6   # triangle + split quad + 3 ears of the pentagon; the 2-vertex face is dropped


@pytest.mark.parametrize("name", IMAGES)
def test_image_load_equals_stb(rt, refio, reference_assets, name):
    """rt_image_load gives Surface::LoadImage's texels (stbi_load) for the reference's PNGs."""
    path = os.path.join(reference_assets, name + ".png")
    want, _ = refio.load_image(path)
    got = rt.load_image(path)
    assert got.shape == want.shape and np.array_equal(got, want)


CASES = [(0, 1, 1), (0, 2, 1), (0, 4, 1), (0, 8, 1), (0, 16, 1), (2, 8, 3), (2, 16, 3), (3, 1, 1), (3, 2, 1),
         (3, 4, 1), (3, 8, 1), (4, 8, 2), (4, 16, 2), (6, 8, 4), (6, 16, 4)]


@pytest.mark.parametrize("ctype,depth,ch", CASES)
def test_png_decode_equals_stb(rt, refio, tmp_path, ctype, depth, ch):
    """Every PNG colour type / bit depth / row filter: rt_image_load == stbi_load + LoadImage's
    packing.  Grey+alpha (stb reports 2 channels): LoadImage reads channels 0..2 of pixel i, i.e.
    grey, alpha and the NEXT pixel's grey -- and for the last pixel one byte past stb's buffer,
    which is undefined, so that one texel is excluded."""
    rng = np.random.default_rng(ctype * 100 + depth)
    h, w = 11, 13
    hi = 1 << depth
    pal = rng.integers(0, 256, size=(hi, 3)) if ctype == 3 else None
    samples = rng.integers(0, hi, size=(h, w, ch))
    f = tmp_path / "t.png"
    f.write_bytes(pngref.encode(samples, ctype, depth, palette=pal))
    want, n = refio.load_image(str(f))
    got = rt.load_image(str(f))
    assert got.shape == want.shape == (h, w)
    if n == 2:
        got, want = got.reshape(-1)[:-1], want.reshape(-1)[:-1]
    assert np.array_equal(got, want)
