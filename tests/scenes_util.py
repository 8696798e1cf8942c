"""Hand-made scenes shared by the parity tests and the fixture generator: the same
primitive list built in the oracle (the checker), and the primitive known-answer set
(edge, vertex, grazing, parallel, inside-sphere, t ~ EPS, exact ties, NaN slabs)."""
import numpy as np


def oracle_scene(rt, oracle, prims, mats, sky=None, textures=(), bvh=None):
    """The primitive list (rt.sphere / plane / triangle / cube / quad records) as an oracle scene;
    bvh = (nodes [n, 32] uint8, indices) replaces the oracle's BuildBVH."""
    import ctypes as C
    L = oracle.lib()
    h = L.or_scene_new()
    f3 = lambda *v: (C.c_float * 3)(*v)
    f16 = lambda T: (C.c_float * 16)(*(np.eye(4, dtype=np.float32).reshape(16) if T is None else T))
    for t in textures:
        t = np.ascontiguousarray(t, np.uint32)
        L.or_scene_add_texture(h, t.shape[1], t.shape[0], t.ctypes.data_as(C.POINTER(C.c_uint32)))
    for m in mats:
        L.or_scene_add_material_tex(h, m.kind, f3(*m.color), f3(*m.color2), m.ior, m.diffuse, m.texture)
    for p in prims:
        v = list(p.v)
        if p.type == rt.SPHERE:
            L.or_scene_add_sphere(h, f3(*v[:3]), v[3], p.material)
        elif p.type == rt.PLANE:
            L.or_scene_add_plane(h, f3(*v[:3]), v[3], p.material)
        elif p.type == rt.CUBE:
            L.or_scene_add_cube(h, f3(*v[:3]), f3(*v[3:6]), f16(getattr(p, "T", None)), p.material)
        elif p.type == rt.QUAD:
            L.or_scene_add_quad(h, v[0], f16(getattr(p, "T", None)), p.material)
        else:
            L.or_scene_add_triangle(h, f3(*v[:3]), f3(*v[3:6]), f3(*v[6:9]), p.material)
    if sky is not None:
        L.or_scene_set_sky(h, sky.shape[1], sky.shape[0], sky.ctypes.data_as(C.POINTER(C.c_uint32)))
    if bvh is None:
        L.or_scene_build_bvh(h)
    else:
        nodes, idx = np.ascontiguousarray(bvh[0], np.uint8), np.ascontiguousarray(bvh[1], np.uint32)
        assert L.or_scene_set_bvh(h, nodes.ctypes.data_as(C.c_void_p), len(nodes),
                                  idx.ctypes.data_as(C.POINTER(C.c_uint32)), len(idx)) == len(nodes)
    o = oracle.Scene.__new__(oracle.Scene)
    o.L, o.h = L, h
    return o




# ---- primitive known-answer set (Primitive.h:64-314, scene.h:285-487)
EPS = np.float32(1e-4)


def kat_scene(rt):
    """Light (prim 0), two triangles sharing an edge, two coincident triangles (exact ties),
    two spheres, a plane (outside the BVH: AABB +-1e30, Primitive.h:322-323)."""
    mats = [rt.material(rt.LIGHT, (24, 24, 22)), rt.material(rt.DIFFUSE, (0.8, 0.8, 0.8)),
            rt.material(rt.MIRROR, (0.9, 0.9, 0.9))]
    prims = [rt.sphere((0, 4, -2), 0.5, 0),
             rt.triangle((0, 0, 5), (1, 0, 5), (0, 1, 5), 1),          # 1: T1
             rt.triangle((1, 0, 5), (1, 1, 5), (0, 1, 5), 1),          # 2: T2, shares T1's hypotenuse
             rt.triangle((-2, -1, 7), (-1, -1, 7), (-2, 0, 7), 1),     # 3: T3a
             rt.triangle((-2, -1, 7), (-1, -1, 7), (-2, 0, 7), 2),     # 4: T3b == T3a (tie)
             rt.sphere((3, 0, 5), 1.0, 2),                             # 5: S1
             rt.sphere((-3, 2, 5), 0.25, 1),                           # 6: S2
             rt.plane((0, 1, 0), 2.0, 1)]                              # 7: y = -2
    return prims, mats


def _ray(o, d, tmax=1e34):
    return [np.float32(o[0]), np.float32(o[1]), np.float32(o[2]), np.float32(d[0]), np.float32(d[1]),
            np.float32(d[2]), np.float32(tmax)]


def kat_rays():
    """Hand-picked rays (7 floats: O, D, tmax) + a jittered cloud around the vertices/edges."""
    up = 1.0 / np.sqrt(np.float32(2))
    R = []
    # T1 / T2: vertices, shared edge (tie between 1 and 2), edges, just outside, centre
    for p in [(0, 0), (1, 0), (0, 1), (1, 1), (0.5, 0.5), (0.25, 0.75), (0.5, 0), (0, 0.5), (1, 0.5), (0.5, 1),
              (0.3, 0.3), (1.0000001, 0.5), (-1e-7, 0.5), (0.5, -1e-7)]:
        R.append(_ray((p[0], p[1], 0), (0, 0, 1)))
        R.append(_ray((p[0], p[1], 10), (0, 0, -1)))                  # back faces (no culling)
    # ray in the triangles' plane, grazing rays
    R.append(_ray((-1, 0.2, 5), (1, 0, 0)))
    R.append(_ray((-1, 0.2, 4.999), (1, 0, 1e-4)))
    R.append(_ray((0.2, 0.2, 4), (0, 1e-7, 1)))
    # t around EPS (t > EPS strict, Primitive.h:270)
    for dz in (1e-4, 9.9e-5, 1.01e-4, 2e-4, 0.0, -1e-5):
        R.append(_ray((0.2, 0.2, np.float32(5) - np.float32(dz)), (0, 0, 1)))
    # exact duplicate triangles: tie -> first tested wins
    for p in [(-1.8, -0.8), (-1.5, -0.5), (-2, -1), (-1, -1), (-2, 0)]:
        R.append(_ray((p[0], p[1], 0), (0, 0, 1)))
    # S1: centre inside (second root), tangent, origin on the surface, just outside, t ~ EPS
    R.append(_ray((3, 0, 5), (0, 0, 1)))
    R.append(_ray((3, 0, 5), (up, up, 0)))
    R.append(_ray((4, -5, 5), (0, 1, 0)))                           # tangent at x = 4
    R.append(_ray((4.0000005, -5, 5), (0, 1, 0)))
    R.append(_ray((3, 0, 4), (0, 0, 1)))                            # starts on the surface
    R.append(_ray((3, 0, np.float32(4) - np.float32(1e-4)), (0, 0, 1)))
    R.append(_ray((3, 0, 0), (0, 0, 1)))
    R.append(_ray((3, 0, 10), (0, 0, -1)))
    R.append(_ray((-3, 2, 0), (0, 0, 1)))
    # plane y = -2: from above, from below, parallel, in the plane
    R.append(_ray((0, 0, 0), (0, -1, 0)))
    R.append(_ray((0, -3, 0), (0, 1, 0)))
    R.append(_ray((0, -1, 0), (1, 0, 0)))
    R.append(_ray((0, -2, 0), (1, 0, 0)))
    R.append(_ray((0, -2, 0), (0, -1, 0)))
    # axis-parallel rays with origins on node slab planes: (slab - O) * inf = NaN
    for o in [(0, 0.5, 0), (1, 0.5, 0), (0.5, 0, 0), (0.5, 1, 0), (0, 0, 0), (-2, -1, 0), (4, 0, 0)]:
        R.append(_ray(o, (0, 0, 1)))
        R.append(_ray(o, (0, 0, -1)))
        R.append(_ray((o[0], o[1], 5), (1, 0, 0)))
        R.append(_ray((o[0], o[1], 5), (-0.0, 1, 0)))
    # shadow-style rays whose tmax ends exactly at / just before / after a surface
    for tm in (5.0, 4.9999995, 5.0000005, 5.0 - 2e-4):
        R.append(_ray((0.2, 0.2, 0), (0, 0, 1), tm))
        R.append(_ray((3, 0, -2), (0, 0, 1), tm))
    rays = np.array(R, np.float32)
    # jittered cloud: rays from random points toward the vertices / edge points +- a few ulps
    rng = np.random.default_rng(2024)
    targets = np.array([[0, 0, 5], [1, 0, 5], [0, 1, 5], [1, 1, 5], [0.5, 0.5, 5], [-2, -1, 7], [-1, -1, 7],
                        [-2, 0, 7], [3, 1, 5], [4, 0, 5], [-3, 2.25, 5]], np.float32)
    n = 4000
    O = rng.uniform(-4, 4, (n, 3)).astype(np.float32)
    O[:, 2] = rng.uniform(-3, 1, n).astype(np.float32)
    T = targets[rng.integers(0, len(targets), n)]
    T = T + rng.integers(-3, 4, (n, 3)).astype(np.float32) * np.float32(1.2e-7)   # a few ulps off
    D = (T - O).astype(np.float32)
    D /= np.linalg.norm(D, axis=1, keepdims=True).astype(np.float32)
    cloud = np.concatenate([O, D.astype(np.float32), np.full((n, 1), 1e34, np.float32)], 1).astype(np.float32)
    return np.concatenate([rays, cloud], 0)


def chain_scene(rt, n_tris=64):
    """A caterpillar tree one primitive per level: the light (prim 0) and n_tris small
    diffuse triangles in front of the default camera, with a prebuilt BVH whose every interior node
    has a leaf child and an interior child -- depth n_tris (64, the most a scene may have), so the LDS stacks
    fill 64 KB (64 entries x 256 lanes x 4 B) and leave no room for the wave walk's words or the work
    map's counters.  Boxes are the unions of their primitives' boxes (nested).  Returns prims,
    materials, (nodes [n, 32] uint8, indices)."""
    mats = [rt.material(rt.LIGHT, (24, 24, 22)), rt.material(rt.DIFFUSE, (0.8, 0.7, 0.6)),
            rt.material(rt.MIRROR, (0.9, 0.9, 0.9))]
    prims = [rt.sphere((0.0, 4.0, -2.0), 0.5, 0)]
    boxes = [(np.float32([-0.5, 3.5, -2.5]), np.float32([0.5, 4.5, -1.5]))]
    cols = 10
    for k in range(n_tris):
        x0 = -3.0 + 0.6 * (k % cols)
        y0 = -1.8 + 0.6 * (k // cols)
        z = 2.5 + 0.01 * k
        a, b, c = (x0, y0, z), (x0 + 0.5, y0 + 0.05, z + 0.1), (x0 + 0.1, y0 + 0.5, z - 0.1)
        prims.append(rt.triangle(a, b, c, 1 + (k % 7 == 3)))
        v = np.float32([a, b, c])
        boxes.append((v.min(axis=0), v.max(axis=0)))
    P = len(prims)
    nodes = np.zeros((2 * P, 8), np.uint32)
    f = nodes.view(np.float32)

    def put(i, lo, hi, left_first, count):
        f[i, 0:3], f[i, 3:6] = lo, hi
        nodes[i, 6], nodes[i, 7] = left_first, count

    def union(j):   # primitives j .. P-1
        lo = np.min([boxes[q][0] for q in range(j, P)], axis=0)
        hi = np.max([boxes[q][1] for q in range(j, P)], axis=0)
        return lo, hi

    put(0, *union(0), 2, 0)
    for j in range(P - 1):   # pair (2 + 2j, 3 + 2j): leaf of prim j, then the rest of the chain
        put(2 + 2 * j, *boxes[j], j, 1)
        if j == P - 2:
            put(3 + 2 * j, *boxes[P - 1], P - 1, 1)
        else:
            put(3 + 2 * j, *union(j + 1), 4 + 2 * j, 0)
    return prims, mats, (nodes.view(np.uint8).reshape(len(nodes), 32), np.arange(P, dtype=np.uint32))


def _cam(rt, W, H, pos, fwd, right, up):
    """A pinhole camera looking along fwd from pos, the screen one unit ahead spanning
    [-aspect, aspect] x [-1, 1] along right / up (the default camera's shape, camera.h:28-41)."""
    c = rt.Camera.default(W, H)
    pos, fwd, right, up = (np.asarray(v, np.float64) for v in (pos, fwd, right, up))
    a = W / H
    ctr = pos + fwd
    for name, p in (("pos", pos), ("top_left", ctr - a * right + up), ("top_right", ctr + a * right + up),
                    ("bottom_left", ctr - a * right - up)):
        getattr(c, name)[:] = [float(np.float32(x)) for x in p]
    return c


def grazing_cameras(rt, W, H):
    """Cameras aimed at the wave walk's open case: camera rays that graze a
    triangle's plane, where the computed triangle t carries the most rounding error relative to its
    leaf box's entry.  TEAPOT-F: the eye at the floor's height (y = -1.225) looking along the floor,
    and just above it looking slightly down (every floor hit grazing); mig29 x16: the eye in the plane
    of the largest triangle of the first aircraft (a wing), looking at that triangle, with the
    image's middle row in the plane."""
    out = {}
    y = -1.225
    out["teapotF_floor_level"] = ("teapotF", _cam(rt, W, H, (0.0, y, -1.0), (0, 0, 1), (1, 0, 0), (0, 1, 0)))
    f = np.array([0.0, -0.02, 1.0])
    f /= np.linalg.norm(f)
    up = np.cross(f, (1.0, 0.0, 0.0))
    out["teapotF_floor_skim"] = ("teapotF", _cam(rt, W, H, (0.3, y + 0.02, -1.0), f, (1, 0, 0), -up))
    prims, _ = rt.recipe_describe("mig16")
    n1 = 1 + (len(prims) - 1) // 16           # the first aircraft's triangles
    best, area = None, -1.0
    for p in prims[1:n1]:
        v = np.array(list(p.v)[:9], np.float64).reshape(3, 3)
        ar = 0.5 * np.linalg.norm(np.cross(v[1] - v[0], v[2] - v[0]))
        if ar > area:
            best, area = v, ar
    ctr = best.mean(axis=0)
    n = np.cross(best[1] - best[0], best[2] - best[0])
    n /= np.linalg.norm(n)
    d = ctr - np.array([0.0, 0.0, -1.0])      # from the default eye, projected into the plane
    d -= n * d.dot(n)
    d /= np.linalg.norm(d)
    right = np.cross(n, d)
    out["mig16_wing_plane"] = ("mig16", _cam(rt, W, H, ctr - 1.5 * d, d, right, n))
    return out


def sticky_prims(rt, prims, log2_lim=-8):
    """The primitives whose boxes the wave camera walk never culls by distance (rt_device.hip
    mark_sticky): spheres, quads and sliver triangles (smallest corner angle's sine under
    2^log2_lim, from the float vertices in double)."""
    out = np.zeros(len(prims), bool)
    lim = 2.0 ** log2_lim
    for i, p in enumerate(prims):
        if p.type in (rt.SPHERE, rt.QUAD):
            out[i] = True
        elif p.type == rt.TRIANGLE:
            v = np.array(list(p.v)[:9], np.float64).reshape(3, 3)
            e = [v[(k + 1) % 3] - v[k] for k in range(3)]
            ln = sorted(float(np.linalg.norm(x)) for x in e)
            out[i] = not (np.linalg.norm(np.cross(e[0], e[2])) >= lim * ln[1] * ln[2])
    return out
