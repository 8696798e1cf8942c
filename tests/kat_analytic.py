"""Analytic known-answer vectors for Scene::IntersectBVH / IsOccluded, built WITHOUT the oracle.

The scene is a light sphere, two axis-aligned triangles, a sphere and a plane on power-of-two
coordinates, with a hand-written BVH (so every slab outcome follows from the boxes alone).
Each ray's expected closest hit follows in closed form from the reference formulas:

* triangle (Primitive.h:248-275): denom = dot(cross(D, AC), AB); u = dot(cross(-D, AO), AC) / denom;
  v = dot(cross(-D, AB), AO) / denom; t = dot(cross(AO, AB), AC) / denom; accepted when
  0 <= u <= 1, v >= 0, u + v <= 1, EPS < t < ray.t;
* sphere (Primitive.h:150-177): b = dot(oc, D), c = dot(oc, oc) - r^2, d = b^2 - c, no hit for
  d <= 0, else t = -b - sqrt(d), then sqrt(d) - b;  u = 0.5 - atan2(z, x) / 2pi, v = 0.5 - asin(y) / pi
  of the unit vector from the centre (checked only where it is +x: u = v = 0.5 exactly);
* plane (Primitive.h:178-194): t = -(dot(O, N) + d) / dot(D, N); u, v = I.x, -I.z for N = +y;
* slab test (template/scene.h:432-450) with std::min / std::max = (b < a) ? b : a / (a < b) ? b : a,
  so (slab - O) * inf = NaN on a box face poisons the test (the ray misses the box).

The arithmetic is done in exact rationals (fractions.Fraction) and a ray is kept only when
EVERY intermediate of every primitive test is a float32 value (no rounding anywhere, square
roots of perfect squares): the float32 evaluation of the reference formulas in ANY
IEEE-conforming implementation must then reproduce these values bit for bit.  The slab test
is evaluated in numpy float32 (IEEE, no FMA) with the reference's min/max semantics; box
faces and ray directions are powers of two so its products are exact too.
"""
from fractions import Fraction as Fr

import numpy as np

EPS = Fr(np.float32(1e-4).item())       # Primitive.h / renderer.h EPS, as the float constant
T_MAX = 1e34                              # Ray.h:10


class Inexact(Exception):
    pass


def X(v):
    """v (a Fraction) if it is exactly a float32 value, else Inexact."""
    v = Fr(v)
    f = np.float32(float(v))
    if not np.isfinite(f) or Fr(f.item()) != v:
        raise Inexact(v)
    return v


def sub(a, b): return tuple(X(x - y) for x, y in zip(a, b))
def neg(a): return tuple(-x for x in a)


def dot(a, b):
    s = X(a[0] * b[0])
    s = X(s + X(a[1] * b[1]))
    return X(s + X(a[2] * b[2]))


def cross(a, b):
    return (X(X(a[1] * b[2]) - X(a[2] * b[1])), X(X(a[2] * b[0]) - X(a[0] * b[2])), X(X(a[0] * b[1]) - X(a[1] * b[0])))


def div(a, b):
    if b == 0:
        raise Inexact("division by zero")
    return X(a / b)


def isqrt_exact(d):
    n, m = d.numerator, d.denominator
    rn, rm = int(round(n ** 0.5)), int(round(m ** 0.5))
    for a in (rn - 1, rn, rn + 1):
        for b in (rm - 1, rm, rm + 1):
            if a >= 0 and b > 0 and a * a == n and b * b == m:
                return X(Fr(a, b))
    raise Inexact("sqrt")


# ---- the scene: prim ids = creation order (Primitive.h:37-38); the light is prim 0
LIGHT = ((0, 64, 0), 1)
TRI1 = ((0, 0, 4), (2, 0, 4), (0, 2, 4))
TRI2 = ((-8, -8, 16), (-4, -8, 16), (-8, -4, 16))
SPH = ((16, 0, 8), 5)
PLANE = ((0, 1, 0), 16)           # y = -16


def scene(rt):
    mats = [rt.material(rt.LIGHT, (24, 24, 22)), rt.material(rt.DIFFUSE, (0.8, 0.8, 0.8))]
    prims = [rt.sphere(LIGHT[0], LIGHT[1], 0), rt.triangle(*TRI1, 1), rt.triangle(*TRI2, 1),
             rt.sphere(SPH[0], SPH[1], 1), rt.plane(PLANE[0], PLANE[1], 1)]
    return prims, mats


BIG = 1e30       # the plane's AABB, Primitive.h:322-323
# hand-made plain BVH (BVHNode.h:5-14; node 1 unused, sibling pairs at even indices):
#   0 root -> (2, 3); 2 = leaf [light]; 3 -> (4, 5); 4 = leaf [TRI1]; 5 -> (6, 7);
#   6 = leaf [TRI2]; 7 = leaf [sphere, plane]
NODES = [  # (mn, mx, leftFirst, count)
    ((-BIG,) * 3, (BIG,) * 3, 2, 0),
    ((0, 0, 0), (0, 0, 0), 0, 0),
    ((-1, 63, -1), (1, 65, 1), 0, 1),
    ((-BIG,) * 3, (BIG,) * 3, 4, 0),
    ((0, 0, 4), (2, 2, 4), 1, 1),
    ((-BIG,) * 3, (BIG,) * 3, 6, 0),
    ((-8, -8, 16), (-4, -4, 16), 2, 1),
    ((-BIG,) * 3, (BIG,) * 3, 3, 2),
]
PATHS = {0: (2,), 1: (3, 4), 2: (3, 5, 6), 3: (3, 5, 7), 4: (3, 5, 7)}   # non-root nodes above each prim


def bvh():
    nodes = np.zeros((len(NODES), 32), np.uint8)
    for i, (mn, mx, lf, cnt) in enumerate(NODES):
        rec = np.array(list(mn) + list(mx), np.float32).tobytes() + np.array([lf, cnt], np.uint32).tobytes()
        nodes[i] = np.frombuffer(rec, np.uint8)
    return nodes, np.arange(5, dtype=np.uint32)


# ---- slab test, template/scene.h:432-450, in float32 with the reference's min / max
def _min(a, b): return b if b < a else a
def _max(a, b): return b if a < b else a


def slab_hits(O, D, tmax, node):
    mn = [np.float32(v) for v in NODES[node][0]]
    mx = [np.float32(v) for v in NODES[node][1]]
    with np.errstate(all="ignore"):
        O = [np.float32(v) for v in O]
        rD = [np.float32(1) / np.float32(v) for v in D]
        t1 = [(mn[k] - O[k]) * rD[k] for k in range(3)]
        t2 = [(mx[k] - O[k]) * rD[k] for k in range(3)]
    lo, hi = _min(t1[0], t2[0]), _max(t1[0], t2[0])
    for k in (1, 2):
        lo = _max(lo, _min(t1[k], t2[k]))
        hi = _min(hi, _max(t1[k], t2[k]))
    return bool(hi >= lo and lo < np.float32(tmax) and hi > 0)


# ---- primitive tests in exact rationals: (t, u, v) or None; u / v None = not checked
def tri_test(O, D, tri, tmax):
    A, B, C = tri
    AB, AC = sub(B, A), sub(C, A)
    denom = dot(cross(D, AC), AB)
    if abs(denom) < Fr(2.220446049250313e-16):
        return None
    AO = sub(O, A)
    u = div(dot(cross(neg(D), AO), AC), denom)
    if u < 0 or u > 1:
        return None
    v = div(dot(cross(neg(D), AB), AO), denom)
    if v < 0 or X(u + v) > 1:
        return None
    t = div(dot(cross(AO, AB), AC), denom)
    return (t, u, v) if (t < tmax and t > EPS) else None


def sph_test(O, D, sph, tmax):
    pos, r = sph
    oc = sub(O, pos)
    b = dot(oc, D)
    c = X(dot(oc, oc) - X(Fr(r) * r))
    d = X(X(b * b) - c)
    if d <= 0:
        return None
    d = isqrt_exact(d)
    for t in (X(-b - d), X(d - b)):
        if t < tmax and t > EPS:
            I = tuple(X(o + X(t * dd)) for o, dd in zip(O, D))
            rel = sub(I, pos)
            uv = (Fr(1, 2), Fr(1, 2)) if (rel[0] > 0 and rel[1] == 0 and rel[2] == 0) else (None, None)
            return (t,) + uv
    return None


def plane_test(O, D, pl, tmax):
    N, dd = pl
    den = dot(D, N)
    if den == 0:
        return None     # t = +-inf or NaN: never inside (EPS, ray.t)
    t = div(-X(dot(O, N) + dd), den)
    if not (t < tmax and t > EPS):
        return None
    I = tuple(X(o + X(t * d)) for o, d in zip(O, D))
    return (t, I[0], -I[2])      # N = +y: the (N.x < eps && N.z < eps) branch, Primitive.h:187-189


def expected(ray):
    """(t, obj, u, v) of IntersectBVH and the IsOccluded bool for one ray (7 floats), or Inexact."""
    O = tuple(Fr(float(v)) for v in ray[:3])
    D = tuple(Fr(float(v)) for v in ray[3:6])
    tmax = Fr(float(ray[6]))
    tests = [lambda: sph_test(O, D, LIGHT, tmax), lambda: tri_test(O, D, TRI1, tmax),
             lambda: tri_test(O, D, TRI2, tmax), lambda: sph_test(O, D, SPH, tmax),
             lambda: plane_test(O, D, PLANE, tmax)]
    best, best_id, occluded = None, -1, False
    ts = []
    for pid, fn in enumerate(tests):
        r = fn()                            # every primitive must evaluate exactly
        if r is None or not all(slab_hits(ray[:3], ray[3:6], ray[6], n) for n in PATHS[pid]):
            continue
        occluded = True
        ts.append(r[0])
        if best is None or r[0] < best[0]:
            best, best_id = r, pid
    if len(ts) != len(set(ts)):
        raise Inexact("tie")                # ties depend on the visiting order: not analytic
    if best is None:
        return (np.float32(float(tmax)), -1, None, None), False
    t, u, v = best
    f = lambda x: None if x is None else np.float32(float(x))
    return (f(t), best_id, f(u), f(v)), occluded


def rays():
    """Candidate rays on a power-of-two grid; only the fully exact ones are kept."""
    R = []
    dirs = (0.0, 0.125, -0.125, 0.25, -0.25, 0.5, -0.5)
    # TRI1 from the front (z = 0 -> 4) and from behind, inside / on edges / vertices / outside
    for x in np.arange(-0.5, 2.75, 0.25):
        for y in np.arange(-0.5, 2.75, 0.25):
            for dx in dirs[::2]:
                for dy in dirs[::3]:
                    R.append((x, y, 0, dx, dy, 1, T_MAX))
            R.append((x, y, 8, 0.0, 0.0, -1, T_MAX))
            R.append((x + 0.125, y + 0.125, 0, 0.0, -0.0, 1, T_MAX))
    # TRI2 at z = 16 from z = 8 with D.z = 0.5 (t = 16)
    for x in np.arange(-9, -3, 0.5):
        for y in np.arange(-9, -3, 0.5):
            for dx in (0.0, 0.125, -0.25):
                R.append((x, y, 8, dx, 0.0, 0.5, T_MAX))
    # the sphere: Pythagorean offsets (roots 5, 4, 3, 0 = tangent), inside, along +-x / +-y / +-z
    for a, b in [(0, 0), (3, 0), (0, 3), (-3, 0), (0, -3), (4, 0), (0, -4), (3, 4), (5, 0), (0, 5), (6, 0),
                 (4, 3), (-4, -3)]:
        R.append((16 + a, b, 0, 0, 0, 1, T_MAX))
        R.append((16 + a, b, 16, 0, 0, -1, T_MAX))
        R.append((16 + a, 24, 8 + b, 0, -1, 0, T_MAX))
        R.append((36, a, 8 + b, -1, 0, 0, T_MAX))
        R.append((16 + a, b, 8, 0, 0, 2, T_MAX))      # non-unit D: the formula's t, not the distance
    R.append((16, 0, 8, 0, 0, 1, T_MAX))              # from the centre: second root
    R.append((16, 0, 8, 1, 0, 0, T_MAX))
    R.append((21, 0, 8, 0, 0, 1, T_MAX))              # starts on the surface, tangent direction
    R.append((21, 0, 8, -1, 0, 0, T_MAX))             # starts on the surface, going in
    # the plane y = -16: from above, below, oblique, parallel, inside it
    for x in (-4, 0, 3.5, 40):
        for dx, dz in ((0, 0), (0.5, 0.25), (-0.25, 0.125), (2, -1)):
            R.append((x, 0, 30, dx, -1, dz, T_MAX))
            R.append((x, -32, 30, dx, 1, dz, T_MAX))
    R += [(0, -8, 30, 1, 0, 0, T_MAX), (0, -16, 30, 1, 0, 0, T_MAX), (0, -16, 30, 0, -1, 0, T_MAX)]
    # axis-parallel rays from points on TRI1's box faces: (face - O) * inf = NaN -> box missed
    for o in [(0, 0.5, 0), (2, 0.5, 0), (0.5, 0, 0), (0.5, 2, 0), (0, 0, 0), (0.5, 0.5, 0), (1, 1, 0)]:
        R.append((o[0], o[1], o[2], 0.0, 0.0, 1, T_MAX))
        R.append((o[0], o[1], o[2], -0.0, 0.0, 1, T_MAX))
        R.append((o[0], o[1], 8, 0.0, -0.0, -1, T_MAX))
    # shadow-style tmax around the hits (t < ray.t strict, t > EPS strict)
    for tm in (4, 4.0000005, 3.9999998, 5, 1e-4, 2e-4):
        R.append((0.5, 0.5, 0, 0, 0, 1, tm))
        R.append((16, 0, 0, 0, 0, 1, tm))
        R.append((0.5, 0.5, 4 - 1e-4, 0, 0, 1, tm))
    R.append((0.5, 0.5, np.float32(4) - np.float32(2e-4), 0, 0, 1, T_MAX))   # t just above / at EPS
    R.append((0.5, 0.5, np.float32(4) - np.float32(1e-4), 0, 0, 1, T_MAX))
    return np.array(R, np.float32)


def vectors():
    """(rays [n, 7] f32, t f32, obj i32, u f32 (NaN = unchecked), v f32, occluded bool)."""
    keep, T, OBJ, U, V, OCC = [], [], [], [], [], []
    for r in rays():
        try:
            (t, obj, u, v), occ = expected(r)
        except Inexact:
            continue
        keep.append(r)
        T.append(t)
        OBJ.append(obj)
        U.append(np.float32(np.nan) if u is None else u)
        V.append(np.float32(np.nan) if v is None else v)
        OCC.append(occ)
    return (np.array(keep, np.float32), np.array(T, np.float32), np.array(OBJ, np.int32), np.array(U, np.float32),
            np.array(V, np.float32), np.array(OCC, bool))


def check(got_t, got_obj, got_u, got_v, exp):
    """Bit-exact comparison against vectors(); returns a list of mismatch descriptions."""
    rays_, T, OBJ, U, V, _ = exp
    # the rationals carry no sign of zero: an expected 0 accepts +0 and -0 (the zero sign is
    # held bit-exact by the GPU-vs-oracle tests instead)
    same = lambda g, e: np.float32(g).tobytes() == e.tobytes() or (e == 0 and np.float32(g) == 0)
    bad = []
    for i in range(len(rays_)):
        ok = got_obj[i] == OBJ[i] and same(got_t[i], T[i])
        if ok and OBJ[i] >= 0:
            for g, e in ((got_u[i], U[i]), (got_v[i], V[i])):
                if not np.isnan(e) and not same(g, e):
                    ok = False
        if not ok:
            bad.append(f"ray {rays_[i].tolist()}: got (t {got_t[i]!r}, obj {got_obj[i]}, u {got_u[i]!r}, "
                       f"v {got_v[i]!r}) want (t {T[i]!r}, obj {OBJ[i]}, u {U[i]!r}, v {V[i]!r})")
    return bad
