// rt_sbvh.cpp -- opt-in spatial-split BVH (SBVH), the reference's SPATIAL_SPLITS build
// (template/scene.h:521-840, Primitive.h:474-685) rebuilt correct and bounded:
//
//   * object split = binned SAH over the references' centroids (32 bins, as findBestObjectSplit);
//   * a spatial split is tried when the object split's children overlap by more than
//     alpha = 1e-5 of the root's surface (as FindBestSplitPlane, SPATIAL_SPLIT_ALPHA): chopped
//     binning over the node box (32 bins); a triangle reference is clipped to each bin slab as a
//     polygon in double precision and its box rounded OUTWARD to float (the reference's
//     fitInBin computes float edge intersections, and its sphere branch reads an uninitialised /
//     shadowed distance -- Primitive.h:493-503 -- which is where its NaN nodes come from); other
//     primitives are clipped as their box intersected with the slab;
//   * SAH cost of a plane = left refs x left area + right refs x right area, leaf cost =
//     refs x node area (calculateNodeCost); no unsplitting;
//   * straddling references are duplicated with their boxes clipped to each side; the
//     duplicates are budgeted (at most as many extra references as primitives, Stich et al.'s
//     bound) and the node pool grows as needed (the reference's 4N pool overflows on
//     mig29 x16);
//   * node order is the reference's (sibling pairs, DFS pre-order, node 1 unused); leaves index
//     a reference array in which a primitive may appear more than once.
//
// Closest hits equal the plain BVH's except where two primitives are hit at exactly the same
// distance (the visiting order picks the first) -- the boxes only decide which primitives are
// tested, and every reference box contains its part of the primitive (tests/test_gpu_parity.py
// holds it to the oracle's plain-BVH hits).  It is a non-parity tree: the bench and the
// parity suite use the plain BVH.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "rt_internal.h"

namespace rt {
namespace {

struct Bx { float mn[3], mx[3]; };
inline Bx bx_empty() { return {{1e30f, 1e30f, 1e30f}, {-1e30f, -1e30f, -1e30f}}; }
inline void bx_grow(Bx &a, const Bx &b) {
    for (int k = 0; k < 3; ++k) { a.mn[k] = std::min(a.mn[k], b.mn[k]); a.mx[k] = std::max(a.mx[k], b.mx[k]); }
}
inline bool bx_valid(const Bx &b) { return b.mn[0] <= b.mx[0] && b.mn[1] <= b.mx[1] && b.mn[2] <= b.mx[2]; }
inline float bx_area(const Bx &b) {   // aabb::Area (precomp.h:912-917), 0 for an empty box
    if (!bx_valid(b)) return 0.0f;
    // extents capped at 2e18 so that a plane's +-1e30 box (Primitive.h:322-323) keeps a finite area
    const float e0 = std::min(b.mx[0] - b.mn[0], 2e18f), e1 = std::min(b.mx[1] - b.mn[1], 2e18f),
                e2 = std::min(b.mx[2] - b.mn[2], 2e18f);
    return std::max(0.0f, e0 * e1 + e0 * e2 + e1 * e2);
}
inline Bx bx_intersect(const Bx &a, const Bx &b) {
    Bx r;
    for (int k = 0; k < 3; ++k) { r.mn[k] = std::max(a.mn[k], b.mn[k]); r.mx[k] = std::min(a.mx[k], b.mx[k]); }
    return r;
}
inline float down(double v) { float f = (float)v; return (double)f > v ? std::nextafter(f, -INFINITY) : f; }
inline float up(double v) { float f = (float)v; return (double)f < v ? std::nextafter(f, INFINITY) : f; }

struct Ref { uint32_t id; Bx box; };

struct Sbvh {
    const rt_prim *prims;
    std::vector<Bx> pbox;          // each primitive's full box (GetAABBMin/Max)
    Bvh &out;
    std::vector<Node> nodes;
    float root_area = 1.0f;
    size_t budget = 0;             // duplicates still allowed

    Sbvh(const rt_prim *p, std::vector<Bx> &&b, Bvh &o) : prims(p), pbox(std::move(b)), out(o) {}

    // the part of reference r inside [lo, hi] on `axis`, within its current box; false if empty
    bool clip(const Ref &r, int axis, float lo, float hi, Bx &res) const {
        Bx slab = r.box;
        slab.mn[axis] = std::max(slab.mn[axis], lo);
        slab.mx[axis] = std::min(slab.mx[axis], hi);
        if (!bx_valid(slab)) return false;
        const rt_prim &p = prims[r.id];
        if (p.type != RT_TRIANGLE) { res = slab; return true; }
        // Sutherland-Hodgman of the triangle against the slab's 6 planes, in double
        double poly[16][3], tmp[16][3];
        int n = 3;
        for (int v = 0; v < 3; ++v)
            for (int k = 0; k < 3; ++k) poly[v][k] = p.v[3 * v + k];
        for (int k = 0; k < 3 && n; ++k)
            for (int side = 0; side < 2 && n; ++side) {
                const double c = side ? slab.mx[k] : slab.mn[k];
                auto inside = [&](const double *q) { return side ? q[k] <= c : q[k] >= c; };
                int m = 0;
                for (int i = 0; i < n; ++i) {
                    const double *a = poly[i], *b = poly[(i + 1) % n];
                    const bool ia = inside(a), ib = inside(b);
                    if (ia) { std::memcpy(tmp[m++], a, sizeof(double) * 3); }
                    if (ia != ib) {
                        const double t = (c - a[k]) / (b[k] - a[k]);
                        for (int j = 0; j < 3; ++j) tmp[m][j] = j == k ? c : a[j] + t * (b[j] - a[j]);
                        ++m;
                    }
                }
                n = m;
                std::memcpy(poly, tmp, sizeof(double) * 3 * (size_t)m);
            }
        if (n == 0) return false;
        Bx b = bx_empty();
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < 3; ++k) {
                b.mn[k] = std::min(b.mn[k], down(poly[i][k]));
                b.mx[k] = std::max(b.mx[k], up(poly[i][k]));
            }
        res = bx_intersect(b, slab);   // outward-rounded polygon box, never beyond the slab
        return bx_valid(res);
    }

    struct Split {
        int axis = -1;
        float pos = 0.0f;
        double cost = 1e300;
        bool spatial = false;
    };

    Split object_split(const std::vector<Ref> &R, Bx &lb, Bx &rb) const {
        Split best;
        for (int a = 0; a < 3; ++a) {
            float lo = 1e30f, hi = -1e30f;
            for (const Ref &r : R) {
                const float c = 0.5f * (r.box.mn[a] + r.box.mx[a]);
                lo = std::min(lo, c);
                hi = std::max(hi, c);
            }
            if (!(lo < hi)) continue;
            Bx bins[32];
            int cnt[32] = {0};
            for (auto &b : bins) b = bx_empty();
            const float scale = 32.0f / (hi - lo);
            for (const Ref &r : R) {
                int b = (int)((0.5f * (r.box.mn[a] + r.box.mx[a]) - lo) * scale);
                b = std::min(31, std::max(0, b));
                cnt[b]++;
                bx_grow(bins[b], r.box);
            }
            Bx L = bx_empty(), Rb = bx_empty();
            float la[31], ra[31];
            int lc[31], rc[31], ls = 0, rs = 0;
            for (int i = 0; i < 31; ++i) {
                ls += cnt[i]; lc[i] = ls; bx_grow(L, bins[i]); la[i] = bx_area(L);
                rs += cnt[31 - i]; rc[30 - i] = rs; bx_grow(Rb, bins[31 - i]); ra[30 - i] = bx_area(Rb);
            }
            for (int i = 0; i < 31; ++i) {
                if (!lc[i] || !rc[i]) continue;
                const double c = (double)lc[i] * la[i] + (double)rc[i] * ra[i];
                if (c < best.cost) { best.cost = c; best.axis = a; best.pos = lo + (hi - lo) * (float)(i + 1) / 32.0f; }
            }
        }
        lb = bx_empty(); rb = bx_empty();
        if (best.axis >= 0)
            for (const Ref &r : R) bx_grow(0.5f * (r.box.mn[best.axis] + r.box.mx[best.axis]) < best.pos ? lb : rb, r.box);
        return best;
    }

    Split spatial_split(const Bx &node, const std::vector<Ref> &R, double bound) const {
        Split best;
        best.cost = bound;
        for (int a = 0; a < 3; ++a) {
            const float lo = node.mn[a], hi = node.mx[a];
            if (!(lo < hi) || hi - lo > 1e18f) continue;   // no chopped bins over a plane's infinite box
            const float w = (hi - lo) / 32.0f;
            auto edge = [&](int i) { return i == 0 ? lo : i == 32 ? hi : lo + w * (float)i; };
            Bx bins[32];
            int entry[32] = {0}, exitc[32] = {0};
            for (auto &b : bins) b = bx_empty();
            for (const Ref &r : R) {
                int b0 = (int)((r.box.mn[a] - lo) / w), b1 = (int)((r.box.mx[a] - lo) / w);
                b0 = std::min(31, std::max(0, b0));
                b1 = std::min(31, std::max(b0, b1));
                int first = -1, last = -1;
                for (int b = b0; b <= b1; ++b) {
                    Bx c;
                    if (!clip(r, a, edge(b), edge(b + 1), c)) continue;
                    bx_grow(bins[b], c);
                    if (first < 0) first = b;
                    last = b;
                }
                if (first < 0) continue;
                entry[first]++;
                exitc[last]++;
            }
            Bx L = bx_empty(), Rb = bx_empty();
            float la[31], ra[31];
            int lc[31], rc[31], ls = 0, rs = 0;
            for (int i = 0; i < 31; ++i) {
                ls += entry[i]; lc[i] = ls; bx_grow(L, bins[i]); la[i] = bx_area(L);
                rs += exitc[31 - i]; rc[30 - i] = rs; bx_grow(Rb, bins[31 - i]); ra[30 - i] = bx_area(Rb);
            }
            for (int i = 0; i < 31; ++i) {
                if (!lc[i] || !rc[i]) continue;
                const double c = (double)lc[i] * la[i] + (double)rc[i] * ra[i];
                if (c < best.cost) { best.cost = c; best.axis = a; best.pos = edge(i + 1); best.spatial = true; }
            }
        }
        return best;
    }

    static Bx bounds(const std::vector<Ref> &R) {
        Bx b = bx_empty();
        for (const Ref &r : R) bx_grow(b, r.box);
        return b;
    }

    void set_node(uint32_t ni, const Bx &b) {
        for (int k = 0; k < 3; ++k) { nodes[ni].mn[k] = b.mn[k]; nodes[ni].mx[k] = b.mx[k]; }
    }

    void run(std::vector<Ref> &&all) {
        nodes.assign(2, Node{});
        Bx rb = bounds(all);
        root_area = std::max(bx_area(rb), 1e-30f);
        set_node(0, rb);
        struct Job { uint32_t ni; std::vector<Ref> refs; };
        std::vector<Job> st;
        st.push_back({0, std::move(all)});
        // leaves in DFS pre-order: left subtree first (pairs are allocated when a node splits,
        // as Subdivide does: left child = nodesUsed, right = nodesUsed + 1)
        std::vector<std::pair<uint32_t, std::vector<Ref>>> leaves;
        while (!st.empty()) {
            Job job = std::move(st.back());
            st.pop_back();
            std::vector<Ref> &R = job.refs;
            const Bx nb = bounds(R);
            set_node(job.ni, nb);
            const double leaf_cost = (double)R.size() * bx_area(nb);
            Bx ol, orr;
            Split s = R.size() > 1 ? object_split(R, ol, orr) : Split{};
            if (s.axis >= 0 && budget > 0) {
                const float ov = bx_area(bx_intersect(ol, orr));
                if (ov / root_area > 1e-5f) {
                    Split sp = spatial_split(nb, R, s.cost);
                    if (sp.spatial) s = sp;
                }
            }
            const bool must = R.size() > 64;   // keep leaves within the kernels' 255-primitive word
            if (!must && (s.axis < 0 || !(s.cost < leaf_cost))) {
                leaves.push_back({job.ni, std::move(R)});
                continue;
            }
            std::vector<Ref> L, Rr;
            if (s.axis < 0) {
                // no split plane separates the centroids (many references share one centroid):
                // halve the references by index, so every leaf stays within the limit
                const size_t h = R.size() / 2;
                L.assign(R.begin(), R.begin() + (long)h);
                Rr.assign(R.begin() + (long)h, R.end());
            } else if (!s.spatial) {
                for (Ref &r : R) (0.5f * (r.box.mn[s.axis] + r.box.mx[s.axis]) < s.pos ? L : Rr).push_back(r);
            } else {
                for (Ref &r : R) {
                    if (r.box.mx[s.axis] <= s.pos) { L.push_back(r); continue; }
                    if (r.box.mn[s.axis] >= s.pos) { Rr.push_back(r); continue; }
                    Ref a = r, b = r;
                    const bool ha = clip(r, s.axis, -INFINITY, s.pos, a.box);
                    const bool hb = clip(r, s.axis, s.pos, INFINITY, b.box);
                    if (ha && hb && budget > 0) { --budget; L.push_back(a); Rr.push_back(b); }
                    else if (ha && hb) ((0.5f * (r.box.mn[s.axis] + r.box.mx[s.axis]) < s.pos) ? L : Rr).push_back(r);
                    else (ha ? L : Rr).push_back(ha ? a : b);
                }
            }
            if (L.empty() || Rr.empty()) {
                if (!must) { leaves.push_back({job.ni, std::move(R)}); continue; }
                const size_t h = R.size() / 2;   // a split that separated nothing: halve by index
                L.assign(R.begin(), R.begin() + (long)h);
                Rr.assign(R.begin() + (long)h, R.end());
            }
            const uint32_t left = (uint32_t)nodes.size();
            nodes.resize(nodes.size() + 2);
            nodes[job.ni].leftFirst = left;
            nodes[job.ni].count = 0;
            st.push_back({left + 1, std::move(Rr)});   // right pushed first: left is built next (DFS pre-order)
            st.push_back({left, std::move(L)});
        }
        // reference array in leaf (pre-order) order
        out.indices.clear();
        for (auto &lf : leaves) {
            nodes[lf.first].leftFirst = (uint32_t)out.indices.size();
            nodes[lf.first].count = (uint32_t)lf.second.size();
            for (const Ref &r : lf.second) out.indices.push_back(r.id);
        }
        out.nodes = nodes;
        out.nodes_used = (uint32_t)nodes.size();
        out.max_leaf = 0;
        for (const Node &nd : nodes) out.max_leaf = std::max(out.max_leaf, nd.count);
        // depth as Scene::maxDepthBVH: interior levels, a root leaf = 1
        std::vector<std::pair<uint32_t, uint32_t>> q{{0, 0}};
        out.depth = 0;
        while (!q.empty()) {
            auto [k, d] = q.back();
            q.pop_back();
            const Node &nd = out.nodes[k];
            if (nd.count > 0) { out.depth = std::max(out.depth, k == 0 ? 1u : d); continue; }
            q.push_back({nd.leftFirst, d + 1});
            q.push_back({nd.leftFirst + 1, d + 1});
        }
    }
};

}  // namespace

int build_sbvh(const rt_prim *prims, const float *transforms, uint32_t n, Bvh &out) {
    if (n == 0) return fail(RT_ERR_INVALID, "scene has no primitives");
    std::vector<Bx> pb(n);
    std::vector<Ref> refs(n);
    for (uint32_t i = 0; i < n; ++i) {
        PrimX x;
        prim_transform(prims[i], transforms ? transforms + 16 * (size_t)i : nullptr, x);
        PrimGeom g;
        prim_geometry(prims[i], x, g);
        pb[i] = {{g.bmin.x, g.bmin.y, g.bmin.z}, {g.bmax.x, g.bmax.y, g.bmax.z}};
        refs[i] = {i, pb[i]};
    }
    Sbvh b(prims, std::move(pb), out);
    b.budget = n;
    b.run(std::move(refs));
    return RT_OK;
}

}  // namespace rt
