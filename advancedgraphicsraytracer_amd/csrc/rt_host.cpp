// rt_host.cpp -- host-side scene preparation for the MI355X ray-tracing path.
//
// Everything here is a prerequisite of the GPU path, executed once per scene:
//   * OBJ reading with tinyobj's exact number parsing and quad split, so vertex bits
//     and primitive ids equal the reference's (Scene::LoadModel, template/scene.h:156-201);
//   * mat4 construction / products (template/precomp.h:1007-1039, template.cpp:779-792);
//   * the plain binned-SAH BVH (template/scene.h:845-976), built with an explicit work
//     stack and precomputed per-primitive bounds, producing the identical node array;
//   * the SURVEY.md 8(d) benchmark scenes.
#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <limits>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <zlib.h>

#include "rt_internal.h"

namespace rt {

static thread_local std::string g_err;
void set_error(const std::string &msg) { g_err = msg; }
int fail(int code, const std::string &msg) { g_err = msg; return code; }

// ------------------------------------------------------------------ mat4
static void identity(float M[16]) { std::memset(M, 0, 64); M[0] = M[5] = M[10] = M[15] = 1.0f; }
void translate_matrix(float x, float y, float z, float M[16]) { identity(M); M[3] = x; M[7] = y; M[11] = z; }
static void mat_mul(const float *a, const float *b, float *out) {
    float r[16];
    for (int i = 0; i < 16; i += 4)
        for (int j = 0; j < 4; ++j)
            r[i + j] = (a[i + 0] * b[j + 0]) + (a[i + 1] * b[j + 4]) + (a[i + 2] * b[j + 8]) + (a[i + 3] * b[j + 12]);
    std::memcpy(out, r, 64);
}
static void mat_rotate(int axis, float a, float M[16]) {   // precomp.h:1007-1009
    identity(M);
    if (axis == 0) { M[5] = cosf(a); M[6] = -sinf(a); M[9] = sinf(a); M[10] = cosf(a); }
    else if (axis == 1) { M[0] = cosf(a); M[2] = sinf(a); M[8] = -sinf(a); M[10] = cosf(a); }
    else { M[0] = cosf(a); M[1] = -sinf(a); M[4] = sinf(a); M[5] = cosf(a); }
}
static const float kIdentity[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};

// ------------------------------------------------------------------ OBJ (tinyobj restatement)
namespace obj {
inline bool digit(char c) { return (unsigned)(c - '0') < 10u; }

// tryParseDouble, template/tiny_obj_loader.h:887-1016 -- the mantissa is accumulated in
// double exactly as tinyobj does, so the float cast yields the reference's vertex bits.
bool parse_double(const char *s, const char *end, double *out) {
    if (s >= end) return false;
    double mant = 0.0;
    int exponent = 0, read = 0;
    char sign = '+', esign = '+';
    const char *c = s;
    bool more = false, leading_dot = false;
    if (*c == '+' || *c == '-') {
        sign = *c++;
        if (c != end && *c == '.') leading_dot = true;
    } else if (*c == '.') {
        leading_dot = true;
    } else if (!digit(*c)) {
        return false;
    }
    more = (c != end);
    if (!leading_dot) {
        while (more && digit(*c)) { mant *= 10; mant += static_cast<int>(*c - 0x30); ++c; ++read; more = (c != end); }
        if (read == 0) return false;
    }
    if (more) {
        bool exp_next = false;
        if (*c == '.') {
            ++c; read = 1; more = (c != end);
            static const double lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            while (more && digit(*c)) {
                mant += static_cast<int>(*c - 0x30) * (read < 8 ? lut[read] : std::pow(10.0, -read));
                ++read; ++c; more = (c != end);
            }
            exp_next = more;
        } else if (*c == 'e' || *c == 'E') {
            exp_next = true;
        }
        if (exp_next && (*c == 'e' || *c == 'E')) {
            ++c; more = (c != end);
            if (more && (*c == '+' || *c == '-')) esign = *c++;
            else if (!digit(*c)) return false;
            read = 0; more = (c != end);
            while (more && digit(*c)) {
                if (exponent > 2147483647 / 10) return false;
                exponent = exponent * 10 + static_cast<int>(*c - 0x30);
                ++c; ++read; more = (c != end);
            }
            exponent *= (esign == '+' ? 1 : -1);
            if (read == 0) return false;
        }
    }
    *out = (sign == '+' ? 1 : -1) * (exponent ? std::ldexp(mant * std::pow(5.0, exponent), exponent) : mant);
    return true;
}

float real_token(const char *&tok) {   // parseReal, 1019-1027
    tok += std::strspn(tok, " \t");
    const char *end = tok + std::strcspn(tok, " \t\r");
    double v = 0.0;
    parse_double(tok, end, &v);
    tok = end;
    return static_cast<float>(v);
}

bool vertex_index(int idx, int n, int &out) {   // fixIndex, position slot (allow_zero = false)
    if (idx > 0) { out = idx - 1; return true; }
    if (idx == 0) return false;
    out = n + idx;
    return out >= 0;
}

struct Reader {
    std::vector<float> v;
    std::vector<int32_t> f;

    void face(const std::vector<int> &ids) {
        size_t n = ids.size();
        if (n < 3) return;                                   // degenerate face
        if (n == 3) { f.insert(f.end(), ids.begin(), ids.end()); return; }
        if (n == 4) {                                        // 1484-1580: split along the shorter diagonal
            for (int id : ids)
                if (3 * (size_t)id + 2 >= v.size()) return;  // invalid quad is skipped, 1496-1503
            const float *p0 = &v[3 * ids[0]], *p1 = &v[3 * ids[1]], *p2 = &v[3 * ids[2]], *p3 = &v[3 * ids[3]];
            float ax = p2[0] - p0[0], ay = p2[1] - p0[1], az = p2[2] - p0[2];
            float bx = p3[0] - p1[0], by = p3[1] - p1[1], bz = p3[2] - p1[2];
            float s02 = ax * ax + ay * ay + az * az, s13 = bx * bx + by * by + bz * bz;
            const int q[2][6] = {{0, 1, 2, 0, 2, 3}, {0, 1, 3, 1, 2, 3}};
            const int *sel = q[s02 < s13 ? 0 : 1];
            for (int k = 0; k < 6; ++k) f.push_back(ids[sel[k]]);
            return;
        }
        ear_clip(ids);
    }

    // pnpoly, template/tiny_obj_loader.h:1407-1419 (float)
    static bool inside3(const float *vx, const float *vy, float tx, float ty) {
        bool c = false;
        for (int i = 0, j = 2; i < 3; j = i++)
            if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
        return c;
    }

    // Polygons of 5+ corners: tinyobj's built-in ear clipping (tiny_obj_loader.h:1705-1928,
    // TINYOBJLOADER_USE_MAPBOX_EARCUT undefined, real_t = float): project on the two axes
    // picked from the first corner with a non-zero cross product, then cut ears starting at
    // guess_vert, skipping reflex corners and triangles that contain another corner.
    void ear_clip(const std::vector<int> &ids) {
        const size_t nv = v.size();
        size_t npolys = ids.size();
        size_t axes[2] = {1, 2};
        for (size_t k = 0; k < npolys; ++k) {
            const size_t a = (size_t)ids[k % npolys], b = (size_t)ids[(k + 1) % npolys], c = (size_t)ids[(k + 2) % npolys];
            if (3 * a + 2 >= nv || 3 * b + 2 >= nv || 3 * c + 2 >= nv) continue;
            const float e0x = v[3 * b] - v[3 * a], e0y = v[3 * b + 1] - v[3 * a + 1], e0z = v[3 * b + 2] - v[3 * a + 2];
            const float e1x = v[3 * c] - v[3 * b], e1y = v[3 * c + 1] - v[3 * b + 1], e1z = v[3 * c + 2] - v[3 * b + 2];
            const float cx = std::fabs(e0y * e1z - e0z * e1y);
            const float cy = std::fabs(e0z * e1x - e0x * e1z);
            const float cz = std::fabs(e0x * e1y - e0y * e1x);
            const float eps = std::numeric_limits<float>::epsilon();
            if (cx > eps || cy > eps || cz > eps) {
                if (!(cx > cy && cx > cz)) {
                    axes[0] = 0;
                    if (cz > cx && cz > cy) axes[1] = 1;
                }
                break;
            }
        }
        std::vector<int> rem(ids);
        size_t guess = 0, iters = rem.size(), prev = rem.size();
        auto coord = [&](int id, size_t ax) { return (size_t)id * 3 + ax < nv ? v[(size_t)id * 3 + ax] : 0.0f; };
        while (rem.size() > 3 && iters > 0) {
            npolys = rem.size();
            if (guess >= npolys) guess -= npolys;
            if (prev != npolys) { prev = npolys; iters = npolys; }
            else --iters;
            int ind[3];
            float vx[3], vy[3];
            for (size_t k = 0; k < 3; ++k) {
                ind[k] = rem[(guess + k) % npolys];
                const bool ok = (size_t)ind[k] * 3 + axes[0] < nv && (size_t)ind[k] * 3 + axes[1] < nv;
                vx[k] = ok ? v[(size_t)ind[k] * 3 + axes[0]] : 0.0f;
                vy[k] = ok ? v[(size_t)ind[k] * 3 + axes[1]] : 0.0f;
            }
            const float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0], e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
            const float cross = e0x * e1y - e0y * e1x;
            const float area = (vx[0] * vy[1] - vy[0] * vx[1]) * 0.5f;
            if (cross * area < 0.0f) { guess += 1; continue; }   // reflex corner
            bool overlap = false;
            for (size_t o = 3; o < npolys && !overlap; ++o) {
                const int id = rem[(guess + o) % npolys];
                if ((size_t)id * 3 + axes[0] >= nv || (size_t)id * 3 + axes[1] >= nv) continue;
                overlap = inside3(vx, vy, coord(id, axes[0]), coord(id, axes[1]));
            }
            if (overlap) { guess += 1; continue; }
            f.insert(f.end(), ind, ind + 3);                  // the ear
            rem.erase(rem.begin() + (long)((guess + 1) % npolys));
        }
        if (rem.size() == 3) f.insert(f.end(), rem.begin(), rem.end());
    }

    int line(const std::string &ln) {
        const char *t = ln.c_str();
        t += std::strspn(t, " \t");
        if (!*t || *t == '#') return 0;
        if (t[0] == 'v' && (t[1] == ' ' || t[1] == '\t')) {
            t += 2;
            for (int k = 0; k < 3; ++k) v.push_back(real_token(t));
            return 0;
        }
        if (t[0] == 'f' && (t[1] == ' ' || t[1] == '\t')) {
            t += 2;
            t += std::strspn(t, " \t");
            std::vector<int> ids;
            while (*t && *t != '\r' && *t != '\n') {
                int vi;
                if (!vertex_index(std::atoi(t), static_cast<int>(v.size() / 3), vi)) return -1;
                ids.push_back(vi);
                t += std::strcspn(t, " \t\r");
                t += std::strspn(t, " \t\r");
            }
            face(ids);
        }
        return 0;
    }
};
}  // namespace obj

// ------------------------------------------------------------------ primitive geometry
void fast_inverse(const float *c, float *r) {
    std::memcpy(r, kIdentity, sizeof(kIdentity));
    r[0] = c[0], r[1] = c[4], r[2] = c[8];
    r[4] = c[1], r[5] = c[5], r[6] = c[9];
    r[8] = c[2], r[9] = c[6], r[10] = c[10];
    r[3] = -(c[3] * r[0] + c[7] * r[1] + c[11] * r[2]);
    r[7] = -(c[3] * r[4] + c[7] * r[5] + c[11] * r[6]);
    r[11] = -(c[3] * r[8] + c[7] * r[9] + c[11] * r[10]);
}

void prim_transform(const rt_prim &p, const float *T16, PrimX &x) {
    const float *T = T16 ? T16 : kIdentity;
    if (p.type == RT_SPHERE) {
        translate_matrix(p.v[0], p.v[1], p.v[2], x.M);           // createSphere, Primitive.h:690-698
    } else if (p.type == RT_CUBE) {                               // createCube, Primitive.h:717-728
        const f3 pos = mk(p.v[0], p.v[1], p.v[2]);
        if (length(pos) > kFLT_EPSILON) {
            float Tr[16];
            translate_matrix(pos.x, pos.y, pos.z, Tr);
            mat_mul(T, Tr, x.M);
        } else {
            std::memcpy(x.M, T, sizeof(x.M));
        }
    } else if (p.type == RT_QUAD) {
        std::memcpy(x.M, T, sizeof(x.M));
    } else {
        std::memcpy(x.M, kIdentity, sizeof(x.M));
    }
    fast_inverse(x.M, x.Minv);
}

// the 8 cube corners / 4 quad corners in GetAABBMin/Max's order (Primitive.h:325-341)
static int box_corners(const rt_prim &p, const PrimX &x, f3 *c) {
    if (p.type == RT_CUBE) {
        const f3 a = -0.5f * mk(p.v[3], p.v[4], p.v[5]), b = 0.5f * mk(p.v[3], p.v[4], p.v[5]);
        c[0] = tpos(x.M, a);
        c[1] = tpos(x.M, mk(b.x, a.y, a.z));
        c[2] = tpos(x.M, mk(a.x, b.y, a.z));
        c[3] = tpos(x.M, mk(a.x, a.y, b.z));
        c[4] = tpos(x.M, b);
        c[5] = tpos(x.M, mk(a.x, b.y, b.z));
        c[6] = tpos(x.M, mk(b.x, a.y, b.z));
        c[7] = tpos(x.M, mk(b.x, b.y, a.z));
        return 8;
    }
    const float sz = 0.5f * p.v[0];
    c[0] = tpos(x.M, mk(-sz, 0, -sz));
    c[1] = tpos(x.M, mk(-sz, 0, sz));
    c[2] = tpos(x.M, mk(sz, 0, -sz));
    c[3] = tpos(x.M, mk(sz, 0, sz));
    return 4;
}

void prim_geometry(const rt_prim &p, const PrimX &x, PrimGeom &g) {
    if (p.type == RT_CUBE || p.type == RT_QUAD) {
        f3 c[8];
        const int n = box_corners(p, x, c);
        g.centroid = tpos(x.M, mk(0, 0, 0));                      // ctor leaves centroid 0
        g.bmin = g.bmax = c[0];
        for (int i = 1; i < n; ++i) { g.bmin = fmin3(g.bmin, c[i]); g.bmax = fmax3(g.bmax, c[i]); }
    } else if (p.type == RT_SPHERE) {
        f3 c = tpos(x.M, mk(0, 0, 0));
        float r = p.v[3];
        g.centroid = c;                       // centroid float3(0) through Transform
        g.bmin = c - mk(r, r, r);
        g.bmax = c + mk(r, r, r);
    } else if (p.type == RT_PLANE) {
        f3 n = mk(p.v[0], p.v[1], p.v[2]);
        g.centroid = tpos(kIdentity, (-n) * p.v[3]);
        g.bmin = mk(-1e30f, -1e30f, -1e30f);
        g.bmax = mk(1e30f, 1e30f, 1e30f);
    } else {
        f3 d0 = mk(p.v[0], p.v[1], p.v[2]), d1 = mk(p.v[3], p.v[4], p.v[5]), d2 = mk(p.v[6], p.v[7], p.v[8]);
        f3 A = tpos(kIdentity, d0), B = tpos(kIdentity, d1), C = tpos(kIdentity, d2);
        g.centroid = tpos(kIdentity, ((d0 + d1) + d2) / 3.0f);
        g.bmin = fmin3(A, fmin3(B, C));
        g.bmax = fmax3(A, fmax3(B, C));
    }
}

// ------------------------------------------------------------------ BVH
namespace {
struct Box { f3 mn, mx; };
inline Box empty_box() { return {mk(1e34f, 1e34f, 1e34f), mk(-1e34f, -1e34f, -1e34f)}; }   // aabb default
inline void grow(Box &b, f3 p) { b.mn = fmin3(b.mn, p); b.mx = fmax3(b.mx, p); }           // _mm_min/max_ps
inline void grow(Box &b, const Box &o) { b.mn = fmin3(b.mn, o.mn); b.mx = fmax3(b.mx, o.mx); }
inline float area(const Box &b) {                                                      // aabb::Area
    float e0 = b.mx.x - b.mn.x, e1 = b.mx.y - b.mn.y, e2 = b.mx.z - b.mn.z;
    return smax(0.0f, e0 * e1 + e0 * e2 + e1 * e2);
}

// The reference's recursive Subdivide (template/scene.h:866-910) on a thread pool: a node's
// split only reads and reorders its own index range, so subtrees are independent; child
// pairs are allocated in whatever order the workers finish and renumbered afterwards in
// the recursion's pre-order (left subtree before right), which reproduces nodesUsed's
// allocation order.  Nodes, indices, depth: identical to the sequential build.
class Builder {
  public:
    Builder(const std::vector<PrimGeom> &g, Bvh &b) : geo_(g), bvh_(b) {}

    void run(uint32_t n) {
        bvh_.indices.resize(n);
        for (uint32_t i = 0; i < n; ++i) bvh_.indices[i] = i;
        tmp_.assign(2 * (size_t)n + 2, Node{});
        kid_.assign(2 * (size_t)n + 2, 0u);
        tmp_[0].leftFirst = 0;
        tmp_[0].count = n;
        used_ = 2;   // node 1 skipped for 64-byte child pairs (scene.h:849)
        refit(0);
        unsigned hw = std::thread::hardware_concurrency();
        unsigned nt = n < 4 * kTaskMin ? 1u : std::max(1u, std::min(16u, hw ? hw : 1u));
        queue_.push_back(0);
        pending_ = 1;
        std::vector<std::thread> pool;
        for (unsigned t = 1; t < nt; ++t) pool.emplace_back([this] { worker(); });
        worker();
        for (auto &t : pool) t.join();
        renumber();
        bvh_.depth = depth(0);
        bvh_.max_leaf = 0;
        for (uint32_t i = 0; i < bvh_.nodes_used; ++i)
            if (i != 1 && bvh_.nodes[i].count > bvh_.max_leaf) bvh_.max_leaf = bvh_.nodes[i].count;
    }

  private:
    static constexpr uint32_t kTaskMin = 2048;   // smaller subtrees stay with their worker
    const std::vector<PrimGeom> &geo_;
    Bvh &bvh_;
    std::vector<Node> tmp_;            // nodes in allocation order
    std::vector<uint32_t> kid_;        // tmp index of an interior node's left child
    std::atomic<uint32_t> used_{2};
    std::mutex mu_;
    std::condition_variable cv_;
    std::vector<uint32_t> queue_;      // subtrees waiting for a worker
    uint32_t pending_ = 0;             // queued + running subtrees

    void worker() {
        for (;;) {
            uint32_t root;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return !queue_.empty() || pending_ == 0; });
                if (queue_.empty()) return;
                root = queue_.back();
                queue_.pop_back();
            }
            std::vector<uint32_t> work{root};
            while (!work.empty()) {
                const uint32_t ni = work.back();
                work.pop_back();
                uint32_t l;
                if (!split(ni, l)) continue;
                for (uint32_t c : {l + 1, l}) {
                    if (tmp_[c].count >= kTaskMin) {
                        std::lock_guard<std::mutex> lk(mu_);
                        queue_.push_back(c);
                        ++pending_;
                        cv_.notify_one();
                    } else {
                        work.push_back(c);
                    }
                }
            }
            std::lock_guard<std::mutex> lk(mu_);
            if (--pending_ == 0) cv_.notify_all();
        }
    }

    // final ids: pairs handed out in the recursion's pre-order
    void renumber() {
        bvh_.nodes.assign(tmp_.size(), Node{});
        bvh_.nodes_used = 2;
        std::vector<std::pair<uint32_t, uint32_t>> st{{0u, 0u}};   // (tmp id, final id)
        while (!st.empty()) {
            auto [t, f] = st.back();
            st.pop_back();
            Node nd = tmp_[t];
            if (nd.count == 0) {
                const uint32_t pair = bvh_.nodes_used;
                bvh_.nodes_used += 2;
                nd.leftFirst = pair;
                st.push_back({kid_[t] + 1, pair + 1});
                st.push_back({kid_[t], pair});
            }
            bvh_.nodes[f] = nd;
        }
    }

    void refit(uint32_t ni) {   // UpdateNodeBounds
        Node &n = tmp_[ni];
        f3 mn = mk(1e30f, 1e30f, 1e30f), mx = mk(-1e30f, -1e30f, -1e30f);
        for (uint32_t i = 0; i < n.count; ++i) {
            const PrimGeom &g = geo_[bvh_.indices[n.leftFirst + i]];
            mn = fmin3(mn, g.bmin);
            mx = fmax3(mx, g.bmax);
        }
        n.mn[0] = mn.x; n.mn[1] = mn.y; n.mn[2] = mn.z;
        n.mx[0] = mx.x; n.mx[1] = mx.y; n.mx[2] = mx.z;
    }

    float best_plane(const Node &n, int &axis, float &pos) const {   // FindBestSplitPlane
        float best = 1e30f;
        const uint32_t *ix = bvh_.indices.data() + n.leftFirst;
        for (int a = 0; a < 3; ++a) {
            float lo = 1e30f, hi = -1e30f;
            for (uint32_t i = 0; i < n.count; ++i) {
                float c = comp(geo_[ix[i]].centroid, a);
                lo = smin(lo, c);
                hi = smax(hi, c);
            }
            if (lo == hi) continue;
            Box bins[32];
            int cnt[32] = {0};
            for (auto &b : bins) b = empty_box();
            float scale = 32 / (hi - lo);
            for (uint32_t i = 0; i < n.count; ++i) {
                const PrimGeom &g = geo_[ix[i]];
                int b = static_cast<int>((comp(g.centroid, a) - lo) * scale);
                b = b < 31 ? b : 31;
                cnt[b]++;
                grow(bins[b], g.bmin);
                grow(bins[b], g.bmax);
            }
            float la[31], ra[31];
            int lc[31], rc[31];
            Box L = empty_box(), R = empty_box();
            int ls = 0, rs = 0;
            for (int i = 0; i < 31; ++i) {
                ls += cnt[i]; lc[i] = ls; grow(L, bins[i]); la[i] = area(L);
                rs += cnt[31 - i]; rc[30 - i] = rs; grow(R, bins[31 - i]); ra[30 - i] = area(R);
            }
            float step = (hi - lo) / 32;
            for (int i = 0; i < 31; ++i) {
                float cost = (float)lc[i] * la[i] + (float)rc[i] * ra[i];
                if (cost < best) { axis = a; pos = lo + step * (float)(i + 1); best = cost; }
            }
        }
        return best;
    }

    bool split(uint32_t ni, uint32_t &left) {   // Subdivide, minus the recursion
        Node n = tmp_[ni];
        int axis = 0;
        float pos = 0.0f;
        float cost = best_plane(n, axis, pos);
        float ex = n.mx[0] - n.mn[0], ey = n.mx[1] - n.mn[1], ez = n.mx[2] - n.mn[2];
        if (cost >= (float)n.count * (ex * ey + ey * ez + ez * ex)) return false;
        int i = (int)n.leftFirst, j = i + (int)n.count - 1;
        uint32_t *ix = bvh_.indices.data();
        while (i <= j) {
            if (comp(geo_[ix[i]].centroid, axis) < pos) ++i;
            else std::swap(ix[i], ix[j--]);
        }
        int lcount = i - (int)n.leftFirst;
        if (lcount == 0 || lcount == (int)n.count) return false;
        left = used_.fetch_add(2);
        Node &l = tmp_[left], &r = tmp_[left + 1];
        l.leftFirst = n.leftFirst; l.count = (uint32_t)lcount;
        r.leftFirst = (uint32_t)i; r.count = n.count - (uint32_t)lcount;
        kid_[ni] = left;
        tmp_[ni].leftFirst = left;
        tmp_[ni].count = 0;
        refit(left);
        refit(left + 1);
        return true;
    }

    uint32_t depth(uint32_t ni) const {   // maxDepthBVH, iterative
        std::vector<std::pair<uint32_t, uint32_t>> st{{ni, 0}};
        uint32_t best = 0;
        while (!st.empty()) {
            auto [k, d] = st.back();
            st.pop_back();
            const Node &n = bvh_.nodes[k];
            if (n.count > 0) { best = std::max(best, k == 0 ? 1u : d); continue; }
            st.push_back({n.leftFirst, d + 1});
            st.push_back({n.leftFirst + 1, d + 1});
        }
        return best;
    }
};
}  // namespace

int build_bvh(const rt_prim *prims, const float *transforms, uint32_t n, Bvh &out) {
    if (n == 0) return fail(RT_ERR_INVALID, "scene has no primitives");
    std::vector<PrimGeom> geo(n);
    for (uint32_t i = 0; i < n; ++i) {
        PrimX x;
        prim_transform(prims[i], transforms ? transforms + 16 * (size_t)i : nullptr, x);
        prim_geometry(prims[i], x, geo[i]);
    }
    Builder(geo, out).run(n);
    return RT_OK;
}

// ------------------------------------------------------------------ mesh container
static int mesh_read(const std::string &path, std::vector<float> &V, std::vector<int32_t> &F) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return fail(RT_ERR_IO, "cannot open " + path);
    char magic[8];
    uint32_t h[2];
    in.read(magic, 8);
    in.read(reinterpret_cast<char *>(h), 8);
    if (!in || std::memcmp(magic, "RTMESH1", 8) != 0) return fail(RT_ERR_IO, "not an RTMESH1 file: " + path);
    V.resize(3 * (size_t)h[0]);
    F.resize(3 * (size_t)h[1]);
    in.read(reinterpret_cast<char *>(V.data()), 4 * V.size());
    in.read(reinterpret_cast<char *>(F.data()), 4 * F.size());
    if (!in) return fail(RT_ERR_IO, "truncated RTMESH1 file: " + path);
    for (int32_t f : F)
        if (f < 0 || (uint32_t)f >= h[0]) return fail(RT_ERR_IO, "face index out of range in " + path);
    return RT_OK;
}

// tinyobj-compatible OBJ read (Scene::LoadModel's LoadObj, template/scene.h:156-161)
static int obj_read(const std::string &path, std::vector<float> &V, std::vector<int32_t> &F) {
    std::ifstream in(path, std::ios::binary);
    if (!in) return fail(RT_ERR_IO, "cannot open " + path);
    obj::Reader rd;
    std::string line;
    size_t lineno = 0;
    while (std::getline(in, line)) {   // '\n' lines; the trailing '\r' of CRLF is dropped
        ++lineno;
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (rd.line(line) != 0) return fail(RT_ERR_IO, "bad face at line " + std::to_string(lineno) + " of " + path);
    }
    V.swap(rd.v);
    F.swap(rd.f);
    return RT_OK;
}

static void append_mesh(const std::vector<float> &V, const std::vector<int32_t> &F, const float M[16], int32_t mat,
                        std::vector<rt_prim> &out) {
    size_t nt = F.size() / 3;
    size_t base = out.size();
    out.resize(base + nt);
    for (size_t f = 0; f < nt; ++f) {
        rt_prim &p = out[base + f];
        p.type = RT_TRIANGLE;
        p.material = mat;
        for (int k = 0; k < 3; ++k) {
            const float *q = &V[3 * (size_t)F[3 * f + k]];
            f3 w = tpos(M, mk(q[0], q[1], q[2]));   // TransformPosition(float3(vx,vy,vz), transform)
            p.v[3 * k] = w.x; p.v[3 * k + 1] = w.y; p.v[3 * k + 2] = w.z;
        }
    }
}

// ------------------------------------------------------------------ SURVEY 8(d) scenes
int recipe_source(const std::string &name, const std::string &dir, SceneSource &out) {
    out.prims.clear();
    out.materials.clear();
    auto material = [&](int32_t kind, f3 c, f3 c2 = mk(0, 0, 0), float ior = 0, float diffuse = -1.0f) {
        rt_material m{};
        m.kind = kind;
        m.color[0] = c.x; m.color[1] = c.y; m.color[2] = c.z;
        m.color2[0] = c2.x; m.color2[1] = c2.y; m.color2[2] = c2.z;
        m.ior = ior;
        m.diffuse = diffuse;
        out.materials.push_back(m);
        return (int32_t)out.materials.size() - 1;
    };
    auto sphere = [&](f3 c, float r, int32_t mat) {
        rt_prim p{};
        p.type = RT_SPHERE; p.material = mat;
        p.v[0] = c.x; p.v[1] = c.y; p.v[2] = c.z; p.v[3] = r;
        out.prims.push_back(p);
    };
    auto tri = [&](f3 a, f3 b, f3 c, int32_t mat) {
        rt_prim p{};
        p.type = RT_TRIANGLE; p.material = mat;
        f3 v[3] = {a, b, c};
        for (int k = 0; k < 3; ++k) { p.v[3 * k] = v[k].x; p.v[3 * k + 1] = v[k].y; p.v[3 * k + 2] = v[k].z; }
        out.prims.push_back(p);
    };
    auto mesh = [&](const char *file, const float M[16], int32_t mat) {
        std::vector<float> V;
        std::vector<int32_t> F;
        // the bundled RTMESH1 file, or the reference's own assets/<file>.obj in that directory
        const std::string base = dir + "/" + file;
        int rc = std::ifstream(base + ".rtmesh").good() ? mesh_read(base + ".rtmesh", V, F) : obj_read(base + ".obj", V, F);
        if (rc == RT_OK) append_mesh(V, F, M, mat, out.prims);
        return rc;
    };
    auto floor2 = [&](int32_t mat) {   // the two checkerboard floor triangles of SURVEY 8(d)
        const float y = -1.225f;
        tri(mk(-20, y, -1), mk(20, y, -1), mk(20, y, 40), mat);
        tri(mk(-20, y, -1), mk(20, y, 40), mk(-20, y, 40), mat);
    };
    auto chain = [](std::initializer_list<const float *> ms, float *M) {
        auto it = ms.begin();
        std::memcpy(M, *it, 64);
        for (++it; it != ms.end(); ++it) mat_mul(M, *it, M);
    };

    int32_t lamp = material(RT_LIGHT, mk(24.0f, 24.0f, 22.0f));          // scene.h:55
    int32_t white = material(RT_DIFFUSE, mk(0.95f, 0.95f, 0.95f));       // scene.h:46
    int32_t green = material(RT_DIFFUSE, mk(0.05f, 0.95f, 0.05f));       // scene.h:44
    int32_t check = material(RT_CHECKERBOARD, mk(0.1f, 0.1f, 0.1f), mk(0.9f, 0.9f, 0.9f));   // scene.h:50
    bool high_light = (name == "teapot" || name == "mig16" || name == "default");
    sphere(high_light ? mk(0.0f, 6.0f, 5.0f) : mk(0.0f, 4.0f, -2.0f), 0.5f, lamp);

    float T[16], R[16], R2[16], R3[16], S[16], M[16];
    int rc = RT_OK;
    if (name == "teapotF" || name == "teapot") {
        bool f = (name == "teapotF");
        translate_matrix(0, 0, f ? 2.0f : 1.5f, T);
        mat_rotate(1, 0.5f * kPI, R);
        identity(S); S[0] = S[5] = S[10] = f ? 2.5f : 1.5f;
        chain({T, R, S}, M);
        rc = mesh("teapot", M, white);
        if (f) floor2(check);
    } else if (name == "mig16") {
        for (int i = 0; i < 16 && rc == RT_OK; ++i) {
            float x = (float)(i % 4) - 1.5f, y = (float)(i / 4) - 1.5f;
            translate_matrix(x * 1.8f, y * 1.1f - 0.3f, 2.5f, T);
            mat_rotate(0, 0.3f * kPI, R);
            identity(S); S[0] = S[5] = S[10] = 0.01f;
            chain({T, R, S}, M);
            rc = mesh("mig29", M, green);
        }
    } else if (name == "cfg3") {
        int32_t glass = material(RT_DIELECTRIC, mk(0.5f, 0.5f, 0.5f), mk(0, 0, 0), 1.52f);
        int32_t mirror = material(RT_MIRROR, mk(0.9f, 0.75f, 0.0f));
        translate_matrix(0, -1, 2, T);
        identity(S); S[0] = S[5] = S[10] = 8.0f;
        chain({T, S}, M);
        rc = mesh("Shiba", M, glass);
        if (rc == RT_OK) {   // glider transform, template/scene.h:88
            translate_matrix(1.0f, 0.0f, 0.0f, T);
            mat_rotate(2, -0.15f * kPI, R); mat_rotate(1, 0.05f * kPI, R2); mat_rotate(0, -0.55f * kPI, R3);
            identity(S); S[0] = S[5] = S[10] = 0.025f;
            chain({T, R, R2, R3, S}, M);
            rc = mesh("glider", M, mirror);
        }
        floor2(check);
    } else if (name == "default") {
        // the reference's as-shipped Scene() (template/scene.h:40-128): light (0,6,5), then
        // cloud.obj, airways.obj, glider, piper_pa18.obj, mig29 -- cloud, airways and piper are
        // not in assets/, and LoadModel returns without triangles for them (scene.h:164-168)
        int32_t red = material(RT_DIFFUSE, mk(0.95f, 0.05f, 0.05f));     // scene.h:43
        translate_matrix(1.0f, 0.0f, 0.0f, T);                            // scene.h:88
        mat_rotate(2, -0.15f * kPI, R); mat_rotate(1, 0.05f * kPI, R2); mat_rotate(0, -0.55f * kPI, R3);
        identity(S); S[0] = S[5] = S[10] = 0.025f;
        chain({T, R, R2, R3, S}, M);
        rc = mesh("glider", M, red);
        if (rc == RT_OK) {                                                // scene.h:94
            translate_matrix(0.1f, 0.2f, -0.2f, T);
            mat_rotate(2, 1.1f * kPI, R); mat_rotate(1, 0.05f * kPI, R2); mat_rotate(0, 0.2f * kPI, R3);
            identity(S); S[0] = S[5] = S[10] = 0.001f;
            chain({T, R, R2, R3, S}, M);
            rc = mesh("mig29", M, green);
        }
    } else if (name == "cfg5") {
        translate_matrix(0, -1.2f, 2.5f, T);
        identity(S); S[0] = S[5] = S[10] = 12.0f;
        chain({T, S}, M);
        rc = mesh("Shiba", M, white);
        floor2(check);
    } else {
        return fail(RT_ERR_INVALID, "unknown scene recipe '" + name + "'");
    }
    return rc;
}

}  // namespace rt

using namespace rt;

// ------------------------------------------------------------------ C-ABI: host-side entry points
extern "C" {

int rt_abi_version(void) { return RT_ABI_VERSION; }
const char *rt_last_error(void) { return g_err.c_str(); }
void rt_free(void *p) { std::free(p); }

int rt_obj_load(const char *path, float **verts, uint32_t *nv, int32_t **faces, uint32_t *nt) {
    if (!path || !verts || !nv || !faces || !nt) return fail(RT_ERR_INVALID, "rt_obj_load: null argument");
    std::vector<float> V;
    std::vector<int32_t> F;
    int rc = obj_read(path, V, F);
    if (rc != RT_OK) return rc;
    *nv = (uint32_t)(V.size() / 3);
    *nt = (uint32_t)(F.size() / 3);
    *verts = static_cast<float *>(std::malloc(sizeof(float) * (V.size() ? V.size() : 1)));
    *faces = static_cast<int32_t *>(std::malloc(sizeof(int32_t) * (F.size() ? F.size() : 1)));
    std::memcpy(*verts, V.data(), sizeof(float) * V.size());
    std::memcpy(*faces, F.data(), sizeof(int32_t) * F.size());
    return RT_OK;
}

// ------------------------------------------------------------------ PNG (Surface::LoadImage)
namespace png {
inline uint32_t be32(const uint8_t *p) { return (uint32_t(p[0]) << 24) | (uint32_t(p[1]) << 16) | (uint32_t(p[2]) << 8) | p[3]; }
inline int paeth(int a, int b, int c) {
    int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}
// decode to 8-bit channels the way stbi_load(.., req_comp 0) reports them: grey 1, grey+alpha 2,
// RGB 3, RGBA 4, palette 3 (4 with tRNS); 16-bit samples keep their high byte, 1/2/4-bit grey
// is scaled to 0..255
int decode(const std::vector<uint8_t> &f, std::vector<uint8_t> &out, uint32_t &W, uint32_t &H, int &n) {
    static const uint8_t sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) return fail(RT_ERR_IO, "not a PNG file");
    size_t i = 8;
    int depth = 0, ctype = -1, interlace = 0;
    std::vector<uint8_t> idat, plte;
    bool trns = false;
    while (i + 8 <= f.size()) {
        const uint32_t len = be32(&f[i]);
        const uint8_t *type = &f[i + 4];
        if (i + 12 + (size_t)len > f.size()) return fail(RT_ERR_IO, "truncated PNG chunk");
        const uint8_t *d = &f[i + 8];
        if (!std::memcmp(type, "IHDR", 4)) {
            if (len < 13) return fail(RT_ERR_IO, "bad IHDR");
            W = be32(d); H = be32(d + 4); depth = d[8]; ctype = d[9]; interlace = d[12];
        } else if (!std::memcmp(type, "PLTE", 4)) {
            plte.assign(d, d + len);
        } else if (!std::memcmp(type, "tRNS", 4)) {
            trns = true;
        } else if (!std::memcmp(type, "IDAT", 4)) {
            idat.insert(idat.end(), d, d + len);
        } else if (!std::memcmp(type, "IEND", 4)) {
            break;
        }
        i += 12 + (size_t)len;
    }
    if (ctype < 0 || !W || !H) return fail(RT_ERR_IO, "PNG without IHDR");
    if (interlace) return fail(RT_ERR_UNSUPPORTED, "interlaced PNG");
    int ch;
    switch (ctype) {
    case 0: ch = 1; break;
    case 2: ch = 3; break;
    case 3: ch = 1; break;
    case 4: ch = 2; break;
    case 6: ch = 4; break;
    default: return fail(RT_ERR_IO, "bad PNG colour type");
    }
    if (!(depth == 8 || depth == 16 || ((ctype == 0 || ctype == 3) && (depth == 1 || depth == 2 || depth == 4))))
        return fail(RT_ERR_UNSUPPORTED, "PNG bit depth");
    if (ctype == 3 && plte.size() < 3) return fail(RT_ERR_IO, "palette PNG without PLTE");
    const size_t bits = (size_t)W * ch * depth, stride = (bits + 7) / 8;
    const size_t bpp = std::max<size_t>(1, (size_t)ch * depth / 8);
    std::vector<uint8_t> raw((stride + 1) * H);
    uLongf rawlen = (uLongf)raw.size();
    if (uncompress(raw.data(), &rawlen, idat.data(), (uLong)idat.size()) != Z_OK || rawlen != raw.size())
        return fail(RT_ERR_IO, "PNG image data does not inflate to the expected size");
    std::vector<uint8_t> cur(stride), prev(stride, 0);
    n = ctype == 3 ? (trns ? 4 : 3) : ch;
    out.assign((size_t)W * H * n, 0);
    for (uint32_t y = 0; y < H; ++y) {
        const uint8_t *r = &raw[(stride + 1) * y];
        const int ft = r[0];
        for (size_t x = 0; x < stride; ++x) {
            const int a = x >= bpp ? cur[x - bpp] : 0, b = prev[x], c = x >= bpp ? prev[x - bpp] : 0;
            int v = r[1 + x];
            switch (ft) {
            case 0: break;
            case 1: v += a; break;
            case 2: v += b; break;
            case 3: v += (a + b) >> 1; break;
            case 4: v += paeth(a, b, c); break;
            default: return fail(RT_ERR_IO, "bad PNG filter type");
            }
            cur[x] = (uint8_t)v;
        }
        uint8_t *o = &out[(size_t)W * n * y];
        for (uint32_t x = 0; x < W; ++x) {
            for (int k = 0; k < ch; ++k) {
                int s;
                if (depth == 16) s = cur[2 * ((size_t)x * ch + k)];
                else if (depth == 8) s = cur[(size_t)x * ch + k];
                else {   // 1/2/4-bit grey or palette index
                    const size_t bit = (size_t)x * depth;
                    s = (cur[bit >> 3] >> (8 - depth - (bit & 7))) & ((1 << depth) - 1);
                    if (ctype == 0) s *= depth == 1 ? 0xff : depth == 2 ? 0x55 : 0x11;
                }
                if (ctype == 3) {
                    if ((size_t)s * 3 + 2 >= plte.size()) return fail(RT_ERR_IO, "palette index out of range");
                    o[(size_t)x * n + 0] = plte[3 * s]; o[(size_t)x * n + 1] = plte[3 * s + 1];
                    o[(size_t)x * n + 2] = plte[3 * s + 2];
                    if (n == 4) o[(size_t)x * n + 3] = 255;
                } else {
                    o[(size_t)x * n + k] = (uint8_t)s;
                }
            }
        }
        std::swap(cur, prev);
    }
    return RT_OK;
}
}  // namespace png

int rt_image_load(const char *path, uint32_t **pixels, uint32_t *width, uint32_t *height) {
    if (!path || !pixels || !width || !height) return fail(RT_ERR_INVALID, "rt_image_load: null argument");
    std::ifstream in(path, std::ios::binary);
    if (!in) return fail(RT_ERR_IO, std::string("File not found: ") + path);
    std::vector<uint8_t> f((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
    std::vector<uint8_t> d;
    uint32_t W = 0, H = 0;
    int n = 0;
    int rc = png::decode(f, d, W, H, n);
    if (rc != RT_OK) return rc;
    const size_t s = (size_t)W * H;
    uint32_t *px = (uint32_t *)std::malloc(sizeof(uint32_t) * s);
    if (!px) return fail(RT_ERR_INVALID, "out of memory");
    if (n == 1) {                      // template/template.cpp:1587-1593
        for (size_t i = 0; i < s; ++i) { const uint32_t p = d[i]; px[i] = p + (p << 8) + (p << 16); }
    } else {                           // 1597: bytes i*n .. i*n+2 (past the end reads as 0)
        auto at = [&](size_t k) -> uint32_t { return k < d.size() ? d[k] : 0u; };
        for (size_t i = 0; i < s; ++i) px[i] = (at(i * n) << 16) + (at(i * n + 1) << 8) + at(i * n + 2);
    }
    *pixels = px; *width = W; *height = H;
    return RT_OK;
}

int rt_mesh_load(const char *path, float **verts, uint32_t *nv, int32_t **faces, uint32_t *nt) {
    if (!path || !verts || !nv || !faces || !nt) return fail(RT_ERR_INVALID, "rt_mesh_load: null argument");
    std::vector<float> V;
    std::vector<int32_t> F;
    int rc = mesh_read(path, V, F);
    if (rc != RT_OK) return rc;
    *nv = (uint32_t)(V.size() / 3);
    *nt = (uint32_t)(F.size() / 3);
    *verts = static_cast<float *>(std::malloc(sizeof(float) * (V.size() ? V.size() : 1)));
    *faces = static_cast<int32_t *>(std::malloc(sizeof(int32_t) * (F.size() ? F.size() : 1)));
    std::memcpy(*verts, V.data(), sizeof(float) * V.size());
    std::memcpy(*faces, F.data(), sizeof(int32_t) * F.size());
    return RT_OK;
}

int rt_mesh_save(const char *path, const float *verts, uint32_t nv, const int32_t *faces, uint32_t nt) {
    if (!path || (nv && !verts) || (nt && !faces)) return fail(RT_ERR_INVALID, "rt_mesh_save: null argument");
    std::ofstream out(path, std::ios::binary);
    if (!out) return fail(RT_ERR_IO, std::string("cannot write ") + path);
    uint32_t h[2] = {nv, nt};
    out.write("RTMESH1", 8);
    out.write(reinterpret_cast<const char *>(h), 8);
    out.write(reinterpret_cast<const char *>(verts), 12 * (size_t)nv);
    out.write(reinterpret_cast<const char *>(faces), 12 * (size_t)nt);
    return out ? RT_OK : fail(RT_ERR_IO, std::string("short write to ") + path);
}

int rt_mat4_translate(float x, float y, float z, float out[16]) {
    if (!out) return fail(RT_ERR_INVALID, "null matrix");
    translate_matrix(x, y, z, out);
    return RT_OK;
}
int rt_mat4_scale(float s, float out[16]) {
    if (!out) return fail(RT_ERR_INVALID, "null matrix");
    identity(out);
    out[0] = out[5] = out[10] = s;
    return RT_OK;
}
int rt_mat4_rotate(int axis, float angle, float out[16]) {
    if (!out || axis < 0 || axis > 2) return fail(RT_ERR_INVALID, "rt_mat4_rotate: axis must be 0, 1 or 2");
    mat_rotate(axis, angle, out);
    return RT_OK;
}
int rt_mat4_mul(const float a[16], const float b[16], float out[16]) {
    if (!a || !b || !out) return fail(RT_ERR_INVALID, "null matrix");
    mat_mul(a, b, out);
    return RT_OK;
}

int rt_mesh_to_prims(const float *verts, uint32_t nv, const int32_t *faces, uint32_t nt, const float M[16],
                     int32_t material, rt_prim *out) {
    if (!verts || !faces || !M || !out) return fail(RT_ERR_INVALID, "rt_mesh_to_prims: null argument");
    for (uint32_t i = 0; i < 3 * nt; ++i)
        if (faces[i] < 0 || (uint32_t)faces[i] >= nv) return fail(RT_ERR_INVALID, "face index out of range");
    std::vector<float> V(verts, verts + 3 * (size_t)nv);
    std::vector<int32_t> F(faces, faces + 3 * (size_t)nt);
    std::vector<rt_prim> tmp;
    append_mesh(V, F, M, material, tmp);
    std::memcpy(out, tmp.data(), sizeof(rt_prim) * tmp.size());
    return RT_OK;
}

int rt_recipe_describe(const char *name, const char *mesh_dir, rt_prim *prims, uint32_t *num_prims,
                       rt_material *materials, uint32_t *num_materials) {
    if (!name || !mesh_dir || !num_prims || !num_materials) return fail(RT_ERR_INVALID, "rt_recipe_describe: null argument");
    SceneSource src;
    int rc = recipe_source(name, mesh_dir, src);
    if (rc != RT_OK) return rc;
    if (prims) {
        if (*num_prims < src.prims.size() || *num_materials < src.materials.size() || !materials)
            return fail(RT_ERR_INVALID, "rt_recipe_describe: arrays too small");
        std::memcpy(prims, src.prims.data(), sizeof(rt_prim) * src.prims.size());
        std::memcpy(materials, src.materials.data(), sizeof(rt_material) * src.materials.size());
    }
    *num_prims = (uint32_t)src.prims.size();
    *num_materials = (uint32_t)src.materials.size();
    return RT_OK;
}

int rt_bvh_build_host(const rt_prim *prims, const float *transforms, uint32_t n, void *nodes, uint32_t *indices,
                      rt_scene_info *info) {
    if (!prims || !nodes || !indices) return fail(RT_ERR_INVALID, "rt_bvh_build_host: null argument");
    Bvh b;
    int rc = build_bvh(prims, transforms, n, b);
    if (rc != RT_OK) return rc;
    std::memcpy(nodes, b.nodes.data(), sizeof(Node) * b.nodes.size());
    std::memcpy(indices, b.indices.data(), sizeof(uint32_t) * n);
    if (info) { info->num_prims = n; info->nodes_used = b.nodes_used; info->depth = b.depth; info->max_leaf = b.max_leaf; info->num_refs = n; }
    return RT_OK;
}

int rt_sbvh_build_host(const rt_prim *prims, const float *transforms, uint32_t n, void **nodes, uint32_t **indices,
                       rt_scene_info *info) {
    if (!prims || !nodes || !indices) return fail(RT_ERR_INVALID, "rt_sbvh_build_host: null argument");
    *nodes = nullptr;
    *indices = nullptr;
    Bvh b;
    int rc = build_sbvh(prims, transforms, n, b);
    if (rc != RT_OK) return rc;
    *nodes = std::malloc(sizeof(Node) * b.nodes_used);
    *indices = static_cast<uint32_t *>(std::malloc(sizeof(uint32_t) * std::max<size_t>(1, b.indices.size())));
    if (!*nodes || !*indices) return fail(RT_ERR_INVALID, "rt_sbvh_build_host: out of memory");
    std::memcpy(*nodes, b.nodes.data(), sizeof(Node) * b.nodes_used);
    std::memcpy(*indices, b.indices.data(), sizeof(uint32_t) * b.indices.size());
    if (info) {
        info->num_prims = n; info->nodes_used = b.nodes_used; info->depth = b.depth; info->max_leaf = b.max_leaf;
        info->num_refs = (uint32_t)b.indices.size();
    }
    return RT_OK;
}

int rt_camera_default(uint32_t W, uint32_t H, rt_camera *c) {   // camera.h:28-41, 93-100
    if (!c || !W || !H) return fail(RT_ERR_INVALID, "rt_camera_default: bad argument");
    float aperture = (float)0.000005;
    float lens = aperture / 2.0f, focus = 1.0f, fov = 1.0f;
    float aspect = (float)W / (float)H;
    f3 pos = mk(0, 0, -fov);
    f3 tl = pos + focus * mk(-aspect, 1, fov), tr = pos + focus * mk(aspect, 1, fov), bl = pos + focus * mk(-aspect, -1, fov);
    const f3 *src[4] = {&pos, &tl, &tr, &bl};
    float *dst[4] = {c->pos, c->top_left, c->top_right, c->bottom_left};
    for (int i = 0; i < 4; ++i) { dst[i][0] = src[i]->x; dst[i][1] = src[i]->y; dst[i][2] = src[i]->z; }
    c->lens_radius = lens;
    return RT_OK;
}

}  // extern "C"
