// xaccel_check.cpp — CPU check of the Mode X acceleration structure built by libgi's host code
// (gi_build.cpp + gi_bvh.cpp, compiled here by g++ from the same sources).
//
//  * structure: every primitive in exactly one leaf (BVH) / at least one leaf (octree, and the
//    spatial-split BVH of scenes over 8192 primitives: scene 2), every fp32 child box of a BVH
//    without spatial splits contains its subtree's fp64 primitive bounds, parent pointers consistent,
//    depth within the 16 mask levels of the traversal;
//  * traversal: the kernel's stackless front-to-back walk (k_mode_x, restated here step for step:
//    per-level 8-bit child masks, slot k ^ octant order, re-cull against the current best t)
//    returns the same closest hit (t, primitive) as a brute-force loop over all primitives, for
//    closest and any-hit (shadow) queries, on random soups and on the Cornell box.
//   xaccel_check <n_rays>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "gi.h"
#include "gi_scene.h"

namespace gi {
bool build_host_scene(const gi_scene_desc& desc, HostScene& hs, std::string& err);
}
using namespace gi;

static uint64_t g_rng = 0x2019;
static double urand() {
    g_rng += 0x9E3779B97F4A7C15ULL;
    uint64_t z = g_rng;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return (double)(z >> 11) * 0x1.0p-53;
}

static double prim_t(const XHot& p, V3 o, V3 d, double tmin) {   // the kernel's x_prim_t
    if (p.kind == 0) {
        const V3 e1 = ld3(p.b), e2 = ld3(p.c);
        const V3 pv = fcross(d, e2);
        const double det = fdot(e1, pv);
        if (det == 0.0) return INFINITY;
        const V3 tv = o - ld3(p.a);
        const double un = fdot(tv, pv);
        if (det > 0.0 ? (un < 0.0 || un > det) : (un > 0.0 || un < det)) return INFINITY;
        const V3 qv = fcross(tv, e1);
        const double vn = fdot(d, qv);
        const double uvn = un + vn;
        if (det > 0.0 ? (vn < 0.0 || uvn > det) : (vn > 0.0 || uvn < det)) return INFINITY;
        const double t = fdot(e2, qv) / det;
        return (t > tmin) ? t : INFINITY;
    }
    const V3 oc = o - ld3(p.a);
    const double b = fdot(oc, d);
    const double r = p.b[0];
    const double c2 = gfma(-r, r, fdot(oc, oc));
    const double disc = gfma(b, b, -c2);
    if (disc < 0.0) return INFINITY;
    const double sq = std::sqrt(disc);
    double t = -b - sq;
    if (t > tmin) return t;
    t = -b + sq;
    return (t > tmin) ? t : INFINITY;
}

static XHot hot_of(const XPrim& p, int i) {
    XHot h;
    for (int k = 0; k < 3; ++k) { h.a[k] = p.a[k]; h.b[k] = p.b[k]; h.c[k] = p.c[k]; }
    h.prim = i;
    h.kind = p.kind;
    return h;
}

static float up32(double v) {
    float f = (float)v;
    if ((double)f < v) f = std::nextafter(f, INFINITY);
    return f;
}
struct F3 { float x, y, z; };
// the kernel's inv_dir: reciprocal clamped to +-1e30 (finite plane distances for axis-parallel rays)
static float inv_clamp(float v) { return std::fmin(std::fmax(1.0f / v, -1e30f), 1e30f); }
// pass 3: the quantised nodes with the kernel's fused arithmetic (children_mask(const XCNode*)):
// t = fma(q, 2^e * iv, fma(org, iv, -(o * iv))) per bound, set while g_xc is non-null
static const XCNode* g_xc = nullptr;
static const XWNode* g_xw_base = nullptr;
static bool child_hit_xc(const XCNode& n, int c, F3 of, F3 ivf, float tmax) {
    const float iv[3] = {ivf.x, ivf.y, ivf.z}, o[3] = {of.x, of.y, of.z};
    float tn = 0.0f, tf = tmax;
    for (int a = 0; a < 3; ++a) {
        const float no = -(o[a] * iv[a]);
        const float siv = std::ldexp(1.0f, n.ex[a]) * iv[a], base = std::fmaf(n.org[a], iv[a], no);
        const float tl = std::fmaf((float)n.qlo[a][c], siv, base), th = std::fmaf((float)n.qhi[a][c], siv, base);
        const bool neg = std::signbit(iv[a]);
        tn = std::fmax(tn, neg ? th : tl);
        tf = std::fmin(tf, neg ? tl : th);
    }
    return tn <= tf;
}
// the kernel's form: plane distance fma(b, iv, -(o * iv))
static bool child_hit(const XWNode* nd, int c, F3 of, F3 ivf, float tmax) {
    if (g_xc) return child_hit_xc(g_xc[nd - g_xw_base], c, of, ivf, tmax);
    const float nx = -(of.x * ivf.x), ny = -(of.y * ivf.y), nz = -(of.z * ivf.z);
    const float tx0 = std::fmaf(nd->lo[0][c], ivf.x, nx), tx1 = std::fmaf(nd->hi[0][c], ivf.x, nx);
    const float ty0 = std::fmaf(nd->lo[1][c], ivf.y, ny), ty1 = std::fmaf(nd->hi[1][c], ivf.y, ny);
    const float tz0 = std::fmaf(nd->lo[2][c], ivf.z, nz), tz1 = std::fmaf(nd->hi[2][c], ivf.z, nz);
    const float tn = std::fmax(std::fmax(std::fmin(tx0, tx1), std::fmin(ty0, ty1)), std::fmax(std::fmin(tz0, tz1), 0.0f));
    const float tf = std::fmin(std::fmin(std::fmax(tx0, tx1), std::fmax(ty0, ty1)), std::fmin(std::fmax(tz0, tz1), tmax));
    return tn <= tf;
}
// skip: a plane group whose leaf children are left out (the kernels' own-plane skip; -1 none)
static uint32_t children_mask(const XWNode* nd, F3 of, F3 ivf, float tmax, int dmask, int skip = -1) {
    uint32_t m = 0;
    const uint8_t* pg = reinterpret_cast<const uint8_t*>(nd->pad);
    for (int c = 0; c < 8; ++c)
        if (nd->child[c] != XEMPTY && child_hit(nd, c, of, ivf, tmax) && !(nd->child[c] < 0 && pg[c] == skip))
            m |= 1u << (c ^ dmask);
    return m;
}
static uint32_t lvl_get(uint64_t lo, uint64_t hi, int l) { return (uint32_t)((l < 8 ? lo >> (8 * l) : hi >> (8 * (l - 8))) & 0xFF); }
static void lvl_set(uint64_t& lo, uint64_t& hi, int l, uint32_t m) {
    if (l < 8) lo = (lo & ~(0xFFull << (8 * l))) | ((uint64_t)m << (8 * l));
    else hi = (hi & ~(0xFFull << (8 * (l - 8)))) | ((uint64_t)m << (8 * (l - 8)));
}

// k_mode_x's traversal of one ray; shadow: any hit with t < tmax
static long g_prim_tests = 0;
static int traverse(const HostScene& s, V3 o, V3 d, bool shadow, double tmax, double& tbest, long& visits, int skip = -1) {
    // the device uses v_rcp_f32 (1 ulp) here; the correctly rounded fp32 reciprocal stands in for it
    const F3 of = {(float)o.x, (float)o.y, (float)o.z}, ivf = {inv_clamp((float)d.x), inv_clamp((float)d.y), inv_clamp((float)d.z)};
    const int dmask = (d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0);
    tbest = shadow ? tmax : INFINITY;
    float tbest_f = shadow ? up32(tmax) : INFINITY;
    int best = -1, node = 0, level = 0;
    uint64_t mlo = 0, mhi = 0;
    const uint32_t rm = children_mask(&s.xwnodes[0], of, ivf, tbest_f, dmask, skip);
    lvl_set(mlo, mhi, 0, rm);
    bool raying = rm != 0;
    while (raying) {   // one iteration = one traversal step of k_mode_x
        const uint32_t msk = lvl_get(mlo, mhi, level);
        const int k = __builtin_ctz(msk);
        lvl_set(mlo, mhi, level, msk & (msk - 1));
        const int c = k ^ dmask;
        const XWNode* nd = &s.xwnodes[node];
        const int ch = nd->child[c];
        const bool keep = shadow || best < 0 || child_hit(nd, c, of, ivf, tbest_f);
        if (keep) {
            if (ch < 0) {
                for (int j = 0; j < nd->cnt[c]; ++j) {
                    const XHot& h = s.xhot[~ch + j];
                    const double t = prim_t(h, o, d, 1e-7);
                    ++g_prim_tests;
                    if (shadow) {
                        if (t < tmax) return h.prim;
                    } else if (t < tbest || (t == tbest && h.prim < best)) {
                        tbest = t;
                        best = h.prim;
                        tbest_f = up32(t);
                    }
                }
            } else {
                ++visits;
                const uint32_t cm = children_mask(&s.xwnodes[ch], of, ivf, tbest_f, dmask, skip);
                if (cm) {
                    node = ch;
                    ++level;
                    if (level > 15) { std::printf("depth overflow\n"); std::exit(3); }
                    lvl_set(mlo, mhi, level, cm);
                }
            }
        }
        uint32_t rest = lvl_get(mlo, mhi, level);
        while (rest == 0 && level > 0) {
            node = s.xwnodes[node].parent;
            --level;
            rest = lvl_get(mlo, mhi, level);
        }
        if (rest == 0) raying = false;
    }
    return best;
}

static int brute(const HostScene& s, V3 o, V3 d, bool shadow, double tmax, double& tbest) {
    tbest = INFINITY;
    int best = -1;
    for (size_t i = 0; i < s.xprims.size(); ++i) {
        const double t = prim_t(hot_of(s.xprims[i], (int)i), o, d, 1e-7);
        if (shadow) {
            if (t < tmax) return (int)i;
        } else if (t < tbest) {
            tbest = t;
            best = (int)i;
        }
    }
    return best;
}

static int check_structure(const HostScene& s, bool exact_once) {
    std::vector<int> seen(s.xprims.size(), 0);
    for (size_t w = 0; w < s.xwnodes.size(); ++w) {
        const XWNode& n = s.xwnodes[w];
        for (int c = 0; c < 8; ++c) {
            if (n.child[c] == XEMPTY) continue;
            if (n.child[c] >= 0) {
                if (s.xwnodes[n.child[c]].parent != (int)w) { std::printf("parent mismatch\n"); return 1; }
                continue;
            }
            for (int j = 0; j < n.cnt[c]; ++j) {
                const XHot& h = s.xhot[~n.child[c] + j];
                ++seen[h.prim];
                const XPrim& p = s.xprims[h.prim];
                double mn[3], mx[3];
                for (int k = 0; k < 3; ++k) {
                    if (p.kind == 1) { mn[k] = p.a[k] - p.b[0]; mx[k] = p.a[k] + p.b[0]; }
                    else {
                        const double v0 = p.a[k], v1 = p.a[k] + p.b[k], v2 = p.a[k] + p.c[k];
                        mn[k] = std::fmin(std::fmin(v0, v1), v2);
                        mx[k] = std::fmax(std::fmax(v0, v1), v2);
                    }
                    // the BVH pads with 1e-5*extent, far above the rounding of p.a + p.b (the octree
                    // clips a primitive's box to each cell it overlaps, so only the BVH contains it)
                    if (exact_once && ((double)n.lo[k][c] > mn[k] || (double)n.hi[k][c] < mx[k])) {
                        std::printf("box does not contain prim\n");
                        return 1;
                    }
                }
            }
        }
    }
    for (size_t i = 0; i < seen.size(); ++i)
        if (seen[i] == 0 || (exact_once && seen[i] != 1)) { std::printf("prim %zu seen %d times\n", i, seen[i]); return 1; }
    return 0;
}

// Quantised nodes (XCNode, the HBM-resident kernel's): every decoded child box -- fma(q, 2^e, org)
// in fp32, as the kernel decodes it -- must contain the XWNode box; returns the nodes with the
// decoded boxes, so that the traversal can be checked on them as well.
static int check_quantised(const HostScene& s, std::vector<XWNode>& dec) {
    std::vector<XCNode> q;
    dec = s.xwnodes;
    if (!encode_xcnodes(s.xwnodes, q)) {   // a leaf of more than 255 records: the scene keeps XWNode
        std::printf("quantised nodes: not encodable, XWNode kept\n");
        return 0;
    }
    for (size_t w = 0; w < q.size(); ++w) {
        const XCNode& n = q[w];
        if (n.exists != (uint8_t)s.xwnodes[w].exists || n.parent != s.xwnodes[w].parent) { std::printf("xc header\n"); return 1; }
        for (int c = 0; c < 8; ++c) {
            if (n.child[c] != s.xwnodes[w].child[c] || n.cnt[c] != s.xwnodes[w].cnt[c]) { std::printf("xc refs\n"); return 1; }
            if (!((n.exists >> c) & 1)) continue;
            for (int a = 0; a < 3; ++a) {
                const float sc = std::ldexp(1.0f, n.ex[a]);
                const float lo = std::fmaf((float)n.qlo[a][c], sc, n.org[a]), hi = std::fmaf((float)n.qhi[a][c], sc, n.org[a]);
                if (!(lo <= s.xwnodes[w].lo[a][c] && hi >= s.xwnodes[w].hi[a][c])) {
                    std::printf("quantised box does not contain node %zu child %d axis %d\n", w, c, a);
                    return 1;
                }
                dec[w].lo[a][c] = lo;
                dec[w].hi[a][c] = hi;
            }
        }
    }
    return 0;
}

static gi_entity_desc tri(double* v) {
    gi_entity_desc e{};
    e.kind = GI_IMP_TRIANGLE;
    for (int k = 0; k < 9; ++k) e.args[k] = v[k];
    return e;
}

// optional: a .scn file (impsphere / imptriangle lines only), e.g. the Cornell box
static bool read_scn(const char* path, std::vector<gi_entity_desc>& ents) {
    std::ifstream f(path);
    std::string line;
    while (std::getline(f, line)) {
        std::istringstream is(line);
        std::string kw;
        is >> kw;
        std::vector<double> v;
        double x;
        while (is >> x) v.push_back(x);
        gi_entity_desc e{};
        if (kw == "imptriangle") e.kind = GI_IMP_TRIANGLE;
        else if (kw == "impsphere") e.kind = GI_IMP_SPHERE;
        else continue;
        for (size_t k = 0; k < v.size() && k < 11; ++k) e.args[k] = v[k];
        ents.push_back(e);
    }
    return !ents.empty();
}

// The own-plane skip (gi_build.cpp assign_plane_groups; gi_wf.hip x_segment): rays leaving a hit
// point on a grouped triangle -- the hit computed as the kernel does, P = o + t d with t from the exact
// test -- toward random targets (shadow: any hit before tmax) and in directions of prescribed incidence
// |d . n| from 1 down to just above the scene's bound, with the origin's group skipped when the
// incidence clears the bound: the same closest hit (t, primitive) / the same any-hit answer as brute
// force.  Below the bound the kernels do not skip; those rays are checked unskipped.  Returns mismatches.
static long check_plane_skip(const HostScene& hs, int nrays, long& skipped, long& total) {
    long bad = 0;
    const int np = (int)hs.xprims.size();
    if (np == 0) return 0;
    for (int r = 0; r < nrays; ++r) {
        const int i = (int)(urand() * np) % np;
        const XPrim& x = hs.xprims[i];
        if (x.kind != 0 || x.pad[0] == 255) continue;
        const V3 o = (r % 4 == 0) ? v3(-10, 0, 0) : v3(urand() * 12 - 1, urand() * 12 - 6, urand() * 12 - 6);
        double a = urand(), b = urand();
        if (a + b > 1) { a = 1 - a; b = 1 - b; }
        const V3 tgt = ld3(x.a) + ld3(x.b) * a + ld3(x.c) * b;
        const V3 d = normalize(tgt - o);
        const double t = prim_t(hot_of(x, i), o, d, 1e-7);
        if (!std::isfinite(t)) continue;
        const V3 P = o + t * d;   // as x_segment computes the hit point
        const V3 n = ld3(x.n);
        const double cmin = hs.x_skip_a * std::max(std::fabs(o.x), std::max(std::fabs(o.y), std::fabs(o.z))) + hs.x_skip_b;
        V3 d2;
        double tmax = INFINITY;
        const int kind = r % 5;
        if (kind == 0) {   // shadow ray toward a random point
            const V3 L = v3(urand() * 12 - 1, urand() * 12 - 6, urand() * 12 - 6);
            tmax = std::sqrt(sq3(L - P));
            d2 = normalize(L - P);
        } else {           // incidence c: random tangent direction tilted to |d . n| = c, either side
            const double c = kind == 1 ? urand() : kind == 2 ? cmin * (1.0 + 3.0 * urand()) : kind == 3 ? cmin * (1.0 + 1e-3 * urand()) : cmin * 0.5;
            V3 tg = cross(n, v3(urand() - 0.5, urand() - 0.5, urand() - 0.5));
            if (sq3(tg) == 0.0) continue;
            tg = normalize(tg);
            const double sg = urand() < 0.5 ? -1.0 : 1.0;
            d2 = normalize(tg * std::sqrt(std::max(0.0, 1.0 - c * c)) + n * (sg * c));
        }
        const bool shadow = kind == 0;
        const int skip = std::fabs(dot(d2, n)) >= cmin ? x.pad[0] : -1;
        double t1, t2;
        long v = 0;
        const int p1 = traverse(hs, P, d2, shadow, tmax, t1, v, skip);
        const int p2 = brute(hs, P, d2, shadow, tmax, t2);
        ++total;
        skipped += skip >= 0;
        if (shadow ? ((p1 >= 0) != (p2 >= 0)) : (p1 != p2 || !(t1 == t2 || (std::isinf(t1) && std::isinf(t2))))) {
            if (++bad < 5) std::printf("plane skip mismatch: prim %d kind %d skip %d got %d want %d (t %.17g %.17g)\n", i, kind, skip, p1, p2, t1, t2);
        }
    }
    return bad;
}

int main(int argc, char** argv) {
    const int nrays = argc > 1 ? std::atoi(argv[1]) : 20000;
    long mism = 0, total = 0, visits = 0;
    const int first_scene = argc > 2 ? 4 : 0, last_scene = argc > 2 ? 5 : 4;
    for (int scene = first_scene; scene < last_scene; ++scene) {
        std::vector<gi_entity_desc> ents;
        if (scene == 4 && !read_scn(argv[2], ents)) return 2;
        const int ntri = scene == 0 ? 40 : scene == 1 ? 3000 : scene == 2 ? 20000 : scene == 3 ? 300 : 0;
        for (int i = 0; scene == 0 && i < 60; ++i) {   // tilted quads: two triangles in one plane each
            const V3 c = v3(urand() * 10, urand() * 10 - 5, urand() * 10 - 5);
            const V3 u = normalize(v3(urand() - 0.5, urand() - 0.5, urand() - 0.5));
            const V3 w = normalize(cross(u, v3(urand() - 0.5, urand() - 0.5, urand() - 0.5)));
            const double su = 0.3 + urand(), sw = 0.3 + urand();
            const V3 q[4] = {c - u * su - w * sw, c + u * su - w * sw, c + u * su + w * sw, c - u * su + w * sw};
            double v1[9] = {q[0].x, q[0].y, q[0].z, q[1].x, q[1].y, q[1].z, q[2].x, q[2].y, q[2].z};
            double v2[9] = {q[0].x, q[0].y, q[0].z, q[2].x, q[2].y, q[2].z, q[3].x, q[3].y, q[3].z};
            ents.push_back(tri(v1));
            ents.push_back(tri(v2));
        }
        for (int i = 0; i < ntri; ++i) {
            double c[3] = {urand() * 10, urand() * 10 - 5, urand() * 10 - 5}, v[9];
            const double sz = scene == 3 ? 6.0 : 0.6;   // scene 3: large overlapping triangles
            for (int k = 0; k < 9; ++k) v[k] = c[k % 3] + sz * (2 * urand() - 1);
            ents.push_back(tri(v));
        }
        for (int i = 0; i < (scene < 4 ? 6 : 0); ++i) {   // spheres
            gi_entity_desc e{};
            e.kind = GI_IMP_SPHERE;
            e.args[0] = urand() * 10; e.args[1] = urand() * 10 - 5; e.args[2] = urand() * 10 - 5; e.args[3] = 0.3 + urand();
            ents.push_back(e);
        }
        gi_scene_desc sd{};
        for (int k = 0; k < 3; ++k) { sd.octree_min[k] = -20; sd.octree_max[k] = 20; }
        sd.n_entities = (int32_t)ents.size();
        sd.entities = ents.data();
        HostScene hs;
        std::string err;
        if (!build_host_scene(sd, hs, err)) { std::printf("build failed: %s\n", err.c_str()); return 2; }
        const bool bvh = hs.xnodes.empty();
        // the spatial-split build puts a primitive in several leaves, each boxing a part of it
        if (check_structure(hs, bvh && !hs.x_spatial)) return 1;
        std::vector<XWNode> dec;
        if (check_quantised(hs, dec)) return 1;
        std::vector<XCNode> xc;
        const bool have_xc = encode_xcnodes(hs.xwnodes, xc);
        const std::vector<XWNode> orig = hs.xwnodes;
        const long visits0 = visits, prims0 = g_prim_tests;
        // the XWNode boxes; the decoded quantised boxes; the quantised nodes with the kernel's
        // fused slab arithmetic
        for (int pass = 0; pass < (have_xc ? 3 : 2); ++pass) {
        if (pass == 1) hs.xwnodes = dec;
        if (pass == 2) { hs.xwnodes = orig; g_xc = xc.data(); g_xw_base = hs.xwnodes.data(); }
        for (int r = 0; r < nrays; ++r) {
            V3 o, tgt;
            if (r % 2 == 0) o = v3(-10, 0, 0);
            else o = v3(urand() * 12 - 1, urand() * 12 - 6, urand() * 12 - 6);
            tgt = v3(urand() * 12 - 1, urand() * 12 - 6, urand() * 12 - 6);
            if (r % 7 == 0) tgt.y = o.y;   // axis-parallel components
            const V3 d = normalize(tgt - o);
            const bool shadow = (r % 3) == 0;
            const double tmax = shadow ? 3.0 + 10 * urand() : INFINITY;
            double t1, t2;
            const int a = traverse(hs, o, d, shadow, tmax, t1, visits);
            const int b = brute(hs, o, d, shadow, tmax, t2);
            ++total;
            if (shadow ? ((a >= 0) != (b >= 0)) : (a != b || !(t1 == t2 || (std::isinf(t1) && std::isinf(t2))))) ++mism;
        }
        }
        g_xc = nullptr;
        {
            long skipped = 0, tot = 0;
            const long pb = check_plane_skip(hs, 4 * nrays, skipped, tot);
            mism += pb;
            std::printf("scene %d plane skip: %ld rays, %ld skipping, bound %.3g + %.3g |cam|, mismatches %ld\n", scene, tot, skipped,
                        hs.x_skip_b, hs.x_skip_a, pb);
        }
        std::printf("scene %d: %zu prims, %zu wide nodes, %zu leaf records, depth %d; per ray: %.2f node visits, %.2f prim tests"
                    " (SAH estimate %.2f / %.2f)\n",
                    scene, hs.xprims.size(), hs.xwnodes.size(), hs.xhot.size(), hs.x_max_depth,
                    (double)(visits - visits0) / ((have_xc ? 3.0 : 2.0) * nrays),
                    (double)(g_prim_tests - prims0) / ((have_xc ? 3.0 : 2.0) * nrays), hs.x_est_nodes,
                    hs.x_est_prims);
    }
    std::printf("rays %ld mismatches %ld wide-node visits %ld\n", total, mism, visits);
    return mism == 0 ? 0 : 1;
}
