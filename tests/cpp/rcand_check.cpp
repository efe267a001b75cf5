// rcand_check.cpp — CPU check of Mode R's candidate reconstruction (gi_kernels.hip
// trace_mode_r_cand, host structures from gi_bvh.cpp build_rcand) against the reference-order walk
// (trace_mode_r: the reverse DFS over the reference octree, first success = the reference's last
// hitting candidate).  Both are restated here step for step on the host, over libgi's
// own scene builder, on seeded random rays through random mixed scenes (spheres, triangles, quads,
// rectangles, boxes) and, given .scn files, through those scenes; the hit entity and the fp64
// point/normal must agree bit for bit.
//   rcand_check <n_rays> [scene.scn ...]
#include <cfloat>
#include <cmath>
#include <functional>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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

static uint64_t g_rng = 0x2019abcdULL;
static double urand() {
    g_rng += 0x9E3779B97F4A7C15ULL;
    uint64_t z = g_rng;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    z ^= z >> 31;
    return (double)(z >> 11) * 0x1.0p-53;
}

// the kernel's ent_hit (entity intersect as the reference computes it)
static bool ent_hit(const HostScene& s, const REnt& e, V3 o, V3 d, V3& P, V3& N) {
    if (e.kind == K_IMP_SPHERE) return sphere_hit(ld3(e.pos), e.radius, o, d, P, N);
    if (e.kind == K_IMP_TRIANGLE) return tri_hit(s.tris[e.tri_first], o, d, P, N);
    if (e.kind == K_EXP_RECTANGLE) {
        if (tri_hit(s.tris[e.tri_first], o, d, P, N)) return true;
        return tri_hit(s.tris[e.tri_first + 1], o, d, P, N);
    }
    if (e.kind == K_EXP_BOX) {
        bool any = false;
        for (int f = 0; f < 6; ++f) {
            V3 p, n;
            bool h = tri_hit(s.tris[e.tri_first + 2 * f], o, d, p, n);
            if (!h) h = tri_hit(s.tris[e.tri_first + 2 * f + 1], o, d, p, n);
            if (h) {
                if (sq3(p - o) < DBL_MAX) { P = p; N = n; }
                any = true;
            }
        }
        return any;
    }
    bool flag = false;
    double md = DBL_MAX;
    V3 mi = v3(DBL_MAX, DBL_MAX, DBL_MAX), cn = v3(0, 0, 0);
    for (int t = 0; t < e.tri_count; ++t) {
        V3 p, n;
        if (tri_hit(s.tris[e.tri_first + t], o, d, p, n)) {
            const double dd = sq3(p - o);
            if (dd <= md) { mi = p; cn = n; md = dd; }
            flag = true;
        }
    }
    P = mi;
    N = cn;
    return flag;
}

struct Res {
    int ent = -1;
    V3 P = v3(0, 0, 0), N = v3(0, 0, 0);
};

// the kernel's trace_mode_r (reverse DFS, first success)
static Res reverse_dfs(const HostScene& s, V3 o, V3 d) {
    Res r;
    auto scan = [&](const RNode& nd) {
        for (int k = nd.ent_cnt - 1; k >= 0; --k) {
            const int e = s.leaf_ents[nd.ent_off + k];
            V3 P, N;
            if (ent_hit(s, s.ents[e], o, d, P, N) && sq3(P - o) < DBL_MAX) {
                r.ent = e; r.P = P; r.N = N;
                return true;
            }
        }
        return false;
    };
    const RNode& root = s.rnodes[0];
    if (root.child0 < 0) { scan(root); return r; }
    int parent = 0, pc0 = root.child0, slot = 7;
    for (;;) {
        if (slot < 0) {
            if (parent == 0) return r;
            const int pp = s.rnodes[parent].parent, ppc0 = s.rnodes[pp].child0;
            slot = parent - ppc0 - 1;
            parent = pp;
            pc0 = ppc0;
            continue;
        }
        const int c = pc0 + slot;
        const RNode& nd = s.rnodes[c];
        if (nd.ent_cnt == 0 || !box_hit(ld3(nd.mn), ld3(nd.mx), o, d)) { --slot; continue; }
        if (nd.child0 < 0) {
            if (scan(nd)) return r;
            --slot;
            continue;
        }
        parent = c;
        pc0 = nd.child0;
        slot = 7;
    }
}

// the kernel's trace_mode_r_cand (fp32 slab math restated with correctly rounded reciprocals)
static uint32_t mask_line(const XWNode& nd, const float of[3], const float iv[3], float tau) {
    uint32_t m = 0;
    for (int c = 0; c < 8; ++c) {
        if (!((nd.exists >> c) & 1)) continue;
        float tn = -INFINITY, tf = INFINITY;
        for (int k = 0; k < 3; ++k) {
            const float t0 = ((nd.lo[k][c] - tau) - of[k]) * iv[k], t1 = ((nd.hi[k][c] + tau) - of[k]) * iv[k];
            tn = std::fmax(tn, std::fmin(t0, t1));
            tf = std::fmin(tf, std::fmax(t0, t1));
        }
        if (tn <= tf) m |= 1u << c;
    }
    return m;
}
static bool reachable(const HostScene& s, int leaf, V3 o, V3 d) {
    for (int i = s.rpath_off[leaf]; i < s.rpath_off[leaf + 1]; ++i) {
        const RNode& nd = s.rnodes[s.rpath[i]];
        if (nd.ent_cnt == 0 || !box_hit(ld3(nd.mn), ld3(nd.mx), o, d)) return false;
    }
    return true;
}
static Res candidates(const HostScene& s, V3 o, V3 d, long& considered) {
    Res r;
    long long best = -1;
    auto consider = [&](int e) {
        ++considered;
        const int a0 = s.app_off[e], a1 = s.app_off[e + 1];
        if (a0 == a1 || s.app_rank[a0] <= best) return;
        V3 P, N;
        if (!ent_hit(s, s.ents[e], o, d, P, N) || !(sq3(P - o) < DBL_MAX)) return;
        for (int i = a0; i < a1 && s.app_rank[i] > best; ++i)
            if (reachable(s, s.app_leaf[i], o, d)) { best = s.app_rank[i]; r.ent = e; r.P = P; r.N = N; return; }
    };
    for (int e : s.r_always) consider(e);
    const double reach = std::fmax(std::fabs(o.x), std::fmax(std::fabs(o.y), std::fabs(o.z))) + s.rc_ext;
    const float tau = (float)(1e-5 * reach + 1e-30);
    const float of[3] = {(float)o.x, (float)o.y, (float)o.z};
    // the kernel's inv_dir: reciprocal clamped to +-1e30
    auto inv = [](float v) { return std::fmin(std::fmax(1.0f / v, -1e30f), 1e30f); };
    const float iv[3] = {inv((float)d.x), inv((float)d.y), inv((float)d.z)};
    // the kernels' walk: depth first in slot order, a level dropped once a popped slot's highest
    // rank (rc_maxkey; slots sorted by it) is <= the best rank found
    std::function<void(int)> visit = [&](int n) {
        const XWNode& nd = s.rc_nodes[n];
        const uint32_t m = mask_line(nd, of, iv, tau);
        for (int c = 0; c < 8; ++c) {
            if (!((m >> c) & 1)) continue;
            if (s.rc_maxkey[(size_t)n * 8 + c] <= best) return;
            if (nd.child[c] >= 0) visit(nd.child[c]);
            else for (int j = 0; j < nd.cnt[c]; ++j) consider(s.rc_ent[~nd.child[c] + j]);
        }
    };
    if (!s.rc_nodes.empty()) visit(0);
    return r;
}

static bool same(const Res& a, const Res& b) {
    if (a.ent != b.ent) return false;
    if (a.ent < 0) return true;
    const double x[6] = {a.P.x, a.P.y, a.P.z, a.N.x, a.N.y, a.N.z}, y[6] = {b.P.x, b.P.y, b.P.z, b.N.x, b.N.y, b.N.z};
    return std::memcmp(x, y, sizeof x) == 0;
}

static bool read_scn(const char* path, std::vector<gi_entity_desc>& ents, double box[6]) {
    std::ifstream f(path);
    std::string line;
    const char* kws[] = {"", "impsphere", "imptriangle", "expquad", "expsphere", "expcube", "expcone", "exprectangle", "expbox"};
    while (std::getline(f, line)) {
        std::istringstream is(line);
        std::string kw;
        is >> kw;
        std::vector<double> v;
        double x;
        while (is >> x) v.push_back(x);
        if (kw == "octree" && v.size() >= 6) { for (int k = 0; k < 6; ++k) box[k] = v[k]; continue; }
        for (int k = 1; k <= 8; ++k)
            if (kw == kws[k]) {
                gi_entity_desc e{};
                e.kind = k;
                for (size_t i = 0; i < v.size() && i < 11; ++i) e.args[i] = v[i];
                ents.push_back(e);
            }
    }
    return !ents.empty();
}

static int run(const std::vector<gi_entity_desc>& ents, const double box[6], int nrays, const char* name, long& mism) {
    gi_scene_desc sd{};
    for (int k = 0; k < 3; ++k) { sd.octree_min[k] = box[k]; sd.octree_max[k] = box[3 + k]; }
    sd.n_entities = (int32_t)ents.size();
    sd.entities = ents.data();
    HostScene hs;
    std::string err;
    if (!build_host_scene(sd, hs, err)) { std::printf("build failed: %s\n", err.c_str()); return 2; }
    long hits = 0, considered = 0, bad = 0;
    // the device's records restate rpath / rnodes and app_rank / app_leaf exactly
    if (hs.rpath_rec.size() != hs.rpath.size() || hs.app_rec.size() != hs.app_rank.size()) ++bad;
    for (size_t i = 0; i < hs.rpath_rec.size() && i < hs.rpath.size(); ++i) {
        const RNode& nd = hs.rnodes[(size_t)hs.rpath[i]];
        const RPathRec& q = hs.rpath_rec[i];
        bool ok = q.node == hs.rpath[i] && q.ent_cnt == nd.ent_cnt;
        for (int k = 0; k < 3; ++k) ok = ok && q.mn[k] == nd.mn[k] && q.mx[k] == nd.mx[k];
        if (!ok) { ++bad; if (bad < 5) std::printf("  path record %zu differs\n", i); }
    }
    for (size_t a = 0; a < hs.app_rec.size() && a < hs.app_rank.size(); ++a) {
        const int lf = hs.app_leaf[a];
        if (hs.app_rec[a].rank != hs.app_rank[a] || hs.app_rec[a].p0 != hs.rpath_off[(size_t)lf] ||
            hs.app_rec[a].p1 != hs.rpath_off[(size_t)lf + 1]) { ++bad; if (bad < 5) std::printf("  appearance record %zu differs\n", a); }
    }
    for (int r = 0; r < nrays; ++r) {
        V3 o = (r % 2 == 0) ? v3(-10, 0, 0) : v3(urand() * 24 - 12, urand() * 24 - 12, urand() * 24 - 12);
        V3 tgt = v3(urand() * 16 - 4, urand() * 14 - 7, urand() * 14 - 7);
        if (r % 9 == 0) tgt.y = o.y;   // axis-parallel components
        if (r % 13 == 0) tgt.z = o.z;
        const V3 d = normalize(tgt - o);
        const Res a = reverse_dfs(hs, o, d), b = candidates(hs, o, d, considered);
        hits += a.ent >= 0;
        if (!same(a, b)) { ++bad; if (bad < 5) std::printf("  mismatch ray %d: dfs %d cand %d\n", r, a.ent, b.ent); }
    }
    std::printf("%s: %zu entities, %zu leaf appearances, %zu line-BVH nodes, %zu always; %d rays, %ld hits, "
                "%.2f entities considered per ray, %ld mismatches\n",
                name, ents.size(), hs.app_rank.size(), hs.rc_nodes.size(), hs.r_always.size(), nrays, hits,
                (double)considered / nrays, bad);
    mism += bad;
    return 0;
}

int main(int argc, char** argv) {
    const int nrays = argc > 1 ? std::atoi(argv[1]) : 20000;
    long mism = 0;
    const double box[6] = {-20, -20, -20, 20, 20, 20};
    for (int scene = 0; scene < 3; ++scene) {   // random mixed scenes
        std::vector<gi_entity_desc> ents;
        const int ntri = scene == 0 ? 30 : scene == 1 ? 400 : 3000;
        for (int i = 0; i < ntri; ++i) {
            gi_entity_desc e{};
            e.kind = GI_IMP_TRIANGLE;
            const double c[3] = {urand() * 10, urand() * 10 - 5, urand() * 10 - 5};
            const double sz = scene == 2 ? 0.3 : 2.0;
            for (int k = 0; k < 9; ++k) e.args[k] = c[k % 3] + sz * (2 * urand() - 1);
            ents.push_back(e);
        }
        for (int i = 0; i < 4; ++i) {
            gi_entity_desc e{};
            e.kind = GI_IMP_SPHERE;
            e.args[0] = urand() * 10; e.args[1] = urand() * 10 - 5; e.args[2] = urand() * 10 - 5; e.args[3] = 0.5 + urand();
            e.args[4] = 1; e.args[5] = 0; e.args[6] = 1;
            ents.push_back(e);
        }
        {
            gi_entity_desc e{};
            e.kind = GI_EXP_QUAD;
            const double q[9] = {1.0, 0.5, -0.5, 3, 2, 0.7, 1, 1, 0};
            for (int k = 0; k < 9; ++k) e.args[k] = q[k];
            ents.push_back(e);
            gi_entity_desc b{};
            b.kind = GI_EXP_BOX;
            const double bx[6] = {2.0, 4.0, -5.0, 4.0, 6.0, -3.0};
            for (int k = 0; k < 6; ++k) b.args[k] = bx[k];
            ents.push_back(b);
            gi_entity_desc rc{};
            rc.kind = GI_EXP_RECTANGLE;
            const double rr[9] = {1.0, -6.0, -3.0, 1.0, -3.0, 0.0, 1.0, -6.0, 0.0};
            for (int k = 0; k < 9; ++k) rc.args[k] = rr[k];
            ents.push_back(rc);
        }
        char name[32];
        std::snprintf(name, sizeof name, "random%d", scene);
        if (run(ents, box, nrays, name, mism)) return 2;
    }
    for (int i = 2; i < argc; ++i) {
        std::vector<gi_entity_desc> ents;
        double b[6] = {-20, -20, -20, 20, 20, 20};
        if (!read_scn(argv[i], ents, b)) return 2;
        if (run(ents, b, nrays, argv[i], mism)) return 2;
    }
    std::printf("mismatches %ld\n", mism);
    return mism == 0 ? 0 : 1;
}
