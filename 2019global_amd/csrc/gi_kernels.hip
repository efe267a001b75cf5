// gi_kernels.hip — gfx950 (CDNA4) kernels for the per-pixel radiance path.
//
// Work decomposition: 8x8 pixel tiles dealt round-robin over shard ranks (tile t belongs to rank
// t % shard_count), so the same kernels serve 1 GPU and N-GPU tile sharding; four waves per
// 256-thread workgroup.  Mode R: one wave64 per tile (lane = pixel).  Mode X: persistent waves
// taking (pixel, run of samples) units from a device work list.
//
// Mode R (reference semantics):
//   The reference builds the full candidate list of Octree::intersect (octree.h:132-155, DFS over
//   children 0..7, ExpBox node test) and keeps the LAST candidate whose intersect() succeeds
//   (raytracer.h:53-74, A.1).  The kernel reconstructs that answer from the entities the ray's line
//   passes near (a line BVH), their exact tests and the reachability of their leaves (the same
//   node tests on those leaves' root paths only): trace_mode_r_cand.  The reference-order walk --
//   the last hit in DFS order is the first hit in reverse DFS order, children 7..0, leaf lists
//   backwards, first success -- stays available (trace_mode_r, GI_FLAG_R_DFS); both give the same
//   frame bit for bit.  Same primitive math (gi_math.h) as the reference.
// Mode X (build-defined): classify pass (background pixels) -> persistent path-tracing
//   kernel over (pixel, run of samples) work units, closest-hit + shadow any-hit through the 8-wide
//   BVH (front-to-back child slots by ray-direction octant) -> in-order per-sample reduce.
//
// Build: hipcc --offload-arch=gfx950 -O3 -ffp-contract=off (bit-level parity needs no FMA
// contraction; f64 div/sqrt are correctly rounded on gfx950).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <cstdlib>
#include <mutex>

#include "gi.h"
#include "gi_dev.h"
#include "gi_scene.h"

namespace gi {

namespace {

// ---------------------------------------------------------------------------------------------
// Mode R device pieces
// ---------------------------------------------------------------------------------------------
// TRI: every entity of the scene is an ImpTriangle (DevScene::r_tri_only; the other kinds' code and
// registers drop out of the Mode R kernels)
template <bool TRI = false>
__device__ bool ent_hit(const DevScene& sc, const REnt& e, V3 o, V3 d, V3& P, V3& N, uint32_t& nprim) {
    if (TRI) {
        ++nprim;
        return tri_hit(sc.tris[e.tri_first], o, d, P, N);
    }
    if (e.kind == K_IMP_SPHERE) {
        ++nprim;
        return sphere_hit(ld3(e.pos), e.radius, o, d, P, N);
    }
    if (e.kind == K_IMP_TRIANGLE) {
        ++nprim;
        return tri_hit(sc.tris[e.tri_first], o, d, P, N);
    }
    if (e.kind == K_EXP_RECTANGLE) {   // entities.h:326-336: t1, else t2
        nprim += 1;
        if (tri_hit(sc.tris[e.tri_first], o, d, P, N)) return true;
        nprim += 1;
        return tri_hit(sc.tris[e.tri_first + 1], o, d, P, N);
    }
    if (e.kind == K_EXP_BOX) {   // entities.h:415-440: every face; the LAST hitting face's point wins
        bool any = false;
        for (int f = 0; f < 6; ++f) {
            V3 p, n;
            ++nprim;
            bool h = tri_hit(sc.tris[e.tri_first + 2 * f], o, d, p, n);
            if (!h) {
                ++nprim;
                h = tri_hit(sc.tris[e.tri_first + 2 * f + 1], o, d, p, n);
            }
            if (h) {
                if (sq3(p - o) < DBL_MAX) { P = p; N = n; }
                any = true;
            }
        }
        return any;
    }
    // ExpQuad / ExpSphere / ExpCube / ExpCone ::intersect (entities.h:596-620, 514-536, 736-760,
    // 906-930): nearest by <= over the triangles (ties -> later); outputs overwritten on a miss
    bool flag = false;
    double md = DBL_MAX;
    V3 mi = v3(DBL_MAX, DBL_MAX, DBL_MAX), cn = v3(0, 0, 0);
    for (int t = 0; t < e.tri_count; ++t) {
        V3 p, n;
        ++nprim;
        if (tri_hit(sc.tris[e.tri_first + t], o, d, p, n)) {
            const double dd = sq3(p - o);
            if (dd <= md) { mi = p; cn = n; md = dd; }
            flag = true;
        }
    }
    P = mi;
    N = cn;
    return flag;
}

// getTextureCoord (entities.h:108-130, 277-303, 630-641) with the device's f64 acos/sin/cos
template <bool TRI = false>
__device__ void tex_coord(const DevScene& sc, const REnt& e, V3 ip, int32_t& x, int32_t& y) {
    if (!TRI && e.kind == K_IMP_SPHERE) {
        const double r = e.radius;
        const double unit_v = 2.0 * REF_PI * r / 320.0;
        const V3 to = ip - ld3(e.pos);
        const double cos_vert = dot(to, v3(0, 0, r)) / (r * r);
        const double ang = acos(cos_vert);
        y = x86_trunc((r * ang) / unit_v);
        const double small_r = r * sin(ang);
        const double cos_hori = dot(v3(to.x, to.y, 0), v3(0, small_r, 0)) / (small_r * small_r);
        const double unit_h = 2.0 * REF_PI * small_r / 320.0;
        x = x86_trunc(small_r * acos(cos_hori) / unit_h);
    } else if (TRI || e.kind == K_IMP_TRIANGLE) {   // per-triangle constants precomputed by the builder
        const V3 p1 = ld3(e.qv0), p21 = ld3(e.qv1), i1 = ip - p1;
        const double i1l = gsqrt(sq3(i1));
        const double theta = acos(dot(p21, i1) / (e.qv2[0] * i1l));
        const double ixl = i1l * sin(theta);
        y = x86_trunc(i1l / e.qv2[2]);
        x = x86_trunc(ixl / e.qv2[1]);
    } else if (e.kind == K_EXP_QUAD) {
        const double uv = (double)e.width / 160.0, uh = (double)e.length / 160.0;
        const V3 rv = ld3(e.qv0) - ld3(e.qv1);
        const V3 i1 = ip - ld3(e.qv1);
        const double i1l = gsqrt(sq3(i1));
        const double theta = acos(dot(i1, rv) / ((double)e.width * i1l));
        y = x86_trunc(i1l * sin(theta) / uh);
        x = x86_trunc(i1l * cos(theta) / uv);
    } else if (e.kind == K_EXP_SPHERE) {   // entities.h:549-571 (latitude measured from the equator)
        const double r = e.radius;
        const double unit_v = 2.0 * REF_PI * r / 320.0;
        const V3 to = ip - ld3(e.pos);
        const double ang = acos(dot(to, v3(0, 0, r)) / (r * r));
        y = x86_trunc((0.5 * REF_PI * r - r * ang) / unit_v);
        const double small_r = r * sin(ang);
        const double cos_hori = dot(v3(to.x, to.y, 0), v3(0, small_r, 0)) / (small_r * small_r);
        const double unit_h = 2.0 * REF_PI * small_r / 320.0;
        x = x86_trunc(small_r * acos(cos_hori) / unit_h);
    } else if (e.kind == K_EXP_CUBE) {     // entities.h:769-811
        const double uv = (double)e.width / 160.0, uh = (double)e.length / 160.0;
        const V3 i1 = ip - ld3(e.qv0);
        const double l = gsqrt(sq3(i1));
        const double theta = acos(dot(i1, v3(0, (double)e.width, 0)) / ((double)e.width * l));
        y = x86_trunc(l * sin(theta) / uh);
        x = x86_trunc(l * cos(theta) / uv);
    } else if (e.kind == K_EXP_CONE) {     // entities.h:942-961
        const double R = e.radius, H = e.height;
        const double unit_h = gsqrt(R * R + H * H) / 320.0;
        const V3 pos = ld3(e.pos);
        const double ylen = gsqrt(sq3(ip - pos));
        y = x86_trunc(ylen / unit_h);
        const V3 center = v3((float)pos.x, (float)pos.y, (float)ip.z);   // glm::vec3
        const double rp = ylen * e.sin_theta;
        const V3 left = v3(0, (float)rp, 0);                              // glm::vec3
        const V3 ic = ip - center;
        const double unit_v = 2.0 * REF_PI * rp / 320.0;
        double alpha = acos(dot(ic, left) / (rp * rp));
        if (alpha > REF_PI / 4.0) alpha = acos(dot(ic, -left) / (rp * rp));
        x = x86_trunc(rp * alpha / unit_v);
    } else if (e.kind == K_EXP_RECTANGLE) {   // entities.h:346-365 (acos of an angle, as written)
        const V3 p1 = ld3(e.qv0), p31 = ld3(e.qv1) - p1, p41 = ld3(e.qv2) - p1;
        const double width = gsqrt(sq3(p41)), length = gsqrt(sq3(p31));
        const V3 i1 = ip - p1;
        const double l = gsqrt(sq3(i1));
        const double ct = acos(dot(i1, p31) / (length * l));
        x = x86_trunc(l * sin(acos(ct)) / (length / 64.0));
        y = x86_trunc(l * ct / (width / 64.0));
    } else {   // ExpBox: (0, 0) (entities.h:448-451)
        x = 0;
        y = 0;
    }
}

// Material::blinn_phong_texture (material.h:48-62)
__device__ V3 shade_ref(const REnt& e, V3 dir, V3 light, V3 ip, V3 n, int32_t u, int32_t v) {
    const V3 tc = texel(ld3(e.color), u, v);
    const V3 tdc = tc * 0.5;
    const V3 la = tc * e.shader[0];
    const V3 ld = (smax(0.0, dot(n, normalize(light - ip))) * tdc) * e.shader[1];
    const V3 bis = normalize(normalize(-dir) + normalize(light - ip));
    const double p = pow(smax(0.0, dot(n, bis)), e.spec_pow);
    const V3 ls = (p * v3(1, 1, 1)) * e.shader[2];
    const V3 out = (la + ld) + ls;
    return v3(smin(out.x, 1.0), smin(out.y, 1.0), smin(out.z, 1.0));
}

struct RResult {
    int32_t ent;
    V3 P, N;
};

// scan one leaf list backwards; true when the last hitting candidate of this leaf is found
__device__ bool scan_leaf_rev(const DevScene& sc, const RNode& nd, V3 o, V3 d, RResult& r, uint32_t& nprim) {
    for (int k = nd.ent_cnt - 1; k >= 0; --k) {
        const int32_t e = sc.leaf_ents[nd.ent_off + k];
        V3 P, N;
        if (ent_hit(sc, sc.ents[e], o, d, P, N, nprim)) {
            if (sq3(P - o) < DBL_MAX) {   // raytracer.h:63-65 with min_dist_square == DBL_MAX
                r.ent = e;
                r.P = P;
                r.N = N;
                return true;
            }
        }
    }
    return false;
}

// Last hitting candidate of Octree::intersect's list = first hit of the reverse DFS.
__device__ void trace_mode_r(const DevScene& sc, V3 o, V3 d, RResult& r, uint32_t& nnode, uint32_t& nprim) {
    r.ent = -1;
    const RNode* nodes = sc.rnodes;
    const RNode root = nodes[0];
    if (root.child0 < 0) {
        scan_leaf_rev(sc, root, o, d, r, nprim);
        return;
    }
    int parent = 0, parent_child0 = root.child0, slot = 7;
    for (;;) {
        if (slot < 0) {
            if (parent == 0) return;
            const int pp = nodes[parent].parent;
            const int pc0 = nodes[pp].child0;
            slot = parent - pc0 - 1;
            parent = pp;
            parent_child0 = pc0;
            continue;
        }
        const int c = parent_child0 + slot;
        const RNode nd = nodes[c];
        if (nd.ent_cnt == 0) { --slot; continue; }   // octree.h:140
        ++nnode;
        if (!box_hit(ld3(nd.mn), ld3(nd.mx), o, d)) { --slot; continue; }
        if (nd.child0 < 0) {
            if (scan_leaf_rev(sc, nd, o, d, r, nprim)) return;
            --slot;
            continue;
        }
        parent = c;
        parent_child0 = nd.child0;
        slot = 7;
    }
}

// ---------------------------------------------------------------------------------------------
// Mode R, candidate reconstruction (gi_bvh.cpp build_rcand).  The reference keeps the LAST hitting
// candidate of Octree::intersect's list; a candidate's list position is (its leaf's rank in the
// static DFS order, its index in the leaf's list), and a leaf is in the list iff every node of its
// root path is non-empty and passes the exact ExpBox node test.  So: collect the entities whose
// boxes the ray's LINE crosses (no t > 0 in the reference's tests, A.2/A.3) from a line BVH, test
// each exactly (ent_hit), and keep the hitting entity whose latest reachable appearance is latest
// (reachability = the same node tests, on that leaf's path only).  Same answer as the reference's
// full DFS, with node tests only on the paths of hitting entities.
// ---------------------------------------------------------------------------------------------
// the 8 children of a line-BVH node against the whole line o + t d (t real), boxes widened by tau
__device__ __forceinline__ uint32_t children_mask_line(const XWNode* nd, F3 of, F3 ivf, float tau) {
    const float4* b = reinterpret_cast<const float4*>(nd);
    // near / far planes by the sign of the (clamped) reciprocal, as in the Mode X node tests: the
    // distance ((b -+ tau) - o) * iv is monotone in b, so no per-child min / max; the planes' quads
    // are addressed directly (lo of axis a at quad 2a, hi at 6 + 2a)
    const int sm = iv_signs(ivf);
    const int ex = nd->exists;
    float4 q[12];   // near[3][8] then far[3][8]
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int nq = ((sm >> a) & 1) ? 6 + 2 * a : 2 * a, fq = ((sm >> a) & 1) ? 2 * a : 6 + 2 * a;
        q[2 * a] = b[nq];
        q[2 * a + 1] = b[nq + 1];
        q[6 + 2 * a] = b[fq];
        q[6 + 2 * a + 1] = b[fq + 1];
    }
    const float* v = reinterpret_cast<const float*>(q);
    const float sx = (sm & 1) ? tau : -tau, sy = (sm & 2) ? tau : -tau, sz = (sm & 4) ? tau : -tau;
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float tn = fmaxf(fmaxf(((v[c] + sx) - of.x) * ivf.x, ((v[8 + c] + sy) - of.y) * ivf.y),
                               ((v[16 + c] + sz) - of.z) * ivf.z);
        const float tf = fminf(fminf(((v[24 + c] - sx) - of.x) * ivf.x, ((v[32 + c] - sy) - of.y) * ivf.y),
                               ((v[40 + c] - sz) - of.z) * ivf.z);
        m |= (uint32_t)((tn <= tf) & ((ex >> c) & 1)) << c;
    }
    return m;
}

// The same 8 tests spread over the NSUB (>= 8) lanes of a pixel group that walk one line
// (k_mode_r_batch's top two levels): lane sub tests child sub & 7 only -- its six bounds are one float
// each, and the group's 8 lanes read 8 consecutive floats of each plane array -- and a ballot gathers
// the mask, the same in every lane.  Per child the arithmetic is children_mask_line's, so the mask is
// identical.
template <int NSUB>
__device__ __forceinline__ uint32_t children_mask_line_coop(const XWNode* nd, F3 of, F3 ivf, float tau, int sub) {
    const int c = sub & 7;
    const int sm = iv_signs(ivf);
    const float nx = (sm & 1) ? nd->hi[0][c] : nd->lo[0][c], fx = (sm & 1) ? nd->lo[0][c] : nd->hi[0][c];
    const float ny = (sm & 2) ? nd->hi[1][c] : nd->lo[1][c], fy = (sm & 2) ? nd->lo[1][c] : nd->hi[1][c];
    const float nz = (sm & 4) ? nd->hi[2][c] : nd->lo[2][c], fz = (sm & 4) ? nd->lo[2][c] : nd->hi[2][c];
    const float sx = (sm & 1) ? tau : -tau, sy = (sm & 2) ? tau : -tau, sz = (sm & 4) ? tau : -tau;
    const float tn = fmaxf(fmaxf(((nx + sx) - of.x) * ivf.x, ((ny + sy) - of.y) * ivf.y), ((nz + sz) - of.z) * ivf.z);
    const float tf = fminf(fminf(((fx - sx) - of.x) * ivf.x, ((fy - sy) - of.y) * ivf.y), ((fz - sz) - of.z) * ivf.z);
    const bool hit = (tn <= tf) & ((nd->exists >> c) & 1);
    const unsigned long long b = __ballot(hit);
    const int base = (int)(threadIdx.x & 63) & ~(NSUB - 1);
    return (uint32_t)((b >> base) & 0xFFull);
}

// Per-ray memo of node-test results (k_mode_r_batch, k_rf_reach): the candidates' root paths share their upper
// levels -- every path starts at the root -- and an exact ExpBox node test is ~12 fp32/fp64 triangle
// solves, so a ray that walks many appearances' paths would repeat the same tests.  Direct-mapped,
// RMEMO entries per ray in LDS, shared by the NSUB lanes of the pixel (one ray, so a result found
// by any of them holds for all); an entry is (node << 1) | passed, -1 when empty.  A lost or stale
// slot only costs a recomputation: the answer never depends on the memo.
#ifndef GI_R_MEMO
#define GI_R_MEMO 64   // entries per ray (power of two); 0 disables the memo
#endif
struct RMemo {
    int* e;        // GI_R_MEMO entries of this ray, or nullptr
    int tag = 0;   // k_rf_reach: (the lane's run of equal tiles in its chunk) << 1 -- a row serves the same
                   // pixel slot of the chunk's tiles, and the memo is cleared at every chunk
};
__device__ __forceinline__ int r_memo_slot(int node) { return (int)(((unsigned)node * 2654435761u) >> 26) & (GI_R_MEMO - 1); }

// is the leaf whose root path is rpath_rec[p0 .. p1) in the ray's candidate list?  (octree.h:139-150
// on that path, top-down: every node non-empty and hit by the exact ExpBox test.)  The path's node
// records are consecutive, so the next one is loaded before the current one's test -- the walk waits
// on one load round trip per path, not two per node (rpath[i], then rnodes[rpath[i]]).
struct RPathR {
    union {
        int4 q[4];
        RPathRec r;
    };
};
__device__ __forceinline__ RPathR load_rpath(const RPathRec* p) {
    const int4* s = reinterpret_cast<const int4*>(p);
    RPathR r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r.q[i] = s[i];
    return r;
}
// G > 1 (k_rf_reach's lane groups): G consecutive lanes hold the same ray and walk the same path in
// step; each tests its part of the 12 ExpBox faces (box_hit_part) and a ballot ORs the group's parts,
// so every decision below is the group's and its lanes never diverge.  Needs the group's lanes active.
template <int G>
__device__ __forceinline__ bool r_box_test(V3 mn, V3 mx, V3 o, V3 d) {
    if constexpr (G == 1) {
        return box_hit(mn, mx, o, d);
    } else {
        static_assert(G == 4, "box_hit_part splits the faces over 4 lanes");
        const int lane = (int)(threadIdx.x & 63);
        const unsigned long long b = __ballot(box_hit_part(mn, mx, o, d, lane & 3));
        return ((b >> (lane & ~3)) & 0xFull) != 0;
    }
}
template <int G = 1>
__device__ __forceinline__ bool r_path_reachable(const DevScene& sc, int p0, int p1, V3 o, V3 d, uint32_t& nnode,
                                                 RMemo memo = RMemo{nullptr}) {
    if (p0 >= p1) return true;
    RPathR cur = load_rpath(sc.rpath_rec + p0);
    for (int i = p0; i < p1; ++i) {
        const RPathR nd = cur;
        if (i + 1 < p1) cur = load_rpath(sc.rpath_rec + i + 1);
        if (nd.r.ent_cnt == 0) return false;   // octree.h:140
        const int ni = nd.r.node;
        if (GI_R_MEMO > 0 && memo.e) {
            int* slot = memo.e + r_memo_slot(ni);
            const int m = *slot;   // (a group's lanes read it in one instruction: the same value)
            const int key = (ni << 9) | memo.tag;   // (the scenes using a memo have < 2^22 nodes)
            if ((m & ~1) == key) {
                if (!(m & 1)) return false;
                continue;
            }
            ++nnode;
            const bool ok = r_box_test<G>(ld3(nd.r.mn), ld3(nd.r.mx), o, d);
            *slot = key | (ok ? 1 : 0);
            if (!ok) return false;
            continue;
        }
        ++nnode;
        if (!r_box_test<G>(ld3(nd.r.mn), ld3(nd.r.mx), o, d)) return false;
    }
    return true;
}

// entity e as a candidate: exact test, then its latest reachable appearance against the best so far
template <bool TRI = false>
__device__ __forceinline__ void r_consider(const DevScene& sc, int e, V3 o, V3 d, long long& best, RResult& r,
                                           uint32_t& nnode, uint32_t& nprim, RMemo memo = RMemo{nullptr}) {
    const int a0 = sc.app_off[e], a1 = sc.app_off[e + 1];
    if (a0 == a1 || sc.app_rec[a0].rank <= best) return;
    V3 P, N;
    if (!ent_hit<TRI>(sc, sc.ents[e], o, d, P, N, nprim) || !(sq3(P - o) < DBL_MAX)) return;   // raytracer.h:58-65
    for (int i = a0; i < a1; ++i) {
        const RApp ap = sc.app_rec[i];
        const long long rk = ap.rank;
        if (rk <= best) return;
        if (r_path_reachable(sc, ap.p0, ap.p1, o, d, nnode, memo)) {
            best = rk;
            r.ent = e;
            r.P = P;
            r.N = N;
            return;
        }
    }
}

__device__ __forceinline__ void trace_mode_r_cand(const DevScene& sc, V3 o, V3 d, float tau, RResult& r, uint32_t& nnode,
                                  uint32_t& nprim) {
    r.ent = -1;
    long long best = -1;
    for (int i = 0; i < sc.n_r_always; ++i) r_consider(sc, sc.r_always[i], o, d, best, r, nnode, nprim);
    const XWNode* W = sc.rc_nodes;
    const F3 of = f3((float)o.x, (float)o.y, (float)o.z);
    const F3 ivf = inv_dir(d);   // clamped to +-1e30: finite plane distances, near / far by sign
    uint64_t mlo = 0, mhi = 0;
    int node = 0, level = 0;
    const uint32_t rm = children_mask_line(W, of, ivf, tau);
    lvl_set(mlo, mhi, 0, rm);
    bool going = rm != 0;
    while (going) {   // stackless: 8-bit "children left" mask per level, parent pointers
        const uint32_t msk = lvl_get(mlo, mhi, level);
        const int c = __builtin_ctz(msk);
        lvl_set(mlo, mhi, level, msk & (msk - 1));
        const XWNode* nd = W + node;
        const int ch = nd->child[c];
        if (sc.rc_maxkey[node * 8 + c] <= best) {   // rank order: no better candidate here or after
            lvl_set(mlo, mhi, level, 0);
        } else if (ch < 0) {
            const int cnt = nd->cnt[c];
            for (int j = 0; j < cnt; ++j) r_consider(sc, sc.rc_ent[~ch + j], o, d, best, r, nnode, nprim);
        } else {
            const uint32_t cm = children_mask_line(W + ch, of, ivf, tau);
            if (cm) {
                node = ch;
                ++level;
                lvl_set(mlo, mhi, level, cm);
            }
        }
        uint32_t rest = lvl_get(mlo, mhi, level);
        while (rest == 0 && level > 0) {
            --level;
            node = level == 0 ? 0 : W[node].parent;
            rest = lvl_get(mlo, mhi, level);
        }
        going = rest != 0;
    }
}

// Mode R for large scenes (more than 4096 entities).  A one-lane-per-pixel walk (k_mode_r) spends
// the 100k soup's frame on a few pixels' serial work -- their lines cross ~100 entity boxes -- so
// these scenes run the flat phases below (k_rf_*), chip-wide and dense, and k_mode_r_batch renders
// the tiles whose candidates do not fit the flat phases' buffers.  Both answer as trace_mode_r_cand:
// the hitting candidate of highest reachable list rank (A.1), bit for bit.

// maximum over the NSUB lanes of a pixel group
template <int NSUB>
__device__ __forceinline__ long long group_max(long long v) {
#pragma unroll
    for (int off = 1; off < NSUB; off <<= 1) {
        const long long u = __shfl_xor(v, off);
        v = u > v ? u : v;
    }
    return v;
}

// the pixel from a group's candidates: the lowest sub-lane holding the group's highest rank (ranks are
// unique: one lane at most) shades it; none: black
template <int NSUB, bool TRI>
__device__ __forceinline__ void r_group_write(const DevScene& sc, V3 d, V3 light, const RResult& r, long long mine,
                                              int sub, long long idx, double* rgb, uint8_t* rgb8) {
    const long long gmax = group_max<NSUB>(mine);
    const unsigned long long m_win = __ballot(mine == gmax);
    const int base = (int)(threadIdx.x & 63) & ~(NSUB - 1);
    const unsigned long long gm = NSUB >= 64 ? ~0ull : ((1ull << (NSUB & 63)) - 1);
    const bool writer = gmax < 0 ? sub == 0 : (int)(threadIdx.x & 63) == base + __builtin_ctzll((m_win >> base) & gm);
    if (writer) {
        double c0 = 0, c1 = 0, c2 = 0;
        if (gmax >= 0) {
            const REnt& e = sc.ents[r.ent];
            int32_t u, v;
            tex_coord<TRI>(sc, e, r.P, u, v);
            const V3 col = shade_ref(e, d, light, r.P, r.N, u, v);
            c0 = col.x; c1 = col.y; c2 = col.z;
        }
        if (rgb) { rgb[3 * idx] = c0; rgb[3 * idx + 1] = c1; rgb[3 * idx + 2] = c2; }
        if (rgb8) quantize(c0, c1, c2, rgb8 + 3 * idx);
    }
}

// a candidate considered by one lane of the group: on a better reachable hit, the group's best rank
// (LDS, atomic max) is raised
template <bool TRI>
__device__ __forceinline__ void r_group_consider(const DevScene& sc, int e, V3 o, V3 d, unsigned long long* gb, long long& best,
                                                 long long& mine, RResult& r, uint32_t& nnode, uint32_t& nprim, RMemo memo) {
    const long long before = best;
    r_consider<TRI>(sc, e, o, d, best, r, nnode, nprim, memo);
    if (best != before) {
        mine = best;
        atomicMax(gb, (unsigned long long)(best + 1));
    }
}
// the items of a pixel's walk: the root's hit slots, an interior one replaced by its own hit slots
// (cooperative node tests), in rank order -- (node << 3) | slot, at most 64; written by sub-lane 0
template <int NSUB>
__device__ __forceinline__ int r_items(const XWNode* W, F3 of, F3 ivf, float tau, int sub, int* items) {
    int n = 0;
    uint32_t rm = children_mask_line_coop<NSUB>(W, of, ivf, tau, sub);
    while (rm) {
        const int c = __builtin_ctz(rm);
        rm &= rm - 1;
        const int ch = W[0].child[c];
        if (ch < 0) {
            if (sub == 0) items[n] = c;
            ++n;
        } else {
            uint32_t cm = children_mask_line_coop<NSUB>(W + ch, of, ivf, tau, sub);
            while (cm) {
                const int c2 = __builtin_ctz(cm);
                cm &= cm - 1;
                if (sub == 0) items[n] = (ch << 3) | c2;
                ++n;
            }
        }
    }
    __builtin_amdgcn_wave_barrier();
    return n;
}

// Mode R in rounds, 8 lanes per pixel (k_mode_r_batch; the flat phases' fallback).  The group walks
// the line BVH's top two levels together into <= 64 items in rank order; every lane then alternates a
// walk phase of at most GI_R_BATCH_STEPS node steps over the items it takes from the group's LDS
// counter, which only queues the entities of the leaves it meets (those whose highest rank beats the
// group's best) in the lane's LDS segment, and a test phase in which the pixel's 8 lanes share the
// group's queued candidates (compacted, candidate j by lane j mod 8) -- the exact tests of a wave's 8
// pixels in one dense block.  Pruning only skips slots whose bound is <= a rank found, and every
// candidate is considered by one lane, so the answer is the highest reachable hitting rank.
// Work items are 32 pixel slots (one per 8-lane group of the workgroup): the whole frame
// (tiles == nullptr) or both halves of each of the *n_tiles listed tiles.
#ifndef GI_R_BATCH_STEPS
#define GI_R_BATCH_STEPS 16   // node steps a lane's walk takes per round (R-C4: 2 4.04, 4 3.56, 8 3.41,
                             // 16 3.19, 32 3.33 ms)
#endif
#ifndef GI_R_BATCH_SEG
#define GI_R_BATCH_SEG 8     // candidates a lane queues per round (4 and 16: equal or slower)
#endif
template <bool STATS, bool TRI>
__global__ __launch_bounds__(256) void k_mode_r_batch(DevScene sc, CamDev cam, V3 light, TileMap m, double* rgb,
                                                      uint8_t* rgb8, unsigned long long* stats, float tau,
                                                      const unsigned* tiles, const unsigned* n_tiles) {
    constexpr int NSUB = 8, SEG = GI_R_BATCH_SEG;   // lanes per pixel; queued candidates per lane and round
    const int sub = (int)(threadIdx.x % NSUB), grp = threadIdx.x / NSUB;
    __shared__ int s_memo[GI_R_MEMO > 0 ? (256 / NSUB) * GI_R_MEMO : 1];
    __shared__ unsigned long long s_best[256 / NSUB];   // the group's best rank + 1 (0: none)
    __shared__ int s_item[256 / NSUB][64];              // (node << 3) | slot, in rank order
    __shared__ unsigned s_next[256 / NSUB];             // the group's next item
    __shared__ int s_seg[256 / NSUB][NSUB * SEG];       // each lane's queued candidates (SEG slots)
    __shared__ int s_cand[256 / NSUB][NSUB * SEG];      // the group's candidates of the round, compacted
    // (memo keys are node << 9: scenes of 2^22 nodes or more run without the memo)
    RMemo memo{(GI_R_MEMO > 0 && sc.n_rnodes < (1 << 22)) ? s_memo + grp * GI_R_MEMO : nullptr};
    const long long n_items = tiles ? 2ll * (long long)*n_tiles : (m.n_local * (kTile * kTile) + 31) / 32;
    uint32_t nnode = 0, nprim = 0, npx = 0;
    for (long long item = blockIdx.x; item < n_items; item += gridDim.x) {   // uniform over the workgroup
        const long long ps = (tiles ? (long long)tiles[item >> 1] * 64 + (item & 1) * 32 : item * 32) + grp;
        if (memo.e)
            for (int k = sub; k < GI_R_MEMO; k += NSUB) memo.e[k] = -1;
        if (sub == 0) {
            s_best[grp] = 0ull;
            s_next[grp] = 0u;
        }
        __builtin_amdgcn_wave_barrier();
        const long long lt = ps >> 6;
        long long idx = -1;
        int x = 0, y = 0;
        const bool ok = lt < m.n_local && slot_pixel(m, lt, (int)(ps & 63), idx, x, y);
        y += m.y0;
        if (ok) {
            if (sub == 0) ++npx;
            const V3 o = cam.pos;
            const V3 d = normalize(primary_dir(cam, (double)x, (double)y));
            unsigned long long* gb = s_best + grp;
            RResult r;
            r.ent = -1;
            long long best = -1, mine = -1;
            for (int i = sub; i < sc.n_r_always; i += NSUB) r_group_consider<TRI>(sc, sc.r_always[i], o, d, gb, best, mine, r, nnode, nprim, memo);
            const XWNode* W = sc.rc_nodes;
            const F3 of = f3((float)o.x, (float)o.y, (float)o.z);
            const F3 ivf = inv_dir(d);
            const int n = r_items<NSUB>(W, of, ivf, tau, sub, s_item[grp]);
            int* seg = s_seg[grp] + sub * SEG;
            int* cand = s_cand[grp];
            // the lane's walk: (root, node, level, masks) while walking; a leaf's entities [pcur, pend)
            // still to queue; done once the group's items are all taken
            bool walking = false, done = false;
            int root = 0, node = 0, level = 0, pcur = 0, pend = 0;
            uint64_t mlo = 0, mhi = 0;
            for (;;) {
                // ---- walk phase: queue up to SEG candidates within GI_R_BATCH_STEPS node steps
                int nq = 0, steps = 0;
                while (nq < SEG) {
                    best = max(best, (long long)*(volatile unsigned long long*)gb - 1);
                    if (pcur < pend) {   // the current leaf's entities: those that can still win
                        const int e = sc.rc_ent[pcur++];
                        const int a0 = sc.app_off[e];
                        if (a0 != sc.app_off[e + 1] && sc.app_rec[a0].rank > best) seg[nq++] = e;
                        continue;
                    }
                    if (steps >= GI_R_BATCH_STEPS || done) break;
                    ++steps;
                    if (!walking) {      // the group's next item
                        const int i = (int)atomicAdd(s_next + grp, 1u);
                        if (i >= n) {
                            done = true;
                            break;
                        }
                        const int it = s_item[grp][i];
                        const int in = it >> 3, ic = it & 7;
                        if (sc.rc_maxkey[in * 8 + ic] <= best) continue;
                        const int ch = W[in].child[ic];
                        if (ch < 0) {
                            pcur = ~ch;
                            pend = ~ch + W[in].cnt[ic];
                        } else {
                            ++nnode;
                            const uint32_t cm = children_mask_line(W + ch, of, ivf, tau);
                            if (cm) {
                                root = node = ch;
                                level = 0;
                                mlo = mhi = 0;
                                lvl_set(mlo, mhi, 0, cm);
                                walking = true;
                            }
                        }
                        continue;
                    }
                    // one step of the item's subtree walk (stackless, rank order)
                    const uint32_t msk = lvl_get(mlo, mhi, level);
                    const int c = __builtin_ctz(msk);
                    lvl_set(mlo, mhi, level, msk & (msk - 1));
                    const XWNode* nd = W + node;
                    const int ch = nd->child[c];
                    if (sc.rc_maxkey[node * 8 + c] <= best) {
                        lvl_set(mlo, mhi, level, 0);
                    } else if (ch < 0) {
                        pcur = ~ch;
                        pend = ~ch + nd->cnt[c];
                    } else {
                        ++nnode;
                        const uint32_t cm = children_mask_line(W + ch, of, ivf, tau);
                        if (cm) {
                            node = ch;
                            ++level;
                            lvl_set(mlo, mhi, level, cm);
                        }
                    }
                    uint32_t rest = lvl_get(mlo, mhi, level);
                    while (rest == 0 && level > 0) {
                        --level;
                        node = level == 0 ? root : W[node].parent;
                        rest = lvl_get(mlo, mhi, level);
                    }
                    walking = rest != 0;
                }
                // ---- the group's queue, compacted (inclusive prefix of the lanes' counts)
                int incl = nq;
#pragma unroll
                for (int off = 1; off < NSUB; off <<= 1) {
                    const int t = __shfl_up(incl, off, NSUB);
                    if (sub >= off) incl += t;
                }
                const int total = __shfl(incl, NSUB - 1, NSUB);
                for (int k = 0; k < nq; ++k) cand[incl - nq + k] = seg[k];
                __builtin_amdgcn_wave_barrier();
                // ---- test phase: candidate j by lane j mod 8
                for (int j = sub; j < total; j += NSUB) {
                    best = max(best, (long long)*(volatile unsigned long long*)gb - 1);
                    r_group_consider<TRI>(sc, cand[j], o, d, gb, best, mine, r, nnode, nprim, memo);
                }
                __builtin_amdgcn_wave_barrier();
                // the wave leaves the loop once none of its lanes has anything left (groups stay in step)
                if (__ballot(!(done && !walking && pcur >= pend)) == 0) break;
            }
            r_group_write<NSUB, TRI>(sc, d, light, r, mine, sub, idx, rgb, rgb8);
        } else if (sub == 0 && idx >= 0 && m.shard_count > 1) {   // padding slot of a packed tile
            if (rgb) { rgb[3 * idx] = 0; rgb[3 * idx + 1] = 0; rgb[3 * idx + 2] = 0; }
            if (rgb8) { rgb8[3 * idx] = 0; rgb8[3 * idx + 1] = 0; rgb8[3 * idx + 2] = 0; }
        }
        __builtin_amdgcn_wave_barrier();   // the group's LDS state is reset for the next item
    }
    if (STATS) wave_add_stats(stats, npx, nnode, nprim, npx);
}

// Flat Mode R (VERDICT r03's chip-wide phases; the default for large scenes).  k_rf_walk: one lane per
// pixel slot walks the whole line BVH (no rank pruning) and stores a (slot, entity) pair for every
// entity of every leaf its line crosses; k_rf_hit: ent_hit over the pairs, the hitting ones kept;
// k_rf_scan + k_rf_reach: per hitting pair, the entity's appearances latest first against the pixel's
// best rank so far (atomic max), the first reachable one raising it; k_rf_shade: per pixel, the
// entity of the best rank (r_leaf_of_rank) tested again for its hit point and normal, shaded.  The
// answer -- the highest reachable hitting rank -- is k_mode_r's.
// Storage, no device-wide append counter (a first version appended every wave's pairs through one:
// the atomics serialised, k_rf_hit waited 95% of its cycles): the walk's wave for tile t owns tile
// t's region -- GI_RF_S0 pairs of its own, then pool pages of GI_RF_PAGE pairs taken with one atomic
// per page run (only tiles with many candidates take any), at most GI_RF_KMAX; rcnt[t] its pairs.  A
// pair is one word, (slot in the tile << 26) | entity.  k_rf_hit compacts a region's hitting pairs in
// place; persistent waves take regions in turn.  A tile that needs more pages than it may take, or
// finds the pool empty, is marked overflowed (rcnt = kRfOvf) and listed; the other phases skip it and
// k_mode_r_batch, launched behind them over that list, renders exactly those tiles.
#ifndef GI_RF_BUF
#define GI_RF_BUF 16   // k_rf_walk: pairs a lane buffers in LDS before the wave flushes
#endif
#define GI_RF_S0 512u     // pairs of a tile's own region (8 per pixel slot)
#define GI_RF_PAGE 512u   // pairs per pool page
#define GI_RF_KMAX 64u    // pool pages a tile may take (so at most 33,280 pairs per tile)
constexpr unsigned kRfOvf = 0xFFFFFFFFu;
constexpr unsigned kRfEntMask = (1u << 26) - 1u;   // scenes of more entities run k_mode_r_batch
struct RFlat {
    unsigned* pairs;            // n_regions x GI_RF_S0: each tile's own region
    unsigned* pool;             // n_pages x GI_RF_PAGE
    unsigned* pt;               // per tile: GI_RF_KMAX pool page ids (those taken)
    unsigned long long* best;   // per pixel slot: best rank + 1
    unsigned* cnt;              // [0] pool pages taken, [1] overflowed tiles
    unsigned* ovf;              // the overflowed tiles (cnt[1] of them)
    unsigned* rcnt;             // per tile: pairs, or kRfOvf
    unsigned* soff;             // per tile: its first segment of GI_RF_SEG pairs (k_rf_scan); [n_regions]: the total
    unsigned* shc;              // per segment: its hitting pairs (compacted to the segment's start)
    unsigned* sreg;             // per segment: its region
    unsigned* hoff;             // per segment: the hits before it (k_rf_scan); [segments]: the total
    double* dir;                // per pixel slot: its primary direction (k_rf_walk writes, the others read)
    unsigned n_pages;
};
__device__ __forceinline__ V3 rf_dir(const RFlat& f, unsigned slot) {
    const double* q = f.dir + 3 * (size_t)slot;
    return v3(q[0], q[1], q[2]);
}
// the page index (0 .. GI_RF_KMAX-1) holding pair i of a region beyond its own GI_RF_S0 (0 below)
__device__ __forceinline__ int rf_page(unsigned i) {
    return i < GI_RF_S0 ? 0 : (int)min((i - GI_RF_S0) / GI_RF_PAGE, GI_RF_KMAX - 1u);
}
// pair i of region r; pg: the id of its pool page (rf_page(i)-th of the region's pages)
__device__ __forceinline__ unsigned* rf_pair(const RFlat& f, long long r, unsigned i, unsigned pg) {
    return i < GI_RF_S0 ? f.pairs + (size_t)r * GI_RF_S0 + i : f.pool + (size_t)pg * GI_RF_PAGE + (i - GI_RF_S0) % GI_RF_PAGE;
}
// lane k: the id of region r's k-th pool page (only regions beyond their own pairs have any)
__device__ __forceinline__ unsigned rf_pages_of(const RFlat& f, long long r, unsigned n, int lane) {
    return (n > GI_RF_S0 && (unsigned)lane < GI_RF_KMAX) ? f.pt[(size_t)r * GI_RF_KMAX + lane] : 0u;
}
// k_rf_walk: a wave per tile walks the line BVH ONCE for all 64 of its pixels' lines.  The lines
// of a tile's pixels lie in the convex cone (apex at the camera) over the tile's 4 corner directions
// -- the primary direction is affine in the pixel coordinates (raytracer.h:41-43) -- so a node box
// that misses both nappes of that cone (a necessary-condition test against its 4 side planes, in
// fp64, the box widened by 2 tau) holds no pixel's candidate.  The wave pops up to 8 nodes per round
// from its LDS stack and tests their 64 children together, one per lane; hit interior children are
// pushed, hit leaf slots are then tested by every lane against its own line with the per-line slab
// test of the per-pixel walk (box_hit_line: children_mask_line's arithmetic), and a passing lane queues the
// slot's entities.  Since a node's box contains its children's, the pairs are exactly those of a
// per-pixel walk; a tile's loads are the same for all its lanes (broadcasts) instead of 64
// divergent walks.  A stack that would exceed GI_RF_STK marks the tile overflowed (k_mode_r_batch).
#define GI_RF_STK 512u   // traversal stack entries per wave (tile)
// one existing child's box (lo xyz, hi xyz) against the line: children_mask_line's arithmetic
__device__ __forceinline__ bool box_hit_line(const float* b, F3 of, F3 ivf, float tau) {
    const int sm = iv_signs(ivf);
    const float nx = (sm & 1) ? b[3] : b[0], fx = (sm & 1) ? b[0] : b[3];
    const float ny = (sm & 2) ? b[4] : b[1], fy = (sm & 2) ? b[1] : b[4];
    const float nz = (sm & 4) ? b[5] : b[2], fz = (sm & 4) ? b[2] : b[5];
    const float sx = (sm & 1) ? tau : -tau, sy = (sm & 2) ? tau : -tau, sz = (sm & 4) ? tau : -tau;
    const float tn = fmaxf(fmaxf(((nx + sx) - of.x) * ivf.x, ((ny + sy) - of.y) * ivf.y), ((nz + sz) - of.z) * ivf.z);
    const float tf = fminf(fminf(((fx - sx) - of.x) * ivf.x, ((fy - sy) - of.y) * ivf.y), ((fz - sz) - of.z) * ivf.z);
    return tn <= tf;
}
// may some line of the tile's double cone (side-plane normals n[4], through the camera c) meet the
// box [lo - wd, hi + wd]?  Forward nappe: every side plane has part of the box on its inner side;
// backward nappe: every side plane has part of it on its outer side.  Conservative (margin eps).
__device__ __forceinline__ bool box_meets_cone(const float* lo, const float* hi, double wd, V3 c, const V3* n) {
    const double l[3] = {(double)lo[0] - wd - c.x, (double)lo[1] - wd - c.y, (double)lo[2] - wd - c.z};
    const double h[3] = {(double)hi[0] + wd - c.x, (double)hi[1] + wd - c.y, (double)hi[2] + wd - c.z};
    const double ext = fmax(fmax(fabs(l[0]), fabs(h[0])), fmax(fmax(fabs(l[1]), fabs(h[1])), fmax(fabs(l[2]), fabs(h[2]))));
    bool fwd = true, bwd = true;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        const double nn[3] = {n[a].x, n[a].y, n[a].z};
        double mx = 0.0, mn = 0.0, an = 0.0;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
            const double u = nn[k] * l[k], v = nn[k] * h[k];
            mx += fmax(u, v);
            mn += fmin(u, v);
            an += fabs(nn[k]);
        }
        const double eps = 1e-9 * an * ext;
        fwd = fwd && mx >= -eps;
        bwd = bwd && mn <= eps;
    }
    return fwd || bwd;
}
template <bool STATS>
__global__ __launch_bounds__(256) void k_rf_walk(DevScene sc, CamDev cam, TileMap m, float tau, RFlat f,
                                                 unsigned long long* stats) {
    __shared__ int s_buf[256][GI_RF_BUF];
    __shared__ unsigned s_pt[4][GI_RF_KMAX];   // the wave's pool pages
    __shared__ int s_stk[4][GI_RF_STK];        // the tile's traversal stack (line-BVH nodes)
    __shared__ int s_leaf[4][64];              // a round's hit leaf slots: (node << 3) | slot
    __shared__ float s_lb[4][64][6];           //   their boxes (lo xyz, hi xyz)
    __shared__ int s_le[4][64][6];             //   their first entity, count and first 4 entity ids
    const long long slot = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long region = slot >> 6;
    const int lane = threadIdx.x & 63;
    int* buf = s_buf[threadIdx.x];
    unsigned* pt = s_pt[threadIdx.x >> 6];
    int* stk = s_stk[threadIdx.x >> 6];
    int* leaves = s_leaf[threadIdx.x >> 6];
    float (*lb)[6] = s_lb[threadIdx.x >> 6];
    int (*le)[6] = s_le[threadIdx.x >> 6];
    long long idx = -1;
    int x = 0, y = 0;
    const bool in = slot < m.n_local * 64;
    const bool ok = in && slot_pixel(m, slot >> 6, (int)(slot & 63), idx, x, y);
    if (in) f.best[slot] = 0ull;
    if (__ballot(in) == 0) return;   // (a wave is one tile: all of it beyond the shard's tiles)
    uint32_t nnode = 0;
    const XWNode* W = sc.rc_nodes;
    int nb = 0;
    unsigned fill = 0, npg = 0;   // the wave's pairs and pool pages so far (the same in every lane)
    bool ovf = false;
    const unsigned tag = (unsigned)(slot & 63) << 26;
    const F3 of = f3((float)cam.pos.x, (float)cam.pos.y, (float)cam.pos.z);
    F3 ivf = f3(1, 1, 1);
    if (ok) {
        const V3 d = normalize(primary_dir(cam, (double)x, (double)(y + m.y0)));
        double* qd = f.dir + 3 * slot;
        qd[0] = d.x; qd[1] = d.y; qd[2] = d.z;
        ivf = inv_dir(d);
    }
    // flush the wave's buffers into its region (pool pages taken as needed: one atomic)
    auto flush = [&]() {
        int incl = nb;
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const int t = __shfl_up(incl, off);
            if (lane >= off) incl += t;
        }
        const unsigned tot = (unsigned)__shfl(incl, 63);
        const unsigned end = fill + tot;
        const unsigned need = end > GI_RF_S0 ? (end - GI_RF_S0 + GI_RF_PAGE - 1) / GI_RF_PAGE : 0u;
        if (need > npg && !ovf) {
            unsigned b = 0;
            if (lane == 0 && need <= GI_RF_KMAX) b = atomicAdd(f.cnt, need - npg);
            b = __shfl(b, 0);
            if (need > GI_RF_KMAX || b + (need - npg) > f.n_pages) {
                ovf = true;   // (pages taken past the pool's end are simply unused)
            } else {
                if ((unsigned)lane >= npg && (unsigned)lane < need) {
                    pt[lane] = b + (unsigned)lane - npg;
                    f.pt[(size_t)region * GI_RF_KMAX + lane] = b + (unsigned)lane - npg;
                }
                npg = need;
                __builtin_amdgcn_wave_barrier();
            }
        }
        if (!ovf) {
            for (int k = 0; k < nb; ++k) {
                const unsigned j = fill + (unsigned)(incl - nb + k);
                *rf_pair(f, region, j, pt[rf_page(j)]) = (unsigned)buf[k];
            }
        }
        fill = end;
        nb = 0;
    };
    // every ray's ImpSpheres (build_rcand keeps them out of the line BVH)
    for (int k = 0; k < sc.n_r_always; ++k) {
        if (__ballot(nb >= (int)GI_RF_BUF) != 0) flush();
        if (ok) buf[nb++] = (int)(tag | (unsigned)sc.r_always[k]);
    }
    // the tile's cone: corner directions from its pixels' extents (uniform)
    int x0 = ok ? x : INT_MAX, x1 = ok ? x : INT_MIN, y0 = ok ? y : INT_MAX, y1 = ok ? y : INT_MIN;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        x0 = min(x0, __shfl_xor(x0, off));
        x1 = max(x1, __shfl_xor(x1, off));
        y0 = min(y0, __shfl_xor(y0, off));
        y1 = max(y1, __shfl_xor(y1, off));
    }
    int sp = 0;   // stack entries (uniform)
    V3 n[4];
    if (x0 <= x1) {
        const V3 da = primary_dir(cam, (double)x0, (double)(y0 + m.y0)), db = primary_dir(cam, (double)x1, (double)(y0 + m.y0));
        const V3 dc = primary_dir(cam, (double)x1, (double)(y1 + m.y0)), dd = primary_dir(cam, (double)x0, (double)(y1 + m.y0));
        const V3 mid = ((da + db) + (dc + dd)) * 0.25;
        n[0] = cross(da, db);
        n[1] = cross(db, dc);
        n[2] = cross(dc, dd);
        n[3] = cross(dd, da);
#pragma unroll
        for (int a = 0; a < 4; ++a)
            if (dot(n[a], mid) < 0) n[a] = -n[a];
        if (lane == 0) stk[0] = 0;   // the root
        sp = 1;
        __builtin_amdgcn_wave_barrier();
    }
    const double wd = 2.0 * (double)tau;
    const V3 cp = cam.pos;
    while (sp > 0 && !ovf) {
        // ---- up to 8 nodes from the stack, their 64 children one per lane
        const int nt = min(sp, 8);
        const int j = lane >> 3, c = lane & 7;
        int ch = 0;
        bool hit = false;
        if (j < nt) {
            const int nd_i = stk[sp - 1 - j];
            const XWNode* nd = W + nd_i;
            if ((nd->exists >> c) & 1) {
                const float lo[3] = {nd->lo[0][c], nd->lo[1][c], nd->lo[2][c]};
                const float hi[3] = {nd->hi[0][c], nd->hi[1][c], nd->hi[2][c]};
                hit = box_meets_cone(lo, hi, wd, cp, n);
                ch = nd->child[c];
                if (hit && ch < 0) ch = ~((nd_i << 3) | c);   // a leaf slot: (node << 3) | slot, negated
            }
            if (c == 0) ++nnode;
        }
        __builtin_amdgcn_wave_barrier();
        sp -= nt;
        const unsigned long long m_in = __ballot(hit && ch >= 0), m_lf = __ballot(hit && ch < 0);
        const int n_in = __popcll(m_in), n_lf = __popcll(m_lf);
        if ((unsigned)(sp + n_in) > GI_RF_STK) {
            ovf = true;
            break;
        }
        if (hit && ch >= 0) stk[sp + __popcll(m_in & ((1ull << lane) - 1))] = ch;
        if (hit && ch < 0) leaves[__popcll(m_lf & ((1ull << lane) - 1))] = ~ch;
        sp += n_in;
        __builtin_amdgcn_wave_barrier();
        // ---- the round's leaf slots against every lane's own line.  Their records are fetched first,
        // lane j those of slot j, into LDS (one memory round trip for the round instead of one per
        // slot); then every slot is tested by every lane from LDS
        if (lane < n_lf) {
            const int it = leaves[lane];
            const XWNode* nd = W + (it >> 3);
            const int sl = it & 7;
#pragma unroll
            for (int a = 0; a < 3; ++a) {
                lb[lane][a] = nd->lo[a][sl];
                lb[lane][3 + a] = nd->hi[a][sl];
            }
            const int e0 = ~nd->child[sl], cnt = nd->cnt[sl];
            le[lane][0] = e0;
            le[lane][1] = cnt;
#pragma unroll
            for (int k = 0; k < 4; ++k) le[lane][2 + k] = k < cnt ? sc.rc_ent[e0 + k] : 0;
        }
        __builtin_amdgcn_wave_barrier();
        for (int i = 0; i < n_lf; ++i) {
            const bool pass = ok && box_hit_line(lb[i], of, ivf, tau);
            const int e0 = le[i][0], cnt = le[i][1];   // (uniform: one leaf for the wave)
            for (int k0 = 0; k0 < cnt; k0 += (int)GI_RF_BUF / 2) {
                const int kk = min(cnt - k0, (int)GI_RF_BUF / 2);
                if (__ballot(nb + kk > (int)GI_RF_BUF) != 0) flush();
                if (pass)
                    for (int k = 0; k < kk; ++k) {
                        const int q = k0 + k;
                        buf[nb++] = (int)(tag | (unsigned)(q < 4 ? le[i][2 + q] : sc.rc_ent[e0 + q]));
                    }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    flush();
    if (in && lane == 0) {
        f.rcnt[region] = ovf ? kRfOvf : fill;
        if (ovf) f.ovf[atomicAdd(f.cnt + 1, 1u)] = (unsigned)region;
    }
    if (STATS) {
        wave_add_stats(stats, 0, nnode, 0, 0);
        if (in && lane == 0) {
            atomicAdd(stats + GI_STAT_R_PAIRS, (unsigned long long)fill);
            if (ovf) atomicAdd(stats + GI_STAT_R_OVF_TILES, 1ull);
        }
    }
}
// the last index k in [0, n) with off[k] <= v (off ascending from off[0] = 0)
__device__ __forceinline__ long long rf_find(const unsigned* off, long long n, long long v) {
    long long lo = 0, hi = n - 1;
    while (lo < hi) {
        const long long mid = (lo + hi + 1) >> 1;
        if ((long long)off[mid] <= v) lo = mid;
        else hi = mid - 1;
    }
    return lo;
}
// The pairs' exact entity tests, per segment of GI_RF_SEG pairs of a region (k_rf_scan numbers them),
// its hitting pairs compacted to the segment's start.  Persistent waves take segments in turn, so the
// thousands of pairs of a soup-core tile are tested by many waves at once, not by one in sequence.
#ifndef GI_RF_SEG
#define GI_RF_SEG 512u   // pairs per segment (8 chunks of 64)
#endif
template <bool STATS, bool TRI>
__global__ __launch_bounds__(64) void k_rf_hit(DevScene sc, CamDev cam, TileMap m, RFlat f, unsigned long long* stats) {
    const int lane = threadIdx.x & 63;
    const long long n_regions = m.n_local;
    const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_w = ((long long)gridDim.x * blockDim.x) >> 6;
    const long long n_seg = f.soff[n_regions];
    uint32_t nprim = 0;
    long long cur = -1;
    unsigned pg = 0, n = 0;
    for (long long sg = gw; sg < n_seg; sg += n_w) {
        const long long r = rf_find(f.soff, n_regions, sg);
        if (r != cur) {
            n = f.rcnt[r];   // (overflowed tiles have no segment)
            pg = rf_pages_of(f, r, n, lane);
            cur = r;
        }
        const unsigned p0 = (unsigned)(sg - (long long)f.soff[r]) * GI_RF_SEG, p1 = min(n, p0 + GI_RF_SEG);
        unsigned kept = 0;
        for (unsigned i0 = p0; i0 < p1; i0 += 64) {
            const unsigned i = i0 + lane;
            const unsigned pin = __shfl(pg, rf_page(i));
            bool hit = false;
            unsigned pr = 0;
            if (i < p1) {
                pr = *rf_pair(f, r, i, pin);
                const unsigned slot = (unsigned)r * 64u + (pr >> 26);
                const V3 d = rf_dir(f, slot);
                V3 P, N;
                hit = ent_hit<TRI>(sc, sc.ents[pr & kRfEntMask], cam.pos, d, P, N, nprim) && sq3(P - cam.pos) < DBL_MAX;   // raytracer.h:58-65
            }
            const unsigned long long mh = __ballot(hit);
            const unsigned k = p0 + kept + (unsigned)__popcll(mh & ((1ull << lane) - 1));
            const unsigned pout = __shfl(pg, rf_page(k));
            if (hit) *rf_pair(f, r, k, pout) = pr;   // at or before its own position, already read
            kept += (unsigned)__popcll(mh);
        }
        if (lane == 0) {
            f.shc[sg] = kept;
            f.sreg[sg] = (unsigned)r;
        }
    }
    if (STATS) wave_add_stats(stats, 0, 0, nprim, 0);
}
// out[k] = sum of ceil(in[j] / div) over j < k, out[n] = the total (in[j] == kRfOvf counts 0); n from
// the device (n_dev) or the host.  One workgroup: tiles of 8192 entries, a coalesced load of their
// counts into LDS, 8 consecutive ones per thread, wave prefix sums by shuffles, the 16 wave totals, a
// coalesced store (the first version -- 32 strided entries per thread -- took ~50 us for the 32,400
// tiles of a 1080p frame; this one ~15 us).
__global__ __launch_bounds__(1024) void k_rf_scan(const unsigned* in, unsigned* out, const unsigned* n_dev, long long n_host,
                                                 unsigned div) {
    __shared__ unsigned s_v[8192];
    __shared__ unsigned s_w[16];
    const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
    const long long n = n_dev ? (long long)*n_dev : n_host;
    unsigned carry = 0;
    for (long long base = 0; base < n; base += 8192) {
        for (int k = t; k < 8192; k += 1024) {
            const long long r = base + k;
            const unsigned v = r < n ? in[r] : 0u;
            s_v[k] = v == kRfOvf ? 0u : (v + div - 1u) / div;
        }
        __syncthreads();
        unsigned v[8], sum = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            v[k] = s_v[8 * t + k];
            sum += v[k];
        }
        unsigned incl = sum;   // inclusive prefix over the wave's lanes
#pragma unroll
        for (int off = 1; off < 64; off <<= 1) {
            const unsigned u = __shfl_up(incl, off);
            if (lane >= off) incl += u;
        }
        if (lane == 63) s_w[wv] = incl;
        __syncthreads();
        unsigned before = carry, tot = 0;
#pragma unroll
        for (int w = 0; w < 16; ++w) {
            before += w < wv ? s_w[w] : 0u;
            tot += s_w[w];
        }
        unsigned run = before + incl - sum;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            s_v[8 * t + k] = run;
            run += v[k];
        }
        __syncthreads();
        for (int k = t; k < 8192; k += 1024) {
            const long long r = base + k;
            if (r < n) out[r] = s_v[k];
        }
        carry += tot;
        __syncthreads();
    }
    if (t == 0) out[n] = carry;
}
// per hitting pair: its entity's latest reachable appearance that beats the pixel's best rank.
// Persistent waves take chunks of 64 / G consecutive hits of the whole frame in turn (hoff numbers
// them across the segments, so chunks are full; a chunk's first segment by a binary search, each
// hit's from there), so the hits of a soup-core tile are shared by many waves.  G lanes per hit (G =
// 4: each tests 3 of a node's 12 ExpBox faces, r_box_test): a wave's node-test step runs the union
// of its lanes' face tests, which with 64 hits of mixed outcomes is nearly all 12 whether or not a
// face accepts early, so splitting the faces shortens every hit's chain of tests about G-fold for
// the same instructions per hit -- what a sparse launch (an eighth of R-C4: ~500 chunks of 64 on a
// chip of 2,560 wave slots) waits on.  One wave per workgroup: its LDS holds a node-test memo
// (RMemo, GI_R_MEMO entries) per pixel slot of a tile, cleared at every chunk and each entry tagged
// with its hit's run of equal tiles in the chunk, so hits of different tiles never read each
// other's results.
template <bool STATS, int G>
__device__ __forceinline__ void rf_reach_chunks(const DevScene& sc, const CamDev& cam, const RFlat& f, unsigned long long* stats,
                                                int* s_memo, long long n_seg, long long n_hits) {
    constexpr int H = 64 / G;   // hits per chunk
    const int lane = threadIdx.x & 63;
    const int hl = lane / G;   // this lane's hit in the chunk; lane % G its part of the face tests
    const long long gw = ((long long)blockIdx.x * blockDim.x + threadIdx.x) >> 6, n_w = ((long long)gridDim.x * blockDim.x) >> 6;
    const bool use_memo = GI_R_MEMO > 0 && sc.n_rnodes < (1 << 22);
    uint32_t nnode = 0;
    // (chunks from a device counter instead, as waves free up: R-C4 0.80 -> 0.88 ms)
    for (long long c = gw; H * c < n_hits; c += n_w) {
        const long long i = H * c + hl;
        long long sg = rf_find(f.hoff, n_seg, H * c);   // the chunk's first segment (uniform)
        long long r = -1;
        if (i < n_hits) {
            while (sg + 1 < n_seg && (long long)f.hoff[sg + 1] <= i) ++sg;   // this hit's
            r = f.sreg[sg];
        }
        // the memo is the chunk's: cleared here (each lane a row), its entries tagged with the hit's
        // run of equal tiles in the chunk (<= 64 runs, so the tag fits its 8 bits).  Two hits share a
        // tag only if they hold the same tile, hence with the same row the same pixel: no entry is
        // ever read for another ray (a tag of the tile's low bits alone let tiles r and r + 256 of
        // one chunk, or of the wave's earlier chunks, read each other's results)
        const long long r_prev = __shfl(r, lane >= G ? lane - G : 0);
        const unsigned long long runs = __ballot(lane % G == 0 && r >= 0 && (hl == 0 || r != r_prev));
        const int run_ord = __popcll(runs & ((2ull << lane) - 1)) - 1;
        if (use_memo) {
            int4* row = reinterpret_cast<int4*>(s_memo + lane * GI_R_MEMO);
            for (int k = 0; k < GI_R_MEMO / 4; ++k) row[k] = make_int4(-1, -1, -1, -1);   // (matches no key)
        }
        __builtin_amdgcn_wave_barrier();
        if (r >= 0) {   // (every value below is the hit's: a group's lanes stay together)
            const unsigned p = (unsigned)(sg - (long long)f.soff[r]) * GI_RF_SEG + (unsigned)(i - (long long)f.hoff[sg]);
            const unsigned pg = p < GI_RF_S0 ? 0u : f.pt[(size_t)r * GI_RF_KMAX + rf_page(p)];
            const unsigned pr = *rf_pair(f, r, p, pg);
            const unsigned slot = (unsigned)r * 64u + (pr >> 26);
            const int e = (int)(pr & kRfEntMask);
            const RMemo memo{use_memo ? s_memo + (pr >> 26) * GI_R_MEMO : nullptr, run_ord << 1};
            const V3 d = rf_dir(f, slot);
            const int a1 = sc.app_off[e + 1];
            for (int a = sc.app_off[e]; a < a1; ++a) {
                const RApp ap = sc.app_rec[a];
                const long long rk = ap.rank;
                long long bst = (long long)*(volatile unsigned long long*)(f.best + slot) - 1;
                if (G > 1) bst = __shfl(bst, lane & ~(G - 1));   // one reading for the group (others raise it)
                if (rk <= bst) break;
                if (r_path_reachable<G>(sc, ap.p0, ap.p1, cam.pos, d, nnode, memo)) {
                    if (lane % G == 0) atomicMax(f.best + slot, (unsigned long long)(rk + 1));
                    break;
                }
            }
        }
    }
    if (STATS) wave_add_stats(stats, 0, lane % G == 0 ? nnode : 0u, 0, 0);   // (node tests per hit, not per lane)
}
// G = 4 for launches of at most kRfGroupHits hits (<= 2,560 chunks of 16: one per resident wave of
// the chip, 10 per CU by the memo's LDS), else G = 1.  R-C4 (266 k hits) and its half and quarter
// shares run faster at G = 1 (whole frame 0.67 against 0.89 ms: where the chip is full, the early
// face exits of the single-lane test save more than the shorter chains); an eighth (33 k hits)
// at G = 4 (rank 0 / 7: 0.33 / 0.37 -> 0.30 / 0.31 ms).  group: 0 chooses, 1 or 4 forces (tests).
constexpr long long kRfGroupHits = 40960;
template <bool STATS>
__global__ __launch_bounds__(64) void k_rf_reach(DevScene sc, CamDev cam, TileMap m, RFlat f, unsigned long long* stats, int group) {
    __shared__ __attribute__((aligned(16))) int s_memo[GI_R_MEMO > 0 ? 64 * GI_R_MEMO : 4];
    const long long n_seg = f.soff[m.n_local], n_hits = f.hoff[n_seg];
    if (group == 4 || (group == 0 && n_hits <= kRfGroupHits)) rf_reach_chunks<STATS, 4>(sc, cam, f, stats, s_memo, n_seg, n_hits);
    else rf_reach_chunks<STATS, 1>(sc, cam, f, stats, s_memo, n_seg, n_hits);
}
// per pixel: the best rank's entity, shaded (overflowed tiles: left to k_mode_r_batch)
template <bool STATS, bool TRI>
__global__ __launch_bounds__(256) void k_rf_shade(DevScene sc, CamDev cam, V3 light, TileMap m, double* rgb, uint8_t* rgb8,
                                                  RFlat f, unsigned long long* stats) {
    const long long slot = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (slot < m.n_local * 64 && f.rcnt[slot >> 6] == kRfOvf) return;   // (uniform: a wave is one tile)
    long long idx = -1;
    int x = 0, y = 0;
    const bool ok = slot < m.n_local * 64 && slot_pixel(m, slot >> 6, (int)(slot & 63), idx, x, y);
    uint32_t nprim = 0;
    if (ok) {
        const V3 d = rf_dir(f, (unsigned)slot);
        const long long b = (long long)f.best[slot] - 1;
        double c0 = 0, c1 = 0, c2 = 0;
        if (b >= 0) {
            const int leaf = sc.r_leaf_of_rank[b >> 32];
            const REnt& e = sc.ents[sc.leaf_ents[sc.rnodes[leaf].ent_off + (int)(b & 0xFFFFFFFFll)]];
            V3 P, N;
            ent_hit<TRI>(sc, e, cam.pos, d, P, N, nprim);
            int32_t u, v;
            tex_coord<TRI>(sc, e, P, u, v);
            const V3 col = shade_ref(e, d, light, P, N, u, v);
            c0 = col.x; c1 = col.y; c2 = col.z;
        }
        if (rgb) { rgb[3 * idx] = c0; rgb[3 * idx + 1] = c1; rgb[3 * idx + 2] = c2; }
        if (rgb8) quantize(c0, c1, c2, rgb8 + 3 * idx);
    } else if (idx >= 0 && m.shard_count > 1) {   // padding slot of a packed tile
        if (rgb) { rgb[3 * idx] = 0; rgb[3 * idx + 1] = 0; rgb[3 * idx + 2] = 0; }
        if (rgb8) { rgb8[3 * idx] = 0; rgb8[3 * idx + 1] = 0; rgb8[3 * idx + 2] = 0; }
    }
    if (STATS) wave_add_stats(stats, ok ? 1 : 0, 0, nprim, ok ? 1 : 0);
}

template <bool STATS>
__global__ __launch_bounds__(256) void k_mode_r(DevScene sc, CamDev cam, V3 light, TileMap m, double* rgb,
                                                 uint8_t* rgb8, unsigned long long* stats, float tau, int dfs) {
    long long idx = -1;
    int x = 0, y = 0;
    const long long lt = (long long)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
    const bool ok = lane_pixel(m, lt, idx, x, y);
    y += m.y0;
    uint32_t nnode = 0, nprim = 0;
    if (ok) {
        const V3 o = cam.pos;
        const V3 d = normalize(primary_dir(cam, (double)x, (double)y));   // Ray ctor (ray.h:6)
        RResult r;
        if (dfs) trace_mode_r(sc, o, d, r, nnode, nprim);   // the reference's list order, reversed (A/B)
        else trace_mode_r_cand(sc, o, d, tau, r, nnode, nprim);
        double c0 = 0, c1 = 0, c2 = 0;
        if (r.ent >= 0) {
            const REnt e = sc.ents[r.ent];
            int32_t u, v;
            tex_coord(sc, e, r.P, u, v);
            const V3 col = shade_ref(e, d, light, r.P, r.N, u, v);
            c0 = col.x; c1 = col.y; c2 = col.z;
        }
        if (rgb) { rgb[3 * idx] = c0; rgb[3 * idx + 1] = c1; rgb[3 * idx + 2] = c2; }
        if (rgb8) quantize(c0, c1, c2, rgb8 + 3 * idx);
    } else if (idx >= 0 && m.shard_count > 1) {   // padding lanes of a packed tile
        if (rgb) { rgb[3 * idx] = 0; rgb[3 * idx + 1] = 0; rgb[3 * idx + 2] = 0; }
        if (rgb8) { rgb8[3 * idx] = 0; rgb8[3 * idx + 1] = 0; rgb8[3 * idx + 2] = 0; }
    }
    if (STATS && lt < m.n_local) wave_add_stats(stats, ok ? 1 : 0, nnode, nprim, ok ? 1 : 0);
}


// Mode X path state machine.  A lane owns one pixel at a time and walks its spp samples in order;
// every loop iteration a lane either makes ONE traversal step of its current ray (pop a node: cull,
// push children, or test a leaf's primitives) or, once its ray has finished, runs the shading
// handler that consumes the hit and spawns the lane's next ray (shadow ray, next bounce, or the
// next sample's primary ray).  When a lane's pixel is complete it writes it and takes the next
// pixel from the device-wide slot counter (wave ballot + one atomic per refill), so lanes never
// wait for each other at sample, bounce or pixel boundaries (a fixed 8x8 tile per wave left ~1/4
// of the lanes idle behind the tile's slowest pixel).  The handler runs once at least half of the
// live lanes have a finished ray, or when none is still traversing, so it executes with a
// well-filled EXEC mask.  The per-path operation sequence is exactly the oracle's (pixel_mode_x in
// oracle/gi_oracle.cpp), so results are bit-identical whatever the schedule.
enum : int { PH_CLOSEST = 0, PH_SHADOW = 1, PH_NEED = 2, PH_START = 3, PH_DEAD = 4, PH_DONEPX = 5, PH_HELP = 6 };

#ifndef GI_X_START_BURST
#define GI_X_START_BURST 16   // primary rays a lane may resolve by the root test per handler run
#endif
#ifndef GI_X_MIN_WAVES
#define GI_X_MIN_WAVES 3       // minimum waves per SIMD, HBM-resident scenes (<= 168 VGPRs)
#endif
#ifndef GI_X_MIN_WAVES_LDS
#define GI_X_MIN_WAVES_LDS 4   // LDS-resident scenes (<= 128 VGPRs; the few spills sit in the handler)
#endif

struct XCounters {
    uint64_t rays = 0, nodes = 0, prims = 0, px = 0, res = 0;   // res: samples resolved without traversal
    uint64_t iters = 0, trav = 0, handle = 0, hlanes = 0, hclose = 0, hshadow = 0;   // wave-level (lane 0)
    uint64_t cyc_trav = 0, cyc_hit = 0, cyc_next = 0, cyc_all = 0;                    // wave clock cycles
    // the longest sample path (primary ray to its end): (wall_clock64 ticks << 32) | (wave iterations
    // << 16) | traversal steps of that lane during it (both saturated at 65535), maximised as one word
    uint64_t path_t0 = 0, path_max = 0;
    uint32_t path_it = 0, path_st = 0;
    // divergence profile (wave-level, lane 0): loop iterations in which some lane ran a node test /
    // a leaf test / an inline bounce restart / a handler start-loop pass, and the lanes that did
    uint64_t it_node = 0, ln_node = 0, it_leaf = 0, ln_leaf = 0, it_rs = 0, ln_rs = 0, it_st = 0, ln_st = 0;
};

// Mode X work list (k_x_classify -> k_mode_x -> k_x_reduce).  A pixel whose every jittered primary
// ray misses the scene's root box is resolved by the classifier (all samples add exactly +0); the
// others are appended to `list` (their slot numbers in tile order).  k_mode_x's unit of work is one
// (listed pixel, run of k consecutive samples), k a power of two <= 8 chosen per launch from the
// amount of work (about 8 units per lane: k = 8 for a whole C3 frame, 1 for an 8-way shard of it).
// Units come in blocks of 64: block b = (group g of 64 listed pixels, run c), so one block is one
// run of 64 pixels; a wave takes a whole block with one atomic and one coalesced load of the
// group's 64 list entries, and hands its units to lanes as they need work (no per-unit round trip).
// With spp > 1 every sample's radiance is stored to part[pixel][sample] and k_x_reduce adds a
// pixel's samples in sample order from +0 (the oracle's sum), so results do not depend on k, on
// the schedule or on the shard count; with spp == 1 the unit writes the pixel.  Splitting pixels
// over lanes keeps every lane busy until the end of the frame (a whole 64-spp pixel per unit left
// the kernel waiting on its last lanes: rendering 1/8 of the C3 frame took 75% of the whole frame's
// time).
struct XWork {
    const unsigned* list;    // listed pixel slots (tile order)
    const unsigned* n_list;  // device count written by k_x_classify
    double* part;            // per-sample radiance [list index][sample][3] (spp > 1)
    unsigned* blocks;        // device counter of blocks taken
    int s0, s1;              // the launch's samples [s0, s1) of the spp (0, spp; or a progressive pass)
};

#ifndef GI_X_UNITS_PER_LANE
#define GI_X_UNITS_PER_LANE 8   // target units per lane when choosing the run length k
#endif
#ifndef GI_X_MAX_RUN
// largest run length k (samples per unit).  1: every unit is one sample -- measured fastest on the
// BASELINE Mode X workloads (C3 7.45 -> 6.72 ms, C5 338 -> 328 ms, X-zoo 7.7 -> 6.0 ms against k = 8;
// fewer wave iterations and fuller handler runs); scenes whose samples are mostly cheap background
// rays pay for the per-unit fetch instead (X-main 0.47 -> 0.72 ms) and are better served by 8
#define GI_X_MAX_RUN 1
#endif

// Shadow-ray handoff (HELP, xflags bit 3).  Once a wave has lanes with no work left (PH_DEAD: the
// end of the frame, or of a small shard), a lane that has shaded a hit whose path continues gives
// that hit's shadow ray to an idle lane and starts its next bounce ray at once, instead of tracing
// the two one after the other: the path's critical path becomes max(shadow_b, closest_{b+1}) per
// bounce instead of their sum.  The owner keeps both candidate sums (Lv lit, Lo dark) as before and
// picks one when the helper's answer arrives, before it shades the next hit, so the operations --
// and the frame, bit for bit -- are the oracle's.  Per lane in LDS (column layout, 256 lanes):
// ray[7][256] (origin, direction, tmax), own[256] (owner lane within the wave, -1: none) and
// res[256] (the owner's answer: 0 pending, 1 lit, 2 occluded).
struct XHelp {
    double* ray;
    int* own;
    int* res;
};
__device__ __forceinline__ int nth_set_bit(unsigned long long m, unsigned n) {
    for (unsigned i = 0; i < n; ++i) m &= m - 1;
    return __ffsll((long long)m) - 1;
}

// NST: the wide-node index of every level of the current traversal path lives in LDS (nst[level *
// 256], one column per lane), so climbing out of exhausted levels is one ds_read instead of a chain
// of dependent parent-pointer loads from HBM / L2 (one per level climbed).
template <bool STATS, bool PAIR, bool PSL, bool NST, bool HELP, bool SH, bool TRI, typename NodeP,
          typename HotP, typename PrimP, typename EntP>
__device__ __forceinline__ void mode_x_wave(const DevScene& sc, NodeP W, HotP H, PrimP XP, EntP EN, double* pslot,
                                            int* nst, XHelp hp_,
                                            const CamDev& cam, V3 light,
                                            const TileMap& m, int spp, int depth, uint64_t seed, double* rgb,
                                            uint8_t* rgb8, unsigned* blk_list, const XWork& wk, int handle8,
                                            int xflags, XCounters& cnt) {
    const int lane = threadIdx.x & 63;
    const unsigned n_list = *wk.n_list;
    // run length k: the largest power of two <= the launch's maximum (xflags bits 8-10: log2, from
    // GI_X_MAX_RUN or the environment variable of that name) and <= spp that still leaves about
    // GI_X_UNITS_PER_LANE units per lane of the grid (every wave computes the same k)
    int k = 1;
    {
        const double lanes = (double)gridDim.x * (double)blockDim.x;
        const double samples = (double)n_list * (double)(wk.s1 - wk.s0);
        const int max_run = 1 << ((xflags >> 8) & 7);
        while (2 * k <= max_run && 2 * k <= wk.s1 - wk.s0 && samples / (2.0 * k) >= GI_X_UNITS_PER_LANE * lanes) k *= 2;
    }
    const unsigned runs = (unsigned)((wk.s1 - wk.s0 + k - 1) / k);    // units per pixel (run c: samples s0 + c k ...)
    const unsigned n_groups = (n_list + 63u) >> 6;
    // xflags bit 5 (pixel-major blocks, launches of >= 64 units per pixel): a block is ONE pixel's
    // 64 consecutive runs instead of 64 pixels' run c, so a wave's lanes start on the same pixel's
    // samples -- nearly the same primary ray -- and walk the same nodes together
    const bool pm = (xflags & 32) != 0 && runs >= 64u;
    const unsigned rpb = (runs + 63u) >> 6;   // (pm) blocks per pixel
    const unsigned n_blocks = pm ? n_list * rpb : n_groups * runs;
    // xflags bit 4 (spread): group g holds list entries g, g + G, g + 2G, ... (G groups) instead of
    // 64 consecutive ones, so a wave's 64 pixels come from all over the frame: the expensive pixels
    // of a frame cluster in space (the soup's core), and consecutive entries would give all of them
    // to a few waves, whose lanes then pace each other (every loop iteration waits for the others'
    // shading) while the rest of the chip idles.  Spread, each long path shares its wave with
    // cheap ones that finish early (fast iterations, idle lanes for its shadow rays).
    const bool spread = (xflags & 16) != 0;
    // the wave's current block lives in its LDS row: blk_list[0..63] = the group's list entries,
    // blk_meta = {units handed out, group, run}; lanes that do not run the handler keep no copy
    unsigned* blk_meta = blk_list + 64;
    if (lane == 0) { blk_meta[0] = 64u; blk_meta[3] = 0u; }
    __builtin_amdgcn_wave_barrier();
    const bool inline_shadow = (xflags & 1) != 0;
    const bool no_shadow = (xflags & 4) != 0;   // GI_FLAG_X_NO_SHADOW (tests): every light visible
    const bool handoff = HELP && (xflags & 8) != 0 && !no_shadow;
    const int tid = threadIdx.x, wbase = tid & ~63;
    if (HELP) {
        hp_.own[tid] = -1;
        hp_.res[tid] = 0;
    }
    bool pend = false;       // this lane's last shadow ray is being traced by a helper
    bool any_gave = false;   // some lane of the wave handed a shadow ray over in the last iteration
    int howner = 0;          // PH_HELP: the owner lane
    uint32_t nnode = 0, nprim = 0, nrays = 0, nres = 0, npx = 0, nsteps = 0;
    long long idx = -1;
    int x = 0, y = 0;
    uint64_t key = 0;

    int phase = PH_NEED;
    int smp = 0, b = 0;
    // current ray
    V3 o = cam.pos, d = v3(1, 0, 0);
    int dmask = 0, best = -1, node = 0, level = 0;
    bool raying = false;
    // MERGE (LDS kernel): the step's interior-node test and a restarted ray's root test share one
    // children_mask call at the end of the step
    constexpr bool MERGE = PAIR && PSL && !NST;
    // UL (quantised-node HBM scenes): one load round trip per step for the node-test and leaf-test
    // lanes together
    // (round 5: in the build without the shadow handoff -- long launches, C5 -- the merged round
    // trip costs more than it saves: C5 178.3 -> 176.8 ms without it, C4 +2% without it, so it stays
    // in the handoff build only)
    constexpr bool UL = !PAIR && HELP &&
                        std::is_same<std::remove_cv_t<std::remove_pointer_t<NodeP>>, XCNode>::value;
    bool desc = false, rs = false;   // MERGE: this step descends into xch / restarts at the root
    int xch = 0;
    uint64_t mlo = 0, mhi = 0;
    double tbest = INFINITY, tmax = INFINITY;
    float tbest_f = INFINITY;
    F3 of = f3(0, 0, 0), ivf = f3(1, 1, 1);
    // path: Lv = L while the closest ray is traced; across the shadow ray Lv / Lo hold the two
    // candidate sums L + T*lit (light visible) and L + T*dark (occluded), and T already holds the
    // next bounce's throughput (the oracle's operations, split around the shadow query)
    V3 Lv = v3(0, 0, 0), Lo = v3(0, 0, 0), T = v3(1, 1, 1);
    V3 nextd = v3(0, 0, 0);   // carried across the shadow ray (its origin = the shadow ray's)
    bool has_next = false;

    // fp64 primitive tests of one leaf's records hp[0 .. cntl) (these decide the result): global
    // records fetched one ahead of the test; LDS records (PAIR) two at a time, the two fp64
    // dependency chains interleaved.  A shadow ray (own or a helper's) stops at any hit.
    // leaf_test_from: global records, the first one already in registers (cur; UL below)
    auto leaf_test_from = [&](XHotR cur, const auto* hp, int cntl) {
        for (int j = 0; j < cntl; ++j) {
            const XHotR rec = cur;
            // long launches (no handoff build): no load after the leaf's last record (C5 182.3 ->
            // 180.2 ms); the handoff build keeps the unconditional one-ahead load (C4 +3% without)
            if (HELP || j + 1 < cntl) cur = load_hot(hp + min(j + 1, cntl - 1));
            ++nprim;
            const double t = x_prim_t<TRI>(rec.h, o, d, MX_TMIN);
            const int pi = rec.h.prim;
            if (phase != PH_CLOSEST) {
                if (t < tmax) { best = pi; raying = false; return; }   // any hit occludes
            } else {   // (selects, not branches: | and & do not short-circuit)
                const bool u = (t < tbest) | ((t == tbest) & (pi < best));
                tbest = u ? t : tbest;
                best = u ? pi : best;
                tbest_f = u ? up32(t) : tbest_f;
            }
        }
    };
    auto leaf_test = [&](const auto* hp, int cntl) {
        if constexpr (!PAIR) {
            leaf_test_from(load_hot(hp), hp, cntl);
        } else {
            for (int j = 0; j < cntl; j += 2) {
                const bool two = j + 1 < cntl;
                const XHotR r0 = load_hot(hp + j), r1 = load_hot(hp + (two ? j + 1 : j));
                const double ta = x_prim_t<TRI>(r0.h, o, d, MX_TMIN);
                const double tb = two ? x_prim_t<TRI>(r1.h, o, d, MX_TMIN) : INFINITY;
                nprim += two ? 2 : 1;
                if (phase != PH_CLOSEST) {
                    if ((ta < tmax) | (tb < tmax)) {   // any hit occludes
                        best = ta < tmax ? r0.h.prim : r1.h.prim;
                        raying = false;
                        return;
                    }
                } else {   // (selects, not branches)
                    const bool ua = (ta < tbest) | ((ta == tbest) & (r0.h.prim < best));
                    tbest = ua ? ta : tbest;
                    best = ua ? r0.h.prim : best;
                    const bool ub = (tb < tbest) | ((tb == tbest) & (r1.h.prim < best));
                    tbest = ub ? tb : tbest;
                    best = ub ? r1.h.prim : best;
                    tbest_f = up32(tbest);
                }
            }
        }
    };


    // PF (HBM-resident scenes): the next pop's child reference and leaf count are fetched at the
    // end of the step that sets up the level (descend, climb or ray start), so the pop itself waits
    // for no load: one dependent round trip per step (the child's node or leaf records) instead of
    // two.  (lvl mask, node) do not change between that fetch and the pop.
    constexpr bool PF = !PAIR;   // (LDS-resident scenes: a ds_read away; +3% with PF)
    int pf_ch = 0, pf_cnt = 0;
    auto prefetch = [&]() {
        const uint32_t m = lvl_get<SH>(mlo, mhi, level);
        if (m) {
            const int c = __builtin_ctz(m) ^ dmask;
            pf_ch = W[node].child[c];
            pf_cnt = W[node].cnt[c];
        }
    };

    const uint64_t t_begin = STATS ? clock64() : 0;
    for (;;) {
        if (HELP && any_gave && phase == PH_DEAD) {   // an idle lane given a shadow ray starts it
            const int ow = hp_.own[tid];
            if (ow >= 0) {
                hp_.own[tid] = -1;
                howner = ow & 0xFF;
                const double* r = hp_.ray + tid;
                o = v3(r[0], r[256], r[512]);
                d = v3(r[768], r[1024], r[1280]);
                of = f3((float)o.x, (float)o.y, (float)o.z);
                ivf = inv_dir(d);
                dmask = (d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0);
                level = 0;
                mlo = mhi = 0;
                // a shadow ray
                tmax = r[1536];
                tbest = tmax;
                tbest_f = up32(tmax);
                phase = PH_HELP;
                best = -1;
                const uint32_t rm = children_mask<PAIR>(W, of, ivf, tbest_f, dmask);
                node = 0;
                lvl_set<SH>(mlo, mhi, 0, rm);
                raying = rm != 0;
                if (PF && raying) prefetch();
            }
        }
        const unsigned long long m_live = __ballot(phase != PH_DEAD);
        if (m_live == 0) break;
        const unsigned long long m_idle = HELP ? ~m_live : 0ull;   // lanes free to take a shadow ray
        bool gave = false;
        const bool trav = raying;
        const unsigned long long m_trav = __ballot(trav);
        const int n_wait = __popcll(m_live & ~m_trav);
        const bool handle = phase != PH_DEAD && !trav &&
                            (8 * n_wait >= handle8 * __popcll(m_live) || m_trav == 0);
        if (STATS) {   // ballots over the whole wave, accumulated by lane 0
            const unsigned long long m_h = __ballot(handle);
            const unsigned long long m_hc = __ballot(handle && phase == PH_CLOSEST);
            const unsigned long long m_hs = __ballot(handle && phase == PH_SHADOW);
            if (lane == 0) {
                ++cnt.iters;
                if (m_h) {
                    ++cnt.handle;
                    cnt.hlanes += __popcll(m_h);
                    cnt.hclose += __popcll(m_hc);
                    cnt.hshadow += __popcll(m_hs);
                }
            }
        }
        const uint64_t t0 = STATS ? clock64() : 0;
        if (STATS) ++cnt.path_it;
        if (trav) {
            if (STATS) {
                ++nsteps;
                ++cnt.path_st;
            }
            // ---- one traversal step (stackless: 8-bit "children left" mask per level).  Invariant:
            // the current level has a child left; the step pops it, then climbs past exhausted
            // levels, so a ray ends in the step that exhausts the root level (no empty iteration).
            const auto* nd = W + node;
            const uint32_t msk = lvl_get<SH>(mlo, mhi, level);
            const int kc = __builtin_ctz(msk);         // next child in front-to-back order
            lvl_set<SH>(mlo, mhi, level, msk & (msk - 1));
            const int c = kc ^ dmask;
            const int ch = PF ? pf_ch : nd->child[c];
            xch = ch;
            desc = false;
            // a closer hit may have arrived since the mask was computed: re-cull this child -- in
            // the LDS kernel only: in HBM-resident scenes an interior child's own node test culls its
            // children against the same t, and skipping the re-cull drops a node-record fetch and ~60
            // instructions from the step (round 3: C5 214 -> 199 ms, C4 1.96 -> 1.82; leaves: their
            // fp64 tests run against the best t as it stands; the LDS kernel, whose re-cull is cheaper
            // than a node test, keeps it: C3 +0.9% without)
            bool keep = true;
            if (PAIR && phase == PH_CLOSEST && best >= 0) keep = child_hit(nd, c, of, ivf, tbest_f);
            if (STATS) {
                const unsigned long long mn = __ballot(keep && ch >= 0), ml = __ballot(keep && ch < 0);
                if (lane == 0) {
                    cnt.it_node += mn != 0;
                    cnt.ln_node += __popcll(mn);
                    cnt.it_leaf += ml != 0;
                    cnt.ln_leaf += __popcll(ml);
                }
            }
            if (UL) {   // (keep is always true in HBM-resident scenes: no re-cull)
                // one memory round trip for the wave's node-test AND leaf-test lanes: each lane's
                // load (the child's 64 slab bytes, or its leaf's first record) is issued before
                // either test waits, instead of a node-test block and a leaf-test block each
                // waiting on its own load
                XHotR ur;
                const int cntl = ch < 0 ? (PF ? pf_cnt : (int)nd->cnt[c]) : 0;
                if (ch < 0) {
                    ur = load_hot(H + ~ch);
                } else {
                    const int4* qb = reinterpret_cast<const int4*>(W + ch);
                    ur.q[0] = qb[0];
                    ur.q[1] = qb[1];
                    ur.q[2] = qb[2];
                    ur.q[3] = qb[3];
                }
                if (ch < 0) leaf_test_from(ur, H + ~ch, cntl);
                if (ch >= 0) {
                    ++nnode;
                    const uint32_t cm = children_mask_q(ur.q[0], ur.q[1], ur.q[2], ur.q[3], of, ivf, tbest_f, dmask);
                    if (cm) {
                        node = ch;
                        ++level;
                        lvl_set<SH>(mlo, mhi, level, cm);
                        if (NST) nst[level * 256] = ch;
                    }
                }
            } else if (keep) {
                if (ch < 0) {             // leaf: fp64 primitive tests (these decide the result)
                    leaf_test(H + ~ch, PF ? pf_cnt : (int)nd->cnt[c]);
                } else if (MERGE) {       // the node test runs below, shared with the restarts
                    desc = true;
                } else {                  // descend if any of the child's 8 children is hit (fp32)
                    ++nnode;
                    const uint32_t cm = children_mask<PAIR>(W + ch, of, ivf, tbest_f, dmask);
                    if (cm) {
                        node = ch;
                        ++level;
                        lvl_set<SH>(mlo, mhi, level, cm);
                        if (NST) nst[level * 256] = ch;
                    }
                }
            }
            if (raying && !desc) {        // climb to the nearest level with children left
                uint32_t rest = lvl_get<SH>(mlo, mhi, level);
                if constexpr (NST) {
                    if (rest == 0 && level > 0) {
                        // the deepest level below with children left, by one leading-zero count
                        const uint64_t lm = level >= 8 ? mlo : mlo & ((1ull << (8 * level)) - 1);
                        const uint64_t hm = level <= 8 ? 0ull : mhi & ((1ull << (8 * (level - 8))) - 1);
                        level = hm ? 8 + (63 - __clzll((long long)hm)) / 8 : lm ? (63 - __clzll((long long)lm)) / 8 : 0;
                        rest = lvl_get<SH>(mlo, mhi, level);
                        node = level == 0 ? 0 : nst[level * 256];
                    }
                } else {
                    while (rest == 0 && level > 0) {
                        --level;
                        node = level == 0 ? 0 : W[node].parent;   // the root is node 0: no load
                        rest = lvl_get<SH>(mlo, mhi, level);
                    }
                }
                if (rest == 0) raying = false;   // ray finished
            }
            if (PF && raying && !desc) prefetch();   // (MERGE: descending lanes below)
            // a finished shadow ray whose path continues: resolve it and start the next bounce
            // right here (the bounce direction was drawn when the hit was shaded), so the lane
            // keeps traversing instead of waiting for the shading handler (short-traversal scenes;
            // for long ones the extra divergent root test costs more than it saves)
            if (STATS) {
                const unsigned long long mr = __ballot(inline_shadow && !raying && phase == PH_SHADOW && has_next);
                if (lane == 0) {
                    cnt.it_rs += mr != 0;
                    cnt.ln_rs += __popcll(mr);
                }
            }
            if (inline_shadow && !raying && phase == PH_SHADOW && has_next) {
                ++nrays;
                if (best >= 0) Lv = PSL ? v3(pslot[0], pslot[1], pslot[2]) : Lo;   // occluded: ambient term only
                d = PSL ? v3(pslot[3], pslot[4], pslot[5]) : nextd;                // o is still the hit point
                ++b;
                phase = PH_CLOSEST;
                tmax = INFINITY;
                tbest = INFINITY;
                tbest_f = INFINITY;
                of = f3((float)o.x, (float)o.y, (float)o.z);
                ivf = inv_dir(d);
                dmask = (d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0);
                best = -1;
                if (MERGE) {         // the root test runs in the shared node test below
                    rs = true;
                } else {
                    const uint32_t rm = children_mask<PAIR>(W, of, ivf, tbest_f, dmask);
                    node = 0;
                    level = 0;
                    mlo = mhi = 0;
                    lvl_set<SH>(mlo, mhi, 0, rm);
                    raying = rm != 0;
                    if (PF && raying) prefetch();
                }
            }
            // MERGE: one node test per step for the lanes that descend into an interior child and
            // the lanes whose next bounce starts here (the root) -- one block instead of two
            if (MERGE && (desc || rs)) {
                if (desc) ++nnode;
                const uint32_t cm = children_mask<PAIR>(W + (rs ? 0 : xch), of, ivf, tbest_f, dmask);
                if (rs) {
                    node = 0;
                    level = 0;
                    mlo = mhi = 0;
                    lvl_set<SH>(mlo, mhi, 0, cm);
                    raying = cm != 0;
                } else if (cm) {
                    node = xch;
                    ++level;
                    lvl_set<SH>(mlo, mhi, level, cm);
                } else {   // the child's children all missed: climb as an unmerged step would have
                    uint32_t rest = lvl_get<SH>(mlo, mhi, level);
                    while (rest == 0 && level > 0) {
                        --level;
                        node = level == 0 ? 0 : W[node].parent;
                        rest = lvl_get<SH>(mlo, mhi, level);
                    }
                    // a ray that ends here waits for the handler (which continues a shadow ray's path)
                    if (rest == 0) raying = false;
                }
                if (PF && raying) prefetch();
                rs = false;
                desc = false;
            }
        }
        const uint64_t t1 = STATS ? clock64() : 0;
        uint64_t t2 = t1;
        if (HELP && handle && phase == PH_HELP) {   // a helper's answer to its owner; idle again
            ++nrays;
            hp_.res[wbase + howner] = best >= 0 ? 2 : 1;
            phase = PH_DEAD;
        }
        bool hold = false;   // an owner whose helper has not answered yet: no handling this time
        if (HELP) {
            __builtin_amdgcn_wave_barrier();
            if (handle && pend) {
                const int r = hp_.res[tid];
                if (r == 0) {
                    hold = true;
                } else {
                    if (r == 2) Lv = PSL ? v3(pslot[0], pslot[1], pslot[2]) : Lo;   // occluded: ambient only
                    hp_.res[tid] = 0;
                    pend = false;
                }
            }
        }
        if (handle && !hold && phase != PH_DEAD) {
            // ---- the lane's ray is finished: consume it, spawn the next one --------------------
            bool end_path = false;
            if (phase == PH_CLOSEST) {
                ++nrays;
                if (best < 0) {
                    end_path = true;
                } else {
                    const V3 din = d;   // the incoming direction
                    const V3 P = o + tbest * d;
                    const XPrim& p = XP[best];   // by reference: only used fields are loaded
                    const REnt& e = EN[p.ent];
                    V3 N = (TRI || p.kind == 0) ? ld3(p.n) : normalize(P - ld3(p.a));
                    if (!(dot(din, N) < 0)) N = -N;
                    int32_t tu, tv;
                    x_texcoord<TRI>(sc, e, P, tu, tv);
                    const V3 tc = texel(ld3(e.color), tu, tv);
                    const V3 lv = light - P;
                    const double ldist = gsqrt(dot(lv, lv));
                    const V3 Ld = normalize(lv);
                    const V3 la = tc * e.shader[0];
                    const V3 ldf = (smax(0.0, dot(N, Ld)) * (tc * 0.5)) * e.shader[1];
                    const V3 bis = normalize(normalize(-din) + Ld);
                    const double spw = mx_pow(smax(0.0, dot(N, bis)), e.spec_pow);
                    const V3 ls = v3(spw, spw, spw) * e.shader[2];
                    const V3 lo = (la + ldf) + ls;
                    if (PSL) T = v3(pslot[6], pslot[7], pslot[8]);
                    Lo = Lv + vmul(T, v3(smin(la.x, 1.0), smin(la.y, 1.0), smin(la.z, 1.0)));
                    if (PSL) { pslot[0] = Lo.x; pslot[1] = Lo.y; pslot[2] = Lo.z; }
                    Lv = Lv + vmul(T, v3(smin(lo.x, 1.0), smin(lo.y, 1.0), smin(lo.z, 1.0)));
                    has_next = false;
                    // mirror bounce with probability e.refl (uniform dim 4): T unchanged, d reflected
                    // about the facing normal; otherwise the diffuse bounce below
                    const bool mirror = b != depth - 1 && e.refl > 0.0 &&
                                        mx_u01k(PSL ? reinterpret_cast<const uint64_t*>(pslot)[9] : key, smp, b, 4) < e.refl;
                    if (mirror) {
                        nextd = normalize(din - N * (2.0 * dot(din, N)));
                        if (PSL) { pslot[3] = nextd.x; pslot[4] = nextd.y; pslot[5] = nextd.z; }
                        has_next = true;
                    } else if (b != depth - 1) {
                        const V3 Tn = vmul(T, tc * 0.5);
                        T = Tn;
                        if (PSL) { pslot[6] = Tn.x; pslot[7] = Tn.y; pslot[8] = Tn.z; }
                        if (!(Tn.x == 0.0 && Tn.y == 0.0 && Tn.z == 0.0)) {
                            double sx, sy, r2;   // cosine-weighted: concentric disk + Malley
                            const uint64_t kk = PSL ? reinterpret_cast<const uint64_t*>(pslot)[9] : key;
                            mx_disk(mx_u01k(kk, smp, b, 2), mx_u01k(kk, smp, b, 3), sx, sy, r2);
                            const double sz = gsqrt(1.0 - r2);
                            const double sg = N.z >= 0.0 ? 1.0 : -1.0;
                            const double aa = -1.0 / (sg + N.z);
                            const double bb = N.x * N.y * aa;
                            const V3 bt1 = v3(1.0 + sg * N.x * N.x * aa, sg * bb, -sg * N.x);
                            const V3 bt2 = v3(bb, sg + N.y * N.y * aa, -N.y);
                            nextd = normalize((bt1 * sx + bt2 * sy) + N * sz);
                            if (PSL) { pslot[3] = nextd.x; pslot[4] = nextd.y; pslot[5] = nextd.z; }
                            has_next = true;
                        }
                    }
                    // shadow ray toward the point light: handed to an idle lane of the wave when the
                    // path continues and one is free (the k-th giver takes the k-th idle lane), the
                    // lane then starts its next bounce at once; else traced here first
                    bool give = handoff && has_next;
                    if (HELP) {
                        const unsigned long long m_give = __ballot(give);
                        if (give) {
                            const unsigned r = (unsigned)__popcll(m_give & ((1ull << lane) - 1));
                            give = r < (unsigned)__popcll(m_idle);
                            if (give) {
                                const int ht = wbase + nth_set_bit(m_idle, r);
                                double* hr = hp_.ray + ht;
                                hr[0] = P.x; hr[256] = P.y; hr[512] = P.z;
                                hr[768] = Ld.x; hr[1024] = Ld.y; hr[1280] = Ld.z;
                                hr[1536] = ldist;
                                hp_.own[ht] = lane;
                                pend = true;
                                gave = true;
                                o = P;
                                d = PSL ? v3(pslot[3], pslot[4], pslot[5]) : nextd;
                                ++b;
                                phase = PH_CLOSEST;
                                tmax = INFINITY;
                                tbest = INFINITY;
                                tbest_f = INFINITY;
                            }
                        }
                    }
                    if (!give) {
                        phase = PH_SHADOW;
                        o = P;
                        d = Ld;
                        tmax = ldist;
                        tbest = ldist;
                        tbest_f = up32(ldist);
                    }
                }
            } else if (phase == PH_SHADOW) {
                ++nrays;
                if (best >= 0) Lv = PSL ? v3(pslot[0], pslot[1], pslot[2]) : Lo;   // occluded: ambient term only
                if (!has_next) {
                    end_path = true;
                } else {
                    d = PSL ? v3(pslot[3], pslot[4], pslot[5]) : nextd;   // o is still the hit point
                    ++b;
                    phase = PH_CLOSEST;
                    tmax = INFINITY;
                    tbest = INFINITY;
                    tbest_f = INFINITY;
                }
            }
            if (end_path) {
                if (STATS)
                    cnt.path_max = max(cnt.path_max, (((uint64_t)wall_clock64() - cnt.path_t0) << 32) |
                                                         ((uint64_t)min(cnt.path_it, 65535u) << 16) |
                                                         (uint64_t)min(cnt.path_st, 65535u));
                if (spp == 1) {   // the pixel: min((0 + L) / 1, 1), the reduce pass's operations
                    const double c0 = smin((0.0 + Lv.x) / 1.0, 1.0), c1 = smin((0.0 + Lv.y) / 1.0, 1.0),
                                 c2 = smin((0.0 + Lv.z) / 1.0, 1.0);
                    if (rgb) { rgb[3 * idx] = c0; rgb[3 * idx + 1] = c1; rgb[3 * idx + 2] = c2; }
                    if (rgb8) quantize(c0, c1, c2, rgb8 + 3 * idx);
                } else {   // the sample's radiance; k_x_reduce sums a pixel's samples in order
                    double* q = wk.part + 3 * ((size_t)idx * (size_t)spp + (size_t)smp);
                    q[0] = Lv.x; q[1] = Lv.y; q[2] = Lv.z;
                }
                ++smp;
                phase = (smp < wk.s1 && ((smp - wk.s0) & (k - 1)) != 0) ? PH_START : PH_DONEPX;
            }
            if (STATS) t2 = clock64();
            // ---- the lane's next ray.  A primary ray that misses every child box of the root
            // cannot hit anything: its sample adds exactly +0 to the pixel sums (the oracle traces
            // it and adds L = 0), so it is resolved here and the lane moves on to its next sample,
            // next pixel (fetched from the slot counter, one atomic per wave) -- up to
            // GI_X_START_BURST primary rays per lane per handler run.
            int burst = 0;
            for (;;) {
                if (STATS) {
                    const unsigned long long mb = __ballot(true);
                    if (lane == 0) {
                        cnt.it_st += 1;
                        cnt.ln_st += __popcll(mb);
                    }
                }
                if (phase == PH_DONEPX) phase = PH_NEED;   // unit complete (its samples are stored)
                const unsigned long long m_need = __ballot(phase == PH_NEED);
                if (m_need) {
                    // units of the wave's current block first, then of one new block (a refill asks
                    // for at most 64 units = one block).  The block's 64 list entries live in this
                    // wave's LDS row (the lanes that run the handler load them; the others may be
                    // traversing), so handing out a unit costs one ds_read.
                    const unsigned rank = (unsigned)__popcll(m_need & ((1ull << lane) - 1));
                    const unsigned n_need = (unsigned)__popcll(m_need);
                    const int leader = __ffsll((long long)m_need) - 1;
                    const unsigned used = blk_meta[0];
                    unsigned g = blk_meta[1], c = blk_meta[2];
                    const unsigned avail = 64u - used;
                    unsigned j = used + rank;
                    bool have = rank < avail;
                    unsigned ps = have ? blk_list[j] : 0u;
                    unsigned used_new = used + n_need;
                    if (n_need > avail) {                          // take the next block
                        // once the wave has seen the block counter run out (blk_meta[3]), no more atomics:
                        // each would be an L2 round trip for nothing (C4 spends ~90% of its loop
                        // iterations after that point, ending ~100 paths per wave)
                        unsigned nb = n_blocks;
                        if (blk_meta[3] == 0u) {
                            if (lane == leader) nb = atomicAdd(wk.blocks, 1u);
                            nb = __shfl(nb, leader);
                        }
                        used_new = 64u;
                        if (nb < n_blocks) {
                            // (pm: ng = the pixel's list index, nc = its block's first run)
                            const unsigned ng = pm ? nb / rpb : nb / runs, nc = pm ? (nb - ng * rpb) * 64u : nb - ng * runs;
                            const unsigned long long m_act = __ballot(true);
                            const unsigned ra = (unsigned)__popcll(m_act & ((1ull << lane) - 1));
                            const unsigned na = (unsigned)__popcll(m_act);
                            __builtin_amdgcn_wave_barrier();
                            const unsigned pm_ps = pm ? wk.list[ng] : 0u;
                            for (unsigned e = ra; e < 64u; e += na) {
                                if (pm) {
                                    blk_list[e] = nc + e < runs ? pm_ps : 0xFFFFFFFFu;
                                } else {
                                    const unsigned li = spread ? e * n_groups + ng : ng * 64u + e;
                                    blk_list[e] = li < n_list ? wk.list[li] : 0xFFFFFFFFu;
                                }
                            }
                            __builtin_amdgcn_wave_barrier();
                            used_new = n_need - avail;
                            if (lane == leader) { blk_meta[1] = ng; blk_meta[2] = nc; }
                            if (!have) {
                                j = rank - avail;
                                ps = blk_list[j];
                                c = nc;
                                g = ng;
                                have = true;
                            }
                        } else if (!have && phase == PH_NEED) {
                            phase = PH_DEAD;                        // no work left
                        }
                        if (nb >= n_blocks && lane == leader) blk_meta[3] = 1u;   // the frame's work is all handed out
                    }
                    if (lane == leader) blk_meta[0] = used_new;
                    __builtin_amdgcn_wave_barrier();
                    if (phase == PH_NEED && have) {
                        const unsigned i = pm ? g : spread ? j * n_groups + g : g * 64u + j;   // list index
                        const unsigned cu = pm ? c + j : c;        // the unit's run
                        if (ps != 0xFFFFFFFFu) {                   // else a padding unit: take another
                            slot_pixel(m, (long long)(ps >> 6), (int)(ps & 63), idx, x, y);
                            y += m.y0;
                            if (spp > 1) idx = (long long)i;        // per-sample radiance row
                            key = mx_key(seed, (uint64_t)y * (uint64_t)m.w + (uint64_t)x);
                            if (PSL) reinterpret_cast<uint64_t*>(pslot)[9] = key;
                            smp = wk.s0 + (int)cu * k;
                            phase = PH_START;
                            if (cu == 0) ++npx;
                        }
                    }
                }
                if (phase == PH_NEED) continue;   // got a padding unit: take another
                if (phase == PH_DEAD) break;
                if (phase == PH_START) {
                    double jx = 0.0, jy = 0.0;
                    if (spp > 1) {
                        const uint64_t kk = PSL ? reinterpret_cast<const uint64_t*>(pslot)[9] : key;
                        jx = mx_u01k(kk, smp, 0xFFFF, 0);
                        jy = mx_u01k(kk, smp, 0xFFFF, 1);
                    }
                    const V3 d0 = primary_dir(cam, (double)x + jx, (double)y + jy);
                    if (burst < GI_X_START_BURST) {
                        // conservative fp32 test of the scene's root box on the unnormalised
                        // direction (slab test is scale-invariant; the padding covers rounding)
                        const F3 iv0 = f3(__builtin_amdgcn_rcpf((float)d0.x), __builtin_amdgcn_rcpf((float)d0.y),
                                          __builtin_amdgcn_rcpf((float)d0.z));
                        if (!root_hit(sc, f3((float)cam.pos.x, (float)cam.pos.y, (float)cam.pos.z), iv0)) {
                            ++nrays;   // background sample: L = 0
                            ++nres;
                            if (spp > 1) {
                                double* q = wk.part + 3 * ((size_t)idx * (size_t)spp + (size_t)smp);
                                q[0] = 0.0; q[1] = 0.0; q[2] = 0.0;
                            } else {   // spp == 1: the pixel is 0
                                if (rgb) { rgb[3 * idx] = 0.0; rgb[3 * idx + 1] = 0.0; rgb[3 * idx + 2] = 0.0; }
                                if (rgb8) { rgb8[3 * idx] = 0; rgb8[3 * idx + 1] = 0; rgb8[3 * idx + 2] = 0; }
                            }
                            ++burst;
                            ++smp;
                            phase = (smp < wk.s1 && ((smp - wk.s0) & (k - 1)) != 0) ? PH_START : PH_DONEPX;
                            continue;
                        }
                    }
                    if (STATS) {
                        cnt.path_t0 = (uint64_t)wall_clock64();
                        cnt.path_it = 0;
                        cnt.path_st = 0;
                    }
                    o = cam.pos;
                    d = normalize(d0);
                    Lv = v3(0, 0, 0);
                    T = v3(1, 1, 1);
                    if (PSL) { pslot[6] = 1.0; pslot[7] = 1.0; pslot[8] = 1.0; }
                    b = 0;
                    tmax = INFINITY;
                    tbest = INFINITY;
                    tbest_f = INFINITY;
                }
                if (no_shadow && phase == PH_SHADOW) {   // unoccluded without a query
                    best = -1;
                    raying = false;
                    break;
                }
                // start traversing the lane's ray (fp32 reciprocal, 1 ulp: the culling error stays
                // far inside the 1e-5*extent box padding)
                of = f3((float)o.x, (float)o.y, (float)o.z);
                ivf = inv_dir(d);
                dmask = (d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0);
                const uint32_t rm = children_mask<PAIR>(W, of, ivf, tbest_f, dmask);
                if (phase == PH_START) phase = PH_CLOSEST;
                best = -1;
                node = 0;   // root wide node
                level = 0;
                mlo = mhi = 0;
                lvl_set<SH>(mlo, mhi, 0, rm);
                raying = rm != 0;   // no root child hit: finished (consumed by the next handler run)
                if (PF && raying) prefetch();
                break;
            }
        }
        if (HELP) any_gave = __ballot(gave) != 0;
        if (STATS) {
            const uint64_t t3 = clock64();
            cnt.cyc_trav += t1 - t0;
            cnt.cyc_hit += t2 - t1;
            cnt.cyc_next += t3 - t2;
        }
    }
    if (STATS) cnt.cyc_all += clock64() - t_begin;
    if (STATS) {   // lane traversal steps, summed over the wave into lane 0
        uint64_t ns = nsteps;
        for (int off = 32; off > 0; off >>= 1) ns += __shfl_xor(ns, off);
        cnt.trav += ns;
    }
    cnt.rays += nrays;
    cnt.nodes += nnode;
    cnt.prims += nprim;
    cnt.px += npx;
    cnt.res += nres;
}

// Persistent waves: the grid is sized to the resident capacity; every lane pulls pixel slots
// from one device counter (SURVEY §7 hard part 4: per-ray cost varies ~10x between background
// and scene pixels), so no lane idles behind a sibling, a workgroup or the grid tail.
// LDS: small scenes (sc.x_lds_bytes > 0) keep the whole traversal structure -- wide nodes and
// leaf records -- in LDS, copied once by each resident workgroup; every traversal load is then a
// ds_read instead of a vector-memory round trip.
// W4: 4 waves per SIMD (<= 128 VGPRs) for LDS-resident scenes whose shading is light (triangles
// without acos texture mapping: +7% on the Cornell box); scenes with spheres / cones / rectangles
// keep 3 (their heavier handler spills at 128 VGPRs: -45% on the main.cpp scene at 4).
// For HBM-resident scenes (!LDS) W4 selects the shadow-ray handoff build (XHelp): chosen
// per launch for small launches, whose frame time is their longest paths' latency (C4: 3.01 ->
// 2.64 ms, with spread work groups 2.40 ms); in long launches (C5) the handoff build's heavier code
// costs 8%, so they run without.
// CN (HBM-resident scenes): traverse the quantised nodes (DevScene::xcnodes) instead of XWNode.
// TR (HBM-resident scenes): the scene is triangle meshes of the 4-wave kinds only (DevScene::x_tri_only,
// e.g. the 100k soup): mode_x_wave's TRI specialisation
template <bool STATS, bool LDS, bool W4, bool CN, bool SH, bool TR = false>
__global__ __launch_bounds__(256, (LDS && W4) ? GI_X_MIN_WAVES_LDS : GI_X_MIN_WAVES) void k_mode_x(DevScene sc, CamDev cam, V3 light, TileMap m, int spp, int depth,
                                                 uint64_t seed, double* rgb, uint8_t* rgb8,
                                                 unsigned long long* stats, XWork wk, int handle8, int xflags) {
    XCounters c;
    __shared__ unsigned s_blk[kWavesPerBlock][68];   // per wave: current block's list entries + state
    unsigned* blk = s_blk[threadIdx.x >> 6];
    if (LDS) {
        extern __shared__ int4 lds_scene[];
        // traversal records and shading records (primitives, entities): the shading handler then
        // issues no global load, so its waits never include the lane's outstanding stores
        const int nw = sc.n_xwnodes * (int)(sizeof(XWNode) / sizeof(int4));
        const int nh = sc.n_xhot * (int)(sizeof(XHot) / sizeof(int4));
        const int np = sc.n_xprims * (int)(sizeof(XPrim) / sizeof(int4));
        const int ne = sc.n_ents * (int)(sizeof(REnt) / sizeof(int4));
        const int4* gw = reinterpret_cast<const int4*>(sc.xwnodes);
        const int4* gh = reinterpret_cast<const int4*>(sc.xhot);
        const int4* gp = reinterpret_cast<const int4*>(sc.xprims);
        const int4* ge = reinterpret_cast<const int4*>(sc.ents);
        for (int i = threadIdx.x; i < nw; i += blockDim.x) lds_scene[i] = gw[i];
        for (int i = threadIdx.x; i < nh; i += blockDim.x) lds_scene[nw + i] = gh[i];
        for (int i = threadIdx.x; i < np; i += blockDim.x) lds_scene[nw + nh + i] = gp[i];
        for (int i = threadIdx.x; i < ne; i += blockDim.x) lds_scene[nw + nh + np + i] = ge[i];
        __syncthreads();
        const XWNode* W = reinterpret_cast<const XWNode*>(lds_scene);
        const XHot* H = reinterpret_cast<const XHot*>(lds_scene + nw);
        const XPrim* XP = reinterpret_cast<const XPrim*>(lds_scene + nw + nh);
        const REnt* EN = reinterpret_cast<const REnt*>(lds_scene + nw + nh + np);
        // 4-wave kernel: path values used only by the shading handler and at the shadow ray's end
        // (occluded sum, next direction, throughput T, RNG key) live in a per-lane LDS slot after
        // the scene instead of in VGPRs / scratch
        double* pslot = reinterpret_cast<double*>(lds_scene + nw + nh + np + ne) + 10 * threadIdx.x;
        mode_x_wave<STATS, true, W4, false, false, SH, W4>(sc, W, H, XP, EN, pslot, nullptr, XHelp{},
                                                                        cam, light, m, spp, depth, seed, rgb, rgb8, blk,
                                                                        wk, handle8, xflags, c);
    } else {
        // dynamic LDS: the 16 levels x 256 lanes of node indices, then the handoff
        // slots (7 x 256 doubles, 2 x 256 ints)
        extern __shared__ int lds_nst[];
        XHelp hp;
        hp.ray = reinterpret_cast<double*>(lds_nst + 16 * 256);
        hp.own = reinterpret_cast<int*>(hp.ray + 7 * 256);
        hp.res = hp.own + 256;
        if constexpr (CN)   // quantised nodes (the default for large HBM-resident scenes)
            mode_x_wave<STATS, false, false, true, W4, SH, TR>(sc, sc.xcnodes, sc.xhot, sc.xprims,
                                                                            sc.ents, nullptr, lds_nst + threadIdx.x, hp,
                                                                            cam, light, m, spp, depth, seed, rgb, rgb8,
                                                                            blk, wk, handle8, xflags, c);
        else
            mode_x_wave<STATS, false, false, true, W4, SH, TR>(sc, sc.xwnodes, sc.xhot, sc.xprims,
                                                                            sc.ents, nullptr, lds_nst + threadIdx.x, hp,
                                                                            cam, light, m, spp, depth, seed, rgb, rgb8,
                                                                            blk, wk, handle8, xflags, c);
    }
    if (STATS) {
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(stats + GI_STAT_X_ITERS, (unsigned long long)c.iters);
            atomicAdd(stats + GI_STAT_X_TRAV, (unsigned long long)c.trav);
            atomicAdd(stats + GI_STAT_X_HANDLE, (unsigned long long)c.handle);
            atomicAdd(stats + GI_STAT_X_HLANES, (unsigned long long)c.hlanes);
            atomicAdd(stats + GI_STAT_X_HCLOSE, (unsigned long long)c.hclose);
            atomicAdd(stats + GI_STAT_X_HSHADOW, (unsigned long long)c.hshadow);
            atomicAdd(stats + GI_STAT_X_CYC_TRAV, (unsigned long long)c.cyc_trav);
            atomicAdd(stats + GI_STAT_X_CYC_HIT, (unsigned long long)c.cyc_hit);
            atomicAdd(stats + GI_STAT_X_CYC_NEXT, (unsigned long long)c.cyc_next);
            atomicAdd(stats + GI_STAT_X_CYC_ALL, (unsigned long long)c.cyc_all);
            atomicAdd(stats + GI_STAT_X_IT_NODE, (unsigned long long)c.it_node);
            atomicAdd(stats + GI_STAT_X_LN_NODE, (unsigned long long)c.ln_node);
            atomicAdd(stats + GI_STAT_X_IT_LEAF, (unsigned long long)c.it_leaf);
            atomicAdd(stats + GI_STAT_X_LN_LEAF, (unsigned long long)c.ln_leaf);
            atomicAdd(stats + GI_STAT_X_IT_RS, (unsigned long long)c.it_rs);
            atomicAdd(stats + GI_STAT_X_LN_RS, (unsigned long long)c.ln_rs);
            atomicAdd(stats + GI_STAT_X_IT_ST, (unsigned long long)c.it_st);
            atomicAdd(stats + GI_STAT_X_LN_ST, (unsigned long long)c.ln_st);
        }
        wave_add_stats(stats, c.rays, c.nodes, c.prims, c.px);
        uint64_t cr = c.res, pm = c.path_max;
        for (int off = 32; off > 0; off >>= 1) {
            cr += __shfl_xor(cr, off);
            pm = max(pm, (uint64_t)__shfl_xor(pm, off));
        }
        if ((threadIdx.x & 63) == 0) {
            atomicAdd(stats + GI_STAT_X_RESOLVED, (unsigned long long)cr);
            atomicMax(stats + GI_STAT_X_PATH_MAX, (unsigned long long)pm);
        }
    }
}

// Mode X pass 1: one thread per pixel slot (tile order; a wave = one 8x8 tile).  A pixel none of
// whose jittered primary rays can meet the scene's root box (conservative fp64 frustum test) is 0:
// every sample adds exactly +0, as in the oracle, which traces them.  Padding slots of a packed
// tile are zeroed.  The other pixels are appended to the work list: one atomic per 1024-thread
// workgroup (the waves' counts combined in LDS) -- one per wave on the single n_list counter
// serialised at L2: 49 us per frame for C2 and C3 alike.
// zero2: two words zeroed by the first thread (the wavefront forms' unit counters), saving a memset
// launch per frame.
constexpr int kClassifyBlock = 1024;
template <bool STATS>
__global__ __launch_bounds__(kClassifyBlock) void k_x_classify(DevScene sc, CamDev cam, TileMap m, int spp, double* rgb,
                                                     uint8_t* rgb8, unsigned* list, unsigned* n_list,
                                                     unsigned long long* stats, unsigned* zero2) {
    if (zero2 && blockIdx.x == 0 && threadIdx.x < 2) zero2[threadIdx.x] = 0u;
    const long long s = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const long long lt = s >> 6;
    const int lane = threadIdx.x & 63;
    long long idx = -1;
    int x = 0, y = 0;
    bool scene = false, zero = false, bg = false;
    if (lt < m.n_local) {
        if (slot_pixel(m, lt, lane, idx, x, y)) {
            bg = pixel_misses_box(cam, x, y + m.y0, sc.root_lo, sc.root_hi);
            scene = !bg;
            zero = bg;
        } else {
            zero = idx >= 0 && m.shard_count > 1;   // padding slot of a packed tile
        }
    }
    if (zero) {
        if (rgb) { rgb[3 * idx] = 0; rgb[3 * idx + 1] = 0; rgb[3 * idx + 2] = 0; }
        if (rgb8) { rgb8[3 * idx] = 0; rgb8[3 * idx + 1] = 0; rgb8[3 * idx + 2] = 0; }
    }
    const unsigned long long ms = __ballot(scene && list != nullptr);   // (a progressive pass after the
    __shared__ unsigned s_cnt[kClassifyBlock / 64 + 1];                  //  first keeps the frame's list)
    const int wv = threadIdx.x >> 6;
    if (lane == 0) s_cnt[wv] = (unsigned)__popcll(ms);
    __syncthreads();
    if (threadIdx.x == 0) {   // exclusive offsets of the waves, then one atomic for the workgroup
        unsigned acc = 0;
        for (int k = 0; k < kClassifyBlock / 64; ++k) {
            const unsigned c = s_cnt[k];
            s_cnt[k] = acc;
            acc += c;
        }
        s_cnt[kClassifyBlock / 64] = acc ? atomicAdd(n_list, acc) : 0u;   // (acc > 0 only with a list)
    }
    __syncthreads();
    if (scene && list) list[s_cnt[kClassifyBlock / 64] + s_cnt[wv] + (unsigned)__popcll(ms & ((1ull << lane) - 1))] = (unsigned)s;
    if (STATS && (s & ~63ll) < m.n_local * 64) {
        wave_add_stats(stats, bg ? (uint64_t)spp : 0, 0, 0, bg ? 1 : 0);
        uint64_t r = bg ? (uint64_t)spp : 0;   // samples resolved here, without traversal
        for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off);
        if (lane == 0 && r) atomicAdd(stats + GI_STAT_X_RESOLVED, (unsigned long long)r);
    }
}

// Mode X pass 3 (spp > 1): a listed pixel's per-sample radiance added in sample order from +0, then
// min(sum / spp, 1) and the 8-bit store -- the oracle's operations (pixel_mode_x).  A progressive
// pass sums its frame's samples [0, s1): the frame of spp = s1, the one-shot frame for s1 = spp.
__global__ __launch_bounds__(256) void k_x_reduce(TileMap m, XWork wk, int spp, double* rgb, uint8_t* rgb8) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= *wk.n_list) return;
    const unsigned ps = wk.list[i];
    long long idx = -1;
    int x = 0, y = 0;
    slot_pixel(m, (long long)(ps >> 6), (int)(ps & 63), idx, x, y);
    double a = 0, b = 0, c = 0;
    const double* p = wk.part + 3 * (size_t)i * (size_t)spp;
    int s = 0;
    if ((spp & 1) == 0) {
        // even spp: the row is 16-byte aligned, so two samples (six doubles) come in three 16-byte
        // loads -- half the load instructions; the lanes' rows are 1.5 KB apart, so each load
        // instruction is 64 separate lines for the address unit, which bounds this kernel.  The
        // sums take the samples in the same order.
        const double2* q = reinterpret_cast<const double2*>(p);
        for (; s + 1 < wk.s1; s += 2) {
            const double2 v0 = q[3 * (s >> 1)], v1 = q[3 * (s >> 1) + 1], v2 = q[3 * (s >> 1) + 2];
            a = a + v0.x;
            b = b + v0.y;
            c = c + v1.x;
            a = a + v1.y;
            b = b + v2.x;
            c = c + v2.y;
        }
    }
    for (; s < wk.s1; ++s) {
        a = a + p[3 * s];
        b = b + p[3 * s + 1];
        c = c + p[3 * s + 2];
    }
    const double n = (double)wk.s1;
    const double c0 = smin(a / n, 1.0), c1 = smin(b / n, 1.0), c2 = smin(c / n, 1.0);
    if (rgb) { rgb[3 * idx] = c0; rgb[3 * idx + 1] = c1; rgb[3 * idx + 2] = c2; }
    if (rgb8) quantize(c0, c1, c2, rgb8 + 3 * idx);
}

// ---------------------------------------------------------------------------------------------
// unshard: packed per-rank tiles -> row-major frame
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_unshard(TileMap m, const double* packed, const uint8_t* packed8, double* rgb,
                                                  uint8_t* rgb8) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;   // global pixel slot in tile order
    const long long t = i / (kTile * kTile);
    if (t >= m.n_tiles) return;
    const int lane = (int)(i % (kTile * kTile));
    const int ty = (int)(t / m.tiles_x), tx = (int)(t % m.tiles_x);
    const int x = tx * kTile + (lane & 7), y = ty * kTile + (lane >> 3);
    if (x >= m.w || y >= m.h) return;
    const long long r = t % m.shard_count, lt = t / m.shard_count;
    const long long src = (r * m.n_local + lt) * (kTile * kTile) + lane;
    const long long dst = (long long)y * m.w + x;
    if (rgb) { rgb[3 * dst] = packed[3 * src]; rgb[3 * dst + 1] = packed[3 * src + 1]; rgb[3 * dst + 2] = packed[3 * src + 2]; }
    if (rgb8) { rgb8[3 * dst] = packed8[3 * src]; rgb8[3 * dst + 1] = packed8[3 * src + 1]; rgb8[3 * dst + 2] = packed8[3 * src + 2]; }
}

__global__ __launch_bounds__(256) void k_box_kat(int n, const double* recs, int32_t* out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double* q = recs + 12 * (size_t)i;
    out[i] = box_hit(v3(q[0], q[1], q[2]), v3(q[3], q[4], q[5]), v3(q[6], q[7], q[8]),
                     normalize(v3(q[9], q[10], q[11]))) ? 1 : 0;
}

__global__ __launch_bounds__(64) void k_trace_ray(DevScene sc, V3 o, V3 d, V3 light, int32_t* out_i, double* out_d) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    RResult r;
    uint32_t nn = 0, np = 0;
    const double reach = fmax(fabs(o.x), fmax(fabs(o.y), fabs(o.z))) + (double)sc.rc_ext;
    trace_mode_r_cand(sc, o, d, (float)(1e-5 * reach + 1e-30), r, nn, np);
    out_i[0] = r.ent;
    out_i[1] = out_i[2] = 0;
    for (int k = 0; k < 9; ++k) out_d[k] = 0;
    if (r.ent >= 0) {
        const REnt e = sc.ents[r.ent];
        int32_t u, v;
        tex_coord(sc, e, r.P, u, v);
        const V3 col = shade_ref(e, d, light, r.P, r.N, u, v);
        out_i[1] = u; out_i[2] = v;
        out_d[0] = r.P.x; out_d[1] = r.P.y; out_d[2] = r.P.z;
        out_d[3] = r.N.x; out_d[4] = r.N.y; out_d[5] = r.N.z;
        out_d[6] = col.x; out_d[7] = col.y; out_d[8] = col.z;
    }
}


}  // namespace

long long shard_tiles(int w, int h, int shard_count) { return make_map(w, h, shard_count, 0).n_local; }

// Read once per process from the environment (thread-safe; several host threads may each drive their
// own device and scene).  One user knob: GI_X_MAX_RUN, the largest Mode X work-unit run length (scenes
// of cheap background samples such as the main.cpp scene prefer 8).  The rest are TEST hooks that pick
// among kernels whose frames are identical bit for bit (tests/test_gpu_parity.py compares them):
// GI_X_WF (0/1/2: force a Mode X form for a whole suite run), GI_X_HELP=0 (no shadow-ray handoff),
// GI_R_FLAT (0/1/2: force a Mode R kernel), GI_RF_PER_SLOT (the flat Mode R pool size: 0 forces the
// per-tile overflow path), GI_RF_GROUP (1/4: force k_rf_reach's lanes per hit).
struct XEnv {
    int run_log2 = 0, help = 1, wf = -1;
    int r_flat = -1;                  // Mode R kernels (GI_R_FLAT): 1 the flat phases for every scene, 0 k_mode_r
                                      // for every scene, 2 k_mode_r_batch for the whole frame (tests); -1 by size
    int rf_per_slot = 16;             // flat Mode R: pool pairs per pixel slot of the frame (GI_RF_PER_SLOT)
    int rf_group = 0;                 // k_rf_reach lanes per hit (GI_RF_GROUP): 0 by the launch's hits, 1 or 4 (tests)
};
const XEnv& x_env() {
    static XEnv env;
    static std::once_flag once;
    std::call_once(once, [] {
        if (const char* v = std::getenv("GI_X_HELP")) env.help = std::atoi(v) != 0;
        if (const char* v = std::getenv("GI_R_FLAT")) env.r_flat = std::atoi(v);
        if (const char* v = std::getenv("GI_RF_PER_SLOT")) env.rf_per_slot = std::max(0, std::min(1024, std::atoi(v)));
        if (const char* v = std::getenv("GI_X_WF")) env.wf = std::atoi(v);
        if (const char* v = std::getenv("GI_RF_GROUP")) env.rf_group = (std::atoi(v) == 1 || std::atoi(v) == 4) ? std::atoi(v) : 0;
        const char* v = std::getenv("GI_X_MAX_RUN");
        const int r = v ? std::max(1, std::min(128, std::atoi(v))) : GI_X_MAX_RUN;
        int lg = 0;
        while ((2 << lg) <= r) ++lg;
        env.run_log2 = lg;
    });
    return env;
}

// wavefront Mode X (gi_wf.hip)
hipError_t launch_wf(const DevScene& sc, int kv, size_t lds_bytes, int resident, int form, const CamDev& cam, V3 light,
                     int w, int h, int y0, const gi_opts& o, double* rgb, uint8_t* rgb8, const XScratch& xs,
                     const unsigned* n_list_dev, unsigned long long* stats, int xflags, hipStream_t stream,
                     hipEvent_t ev_begin, hipEvent_t ev_end);
hipError_t wf_occupancy(const DevScene& sc, int kv, size_t lds_bytes, int form, int* per_cu);
size_t wf_slot_bytes();
size_t wf_scene_lds_bytes(const DevScene& sc);

#ifndef GI_WF_MAX_DEPTH
#define GI_WF_MAX_DEPTH 64   // the wavefront form launches once per bounce: deeper paths run k_mode_x
#endif
// Mode X form of a launch: 0 the persistent path-state kernel (k_mode_x), 1 the wavefront form
// (k_wf_bounce once per bounce over compacted queues), 2 the segment-synchronous form (k_seg).
// GI_FLAG_X_MEGA / _WF / _SEG force one (tests, A/B), then GI_X_WF=0/1/2.  By default (DESIGN.md §5,
// round-4 A/B): scenes staged in LDS run k_seg (C3 5.8 -> 5.2 ms, C2 0.29 -> 0.15-0.17 ms; short
// traversals, so a wave's lanes finish a segment together); large HBM-resident scenes keep
// k_mode_x, whose lanes refill independently (C4: k_seg 3.2 against 1.7 ms -- one long traversal
// would hold its whole wave).  The wavefront form loses everywhere (queue traffic and its
// atomics: C3 12.5-20 ms); it stays selectable.
int x_form_choice(const DevScene& sc, const XLaunchCfg& xc, const gi_opts& o) {
    if (o.mode != GI_MODE_X || (o.flags & GI_FLAG_X_MEGA)) return 0;
    if (o.flags & GI_FLAG_X_SEG) return 2;
    if (o.flags & GI_FLAG_X_WF) return o.depth <= GI_WF_MAX_DEPTH ? 1 : 0;
    const XEnv& env = x_env();
    if (env.wf >= 0) return env.wf == 1 ? (o.depth <= GI_WF_MAX_DEPTH ? 1 : 0) : env.wf == 2 ? 2 : 0;
    // small HBM-resident trees (<= 1 MB of wide nodes: L2-resident, short traversals -- X-zoo 5.7 ->
    // 4.8-5.0 ms, the 1k soup even) run k_seg too
    return (xc.kv >= 2 || (size_t)sc.n_xwnodes * sizeof(XWNode) <= ((size_t)1 << 20)) ? 2 : 0;
}
long long x_wf_chunk() { return 8ll << 20; }   // wavefront Mode X: units (pixel samples) per chunk = queue capacity
int x_env_rf_per_slot() { return x_env().rf_per_slot; }
unsigned rf_own_pairs() { return GI_RF_S0; }
unsigned rf_page_pairs() { return GI_RF_PAGE; }
unsigned rf_max_pages() { return GI_RF_KMAX; }
unsigned rf_seg_pairs() { return GI_RF_SEG; }
// Mode R kernel of a launch: 0 k_mode_r (one lane per pixel; small scenes, the reverse-DFS flag, an
// octree that never split), 1 the flat phases (scenes of more than 4096 entities; their overflowed
// tiles through k_mode_r_batch), 2 k_mode_r_batch for the whole frame (GI_R_FLAT=2, tests; and
// scenes of 2^26 entities or more, beyond the flat phases' one-word pairs)
int r_kernel_choice(const DevScene& sc, const gi_opts& o) {
    if (o.mode != GI_MODE_R || (o.flags & GI_FLAG_R_DFS) || sc.n_rnodes <= 1) return 0;
    const XEnv& env = x_env();
    const bool large = env.r_flat >= 0 ? env.r_flat != 0 : sc.n_ents > 4096;
    if (!large) return 0;
    return (env.r_flat == 2 || (unsigned)sc.n_ents > kRfEntMask) ? 2 : 1;
}

hipError_t x_launch_config(const DevScene& sc, int device, XLaunchCfg& cfg) {
    const bool lds = sc.x_lds_bytes > 0;
    cfg.lds_bytes = lds ? (size_t)sc.x_lds_bytes + (sc.x_waves4 ? 256 * 10 * sizeof(double) : 0)
                        : 16 * 256 * sizeof(int) + 256 * (7 * sizeof(double) + 2 * sizeof(int));
    cfg.kv = 2 * (int)lds + ((lds && sc.x_waves4) ? 1 : 0);   // 0 / 1 (per launch, HELP): HBM-resident
    int cus = 0, per_cu = 0;
    hipError_t e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device);
    if (e != hipSuccess) return e;
    e = hipOccupancyMaxActiveBlocksPerMultiprocessor(
        &per_cu, cfg.kv == 3 ? reinterpret_cast<const void*>(k_mode_x<false, true, true, false, false>)
                 : cfg.kv == 2 ? reinterpret_cast<const void*>(k_mode_x<false, true, false, false, false>)
                 : sc.xcnodes  ? (sc.x_tri_only ? reinterpret_cast<const void*>(k_mode_x<false, false, false, true, false, true>)
                                                : reinterpret_cast<const void*>(k_mode_x<false, false, false, true, false>))
                 : sc.x_tri_only ? reinterpret_cast<const void*>(k_mode_x<false, false, false, false, false, true>)
                               : reinterpret_cast<const void*>(k_mode_x<false, false, false, false, false>),
        64 * kWavesPerBlock, cfg.lds_bytes);
    if (e != hipSuccess) return e;
    cfg.resident = std::max(1, cus) * std::max(1, per_cu);
    cfg.wf_lds_bytes = (lds ? wf_scene_lds_bytes(sc) : 16 * 256 * sizeof(int)) + wf_slot_bytes();
    e = wf_occupancy(sc, cfg.kv, cfg.wf_lds_bytes, 1, &per_cu);
    if (e != hipSuccess) return e;
    cfg.wf_resident = std::max(1, cus) * std::max(1, per_cu);
    e = wf_occupancy(sc, cfg.kv, cfg.wf_lds_bytes, 2, &per_cu);
    if (e != hipSuccess) return e;
    cfg.seg_resident = std::max(1, cus) * std::max(1, per_cu);
    return hipSuccess;
}

hipError_t launch_render(const DevScene& sc, const XLaunchCfg& xc, const CamDev& cam, V3 light, int w, int h, int y0,
                         const gi_opts& o, double* rgb, uint8_t* rgb8, const XScratch& xs, KTimer* kt,
                         hipStream_t stream) {
    // GI_FLAG_TIME: events on the launch stream around the dominant kernel only (slot chosen by
    // the caller, gi_capi.cpp, which folds a reused pair before this call)
    const bool timed = (o.flags & GI_FLAG_TIME) && kt && kt->ev0[0];
    const int slot = timed ? (int)(kt->recorded % KTimer::kRing) : 0;
    hipEvent_t ev_begin = timed ? static_cast<hipEvent_t>(kt->ev0[slot]) : nullptr;
    hipEvent_t ev_end = timed ? static_cast<hipEvent_t>(kt->ev1[slot]) : nullptr;
    auto mark = [&](hipEvent_t ev) { if (timed) (void)hipEventRecord(ev, stream); };
    const TileMap m = make_map(w, h, o.shard_count, o.shard_index, y0);
    if (m.n_local == 0) return hipSuccess;
    const dim3 grid((unsigned)((m.n_local + kWavesPerBlock - 1) / kWavesPerBlock)), block(64 * kWavesPerBlock);
    unsigned long long* st = reinterpret_cast<unsigned long long*>(o.stats);
    const bool stats = (o.flags & GI_FLAG_STATS) && st;
    if (o.mode == GI_MODE_R) {
        // line-BVH widening: the prefilter's 1e-12|oc|^2 slack (<= 1e-6 |oc|) and fp32 slab rounding
        const double reach = std::max(std::fabs(cam.pos.x), std::max(std::fabs(cam.pos.y), std::fabs(cam.pos.z))) + (double)sc.rc_ext;
        const float tau = (float)(1e-5 * reach + 1e-30);
        // an octree that never split is one leaf: its list scanned backwards (first success) is
        // already the least work
        const int dfs = ((o.flags & GI_FLAG_R_DFS) || sc.n_rnodes <= 1) ? 1 : 0;
        const int rk = r_kernel_choice(sc, o);
        const bool tri = sc.r_tri_only != 0;   // ImpTriangle-only scenes: the other entity kinds' code dropped
        mark(ev_begin);
        if (rk == 1 && xs.rf_pairs && xs.rf_slots >= m.n_local * (kTile * kTile)) {   // flat phases
            const RFlat f{xs.rf_pairs, xs.rf_pairs + (size_t)(xs.rf_slots / 64) * GI_RF_S0, xs.rf_pt, xs.rf_best, xs.rf_cnt,
                          xs.rf_ovf, xs.rf_rcnt, xs.rf_soff, xs.rf_shc, xs.rf_sreg, xs.rf_hoff, xs.rf_dir, xs.rf_pages};
            const dim3 pgrid((unsigned)((m.n_local * (kTile * kTile) + 255) / 256)), fgrid(4096);
            hipError_t e1 = hipMemsetAsync(xs.rf_cnt, 0, 2 * sizeof(unsigned), stream);
            if (e1 != hipSuccess) return e1;
            // the overflowed tiles' fallback: half a tile per workgroup item, a grid that returns at once
            // when the list is empty
            const dim3 bgrid((unsigned)std::min<long long>(2 * m.n_local, 2048));
            const dim3 hgrid(16384);   // k_rf_hit: persistent waves (one per workgroup) over the segments
            const int rgroup = x_env().rf_group;
            if (stats) hipLaunchKernelGGL(k_rf_walk<true>, pgrid, block, 0, stream, sc, cam, m, tau, f, st);
            else hipLaunchKernelGGL(k_rf_walk<false>, pgrid, block, 0, stream, sc, cam, m, tau, f, st);
#define GI_LAUNCH_RF(S, T)                                                                                                \
    do {                                                                                                                  \
        hipLaunchKernelGGL(k_rf_scan, dim3(1), dim3(1024), 0, stream, f.rcnt, f.soff, nullptr, m.n_local, GI_RF_SEG);    \
        hipLaunchKernelGGL((k_rf_hit<S, T>), hgrid, dim3(64), 0, stream, sc, cam, m, f, st);                              \
        hipLaunchKernelGGL(k_rf_scan, dim3(1), dim3(1024), 0, stream, f.shc, f.hoff, f.soff + m.n_local, 0ll, 1u);       \
        hipLaunchKernelGGL(k_rf_reach<S>, dim3(4 * fgrid.x), dim3(64), 0, stream, sc, cam, m, f, st, rgroup);              \
        hipLaunchKernelGGL((k_rf_shade<S, T>), pgrid, block, 0, stream, sc, cam, light, m, rgb, rgb8, f, st);             \
        hipLaunchKernelGGL((k_mode_r_batch<S, T>), bgrid, block, 0, stream, sc, cam, light, m, rgb, rgb8, st, tau,        \
                           (const unsigned*)xs.rf_ovf, (const unsigned*)(xs.rf_cnt + 1));                                 \
    } while (0)
            if (stats) { if (tri) GI_LAUNCH_RF(true, true); else GI_LAUNCH_RF(true, false); }
            else { if (tri) GI_LAUNCH_RF(false, true); else GI_LAUNCH_RF(false, false); }
#undef GI_LAUNCH_RF
        } else if (rk) {   // k_mode_r_batch over the whole frame
            const dim3 sgrid((unsigned)((m.n_local * (kTile * kTile) + 31) / 32));
            if (stats) { if (tri) hipLaunchKernelGGL((k_mode_r_batch<true, true>), sgrid, block, 0, stream, sc, cam, light, m, rgb, rgb8, st, tau, nullptr, nullptr);
                         else hipLaunchKernelGGL((k_mode_r_batch<true, false>), sgrid, block, 0, stream, sc, cam, light, m, rgb, rgb8, st, tau, nullptr, nullptr); }
            else { if (tri) hipLaunchKernelGGL((k_mode_r_batch<false, true>), sgrid, block, 0, stream, sc, cam, light, m, rgb, rgb8, st, tau, nullptr, nullptr);
                   else hipLaunchKernelGGL((k_mode_r_batch<false, false>), sgrid, block, 0, stream, sc, cam, light, m, rgb, rgb8, st, tau, nullptr, nullptr); }
        } else if (stats) {
            hipLaunchKernelGGL(k_mode_r<true>, grid, block, 0, stream, sc, cam, light, m, rgb, rgb8, st, tau, dfs);
        } else {
            hipLaunchKernelGGL(k_mode_r<false>, grid, block, 0, stream, sc, cam, light, m, rgb, rgb8, st, tau, dfs);
        }
        mark(ev_end);
    } else {
        // persistent grid: as many 4-wave blocks as can be resident (xc, per scene), each wave pulls
        // blocks of work units
        const XEnv& env = x_env();
        const long long n_slots = m.n_local * (kTile * kTile);
        // HBM-resident scenes: the shadow-ray handoff build (and spread work groups) for launches of
        // at most 32 samples per resident lane -- their time is the longest paths' latency and lanes
        // run out of work early (C4: 10 per lane; X-soup1000, 169 per lane, is throughput-bound and
        // 25% slower spread)
        const bool help = xc.kv == 0 && env.help &&
                          n_slots * (long long)o.spp <= 32ll * 256ll * (long long)xc.resident;
        const int kv = xc.kv + (help ? 1 : 0);
        const size_t lds_bytes = xc.lds_bytes;
        // up to one lane per (pixel slot, sample): single-sample units can occupy that many lanes
        const long long want = (n_slots * (long long)o.spp / 64 + kWavesPerBlock - 1) / kWavesPerBlock;
        const dim3 pgrid((unsigned)std::max<long long>(1, std::min<long long>(want, xc.resident)));
        if (!xs.list || (unsigned long long)xs.cap < (unsigned long long)n_slots || (o.spp > 1 && (!xs.part || xs.spp < o.spp)))
            return hipErrorInvalidValue;
        // the launch's samples: the whole spp, or a progressive pass [sample_begin, sample_end) -- a pass
        // after the first continues the frame: its work list (and count, work[1]) and the earlier
        // passes' per-sample rows stay; classify only rewrites the background pixels
        const int s0 = o.sample_end > 0 ? o.sample_begin : 0, s1 = o.sample_end > 0 ? o.sample_end : o.spp;
        const bool cont = s0 > 0;
        hipError_t e = hipMemsetAsync(sc.work, 0, (cont ? 1 : 16) * sizeof(unsigned), stream);
        if (e == hipSuccess && cont) e = hipMemsetAsync(sc.work + 2, 0, 14 * sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
        XWork wk;
        wk.list = xs.list;
        wk.n_list = sc.work + 1;
        wk.part = xs.part;
        wk.blocks = sc.work;
        wk.s0 = s0;
        wk.s1 = s1;
        const dim3 sgrid((unsigned)((n_slots + 255) / 256));
        const dim3 cgrid((unsigned)((n_slots + kClassifyBlock - 1) / kClassifyBlock));
        const int form = x_form_choice(sc, xc, o);
        unsigned* zero2 = form == 2 ? xs.wcnt : nullptr;   // k_seg's unit counter, zeroed by the classify pass
        unsigned* cl = cont ? nullptr : xs.list;
        if (stats) hipLaunchKernelGGL(k_x_classify<true>, cgrid, dim3(kClassifyBlock), 0, stream, sc, cam, m, s1 - s0, rgb, rgb8, cl, sc.work + 1, st, zero2);
        else hipLaunchKernelGGL(k_x_classify<false>, cgrid, dim3(kClassifyBlock), 0, stream, sc, cam, m, s1 - s0, rgb, rgb8, cl, sc.work + 1, st, zero2);
        // shading-handler threshold (eighths of the live lanes that must wait): the builder's
        // estimate for the scene (DevScene::x_handle8)
        const int h8 = sc.x_handle8;
        // schedule flags (bit 0: inline shadow, bit 2: no shadow rays, bit 3: shadow handoff, bit 4:
        // spread work groups -- with the handoff build, bit 5: pixel-major work blocks) and the
        // maximum run length (log2, bits 8-10)
        const int xf = sc.x_flags | (env.run_log2 << 8) | ((o.flags & GI_FLAG_X_NO_SHADOW) ? 4 : 0) | (env.help ? 8 : 0) |
                       (help ? 16 : 0) | 32;
        if (form) {   // gi_wf.hip's forms, timed as one pass
            if (!xs.wcnt || (form == 1 && (!xs.wq[0] || !xs.wq[1] || xs.wcap <= 0))) return hipErrorInvalidValue;
            e = launch_wf(sc, xc.kv, xc.wf_lds_bytes, form == 2 ? xc.seg_resident : xc.wf_resident, form, cam, light, w, h, y0,
                          o, rgb, rgb8, xs, sc.work + 1, stats ? st : nullptr, xf, stream, ev_begin, ev_end);
            if (e != hipSuccess) return e;
            if (o.spp > 1) hipLaunchKernelGGL(k_x_reduce, sgrid, dim3(256), 0, stream, m, wk, o.spp, rgb, rgb8);
            if (timed) kt->recorded++;
            return hipGetLastError();
        }
        const bool cn = kv < 2 && sc.xcnodes != nullptr;
#define GI_LAUNCH_X2(S, L, W, SH, TR) hipLaunchKernelGGL((k_mode_x<S, L, W, false, SH, TR>), pgrid, block, lds_bytes, stream, sc, cam, light, m, o.spp, \
                                           o.depth, o.seed, rgb, rgb8, st, wk, h8, xf)
#define GI_LAUNCH_XC2(S, W, SH, TR) hipLaunchKernelGGL((k_mode_x<S, false, W, true, SH, TR>), pgrid, block, lds_bytes, stream, sc, cam, light, m, \
                                          o.spp, o.depth, o.seed, rgb, rgb8, st, wk, h8, xf)
        // TR: triangle-only HBM-resident scenes (the LDS kernels do not use it: theirs is W4)
#define GI_LAUNCH_X1(S, L, W, SH) do { if (!(L) && sc.x_tri_only) GI_LAUNCH_X2(S, L, W, SH, true); else GI_LAUNCH_X2(S, L, W, SH, false); } while (0)
#define GI_LAUNCH_XC1(S, W, SH) do { if (sc.x_tri_only) GI_LAUNCH_XC2(S, W, SH, true); else GI_LAUNCH_XC2(S, W, SH, false); } while (0)
        // SH: the per-level masks in one 64-bit word when the tree has at most 8 levels
        const bool sh = sc.x_max_depth <= 7;
#define GI_LAUNCH_X(S, L, W) do { if (sh) GI_LAUNCH_X1(S, L, W, true); else GI_LAUNCH_X1(S, L, W, false); } while (0)
#define GI_LAUNCH_XC(S, W) do { if (sh) GI_LAUNCH_XC1(S, W, true); else GI_LAUNCH_XC1(S, W, false); } while (0)
        mark(ev_begin);
        if (stats) {
            if (kv == 3) GI_LAUNCH_X(true, true, true); else if (kv == 2) GI_LAUNCH_X(true, true, false);
            else if (cn) { if (kv == 1) GI_LAUNCH_XC(true, true); else GI_LAUNCH_XC(true, false); }
            else if (kv == 1) GI_LAUNCH_X(true, false, true); else GI_LAUNCH_X(true, false, false);
        } else {
            if (kv == 3) GI_LAUNCH_X(false, true, true); else if (kv == 2) GI_LAUNCH_X(false, true, false);
            else if (cn) { if (kv == 1) GI_LAUNCH_XC(false, true); else GI_LAUNCH_XC(false, false); }
            else if (kv == 1) GI_LAUNCH_X(false, false, true); else GI_LAUNCH_X(false, false, false);
        }
        mark(ev_end);
#undef GI_LAUNCH_X
#undef GI_LAUNCH_XC
#undef GI_LAUNCH_X1
#undef GI_LAUNCH_XC1
#undef GI_LAUNCH_X2
#undef GI_LAUNCH_XC2
        if (o.spp > 1) hipLaunchKernelGGL(k_x_reduce, sgrid, dim3(256), 0, stream, m, wk, o.spp, rgb, rgb8);
    }
    if (timed) kt->recorded++;
    return hipGetLastError();
}

hipError_t launch_unshard(int w, int h, int shard_count, const double* packed, const uint8_t* packed8, double* rgb,
                          uint8_t* rgb8, hipStream_t stream) {
    const TileMap m = make_map(w, h, shard_count, 0);
    const long long n = m.n_tiles * kTile * kTile;
    hipLaunchKernelGGL(k_unshard, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, m, packed, packed8, rgb, rgb8);
    return hipGetLastError();
}

hipError_t launch_box_kat(int n, const double* recs, int32_t* out, hipStream_t stream) {
    if (n > 0) hipLaunchKernelGGL(k_box_kat, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, n, recs, out);
    return hipGetLastError();
}

hipError_t launch_trace_ray(const DevScene& sc, V3 o, V3 d, V3 light, int32_t* out_i, double* out_d, hipStream_t stream) {
    hipLaunchKernelGGL(k_trace_ray, dim3(1), dim3(64), 0, stream, sc, o, d, light, out_i, out_d);
    return hipGetLastError();
}

}  // namespace gi
