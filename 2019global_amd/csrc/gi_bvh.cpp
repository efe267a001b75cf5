// gi_bvh.cpp — Mode X acceleration structure: an 8-wide bounding volume hierarchy (host build).
//
// Mode X's result is defined by its primitive tests alone (closest t > 1e-7, ties to the lower
// primitive index), so the acceleration structure is free.  The measured cost of one wide-node
// visit is ~4 fp64 triangle tests (dependent loads dominate), so the build minimises node visits:
//   1. binary BVH, binned SAH (32 bins per axis), leaves of <= leaf_max primitives;
//   2. collapse to 8-wide: a wide node takes its binary node's children and repeatedly opens the
//      interior child of largest surface area until it has 8 children (Wald et al. 2008);
//   3. child slots ordered so that visiting slot k ^ octant(ray) for k = 0..7 is approximately
//      front to back for every ray octant (the slot assignment of Ylitie, Karras & Laine 2017):
//      the assignment of children to slots that minimises the summed cost -(octant direction of
//      the slot . offset of the child's centroid from the parent's), by a DP over slot subsets;
//   4. each primitive appears in exactly one leaf; a leaf's records (XHot) are contiguous.
// The fp32 child boxes are rounded outward and padded, so culling is conservative and the fp64
// primitive tests alone decide hits (bit-exact with the oracle's brute force).
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "gi_scene.h"

namespace gi {

namespace {

struct BBox {
    double mn[3], mx[3];
    void reset() {
        for (int k = 0; k < 3; ++k) { mn[k] = INFINITY; mx[k] = -INFINITY; }
    }
    void grow(const BBox& b) {
        for (int k = 0; k < 3; ++k) { mn[k] = std::min(mn[k], b.mn[k]); mx[k] = std::max(mx[k], b.mx[k]); }
    }
    double area() const {
        const double dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        if (!(dx >= 0 && dy >= 0 && dz >= 0)) return 0.0;
        return 2.0 * (dx * dy + dy * dz + dz * dx);
    }
    double centre(int k) const { return 0.5 * (mn[k] + mx[k]); }
};

struct BNode {
    BBox box;
    int left = -1, right = -1;   // interior: children; leaf: left < 0
    int first = 0, count = 0;    // leaf: range in the primitive order array
};

struct Builder {
    const std::vector<BBox>* pb;
    std::vector<int32_t> order;
    std::vector<double> cen;   // 3 per primitive
    std::vector<BNode> nodes;
    int leaf_max = 4;
    static constexpr int kMaxBins = 128;
    int kBins = 32;   // SAH bins per axis (GI_XSAH_BINS, <= kMaxBins)
    // SAH cost of a (binary) node visit relative to one primitive test.  Measured on the 100k soup
    // (GI_XSAH_CT sweep, profiles/r02_s4_sah.txt): 0.35 against 1.0 gives C4 2.10 -> 1.93 ms and C5
    // 231 -> 218 ms (smaller leaves: fewer fp64 record tests per ray, the 8-wide collapse absorbs
    // the extra binary levels); 2 and 4 are 15-20% slower; the Cornell box and the 1k soup are
    // unchanged within noise.
    double kTraverse = 0.35;
    // > 0: every binary node at this depth is a leaf (GI_XFLAT, tuning knob for tiny scenes: depth 3
    // gives at most 8 leaves, i.e. one wide root whose children are all leaves)

    int build(int first, int count, int depth) {
        const int ni = (int)nodes.size();
        nodes.emplace_back();
        BBox box, cb;
        box.reset();
        cb.reset();
        for (int i = first; i < first + count; ++i) {
            const int32_t p = order[i];
            box.grow((*pb)[p]);
            for (int k = 0; k < 3; ++k) { cb.mn[k] = std::min(cb.mn[k], cen[3 * p + k]); cb.mx[k] = std::max(cb.mx[k], cen[3 * p + k]); }
        }
        nodes[ni].box = box;
        nodes[ni].first = first;
        nodes[ni].count = count;
        if (count <= 1 || depth > 60) return ni;
        // binned SAH over the centroid bounds
        int best_axis = -1, best_split = -1;
        double best_cost = INFINITY;
        for (int k = 0; k < 3; ++k) {
            const double lo = cb.mn[k], ext = cb.mx[k] - cb.mn[k];
            if (!(ext > 0)) continue;
            BBox bb[kMaxBins];
            int bn[kMaxBins] = {0};
            for (auto& b : bb) b.reset();
            const double sc = kBins / ext;
            for (int i = first; i < first + count; ++i) {
                const int32_t p = order[i];
                int bi = (int)((cen[3 * p + k] - lo) * sc);
                bi = std::min(std::max(bi, 0), kBins - 1);
                ++bn[bi];
                bb[bi].grow((*pb)[p]);
            }
            double ra[kMaxBins];
            int rn[kMaxBins];
            BBox acc;
            acc.reset();
            int n = 0;
            for (int i = kBins - 1; i > 0; --i) {
                acc.grow(bb[i]);
                n += bn[i];
                ra[i] = acc.area();
                rn[i] = n;
            }
            acc.reset();
            n = 0;
            for (int i = 0; i < kBins - 1; ++i) {
                acc.grow(bb[i]);
                n += bn[i];
                if (n == 0 || rn[i + 1] == 0) continue;
                const double c = acc.area() * n + ra[i + 1] * rn[i + 1];
                if (c < best_cost) { best_cost = c; best_axis = k; best_split = i; }
            }
        }
        const double parea = box.area();
        const double split_cost = parea > 0 ? kTraverse + best_cost / parea : INFINITY;
        if (count <= leaf_max && !(split_cost < (double)count)) return ni;   // SAH prefers a leaf
        int mid;
        if (best_axis < 0) {   // all centroids equal: object median
            mid = first + count / 2;
        } else {
            const double lo = cb.mn[best_axis], sc = kBins / (cb.mx[best_axis] - cb.mn[best_axis]);
            auto it = std::partition(order.begin() + first, order.begin() + first + count, [&](int32_t p) {
                int bi = (int)((cen[3 * p + best_axis] - lo) * sc);
                bi = std::min(std::max(bi, 0), kBins - 1);
                return bi <= best_split;
            });
            mid = (int)(it - order.begin());
            if (mid == first || mid == first + count) mid = first + count / 2;
        }
        const int l = build(first, mid - first, depth + 1);
        const int r = build(mid, first + count - mid, depth + 1);
        nodes[ni].left = l;
        nodes[ni].right = r;
        return ni;
    }
};

// Spatial-split BVH (Stich, Friedrich & Dietrich 2009, "SBVH"): the binary build over *references*
// -- a primitive and the box of its part inside the node's region -- where a node may also be split
// by a plane that cuts references in two (each half's box = the bounds of the triangle's part on that
// side, intersected with the reference's box), when that beats the best object split by SAH.  Only
// tried where the object split's children overlap (area of their intersection > alpha * root area),
// and while the references stay within a budget of the primitive count; spheres are never cut (a
// straddling sphere goes to both sides with its box clipped to each).  The result has the Builder's
// shape (nodes, order = primitive ids of the leaves, a primitive possibly in several leaves), so the
// 8-wide collapse and the leaf emission below are shared.  Culling stays conservative: every part of
// a triangle lies in some reference's box, and the fp64 primitive test of the whole triangle decides.
struct SRef {
    int32_t prim;
    BBox box;
};
struct SBuilder {
    const std::vector<XPrim>* prims;
    std::vector<BNode> nodes;
    std::vector<int32_t> order;   // leaf primitive ids, leaf after leaf
    int leaf_max = 4;
    int kBins = 32;
    double kTraverse = 0.35;
    double alpha_area = 0;        // overlap threshold (alpha * root area)
    size_t ref_budget = 0;        // stop spatial splits when this many references exist
    size_t n_refs = 0;
    int max_split_depth = 10;     // spatial splits only this close to the root (deeper: +2.7 s of
                                  // build on the 100k soup for 0.3% fewer node visits)

    // the bounds of primitive r's part on each side of plane x_axis = pos, within r.box
    void split_ref(const SRef& r, int axis, double pos, BBox& lb, BBox& rb) const {
        lb.reset();
        rb.reset();
        const XPrim& p = (*prims)[r.prim];
        if (p.kind == 0) {
            double v[3][3];
            for (int k = 0; k < 3; ++k) { v[0][k] = p.a[k]; v[1][k] = p.a[k] + p.b[k]; v[2][k] = p.a[k] + p.c[k]; }
            auto add = [](BBox& b, const double* x) {
                for (int k = 0; k < 3; ++k) { b.mn[k] = std::min(b.mn[k], x[k]); b.mx[k] = std::max(b.mx[k], x[k]); }
            };
            for (int e = 0; e < 3; ++e) {
                const double* a = v[e];
                const double* b = v[(e + 1) % 3];
                if (a[axis] <= pos) add(lb, a);
                if (a[axis] >= pos) add(rb, a);
                if ((a[axis] < pos && b[axis] > pos) || (a[axis] > pos && b[axis] < pos)) {
                    const double t = (pos - a[axis]) / (b[axis] - a[axis]);
                    double x[3];
                    for (int k = 0; k < 3; ++k) x[k] = a[k] + t * (b[k] - a[k]);
                    x[axis] = pos;
                    add(lb, x);
                    add(rb, x);
                }
            }
        } else {   // a sphere is not cut: its box on each side
            lb = r.box;
            rb = r.box;
        }
        // within the reference's box and its side of the plane
        lb.mx[axis] = std::min(lb.mx[axis], pos);
        rb.mn[axis] = std::max(rb.mn[axis], pos);
        for (int k = 0; k < 3; ++k) {
            lb.mn[k] = std::max(lb.mn[k], r.box.mn[k]); lb.mx[k] = std::min(lb.mx[k], r.box.mx[k]);
            rb.mn[k] = std::max(rb.mn[k], r.box.mn[k]); rb.mx[k] = std::min(rb.mx[k], r.box.mx[k]);
        }
    }

    static bool valid(const BBox& b) { return b.mn[0] <= b.mx[0] && b.mn[1] <= b.mx[1] && b.mn[2] <= b.mx[2]; }

    int build(std::vector<SRef>& refs, int depth) {
        const int ni = (int)nodes.size();
        nodes.emplace_back();
        BBox box, cb;
        box.reset();
        cb.reset();
        for (const SRef& r : refs) {
            box.grow(r.box);
            for (int k = 0; k < 3; ++k) { cb.mn[k] = std::min(cb.mn[k], r.box.centre(k)); cb.mx[k] = std::max(cb.mx[k], r.box.centre(k)); }
        }
        nodes[ni].box = box;
        const int count = (int)refs.size();
        auto make_leaf = [&]() {
            // a primitive at most once per leaf (its parts may meet again after later splits)
            std::vector<int32_t> ids;
            for (const SRef& r : refs) ids.push_back(r.prim);
            std::sort(ids.begin(), ids.end());
            ids.erase(std::unique(ids.begin(), ids.end()), ids.end());
            nodes[ni].first = (int)order.size();
            nodes[ni].count = (int)ids.size();
            order.insert(order.end(), ids.begin(), ids.end());
            return ni;
        };
        if (count <= 1 || depth > 60) return make_leaf();
        const double parea = box.area();
        // object split: binned SAH over the references' centroids (as Builder)
        int ob_axis = -1, ob_split = -1;
        double ob_cost = INFINITY;
        BBox ob_l, ob_r;
        for (int k = 0; k < 3; ++k) {
            const double lo = cb.mn[k], ext = cb.mx[k] - cb.mn[k];
            if (!(ext > 0)) continue;
            std::vector<BBox> bb(kBins);
            std::vector<int> bn(kBins, 0);
            for (auto& b : bb) b.reset();
            const double sc = kBins / ext;
            for (const SRef& r : refs) {
                int bi = std::min(std::max((int)((r.box.centre(k) - lo) * sc), 0), kBins - 1);
                ++bn[bi];
                bb[bi].grow(r.box);
            }
            std::vector<BBox> racc(kBins);
            std::vector<int> rn(kBins);
            BBox acc;
            acc.reset();
            int n = 0;
            for (int i = kBins - 1; i > 0; --i) { acc.grow(bb[i]); n += bn[i]; racc[i] = acc; rn[i] = n; }
            acc.reset();
            n = 0;
            for (int i = 0; i < kBins - 1; ++i) {
                acc.grow(bb[i]);
                n += bn[i];
                if (n == 0 || rn[i + 1] == 0) continue;
                const double c = acc.area() * n + racc[i + 1].area() * rn[i + 1];
                if (c < ob_cost) { ob_cost = c; ob_axis = k; ob_split = i; ob_l = acc; ob_r = racc[i + 1]; }
            }
        }
        // spatial split: bins over the node box; a reference counts on the left of every plane past
        // its first bin and on the right of every plane before its last
        int sp_axis = -1;
        double sp_pos = 0, sp_cost = INFINITY;
        bool try_spatial = n_refs < ref_budget && ob_axis >= 0 && depth <= max_split_depth;
        if (try_spatial) {
            BBox ov;
            for (int k = 0; k < 3; ++k) { ov.mn[k] = std::max(ob_l.mn[k], ob_r.mn[k]); ov.mx[k] = std::min(ob_l.mx[k], ob_r.mx[k]); }
            try_spatial = valid(ov) && ov.area() > alpha_area;
        }
        if (try_spatial) {
            for (int k = 0; k < 3; ++k) {
                const double lo = box.mn[k], ext = box.mx[k] - box.mn[k];
                if (!(ext > 0)) continue;
                const double w = ext / kBins;
                std::vector<BBox> bb(kBins);
                std::vector<int> enter(kBins, 0), leave(kBins, 0);
                for (auto& b : bb) b.reset();
                for (const SRef& r : refs) {
                    int b0 = std::min(std::max((int)((r.box.mn[k] - lo) / w), 0), kBins - 1);
                    int b1 = std::min(std::max((int)((r.box.mx[k] - lo) / w), 0), kBins - 1);
                    ++enter[b0];
                    ++leave[b1];
                    SRef cur = r;
                    for (int bi = b0; bi < b1; ++bi) {   // chop the reference at each bin plane
                        BBox lb, rb;
                        split_ref(cur, k, lo + w * (bi + 1), lb, rb);
                        if (valid(lb)) bb[bi].grow(lb);
                        if (!valid(rb)) { cur.box.reset(); break; }
                        cur.box = rb;
                    }
                    if (valid(cur.box)) bb[b1].grow(cur.box);
                }
                std::vector<BBox> racc(kBins);
                std::vector<int> rn(kBins);
                BBox acc;
                acc.reset();
                int n = 0;
                for (int i = kBins - 1; i > 0; --i) { acc.grow(bb[i]); n += leave[i]; racc[i] = acc; rn[i] = n; }
                acc.reset();
                n = 0;
                for (int i = 0; i < kBins - 1; ++i) {
                    acc.grow(bb[i]);
                    n += enter[i];
                    if (n == 0 || rn[i + 1] == 0) continue;
                    const double c = acc.area() * n + racc[i + 1].area() * rn[i + 1];
                    if (c < sp_cost) { sp_cost = c; sp_axis = k; sp_pos = lo + w * (i + 1); }
                }
            }
        }
        const double best_cost = std::min(ob_cost, sp_cost);
        const double split_cost = parea > 0 ? kTraverse + best_cost / parea : INFINITY;
        if (count <= leaf_max && !(split_cost < (double)count)) return make_leaf();
        std::vector<SRef> lr, rr;
        if (sp_axis >= 0 && sp_cost < ob_cost) {
            for (const SRef& r : refs) {
                if (r.box.mx[sp_axis] <= sp_pos) lr.push_back(r);
                else if (r.box.mn[sp_axis] >= sp_pos) rr.push_back(r);
                else {
                    BBox lb, rb;
                    split_ref(r, sp_axis, sp_pos, lb, rb);
                    if (valid(lb)) lr.push_back(SRef{r.prim, lb});
                    if (valid(rb)) rr.push_back(SRef{r.prim, rb});
                }
            }
            n_refs += lr.size() + rr.size() - refs.size();
        }
        if (lr.empty() || rr.empty()) {   // object split (or a spatial split that did not divide)
            lr.clear();
            rr.clear();
            if (ob_axis < 0) {   // all centroids equal: halves
                for (int i = 0; i < count; ++i) (i < count / 2 ? lr : rr).push_back(refs[i]);
            } else {
                const double lo = cb.mn[ob_axis], sc = kBins / (cb.mx[ob_axis] - cb.mn[ob_axis]);
                for (const SRef& r : refs) {
                    const int bi = std::min(std::max((int)((r.box.centre(ob_axis) - lo) * sc), 0), kBins - 1);
                    (bi <= ob_split ? lr : rr).push_back(r);
                }
                if (lr.empty() || rr.empty()) {
                    lr.clear();
                    rr.clear();
                    for (int i = 0; i < count; ++i) (i < count / 2 ? lr : rr).push_back(refs[i]);
                }
            }
        }
        std::vector<SRef>().swap(refs);   // release the parent's references before recursing
        const int l = build(lr, depth + 1);
        const int r = build(rr, depth + 1);
        nodes[ni].left = l;
        nodes[ni].right = r;
        return ni;
    }
};

}  // namespace

// Builds hs.xwnodes / xhot / xbox from the Mode X primitives and their fp64 bounds.
void build_xbvh(const std::vector<XPrim>& prims, const std::vector<double>& bounds, int leaf_max, HostScene& hs,
                bool geometric) {
    const size_t np = prims.size();
    std::vector<BBox> pb(np);
    BBox scene;
    scene.reset();
    for (size_t i = 0; i < np; ++i) {
        for (int k = 0; k < 3; ++k) { pb[i].mn[k] = bounds[6 * i + k]; pb[i].mx[k] = bounds[6 * i + 3 + k]; }
        scene.grow(pb[i]);
    }
    double ext = 1.0;
    for (int k = 0; k < 3; ++k)
        if (np) ext = std::max(ext, std::max(std::fabs(scene.mn[k]), std::fabs(scene.mx[k])));
    const double pad32 = 1e-5 * ext;
    auto lo32 = [&](double v) {
        float f = (float)(v - pad32);
        if ((double)f > v - pad32) f = std::nextafter(f, -INFINITY);
        return f;
    };
    auto hi32 = [&](double v) {
        float f = (float)(v + pad32);
        if ((double)f < v + pad32) f = std::nextafter(f, INFINITY);
        return f;
    };

    hs.xwnodes.clear();
    hs.xhot.clear();
    hs.xbox.clear();
    XWNode blank;
    for (int c = 0; c < 8; ++c) {
        for (int k = 0; k < 3; ++k) { blank.lo[k][c] = INFINITY; blank.hi[k][c] = -INFINITY; }
        blank.child[c] = XEMPTY;
        blank.cnt[c] = 0;
    }
    blank.parent = -1;
    blank.exists = 0;
    blank.pad[0] = blank.pad[1] = 0;
    hs.xwnodes.push_back(blank);   // root
    hs.x_max_depth = 0;
    if (np == 0) {
        finalize_xwnodes(hs.xwnodes);
        return;
    }

    Builder b;
    b.pb = &pb;
    b.leaf_max = std::max(1, leaf_max);
    b.order.resize(np);
    b.cen.resize(3 * np);
    for (size_t i = 0; i < np; ++i) {
        b.order[i] = (int32_t)i;
        for (int k = 0; k < 3; ++k) b.cen[3 * i + k] = pb[i].centre(k);
    }
    b.nodes.reserve(2 * np);
    int root;
    // The spatial-split build for scenes of more than kSpatialMin primitives (the HBM-resident
    // ones; the 100k soup: C5 -1.5%, C4 -1%, +9% leaf records, +0.9 s of build,
    // profiles/r03_sbvh.txt): a references' budget of 1.5 x the primitives, splits tried where the
    // object split's children overlap by more than 1e-5 of the scene's area, down to level 10.
    // GI_XSBVH=0/1 forces it off / on (a test hook: the frame does not depend on it)
    constexpr size_t kSpatialMin = 8192;
    const char* sbv = std::getenv("GI_XSBVH");
    hs.x_spatial = geometric && (sbv ? std::atoi(sbv) != 0 : np > kSpatialMin);
    if (hs.x_spatial) {
        SBuilder sb;
        sb.prims = &prims;
        sb.leaf_max = b.leaf_max;
        sb.kBins = b.kBins;
        sb.kTraverse = b.kTraverse;
        sb.ref_budget = (size_t)(1.5 * (double)np);
        std::vector<SRef> refs(np);
        for (size_t i = 0; i < np; ++i) refs[i] = SRef{(int32_t)i, pb[i]};
        sb.alpha_area = 1e-5 * scene.area();
        sb.n_refs = np;
        root = sb.build(refs, 0);
        b.nodes = std::move(sb.nodes);
        b.order = std::move(sb.order);
    } else {
        root = b.build(0, (int)np, 0);
    }

    auto emit_leaf = [&](int first, int count) {   // -> ~offset into xhot
        const int32_t off = (int32_t)hs.xhot.size();
        std::vector<int32_t> ids(b.order.begin() + first, b.order.begin() + first + count);
        std::sort(ids.begin(), ids.end());   // ascending primitive index inside a leaf
        for (int32_t pi : ids) {
            const XPrim& p = prims[pi];
            XHot h;
            memcpy(h.a, p.a, sizeof h.a);
            memcpy(h.b, p.b, sizeof h.b);
            memcpy(h.c, p.c, sizeof h.c);
            h.prim = pi;
            h.kind = p.kind;
            hs.xhot.push_back(h);
            XBox bx;
            for (int a = 0; a < 3; ++a) { bx.lo[a] = lo32(pb[pi].mn[a]); bx.hi[a] = hi32(pb[pi].mx[a]); }
            bx.pad[0] = pi;
            bx.pad[1] = p.kind;
            hs.xbox.push_back(bx);
        }
        return off;
    };
    // collect all primitives under a binary subtree into one leaf range (depth cap fallback)
    std::function<void(int, std::vector<int32_t>&)> gather = [&](int n, std::vector<int32_t>& out) {
        const BNode& bn = b.nodes[n];
        if (bn.left < 0) {
            out.insert(out.end(), b.order.begin() + bn.first, b.order.begin() + bn.first + bn.count);
            return;
        }
        gather(bn.left, out);
        gather(bn.right, out);
    };

    // child-to-slot assignment of minimum total cost (C3 kernel -1% against the greedy one, the
    // soups unchanged, profiles/r02_s4_sah.txt)
    // fill wide node `wi` (depth `wd`) from binary node `bn`'s subtree
    std::function<void(int, int, int)> fill = [&](int wi, int bn, int wd) {
        hs.x_max_depth = std::max(hs.x_max_depth, wd);
        std::vector<int> kids;
        if (b.nodes[bn].left < 0) {
            kids.push_back(bn);   // root that is a single leaf
        } else {
            kids.push_back(b.nodes[bn].left);
            kids.push_back(b.nodes[bn].right);
            while (kids.size() < 8) {
                int pick = -1;
                double best = -1;
                for (int i = 0; i < (int)kids.size(); ++i) {
                    const BNode& k = b.nodes[kids[i]];
                    if (k.left >= 0 && k.box.area() > best) { best = k.box.area(); pick = i; }
                }
                if (pick < 0) break;
                const int n = kids[pick];
                kids[pick] = b.nodes[n].left;
                kids.push_back(b.nodes[n].right);
            }
        }
        // slot assignment: child centroid offset vs octant direction of each slot (greedy)
        const BBox& pbox = b.nodes[bn].box;
        const int nk = (int)kids.size();
        double cost[8][8];
        for (int i = 0; i < nk; ++i)
            for (int s = 0; s < 8; ++s) {
                double c = 0;
                for (int k = 0; k < 3; ++k) {
                    const double off = b.nodes[kids[i]].box.centre(k) - pbox.centre(k);
                    c -= ((s >> k) & 1 ? 1.0 : -1.0) * off;
                }
                cost[i][s] = c;
            }
        int slot_of[8];
        {   // minimum-cost assignment: DP over the set of slots taken by kids 0..i-1
            double dp[256];
            int8_t pick[9][256];
            for (int m = 0; m < 256; ++m) dp[m] = INFINITY;
            dp[0] = 0.0;
            for (int i = 0; i < nk; ++i) {
                double nd[256];
                for (int m = 0; m < 256; ++m) nd[m] = INFINITY;
                for (int m = 0; m < 256; ++m) {
                    if (dp[m] == INFINITY || __builtin_popcount(m) != i) continue;
                    for (int sl = 0; sl < 8; ++sl) {
                        if (m & (1 << sl)) continue;
                        const double c = dp[m] + cost[i][sl];
                        if (c < nd[m | (1 << sl)]) { nd[m | (1 << sl)] = c; pick[i][m | (1 << sl)] = (int8_t)sl; }
                    }
                }
                for (int m = 0; m < 256; ++m) dp[m] = nd[m];
            }
            int bm = -1;
            for (int m = 0; m < 256; ++m)
                if (__builtin_popcount(m) == nk && dp[m] < INFINITY && (bm < 0 || dp[m] < dp[bm])) bm = m;
            for (int i = nk - 1; i >= 0; --i) {
                slot_of[i] = pick[i][bm];
                bm &= ~(1 << slot_of[i]);
            }
        }
        for (int i = 0; i < nk; ++i) {
            const int s = slot_of[i];
            const BNode& k = b.nodes[kids[i]];
            {
                XWNode& w = hs.xwnodes[wi];
                for (int a = 0; a < 3; ++a) { w.lo[a][s] = lo32(k.box.mn[a]); w.hi[a][s] = hi32(k.box.mx[a]); }
            }
            if (k.left < 0) {
                const int32_t off = emit_leaf(k.first, k.count);
                XWNode& w = hs.xwnodes[wi];
                w.child[s] = ~off;
                w.cnt[s] = (uint16_t)std::min(k.count, 65535);
            } else if (wd + 1 > 15) {   // traversal keeps 16 levels of child masks: flatten below
                std::vector<int32_t> ids;
                gather(kids[i], ids);
                const int32_t off = (int32_t)hs.xhot.size();
                for (int32_t pi : ids) {   // emit_leaf on an explicit id list
                    const XPrim& p = prims[pi];
                    XHot h;
                    memcpy(h.a, p.a, sizeof h.a);
                    memcpy(h.b, p.b, sizeof h.b);
                    memcpy(h.c, p.c, sizeof h.c);
                    h.prim = pi;
                    h.kind = p.kind;
                    hs.xhot.push_back(h);
                    XBox bx;
                    for (int a = 0; a < 3; ++a) { bx.lo[a] = lo32(pb[pi].mn[a]); bx.hi[a] = hi32(pb[pi].mx[a]); }
                    bx.pad[0] = pi;
                    bx.pad[1] = p.kind;
                    hs.xbox.push_back(bx);
                }
                XWNode& w = hs.xwnodes[wi];
                w.child[s] = ~off;
                w.cnt[s] = (uint16_t)std::min<size_t>(ids.size(), 65535);
            } else {
                const int ci = (int)hs.xwnodes.size();
                hs.xwnodes.push_back(blank);
                hs.xwnodes[ci].parent = wi;
                hs.xwnodes[wi].child[s] = ci;
                fill(ci, kids[i], wd + 1);
            }
        }
    };
    fill(0, root, 0);
    finalize_xwnodes(hs.xwnodes);

    // surface-area estimates of the work per ray (a random line through the root box meets a box
    // with probability area(box) / area(root)): wide nodes entered and primitives tested
    const double aroot = b.nodes[root].box.area();
    double est_nodes = 0, est_prims = 0;
    if (aroot > 0) {
        for (const XWNode& w : hs.xwnodes)
            for (int c = 0; c < 8; ++c) {
                if (w.child[c] == XEMPTY) continue;
                BBox cb;
                for (int k = 0; k < 3; ++k) { cb.mn[k] = w.lo[k][c]; cb.mx[k] = w.hi[k][c]; }
                const double p = std::min(1.0, cb.area() / aroot);
                if (w.child[c] >= 0) est_nodes += p;
                else est_prims += p * w.cnt[c];
            }
    }
    hs.x_est_nodes = est_nodes;
    hs.x_est_prims = est_prims;
    // k_mode_x's shading handler runs once this many eighths of a wave's live lanes wait.  Short
    // traversals (few node visits per ray) gain from shading whole waves at once; long ones lose
    // more to lanes idling at the threshold (measured: Cornell / main / 1k soup best at 8/8, the
    // 100k soup at 3/8 in round 2 and 4/8 with UL: C4 1.72 -> 1.67-1.69 ms, C5 equal).  One node
    // visit costs ~4 primitive tests.
    const bool long_traversal = est_nodes + 0.25 * est_prims > 16.0;
    hs.x_handle8 = long_traversal ? 4 : 8;
    // short traversals also continue a path from its finished shadow ray inside the traversal
    // branch (measured +14% on the Cornell box, -5% on the 100k soup)
    hs.x_flags = long_traversal ? 0 : 1;
}

// Mode R candidate reconstruction.  The reference's pixel is the LAST candidate of
// Octree::intersect's list (octree.h:132-155, DFS over children 0..7) whose intersect() succeeds
// (raytracer.h:53-74, A.1).  A leaf L is in the list iff every node on its path below the root is
// non-empty (:140) and passes the ExpBox node test (:141-146); its entities appear at list
// position (rank of L in the static DFS order, index in L's list).  So the answer is the hitting
// entity whose latest reachable appearance is latest -- computable from the few entities the ray's
// LINE passes near (the reference has no t > 0 test, A.2/A.3), without walking the tree:
//   * every entity's appearances, by decreasing (leaf rank, position);
//   * every leaf's root path, top-down, for the reachability check;
//   * a line BVH over the entities that appear in some leaf, each boxed by the union of its
//     triangles' prefilter spheres (gi_math.h tri_may_hit: a line outside them cannot produce a
//     hit; the kernel widens the boxes by a margin covering the prefilter's 1e-12|oc|^2 slack and
//     fp32 slab rounding).  ImpSpheres (a line test with fp32 coefficients, A.2) are not boxed:
//     every ray tests them.
void build_rcand(HostScene& hs) {
    const int nn = (int)hs.rnodes.size(), ne = (int)hs.ents.size();
    // static DFS order of the leaves and their paths
    std::vector<int64_t> leaf_rank((size_t)nn, -1);
    std::vector<std::vector<int32_t>> paths((size_t)nn);
    std::vector<int32_t> path;
    int64_t next = 0;
    std::function<void(int)> dfs = [&](int n) {
        const RNode& r = hs.rnodes[n];
        if (r.child0 < 0) {
            leaf_rank[n] = next++;
            paths[n] = path;
            return;
        }
        for (int c = 0; c < 8; ++c) {
            path.push_back(r.child0 + c);
            dfs(r.child0 + c);
            path.pop_back();
        }
    };
    if (nn > 0) dfs(0);
    hs.r_leaf_of_rank.assign((size_t)next, -1);
    for (int n = 0; n < nn; ++n)
        if (leaf_rank[n] >= 0) hs.r_leaf_of_rank[(size_t)leaf_rank[n]] = n;
    hs.rpath_off.assign((size_t)nn + 1, 0);
    hs.rpath.clear();
    for (int n = 0; n < nn; ++n) {
        hs.rpath.insert(hs.rpath.end(), paths[n].begin(), paths[n].end());
        hs.rpath_off[n + 1] = (int32_t)hs.rpath.size();
    }
    // appearances per entity, latest first
    std::vector<std::vector<std::pair<int64_t, int32_t>>> app((size_t)ne);
    for (int n = 0; n < nn; ++n) {
        const RNode& r = hs.rnodes[n];
        if (r.child0 >= 0) continue;
        for (int p = 0; p < r.ent_cnt; ++p)
            app[hs.leaf_ents[r.ent_off + p]].push_back({(leaf_rank[n] << 32) | (int64_t)p, n});
    }
    hs.app_off.assign((size_t)ne + 1, 0);
    hs.app_leaf.clear();
    hs.app_rank.clear();
    for (int e = 0; e < ne; ++e) {
        std::sort(app[e].begin(), app[e].end(), [](const std::pair<int64_t, int32_t>& a,
                                                   const std::pair<int64_t, int32_t>& b) { return a.first > b.first; });
        for (const auto& a : app[e]) {
            hs.app_rank.push_back(a.first);
            hs.app_leaf.push_back(a.second);
        }
        hs.app_off[e + 1] = (int32_t)hs.app_rank.size();
    }
    // the device's records: every path entry's node box, every appearance's rank and path range
    hs.rpath_rec.resize(hs.rpath.size());
    for (size_t i = 0; i < hs.rpath.size(); ++i) {
        const RNode& r = hs.rnodes[(size_t)hs.rpath[i]];
        RPathRec& q = hs.rpath_rec[i];
        for (int k = 0; k < 3; ++k) { q.mn[k] = r.mn[k]; q.mx[k] = r.mx[k]; }
        q.node = hs.rpath[i];
        q.ent_cnt = r.ent_cnt;
        q.pad[0] = q.pad[1] = 0;
    }
    hs.app_rec.resize(hs.app_rank.size());
    for (size_t a = 0; a < hs.app_rank.size(); ++a)
        hs.app_rec[a] = RApp{hs.app_rank[a], hs.rpath_off[(size_t)hs.app_leaf[a]], hs.rpath_off[(size_t)hs.app_leaf[a] + 1]};
    // line BVH over the entities that appear somewhere
    std::vector<XPrim> atoms;
    std::vector<double> bounds;
    std::vector<int32_t> atom_ent;
    hs.r_always.clear();
    hs.rc_ext = 0;
    for (int e = 0; e < ne; ++e) {
        if (app[e].empty()) continue;
        const REnt& E = hs.ents[e];
        if (E.kind == K_IMP_SPHERE || E.tri_count <= 0) {
            hs.r_always.push_back(e);
            continue;
        }
        double mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
        bool finite = true;
        for (int t = 0; t < E.tri_count; ++t) {
            const TriRec& T = hs.tris[E.tri_first + t];
            const V3 p1 = ld3(T.p1), p2 = ld3(T.p2), p3 = ld3(T.p3);
            const V3 c = (p1 + p2 + p3) * (1.0 / 3.0);   // tri_may_hit's sphere
            const double r2 = smax(smax(sq3(p1 - c), sq3(p2 - c)), sq3(p3 - c));
            const double R = std::sqrt(r2 * 1.0201) * (1.0 + 1e-9) + 1e-300;
            const double cc[3] = {c.x, c.y, c.z};
            for (int k = 0; k < 3; ++k) {
                mn[k] = std::min(mn[k], cc[k] - R);
                mx[k] = std::max(mx[k], cc[k] + R);
            }
            finite = finite && std::isfinite(R) && std::isfinite(c.x) && std::isfinite(c.y) && std::isfinite(c.z);
        }
        if (!finite) {   // degenerate coordinates: no box can bound it, test it on every ray
            hs.r_always.push_back(e);
            continue;
        }
        XPrim p;
        memset(&p, 0, sizeof p);
        p.ent = e;
        atoms.push_back(p);
        for (int k = 0; k < 3; ++k) bounds.push_back(mn[k]);
        for (int k = 0; k < 3; ++k) bounds.push_back(mx[k]);
        for (int k = 0; k < 3; ++k) hs.rc_ext = std::max(hs.rc_ext, std::max(std::fabs(mn[k]), std::fabs(mx[k])));
        atom_ent.push_back(e);
    }
    HostScene tmp;
    build_xbvh(atoms, bounds, 4, tmp);
    hs.rc_nodes = std::move(tmp.xwnodes);
    hs.rc_ent.resize(tmp.xhot.size());
    for (size_t j = 0; j < tmp.xhot.size(); ++j) hs.rc_ent[j] = atom_ent[tmp.xhot[j].prim];
    // Rank order: every slot carries the highest list rank of the entities below it (an entity's
    // first appearance is its latest), and each node's slots are sorted by it, highest first.  The
    // answer is the hitting candidate of highest reachable rank, so a walk in slot order meets the
    // likely winners first, and once a popped slot's bound is <= the best rank found, neither it nor
    // its later siblings can hold a better candidate (the kernels drop the rest of that level).
    // Children follow their parent in rc_nodes (fill pushes them), so one backward pass suffices.
    const int nw = (int)hs.rc_nodes.size();
    hs.rc_maxkey.assign((size_t)nw * 8, -1);
    for (int w = nw - 1; w >= 0; --w) {
        XWNode& nd = hs.rc_nodes[w];
        int64_t key[8];
        for (int c = 0; c < 8; ++c) {
            key[c] = -1;
            if (nd.child[c] == XEMPTY) continue;
            if (nd.child[c] >= 0) {
                for (int k = 0; k < 8; ++k) key[c] = std::max(key[c], hs.rc_maxkey[(size_t)nd.child[c] * 8 + k]);
            } else {
                for (int j = 0; j < nd.cnt[c]; ++j) {
                    const int e = hs.rc_ent[~nd.child[c] + j];
                    key[c] = std::max(key[c], hs.app_rank[hs.app_off[e]]);
                }
            }
        }
        int perm[8] = {0, 1, 2, 3, 4, 5, 6, 7};
        std::stable_sort(perm, perm + 8, [&](int a, int b) {
            const bool ea = nd.child[a] == XEMPTY, eb = nd.child[b] == XEMPTY;
            if (ea != eb) return eb;   // empty slots last
            return key[a] > key[b];
        });
        const XWNode old = nd;
        for (int i = 0; i < 8; ++i) {
            const int c = perm[i];
            for (int a = 0; a < 3; ++a) { nd.lo[a][i] = old.lo[a][c]; nd.hi[a][i] = old.hi[a][c]; }
            nd.child[i] = old.child[c];
            nd.cnt[i] = old.cnt[c];
            hs.rc_maxkey[(size_t)w * 8 + i] = key[c];
        }
    }
    finalize_xwnodes(hs.rc_nodes);
}


// Quantised nodes (XCNode): per axis, org = the children's union minimum and the smallest scale 2^e
// with (union max - org) / 2^e <= 255; each child's q are rounded outward and then checked -- and
// moved outward while needed -- with the device's arithmetic (fmaf), so every decoded box contains
// the padded fp32 box of XWNode.  Should the largest q need 256, the axis takes the next exponent.
bool encode_xcnodes(const std::vector<XWNode>& w, std::vector<XCNode>& out) {
    out.assign(w.size(), XCNode());
    for (size_t i = 0; i < w.size(); ++i) {
        const XWNode& n = w[i];
        XCNode& q = out[i];
        std::memset(&q, 0, sizeof q);
        q.exists = (uint8_t)n.exists;
        q.parent = n.parent;
        for (int c = 0; c < 8; ++c) {
            q.child[c] = n.child[c];
            if (n.cnt[c] > 255) return false;
            q.cnt[c] = (uint8_t)n.cnt[c];
        }
        for (int a = 0; a < 3; ++a) {
            float ulo = INFINITY, uhi = -INFINITY;
            for (int c = 0; c < 8; ++c)
                if ((n.exists >> c) & 1) { ulo = std::min(ulo, n.lo[a][c]); uhi = std::max(uhi, n.hi[a][c]); }
            if (!(ulo <= uhi)) { ulo = 0.0f; uhi = 0.0f; }   // no child
            q.org[a] = ulo;
            const double span = (double)uhi - (double)ulo;
            int e = -126;
            while (e < 127 && std::ldexp(255.0, e) < span) ++e;
            for (;; ++e) {
                if (e > 127) return false;
                const float sc = std::ldexp(1.0f, e);
                bool ok = true;
                for (int c = 0; c < 8 && ok; ++c) {
                    if (!((n.exists >> c) & 1)) { q.qlo[a][c] = 0; q.qhi[a][c] = 0; continue; }
                    double fl = std::floor(((double)n.lo[a][c] - (double)ulo) / std::ldexp(1.0, e));
                    double fh = std::ceil(((double)n.hi[a][c] - (double)ulo) / std::ldexp(1.0, e));
                    int lo = (int)std::max(0.0, std::min(255.0, fl)), hi = (int)std::max(0.0, std::min(255.0, fh));
                    while (lo > 0 && !(std::fmaf((float)lo, sc, ulo) <= n.lo[a][c])) --lo;
                    while (hi <= 255 && !(std::fmaf((float)hi, sc, ulo) >= n.hi[a][c])) ++hi;
                    if (!(std::fmaf((float)lo, sc, ulo) <= n.lo[a][c]) || hi > 255) { ok = false; break; }
                    q.qlo[a][c] = (uint8_t)lo;
                    q.qhi[a][c] = (uint8_t)hi;
                }
                if (ok) { q.ex[a] = (int8_t)e; break; }
            }
        }
    }
    return true;
}

}  // namespace gi
