// gi_scene.h — device-resident scene layout (HBM) and the host-side builder interface.
//
// Mode R keeps the reference octree exactly (octree.h:12-163, including SURVEY A.4-A.6, A.14):
//   RNode[]   64 B/node: AABB (fp64) + child0 / parent / leaf list range.  Children of a node are
//             8 consecutive records in octant order 0..7 (octree.h:94-108).
//   leaf_ents int32 entity indices, each leaf's list in push order.
//   REnt[]    entity records (kind, material, sphere/quad parameters) + TriRec[] triangles.
// Mode X uses its own tight octree over primitives (XWNode[] traversal nodes, XHot[] leaf records,
// XPrim[] shading records).
#pragma once
#include <stdint.h>
#include <vector>

#include "gi_math.h"

namespace gi {

enum EntKind : int32_t { K_IMP_SPHERE = 1, K_IMP_TRIANGLE = 2, K_EXP_QUAD = 3, K_EXP_SPHERE = 4, K_EXP_CUBE = 5,
                         K_EXP_CONE = 6, K_EXP_RECTANGLE = 7, K_EXP_BOX = 8 };

struct RNode {             // 64 bytes
    double mn[3], mx[3];
    int32_t child0;        // -1: leaf
    int32_t parent;        // -1: root
    int32_t ent_off;       // leaves: offset into leaf_ents
    int32_t ent_cnt;       // size of the node's _entities (interior: only emptiness is used, octree.h:140)
};
static_assert(sizeof(RNode) == 64, "RNode layout");

// Mode R reachability records (the flat reach phase and the candidate walks, round 5): a leaf's root
// path laid out as consecutive node records, so a walk down it streams one record after another (the
// next load issued before the current exact node test) instead of chasing rpath[i] -> rnodes[...].
struct RPathRec {          // 64 bytes: the node's box, its id (memo key) and emptiness
    double mn[3], mx[3];
    int32_t node;
    int32_t ent_cnt;
    int32_t pad[2];
};
static_assert(sizeof(RPathRec) == 64, "RPathRec layout");
struct RApp {              // 16 bytes: one appearance of an entity, by decreasing rank
    int64_t rank;          // (leaf's rank in the reference's DFS order << 32) | position
    int32_t p0, p1;        // its leaf's root path: rpath_rec[p0 .. p1), top-down
};
static_assert(sizeof(RApp) == 16, "RApp layout");

struct REnt {              // 208 bytes
    int32_t kind, tri_first, tri_count, pad0;
    double pos[3];         // ImpSphere / ExpSphere / ExpCone centre, ExpQuad / ExpCube pos
    float radius, width, length, alpha;
    double qv0[3], qv1[3], qv2[3];   // texture frames: ExpQuad vertices[0], [1] (entities.h:634-635);
                                     // ExpCube vertices[0] (:772); ExpRectangle p1, p3, p4 (:346-350)
    double color[3], shader[3];
    double spec_pow;
    float height, pad1;    // ExpCube / ExpCone height
    double sin_theta;      // ExpCone: sin(cone_theta), cone_theta = float atan(radius/height) (:950-953)
    double refl;           // Mode X mirror-reflection probability (gi_entity_desc::mat_reflectivity)
};
static_assert(sizeof(REnt) == 208, "REnt layout");

// Mode X primitive: triangle (v0, e1, e2, n) or sphere (c, r)
struct XPrim {             // 112 bytes
    double a[3];           // triangle v0 | sphere centre
    double b[3];           // triangle e1 | sphere (r, 0, 0)
    double c[3];           // triangle e2
    double n[3];           // triangle geometric normal normalize(cross(e1,e2))
    int32_t kind;          // 0 triangle, 1 sphere
    int32_t ent;
    int32_t pad[2];        // pad[0]: plane group (gi_build.cpp assign_plane_groups; 255 none)
};
static_assert(sizeof(XPrim) == 112, "XPrim layout");

struct XNode {             // 64 bytes
    double mn[3], mx[3];   // conservative AABB of the cell
    int32_t child_base;    // interior: index of the first existing child (children contiguous)
    int32_t child_mask;    // interior: bit c set if octant c exists; 0 for a leaf
    int32_t prim_off;      // leaf: range in xprim_idx
    int32_t prim_cnt;
};
static_assert(sizeof(XNode) == 64, "XNode layout");

// Mode X traversal node: the 8 children of one octree cell, each child's tight box in fp32
// rounded outward and padded (conservative culling; the fp64 primitive tests decide hits).
constexpr int32_t XEMPTY = (int32_t)0x80000000;
struct XWNode {            // 256 bytes, 2 cache lines
    float lo[3][8];        // child box minima, SoA over the 8 octants
    float hi[3][8];
    int32_t child[8];      // >= 0: wide node; < 0 (not XEMPTY): leaf = ~(offset into xhot[]); XEMPTY: none
    int32_t parent;        // wide node of the parent cell, -1 at the root (stackless traversal)
    uint16_t cnt[8];       // leaf children: number of xhot records
    int32_t exists;        // bit c set iff child[c] != XEMPTY (branch-free culling)
    int32_t pad[2];        // byte c: plane group of leaf child c, 255 none (Mode X scene nodes)
};
static_assert(sizeof(XWNode) == 256, "XWNode layout");
// The same node quantised into one 128-byte cache line (HBM-resident scenes, k_mode_x): child c's
// box on axis a is lo = fma(qlo[a][c], 2^ex[a], org[a]), hi = fma(qhi[a][c], 2^ex[a], org[a]) in
// fp32, with the 8-bit q chosen on the host -- by the device's own fused arithmetic -- so that the
// decoded box contains XWNode's padded box (culling stays conservative).  Children, counts and
// parent as in XWNode (counts <= 255; a scene with a larger leaf keeps XWNode).
struct XCNode {            // 128 bytes
    float org[3];
    int8_t ex[3];
    uint8_t exists;        // bit c set iff child[c] != XEMPTY
    uint8_t qlo[3][8];
    uint8_t qhi[3][8];     // bytes 0..63: what the slab tests read (four 16-byte loads)
    int32_t child[8];
    uint8_t cnt[8];
    int32_t parent;
    int32_t pad[5];
};
static_assert(sizeof(XCNode) == 128, "XCNode layout");
// Encodes w as XCNode (the decode above contains every child's box); false if a count exceeds 255.
bool encode_xcnodes(const std::vector<XWNode>& w, std::vector<XCNode>& out);

// Leaf primitive records, duplicated per leaf reference and stored contiguously per leaf, so a
// leaf costs one dependent load level: exactly what Moller-Trumbore / the sphere test read.
struct XHot {              // 80 bytes
    double a[3], b[3], c[3];   // triangle v0, e1, e2 | sphere centre, (r, 0, 0)
    int32_t prim;          // global primitive index (tie-break, shading record)
    int32_t kind;          // 0 triangle, 1 sphere
};
static_assert(sizeof(XHot) == 80, "XHot layout");
// fp32 prefilter record parallel to xhot[]: the primitive's AABB rounded outward and padded, so a
// ray that misses it cannot hit the primitive; the 80-B fp64 record is fetched only otherwise.
struct XBox {              // 32 bytes
    float lo[3], hi[3];
    int32_t pad[2];
};
static_assert(sizeof(XBox) == 32, "XBox layout");
struct XLeaf {
    int32_t off, cnt;      // host build only: range in xprim_idx
};

struct HostScene {
    // Mode R
    std::vector<RNode> rnodes;
    std::vector<int32_t> leaf_ents;
    std::vector<REnt> ents;
    std::vector<TriRec> tris;
    int32_t max_depth = 0, n_leaves = 0, n_reachable = 0, n_dropped = 0;
    // Mode X
    std::vector<XNode> xnodes;
    std::vector<XWNode> xwnodes;
    std::vector<XCNode> xcnodes;     // xwnodes quantised (encode_xcnodes), for HBM-resident scenes
    std::vector<XLeaf> xleaves;
    std::vector<int32_t> xprim_idx;
    std::vector<XHot> xhot;
    std::vector<XBox> xbox;
    std::vector<XPrim> xprims;
    int32_t x_max_depth = 0;
    // Mode R candidate reconstruction (gi_bvh.cpp build_rcand; DESIGN.md §5 k_mode_r)
    std::vector<int32_t> app_off;    // per entity (n_ents + 1): its appearances in leaf lists
    std::vector<int32_t> app_leaf;   //   leaf node of each appearance, by decreasing rank
    std::vector<int64_t> app_rank;   //   (leaf's rank in the reference's DFS order << 32) | position
    std::vector<int32_t> rpath_off;  // per node (n_rnodes + 1): its path below the root, top-down
    std::vector<int32_t> rpath;      //   (filled for leaves; the leaf itself is the last entry)
    std::vector<RPathRec> rpath_rec; // rpath's node records, in the same order (the device reads these)
    std::vector<RApp> app_rec;       // app_rank / app_leaf as (rank, path range) records (device)
    std::vector<XWNode> rc_nodes;    // line BVH over the non-sphere entities that appear in a leaf
    std::vector<int32_t> rc_ent;     //   entity of each leaf record
    std::vector<int64_t> rc_maxkey;  //   per node slot (8 per node): the highest app_rank under it;
                                     //   a node's slots are in decreasing order of it
    std::vector<int32_t> r_always;   // ImpSpheres that appear in a leaf (tested by every ray)
    std::vector<int32_t> r_leaf_of_rank;   // leaf node of each DFS rank (app_rank >> 32)
    double rc_ext = 0;               // max |coordinate| of the line BVH's boxes
    int32_t x_handle8 = 6;   // Mode X handler threshold (eighths), chosen by the builder
    int32_t x_flags = 0;     // Mode X schedule flags (DevScene::x_flags), chosen by the builder
    double x_est_nodes = 0, x_est_prims = 0;   // SAH estimates per random ray through the root
    bool x_spatial = false;  // the Mode X BVH was built with spatial splits (a primitive in several leaves)
    double x_skip_a = 0.0, x_skip_b = 2.0;   // own-plane leaf skip: |d . n| >= a * max|cam| + b (gi_build.cpp)
};

// Sets XWNode::exists from the child references (both Mode X builders call it last).
inline void finalize_xwnodes(std::vector<XWNode>& w) {
    for (XWNode& n : w) {
        n.exists = 0;
        for (int c = 0; c < 8; ++c)
            if (n.child[c] != XEMPTY) n.exists |= 1 << c;
    }
}

// Mode X 8-wide BVH over the primitives (gi_bvh.cpp); bounds: 6 doubles (min xyz, max xyz) each.
// geometric: the prims hold their geometry (Mode X), so large scenes may use spatial splits; the
// Mode R line BVH passes boxes only.
void build_xbvh(const std::vector<XPrim>& prims, const std::vector<double>& bounds, int leaf_max, HostScene& hs,
                bool geometric = false);
// Mode R candidate reconstruction structures (HostScene app_* / rpath* / rc_* / r_always) from the
// reference octree (rnodes, leaf_ents) and the entities' triangles.
void build_rcand(HostScene& hs);

// Device view passed to kernels by value.
struct DevScene {
    const RNode* rnodes;
    const int32_t* leaf_ents;
    const REnt* ents;
    const TriRec* tris;
    const XWNode* xwnodes;
    const XCNode* xcnodes;   // quantised copy of xwnodes (null: the scene keeps XWNode everywhere)
    const XHot* xhot;
    const XBox* xbox;
    const XPrim* xprims;
    unsigned* work;        // 16 device counters (persistent-kernel tile queue), reset per launch
    int32_t n_rnodes, n_ents, n_xwnodes, n_xprims;
    int32_t x_max_depth;
    int32_t x_handle8;     // Mode X shading-handler threshold, eighths of the live lanes (set at upload)
    int32_t x_flags;       // Mode X schedule flags: bit 0 = continue paths from shadow rays in traversal
    int32_t n_xhot;
    int32_t x_lds_bytes;   // > 0: xwnodes + xhot fit in LDS and are staged there by each workgroup
    int32_t x_waves4;      // LDS-resident scene with light shading: k_mode_x at 4 waves per SIMD
    int32_t x_tri_only;    // every primitive a triangle, every entity ImpTriangle / ExpQuad / ExpCube /
                           // ExpBox (the 4-wave kinds): HBM-resident k_mode_x's TRI specialisation
    int32_t r_tri_only;    // every entity an ImpTriangle: the Mode R kernels' TRI specialisation
    float root_lo[3], root_hi[3];   // Mode X: union of the root's fp32 child boxes (conservative)
    double x_skip_a, x_skip_b;      // Mode X own-plane leaf skip bound (HostScene, gi_build.cpp)
    // Mode R candidate reconstruction (HostScene fields of the same names)
    const int32_t* app_off;
    const RApp* app_rec;
    const RPathRec* rpath_rec;
    const XWNode* rc_nodes;
    const int32_t* rc_ent;
    const int64_t* rc_maxkey;
    const int32_t* r_always;
    const int32_t* r_leaf_of_rank;
    int32_t n_r_always;
    float rc_ext;
};

// HIP events bracketing the dominant kernel of renders issued with GI_FLAG_TIME (owned by the
// scene handle, created on first use): a ring of kRing pairs, so frames stay asynchronous; a pair
// about to be reused is folded into the running sum first (it ended kRing frames ago).
struct KTimer {
    static constexpr int kRing = 64;
    void* ev0[kRing] = {};   // hipEvent_t
    void* ev1[kRing] = {};
    long long recorded = 0;  // pairs recorded since the last read
    double sum_ms = 0.0;     // folded pairs
    long long folded = 0;
};

// Mode X per-launch work buffers, owned by the scene handle (gi_capi.cpp) and grown on demand:
// the list of pixel slots left after the background test and, for spp > 1, every listed pixel's
// per-sample radiance (summed in sample order by k_x_reduce).
struct XScratch {
    unsigned* list = nullptr;   // cap entries
    double* part = nullptr;     // cap * spp * 3 doubles
    long long cap = 0;          // pixel slots the buffers hold
    int spp = 0;                // samples per pixel the part buffer was sized for
    // wavefront Mode X (gi_wf.hip): two path queues of wcap entries (SoA: 12 fp64 fields + a
    // (list index, sample) pair = 104 B per entry) and 2 device counters per bounce
    double* wq[2] = {nullptr, nullptr};
    unsigned* wid[2] = {nullptr, nullptr};
    unsigned* wcnt = nullptr;
    long long wcap = 0;
    // flat Mode R (gi_kernels.hip k_rf_*): candidate pairs, one word each -- every tile's own region
    // of GI_RF_S0, then the pool of rf_pages pages of GI_RF_PAGE (rf_pairs holds both); per tile its
    // pool page ids (GI_RF_KMAX), its pairs / hits and its first chunk of hits; per pixel slot the best
    // rank + 1 and the primary direction; the counters (pool pages taken, overflowed tiles) and the
    // overflowed tiles' list; the segment offsets and hit counts.  Sized for rf_slots pixel slots.
    unsigned* rf_pairs = nullptr;
    unsigned* rf_pt = nullptr;
    unsigned long long* rf_best = nullptr;
    double* rf_dir = nullptr;
    unsigned* rf_cnt = nullptr;
    unsigned* rf_ovf = nullptr;
    unsigned* rf_rcnt = nullptr;
    unsigned* rf_soff = nullptr;    // per tile + 1: its first segment of pairs (k_rf_hit's unit)
    unsigned* rf_shc = nullptr;     // per segment: its hits
    unsigned* rf_sreg = nullptr;    // per segment: its tile
    unsigned* rf_hoff = nullptr;    // per segment + 1: the hits before it (k_rf_reach's chunks of 64)
    unsigned rf_pages = 0;
    long long rf_slots = 0;
    size_t rf_bytes = 0;
    long long rf_failed = 0;   // pixel slots for which the allocation failed (0: none): not retried for
                               // that many or more; such frames render through k_mode_r_batch
};

// Mode X launch configuration, computed once per scene when it is created (gi_capi.cpp, on the
// scene's device): kernel variant, dynamic LDS bytes and the resident persistent grid.
struct XLaunchCfg {
    int kv = 0;              // kernel variant: 2 * (LDS-resident scene) + (4 waves per SIMD)
    size_t lds_bytes = 0;    // dynamic LDS per workgroup
    int resident = 1;        // resident 256-thread workgroups on the device (occupancy x CUs)
    size_t wf_lds_bytes = 0; // wavefront Mode X (k_wf_bounce, k_seg): dynamic LDS per workgroup
    int wf_resident = 1;     //   and the resident workgroups of k_wf_bounce
    int seg_resident = 1;    //   and of k_seg
};

}  // namespace gi
