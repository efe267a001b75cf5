// gi_wf.hip — Mode X in wavefront form (WF): one kernel launch per bounce over a compacted queue of
// live paths, instead of the persistent path-state machine of k_mode_x (gi_kernels.hip).
//
// Per bounce b every lane of a wave runs the same sequence on one path (the per-pixel
// body raytracer.h:41-84 extended by the build-defined integrator, DESIGN.md "Mode X"):
//   closest-hit traversal -> hit point, light direction -> shadow any-hit traversal -> shading
//   (texture, Blinn-Phong with the shadow answer) -> L += T * local -> next direction (mirror /
//   cosine-weighted) -> the path is appended to the next bounce's queue, or its radiance stored.
// The queue is compacted with one ballot + prefix count + one atomic per wave (paths that end drop
// out), so bounce b + 1 launches over exactly the live paths.  Bounce 0 enumerates the work list's
// (pixel, sample) units directly (no queue: a primary ray is regenerated from its unit).  Path
// records are SoA in HBM (o, d, L, T in fp64 + (list index, sample): 104 B); a frame whose units
// exceed a queue's capacity runs in chunks of units, each chunk depth launches.
//
// Results: every path runs exactly the oracle's operations (oracle/gi_oracle.cpp sample_mode_x);
// the closest hit is the minimum of (t, primitive index) whatever the traversal order, and the
// per-sample radiance rows are summed in sample order by k_x_reduce as for k_mode_x -- so frames
// are bit-identical to k_mode_x's and the oracle's (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>

#include "gi.h"
#include "gi_dev.h"
#include "gi_scene.h"

namespace gi {
namespace {

#ifndef GI_WF_MIN_WAVES_LDS
#define GI_WF_MIN_WAVES_LDS 4   // LDS-resident scenes, light shading (<= 128 VGPRs)
#endif
#ifndef GI_WF_MIN_WAVES
#define GI_WF_MIN_WAVES 3       // other scenes
#endif
#ifndef GI_WF_PSL
// a path's L and T wait out the two traversals in a per-lane LDS slot (column layout, 6 x 256 fp64 per
// workgroup) instead of VGPRs: the 4-wave kernel stays within 128 VGPRs
#define GI_WF_PSL 1
#endif
constexpr size_t kWfSlotBytes = GI_WF_PSL ? 6 * 256 * sizeof(double) : 0;

// one queue of path records: field f (o.xyz, d.xyz, L.xyz, T.xyz) of entry j at r[f * cap + j]
struct WFQ {
    double* r;
    uint2* id;   // (work-list index, sample)
    long long cap;
};

// Closest hit (ANY = false: the (t, primitive) minimum over t > MX_TMIN) or any hit before tmax
// (ANY: a shadow ray; true on the first primitive found) of the ray o + t d through the 8-wide BVH.
// Stackless: 8-bit "children left" mask per level (SH: one 64-bit word, trees of <= 8 levels);
// climbing by parent pointers (LDS-resident scenes) or the per-lane level stack nst (HBM).
// PAIR: leaf records two at a time (two interleaved fp64 chains; LDS records); otherwise global
// records fetched one ahead of their test.  RECULL (closest, LDS): a popped child is re-tested
// against the current best t (its box is a ds_read away).
template <bool ANY, bool PAIR, bool AXIS, bool SH, bool TRI, bool NST, typename NodeP, typename HotP>
__device__ __forceinline__ int wf_trace(NodeP W, HotP H, V3 o, V3 d, double tmax, bool act, int* nst, double& t_out,
                                        uint32_t& nnode, uint32_t& nprim) {
    const F3 of = f3((float)o.x, (float)o.y, (float)o.z);
    const F3 ivf = inv_dir(d);
    const int dmask = (d.x < 0 ? 1 : 0) | (d.y < 0 ? 2 : 0) | (d.z < 0 ? 4 : 0);
    double tb = tmax;
    float tbf = up32(tmax);
    int best = -1;
    uint64_t mlo = 0, mhi = 0;
    int node = 0, level = 0;
    bool raying = false;
    if (act) {
        const uint32_t rm = children_mask<AXIS>(W, of, ivf, tbf, dmask);
        lvl_set<SH>(mlo, mhi, 0, rm);
        raying = rm != 0;
    }
    while (raying) {
        const auto* nd = W + node;
        const uint32_t msk = lvl_get<SH>(mlo, mhi, level);
        const int kc = __builtin_ctz(msk);   // next child in front-to-back order
        lvl_set<SH>(mlo, mhi, level, msk & (msk - 1));
        const int c = kc ^ dmask;
        const int ch = nd->child[c];
        bool keep = true;
        if (!ANY && PAIR && best >= 0) keep = child_hit(nd, c, of, ivf, tbf);
        if (keep) {
            if (ch < 0) {   // leaf: the fp64 primitive tests decide
                const int cnt = nd->cnt[c];
                const auto* hp = H + ~ch;
                if constexpr (PAIR) {
                    for (int j = 0; j < cnt; j += 2) {
                        const bool two = j + 1 < cnt;
                        const XHotR r0 = load_hot(hp + j), r1 = load_hot(hp + (two ? j + 1 : j));
                        const double ta = x_prim_t<TRI>(r0.h, o, d, MX_TMIN);
                        const double tq = two ? x_prim_t<TRI>(r1.h, o, d, MX_TMIN) : INFINITY;
                        nprim += two ? 2 : 1;
                        if (ANY) {
                            if (ta < tmax || tq < tmax) {
                                best = ta < tmax ? r0.h.prim : r1.h.prim;
                                break;
                            }
                        } else {
                            if (ta < tb || (ta == tb && r0.h.prim < best)) { tb = ta; best = r0.h.prim; }
                            if (tq < tb || (tq == tb && r1.h.prim < best)) { tb = tq; best = r1.h.prim; }
                            tbf = up32(tb);
                        }
                    }
                } else {
                    XHotR cur = load_hot(hp);
                    for (int j = 0; j < cnt; ++j) {
                        const XHotR rec = cur;
                        if (j + 1 < cnt) cur = load_hot(hp + j + 1);
                        ++nprim;
                        const double t = x_prim_t<TRI>(rec.h, o, d, MX_TMIN);
                        if (ANY) {
                            if (t < tmax) { best = rec.h.prim; break; }
                        } else if (t < tb || (t == tb && rec.h.prim < best)) {
                            tb = t;
                            best = rec.h.prim;
                            tbf = up32(t);
                        }
                    }
                }
            } else {        // interior: descend if any of its children is hit (fp32 slabs)
                ++nnode;
                const uint32_t cm = children_mask<AXIS>(W + ch, of, ivf, tbf, dmask);
                if (cm) {
                    node = ch;
                    ++level;
                    lvl_set<SH>(mlo, mhi, level, cm);
                    if (NST) nst[level * 256] = ch;
                }
            }
        }
        if (ANY && best >= 0) break;
        uint32_t rest = lvl_get<SH>(mlo, mhi, level);
        if (rest == 0 && level > 0) {   // climb to the nearest level with children left
            if constexpr (NST) {
                const uint64_t lm = level >= 8 ? mlo : mlo & ((1ull << (8 * level)) - 1);
                const uint64_t hm = level <= 8 ? 0ull : mhi & ((1ull << (8 * (level - 8))) - 1);
                level = hm ? 8 + (63 - __clzll((long long)hm)) / 8 : lm ? (63 - __clzll((long long)lm)) / 8 : 0;
                rest = lvl_get<SH>(mlo, mhi, level);
                node = level == 0 ? 0 : nst[level * 256];
            } else {
                do {
                    --level;
                    node = level == 0 ? 0 : W[node].parent;   // the root is node 0: no load
                    rest = lvl_get<SH>(mlo, mhi, level);
                } while (rest == 0 && level > 0);
            }
        }
        raying = rest != 0;
    }
    t_out = tb;
    return best;
}

struct WFArgs {
    const unsigned* list;      // k_x_classify's work list (pixel slots, tile order)
    const unsigned* n_list;    // its length (device)
    double* part;              // per-sample radiance rows (spp > 1)
    unsigned* take;            // this bounce's input entries handed out (device counter)
    const unsigned* n_in;      // this bounce's input length (bounce > 0: the previous bounce's n_out)
    unsigned* n_out;           // entries appended to qout
    unsigned long long u0, u1; // bounce 0: the chunk's units [u0, u1) of n_list * spp
};

// One bounce of every live path.  Persistent grid: each wave takes 64 queue entries with one atomic
// until the queue is exhausted.  LDS: the scene (wide nodes, leaf records, primitives, entities) is
// staged in LDS by each workgroup, as in k_mode_x; otherwise HBM-resident (CN: quantised nodes).
template <bool STATS, bool LDS, bool W4, bool SH, bool TRI, bool CN>
__global__ __launch_bounds__(256, (LDS && W4) ? GI_WF_MIN_WAVES_LDS : GI_WF_MIN_WAVES) void k_wf_bounce(
    DevScene sc, CamDev cam, V3 light, TileMap m, int spp, int depth, uint64_t seed, int b, double* rgb, uint8_t* rgb8,
    unsigned long long* stats, WFArgs a, WFQ qin, WFQ qout, int xflags) {
    // the bounce's input length: bounce 0, the chunk's units of the work list; else the queue
    unsigned n_in;
    if (b == 0) {
        const unsigned long long tot = (unsigned long long)*a.n_list * (unsigned long long)spp;
        n_in = (unsigned)(min(tot, a.u1) > a.u0 ? min(tot, a.u1) - a.u0 : 0ull);
    } else {
        n_in = *a.n_in;
    }
    if (*(volatile unsigned*)a.take >= n_in) return;   // nothing left (before staging the scene)
    extern __shared__ int4 lds_dyn[];
    const XWNode* LW = nullptr;
    const XHot* LH = nullptr;
    const XPrim* XP = sc.xprims;
    const REnt* EN = sc.ents;
    int* nst = nullptr;
    double* pl = nullptr;   // GI_WF_PSL: this lane's L (fields 0-2) and T (3-5), pl[f * 256]
    if constexpr (LDS) {
        const int nw = sc.n_xwnodes * (int)(sizeof(XWNode) / sizeof(int4));
        const int nh = sc.n_xhot * (int)(sizeof(XHot) / sizeof(int4));
        const int np = sc.n_xprims * (int)(sizeof(XPrim) / sizeof(int4));
        const int ne = sc.n_ents * (int)(sizeof(REnt) / sizeof(int4));
        const int4* gw = reinterpret_cast<const int4*>(sc.xwnodes);
        const int4* gh = reinterpret_cast<const int4*>(sc.xhot);
        const int4* gp = reinterpret_cast<const int4*>(sc.xprims);
        const int4* ge = reinterpret_cast<const int4*>(sc.ents);
        for (int i = threadIdx.x; i < nw; i += blockDim.x) lds_dyn[i] = gw[i];
        for (int i = threadIdx.x; i < nh; i += blockDim.x) lds_dyn[nw + i] = gh[i];
        for (int i = threadIdx.x; i < np; i += blockDim.x) lds_dyn[nw + nh + i] = gp[i];
        for (int i = threadIdx.x; i < ne; i += blockDim.x) lds_dyn[nw + nh + np + i] = ge[i];
        __syncthreads();
        LW = reinterpret_cast<const XWNode*>(lds_dyn);
        LH = reinterpret_cast<const XHot*>(lds_dyn + nw);
        XP = reinterpret_cast<const XPrim*>(lds_dyn + nw + nh);
        EN = reinterpret_cast<const REnt*>(lds_dyn + nw + nh + np);
        pl = reinterpret_cast<double*>(lds_dyn + nw + nh + np + ne) + threadIdx.x;
    } else {
        nst = reinterpret_cast<int*>(lds_dyn) + threadIdx.x;   // 16 levels x 256 lanes
        pl = reinterpret_cast<double*>(reinterpret_cast<int*>(lds_dyn) + 16 * 256) + threadIdx.x;
    }
    const bool no_shadow = (xflags & 4) != 0;
    const int lane = threadIdx.x & 63;
    uint32_t nnode = 0, nprim = 0, nrays = 0, nres = 0, npx = 0;
    const long long qc = qin.cap, oc = qout.cap;
    for (;;) {
        unsigned base = 0;
        if (lane == 0) base = atomicAdd(a.take, 64u);
        base = __shfl(base, 0);
        if (base >= n_in) break;
        const unsigned j = base + (unsigned)lane;
        bool act = j < n_in;
        unsigned li = 0, smp = 0;
        V3 o = cam.pos, d = v3(1, 0, 0), L = v3(0, 0, 0), T = v3(1, 1, 1);
        long long idx = -1;
        int x = 0, y = 0;
        uint64_t key = 0;
        if (act) {
            if (b == 0) {
                const unsigned long long u = a.u0 + j;
                if (u < (1ull << 32)) {   // 32-bit division where it suffices
                    li = (unsigned)u / (unsigned)spp;
                    smp = (unsigned)u - li * (unsigned)spp;
                } else {
                    li = (unsigned)(u / (unsigned long long)spp);
                    smp = (unsigned)(u - (unsigned long long)li * (unsigned long long)spp);
                }
            } else {
                const uint2 id = qin.id[j];
                li = id.x;
                smp = id.y;
                const double* r = qin.r + j;
                o = v3(r[0], r[qc], r[2 * qc]);
                d = v3(r[3 * qc], r[4 * qc], r[5 * qc]);
                L = v3(r[6 * qc], r[7 * qc], r[8 * qc]);
                T = v3(r[9 * qc], r[10 * qc], r[11 * qc]);
            }
            const unsigned ps = a.list[li];
            slot_pixel(m, (long long)(ps >> 6), (int)(ps & 63), idx, x, y);
            y += m.y0;
            if (spp > 1) idx = (long long)li;   // the per-sample radiance row
            key = mx_key(seed, (uint64_t)y * (uint64_t)m.w + (uint64_t)x);
            if (b == 0) {   // the unit's primary ray
                double jx = 0.0, jy = 0.0;
                if (spp > 1) {
                    jx = mx_u01k(key, smp, 0xFFFF, 0);
                    jy = mx_u01k(key, smp, 0xFFFF, 1);
                }
                const V3 d0 = primary_dir(cam, (double)x + jx, (double)y + jy);
                if (smp == 0) ++npx;
                // conservative fp32 test of the scene's root box on the unnormalised direction: a
                // miss adds exactly +0 (the oracle traces it and adds L = 0)
                const F3 iv0 = f3(__builtin_amdgcn_rcpf((float)d0.x), __builtin_amdgcn_rcpf((float)d0.y),
                                  __builtin_amdgcn_rcpf((float)d0.z));
                if (!root_hit(sc, f3((float)cam.pos.x, (float)cam.pos.y, (float)cam.pos.z), iv0)) {
                    ++nrays;
                    ++nres;
                    act = false;
                    if (spp > 1) {
                        double* q = a.part + 3 * ((size_t)idx * (size_t)spp + (size_t)smp);
                        q[0] = 0.0; q[1] = 0.0; q[2] = 0.0;
                    } else {
                        if (rgb) { rgb[3 * idx] = 0.0; rgb[3 * idx + 1] = 0.0; rgb[3 * idx + 2] = 0.0; }
                        if (rgb8) { rgb8[3 * idx] = 0; rgb8[3 * idx + 1] = 0; rgb8[3 * idx + 2] = 0; }
                    }
                } else {
                    d = normalize(d0);
                }
            }
            if (GI_WF_PSL) {
                pl[0] = L.x; pl[256] = L.y; pl[512] = L.z;
                pl[768] = T.x; pl[1024] = T.y; pl[1280] = T.z;
            }
        }
        // ---- closest hit
        double tbest = INFINITY;
        int best;
        if constexpr (LDS) best = wf_trace<false, true, true, SH, TRI, false>(LW, LH, o, d, INFINITY, act, nst, tbest, nnode, nprim);
        else if constexpr (CN) best = wf_trace<false, false, false, SH, TRI, true>(sc.xcnodes, sc.xhot, o, d, INFINITY, act, nst, tbest, nnode, nprim);
        else best = wf_trace<false, false, false, SH, TRI, true>(sc.xwnodes, sc.xhot, o, d, INFINITY, act, nst, tbest, nnode, nprim);
        if (act) ++nrays;
        const bool hit = act && best >= 0;
        // ---- the hit point and its shadow ray toward the point light
        V3 P = o, Ld = v3(0, 0, 1);
        double ldist = 0.0;
        if (hit) {
            P = o + tbest * d;
            const V3 lv = light - P;
            ldist = gsqrt(dot(lv, lv));
            Ld = normalize(lv);
        }
        bool occl = false;
        if (!no_shadow) {
            double tdummy;
            int sb;
            if constexpr (LDS) sb = wf_trace<true, true, true, SH, TRI, false>(LW, LH, P, Ld, ldist, hit, nst, tdummy, nnode, nprim);
            else if constexpr (CN) sb = wf_trace<true, false, false, SH, TRI, true>(sc.xcnodes, sc.xhot, P, Ld, ldist, hit, nst, tdummy, nnode, nprim);
            else sb = wf_trace<true, false, false, SH, TRI, true>(sc.xwnodes, sc.xhot, P, Ld, ldist, hit, nst, tdummy, nnode, nprim);
            occl = sb >= 0;
        }
        // ---- shading (the oracle's operations: local = ambient, + diffuse + specular when lit)
        bool cont = false;
        if (hit) {
            ++nrays;   // the shadow ray
            if (GI_WF_PSL) {
                L = v3(pl[0], pl[256], pl[512]);
                T = v3(pl[768], pl[1024], pl[1280]);
            }
            const XPrim& p = XP[best];   // the facing normal (after the shadow ray: fewer live values)
            V3 N = (TRI || p.kind == 0) ? ld3(p.n) : normalize(P - ld3(p.a));
            if (!(dot(d, N) < 0)) N = -N;
            const REnt& e = EN[p.ent];
            int32_t tu, tv;
            x_texcoord<TRI>(sc, e, P, tu, tv);
            const V3 tc = texel(ld3(e.color), tu, tv);
            const V3 la = tc * e.shader[0];
            V3 loc = la;
            if (!occl) {
                const V3 ldf = (smax(0.0, dot(N, Ld)) * (tc * 0.5)) * e.shader[1];
                const V3 bis = normalize(normalize(-d) + Ld);
                const double spw = mx_pow(smax(0.0, dot(N, bis)), e.spec_pow);
                const V3 ls = v3(spw, spw, spw) * e.shader[2];
                loc = (la + ldf) + ls;
            }
            L = L + vmul(T, v3(smin(loc.x, 1.0), smin(loc.y, 1.0), smin(loc.z, 1.0)));
            if (b != depth - 1) {
                // mirror bounce with probability e.refl (uniform dim 4): T unchanged, d reflected
                // about the facing normal; otherwise T *= texel / 2 and a cosine-weighted direction
                if (e.refl > 0.0 && mx_u01k(key, smp, b, 4) < e.refl) {
                    d = normalize(d - N * (2.0 * dot(d, N)));
                    cont = true;
                } else {
                    T = vmul(T, tc * 0.5);
                    if (!(T.x == 0.0 && T.y == 0.0 && T.z == 0.0)) {
                        double sx, sy, r2;   // concentric disk + Malley
                        mx_disk(mx_u01k(key, smp, b, 2), mx_u01k(key, smp, b, 3), sx, sy, r2);
                        const double sz = gsqrt(1.0 - r2);
                        const double sg = N.z >= 0.0 ? 1.0 : -1.0;   // Duff et al. 2017 basis
                        const double aa = -1.0 / (sg + N.z);
                        const double bb = N.x * N.y * aa;
                        const V3 bt1 = v3(1.0 + sg * N.x * N.x * aa, sg * bb, -sg * N.x);
                        const V3 bt2 = v3(bb, sg + N.y * N.y * aa, -N.y);
                        d = normalize((bt1 * sx + bt2 * sy) + N * sz);
                        cont = true;
                    }
                }
                o = P;
            }
        }
        // ---- live paths to the next bounce's queue: one atomic per wave, entries in lane order
        const unsigned long long mc = __ballot(cont);
        if (mc) {
            const int leader = __ffsll((long long)mc) - 1;
            unsigned ob = 0;
            if (lane == leader) ob = atomicAdd(a.n_out, (unsigned)__popcll(mc));
            ob = __shfl(ob, leader);
            if (cont) {
                const unsigned k = ob + (unsigned)__popcll(mc & ((1ull << lane) - 1));
                qout.id[k] = make_uint2(li, smp);
                double* r = qout.r + k;
                r[0] = o.x; r[oc] = o.y; r[2 * oc] = o.z;
                r[3 * oc] = d.x; r[4 * oc] = d.y; r[5 * oc] = d.z;
                r[6 * oc] = L.x; r[7 * oc] = L.y; r[8 * oc] = L.z;
                r[9 * oc] = T.x; r[10 * oc] = T.y; r[11 * oc] = T.z;
            }
        }
        // ---- paths that end here: the sample's radiance (k_x_reduce sums a pixel's samples in
        // order) or, with one sample, the pixel itself
        if (act && !cont) {
            if (GI_WF_PSL && !hit) L = v3(pl[0], pl[256], pl[512]);
            if (spp > 1) {
                double* q = a.part + 3 * ((size_t)idx * (size_t)spp + (size_t)smp);
                q[0] = L.x; q[1] = L.y; q[2] = L.z;
            } else {
                const double c0 = smin((0.0 + L.x) / 1.0, 1.0), c1 = smin((0.0 + L.y) / 1.0, 1.0),
                             c2 = smin((0.0 + L.z) / 1.0, 1.0);
                if (rgb) { rgb[3 * idx] = c0; rgb[3 * idx + 1] = c1; rgb[3 * idx + 2] = c2; }
                if (rgb8) quantize(c0, c1, c2, rgb8 + 3 * idx);
            }
        }
    }
    if (STATS) {
        wave_add_stats(stats, nrays, nnode, nprim, npx);
        uint64_t r = nres;
        for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off);
        if (lane == 0 && r) atomicAdd(stats + GI_STAT_X_RESOLVED, (unsigned long long)r);
    }
}

}  // namespace

// dynamic LDS of the bounce kernel beyond the scene / level stack: the per-lane path slots
size_t wf_slot_bytes() { return kWfSlotBytes; }

// resident workgroups per CU of the bounce kernel launch_wf picks for this scene
hipError_t wf_occupancy(const DevScene& sc, int kv, size_t lds_bytes, int* per_cu) {
    const bool lds = kv >= 2, w4 = kv == 3, sh = sc.x_max_depth <= 7, tr = sc.x_tri_only != 0;
    const bool cn = !lds && sc.xcnodes != nullptr;
    const void* f = lds ? (w4 ? (sh ? reinterpret_cast<const void*>(k_wf_bounce<false, true, true, true, true, false>)
                                    : reinterpret_cast<const void*>(k_wf_bounce<false, true, true, false, true, false>))
                              : (sh ? reinterpret_cast<const void*>(k_wf_bounce<false, true, false, true, false, false>)
                                    : reinterpret_cast<const void*>(k_wf_bounce<false, true, false, false, false, false>)))
                  : cn ? (tr ? reinterpret_cast<const void*>(k_wf_bounce<false, false, false, false, true, true>)
                             : reinterpret_cast<const void*>(k_wf_bounce<false, false, false, false, false, true>))
                       : (tr ? reinterpret_cast<const void*>(k_wf_bounce<false, false, false, false, true, false>)
                             : reinterpret_cast<const void*>(k_wf_bounce<false, false, false, false, false, false>));
    return hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, f, 256, lds_bytes);
}

// The wavefront Mode X pass (after k_x_classify, before k_x_reduce): reads the work list's length
// back to the host (one stream synchronisation), then per chunk of units `depth` bounce launches.
// kv: 2 * LDS-resident + light-shading (XLaunchCfg::kv).  Counters: 2 per bounce (take, n_out),
// zeroed per chunk.
hipError_t launch_wf(const DevScene& sc, int kv, size_t lds_bytes, int resident, const CamDev& cam, V3 light, int w,
                     int h, int y0, const gi_opts& o, double* rgb, uint8_t* rgb8, const XScratch& xs,
                     const unsigned* n_list_dev, unsigned long long* stats, int xflags, hipStream_t stream,
                     hipEvent_t ev_begin, hipEvent_t ev_end) {
    const TileMap m = make_map(w, h, o.shard_count, o.shard_index, y0);
    hipError_t e = hipMemcpyAsync(xs.h_nlist, n_list_dev, sizeof(unsigned), hipMemcpyDeviceToHost, stream);
    if (e == hipSuccess) e = hipStreamSynchronize(stream);
    if (e != hipSuccess) return e;
    const unsigned long long units = (unsigned long long)*xs.h_nlist * (unsigned long long)o.spp;
    const int depth = o.depth;
    const bool lds = kv >= 2, w4 = kv == 3;
    const bool sh = sc.x_max_depth <= 7;
    const bool cn = !lds && sc.xcnodes != nullptr;
    const bool tr = sc.x_tri_only != 0;
    const size_t lbytes = lds_bytes;
    const dim3 grid((unsigned)std::max(1, resident)), block(256);
    if (ev_begin) (void)hipEventRecord(ev_begin, stream);
    for (unsigned long long u0 = 0; u0 < units; u0 += (unsigned long long)xs.wcap) {
        e = hipMemsetAsync(xs.wcnt, 0, 2 * (size_t)depth * sizeof(unsigned), stream);
        if (e != hipSuccess) return e;
        for (int b = 0; b < depth; ++b) {
            WFArgs a;
            a.list = xs.list;
            a.n_list = n_list_dev;
            a.part = xs.part;
            a.take = xs.wcnt + 2 * b;
            a.n_in = b > 0 ? xs.wcnt + 2 * (b - 1) + 1 : nullptr;
            a.n_out = xs.wcnt + 2 * b + 1;
            a.u0 = u0;
            a.u1 = std::min(units, u0 + (unsigned long long)xs.wcap);
            WFQ qin, qout;
            qin.cap = qout.cap = xs.wcap;
            qin.r = xs.wq[(b + 1) & 1];
            qin.id = reinterpret_cast<uint2*>(xs.wid[(b + 1) & 1]);
            qout.r = xs.wq[b & 1];
            qout.id = reinterpret_cast<uint2*>(xs.wid[b & 1]);
#define GI_WF_LAUNCH(S, L, W, SHV, T, C) hipLaunchKernelGGL((k_wf_bounce<S, L, W, SHV, T, C>), grid, block, lbytes, stream, sc, cam, \
                                                  light, m, o.spp, depth, o.seed, b, rgb, rgb8, stats, a, qin, qout, xflags)
#define GI_WF_S(S)                                                                                   \
    do {                                                                                             \
        if (lds) {                                                                                   \
            if (w4) { if (sh) GI_WF_LAUNCH(S, true, true, true, true, false); else GI_WF_LAUNCH(S, true, true, false, true, false); } \
            else { if (sh) GI_WF_LAUNCH(S, true, false, true, false, false); else GI_WF_LAUNCH(S, true, false, false, false, false); } \
        } else if (cn) {                                                                             \
            if (tr) GI_WF_LAUNCH(S, false, false, false, true, true); else GI_WF_LAUNCH(S, false, false, false, false, true); \
        } else {                                                                                     \
            if (tr) GI_WF_LAUNCH(S, false, false, false, true, false); else GI_WF_LAUNCH(S, false, false, false, false, false); \
        }                                                                                            \
    } while (0)
            if (stats) GI_WF_S(true);
            else GI_WF_S(false);
#undef GI_WF_S
#undef GI_WF_LAUNCH
        }
    }
    if (ev_end) (void)hipEventRecord(ev_end, stream);
    return hipGetLastError();
}

}  // namespace gi
