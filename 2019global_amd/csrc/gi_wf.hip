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
#include <type_traits>

#include "gi.h"
#include "gi_dev.h"
#include "gi_scene.h"

namespace gi {
namespace {

constexpr long long kWfTile = 8;   // pixel tiles are 8 x 8 (GI_TILE)

#ifndef GI_WF_MIN_WAVES_LDS
#define GI_WF_MIN_WAVES_LDS 4   // LDS-resident scenes, light shading (<= 128 VGPRs)
#endif
#ifndef GI_WF_MIN_WAVES
#define GI_WF_MIN_WAVES 3       // other scenes
#endif
#ifndef GI_WF_TAKE
#define GI_WF_TAKE 16   // most 64-entry batches a wave takes per atomic on the queue's counter
#endif
// a path's L and T wait out the two traversals in a per-lane LDS slot (column layout, 6 x 256 fp64 per
// workgroup) instead of VGPRs: the 4-wave kernel stays within 128 VGPRs.  k_seg also keeps the path's
// RNG key, its output index and sample, and its bounce there (fields 6, 7, 8), read where they are
// used: carried in VGPRs across the traversals they were spilled to scratch (136 -> 56 B per lane).
// LDS-resident scenes test leaf records two at a time (PAIR: two interleaved fp64 chains) and their
// node slab tests issue the 12 loads at once (round 5: C3 4.90 -> 4.81 ms against axis by axis)
constexpr size_t kWfSlotBytes = 9 * 256 * sizeof(double);

// a path's identity where the shading needs it: RNG key, sample, bounce
struct PathId {
    uint64_t key;
    unsigned smp;
    int b;
};
__device__ __forceinline__ void slot_put_u64(double* pl, int f, uint64_t v) { reinterpret_cast<uint64_t*>(pl)[f * 256] = v; }
__device__ __forceinline__ uint64_t slot_get_u64(const double* pl, int f) { return reinterpret_cast<const uint64_t*>(pl)[f * 256]; }

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
// PAIR: leaf records two at a time (two interleaved fp64 chains; LDS records); otherwise records
// fetched one ahead of their test.  LDS-resident scenes (!NST), closest hit: a popped child is
// re-tested against the current best t (its box is a ds_read away).
template <bool ANY, bool PAIR, bool AXIS, bool SH, bool TRI, bool NST, typename NodeP, typename HotP>
__device__ __forceinline__ int wf_trace(NodeP W, HotP H, V3 o, V3 d, double tmax, bool act, int* nst, double& t_out,
                                        uint32_t& nnode, uint32_t& nprim, uint32_t& nsteps, int skip = 254) {
    // the own-plane skip (XWNode scenes; gi_build.cpp assign_plane_groups): leaves of group skip are
    // never entered -- their exact tests would all find t below MX_TMIN for this ray
    constexpr bool kSkip = std::is_same<NodeP, const XWNode*>::value;
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
        uint32_t rm;
        if constexpr (kSkip) rm = children_mask<AXIS, true>(W, of, ivf, tbf, dmask, skip);
        else rm = children_mask<AXIS>(W, of, ivf, tbf, dmask);
        lvl_set<SH>(mlo, mhi, 0, rm);
        raying = rm != 0;
    }
    while (raying) {
        ++nsteps;
        const auto* nd = W + node;
        const uint32_t msk = lvl_get<SH>(mlo, mhi, level);
        const int kc = __builtin_ctz(msk);   // next child in front-to-back order
        lvl_set<SH>(mlo, mhi, level, msk & (msk - 1));
        const int c = kc ^ dmask;
        bool keep = true;
        if (!ANY && !NST && best >= 0) {   // (LDS scenes) re-cull against the current best t
            keep = child_hit(nd, c, of, ivf, tbf);
        }
        const int ch = nd->child[c];
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
                            if ((ta < tmax) | (tq < tmax)) {
                                best = ta < tmax ? r0.h.prim : r1.h.prim;
                                break;
                            }
                        } else {   // (selects, not branches: | and & do not short-circuit)
                            const bool ua = (ta < tb) | ((ta == tb) & (r0.h.prim < best));
                            tb = ua ? ta : tb;
                            best = ua ? r0.h.prim : best;
                            const bool uq = (tq < tb) | ((tq == tb) & (r1.h.prim < best));
                            tb = uq ? tq : tb;
                            best = uq ? r1.h.prim : best;
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
                        } else {
                            const bool u = (t < tb) | ((t == tb) & (rec.h.prim < best));
                            tb = u ? t : tb;
                            best = u ? rec.h.prim : best;
                            tbf = u ? up32(t) : tbf;
                        }
                    }
                }
            } else {        // interior: descend if any of its children is hit (fp32 slabs)
                ++nnode;
                uint32_t cm;
                if constexpr (kSkip) cm = children_mask<AXIS, true>(W + ch, of, ivf, tbf, dmask, skip);
                else cm = children_mask<AXIS>(W + ch, of, ivf, tbf, dmask);
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
    unsigned long long u0, u1; // bounce 0: the chunk's units [u0, u1) of n_list * ns
    unsigned s0, ns;           // the launch's samples [s0, s0 + ns) of the spp (0, spp; or a progressive pass)
};

// The scene views of a bounce / segment kernel.  LDS: wide nodes, leaf records, primitives and
// entities staged in LDS by the workgroup (as k_mode_x does); then the per-lane path slots.
// HBM-resident scenes: the per-lane level stack (16 x 256 ints), then the path slots.
struct WFView {
    const XWNode* LW = nullptr;
    const XHot* LH = nullptr;
    const XPrim* XP = nullptr;
    const REnt* EN = nullptr;
    int* nst = nullptr;
    double* pl = nullptr;   // this lane's L (fields 0-2) and T (3-5), pl[f * 256]
};
template <bool LDS>
__device__ __forceinline__ WFView wf_stage(const DevScene& sc, int4* lds_dyn) {
    WFView v;
    v.XP = sc.xprims;
    v.EN = sc.ents;
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
        v.LW = reinterpret_cast<const XWNode*>(lds_dyn);
        v.LH = reinterpret_cast<const XHot*>(lds_dyn + nw);
        v.XP = reinterpret_cast<const XPrim*>(lds_dyn + nw + nh);
        v.EN = reinterpret_cast<const REnt*>(lds_dyn + nw + nh + np);
        v.pl = reinterpret_cast<double*>(lds_dyn + nw + nh + np + ne) + threadIdx.x;
    } else {
        v.nst = reinterpret_cast<int*>(lds_dyn) + threadIdx.x;   // 16 levels x 256 lanes
        v.pl = reinterpret_cast<double*>(reinterpret_cast<int*>(lds_dyn) + 16 * 256) + threadIdx.x;
    }
    return v;
}

// The unit (work-list index li, sample smp) of a pixel's sample: its pixel, RNG key and primary
// direction (the reference's corner ray, jittered for spp > 1).  idx: the output slot (the
// per-sample radiance row for spp > 1, else the pixel).
__device__ __forceinline__ V3 wf_primary(const CamDev& cam, const TileMap& m, unsigned ps, int spp, uint64_t seed,
                                         unsigned li, unsigned smp, long long& idx, uint64_t& key) {
    int x = 0, y = 0;   // ps: the work list's entry li (the pixel slot)
    slot_pixel(m, (long long)(ps >> 6), (int)(ps & 63), idx, x, y);
    y += m.y0;
    if (spp > 1) idx = (long long)li;
    key = mx_key(seed, (uint64_t)y * (uint64_t)m.w + (uint64_t)x);
    double jx = 0.0, jy = 0.0;
    if (spp > 1) {
        jx = mx_u01k(key, smp, 0xFFFF, 0);
        jy = mx_u01k(key, smp, 0xFFFF, 1);
    }
    return primary_dir(cam, (double)x + jx, (double)y + jy);
}
// conservative fp32 test of the scene's root box on the unnormalised primary direction: a miss adds
// exactly +0 (the oracle traces it and adds L = 0)
__device__ __forceinline__ bool wf_primary_misses(const DevScene& sc, const CamDev& cam, V3 d0) {
    const F3 iv0 = f3(__builtin_amdgcn_rcpf((float)d0.x), __builtin_amdgcn_rcpf((float)d0.y), __builtin_amdgcn_rcpf((float)d0.z));
    return !root_hit(sc, f3((float)cam.pos.x, (float)cam.pos.y, (float)cam.pos.z), iv0);
}
// the path's radiance once it ends: its per-sample row (spp > 1; k_x_reduce adds a pixel's rows in
// sample order) or, with one sample, the pixel: min((0 + L) / 1, 1), the reduce pass's operations
__device__ __forceinline__ void wf_store(double* part, double* rgb, uint8_t* rgb8, int spp, long long idx, unsigned smp, V3 L) {
    if (spp > 1) {
        double* q = part + 3 * ((size_t)idx * (size_t)spp + (size_t)smp);
        q[0] = L.x; q[1] = L.y; q[2] = L.z;
    } else {
        const double c0 = smin((0.0 + L.x) / 1.0, 1.0), c1 = smin((0.0 + L.y) / 1.0, 1.0), c2 = smin((0.0 + L.z) / 1.0, 1.0);
        if (rgb) { rgb[3 * idx] = c0; rgb[3 * idx + 1] = c1; rgb[3 * idx + 2] = c2; }
        if (rgb8) quantize(c0, c1, c2, rgb8 + 3 * idx);
    }
}

// One path segment, bounce b (every lane of the wave runs the same sequence): closest hit -> hit
// point and light direction -> shadow any-hit -> texture and Blinn-Phong with the shadow answer ->
// L += T * local -> the next direction (mirror with probability refl, else T *= texel / 2 and a
// cosine-weighted direction).  The oracle's operations (sample_mode_x).  In: o, d and (in the lane's
// path slot) the path's L and T.  Out: true when the path continues (o, d set to its next ray; L, T in
// registers and in the slot); false when it ends (L final).
// STATS: the wave's traversal-loop iterations (closest, shadow) and the lanes' own steps, summed into
// ws (lane 0) -- the divergence profile of a segment
struct WFSegStats {
    uint64_t it_c = 0, ln_c = 0, it_s = 0, ln_s = 0, segs = 0, live = 0, iters = 0;
    uint64_t cyc_c = 0, cyc_s = 0, cyc_sh = 0, cyc_ref = 0, cyc_all = 0;   // wave clock cycles per phase
};
__device__ __forceinline__ void wf_wave_steps(uint32_t n, uint64_t& it, uint64_t& ln) {
    uint32_t mx = n, sm = n;
    for (int off = 32; off > 0; off >>= 1) {
        mx = max(mx, (uint32_t)__shfl_xor(mx, off));
        sm += __shfl_xor(sm, off);
    }
    if ((threadIdx.x & 63) == 0) { it += mx; ln += sm; }
}
template <bool STATS, bool LDS, bool SH, bool TRI, bool CN, typename KeyF>
__device__ __forceinline__ bool x_segment(const DevScene& sc, const WFView& v, const V3& light, int depth, bool no_shadow, bool act,
                                          const KeyF& id_of, V3& o, V3& d, V3& L, V3& T,
                                          uint32_t& nnode, uint32_t& nprim, uint32_t& nrays, WFSegStats& ws,
                                          double skip_cos = 2.0, int* splane = nullptr) {
    uint32_t st_steps = 0;
    uint64_t c0 = STATS ? clock64() : 0;
    V3 P = o, Ld = v3(0, 0, 1);
    bool occl = false;
    // ---- closest hit
    double tbest = INFINITY;
    int best;
    // the own-plane skip of this ray (k_seg carries it from the previous segment; 254: none)
    const int skip_c = splane ? *splane : 254;
    if constexpr (LDS) best = wf_trace<false, true, false, SH, TRI, false>(v.LW, v.LH, o, d, INFINITY, act, v.nst, tbest, nnode, nprim, st_steps, skip_c);
    else if constexpr (CN) best = wf_trace<false, false, false, SH, TRI, true>(sc.xcnodes, sc.xhot, o, d, INFINITY, act, v.nst, tbest, nnode, nprim, st_steps);
    else best = wf_trace<false, false, false, SH, TRI, true>(sc.xwnodes, sc.xhot, o, d, INFINITY, act, v.nst, tbest, nnode, nprim, st_steps, skip_c);
    if (act) ++nrays;
    if (STATS) {
        wf_wave_steps(st_steps, ws.it_c, ws.ln_c);
        st_steps = 0;
        const uint64_t c1 = clock64();
        ws.cyc_c += c1 - c0;
        c0 = c1;
    }
    const bool hit = act && best >= 0;
    // ---- the hit point and its shadow ray toward the point light
    double ldist = 0.0;
    int pg = 254;   // the hit's plane group: the shadow ray and the next ray leave its plane
    V3 pn = v3(0, 0, 1);
    if (hit) {
        P = o + tbest * d;
        const V3 lv = light - P;
        ldist = gsqrt(dot(lv, lv));
        Ld = normalize(lv);
        const XPrim& px = v.XP[best];
        pg = px.pad[0] < 254 ? px.pad[0] : 254;
        pn = ld3(px.n);
    }
    if (!no_shadow) {
        double tdummy;
        int sb;
        const int skip_s = (pg < 254 && fabs(dot(Ld, pn)) >= skip_cos) ? pg : 254;
        if constexpr (LDS) sb = wf_trace<true, true, false, SH, TRI, false>(v.LW, v.LH, P, Ld, ldist, hit, v.nst, tdummy, nnode, nprim, st_steps, skip_s);
        else if constexpr (CN) sb = wf_trace<true, false, false, SH, TRI, true>(sc.xcnodes, sc.xhot, P, Ld, ldist, hit, v.nst, tdummy, nnode, nprim, st_steps);
        else sb = wf_trace<true, false, false, SH, TRI, true>(sc.xwnodes, sc.xhot, P, Ld, ldist, hit, v.nst, tdummy, nnode, nprim, st_steps, skip_s);
        occl = sb >= 0;
        if (STATS) wf_wave_steps(st_steps, ws.it_s, ws.ln_s);
    }
    if (STATS) {
        const uint64_t c1 = clock64();
        ws.cyc_s += c1 - c0;
        c0 = c1;
    }
    {   // every lane: a lane without a path never uses them, so L and T are dead during
        L = v3(v.pl[0], v.pl[256], v.pl[512]);      // the traversals (conditioned on act, the register copies
        T = v3(v.pl[768], v.pl[1024], v.pl[1280]);  // stayed live for inactive lanes and were spilled)
    }
    // ---- shading (local = ambient, + diffuse + specular when lit)
    bool cont = false;
    if (hit) {
        ++nrays;   // the shadow ray
        const XPrim& p = v.XP[best];   // the facing normal (after the shadow ray: fewer live values)
        V3 N = (TRI || p.kind == 0) ? ld3(p.n) : normalize(P - ld3(p.a));
        N = dot(d, N) < 0 ? N : -N;
        const REnt& e = v.EN[p.ent];
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
        const PathId id = id_of();   // (k_seg: from the lane's slot)
        const uint64_t key = id.key;
        const unsigned smp = id.smp;
        const int b = id.b;
        if (b != depth - 1) {
            if (e.refl > 0.0 && mx_u01k(key, smp, b, 4) < e.refl) {   // mirror: T unchanged
                d = normalize(d - N * (2.0 * dot(d, N)));
                cont = true;
            } else {
                T = vmul(T, tc * 0.5);
                if (!((T.x == 0.0) & (T.y == 0.0) & (T.z == 0.0))) {
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
        if (cont) {
            v.pl[0] = L.x; v.pl[256] = L.y; v.pl[512] = L.z;
            v.pl[768] = T.x; v.pl[1024] = T.y; v.pl[1280] = T.z;
            if (splane) *splane = (pg < 254 && fabs(dot(d, pn)) >= skip_cos) ? pg : 254;
        }
    }
    if (STATS) ws.cyc_sh += clock64() - c0;
    return cont;
}

// One bounce of every live path (the wavefront form).  Persistent grid: each wave takes GI_WF_TAKE
// batches of 64 queue entries per atomic until the queue is exhausted.
template <bool STATS, bool LDS, bool W4, bool SH, bool TRI, bool CN>
__global__ __launch_bounds__(256, (LDS && W4) ? GI_WF_MIN_WAVES_LDS : GI_WF_MIN_WAVES) void k_wf_bounce(
    DevScene sc, CamDev cam, V3 light, TileMap m, int spp, int depth, uint64_t seed, int b, double* rgb, uint8_t* rgb8,
    unsigned long long* stats, WFArgs a, WFQ qin, WFQ qout, int xflags) {
    // the bounce's input length: bounce 0, the chunk's units of the work list; else the queue
    unsigned n_in;
    if (b == 0) {
        const unsigned long long tot = (unsigned long long)*a.n_list * (unsigned long long)a.ns;
        n_in = (unsigned)(min(tot, a.u1) > a.u0 ? min(tot, a.u1) - a.u0 : 0ull);
    } else {
        n_in = *a.n_in;
    }
    if (*(volatile unsigned*)a.take >= n_in) return;   // nothing left (before staging the scene)
    extern __shared__ int4 lds_dyn[];
    const WFView v = wf_stage<LDS>(sc, lds_dyn);
    const bool no_shadow = (xflags & 4) != 0;
    const int lane = threadIdx.x & 63;
    uint32_t nnode = 0, nprim = 0, nrays = 0, nres = 0, npx = 0;
    const long long qc = qin.cap, oc = qout.cap;
    // batches per atomic: up to GI_WF_TAKE, fewer when the queue has fewer than about 8 runs per
    // resident wave (small queues: every wave gets work)
    const unsigned take = (unsigned)max(1u, min((unsigned)GI_WF_TAKE, n_in / (64u * 8u * (gridDim.x * (blockDim.x >> 6)))));
    unsigned base = 0, left = 0;   // the wave's current run of take x 64 entries
    for (;;) {
        if (left == 0) {
            if (lane == 0) base = atomicAdd(a.take, 64u * take);
            base = __shfl(base, 0);
            left = take;
        }
        if (base >= n_in) break;
        const unsigned j = base + (unsigned)lane;
        base += 64u;
        --left;
        bool act = j < n_in;
        unsigned li = 0, smp = 0;
        V3 o = cam.pos, d = v3(1, 0, 0), L = v3(0, 0, 0), T = v3(1, 1, 1);
        long long idx = -1;
        uint64_t key = 0;
        if (act) {
            if (b == 0) {
                const unsigned long long u = a.u0 + j;
                if (u < (1ull << 32)) {   // 32-bit division where it suffices
                    li = (unsigned)u / a.ns;
                    smp = a.s0 + ((unsigned)u - li * a.ns);
                } else {
                    li = (unsigned)(u / (unsigned long long)a.ns);
                    smp = a.s0 + (unsigned)(u - (unsigned long long)li * (unsigned long long)a.ns);
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
            const V3 d0 = wf_primary(cam, m, a.list[li], spp, seed, li, smp, idx, key);
            if (b == 0) {   // the unit's primary ray
                if (smp == 0) ++npx;
                if (wf_primary_misses(sc, cam, d0)) {
                    ++nrays;
                    ++nres;
                    act = false;
                    wf_store(a.part, rgb, rgb8, spp, idx, smp, v3(0, 0, 0));
                } else {
                    d = normalize(d0);
                }
            }
            v.pl[0] = L.x; v.pl[256] = L.y; v.pl[512] = L.z;
            v.pl[768] = T.x; v.pl[1024] = T.y; v.pl[1280] = T.z;
        }
        WFSegStats ws;
        // (the queue carries no plane: the closest ray is not skipped here, the shadow ray is)
        const double skip_cos = sc.x_skip_a * fmax(fabs(cam.pos.x), fmax(fabs(cam.pos.y), fabs(cam.pos.z))) + sc.x_skip_b;
        int splane = 254;
        const bool cont = x_segment<false, LDS, SH, TRI, CN>(sc, v, light, depth, no_shadow, act, [&] { return PathId{key, smp, b}; }, o, d, L, T,
                                                             nnode, nprim, nrays, ws, skip_cos, &splane);
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
        if (act && !cont) wf_store(a.part, rgb, rgb8, spp, idx, smp, L);
    }
    if (STATS) {
        wave_add_stats(stats, nrays, nnode, nprim, npx);
        uint64_t r = nres;
        for (int off = 32; off > 0; off >>= 1) r += __shfl_xor(r, off);
        if (lane == 0 && r) atomicAdd(stats + GI_STAT_X_RESOLVED, (unsigned long long)r);
    }
}

// The segment-synchronous form (SEG): one persistent kernel in which every loop iteration is one
// whole path segment (x_segment) for every lane of the wave -- the wavefront form's uniform per-lane
// sequence, with the path state kept in registers / the lane's LDS slot instead of HBM queues, and
// no launch per bounce.  A lane whose path ends takes the next (pixel, sample) unit at the top of
// the next iteration (units handed out from the wave's run, one atomic per run);
// primary rays that miss the scene's root box are resolved there, up to GI_SEG_BURST per lane.
#ifndef GI_SEG_BURST
#define GI_SEG_BURST 16
#endif
#ifndef GI_SEG_TAKE
#define GI_SEG_TAKE 2       // k_seg: most batches of 64 units per run (one atomic per run)
#endif
#ifndef GI_SEG_TAKE_TRI
#define GI_SEG_TAKE_TRI 1   // the same for LDS-resident triangle-only scenes (the Cornell box)
#endif
template <bool STATS, bool LDS, bool W4, bool SH, bool TRI, bool CN>
__global__ __launch_bounds__(256, (LDS && W4) ? GI_WF_MIN_WAVES_LDS : GI_WF_MIN_WAVES) void k_seg(
    DevScene sc, CamDev cam, V3 light, TileMap m, int spp, int depth, uint64_t seed, double* rgb, uint8_t* rgb8,
    unsigned long long* stats, WFArgs a, int xflags) {
    extern __shared__ int4 lds_dyn[];
    const WFView v = wf_stage<LDS>(sc, lds_dyn);
    const bool no_shadow = (xflags & 4) != 0;
    const int lane = threadIdx.x & 63;
    const unsigned long long total = (unsigned long long)*a.n_list * (unsigned long long)a.ns;
    // run length: up to GI_SEG_TAKE batches of 64 units per atomic (background-heavy frames burn units
    // fast: longer runs, fewer atomics on the one counter), fewer when the launch has less than about
    // 8 runs per resident wave (small launches: every wave gets work).  Round 5, after the spill fix
    // (profiles/r05_ab.txt): 4 -> 2 batches gives C3 5.09 -> 4.95 ms and X-zoo 4.35-4.43 -> 4.17-4.19,
    // X-main and the 1k soup unchanged; 1 batch gives C3 4.89-4.90 but X-main 0.38 -> 0.69 and X-zoo
    // 4.67 (their frames are background-heavy or shading-heavy), so 1 only for LDS-resident
    // triangle-only scenes.  Guided self-scheduling -- run sizes from a relaxed read of the counter --
    // measured 1.2-2.6x slower (the read waits behind the atomics on that L2 line).
    constexpr long long kTake = (LDS && TRI) ? GI_SEG_TAKE_TRI : GI_SEG_TAKE;
    const unsigned long long n_waves = (unsigned long long)gridDim.x * (blockDim.x >> 6);
    const unsigned long long run = 64ull * (unsigned long long)max(1ll, min(kTake, (long long)(total / (64ull * 8ull * n_waves))));
    uint32_t nnode = 0, nprim = 0, nrays = 0, nres = 0, npx = 0;
    unsigned long long cur = 0, cur_end = 0;   // the wave's unhanded units [cur, cur_end) (uniform)
    bool exhausted = false;                    // the frame's units are all handed out (uniform)
    bool live = false;                         // this lane carries a path
    unsigned li = 0, smp = 0;
    long long idx = -1;
    uint64_t key = 0;
    V3 o = cam.pos, d = v3(1, 0, 0), L = v3(0, 0, 0), T = v3(1, 1, 1);
    int splane = 254;   // the own-plane skip of the lane's next ray (254: none; primary rays)
    // (gi_build.cpp assign_plane_groups: the bound on |d . n| above which a surface's own plane is skipped)
    const double skip_cos = sc.x_skip_a * fmax(fabs(cam.pos.x), fmax(fabs(cam.pos.y), fabs(cam.pos.z))) + sc.x_skip_b;
    WFSegStats ws;
    const uint64_t t_begin = STATS ? clock64() : 0;
    for (;;) {
        if (STATS && lane == 0) ++ws.iters;
        const uint64_t t_ref = STATS ? clock64() : 0;
        // ---- lanes without a path take units (primary rays; background samples resolved here)
        for (int burst = 0; burst < GI_SEG_BURST; ++burst) {
            const unsigned long long m_need = __ballot(!live);
            if (m_need == 0 || (exhausted && cur >= cur_end)) break;
            const unsigned rank = (unsigned)__popcll(m_need & ((1ull << lane) - 1));
            const unsigned n_need = (unsigned)__popcll(m_need);
            unsigned long long u = ~0ull;
            const unsigned long long avail = cur_end - cur;
            if (n_need > avail && !exhausted) {   // a new run of units for the lanes beyond it
                unsigned long long nb = 0;
                if (lane == 0) nb = atomicAdd(reinterpret_cast<unsigned long long*>(a.take), run);
                nb = __shfl(nb, 0);
                if (nb >= total) {
                    exhausted = true;
                    if (!live && rank < avail) u = cur + rank;
                    cur = cur_end;
                } else {
                    const unsigned long long ne = min(total, nb + run);
                    if (!live) {
                        if (rank < avail) u = cur + rank;
                        else if (nb + (rank - avail) < ne) u = nb + (rank - avail);
                    }
                    cur = min(ne, nb + (n_need - avail));
                    cur_end = ne;
                    if (ne == total) exhausted = true;
                }
            } else {
                if (!live && rank < avail) u = cur + rank;
                cur += min((unsigned long long)n_need, avail);
            }
            unsigned li_u = 0, smp_u = 0;
            if (u != ~0ull) {
                if (u < (1ull << 32)) {
                    li_u = (unsigned)u / a.ns;
                    smp_u = a.s0 + ((unsigned)u - li_u * a.ns);
                } else {
                    li_u = (unsigned)(u / (unsigned long long)a.ns);
                    smp_u = a.s0 + (unsigned)(u - (unsigned long long)li_u * (unsigned long long)a.ns);
                }
            }
            if (!live && u != ~0ull) {
                li = li_u;
                smp = smp_u;
                const unsigned ps = a.list[li];   // (prefetching a run's entries into lanes: +3%, round 4)
                const V3 d0 = wf_primary(cam, m, ps, spp, seed, li, smp, idx, key);
                if (smp == 0) ++npx;
                if (wf_primary_misses(sc, cam, d0)) {
                    ++nrays;
                    ++nres;
                    wf_store(a.part, rgb, rgb8, spp, idx, smp, v3(0, 0, 0));
                } else {
                    live = true;
                    o = cam.pos;
                    d = normalize(d0);
                    splane = 254;
                    L = v3(0, 0, 0);
                    T = v3(1, 1, 1);
                    v.pl[0] = 0.0; v.pl[256] = 0.0; v.pl[512] = 0.0;
                    v.pl[768] = 1.0; v.pl[1024] = 1.0; v.pl[1280] = 1.0;
                    slot_put_u64(v.pl, 6, key);
                    slot_put_u64(v.pl, 7, (uint64_t)(uint32_t)idx | ((uint64_t)smp << 32));   // (idx < 2^32: work-list index or pixel)
                    slot_put_u64(v.pl, 8, 0ull);
                }
            }
        }
        if (STATS) ws.cyc_ref += clock64() - t_ref;
        if (__ballot(live) == 0) {
            if (exhausted && cur >= cur_end) break;
            continue;
        }
        // ---- one segment of every live path
        if (STATS) {
            const unsigned long long ml = __ballot(live);
            if (lane == 0) { ++ws.segs; ws.live += __popcll(ml); }
        }
        const bool cont = x_segment<STATS, LDS, SH, TRI, CN>(
            sc, v, light, depth, no_shadow, live,
            [&] { return PathId{slot_get_u64(v.pl, 6), (unsigned)(slot_get_u64(v.pl, 7) >> 32), (int)slot_get_u64(v.pl, 8)}; },
            o, d, L, T, nnode, nprim, nrays, ws, skip_cos, &splane);
        if (live) {
            if (cont) {
                slot_put_u64(v.pl, 8, slot_get_u64(v.pl, 8) + 1);
            } else {
                const uint64_t is = slot_get_u64(v.pl, 7);
                wf_store(a.part, rgb, rgb8, spp, (long long)(uint32_t)is, (unsigned)(is >> 32), L);
                live = false;
            }
        }
    }
    if (STATS && lane == 0) {   // the segment divergence profile (bench "schedule")
        atomicAdd(stats + GI_STAT_X_ITERS, (unsigned long long)ws.iters);
        atomicAdd(stats + GI_STAT_X_HANDLE, (unsigned long long)ws.segs);
        atomicAdd(stats + GI_STAT_X_HLANES, (unsigned long long)ws.live);
        atomicAdd(stats + GI_STAT_X_IT_LEAF, (unsigned long long)ws.it_c);
        atomicAdd(stats + GI_STAT_X_LN_LEAF, (unsigned long long)ws.ln_c);
        atomicAdd(stats + GI_STAT_X_IT_NODE, (unsigned long long)ws.it_s);
        atomicAdd(stats + GI_STAT_X_LN_NODE, (unsigned long long)ws.ln_s);
        atomicAdd(stats + GI_STAT_X_CYC_TRAV, (unsigned long long)(ws.cyc_c + ws.cyc_s));
        atomicAdd(stats + GI_STAT_X_IT_RS, (unsigned long long)ws.cyc_c);   // (k_seg: closest-trace cycles)
        atomicAdd(stats + GI_STAT_X_CYC_HIT, (unsigned long long)ws.cyc_sh);
        atomicAdd(stats + GI_STAT_X_CYC_NEXT, (unsigned long long)ws.cyc_ref);
        atomicAdd(stats + GI_STAT_X_CYC_ALL, (unsigned long long)(clock64() - t_begin));
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
// the scene's share of that LDS (LDS-resident scenes): the staged records (entity records included:
// read from global memory by the shading instead, C3 4.65 -> 4.69 ms, and 5 waves per SIMD with them
// there, 96 VGPRs and 120 B of scratch, 4.79 ms; profiles/r06_ab.txt)
size_t wf_scene_lds_bytes(const DevScene& sc) { return (size_t)sc.x_lds_bytes; }

// The kernel variant for a scene: f(LDS, W4, SH, TRI, CN) with each a std::integral_constant<bool>
// (kv: 2 * LDS-resident + light-shading, XLaunchCfg::kv)
template <typename F>
void wf_dispatch(const DevScene& sc, int kv, F&& f) {
    using B = std::true_type;
    using N = std::false_type;
    const bool lds = kv >= 2, w4 = kv == 3, sh = sc.x_max_depth <= 7, tr = sc.x_tri_only != 0;
    const bool cn = !lds && sc.xcnodes != nullptr;
    if (lds) {
        if (w4) { if (sh) f(B{}, B{}, B{}, B{}, N{}); else f(B{}, B{}, N{}, B{}, N{}); }
        else { if (sh) f(B{}, N{}, B{}, N{}, N{}); else f(B{}, N{}, N{}, N{}, N{}); }
    } else if (cn) {
        if (tr) f(N{}, N{}, N{}, B{}, B{}); else f(N{}, N{}, N{}, N{}, B{});
    } else {
        if (tr) f(N{}, N{}, N{}, B{}, N{}); else f(N{}, N{}, N{}, N{}, N{});
    }
}

// resident workgroups per CU of the kernel a form (1: k_wf_bounce, 2: k_seg) runs for this scene
hipError_t wf_occupancy(const DevScene& sc, int kv, size_t lds_bytes, int form, int* per_cu) {
    hipError_t e = hipSuccess;
    wf_dispatch(sc, kv, [&](auto L, auto W, auto SHt, auto T, auto C) {
        constexpr bool l = decltype(L)::value, w = decltype(W)::value, sh = decltype(SHt)::value,
                       t = decltype(T)::value, c = decltype(C)::value;
        const void* f = form == 2 ? reinterpret_cast<const void*>(k_seg<false, l, w, sh, t, c>)
                                  : reinterpret_cast<const void*>(k_wf_bounce<false, l, w, sh, t, c>);
        e = hipOccupancyMaxActiveBlocksPerMultiprocessor(per_cu, f, 256, lds_bytes);
    });
    return e;
}

// The Mode X pass after k_x_classify and before k_x_reduce in the wavefront forms.
//  form 1 (wavefront): per chunk of units (the queue capacity; chunks for the launch's every pixel
//    slot, those past the work list's end return at once on the device) `depth` bounce launches;
//    counters: 2 per bounce (take, n_out), zeroed per chunk.
//  form 2 (segment-synchronous): one persistent launch; counter: a 64-bit unit count at xs.wcnt.
hipError_t launch_wf(const DevScene& sc, int kv, size_t lds_bytes, int resident, int form, const CamDev& cam, V3 light,
                     int w, int h, int y0, const gi_opts& o, double* rgb, uint8_t* rgb8, const XScratch& xs,
                     const unsigned* n_list_dev, unsigned long long* stats, int xflags, hipStream_t stream,
                     hipEvent_t ev_begin, hipEvent_t ev_end) {
    const TileMap m = make_map(w, h, o.shard_count, o.shard_index, y0);
    const int depth = o.depth;
    const int s0 = o.sample_end > 0 ? o.sample_begin : 0, s1 = o.sample_end > 0 ? o.sample_end : o.spp;
    const dim3 grid((unsigned)std::max(1, resident)), block(256);
    hipError_t e = hipSuccess;
    if (form == 2) {   // (the unit counter xs.wcnt[0..1] was zeroed by k_x_classify)
        WFArgs a{};
        a.list = xs.list;
        a.n_list = n_list_dev;
        a.part = xs.part;
        a.take = xs.wcnt;
        a.s0 = (unsigned)s0;
        a.ns = (unsigned)(s1 - s0);
        if (ev_begin) (void)hipEventRecord(ev_begin, stream);
        wf_dispatch(sc, kv, [&](auto L, auto W, auto SHt, auto T, auto C) {
            constexpr bool l = decltype(L)::value, wv = decltype(W)::value, sh = decltype(SHt)::value,
                           t = decltype(T)::value, c = decltype(C)::value;
            if (stats) hipLaunchKernelGGL((k_seg<true, l, wv, sh, t, c>), grid, block, lds_bytes, stream, sc, cam, light, m, o.spp, depth, o.seed, rgb, rgb8, stats, a, xflags);
            else hipLaunchKernelGGL((k_seg<false, l, wv, sh, t, c>), grid, block, lds_bytes, stream, sc, cam, light, m, o.spp, depth, o.seed, rgb, rgb8, stats, a, xflags);
        });
        if (ev_end) (void)hipEventRecord(ev_end, stream);
        return hipGetLastError();
    }
    // chunks for every pixel slot of the launch listed (the list's length stays on the device: no host
    // synchronisation, so the form can be captured in a graph); a chunk beyond the listed units' end
    // finds no input on the device and its bounce kernels return at once
    const unsigned long long units = (unsigned long long)m.n_local * (unsigned long long)(kWfTile * kWfTile) *
                                     (unsigned long long)(s1 - s0);
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
            a.s0 = (unsigned)s0;
            a.ns = (unsigned)(s1 - s0);
            WFQ qin, qout;
            qin.cap = qout.cap = xs.wcap;
            qin.r = xs.wq[(b + 1) & 1];
            qin.id = reinterpret_cast<uint2*>(xs.wid[(b + 1) & 1]);
            qout.r = xs.wq[b & 1];
            qout.id = reinterpret_cast<uint2*>(xs.wid[b & 1]);
            wf_dispatch(sc, kv, [&](auto L, auto W, auto SHt, auto T, auto C) {
                constexpr bool l = decltype(L)::value, wv = decltype(W)::value, sh = decltype(SHt)::value,
                               t = decltype(T)::value, c = decltype(C)::value;
                if (stats) hipLaunchKernelGGL((k_wf_bounce<true, l, wv, sh, t, c>), grid, block, lds_bytes, stream, sc, cam, light, m, o.spp, depth, o.seed, b, rgb, rgb8, stats, a, qin, qout, xflags);
                else hipLaunchKernelGGL((k_wf_bounce<false, l, wv, sh, t, c>), grid, block, lds_bytes, stream, sc, cam, light, m, o.spp, depth, o.seed, b, rgb, rgb8, stats, a, qin, qout, xflags);
            });
        }
    }
    if (ev_end) (void)hipEventRecord(ev_end, stream);
    return hipGetLastError();
}

}  // namespace gi
