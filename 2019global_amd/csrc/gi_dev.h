// gi_dev.h — device code shared by the gfx950 kernel translation units (gi_kernels.hip: Mode R and
// the persistent Mode X kernel; gi_wf.hip: the wavefront Mode X kernels): camera, tile map, the
// Mode X wide-node / leaf-record tests and texture mapping.  Header-only (internal linkage per TU).
#pragma once
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>
#include <type_traits>

#include "gi.h"
#include "gi_scene.h"

namespace gi {
struct CamDev {
    V3 pos, up, left, top_left;
    double rx, ry;
};

namespace {

constexpr int kTile = GI_TILE;
constexpr int kWavesPerBlock = 4;

__device__ __forceinline__ void wave_add_stats(unsigned long long* stats, uint64_t a, uint64_t b, uint64_t c, uint64_t px) {
    for (int off = 32; off > 0; off >>= 1) {
        a += __shfl_xor(a, off);
        b += __shfl_xor(b, off);
        c += __shfl_xor(c, off);
        px += __shfl_xor(px, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAdd(stats + GI_STAT_RAYS, (unsigned long long)a);
        atomicAdd(stats + GI_STAT_NODES, (unsigned long long)b);
        atomicAdd(stats + GI_STAT_PRIMS, (unsigned long long)c);
        atomicAdd(stats + GI_STAT_PIXELS, (unsigned long long)px);
    }
}

struct TileMap {
    int w, h, tiles_x;
    int y0;   // absolute row of the band's first row (progressive gi_render bands)
    long long n_tiles, n_local;
    int shard_count, shard_index;
};

// pixel of this lane; returns false when the lane has no pixel
__device__ __forceinline__ bool lane_pixel(const TileMap& m, long long lt, long long& out_idx, int& x, int& y) {
    const int lane = threadIdx.x & 63;
    if (lt >= m.n_local) return false;
    const long long t = (long long)m.shard_index + lt * m.shard_count;
    if (t >= m.n_tiles) { out_idx = -1; return false; }
    const unsigned tu = (unsigned)t, tyu = tu / (unsigned)m.tiles_x;   // 32-bit: see slot_pixel
    const int ty = (int)tyu, tx = (int)(tu - tyu * (unsigned)m.tiles_x);
    x = tx * kTile + (lane & 7);
    y = ty * kTile + (lane >> 3);
    if (m.shard_count == 1) out_idx = (long long)y * m.w + x;
    else out_idx = lt * (kTile * kTile) + lane;
    return x < m.w && y < m.h;
}

// pixel of slot j (0..63) of local tile lt (row-major 8x8 inside the tile); false: no pixel there
__device__ __forceinline__ bool slot_pixel(const TileMap& m, long long lt, int j, long long& out_idx, int& x, int& y) {
    out_idx = -1;
    const long long t = (long long)m.shard_index + lt * m.shard_count;
    if (t >= m.n_tiles) return false;
    // tile counts stay below 2^32 (check_opts caps a frame at 2^34 pixels, i.e. 2^28 tiles), so
    // the tile row / column come from a 32-bit division (a 64-bit one is a long software routine)
    const unsigned tu = (unsigned)t, tyu = tu / (unsigned)m.tiles_x;
    const int ty = (int)tyu, tx = (int)(tu - tyu * (unsigned)m.tiles_x);
    x = tx * kTile + (j & 7);
    y = ty * kTile + (j >> 3);
    if (m.shard_count == 1) out_idx = (long long)y * m.w + x;
    else out_idx = lt * (kTile * kTile) + j;
    return x < m.w && y < m.h;
}

__host__ __device__ inline TileMap make_map(int w, int h, int shard_count, int shard_index, int y0 = 0) {
    TileMap m;
    m.w = w;
    m.h = h;
    m.y0 = y0;
    m.tiles_x = (w + kTile - 1) / kTile;
    const long long tiles_y = (h + kTile - 1) / kTile;
    m.n_tiles = (long long)m.tiles_x * tiles_y;
    m.shard_count = shard_count;
    m.shard_index = shard_index;
    m.n_local = (m.n_tiles + shard_count - 1) / shard_count;
    return m;
}

__device__ __forceinline__ V3 primary_dir(const CamDev& c, double fx, double fy) {
    // raytracer.h:41: top_left - left*x*res.x - up*y*res.y
    return (c.top_left - (c.left * fx) * c.rx) - (c.up * fy) * c.ry;
}

// ---------------------------------------------------------------------------------------------
// Mode X
// ---------------------------------------------------------------------------------------------
struct F3 {
    float x, y, z;
};
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ F3 f3(float x, float y, float z) { F3 r; r.x = x; r.y = y; r.z = z; return r; }
// Per-level "children left" masks, 8 bits per level in two 64-bit words.  SH (trees of depth <= 7,
// i.e. at most 8 levels): the low word alone, without the per-access choice of word (C3 -3%, C4 -5%,
// C5 -3%).
template <bool SH = false>
__device__ __forceinline__ uint32_t lvl_get(uint64_t lo, uint64_t hi, int l) {
    if (SH) return (uint32_t)((lo >> (8 * l)) & 0xFF);
    return (uint32_t)((l < 8 ? lo >> (8 * l) : hi >> (8 * (l - 8))) & 0xFF);
}
template <bool SH = false>
__device__ __forceinline__ void lvl_set(uint64_t& lo, uint64_t& hi, int l, uint32_t m) {
    if (SH) { lo = (lo & ~(0xFFull << (8 * l))) | ((uint64_t)m << (8 * l)); return; }
    if (l < 8) lo = (lo & ~(0xFFull << (8 * l))) | ((uint64_t)m << (8 * l));
    else hi = (hi & ~(0xFFull << (8 * (l - 8)))) | ((uint64_t)m << (8 * (l - 8)));
}

// smallest float >= v (conservative culling bound)
__device__ __forceinline__ float up32(double v) {
    float f = (float)v;
    if ((double)f < v) f = __int_as_float(__float_as_int(f) + (f >= 0.0f ? 1 : -1));
    return f;
}

// One leaf record in registers: fetched by 5 independent 16-byte loads (one memory round trip),
// so no load waits on a branch of the test.
struct XHotR {
    union {
        int4 q[5];
        XHot h;
    };
};
__device__ __forceinline__ XHotR load_hot(const XHot* p) {
    const int4* s = reinterpret_cast<const int4*>(p);
    XHotR r;
#pragma unroll
    for (int i = 0; i < 5; ++i) r.q[i] = s[i];
    return r;
}

// Möller–Trumbore, two-sided, barycentric tests on the numerators (no 1/det); all products are
// formed before the first branch.  Spheres (kind 1): the geometric quadratic.
// TRI: the scene's primitives are all triangles (kernels chosen per scene): the sphere branch and the
// kind test vanish, so a leaf test is one straight block the compiler schedules as a whole
template <bool TRI = false>
__device__ __forceinline__ double x_prim_t(const XHot& p, V3 o, V3 d, double tmin) {
    if (TRI || p.kind == 0) {
        const V3 e1 = ld3(p.b), e2 = ld3(p.c), v0 = ld3(p.a);
        const V3 pv = fcross(d, e2);
        const double det = fdot(e1, pv);
        const V3 tv = o - v0;
        const double un = fdot(tv, pv);
        const V3 qv = fcross(tv, e1);
        const double vn = fdot(d, qv);
        const double uvn = un + vn;
        const bool pos = det > 0.0;
        // the comparisons combined with | and & (no short circuit: || compiled to nested exec-mask
        // branches, ~35 scalar instructions and their VALU -> SALU latencies per test) -- the same
        // boolean for every input, NaN included
        const bool miss = (det == 0.0) | (pos & ((un < 0.0) | (un > det) | (vn < 0.0) | (uvn > det))) |
                          (!pos & ((un > 0.0) | (un < det) | (vn > 0.0) | (uvn < det)));
        const double t = fdot(e2, qv) / det;   // branch-free: two tests interleave in the leaf loop
        return (!miss & (t > tmin)) ? t : INFINITY;
    }
    const V3 oc = o - ld3(p.a);
    const double b = fdot(oc, d);
    const double r = p.b[0];
    const double c2 = gfma(-r, r, fdot(oc, oc));
    const double disc = gfma(b, b, -c2);
    if (disc < 0.0) return INFINITY;
    const double sq = gsqrt(disc);
    double t = -b - sq;
    if (t > tmin) return t;
    t = -b + sq;
    return (t > tmin) ? t : INFINITY;
}

// fp32 slab test of child c of a wide node against [0, tmax]; boxes are outward-rounded + padded.
// Slab distances as (b - o) * iv = fma(b, iv, -o*iv): one fma per plane.  Its error in position,
// ~2^-24 (|o| + |b - o|), is the subtraction form's order and far inside the 1e-5 * extent padding
// for origins within the scene's extent (bounce origins; the camera of every scene here).
// fp32 reciprocal direction (1 ulp), clamped to +-1e30 so that an axis-parallel ray gives finite
// plane distances (fma(b, inf, -(o * inf)) would be inf - inf = NaN); with |b - o| >= the box
// padding the clamped distances still exceed any t of the scene, so culling stays conservative
__device__ __forceinline__ F3 inv_dir(V3 d) {
    return f3(__builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf((float)d.x), -1e30f, 1e30f),
              __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf((float)d.y), -1e30f, 1e30f),
              __builtin_amdgcn_fmed3f(__builtin_amdgcn_rcpf((float)d.z), -1e30f, 1e30f));
}
__device__ __forceinline__ F3 neg_oiv(F3 of, F3 ivf) { return f3(-(of.x * ivf.x), -(of.y * ivf.y), -(of.z * ivf.z)); }
// Near / far planes: on axis a a box's entry plane is its min plane when iv_a >= 0 and its max
// plane otherwise, for every box -- fma(b, iv, -o*iv) is monotone in the plane b, rounding included
// -- so t_near = t(near plane) and t_far = t(far plane) with no per-box min / max: exactly the
// interval of the min / max form.  The sign comes from the fp32 reciprocal itself (sm: bit a set
// when iv_a < 0), so a -0 direction component (reciprocal -1e30) is ordered correctly too.
__device__ __forceinline__ int iv_signs(F3 ivf) {
    return (int)((__float_as_uint(ivf.x) >> 31) | ((__float_as_uint(ivf.y) >> 31) << 1) |
                 ((__float_as_uint(ivf.z) >> 31) << 2));
}
__device__ __forceinline__ bool child_hit(const XWNode* nd, int c, F3 of, F3 ivf, float tmax) {
    const F3 no = neg_oiv(of, ivf);
    const int sm = iv_signs(ivf);
    const float* L = &nd->lo[0][0];
    const float* Hh = &nd->hi[0][0];
    const float nx = (sm & 1) ? Hh[c] : L[c], fx = (sm & 1) ? L[c] : Hh[c];
    const float ny = (sm & 2) ? Hh[8 + c] : L[8 + c], fy = (sm & 2) ? L[8 + c] : Hh[8 + c];
    const float nz = (sm & 4) ? Hh[16 + c] : L[16 + c], fz = (sm & 4) ? L[16 + c] : Hh[16 + c];
    const float tn = fmaxf(fmaxf(__builtin_fmaf(nx, ivf.x, no.x), __builtin_fmaf(ny, ivf.y, no.y)),
                           fmaxf(__builtin_fmaf(nz, ivf.z, no.z), 0.0f));
    const float tf = fminf(fminf(__builtin_fmaf(fx, ivf.x, no.x), __builtin_fmaf(fy, ivf.y, no.y)),
                           fminf(__builtin_fmaf(fz, ivf.z, no.z), tmax));
    return tn <= tf;
}
__device__ __forceinline__ bool box32_hit(const XBox& b, F3 of, F3 ivf, float tmax) {
    const float tx0 = (b.lo[0] - of.x) * ivf.x, tx1 = (b.hi[0] - of.x) * ivf.x;
    const float ty0 = (b.lo[1] - of.y) * ivf.y, ty1 = (b.hi[1] - of.y) * ivf.y;
    const float tz0 = (b.lo[2] - of.z) * ivf.z, tz1 = (b.hi[2] - of.z) * ivf.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fminf(fmaxf(tx0, tx1), fmaxf(ty0, ty1)), fminf(fmaxf(tz0, tz1), tmax));
    return tn <= tf;
}
// bit c of m moved to bit c ^ dm (three conditional swaps of bit groups)
__device__ __forceinline__ uint32_t xor_permute8(uint32_t m, int dm) {
    m = (dm & 1) ? (((m << 1) & 0xAAu) | ((m >> 1) & 0x55u)) : m;
    m = (dm & 2) ? (((m << 2) & 0xCCu) | ((m >> 2) & 0x33u)) : m;
    m = (dm & 4) ? (((m << 4) & 0xF0u) | ((m >> 4) & 0x0Fu)) : m;
    return m;
}
// bit c set iff child c is a leaf of plane group `skip` (byte c of the node's pad; gi_build.cpp
// assign_plane_groups): SWAR compare of the 8 bytes with skip, zero bytes gathered to bits
__device__ __forceinline__ uint32_t plane_bits(const XWNode* nd, int skip) {
    const uint32_t s4 = (uint32_t)skip * 0x01010101u;
    uint32_t r = 0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        const uint32_t x = (uint32_t)nd->pad[h] ^ s4;
        const uint32_t z = ~(((x & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | x | 0x7F7F7F7Fu);   // 0x80 in the zero bytes
        r |= (((z >> 7) & 1u) | ((z >> 14) & 2u) | ((z >> 21) & 4u) | ((z >> 28) & 8u)) << (4 * h);
    }
    return r;
}
// mask of hit, existing children with bit k for child k ^ dmask (bit order = front-to-back).
// The node's 48 bounds are fetched by 12 independent 16-byte loads (one memory round trip) and
// all 8 slab tests run branch-free; existence comes from the node's precomputed bit mask.
// AXIS: the slab tests accumulate axis by axis (4 float4 live instead of 12: fewer VGPRs at the
// node step, which lets the LDS-resident kernel run 4 waves per SIMD); otherwise all 12 loads are
// issued at once (one memory round trip: the HBM-resident kernel's choice).  Same mask either way.
// SKIP: the leaf children of plane group skip left out (the own-plane skip; skip 254 matches none).
template <bool AXIS, bool SKIP = false>
__device__ __forceinline__ uint32_t children_mask(const XWNode* nd, F3 of, F3 ivf, float tmax, int dmask, int skip = 254) {
    const float4* b = reinterpret_cast<const float4*>(nd);
    const uint32_t ex = SKIP ? ((uint32_t)nd->exists & ~plane_bits(nd, skip)) : (uint32_t)nd->exists;
    const F3 no = neg_oiv(of, ivf);
    const int sm = iv_signs(ivf);   // near / far planes per axis (see child_hit)
    if constexpr (AXIS) {
    float tn[8], tf[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) { tn[c] = 0.0f; tf[c] = tmax; }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        // the near and far planes' quads addressed directly (lo at quad 2a, hi at 6 + 2a)
        const int nq = ((sm >> a) & 1) ? 6 + 2 * a : 2 * a, fq = ((sm >> a) & 1) ? 2 * a : 6 + 2 * a;
        const float4 n0 = b[nq], n1 = b[nq + 1], f0 = b[fq], f1 = b[fq + 1];
        const float o = a == 0 ? no.x : (a == 1 ? no.y : no.z), iv = a == 0 ? ivf.x : (a == 1 ? ivf.y : ivf.z);
        // children in pairs: one packed fma (v_pk_fma_f32) gives two children's plane distances
        const f32x2 nr[4] = {f32x2{n0.x, n0.y}, f32x2{n0.z, n0.w}, f32x2{n1.x, n1.y}, f32x2{n1.z, n1.w}};
        const f32x2 fr[4] = {f32x2{f0.x, f0.y}, f32x2{f0.z, f0.w}, f32x2{f1.x, f1.y}, f32x2{f1.z, f1.w}};
        const f32x2 iv2 = {iv, iv}, o2 = {o, o};
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const f32x2 t0 = __builtin_elementwise_fma(nr[q], iv2, o2), t1 = __builtin_elementwise_fma(fr[q], iv2, o2);
            tn[2 * q] = fmaxf(tn[2 * q], t0.x);
            tf[2 * q] = fminf(tf[2 * q], t1.x);
            tn[2 * q + 1] = fmaxf(tn[2 * q + 1], t0.y);
            tf[2 * q + 1] = fminf(tf[2 * q + 1], t1.y);
        }
    }
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) m |= tn[c] <= tf[c] ? 1u << c : 0u;
    return xor_permute8(m & ex, dmask);
    } else {
    // all 12 quads at once (one memory round trip), the near and far planes' addressed directly
    float4 q[12];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const int nq = ((sm >> a) & 1) ? 6 + 2 * a : 2 * a, fq = ((sm >> a) & 1) ? 2 * a : 6 + 2 * a;
        q[2 * a] = b[nq];
        q[2 * a + 1] = b[nq + 1];
        q[6 + 2 * a] = b[fq];
        q[6 + 2 * a + 1] = b[fq + 1];
    }
    const float* v = reinterpret_cast<const float*>(q);   // near[3][8] then far[3][8]
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const float nx = v[c], fx = v[24 + c], ny = v[8 + c], fy = v[32 + c], nz = v[16 + c], fz = v[40 + c];
        const float tn = fmaxf(fmaxf(__builtin_fmaf(nx, ivf.x, no.x), __builtin_fmaf(ny, ivf.y, no.y)),
                               fmaxf(__builtin_fmaf(nz, ivf.z, no.z), 0.0f));
        const float tf = fminf(fminf(__builtin_fmaf(fx, ivf.x, no.x), __builtin_fmaf(fy, ivf.y, no.y)),
                               fminf(__builtin_fmaf(fz, ivf.z, no.z), tmax));
        m |= tn <= tf ? 1u << c : 0u;
    }
    return xor_permute8(m & ex, dmask);
    }
}

// Quantised nodes (XCNode, HBM-resident scenes): the 64 bytes the slab tests need arrive in four
// 16-byte loads.  A bound's slab distance is taken straight from its 8-bit q: t = fma(q, 2^e * iv,
// fma(org, iv, -o * iv)) -- the decode fma(q, 2^e, org) and the slab fma folded into one; the
// difference from decoding first is a few fp32 ulps of t, inside the 1e-5 * extent padding that
// the host-checked decoded box already exceeds (the CPU checker runs this form).  Near / far
// planes per axis as for XWNode.
__device__ __forceinline__ float xc_scale(int w, int a) {   // 2^e of axis a (e: signed byte a of w)
    const int e = (int)(int8_t)((w >> (8 * a)) & 0xFF);
    return __int_as_float((e + 127) << 23);
}
__device__ __forceinline__ float xc_q(int lo4, int hi4, int c) {   // byte c of the 8-byte pair
    return (float)(((c < 4 ? lo4 : hi4) >> (8 * (c & 3))) & 0xFF);
}
// the slab tests of a quantised node whose first 64 bytes (h, q1..q3) are already in registers
__device__ __forceinline__ uint32_t children_mask_q(int4 h, int4 q1, int4 q2, int4 q3, F3 of, F3 ivf, float tmax,
                                                    int dmask) {
    const F3 no = neg_oiv(of, ivf);
    const int sm = iv_signs(ivf);
    const float iv3[3] = {ivf.x, ivf.y, ivf.z}, no3[3] = {no.x, no.y, no.z};
    const float o3[3] = {__int_as_float(h.x), __int_as_float(h.y), __int_as_float(h.z)};
    const int lw[3][2] = {{q1.x, q1.y}, {q1.z, q1.w}, {q2.x, q2.y}};   // qlo x, y, z
    const int hw[3][2] = {{q2.z, q2.w}, {q3.x, q3.y}, {q3.z, q3.w}};   // qhi x, y, z
    float siv[3], base[3];
    int nw[3][2], fw[3][2];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        siv[a] = xc_scale(h.w, a) * iv3[a];
        base[a] = __builtin_fmaf(o3[a], iv3[a], no3[a]);
        const bool neg = (sm >> a) & 1;
        nw[a][0] = neg ? hw[a][0] : lw[a][0];
        nw[a][1] = neg ? hw[a][1] : lw[a][1];
        fw[a][0] = neg ? lw[a][0] : hw[a][0];
        fw[a][1] = neg ? lw[a][1] : hw[a][1];
    }
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        float tn = 0.0f, tf = tmax;
#pragma unroll
        for (int a = 0; a < 3; ++a) {
            tn = fmaxf(tn, __builtin_fmaf(xc_q(nw[a][0], nw[a][1], c), siv[a], base[a]));
            tf = fminf(tf, __builtin_fmaf(xc_q(fw[a][0], fw[a][1], c), siv[a], base[a]));
        }
        m |= tn <= tf ? 1u << c : 0u;
    }
    return xor_permute8(m & (uint32_t)((h.w >> 24) & 0xFF), dmask);
}
template <bool AXIS>
__device__ __forceinline__ uint32_t children_mask(const XCNode* nd, F3 of, F3 ivf, float tmax, int dmask) {
    const int4* b = reinterpret_cast<const int4*>(nd);
    return children_mask_q(b[0], b[1], b[2], b[3], of, ivf, tmax, dmask);
}
__device__ __forceinline__ bool child_hit(const XCNode* nd, int c, F3 of, F3 ivf, float tmax) {
    const int4* b = reinterpret_cast<const int4*>(nd);
    const int4 h = b[0], q1 = b[1], q2 = b[2], q3 = b[3];
    const F3 no = neg_oiv(of, ivf);
    const int sm = iv_signs(ivf);
    const float iv3[3] = {ivf.x, ivf.y, ivf.z}, no3[3] = {no.x, no.y, no.z};
    const float o3[3] = {__int_as_float(h.x), __int_as_float(h.y), __int_as_float(h.z)};
    const int lw[3][2] = {{q1.x, q1.y}, {q1.z, q1.w}, {q2.x, q2.y}};
    const int hw[3][2] = {{q2.z, q2.w}, {q3.x, q3.y}, {q3.z, q3.w}};
    float tn = 0.0f, tf = tmax;
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float siv = xc_scale(h.w, a) * iv3[a], base = __builtin_fmaf(o3[a], iv3[a], no3[a]);
        const bool neg = (sm >> a) & 1;
        const float tl = __builtin_fmaf(xc_q(lw[a][0], lw[a][1], c), siv, base);
        const float th = __builtin_fmaf(xc_q(hw[a][0], hw[a][1], c), siv, base);
        tn = fmaxf(tn, neg ? th : tl);
        tf = fminf(tf, neg ? tl : th);
    }
    return tn <= tf;
}

__device__ __forceinline__ bool root_hit(const DevScene& sc, F3 of, F3 ivf) {
    const float tx0 = (sc.root_lo[0] - of.x) * ivf.x, tx1 = (sc.root_hi[0] - of.x) * ivf.x;
    const float ty0 = (sc.root_lo[1] - of.y) * ivf.y, ty1 = (sc.root_hi[1] - of.y) * ivf.y;
    const float tz0 = (sc.root_lo[2] - of.z) * ivf.z, tz1 = (sc.root_hi[2] - of.z) * ivf.z;
    const float tn = fmaxf(fmaxf(fminf(tx0, tx1), fminf(ty0, ty1)), fmaxf(fminf(tz0, tz1), 0.0f));
    const float tf = fminf(fmaxf(tx0, tx1), fminf(fmaxf(ty0, ty1), fmaxf(tz0, tz1)));
    return tn <= tf;
}

// Conservative packet test: true only if no ray through pixel (x, y)'s jitter square (corners
// (x, y) .. (x+1, y+1): every jittered primary direction is a convex combination of the corner
// directions) can meet the box, i.e. the box lies strictly outside one side plane of the pixel's
// ray frustum (fp64, with a relative margin far above rounding).
__device__ __forceinline__ bool pixel_misses_box(const CamDev& cam, int x, int y, const float* lo, const float* hi) {
    const double fx = (double)x, fy = (double)y;
    // box as centre (relative to the camera) and half extents: max over its corners of n.(p - o)
    // = n.(centre - o) + sum |n_k| h_k
    const V3 bc = v3(0.5 * ((double)lo[0] + (double)hi[0]), 0.5 * ((double)lo[1] + (double)hi[1]),
                     0.5 * ((double)lo[2] + (double)hi[2])) - cam.pos;
    const V3 bh = v3(0.5 * ((double)hi[0] - (double)lo[0]), 0.5 * ((double)hi[1] - (double)lo[1]),
                     0.5 * ((double)hi[2] - (double)lo[2]));
    const double reach = fabs(bc.x) + fabs(bc.y) + fabs(bc.z) + bh.x + bh.y + bh.z;
    const V3 cc = primary_dir(cam, fx + 0.5, fy + 0.5);
    V3 a = primary_dir(cam, fx, fy);
#pragma unroll 1
    for (int i = 0; i < 4; ++i) {
        const V3 bnext = primary_dir(cam, fx + ((i == 0 || i == 1) ? 1.0 : 0.0), fy + ((i == 1 || i == 2) ? 1.0 : 0.0));
        V3 n = cross(a, bnext);
        if (dot(n, cc) < 0) n = -n;   // inside = the pixel centre's side
        const double mx = dot(n, bc) + (fabs(n.x) * bh.x + fabs(n.y) * bh.y + fabs(n.z) * bh.z);
        const double nl = fabs(n.x) + fabs(n.y) + fabs(n.z);
        if (mx < -1e-9 * nl * reach) return true;
        a = bnext;
    }
    return false;
}

// TRI: only the entity kinds of the 4-wave scenes (triangle meshes without acos texture mapping:
// ImpTriangle, ExpQuad, ExpCube; ExpBox maps to (0, 0)) -- the other kinds' code is not emitted
template <bool TRI = false>
__device__ __forceinline__ void x_texcoord(const DevScene& sc, const REnt& e, V3 ip, int32_t& x, int32_t& y) {
    if (TRI) {
        if (e.kind == K_IMP_TRIANGLE) {
            const V3 p1 = ld3(e.qv0), p21 = ld3(e.qv1), i1 = ip - p1;
            const double i1l = gsqrt(sq3(i1));
            const double c = dot(p21, i1) / (e.qv2[0] * i1l);
            const double ixl = i1l * mx_sin_acos(c);
            y = x86_trunc(i1l / e.qv2[2]);
            x = x86_trunc(ixl / e.qv2[1]);
        } else if (e.kind == K_EXP_QUAD || e.kind == K_EXP_CUBE) {
            const bool q = e.kind == K_EXP_QUAD;
            const double uv = (double)e.width / 160.0, uh = (double)e.length / 160.0;
            const V3 i1 = ip - (q ? ld3(e.qv1) : ld3(e.qv0));
            const double l = gsqrt(sq3(i1));
            const double c = q ? dot(i1, ld3(e.qv0) - ld3(e.qv1)) / ((double)e.width * l)
                               : dot(i1, v3(0, (double)e.width, 0)) / ((double)e.width * l);
            y = x86_trunc(l * mx_sin_acos(c) / uh);
            x = x86_trunc(l * mx_cos_acos(c) / uv);
        } else {
            x = 0;
            y = 0;
        }
        return;
    }
    if (e.kind == K_IMP_SPHERE) {
        const double r = e.radius;
        const double unit_v = 2.0 * REF_PI * r / 320.0;
        const V3 to = ip - ld3(e.pos);
        const double cv = dot(to, v3(0, 0, r)) / (r * r);
        y = x86_trunc((r * mx_acos(cv)) / unit_v);
        const double small_r = r * mx_sin_acos(cv);
        const double ch = dot(v3(to.x, to.y, 0), v3(0, small_r, 0)) / (small_r * small_r);
        const double unit_h = 2.0 * REF_PI * small_r / 320.0;
        x = x86_trunc(small_r * mx_acos(ch) / unit_h);
    } else if (e.kind == K_IMP_TRIANGLE) {
        const V3 p1 = ld3(e.qv0), p21 = ld3(e.qv1), i1 = ip - p1;
        const double i1l = gsqrt(sq3(i1));
        const double c = dot(p21, i1) / (e.qv2[0] * i1l);
        const double ixl = i1l * mx_sin_acos(c);
        y = x86_trunc(i1l / e.qv2[2]);
        x = x86_trunc(ixl / e.qv2[1]);
    } else if (e.kind == K_EXP_QUAD) {
        const double uv = (double)e.width / 160.0, uh = (double)e.length / 160.0;
        const V3 rv = ld3(e.qv0) - ld3(e.qv1), i1 = ip - ld3(e.qv1);
        const double i1l = gsqrt(sq3(i1));
        const double c = dot(i1, rv) / ((double)e.width * i1l);
        y = x86_trunc(i1l * mx_sin_acos(c) / uh);
        x = x86_trunc(i1l * mx_cos_acos(c) / uv);
    } else if (e.kind == K_EXP_SPHERE) {
        const double r = e.radius;
        const double unit_v = 2.0 * REF_PI * r / 320.0;
        const V3 to = ip - ld3(e.pos);
        const double cv = dot(to, v3(0, 0, r)) / (r * r);
        y = x86_trunc((0.5 * REF_PI * r - r * mx_acos(cv)) / unit_v);
        const double small_r = r * mx_sin_acos(cv);
        const double ch = dot(v3(to.x, to.y, 0), v3(0, small_r, 0)) / (small_r * small_r);
        const double unit_h = 2.0 * REF_PI * small_r / 320.0;
        x = x86_trunc(small_r * mx_acos(ch) / unit_h);
    } else if (e.kind == K_EXP_CUBE) {
        const double uv = (double)e.width / 160.0, uh = (double)e.length / 160.0;
        const V3 i1 = ip - ld3(e.qv0);
        const double l = gsqrt(sq3(i1));
        const double c = dot(i1, v3(0, (double)e.width, 0)) / ((double)e.width * l);
        y = x86_trunc(l * mx_sin_acos(c) / uh);
        x = x86_trunc(l * mx_cos_acos(c) / uv);
    } else if (e.kind == K_EXP_CONE) {
        const double R = e.radius, H = e.height;
        const double unit_h = gsqrt(R * R + H * H) / 320.0;
        const V3 pos = ld3(e.pos);
        const double ylen = gsqrt(sq3(ip - pos));
        y = x86_trunc(ylen / unit_h);
        const V3 center = v3((float)pos.x, (float)pos.y, (float)ip.z);
        const double rp = ylen * e.sin_theta;
        const V3 left = v3(0, (float)rp, 0);
        const V3 ic = ip - center;
        const double unit_v = 2.0 * REF_PI * rp / 320.0;
        double alpha = mx_acos(dot(ic, left) / (rp * rp));
        if (alpha > REF_PI / 4.0) alpha = mx_acos(dot(ic, -left) / (rp * rp));
        x = x86_trunc(rp * alpha / unit_v);
    } else if (e.kind == K_EXP_RECTANGLE) {
        const V3 p1 = ld3(e.qv0), p31 = ld3(e.qv1) - p1, p41 = ld3(e.qv2) - p1;
        const double width = gsqrt(sq3(p41)), length = gsqrt(sq3(p31));
        const V3 i1 = ip - p1;
        const double l = gsqrt(sq3(i1));
        const double ct = mx_acos(dot(i1, p31) / (length * l));
        x = x86_trunc(l * mx_sin_acos(ct) / (length / 64.0));
        y = x86_trunc(l * ct / (width / 64.0));
    } else {
        x = 0;
        y = 0;
    }
}

}  // namespace
}  // namespace gi
