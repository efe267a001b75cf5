// gi_math.h — fp64/fp32 vector math with the reference's exact operation order, shared by the host
// scene builder (g++) and the gfx950 kernels (hipcc).  Both sides compile with -ffp-contract=off,
// so every expression rounds exactly like the reference's glm 0.9.8.2 code:
//   dot       (x*x' + y*y') + z*z'                 glm/detail/func_geometric.inl:54-61
//   cross     (y*z'-y'*z, z*x'-z'*x, x*y'-x'*y)    func_geometric.inl:74-85
//   normalize v * (1 / sqrt(dot(v,v)))              func_geometric.inl:88-96, func_exponential.inl:128-133
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GI_HD __host__ __device__ __forceinline__
#else
#define GI_HD inline
#include <cmath>
#endif

namespace gi {

struct V3 {
    double x, y, z;
};
GI_HD V3 v3(double x, double y, double z) { V3 r; r.x = x; r.y = y; r.z = z; return r; }
GI_HD V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
GI_HD V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
GI_HD V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
GI_HD V3 operator*(V3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
GI_HD V3 operator*(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
GI_HD V3 vmul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
GI_HD double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
GI_HD V3 cross(V3 x, V3 y) { return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); }
GI_HD double gsqrt(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_sqrt(x);   // correctly rounded f64 sqrt on gfx950
#else
    return std::sqrt(x);
#endif
}
GI_HD V3 normalize(V3 v) { return v * (1.0 / gsqrt(dot(v, v))); }
// Mode X only (build-defined, not the reference's arithmetic): fused multiply-add, correctly
// rounded on both sides (v_fma_f64 / std::fma), so the oracle restates it exactly.
GI_HD double gfma(double a, double b, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_fma(a, b, c);
#else
    return std::fma(a, b, c);
#endif
}
GI_HD double fdot(V3 a, V3 b) { return gfma(a.z, b.z, gfma(a.y, b.y, a.x * b.x)); }
GI_HD V3 fcross(V3 x, V3 y) {
    return v3(gfma(x.y, y.z, -(y.y * x.z)), gfma(x.z, y.x, -(y.z * x.x)), gfma(x.x, y.y, -(y.x * x.y)));
}

GI_HD double length(V3 v) { return gsqrt(dot(v, v)); }
// pow(v.x,2)+pow(v.y,2)+pow(v.z,2) as the reference writes it (g++ folds pow(x,2) to x*x)
GI_HD double sq3(V3 v) { return v.x * v.x + v.y * v.y + v.z * v.z; }
GI_HD double smin(double a, double b) { return (b < a) ? b : a; }   // std::min
GI_HD double smax(double a, double b) { return (a < b) ? b : a; }   // std::max
GI_HD float sminf(float a, float b) { return (b < a) ? b : a; }
GI_HD float fabsf_(float a) { return a < 0.0f ? -a : (a == 0.0f ? 0.0f : a); }

// x86-64 cvttsd2si semantics for the reference's int() casts: NaN/out of range -> INT_MIN (A.9).
// (gfx950's v_cvt_i32_f64 clamps instead, so this is explicit.)
GI_HD int32_t x86_trunc(double d) {
    if (!(d > -2147483649.0 && d < 2147483648.0)) return (int32_t)0x80000000u;
    return (int32_t)d;
}

const double REF_PI = 3.1415926535;   // entities.h:16

// ImpTriangle derived members (entities.h:139-148), member-initialisation order.
struct TriRec {            // 144 bytes
    double p1[3], p2[3], p3[3];
    double n[3];           // normalize(cross(edge1, edge2))
    double pos[3];         // 0.5*(0.5*(p1+p2)+p3)
    float e1f[3], e2f[3];  // glm::vec3(edge1/edge2) as cast into the fp32 mat3
};

GI_HD V3 ld3(const double* p) { return v3(p[0], p[1], p[2]); }
GI_HD void st3(double* p, V3 v) { p[0] = v.x; p[1] = v.y; p[2] = v.z; }

GI_HD void make_tri(V3 p1, V3 p2, V3 p3, TriRec& t) {
    st3(t.p1, p1); st3(t.p2, p2); st3(t.p3, p3);
    const V3 e1 = p2 - p1, e2 = p3 - p1;
    st3(t.n, normalize(cross(e1, e2)));
    st3(t.pos, 0.5 * (0.5 * (p1 + p2) + p3));
    t.e1f[0] = (float)e1.x; t.e1f[1] = (float)e1.y; t.e1f[2] = (float)e1.z;
    t.e2f[0] = (float)e2.x; t.e2f[1] = (float)e2.y; t.e2f[2] = (float)e2.z;
}

// ImpTriangle::intersect (entities.h:150-249) after its parallel test: the fp32 solve --
// glm::mat3(e1, e2, -dir) transposed, glm's cofactor inverse (func_matrix.inl:272-294) and
// vec3 * mat3 (type_mat3x3.inl:437-443); only sol.z is used -- then the acceptance test on the
// three sub-triangle normals at the computed point.  No t > 0 test (A.3).
GI_HD bool tri_accept(V3 p1, V3 p2, V3 p3, V3 pos, const float* e1f, const float* e2f, V3 o, V3 d, V3& P) {
    const float m00 = e1f[0], m01 = e2f[0], m02 = (float)(-d.x);
    const float m10 = e1f[1], m11 = e2f[1], m12 = (float)(-d.y);
    const float m20 = e1f[2], m21 = e2f[2], m22 = (float)(-d.z);
    const float det = m00 * (m11 * m22 - m21 * m12) - m10 * (m01 * m22 - m21 * m02) + m20 * (m01 * m12 - m11 * m02);
    const float ood = 1.0f / det;
    const float i20 = (m10 * m21 - m20 * m11) * ood;
    const float i21 = (-(m00 * m21 - m20 * m01)) * ood;
    const float i22 = (m00 * m11 - m10 * m01) * ood;
    const V3 right = o - pos;
    const float solz = i20 * (float)right.x + i21 * (float)right.y + i22 * (float)right.z;
    const V3 point = o + (double)solz * d;
    const V3 c1 = cross(p1 - point, p2 - point), c2 = cross(p2 - point, p3 - point), c3 = cross(p3 - point, p1 - point);
    // Exact-safe early rejection (no normalisation): acceptance below needs |d1 - d2|^2 < 1e-3 and
    // |d2 - d3|^2 < 1e-3, i.e. d1.d2 and d2.d3 > 0.9995, or a sub-normal shorter than 1e-3.  With every
    // |c_k| > 1e-100 the normalised d_k have length ~1 (no short one), and c1.c2 <= 0 or c2.c3 <= 0
    // (rounding errors ~1e-16 |c_i||c_j|) puts the pair ~90 degrees or more apart: the test below would
    // reject too.  NaN / inf components fail the length guard or the comparison and take the full test.
    const double n1 = dot(c1, c1), n2 = dot(c2, c2), n3 = dot(c3, c3);
    const double x12 = dot(c1, c2), x23 = dot(c2, c3);
    if ((n1 > 1e-200) & (n2 > 1e-200) & (n3 > 1e-200) & ((x12 <= 0.0) | (x23 <= 0.0))) return false;
    // Both comparisons decided without the normalisations where the answer is clear.  With the
    // c_k's squared lengths in [1e-150, 1e150] the d_k are unit vectors to ~5u, so the computed
    // |d_j - d_k|^2 is 2 - 2 cos(c_j, c_k) to ~50u; cos^2 from the unnormalised dot products (relative
    // rounding ~1e-15) set against the threshold moved by 1e-9 either way: a pair clearly below 1e-3
    // is below it in the reference's arithmetic too, a pair clearly above it is above (and no d_k is
    // short), so the answer is the reference's; within the 1e-9 band the test runs as written.
    if ((n1 > 1e-150) & (n2 > 1e-150) & (n3 > 1e-150) & (n1 < 1e150) & (n2 < 1e150) & (n3 < 1e150)) {
        constexpr double kIn = (1.0 - (1.0e-3 - 1e-9) / 2.0) * (1.0 - (1.0e-3 - 1e-9) / 2.0);
        constexpr double kOut = (1.0 - (1.0e-3 + 1e-9) / 2.0) * (1.0 - (1.0e-3 + 1e-9) / 2.0);
        const double p12 = n1 * n2, p23 = n2 * n3;
        const bool in = (x12 > 0.0) & (x23 > 0.0) & (x12 * x12 > kIn * p12) & (x23 * x23 > kIn * p23);
        const bool out = (x12 <= 0.0) | (x23 <= 0.0) | (x12 * x12 < kOut * p12) | (x23 * x23 < kOut * p23);
        if (in) {
            P = point;
            return true;
        }
        if (out) return false;
    }
    const V3 d1 = normalize(c1);
    const V3 d2 = normalize(c2);
    const V3 d3 = normalize(c3);
    // glm::length(d_k) < 1e-3 branches (:201-230): a normalised vector has length ~1, inf or NaN;
    // test the squared length first so the sqrt only runs when the branch can fire.
    const double q1 = dot(d1, d1), q2 = dot(d2, d2), q3 = dot(d3, d3);
    const bool short_d = (q1 < 1e-5 && gsqrt(q1) < 1.0e-3) || (q2 < 1e-5 && gsqrt(q2) < 1.0e-3) ||
                         (q3 < 1e-5 && gsqrt(q3) < 1.0e-3);
    const bool inside = sq3(d1 - d2) < 1.0e-3 && sq3(d2 - d3) < 1.0e-3;   // :232-237
    if (!(short_d || inside)) return false;
    P = point;
    return true;
}
// ImpTriangle::intersect (entities.h:150-249) with the triangle's derived members n, pos, e1f, e2f
GI_HD bool tri_hit(V3 p1, V3 p2, V3 p3, V3 n, V3 pos, const float* e1f, const float* e2f, V3 o, V3 d,
                   V3& P, V3& N) {
    if (dot(n, d) == 0) return false;
    if (!tri_accept(p1, p2, p3, pos, e1f, e2f, o, d, P)) return false;
    N = dot(d, n) < 0 ? n : -n;
    return true;
}

// Exact-safe early rejection for tri_hit.  The reference's acceptance test (:232-237) needs the
// three normalised sub-triangle normals at the computed point to agree within sqrt(1e-3)
// (~0.03 rad); the point always lies on the ray's line.  Outside the triangle's plane region one
// sub-normal flips (|d_i - d_j|^2 ~ 4); above/below it the side normals tilt apart unless the
// height is < ~3% of the distance to the edges; far away they follow P x edge_k, which differ.
// So every accepted point lies within 1.01x the bounding-sphere radius of the vertex centroid,
// and a line that misses that sphere (with rounding slack) cannot produce a hit.
GI_HD bool tri_may_hit(V3 p1, V3 p2, V3 p3, V3 o, V3 d) {
    const V3 c = (p1 + p2 + p3) * (1.0 / 3.0);
    const double r2 = smax(smax(sq3(p1 - c), sq3(p2 - c)), sq3(p3 - c));
    const V3 oc = c - o;
    const V3 x = cross(oc, d);
    return dot(x, x) <= r2 * 1.0201 + 1e-12 * dot(oc, oc);
}

GI_HD bool tri_hit(const TriRec& t, V3 o, V3 d, V3& P, V3& N) {
    if (!tri_may_hit(ld3(t.p1), ld3(t.p2), ld3(t.p3), o, d)) return false;
    return tri_hit(ld3(t.p1), ld3(t.p2), ld3(t.p3), ld3(t.n), ld3(t.pos), t.e1f, t.e2f, o, d, P, N);
}

// A triangle built on the fly from three corners (ExpBox faces, entities.h:319-324), its normal
// used only by the parallel test dot(normalize(c), d) == 0, c = cross(e1, e2).  normalize scales the
// components of c by one rounded factor s: the computed dot is s sum(c_i d_i (1 + e_i)) plus its own
// rounding, |e_i| <= u, the rounding <= 3u (1 + u) s sum |c_i d_i|; so whenever |sum c_i d_i| exceeds
// ~4.5u sum |c_i d_i| it is nonzero.  dot(c, d) computed (rounding <= 3u sum |c_i d_i|) above 1e-12 of
// sum |c_i d_i| proves that, with c and d in the normal range, and the square root and division of
// the normalisation are skipped; otherwise the test runs as the reference writes it.
GI_HD bool tri_hit_corners(V3 p1, V3 p2, V3 p3, V3 o, V3 d) {
    if (!tri_may_hit(p1, p2, p3, o, d)) return false;
    const V3 e1 = p2 - p1, e2 = p3 - p1;
    const V3 c = cross(e1, e2);
    const double cd = dot(c, d);
    const double ca = fabs(c.x * d.x) + fabs(c.y * d.y) + fabs(c.z * d.z);
    const bool clear = (fabs(cd) > 1e-12 * ca) & (ca > 1e-200) & (ca < 1e200);
    if (!clear && dot(normalize(c), d) == 0) return false;
    const V3 pos = 0.5 * (0.5 * (p1 + p2) + p3);
    const float e1f[3] = {(float)e1.x, (float)e1.y, (float)e1.z};
    const float e2f[3] = {(float)e2.x, (float)e2.y, (float)e2.z};
    V3 P;
    return tri_accept(p1, p2, p3, pos, e1f, e2f, o, d, P);
}

// ExpBox(min,max).intersect (entities.h:379-440) as Octree::Node::intersect uses it: true iff any
// of the 12 face triangles hits; each ExpRectangle(p1,p2,p3) face is t1=(p1,p2,p3) then
// t2=(p1,p2,p4) with p4 = -p3 (default member init runs before pos is set, A.4).
GI_HD bool box_hit(V3 mn, V3 mx, V3 o, V3 d) {
    const V3 dlb = mn, drb = v3(mx.x, mn.y, mn.z), dlt = v3(mn.x, mx.y, mn.z), drt = v3(mx.x, mx.y, mn.z);
    const V3 ulb = v3(mn.x, mn.y, mx.z), urb = v3(mx.x, mn.y, mx.z), ult = v3(mn.x, mx.y, mx.z), urt = mx;
    // the OR of the 12 face tests (ExpBox::faces, entities.h:400-405; || short-circuits like an OR of
    // bools, and the tests have no side effects, so any order gives the same answer)
    // the spurious faces first (A.4: p4 = -p3, triangles through the box's mirror image): they accept
    // most of the rays that pass a node test, so a passing test ends sooner (R-C3 -5%, R-C4 +-0)
    return tri_hit_corners(dlb, urb, -ulb, o, d) || tri_hit_corners(dlb, ult, -dlt, o, d) ||
           tri_hit_corners(dlb, drt, -dlt, o, d) || tri_hit_corners(urt, ulb, -ult, o, d) ||
           tri_hit_corners(urt, drb, -drt, o, d) || tri_hit_corners(urt, dlt, -drt, o, d) ||
           tri_hit_corners(dlb, urb, ulb, o, d) || tri_hit_corners(dlb, ult, dlt, o, d) ||
           tri_hit_corners(dlb, drt, dlt, o, d) || tri_hit_corners(urt, ulb, ult, o, d) ||
           tri_hit_corners(urt, drb, drt, o, d) || tri_hit_corners(urt, dlt, drt, o, d);
}

// box_hit split over four lanes: part j in [0, 4) tests faces j, j + 4, j + 8 of box_hit's order
// (spurious faces 0-5, real faces 6-11), so the OR over the four parts is box_hit's answer.  Face
// f's rectangle k = f % 6 has corners p1 (dlb for k < 3, else urt), p2 and p3 (-p3 for the spurious
// triangle), each corner picked from mn / mx by its 3 bits (x = 1, y = 2, z = 4) -- the same corners
// and triangles as box_hit, selected per lane so that every lane runs the same code.
GI_HD V3 box_corner(V3 mn, V3 mx, int bits) {
    return v3((bits & 1) ? mx.x : mn.x, (bits & 2) ? mx.y : mn.y, (bits & 4) ? mx.z : mn.z);
}
GI_HD bool box_face_hit(V3 mn, V3 mx, V3 o, V3 d, int f) {
    const int k = f >= 6 ? f - 6 : f;
    // p2 and p3 corner bits of rectangles k = 0..5 (urb ult drt ulb drb dlt; ulb dlt dlt ult drt drt), 4 bits each
    const int b2 = (0x214365 >> (4 * k)) & 7, b3 = (0x336224 >> (4 * k)) & 7;
    const V3 p3 = box_corner(mn, mx, b3);
    return tri_hit_corners(box_corner(mn, mx, k < 3 ? 0 : 7), box_corner(mn, mx, b2), f < 6 ? -p3 : p3, o, d);
}
GI_HD bool box_hit_part(V3 mn, V3 mx, V3 o, V3 d, int part) {
    return box_face_hit(mn, mx, o, d, part) || box_face_hit(mn, mx, o, d, part + 4) ||
           box_face_hit(mn, mx, o, d, part + 8);
}

// ImpSphere::intersect (entities.h:53-96): the quadratic in the dominant-axis parameterisation
// with its fp32/fp64 mix; a line test on |root| (A.2).
GI_HD bool sphere_hit(V3 pos, float radius, V3 o, V3 d, V3& P, V3& N) {
    const V3 np = pos - o;
    float a1 = 1, a2 = 1, a3 = 1;
    if (d.x != 0) { a2 = (float)(d.y / d.x); a3 = (float)(d.z / d.x); }
    else if (d.y != 0) { a1 = (float)(d.x / d.y); a3 = (float)(d.z / d.y); }
    else if (d.z != 0) { a2 = (float)(d.y / d.z); a1 = (float)(d.x / d.z); }
    else return false;
    const double A1 = a1, A2 = a2, A3 = a3;
    const float a = (float)(A1 * A1 + A2 * A2 + A3 * A3);
    const float b = (float)(-2.0 * (np.x * A1 + np.y * A2 + np.z * A3));
    const double R = radius;
    const float c = (float)(np.x * np.x + np.y * np.y + np.z * np.z - R * R);
    const double B = b;
    const float ac4 = (4.0f * a) * c;
    const double disc = B * B - (double)ac4;
    if (disc < 0) return false;
    const double s = gsqrt(disc);
    const float a2f = 2.0f * a;
    const float v1 = (float)((-B + s) / (double)a2f);
    const float v2 = (float)((-B - s) / (double)a2f);
    const float base = sminf(fabsf_(v1), fabsf_(v2));
    const V3 ip = v3((double)(base * a1), (double)(base * a2), (double)(base * a3)) + o;
    P = ip;
    N = normalize(ip - pos);
    return true;
}

// ---- Mode X (build-defined) ----------------------------------------------------
// Only + - * / sqrt and comparisons, so host oracle and device agree bit for bit.
const double MX_TMIN = 1e-7;
const double MX_PI = 0x1.921fb54442d18p+1, MX_PIO2 = 0x1.921fb54442d18p+0;

GI_HD uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}
// counter-based uniform in [0,1): key (seed, pixel, sample, bounce, dim)
GI_HD uint64_t mx_key(uint64_t seed, uint64_t pixel) { return mix64(seed + 0x9E3779B97F4A7C15ULL * (pixel + 1)); }
GI_HD double mx_u01k(uint64_t key, uint32_t sample, uint32_t bounce, uint32_t dim) {
    const uint64_t k = mix64(key ^ (((uint64_t)sample << 32) | ((uint64_t)(bounce & 0xFFFF) << 16) | (uint64_t)(dim & 0xFFFF)));
    return (double)(k >> 11) * 0x1.0p-53;
}

GI_HD double mx_asin_small(double y) {   // |y| <= 0.5: 30-term Taylor series, Horner
    const double C[30] = {
        0x1.0000000000000p+0, 0x1.5555555555555p-3, 0x1.3333333333333p-4, 0x1.6db6db6db6db7p-5,
        0x1.f1c71c71c71c7p-6, 0x1.6e8ba2e8ba2e9p-6, 0x1.1c4ec4ec4ec4fp-6, 0x1.c99999999999ap-7,
        0x1.7a87878787878p-7, 0x1.3fde50d79435ep-7, 0x1.12ef3cf3cf3cfp-7, 0x1.df3bd37a6f4dfp-8,
        0x1.a6863d70a3d71p-8, 0x1.782dda12f684cp-8, 0x1.51ba308d3dcb1p-8, 0x1.31683bdef7bdfp-8,
        0x1.15ee9d45d1746p-8, 0x1.fcaf8fb6db6dbp-9, 0x1.d3d2a8e0dd67dp-9, 0x1.b026f57b13b14p-9,
        0x1.90cb77f60c7cep-9, 0x1.750de64d7d05fp-9, 0x1.5c5f56efaaaabp-9, 0x1.464c0950f7d47p-9,
        0x1.3275586c5f2f0p-9, 0x1.208d3570ae5a6p-9, 0x1.1052bc5fa960ap-9, 0x1.018f963c229bfp-9,
        0x1.e82be60d9127ep-10, 0x1.cf7dea5b6e830p-10};
    const double z = y * y;
    double p = C[29];
    for (int k = 28; k >= 0; --k) p = p * z + C[k];
    return y * p;
}
GI_HD double mx_acos(double x) {
    if (!(x >= -1.0 && x <= 1.0)) return __builtin_nan("");
    if (x >= -0.5 && x <= 0.5) return MX_PIO2 - mx_asin_small(x);
    if (x > 0.5) return 2.0 * mx_asin_small(gsqrt((1.0 - x) * 0.5));
    return MX_PI - 2.0 * mx_asin_small(gsqrt((1.0 + x) * 0.5));
}
GI_HD double mx_sin_acos(double c) { return gsqrt(1.0 - c * c); }
GI_HD double mx_cos_acos(double c) { return (c >= -1.0 && c <= 1.0) ? c : __builtin_nan(""); }
GI_HD double mx_powi(double x, int p) {
    double r = 1.0, b = x;
    while (p) {
        if (p & 1) r = r * b;
        b = b * b;
        p >>= 1;
    }
    return r;
}
// x^p for any specular power (Material::specular_power is any double, material.h:29): integer p in
// [0, 64] by square-and-multiply (mx_powi); otherwise exp(p * ln x) with ln from the atanh series of
// the mantissa and exp from a Taylor polynomial, 2^n applied through the exponent bits -- only
// +, -, *, / and exact bit operations on fp64, so host and gfx950 agree bit for bit (DESIGN.md
// "Mode X").  Relative error ~1e-15 against the true power (x in [0, 1] at the call site).
GI_HD double mx_bits_to_f64(uint64_t b) { double d; __builtin_memcpy(&d, &b, 8); return d; }
GI_HD uint64_t mx_f64_to_bits(double d) { uint64_t b; __builtin_memcpy(&b, &d, 8); return b; }
GI_HD double mx_ln(double x) {   // x > 0, finite
    int e = 0;
    if (x < 0x1.0p-1022) { x = x * 0x1.0p+54; e = -54; }   // subnormal: exact rescale
    const uint64_t b = mx_f64_to_bits(x);
    e += (int)((b >> 52) & 0x7FF) - 1023;
    double m = mx_bits_to_f64((b & 0x000FFFFFFFFFFFFFull) | 0x3FF0000000000000ull);   // [1, 2)
    if (m > 1.4142135623730951) { m = m * 0.5; e += 1; }                               // [0.707, 1.414]
    const double s = (m - 1.0) / (m + 1.0), z = s * s;
    double q = 1.0 / 25.0;
    q = q * z + 1.0 / 23.0; q = q * z + 1.0 / 21.0; q = q * z + 1.0 / 19.0; q = q * z + 1.0 / 17.0;
    q = q * z + 1.0 / 15.0; q = q * z + 1.0 / 13.0; q = q * z + 1.0 / 11.0; q = q * z + 1.0 / 9.0;
    q = q * z + 1.0 / 7.0; q = q * z + 1.0 / 5.0; q = q * z + 1.0 / 3.0; q = q * z + 1.0;
    const double de = (double)e;
    return de * 0x1.62e42fee00000p-1 + (de * 0x1.a39ef35793c76p-33 + 2.0 * s * q);
}
GI_HD double mx_exp(double y) {
    if (!(y > -746.0)) return y != y ? y : 0.0;
    if (y > 710.0) return __builtin_inf();
    const int n = (int)(y * 0x1.71547652b82fep+0 + (y >= 0.0 ? 0.5 : -0.5));   // round(y / ln 2)
    const double dn = (double)n;
    const double r = (y - dn * 0x1.62e42fee00000p-1) - dn * 0x1.a39ef35793c76p-33;   // |r| <~ 0.35
    double q = 1.0 / 355687428096000.0;   // 1/17!
    q = q * r + 1.0 / 20922789888000.0; q = q * r + 1.0 / 1307674368000.0; q = q * r + 1.0 / 87178291200.0;
    q = q * r + 1.0 / 6227020800.0; q = q * r + 1.0 / 479001600.0; q = q * r + 1.0 / 39916800.0;
    q = q * r + 1.0 / 3628800.0; q = q * r + 1.0 / 362880.0; q = q * r + 1.0 / 40320.0; q = q * r + 1.0 / 5040.0;
    q = q * r + 1.0 / 720.0; q = q * r + 1.0 / 120.0; q = q * r + 1.0 / 24.0; q = q * r + 1.0 / 6.0;
    q = q * r + 0.5; q = q * r + 1.0; q = q * r + 1.0;
    if (n >= -1022) return q * mx_bits_to_f64((uint64_t)(n + 1023) << 52);
    return (q * mx_bits_to_f64((uint64_t)(n + 1023 + 54) << 52)) * 0x1.0p-54;   // subnormal result
}
GI_HD double mx_pow(double x, double p) {
    if (p >= 0.0 && p <= 64.0 && p == (double)(int)p) return mx_powi(x, (int)p);
    if (p != p || x != x) return __builtin_nan("");
    if (x == 0.0) return p > 0.0 ? 0.0 : __builtin_inf();
    if (x < 0.0) return __builtin_nan("");
    if (x == __builtin_inf()) return p > 0.0 ? x : 0.0;
    return mx_exp(p * mx_ln(x));
}

// Texture (material.h:65-106): 32x32 int checker, colour truncated to int (A.7); a negative
// index (out-of-bounds UB in the reference, A.9) wraps into [0,32).
// Mode X: point on the unit disk from (u1, u2) in [0,1)^2 by the concentric map (Shirley & Chiu
// 1997), loop-free; sin/cos on [-pi/4, pi/4] as degree-17/16 Taylor polynomials in Horner form
// (only +, -, * on fp64: bit-identical on the host and gfx950).  r2 = radius^2.
GI_HD void mx_sincos_q(double p, double& sn, double& cs) {
    const double S[8] = {-0x1.5555555555555p-3, 0x1.1111111111111p-7, -0x1.a01a01a01a01ap-13, 0x1.71de3a556c734p-19,
    -0x1.ae64567f544e4p-26, 0x1.6124613a86d09p-33, -0x1.ae7f3e733b81fp-41, 0x1.952c77030ad4ap-49};
    const double C[8] = {-0x1.0000000000000p-1, 0x1.5555555555555p-5, -0x1.6c16c16c16c17p-10, 0x1.a01a01a01a01ap-16,
    -0x1.27e4fb7789f5cp-22, 0x1.1eed8eff8d898p-29, -0x1.93974a8c07c9dp-37, 0x1.ae7f3e733b81fp-45};
    const double z = p * p;
    double ps = S[7], pc = C[7];
    for (int k = 6; k >= 0; --k) {
        ps = ps * z + S[k];
        pc = pc * z + C[k];
    }
    sn = p + p * (z * ps);
    cs = 1.0 + z * pc;
}
// Branch-free form of the concentric map (the same operations per lane as the two-branch
// statement of the oracle's mx_disk: the octant choice selects operands, one quotient, one
// sincos), so a wave evaluates one polynomial pair instead of both branches' copies.
GI_HD void mx_disk(double u1, double u2, double& dx, double& dy, double& r2) {
    const double a = 2.0 * u1 - 1.0, b = 2.0 * u2 - 1.0;
    const double QPI = 0x1.921fb54442d18p-1;   // pi/4
    const bool ax = (a < 0 ? -a : a) > (b < 0 ? -b : b);
    const double r = ax ? a : b, num = ax ? b : a;
    const double q = num / r;
    double sn, cs;
    mx_sincos_q(QPI * q, sn, cs);
    const bool zero = (a == 0.0) & (b == 0.0);
    dx = zero ? 0.0 : r * (ax ? cs : sn);
    dy = zero ? 0.0 : r * (ax ? sn : cs);
    r2 = zero ? 0.0 : r * r;
}

GI_HD V3 texel(V3 color, int32_t u, int32_t v) {
    // pattern[u % 32][v % 32] with C remainders: the compiled reference reads the FLAT element
    // (u%32)*32 + v%32 of the 32x32 array; inside [0,1024) that is exact, outside it reads stack
    // memory (UB, no parity claim) and this path wraps the flat index into the array (oracle: same).
    int f = (u % 32) * 32 + (v % 32);
    if (f < 0 || f >= 1024) f = ((f % 1024) + 1024) % 1024;
    const int i = f >> 5, j = f & 31;
    const bool white = ((i <= 16) & (j <= 16)) | ((i > 16) & (j > 16));   // (a select, not a branch)
    const V3 c = v3((double)x86_trunc(color.x), (double)x86_trunc(color.y), (double)x86_trunc(color.z));
    return white ? v3(1, 1, 1) : c;
}

// Image::setPixel quantisation (image.h:14-16): (int)(255*c); an out-of-range channel makes the
// QColor invalid, which QImage stores as black.
GI_HD void quantize(double r, double g, double b, uint8_t* q) {
    const int32_t R = x86_trunc(255 * r), G = x86_trunc(255 * g), B = x86_trunc(255 * b);
    if (R < 0 || R > 255 || G < 0 || G > 255 || B < 0 || B > 255) { q[0] = q[1] = q[2] = 0; return; }
    q[0] = (uint8_t)R; q[1] = (uint8_t)G; q[2] = (uint8_t)B;
}

}  // namespace gi
