// Stress test: the exact-safe bounding-sphere prefilter (gi_math.h tri_may_hit) never changes
// the reference ImpTriangle::intersect result (entities.h:150-249) on random, on-edge,
// near-edge and sliver triangles across 6 orders of magnitude of scale.
#include "gi_math.h"
#include <cstdio>
#include <random>
#include <cstdlib>
#include <cmath>
using namespace gi;
static bool raw(V3 p1, V3 p2, V3 p3, V3 o, V3 d) {
    const V3 e1 = p2 - p1, e2 = p3 - p1;
    const V3 n = normalize(cross(e1, e2));
    const V3 pos = 0.5 * (0.5 * (p1 + p2) + p3);
    const float e1f[3] = {(float)e1.x, (float)e1.y, (float)e1.z};
    const float e2f[3] = {(float)e2.x, (float)e2.y, (float)e2.z};
    V3 P, N;
    return tri_hit(p1, p2, p3, n, pos, e1f, e2f, o, d, P, N);
}
// tri_hit without its early rejection (the reference's acceptance test evaluated in full, as round 5
// shipped it): the product's early rejection of unnormalised sub-normals must never change a result
static bool full(V3 p1, V3 p2, V3 p3, V3 o, V3 d) {
    const V3 e1 = p2 - p1, e2 = p3 - p1;
    const V3 n = normalize(cross(e1, e2));
    const V3 pos = 0.5 * (0.5 * (p1 + p2) + p3);
    const float e1f[3] = {(float)e1.x, (float)e1.y, (float)e1.z};
    const float e2f[3] = {(float)e2.x, (float)e2.y, (float)e2.z};
    if (dot(n, d) == 0) return false;
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
    const V3 d1 = normalize(cross(p1 - point, p2 - point));
    const V3 d2 = normalize(cross(p2 - point, p3 - point));
    const V3 d3 = normalize(cross(p3 - point, p1 - point));
    const double q1 = dot(d1, d1), q2 = dot(d2, d2), q3 = dot(d3, d3);
    const bool short_d = (q1 < 1e-5 && gsqrt(q1) < 1.0e-3) || (q2 < 1e-5 && gsqrt(q2) < 1.0e-3) ||
                         (q3 < 1e-5 && gsqrt(q3) < 1.0e-3);
    const bool inside = sq3(d1 - d2) < 1.0e-3 && sq3(d2 - d3) < 1.0e-3;
    return short_d || inside;
}
int main(int argc, char** argv) {
    std::mt19937_64 g(1);
    std::uniform_real_distribution<double> U(-1, 1);
    long n = 0, hits = 0, bad = 0, near = 0;
    const long N = argc > 1 ? atol(argv[1]) : 6000000;
    for (long it = 0; it < N; ++it) {
        double sc = std::pow(10.0, 3 * U(g));
        V3 p1 = v3(U(g), U(g), U(g)) * sc, p2 = v3(U(g), U(g), U(g)) * sc, p3 = v3(U(g), U(g), U(g)) * sc;
        if (it % 3 == 0) { p2 = p1 + (p2 - p1) * 1e-3; }       // slivers
        V3 o = v3(U(g), U(g), U(g)) * (sc * 20);
        V3 tgt;
        int mode = it % 4;
        double a = (U(g) + 1) / 2, b = (U(g) + 1) / 2 * (1 - a);
        if (mode == 0) tgt = p1 + (p2 - p1) * a + (p3 - p1) * b;            // inside
        else if (mode == 1) tgt = p1 + (p2 - p1) * a;                         // on an edge
        else if (mode == 2) tgt = (it % 8 == 2) ? p1 + (p2 - p1) * a + (p3 - p1) * b + cross(p2 - p1, p3 - p1) * (0.02 * U(g) * (a + b) * (1 - a - b) / sc)   // just off the plane: the acceptance angle's edge
                                                : p1 + (p2 - p1) * a + v3(U(g), U(g), U(g)) * (sc * 1e-3);   // near an edge
        else tgt = v3(U(g), U(g), U(g)) * (sc * 2);                           // anywhere
        V3 d = normalize(tgt - o);
        bool r = raw(p1, p2, p3, o, d), f = tri_hit_corners(p1, p2, p3, o, d), u = full(p1, p2, p3, o, d);
        // spurious ExpBox faces (A.4): the third corner reflected through the origin
        bool rs = raw(p1, p2, -p3, o, d), us = full(p1, p2, -p3, o, d), fs = tri_hit_corners(p1, p2, -p3, o, d);
        // nearly parallel rays: tri_hit_corners' parallel test skips the normalisation only when
        // dot(cross(e1, e2), d) is clearly nonzero; here it is 0 or within a few ulps of 0
        const V3 nrm = cross(p2 - p1, p3 - p1);
        V3 dp = d - nrm * (dot(d, nrm) / dot(nrm, nrm));
        if (it % 5 == 0) dp = dp + nrm * (1e-17 * U(g) / std::sqrt(dot(nrm, nrm)));
        if (dot(dp, dp) > 0) {
            dp = normalize(dp);
            const bool rp = raw(p1, p2, p3, o, dp), fp = tri_hit_corners(p1, p2, p3, o, dp);
            if (rp != fp) { ++bad; if (bad < 5) printf("parallel mismatch it=%ld raw=%d corners=%d\n", it, rp, fp); }
        }
        ++n; hits += r;
        if (r != f || r != u || rs != us || rs != fs) { ++bad; if (bad < 5) printf("mismatch it=%ld mode=%d raw=%d full=%d\n", it, mode, r, u); }
        if (mode == 2) near += r;
    }
    // box_hit_part: the OR of its four parts (3 faces each, for four cooperating lanes) is box_hit
    long nb = 0, bhits = 0, bbad = 0;
    for (long it = 0; it < N / 8; ++it) {
        const double sc = std::pow(10.0, 2 * U(g));
        const V3 c = v3(U(g), U(g), U(g)) * (sc * (it % 2 ? 0.5 : 4.0));
        const V3 hw = v3(U(g) + 1.01, U(g) + 1.01, U(g) + 1.01) * (sc * 0.25);
        const V3 mn = c - hw, mx = c + hw;
        const V3 o = v3(U(g), U(g), U(g)) * (sc * 10);
        V3 tgt;
        const int mode = it % 3;
        if (mode == 0) tgt = c + vmul(hw, v3(U(g), U(g), U(g)));               // through the box
        else if (mode == 1) tgt = c + vmul(hw, v3(U(g), U(g), U(g)) * 1.05);   // near its faces
        else tgt = -c + vmul(hw, v3(U(g), U(g), U(g)));                        // its mirror image (A.4)
        const V3 d = normalize(tgt - o);
        const bool b = box_hit(mn, mx, o, d);
        const bool q = box_hit_part(mn, mx, o, d, 0) || box_hit_part(mn, mx, o, d, 1) ||
                       box_hit_part(mn, mx, o, d, 2) || box_hit_part(mn, mx, o, d, 3);
        ++nb; bhits += b;
        if (b != q) { ++bbad; if (bbad < 5) printf("box mismatch it=%ld mode=%d box_hit=%d parts=%d\n", it, mode, b, q); }
    }
    printf("box cases %ld hits %ld box mismatches %ld\n", nb, bhits, bbad);
    bad += bbad;
    printf("cases %ld raw hits %ld near-edge hits %ld mismatches %ld\n", n, hits, near, bad);
    return bad != 0;
}
