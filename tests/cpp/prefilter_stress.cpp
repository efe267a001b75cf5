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
        else if (mode == 2) tgt = p1 + (p2 - p1) * a + v3(U(g), U(g), U(g)) * (sc * 1e-3);   // near an edge
        else tgt = v3(U(g), U(g), U(g)) * (sc * 2);                           // anywhere
        V3 d = normalize(tgt - o);
        bool r = raw(p1, p2, p3, o, d), f = tri_hit_corners(p1, p2, p3, o, d);
        ++n; hits += r; if (r != f) { ++bad; if (bad < 5) printf("mismatch it=%ld mode=%d raw=%d\n", it, mode, r); }
        if (mode == 2) near += r;
    }
    printf("cases %ld raw hits %ld near-edge hits %ld mismatches %ld\n", n, hits, near, bad);
    return bad != 0;
}
