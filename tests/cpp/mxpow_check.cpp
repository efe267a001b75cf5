// CPU check of gi_math.h's mx_pow (Mode X specular power for any double exponent): relative error
// against libm pow over x in (0, 1] and many exponents; special cases.  Prints "maxrel <e> bad <n>".
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>

#include "gi_math.h"

int main() {
    using gi::mx_pow;
    double maxrel = 0.0;
    long bad = 0;
    uint64_t s = 12345;
    auto rnd = [&]() { s = s * 6364136223846793005ULL + 1442695040888963407ULL; return (double)(s >> 11) * 0x1.0p-53; };
    const double ps[] = {0.25, 0.5, 1.5, 2.75, 5.5, 7.0 / 3.0, 31.9, 64.5, 100.0, 1000.0, -0.5, -3.25};
    for (double p : ps) {
        for (int i = 0; i < 200000; ++i) {
            double x = rnd();
            if (i % 4 == 0) x = std::pow(x, 8.0);   // small arguments too
            if (x == 0.0) continue;
            const double r = std::pow(x, p), g = mx_pow(x, p);
            if (r == 0.0 || std::isinf(r)) { if (g != r) ++bad; continue; }
            if (r < 1e-300) continue;   // subnormal results: absolute accuracy only
            const double rel = std::fabs(g - r) / std::fabs(r);
            // the exponent amplifies ln's rounding: |p ln x| * 2^-52 relative, plus a few ulps
            const double tol = 8e-16 + std::fabs(p * std::log(x)) * 8e-16;
            if (!(rel <= tol)) ++bad;
            if (rel > maxrel && rel <= 1.0) maxrel = rel;
        }
    }
    // integer exponents in [0, 64]: square-and-multiply, as before
    for (int p = 0; p <= 64; ++p) {
        const double x = 0.8125;
        if (mx_pow(x, (double)p) != gi::mx_powi(x, p)) ++bad;
    }
    if (mx_pow(0.0, 2.5) != 0.0 || !std::isinf(mx_pow(0.0, -1.5)) || mx_pow(1.0, 5.5) != 1.0 || !std::isnan(mx_pow(NAN, 2.5)))
        ++bad;
    printf("maxrel %.3g bad %ld\n", maxrel, bad);
    return bad ? 1 : 0;
}
