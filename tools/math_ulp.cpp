// Exhaustive accuracy of the shared transcendentals (include/sbmp/sbmp_math.h, D9) over
// the Cody-Waite range, against a double-precision reference.
//
//   g++ -O2 -std=c++17 -fopenmp -ffp-contract=off -I include tools/math_ulp.cpp -o /tmp/math_ulp
//   /tmp/math_ulp [stride] [limit]      (stride 1: every float; limit default 105615)
//
// Every float x with |x| <= limit (both signs, stride apart in bit pattern) is passed to
// sinf_d / cosf_d / tanf_d, and the result is compared with sin / cos / tan of the same
// x in double (glibc, error < 1 ulp of double, i.e. 2^-29 ulp of float).  The error is
// |f(x) - ref| in units of the float ulp of ref (ulp(y) = 2^(floor(log2|y|) - 23),
// 2^-149 below the normal range), the measure CUDA's programming guide uses for its
// single-precision bounds (sinf, cosf: 2 ulp; tanf: 4 ulp; full range).  Printed: the
// maximum per function and per binade of |x|, with the argument where it occurs.
#include <omp.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "sbmp/sbmp_math.h"

static double ulp_of(double y) {
    const double a = std::fabs(y);
    if (a < 0x1p-126) return 0x1p-149;
    int e;
    std::frexp(a, &e);   // a in [2^(e-1), 2^e)
    return std::ldexp(1.0, e - 1 - 23);
}

struct Worst {
    double err = 0.0;
    float x = 0.0f;
};

int main(int argc, char** argv) {
    const uint32_t stride = argc > 1 ? (uint32_t)strtoul(argv[1], nullptr, 10) : 1u;
    const float limit = argc > 2 ? strtof(argv[2], nullptr) : 105615.0f;
    uint32_t top;
    std::memcpy(&top, &limit, 4);
    constexpr int kBins = 160;   // binade of |x|: exponent field (0 = zero / subnormal)
    Worst ws[3][kBins], wt[3];
    unsigned long long n = 0;
#pragma omp parallel
    {
        Worst w[3][kBins], tot[3];
        unsigned long long cnt = 0;
#pragma omp for schedule(dynamic, 1 << 16)
        for (long long u = 0; u <= (long long)top; u += stride) {
            for (int sgn = 0; sgn < 2; ++sgn) {
                const uint32_t bits = (uint32_t)u | (sgn ? 0x80000000u : 0u);
                float x;
                std::memcpy(&x, &bits, 4);
                float s, c;
                sbmp::sincosf_d(x, &s, &c);
                const float t = sbmp::tanf_d(x);
                const double xd = (double)x;
                const double ref[3] = {std::sin(xd), std::cos(xd), std::tan(xd)};
                const float got[3] = {s, c, t};
                const int bin = (int)(((uint32_t)u >> 23) & 0xff);
                for (int f = 0; f < 3; ++f) {
                    const double e = std::fabs((double)got[f] - ref[f]) / ulp_of(ref[f]);
                    if (e > w[f][bin].err) w[f][bin] = {e, x};
                    if (e > tot[f].err) tot[f] = {e, x};
                }
                ++cnt;
            }
        }
#pragma omp critical
        {
            n += cnt;
            for (int f = 0; f < 3; ++f) {
                if (tot[f].err > wt[f].err) wt[f] = tot[f];
                for (int b = 0; b < kBins; ++b)
                    if (w[f][b].err > ws[f][b].err) ws[f][b] = w[f][b];
            }
        }
    }
    const char* names[3] = {"sinf", "cosf", "tanf"};
    printf("sbmp_math.h against double libm: %llu arguments, |x| <= %.9g, stride %u (%s)\n", n, (double)limit, stride,
           stride == 1 ? "every float" : "sampled");
    for (int f = 0; f < 3; ++f)
        printf("%s  max %.4f ulp at x = %.9g (0x%08x)\n", names[f], wt[f].err, (double)wt[f].x,
               [&] { uint32_t b; std::memcpy(&b, &wt[f].x, 4); return b; }());
    printf("\nper binade of |x| (max ulp: sinf cosf tanf)\n");
    for (int b = 0; b < kBins; ++b) {
        if (ws[0][b].err == 0.0 && ws[1][b].err == 0.0 && ws[2][b].err == 0.0) continue;
        printf("  [2^%4d, 2^%4d)  %8.4f %8.4f %8.4f\n", b - 127, b - 126, ws[0][b].err, ws[1][b].err, ws[2][b].err);
    }
    return 0;
}
