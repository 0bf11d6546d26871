// Exhaustive check of the division the kernels use for per-plan constant divisors
// (kgmt_device.h div_by): with y = RN(1/b) (IEEE float division on the host),
//     q0 = RN(a * y);  r = RN(a - q0 * b) (exact, FMA);  q = RN(q0 + r * y)
// must equal the IEEE quotient RN(a / b) bit for bit while the residual r stays
// normal (Markstein's theorem); the kernels take the IEEE division below
// |a| < 2^-100 where the quotient itself is used (dt, v / L), and grid cells use only
// its truncation (D3), which must agree for every input.  All 2^32 float inputs a
// are checked for each divisor given.
//
//   gcc -O2 -mfma -o /tmp/check_fast_division tools/check_fast_division.c -lm
//   /tmp/check_fast_division 1.25 0.15625 10 25 2.5
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

static float f_of(uint32_t u) {
    float f;
    memcpy(&f, &u, 4);
    return f;
}
static uint32_t u_of(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    return u;
}

int main(int argc, char** argv) {
    int bad = 0;
    for (int k = 1; k < argc; ++k) {
        const volatile float b = strtof(argv[k], NULL);
        const volatile float y = 1.0f / b;
        unsigned long long normalMismatch = 0, cellMismatch = 0, tiny = 0;
        for (uint64_t i = 0; i <= 0xffffffffull; ++i) {
            const float a = f_of((uint32_t)i);
            if (isnan(a)) continue;
            const float ref = a / b;
            const float q0 = a * y;
            const float r = fmaf(-q0, b, a);
            const float q = fmaf(r, y, q0);
            if (u_of(q) == u_of(ref)) continue;
            // grid cells use the truncation of the quotient (range-checked, D3)
            const int inR = fabsf(ref) < 2147483648.0f, inQ = fabsf(q) < 2147483648.0f;
            if (inR != inQ || (inR && (int)ref != (int)q)) ++cellMismatch;
            if (fabsf(a) >= 0x1p-100f && isfinite(ref) && isfinite(q0)) {
                if (normalMismatch < 5) printf("  b=%g a=%a ref=%a fast=%a\n", (double)b, a, ref, q);
                ++normalMismatch;
            } else {
                ++tiny;
            }
        }
        printf("b=%-10g y=%a: mismatches |a| >= 2^-100 %llu, below or overflowing %llu, cell mismatches %llu\n", (double)b,
               (double)y, normalMismatch, tiny, cellMismatch);
        bad |= normalMismatch != 0 || cellMismatch != 0;
    }
    return bad;
}
