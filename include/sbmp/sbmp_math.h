// sbmp_math.h — deterministic single-precision sin/cos/tan shared by the HIP
// kernels and the CPU oracle (canonical-semantics decision D9).
//
// The reference calls CUDA libdevice cosf/sinf/tanf inside the propagation
// loop (reference src/statePropagator/statePropagator.cu:34-36).  Neither
// libdevice nor ocml nor glibc produce the same bits as each other, and the
// north star asks for bit-exact accept masks, so the build defines the
// transcendentals once, in plain IEEE float operations, and compiles this one
// header for the host (g++) and for gfx950 (hipcc) with -ffp-contract=off.
// Every multiply-add that should be fused is written as an explicit fmaf, so
// the operation sequence is identical on both sides.
//
// Algorithm (the classic structure libdevice also uses):
//   * |x| <= 105615: Cody-Waite reduction by pi/2 with a 3-part constant and
//     fmaf (exact enough for |quadrant| < 2^17);
//   * larger |x|: Payne-Hanek reduction against 224 bits of 2/pi, integer
//     arithmetic, final scaling in double;
//   * minimax polynomials on [-pi/4, pi/4] (Cephes sinf/cosf/tanf
//     coefficients), quadrant selection.
// Accuracy is checked against float64 libm in tests/test_math.py (<= 2 ulp
// for sin/cos, <= 3 ulp for tan over the tested ranges).
#pragma once

#include <stdint.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define SBMP_HD __host__ __device__ __forceinline__
#else
#define SBMP_HD static inline
#endif

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace sbmp {

SBMP_HD uint32_t f2u(float f) {
    union { float f; uint32_t u; } c;
    c.f = f;
    return c.u;
}
SBMP_HD float u2f(uint32_t u) {
    union { float f; uint32_t u; } c;
    c.u = u;
    return c.f;
}

// 2/pi, most significant 32-bit word first (0.A2F9836E 4E441529 ...).
// tests/test_math.py re-derives these words from an integer Machin series.
#define SBMP_TWO_OVER_PI_WORDS 7

SBMP_HD uint32_t two_over_pi_word(int i) {
    // A switch instead of a table keeps the header free of device globals.
    switch (i) {
        case 0: return 0xA2F9836Eu;
        case 1: return 0x4E441529u;
        case 2: return 0xFC2757D1u;
        case 3: return 0xF534DDC0u;
        case 4: return 0xDB629599u;
        case 5: return 0x3C439041u;
        default: return 0xFE5163ABu;
    }
}

// Payne-Hanek: returns r with x = (q + r/(pi/2)) * pi/2, |r| <= pi/4.
// Precondition: x finite, |x| >= 2^16.
SBMP_HD float reduce_payne_hanek(float x, int* q_out) {
    const uint32_t ix = f2u(x);
    const uint32_t sign = ix >> 31;
    const int E = (int)((ix >> 23) & 0xffu) - 127;        // x in [2^E, 2^(E+1))
    const uint32_t ia = (ix << 8) | 0x80000000u;          // x = ia * 2^(E-31)
    // Q = ia * (2/pi * 2^224), a 256-bit integer held in 8 little-endian words.
    uint32_t Q[SBMP_TWO_OVER_PI_WORDS + 1];
    uint64_t carry = 0;
    for (int i = SBMP_TWO_OVER_PI_WORDS - 1; i >= 0; --i) {   // least significant word first
        const uint64_t p = (uint64_t)ia * (uint64_t)two_over_pi_word(i) + carry;
        Q[SBMP_TWO_OVER_PI_WORDS - 1 - i] = (uint32_t)p;
        carry = p >> 32;
    }
    Q[SBMP_TWO_OVER_PI_WORDS] = (uint32_t)carry;
    // x*2/pi = Q * 2^(E-255): the binary point sits at bit p = 255 - E.
    // Take the 64-bit window W = Q[p-62 .. p+1]: 2 integer bits + 62 fraction bits.
    // 16 <= E <= 127 (|x| >= 2^16, finite), so lo_bit is in [66, 177] and the window
    // starts in word 2..5: three 4-way selects, then two 32-bit funnel shifts
    // (v_alignbit_b32 on the device).  The same bits as shifting the whole of Q.
    const int lo_bit = 255 - E - 62;
    const int wi = lo_bit >> 5;
    const int sh = lo_bit & 31;
    const uint32_t w0 = wi <= 2 ? Q[2] : wi == 3 ? Q[3] : wi == 4 ? Q[4] : Q[5];
    const uint32_t w1 = wi <= 2 ? Q[3] : wi == 3 ? Q[4] : wi == 4 ? Q[5] : Q[6];
    const uint32_t w2 = wi <= 2 ? Q[4] : wi == 3 ? Q[5] : wi == 4 ? Q[6] : Q[7];
#if defined(__HIP_DEVICE_COMPILE__)
    const uint32_t lo = __builtin_amdgcn_alignbit(w1, w0, (uint32_t)sh);
    const uint32_t hi = __builtin_amdgcn_alignbit(w2, w1, (uint32_t)sh);
#else
    const uint32_t lo = (uint32_t)((((uint64_t)w1 << 32) | w0) >> sh);
    const uint32_t hi = (uint32_t)((((uint64_t)w2 << 32) | w1) >> sh);
#endif
    const uint64_t W = ((uint64_t)hi << 32) | lo;
    int q = (int)(W >> 62);
    int64_t f = (int64_t)(W & 0x3fffffffffffffffull);     // fraction in 0.62 fixed point
    if (f >= (int64_t)0x2000000000000000ll) {              // fraction >= 1/2: round quadrant up
        q += 1;
        f -= (int64_t)0x4000000000000000ll;
    }
    double d = (double)f * 3.4061215800865545e-19;         // (pi/2) * 2^-62
    float r = (float)d;
    if (sign) {
        r = -r;
        q = -q;
    }
    *q_out = q;
    return r;
}

// Reduce by pi/2: returns r in about [-pi/4, pi/4] and the quadrant q.
SBMP_HD float reduce_pio2(float x, int* q) {
    const float ax = __builtin_fabsf(x);
    if (ax <= 105615.0f) {
        const float j = __builtin_rintf(x * 0.636619772f);
        float r = __builtin_fmaf(j, -1.57079601e+00f, x);
        r = __builtin_fmaf(j, -3.13916473e-07f, r);
        r = __builtin_fmaf(j, -5.39030253e-15f, r);
        *q = (int)j;
        return r;
    }
    return reduce_payne_hanek(x, q);
}

SBMP_HD float sin_poly(float r) {   // sin on [-pi/4, pi/4]
    const float z = r * r;
    float p = __builtin_fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f);
    p = __builtin_fmaf(p, z, -1.6666654611e-1f);
    return __builtin_fmaf(p * z, r, r);
}

SBMP_HD float cos_poly(float r) {   // cos on [-pi/4, pi/4]
    const float z = r * r;
    float p = __builtin_fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f);
    p = __builtin_fmaf(p, z, 4.166664568298827e-2f);
    return __builtin_fmaf(p * z, z, __builtin_fmaf(-0.5f, z, 1.0f));
}

SBMP_HD float tan_poly(float r) {   // tan on [-pi/4, pi/4]
    const float z = r * r;
    float p = __builtin_fmaf(9.38540185543e-3f, z, 3.11992232697e-3f);
    p = __builtin_fmaf(p, z, 2.44301354525e-2f);
    p = __builtin_fmaf(p, z, 5.34112807005e-2f);
    p = __builtin_fmaf(p, z, 1.33387994085e-1f);
    p = __builtin_fmaf(p, z, 3.33331568548e-1f);
    return __builtin_fmaf(p * z, r, r);
}

SBMP_HD bool finitef(float x) { return (f2u(x) & 0x7f800000u) != 0x7f800000u; }

// sin and cos of one argument with a shared reduction.  Bitwise equal to
// sinf_d(x) / cosf_d(x) below (same operations on the same reduced value).
SBMP_HD void sincosf_d(float x, float* s, float* c) {
    if (!finitef(x)) {
        *s = x - x;
        *c = x - x;
        return;
    }
    int q;
    const float r = reduce_pio2(x, &q);
    const float sp = sin_poly(r);
    const float cp = cos_poly(r);
    // Quadrant q mod 4: (s, c) = (sp, cp), (cp, -sp), (-sp, -cp), (-cp, sp).
    // Branch-free: swap on odd q, then exact sign flips (bit 1 of q for s,
    // bit 1 of q+1 for c).
    const bool odd = (q & 1) != 0;
    const float s0 = odd ? cp : sp;
    const float c0 = odd ? sp : cp;
    *s = u2f(f2u(s0) ^ ((uint32_t)(q & 2) << 30));
    *c = u2f(f2u(c0) ^ ((uint32_t)((q + 1) & 2) << 30));
}

SBMP_HD float sinf_d(float x) {
    float s, c;
    sincosf_d(x, &s, &c);
    return s;
}

SBMP_HD float cosf_d(float x) {
    float s, c;
    sincosf_d(x, &s, &c);
    return c;
}

SBMP_HD float tanf_d(float x) {
    if (!finitef(x)) return x - x;
    int q;
    const float r = reduce_pio2(x, &q);
    const float t = tan_poly(r);
    return (q & 1) ? -1.0f / t : t;
}

}  // namespace sbmp
