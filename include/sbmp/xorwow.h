// xorwow.h — cuRAND-compatible XORWOW for host and device (curandState's
// generator as the reference uses it: curand_init at KGMT.cu:595-600,
// curand_uniform at statePropagator.cu:17-19 and KGMT.cu:395,463).
//
// State: v[5] + the Weyl counter d (24 B; cuRAND's curandState is 48 B because it
// also carries Box-Muller scratch the reference never uses).  Seeding restates
// cuRAND's published curand_init scrambling; the subsequence skip-ahead (2^67 per
// subsequence) needs precomputed GF(2) jump matrices and lives in the library
// (k_init_slots / xorwow_jump.cpp).  PARITY UNPINNED for the seeding constants
// (DESIGN.md §3): no cuRAND output is available here to check them against.
#pragma once

#include "sbmp/sbmp_math.h"

namespace sbmp {

struct Xorwow {
    uint32_t v0, v1, v2, v3, v4, d;
};

// One step of the xorwow recurrence (Marsaglia 2003, as in cuRAND / rocRAND).
SBMP_HD uint32_t xorwow_next(Xorwow& s) {
    const uint32_t t = s.v0 ^ (s.v0 >> 2);
    s.v0 = s.v1;
    s.v1 = s.v2;
    s.v2 = s.v3;
    s.v3 = s.v4;
    s.v4 = (s.v4 ^ (s.v4 << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    return s.v4 + s.d;
}

// curand_init(seed, 0, 0): cuRAND's XORWOW seeding (_curand_init_scratch: salts
// 0xaad26b49 / 0xf7dcefdd, multipliers 1099087573 / 2591861531), no skip-ahead.
SBMP_HD Xorwow xorwow_seed(uint64_t seed) {
    const uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u;
    const uint32_t s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    const uint32_t t0 = 1099087573u * s0;
    const uint32_t t1 = 2591861531u * s1;
    Xorwow st;
    st.d = 6615241u + t1 + t0;
    st.v0 = 123456789u + t0;
    st.v1 = 362436069u ^ t0;
    st.v2 = 521288629u + t1;
    st.v3 = 88675123u ^ t1;
    st.v4 = 5783321u + t0;
    return st;
}

// curand_uniform: x * 2^-32 + 2^-33 (product exact, one rounding), in (0, 1].  Written as
// one fused multiply-add: the product of the converted integer and a power of two is
// exact, so the FMA rounds the same sum once, as the multiply-then-add does (one VALU per
// draw instead of two; the oracle's restatement keeps the two operations, same bits).
SBMP_HD float xorwow_uniform(Xorwow& s) {
    return __builtin_fmaf((float)xorwow_next(s), 2.3283064365386963e-10f, 1.1641532182693481e-10f);
}

}  // namespace sbmp
