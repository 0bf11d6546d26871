// oracle/xorwow_ref.h — TEST INFRASTRUCTURE ONLY (the parity checker; never
// linked into the product library).
//
// CPU restatement of the cuRAND XORWOW generator as the reference uses it:
//   curand_init(seed, subsequence = tid, offset = 0, &state)  (reference src/planners/KGMT.cu:595-600)
//   curand_uniform(&state)                                   (reference src/statePropagator/statePropagator.cu:17-19,
//                                                             src/planners/KGMT.cu:395,463)
// cuRAND is a third-party NVIDIA library (CUDA toolkit, version unpinned by
// the reference's CMakeLists.txt:7) and is absent from this image.  What is
// restated here:
//   * seeding: s0 = lo32(seed) ^ 0xaad26b49, s1 = hi32(seed) ^ 0xf7dcefdd,
//     t0 = 1099087573*s0, t1 = 2591861531*s1, d = 6615241 + t1 + t0,
//     v = {123456789+t0, 362436069^t0, 521288629+t1, 88675123^t1, 5783321+t0}
//     (published cuRAND constants; PARITY UNPINNED against a real cuRAND run —
//     no cuRAND binary or header exists here);
//   * recurrence: Marsaglia xorwow, t = v0^(v0>>2); shift; v4 = (v4^(v4<<4))^(t^(t<<1)); d += 362437; out = v4 + d;
//   * subsequence skip: the state's 160-bit xorshift part is multiplied by
//     A^(2^67 * subsequence) over GF(2); the Weyl counter d is unchanged
//     (2^67 * 362437 = 0 mod 2^32);
//   * uniform: (float)x * 2^-32 + 2^-33 (product exact, one rounding).
// The recurrence and the 2^67 subsequence jump are shared with rocRAND's
// XORWOW (which only differs in its seeding salts/multipliers and uniform
// mapping), so tests/test_xorwow.py pins them against golden vectors produced
// by rocRAND's own engine (tests/golden/xorwow_rocrand_kat.json).
#pragma once

#include <stdint.h>
#include <string.h>
#include <vector>

namespace oracle {

struct XorwowState {
    uint32_t v[5];
    uint32_t d;
};

struct XorwowSeeding {
    uint32_t salt0, salt1, mul0, mul1;
};

static const XorwowSeeding kCurandSeeding = {0xaad26b49u, 0xf7dcefddu, 1099087573u, 2591861531u};
static const XorwowSeeding kRocrandSeeding = {0x2c7f967fu, 0xa03697cbu, 1228688033u, 2073658381u};

inline XorwowState xorwow_seed(uint64_t seed, const XorwowSeeding& k = kCurandSeeding) {
    const uint32_t s0 = (uint32_t)seed ^ k.salt0;
    const uint32_t s1 = (uint32_t)(seed >> 32) ^ k.salt1;
    const uint32_t t0 = k.mul0 * s0;
    const uint32_t t1 = k.mul1 * s1;
    XorwowState st;
    st.d = 6615241u + t1 + t0;
    st.v[0] = 123456789u + t0;
    st.v[1] = 362436069u ^ t0;
    st.v[2] = 521288629u + t1;
    st.v[3] = 88675123u ^ t1;
    st.v[4] = 5783321u + t0;
    return st;
}

inline uint32_t xorwow_next(XorwowState& st) {
    uint32_t t = st.v[0] ^ (st.v[0] >> 2);
    st.v[0] = st.v[1];
    st.v[1] = st.v[2];
    st.v[2] = st.v[3];
    st.v[3] = st.v[4];
    st.v[4] = (st.v[4] ^ (st.v[4] << 4)) ^ (t ^ (t << 1));
    st.d += 362437u;
    return st.v[4] + st.d;
}

inline float curand_uniform_of(uint32_t x) {
    // CURAND_2POW32_INV = 2^-32; (CURAND_2POW32_INV / 2) = 2^-33.
    return (float)x * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
}

inline float xorwow_uniform(XorwowState& st) { return curand_uniform_of(xorwow_next(st)); }

// 160x160 GF(2) matrix, stored by columns: col[i] (5 words) = M * e_i.
struct Gf2Mat {
    uint32_t col[160][5];
};

inline void gf2_apply(const Gf2Mat& m, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int i = 0; i < 160; ++i) {
        if ((in[i >> 5] >> (i & 31)) & 1u) {
            for (int w = 0; w < 5; ++w) r[w] ^= m.col[i][w];
        }
    }
    memcpy(out, r, sizeof(r));
}

inline Gf2Mat gf2_mul(const Gf2Mat& a, const Gf2Mat& b) {   // a * b
    Gf2Mat c;
    for (int i = 0; i < 160; ++i) gf2_apply(a, b.col[i], c.col[i]);
    return c;
}

// One xorshift step as a matrix (the Weyl part is not linear and is skipped).
inline Gf2Mat xorwow_step_matrix() {
    Gf2Mat m;
    for (int i = 0; i < 160; ++i) {
        XorwowState s;
        memset(&s, 0, sizeof(s));
        s.v[i >> 5] = 1u << (i & 31);
        xorwow_next(s);
        memcpy(m.col[i], s.v, sizeof(s.v));
    }
    return m;
}

// J[b] = A^(2^(67+b)): the jump by 2^b subsequences.
class XorwowSubsequenceJumps {
public:
    explicit XorwowSubsequenceJumps(int nbits = 40) {
        Gf2Mat m = xorwow_step_matrix();
        for (int i = 0; i < 67; ++i) m = gf2_mul(m, m);
        for (int b = 0; b < nbits; ++b) {
            jumps_.push_back(m);
            m = gf2_mul(m, m);
        }
    }
    void skip(XorwowState& st, uint64_t subsequence) const {
        for (int b = 0; subsequence; ++b, subsequence >>= 1) {
            if (subsequence & 1u) gf2_apply(jumps_[b], st.v, st.v);
        }
    }
    // One subsequence forward (J[0]).
    void skip_one(XorwowState& st) const { gf2_apply(jumps_[0], st.v, st.v); }

private:
    std::vector<Gf2Mat> jumps_;
};

}  // namespace oracle
