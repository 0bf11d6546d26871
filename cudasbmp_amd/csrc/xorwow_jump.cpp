// xorwow_jump.cpp — host precomputation for curand_init(seed, subsequence, 0)
// (reference src/planners/KGMT.cu:595-600).
//
// cuRAND's XORWOW subsequences are 2^67 draws apart.  The xorshift part of the
// state (160 bits) advances linearly over GF(2): v' = A v.  Jumping s
// subsequences multiplies by A^(2^67 s); with J[b] = A^(2^(67+b)) the jump is
// the product of J[b] over the set bits b of s (the powers commute).  The Weyl
// counter d needs no jump (2^67 * 362437 = 0 mod 2^32).  The matrices are built
// once per process by repeated squaring (67 + nbits squarings of a 160x160
// bit matrix, a few ms) and uploaded for k_init_slots.
#include <mutex>
#include <vector>

#include "kgmt_launch.h"

namespace sbmp {

namespace {

struct Mat {
    uint32_t c[160][5];   // c[i] = A * e_i
};

void apply(const Mat& m, const uint32_t in[5], uint32_t out[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int w = 0; w < 5; ++w) {
        uint32_t bits = in[w];
        while (bits) {
            const int k = __builtin_ctz(bits);
            bits &= bits - 1;
            const uint32_t* col = m.c[w * 32 + k];
            for (int q = 0; q < 5; ++q) r[q] ^= col[q];
        }
    }
    for (int q = 0; q < 5; ++q) out[q] = r[q];
}

Mat square(const Mat& m) {
    Mat r;
    for (int i = 0; i < 160; ++i) apply(m, m.c[i], r.c[i]);
    return r;
}

Mat step_matrix() {
    Mat m;
    for (int i = 0; i < 160; ++i) {
        uint32_t words[5] = {0, 0, 0, 0, 0};
        words[i >> 5] = 1u << (i & 31);
        Xorwow s{words[0], words[1], words[2], words[3], words[4], 0};
        xorwow_next(s);
        m.c[i][0] = s.v0;
        m.c[i][1] = s.v1;
        m.c[i][2] = s.v2;
        m.c[i][3] = s.v3;
        m.c[i][4] = s.v4;
    }
    return m;
}

std::mutex g_mu;
std::vector<uint32_t> g_jumps;   // flattened J[0..g_nbits)
int g_nbits = 0;

}  // namespace

Xorwow curand_seed_state(uint64_t seed) { return xorwow_seed(seed); }

const std::vector<uint32_t>& subsequence_jump_matrices(int nbits) {
    std::lock_guard<std::mutex> lock(g_mu);
    if (nbits <= g_nbits) return g_jumps;
    Mat m = step_matrix();
    for (int i = 0; i < 67; ++i) m = square(m);
    std::vector<uint32_t> out;
    out.reserve((size_t)nbits * 800);
    for (int b = 0; b < nbits; ++b) {
        for (int i = 0; i < 160; ++i)
            for (int q = 0; q < 5; ++q) out.push_back(m.c[i][q]);
        m = square(m);
    }
    g_jumps.swap(out);
    g_nbits = nbits;
    return g_jumps;
}

}  // namespace sbmp
