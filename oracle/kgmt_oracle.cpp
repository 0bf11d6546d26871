// oracle/kgmt_oracle.cpp — TEST INFRASTRUCTURE ONLY.
//
// CPU restatement of the reference KGMT planner, written to follow the
// reference's own structure (boolean G/GNew arrays scanned over all M slots,
// findInd compaction, propagateG / propagateGV2 slot mapping, updateR1,
// updateG), so that the GPU build's different data structures (contiguous
// frontier range, GNew bitmask, fused kernels) are checked against a literal
// restatement.  Every function cites the reference file:line it follows.
// Canonical-semantics decisions D1-D13 resolve the places where
// the reference is racy or undefined.
//
// Pinning: the reference cannot be built here (CUDA/thrust/cub/curand absent,
// SURVEY.md §8c) and ships no tests or golden vectors, so this oracle is pinned
// by (i) the reference's RNG-independent invariants I1-I6 (tests/test_oracle.py),
// (ii) rocRAND known-answer vectors for the XORWOW recurrence and 2^67 jump
// (tests/test_xorwow.py), and (iii) its own committed golden fixtures
// (tests/golden/) for regression.  Bit-parity with a real CUDA run is
// unverifiable here (PARITY UNPINNED for cuRAND seeding constants and CUDA
// libdevice transcendental bits).
#include "kgmt_oracle.h"

#include <algorithm>
#include <climits>
#include <cmath>
#include <cstring>
#include <vector>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "sbmp/sbmp_math.h"
#include "xorwow_ref.h"

#if defined(__GNUC__) && !defined(__clang__)
#pragma GCC optimize("fp-contract=off")
#endif

namespace {

constexpr int SAMPLE_DIM = 7;   // KGMT.cu:5
constexpr int WS_DIM = 2;       // statePropagator.cu:3, collisionCheck.cu:3
constexpr int OWNER_BLOCK = 256;

// reference KGMT.cu:602-609 (getR1).  Float->int is a truncation toward zero;
// an out-of-int-range or NaN quotient (undefined in C++) maps to -1 (D3).
int to_cell(float q, bool* ok) {
    if (!(q > -2147483648.0f && q < 2147483648.0f)) {
        *ok = false;
        return 0;
    }
    *ok = true;
    return (int)q;
}

int getR1(float x, float y, float R1Size, int N) {
    bool okx, oky;
    const int cellX = to_cell(x / R1Size, &okx);
    const int cellY = to_cell(y / R1Size, &oky);
    if (okx && oky && cellX >= 0 && cellX < N && cellY >= 0 && cellY < N) return cellY * N + cellX;
    return -1;
}

// reference KGMT.cu:610-629 (getR2).
int getR2(float x, float y, int r1, float R1Size, int N, float R2Size, int n) {
    if (r1 == -1) return -1;
    const int cellY_R1 = r1 / N;
    const int cellX_R1 = r1 % N;
    // nvcc contracts x - c * R1Size into fma(-c, R1Size, x) (-fmad=true, D10)
    const float localX = fmaf(-(float)cellX_R1, R1Size, x);
    const float localY = fmaf(-(float)cellY_R1, R1Size, y);
    bool okx, oky;
    const int cellX_R2 = to_cell(localX / R2Size, &okx);
    const int cellY_R2 = to_cell(localY / R2Size, &oky);
    if (okx && oky && cellX_R2 >= 0 && cellX_R2 < n && cellY_R2 >= 0 && cellY_R2 < n)
        return r1 * (n * n) + cellY_R2 * n + cellX_R2;
    return -1;
}

// reference collisionCheck.cu:6-14 (isBroadPhaseValid): free iff separated on some axis.
bool isBroadPhaseValid(const float* bbMin, const float* bbMax, const float* obs) {
    for (int d = 0; d < WS_DIM; ++d) {
        if (bbMax[d] <= obs[d] || obs[WS_DIM + d] <= bbMin[d]) return true;
    }
    return false;
}

// reference collisionCheck.cu:16-28 (isMotionValid).
bool isMotionValid(const float* bbMin, const float* bbMax, const float* obstacles, int count) {
    for (int i = 0; i < count; ++i) {
        if (!isBroadPhaseValid(bbMin, bbMax, &obstacles[i * 2 * WS_DIM])) return false;
    }
    return true;
}

// Large obstacle lists (the c5 field: 10,000 boxes): the same boolean as
// isMotionValid, as an order-independent OR over structure-of-arrays copies of the
// boxes in chunks of 64 (branch-free inside a chunk, so the compiler vectorises it;
// early exit between chunks).  Any overlapping box makes the segment invalid, so the
// answer does not depend on the order in which boxes are tested.
struct ObsSoA {
    std::vector<float> x0, y0, x1, y1;
    int n = 0;
    void assign(const float* obstacles, int count) {
        n = count;
        x0.resize(count);
        y0.resize(count);
        x1.resize(count);
        y1.resize(count);
        for (int i = 0; i < count; ++i) {
            x0[i] = obstacles[4 * i];
            y0[i] = obstacles[4 * i + 1];
            x1[i] = obstacles[4 * i + 2];
            y1[i] = obstacles[4 * i + 3];
        }
    }
};
constexpr int kSoAMinObs = 64;

bool isMotionValidSoA(const float* bbMin, const float* bbMax, const ObsSoA& o) {
    const float bx0 = bbMin[0], by0 = bbMin[1], bx1 = bbMax[0], by1 = bbMax[1];
    for (int i0 = 0; i0 < o.n; i0 += 64) {
        const int i1 = std::min(o.n, i0 + 64);
        int hit = 0;
        for (int i = i0; i < i1; ++i)   // isBroadPhaseValid negated, NaN-exact (!(a <= b))
            hit |= (int)(!(bx1 <= o.x0[i])) & (int)(!(o.x1[i] <= bx0)) & (int)(!(by1 <= o.y0[i])) &
                   (int)(!(o.y1[i] <= by0));
        if (hit) return false;
    }
    return true;
}

void segment_aabb(const float* v_state, const float* w_state, float* bbMin, float* bbMax) {
    // statePropagator.cu:52-60
    for (int d = 0; d < WS_DIM; ++d) {
        if (v_state[d] > w_state[d]) {
            bbMin[d] = w_state[d];
            bbMax[d] = v_state[d];
        } else {
            bbMin[d] = v_state[d];
            bbMax[d] = w_state[d];
        }
    }
}

struct PropCfg {
    int numDisc;
    float agentLength, width, height;
    const float* obstacles;
    int obstaclesCount;
    const ObsSoA* soa;   // non-null for large lists (isMotionValidSoA)
};

bool motion_valid(const float* bbMin, const float* bbMax, const PropCfg& c) {
    if (c.soa) return isMotionValidSoA(bbMin, bbMax, *c.soa);
    return isMotionValid(bbMin, bbMax, c.obstacles, c.obstaclesCount);
}

// reference statePropagator.cu:5-76 (propagateAndCheck), car / kinematic bicycle.
// Contraction choices (D10): a = fmaf(u,10,-5); steering in double with one fma (D11);
// x = fmaf(v*cos, dt, x); y likewise; theta = fmaf((v/L)*tan, dt, theta); v = fmaf(a, dt, v).
// tanf(steering) is loop-invariant: evaluated once (bitwise identical to per-step).
bool propagate_car(const float* x0, float* x1, oracle::XorwowState& rs, const PropCfg& c) {
    const float a = fmaf(oracle::xorwow_uniform(rs), 10.0f, -5.0f);
    const float u2 = oracle::xorwow_uniform(rs);
    const float steering = (float)std::fma((double)(u2 * 2.0f), M_PI, -M_PI);
    const float duration = fmaf(oracle::xorwow_uniform(rs), 1.0f, 0.05f);
    const float dt = duration / (float)c.numDisc;
    float x = x0[0], y = x0[1], theta = x0[2], v = x0[3];
    const float tan_steering = sbmp::tanf_d(steering);
    bool motionValid = true;
    for (int i = 0; i < c.numDisc; ++i) {
        const float v_state[WS_DIM] = {x, y};
        float sin_theta, cos_theta;
        sbmp::sincosf_d(theta, &sin_theta, &cos_theta);
        x = fmaf(v * cos_theta, dt, x);
        y = fmaf(v * sin_theta, dt, y);
        if (x <= 0.0f || x >= c.width || y <= 0.0f || y >= c.height) {
            motionValid = false;
            break;
        }
        theta = fmaf((v / c.agentLength) * tan_steering, dt, theta);
        v = fmaf(a, dt, v);
        const float w_state[WS_DIM] = {x, y};
        float bbMin[WS_DIM], bbMax[WS_DIM];
        segment_aabb(v_state, w_state, bbMin, bbMax);
        motionValid = motionValid && motion_valid(bbMin, bbMax, c);
        if (!motionValid) break;
    }
    x1[0] = x;
    x1[1] = y;
    x1[2] = theta;
    x1[3] = v;
    x1[4] = a;
    x1[5] = steering;
    x1[6] = duration;
    return motionValid;
}

// Build extension (no reference counterpart): holonomic R2 point agent
// in the same skeleton.  Controls (vx, vy) in (-1, 1]^2, duration as the car.
bool propagate_point(const float* x0, float* x1, oracle::XorwowState& rs, const PropCfg& c) {
    const float vx = fmaf(oracle::xorwow_uniform(rs), 2.0f, -1.0f);
    const float vy = fmaf(oracle::xorwow_uniform(rs), 2.0f, -1.0f);
    const float duration = fmaf(oracle::xorwow_uniform(rs), 1.0f, 0.05f);
    const float dt = duration / (float)c.numDisc;
    float x = x0[0], y = x0[1];
    bool motionValid = true;
    for (int i = 0; i < c.numDisc; ++i) {
        const float v_state[WS_DIM] = {x, y};
        x = fmaf(vx, dt, x);
        y = fmaf(vy, dt, y);
        if (x <= 0.0f || x >= c.width || y <= 0.0f || y >= c.height) {
            motionValid = false;
            break;
        }
        const float w_state[WS_DIM] = {x, y};
        float bbMin[WS_DIM], bbMax[WS_DIM];
        segment_aabb(v_state, w_state, bbMin, bbMax);
        motionValid = motionValid && motion_valid(bbMin, bbMax, c);
        if (!motionValid) break;
    }
    x1[0] = x;
    x1[1] = y;
    x1[2] = 0.0f;
    x1[3] = 0.0f;
    x1[4] = vx;
    x1[5] = vy;
    x1[6] = duration;
    return motionValid;
}

// CUB BlockReduce<float,256>::Sum in BLOCK_REDUCE_WARP_REDUCTIONS order (D8):
// per 32-lane group a shfl-down tree (offsets 1,2,4,8,16 = balanced pairwise tree),
// then warp aggregates added sequentially.  reference KGMT.cu:520-522.
float cub_block_sum_256(const float* x) {
    float total = 0.0f;
    for (int w = 0; w < 8; ++w) {
        float t[32];
        for (int i = 0; i < 32; ++i) t[i] = x[w * 32 + i];
        for (int off = 1; off < 32; off <<= 1) {
            for (int i = 0; i + off < 32; i += 2 * off) t[i] = t[i] + t[i + off];
        }
        total = (w == 0) ? t[0] : total + t[0];
    }
    return total;
}

struct LocalOut {   // per-slot expansion result, applied to the region tables afterwards
    int r1, r2;
    uint8_t valid, accept;
};

class Oracle {
public:
    explicit Oracle(const oracle_params& p) : p_(p) {
        M_ = p.maxTreeSize;
        R1Size_ = p.width / (float)p.N;           // KGMT.cu:13
        R2Size_ = p.width / (float)(p.n * p.N);   // KGMT.cu:14
        nR1_ = p.N * p.N;
        nR2_ = nR1_ * p.n * p.n;
        P_ = p.nranks > 0 ? p.nranks : 1;
        rank_ = p.rank;
        nSlots_ = p.samplesPerIteration > 0 ? std::min(M_, p.samplesPerIteration) : M_;
    }

    bool owns(int slot) const { return ((slot / OWNER_BLOCK) % P_) == rank_; }

    int begin(const float* initial, const float* goal, const float* obstacles, int nObs, uint64_t seed) {
        // Constructor state (KGMT.cu:16-72): zero-filled vectors, parents -1, R1Score 1.0.
        samples_.assign((size_t)M_ * SAMPLE_DIM, 0.0f);
        unexplored_.assign((size_t)M_ * SAMPLE_DIM, 0.0f);
        parent_.assign(M_, -1);
        uParent_.assign(M_, -1);
        G_.assign(M_, 0);
        GNew_.assign(M_, 0);
        costs_.assign(M_, 0.0f);
        R1_.assign(nR1_, 0);
        R1Avail_.assign(nR1_, 0);
        R1Valid_.assign(nR1_, 0);
        R1Invalid_.assign(nR1_, 0);
        R1Score_.assign(nR1_, 1.0f);
        R2_.assign(nR2_, 0);
        R2Avail_.assign(nR2_, 0);
        R2Valid_.assign(nR2_, 0);
        R2Invalid_.assign(nR2_, 0);
        obstacles_.assign(obstacles, obstacles + (size_t)nObs * 2 * WS_DIM);
        nObs_ = nObs;
        soa_.assign(obstacles, nObs);
        memcpy(goal_, goal, sizeof(goal_));
        logs_.clear();
        samplesGenerated_ = 0;

        // KGMT.cu:85-97: root row, G[0], root region seeds.
        for (int i = 0; i < SAMPLE_DIM; ++i) samples_[i] = initial[i];
        G_[0] = 1;
        const int r1_0 = getR1(initial[0], initial[1], R1Size_, p_.N);
        const int r2_0 = getR2(initial[0], initial[1], r1_0, R1Size_, p_.N, R2Size_, p_.n);
        if (r1_0 >= 0) {   // D3: the reference fills index -1 otherwise (out of bounds)
            R1_[r1_0] = 1;
            R1Avail_[r1_0] = 1;
            R1Valid_[r1_0] = 1;
        }
        if (r2_0 >= 0) R2Avail_[r2_0] = 1;

        // KGMT.cu:109-111: curand_init(seed, subsequence = slot, 0) for every slot (D1).
        rng_.assign(nSlots_, oracle::XorwowState());
        const oracle::XorwowState base = oracle::xorwow_seed(seed);
        int nbits = 1;
        while ((1ll << nbits) < nSlots_) ++nbits;
        oracle::XorwowSubsequenceJumps jumps(nbits + 1);
        const int chunk = 4096;
        const int nChunks = (nSlots_ + chunk - 1) / chunk;
#pragma omp parallel for schedule(dynamic) num_threads(threads())
        for (int c = 0; c < nChunks; ++c) {
            const int s0 = c * chunk;
            const int s1 = std::min(nSlots_, s0 + chunk);
            oracle::XorwowState st = base;
            jumps.skip(st, (uint64_t)s0);
            for (int s = s0; s < s1; ++s) {
                rng_[s] = st;
                jumps.skip_one(st);
            }
        }

        itr_ = 0;
        treeSize_ = 1;       // KGMT.cu:114
        costToGoal_ = 0.0f;  // D4: d_costToGoal is never initialised in the reference
        goalIdx_ = -1;
        terminated_ = false;
        return 0;
    }

    int threads() const { return p_.threads > 0 ? p_.threads : 1; }

    // KGMT.cu:485-538 (updateR1).  D12: the R1Avail scan and R1Threshold are dead.
    void updateR1() {
        std::vector<float> score(256, 0.0f);
        const int nn = p_.n * p_.n;
        const float epsilon = 0.01f;   // KGMT.cu:133
        for (int t = 0; t < nR1_; ++t) {
            float s = 0.0f;
            if (R1Avail_[t] != 0) {
                const int nValid = R1Valid_[t];
                float covR = 0.0f;
                for (int i = t * nn; i < (t + 1) * nn; ++i) covR += (float)R2Avail_[i];
                covR = covR / (float)nn;
                const float freeVol = (epsilon + (float)nValid) / (epsilon + (float)nValid + (float)R1Invalid_[t]);
                // pow(freeVol,4) in float as (fv^2)^2; pow(R1,2) in double (int args promote).
                const float fv2 = freeVol * freeVol;
                const float fv4 = fv2 * fv2;
                const double den = (double)(1.0f + covR) * (1.0 + (double)R1_[t] * (double)R1_[t]);
                s = (float)((double)fv4 / den);
            }
            score[t] = s;
        }
        const float total = cub_block_sum_256(score.data());
        for (int t = 0; t < nR1_; ++t) R1Score_[t] = (R1Avail_[t] == 0) ? 1.0f : score[t] / total;
    }

    int expand_local() {
        local_.clear();
        delta_.assign(4 * nR1_ + 3 * nR2_, 0);
        if (terminated_ || itr_ >= p_.numIterations) {
            terminated_ = true;
            return -1;
        }
        itr_++;
        cur_ = oracle_iter_log{itr_, treeSize_, 0, 0, 0, 0, 0, 0, -1};

        updateR1();   // KGMT.cu:125-136

        // KGMT.cu:139-147: frontier scan + findInd.
        std::vector<int> activeIdx;
        for (int i = 0; i < M_; ++i)
            if (G_[i]) activeIdx.push_back(i);
        const int nG = (int)activeIdx.size();
        cur_.nG = nG;

        // KGMT.cu:151-219 branch.  With samplesPerIteration > 0 the capped extension
        // (SURVEY.md §8d): remaining := min(cap, M - treeSize); |G| > remaining -> the
        // first `remaining` frontier nodes get one child each, the rest stay in G.
        int k = 0, nExp = 0;
        if (nG > 0) {   // D7: a zero-block launch is a no-op
            const long long cap = p_.samplesPerIteration;
            long long remaining = (long long)M_ - treeSize_;
            if (cap > 0) remaining = std::min(remaining, cap);
            if (cap > 0 && p_.batchRule == 1) {
                // D14 (build extension): fill the batch -- every frontier node gets
                // floor(remaining/|G|) children; more frontier than budget: one child
                // each for the first `remaining` nodes.
                if (nG <= remaining) {
                    k = (int)(remaining / nG);
                    nExp = nG;
                } else {
                    k = 1;
                    nExp = (int)remaining;
                }
            } else if (32ll * nG <= remaining) {
                k = 32;
                nExp = nG;
            } else {
                k = (int)((float)remaining / (float)nG);   // KGMT.cu:157
                nExp = nG;
                if (cap > 0 && k == 0) {
                    k = 1;
                    nExp = (int)std::max(0ll, remaining);
                }
            }
        }
        const int S = k * nExp;
        cur_.k = k;
        cur_.nExp = nExp;
        cur_.S = S;
        samplesGenerated_ += S;

        // propagateG / propagateGV2 (KGMT.cu:341-482): expanded frontier nodes leave G
        // (D5: only frontier positions < |G|; V2 clears them even when k = 0).
        for (int g = 0; g < nExp; ++g) G_[activeIdx[g]] = 0;

        // D2: the accept test reads R1Score / R2Avail as of the iteration start.
        std::vector<LocalOut> out(S);
        PropCfg pc{p_.numDisc, p_.agentLength, p_.width, p_.height, obstacles_.data(), nObs_,
                   nObs_ >= kSoAMinObs ? &soa_ : nullptr};
        const bool point = p_.agent == 1;
#pragma omp parallel for schedule(static) num_threads(threads())
        for (int s = 0; s < S; ++s) {
            if (!owns(s)) continue;
            const int g = s / k;                 // slot = g*k + i (propagateG: blockIdx*32 + lane)
            const int x0Idx = activeIdx[g];
            const float* x0 = &samples_[(size_t)x0Idx * SAMPLE_DIM];
            float* x1 = &unexplored_[(size_t)s * SAMPLE_DIM];
            uParent_[s] = x0Idx;
            oracle::XorwowState& rs = rng_[s];
            const bool valid = point ? propagate_point(x0, x1, rs, pc) : propagate_car(x0, x1, rs, pc);
            const int r1 = getR1(x1[0], x1[1], R1Size_, p_.N);
            const int r2 = getR2(x1[0], x1[1], r1, R1Size_, p_.N, R2Size_, p_.n);
            LocalOut o{r1, r2, (uint8_t)valid, 0};
            if (valid) {
                const float rnd = oracle::xorwow_uniform(rs);   // KGMT.cu:395
                // D3: a valid child outside the grid is rejected (reference reads index -1).
                if (r1 >= 0 && r2 >= 0 && (rnd <= R1Score_[r1] || R2Avail_[r2] == 0)) {
                    GNew_[s] = 1;   // stale flags are never cleared here (D6)
                    o.accept = 1;
                }
            }
            out[s] = o;
        }
        // Region counters (KGMT.cu:392-411), as deltas (D3: only in-grid cells).
        int* dR1 = &delta_[0];
        int* dR1Valid = &delta_[nR1_];
        int* dR1Invalid = &delta_[2 * nR1_];
        int* dR1AvailSet = &delta_[3 * nR1_];
        int* dR2AvailSet = &delta_[4 * nR1_];
        int* dR2Valid = &delta_[4 * nR1_ + nR2_];
        int* dR2Invalid = &delta_[4 * nR1_ + 2 * nR2_];
        for (int s = 0; s < S; ++s) {
            if (!owns(s)) continue;
            const LocalOut& o = out[s];
            if (o.r1 >= 0) dR1[o.r1] += 1;
            if (o.r2 >= 0) R2_[o.r2] += 1;   // R2 is written but never read or exported (D13)
            if (o.valid) {
                if (o.r1 >= 0) {
                    dR1AvailSet[o.r1] = 1;
                    dR1Valid[o.r1] += 1;
                }
                if (o.r2 >= 0) {
                    dR2AvailSet[o.r2] = 1;
                    dR2Valid[o.r2] += 1;
                }
            } else {
                if (o.r1 >= 0) dR1Invalid[o.r1] += 1;
                if (o.r2 >= 0) dR2Invalid[o.r2] += 1;
            }
        }
        // KGMT.cu:222-229: exclusive_scan(GNew) + findInd, restricted to owned slots.
        for (int s = 0; s < M_; ++s) {
            if (GNew_[s] && owns(s)) {
                oracle_record r;
                r.slot = s;
                memcpy(r.sample, &unexplored_[(size_t)s * SAMPLE_DIM], sizeof(r.sample));
                r.parent = uParent_[s];
                local_.push_back(r);
            }
        }
        return (int)local_.size();
    }

    // Apply summed deltas + gathered records: KGMT.cu:230-259 (updateG + termination).
    int finish(const oracle_record* recs, int count, const int32_t* sd) {
        if (terminated_) return -1;
        for (int t = 0; t < nR1_; ++t) {
            R1_[t] += sd[t];
            R1Valid_[t] += sd[nR1_ + t];
            R1Invalid_[t] += sd[2 * nR1_ + t];
            if (sd[3 * nR1_ + t] > 0) R1Avail_[t] = 1;
        }
        for (int c = 0; c < nR2_; ++c) {
            if (sd[4 * nR1_ + c] > 0) R2Avail_[c] = 1;
            R2Valid_[c] += sd[4 * nR1_ + nR2_ + c];
            R2Invalid_[c] += sd[4 * nR1_ + 2 * nR2_ + c];
        }
        std::vector<oracle_record> all(recs, recs + count);
        std::sort(all.begin(), all.end(),
                  [](const oracle_record& a, const oracle_record& b) { return a.slot < b.slot; });
        const int A = count;
        // updateG launch: min(|GNew|, floor(M/32)) blocks of 32 (KGMT.cu:231-232).
        const int grid = std::min(A, M_ / 32);
        const int cleared = 32 * grid;   // D6: GNew[0 .. 32*grid) cleared, the rest survives
        for (int s = 0; s < M_; ++s) {
            if (owns(s) && (p_.fixGNewClear || s < cleared)) GNew_[s] = 0;
        }
        int goalIdx = -1;
        const int nIns = std::min(A, cleared);
        for (int j = 0; j < nIns; ++j) {   // KGMT.cu:564-591
            const int dst = treeSize_ + j;
            if (dst >= M_) break;   // D13: the reference writes out of bounds here
            const oracle_record& r = all[j];
            parent_[dst] = r.parent;
            memcpy(&samples_[(size_t)dst * SAMPLE_DIM], r.sample, sizeof(r.sample));
            G_[dst] = 1;
            costs_[dst] = costs_[r.parent] + r.sample[SAMPLE_DIM - 1];   // getCost, KGMT.cu:631-633
            // inGoalRegion (KGMT.cu:635-638) in float: sqrt(dx*dx + dy*dy) < r.
            const float dx = r.sample[0] - goal_[0];
            const float dy = r.sample[1] - goal_[1];
            const float d2 = dx * dx + dy * dy;
            if (std::sqrt(d2) < p_.goalThreshold && goalIdx < 0) goalIdx = dst;   // D4: lowest index
        }
        treeSize_ += A;   // KGMT.cu:249
        cur_.A = A;
        cur_.treeSizeAfter = treeSize_;
        if (goalIdx >= 0) {
            goalIdx_ = goalIdx;
            costToGoal_ = costs_[goalIdx];
        }
        cur_.goalIdx = goalIdx_;
        logs_.push_back(cur_);
        if (costToGoal_ != 0.0f || goalIdx_ >= 0) terminated_ = true;   // KGMT.cu:251-254
        if (treeSize_ >= M_) terminated_ = true;                         // KGMT.cu:255-259
        if (itr_ >= p_.numIterations) terminated_ = true;
        return 1;
    }

    int step() {
        if (expand_local() < 0) return 0;
        finish(local_.data(), (int)local_.size(), delta_.data());
        return 1;
    }

    // --- accessors ---
    oracle_params p_;
    int M_, nR1_, nR2_, P_, rank_, nSlots_;
    float R1Size_, R2Size_;
    std::vector<float> samples_, unexplored_, costs_, R1Score_, obstacles_;
    std::vector<int> parent_, uParent_, R1_, R1Avail_, R1Valid_, R1Invalid_, R2_, R2Avail_, R2Valid_, R2Invalid_;
    std::vector<uint8_t> G_, GNew_;
    std::vector<oracle::XorwowState> rng_;
    std::vector<oracle_record> local_;
    std::vector<int32_t> delta_;
    std::vector<oracle_iter_log> logs_;
    oracle_iter_log cur_{};
    float goal_[SAMPLE_DIM];
    int nObs_ = 0;
    ObsSoA soa_;
    int itr_ = 0, treeSize_ = 0, goalIdx_ = -1;
    float costToGoal_ = 0.0f;
    bool terminated_ = false;
    long long samplesGenerated_ = 0;
};

}  // namespace

extern "C" {

void* oracle_create(const oracle_params* p) {
    if (!p || p->N * p->N != 256 || p->n <= 0 || p->maxTreeSize <= 0 || p->numDisc <= 0) return nullptr;
    if (p->batchRule == 1 && p->samplesPerIteration <= 0) return nullptr;
    if (p->nranks > 1 && (p->rank < 0 || p->rank >= p->nranks)) return nullptr;
    return new Oracle(*p);
}

void oracle_destroy(void* h) { delete static_cast<Oracle*>(h); }

int oracle_begin(void* h, const float initial[7], const float goal[7], const float* obstacles, int n,
                 uint64_t seed) {
    return static_cast<Oracle*>(h)->begin(initial, goal, obstacles, n, seed);
}

int oracle_step(void* h) { return static_cast<Oracle*>(h)->step(); }

int oracle_plan(void* h, const float initial[7], const float goal[7], const float* obstacles, int n,
                uint64_t seed) {
    Oracle* o = static_cast<Oracle*>(h);
    o->begin(initial, goal, obstacles, n, seed);
    int ran = 0;
    while (o->step()) ++ran;
    return ran;
}

int oracle_expand_local(void* h) { return static_cast<Oracle*>(h)->expand_local(); }

int oracle_local_records(void* h, oracle_record* out, int capacity) {
    Oracle* o = static_cast<Oracle*>(h);
    const int n = std::min(capacity, (int)o->local_.size());
    if (n > 0) memcpy(out, o->local_.data(), sizeof(oracle_record) * n);
    return n;
}

int oracle_delta_size(void* h) {
    Oracle* o = static_cast<Oracle*>(h);
    return 4 * o->nR1_ + 3 * o->nR2_;
}

int oracle_local_deltas(void* h, int32_t* out) {
    Oracle* o = static_cast<Oracle*>(h);
    memcpy(out, o->delta_.data(), sizeof(int32_t) * o->delta_.size());
    return (int)o->delta_.size();
}

int oracle_finish(void* h, const oracle_record* records, int count, const int32_t* summedDeltas) {
    return static_cast<Oracle*>(h)->finish(records, count, summedDeltas);
}

int oracle_info(void* h, int* itr, int* treeSize, int* goalIdx, float* costToGoal, int* terminated) {
    Oracle* o = static_cast<Oracle*>(h);
    *itr = o->itr_;
    *treeSize = o->treeSize_;
    *goalIdx = o->goalIdx_;
    *costToGoal = o->costToGoal_;
    *terminated = o->terminated_ ? 1 : 0;
    return 0;
}

int oracle_num_slots(void* h) { return static_cast<Oracle*>(h)->nSlots_; }

int oracle_tree(void* h, float* samples, int* parent, float* costs) {
    Oracle* o = static_cast<Oracle*>(h);
    memcpy(samples, o->samples_.data(), sizeof(float) * o->samples_.size());
    memcpy(parent, o->parent_.data(), sizeof(int) * o->parent_.size());
    memcpy(costs, o->costs_.data(), sizeof(float) * o->costs_.size());
    return 0;
}

int oracle_unexplored(void* h, float* samples, int* uParent) {
    Oracle* o = static_cast<Oracle*>(h);
    memcpy(samples, o->unexplored_.data(), sizeof(float) * o->unexplored_.size());
    memcpy(uParent, o->uParent_.data(), sizeof(int) * o->uParent_.size());
    return 0;
}

int oracle_flags(void* h, uint8_t* G, uint8_t* GNew) {
    Oracle* o = static_cast<Oracle*>(h);
    memcpy(G, o->G_.data(), o->G_.size());
    memcpy(GNew, o->GNew_.data(), o->GNew_.size());
    return 0;
}

int oracle_regions(void* h, int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score, int* R2Avail,
                   int* R2Valid, int* R2Invalid) {
    Oracle* o = static_cast<Oracle*>(h);
    memcpy(R1, o->R1_.data(), sizeof(int) * o->nR1_);
    memcpy(R1Avail, o->R1Avail_.data(), sizeof(int) * o->nR1_);
    memcpy(R1Valid, o->R1Valid_.data(), sizeof(int) * o->nR1_);
    memcpy(R1Invalid, o->R1Invalid_.data(), sizeof(int) * o->nR1_);
    memcpy(R1Score, o->R1Score_.data(), sizeof(float) * o->nR1_);
    memcpy(R2Avail, o->R2Avail_.data(), sizeof(int) * o->nR2_);
    memcpy(R2Valid, o->R2Valid_.data(), sizeof(int) * o->nR2_);
    memcpy(R2Invalid, o->R2Invalid_.data(), sizeof(int) * o->nR2_);
    return 0;
}

int oracle_rng(void* h, uint32_t* states) {
    Oracle* o = static_cast<Oracle*>(h);
    for (size_t s = 0; s < o->rng_.size(); ++s) {
        memcpy(&states[6 * s], o->rng_[s].v, 5 * sizeof(uint32_t));
        states[6 * s + 5] = o->rng_[s].d;
    }
    return (int)o->rng_.size();
}

int oracle_iter_logs(void* h, oracle_iter_log* out, int capacity) {
    Oracle* o = static_cast<Oracle*>(h);
    const int n = std::min(capacity, (int)o->logs_.size());
    if (n > 0) memcpy(out, o->logs_.data(), sizeof(oracle_iter_log) * n);
    return n;
}

long long oracle_samples_generated(void* h) { return static_cast<Oracle*>(h)->samplesGenerated_; }

void oracle_xorwow_init(uint64_t seed, uint64_t subsequence, int seeding, uint32_t state[6]) {
    oracle::XorwowState st = oracle::xorwow_seed(seed, seeding ? oracle::kRocrandSeeding : oracle::kCurandSeeding);
    int nbits = 1;
    while (nbits < 64 && (subsequence >> nbits)) ++nbits;
    oracle::XorwowSubsequenceJumps jumps(nbits);
    jumps.skip(st, subsequence);
    memcpy(state, st.v, 5 * sizeof(uint32_t));
    state[5] = st.d;
}

void oracle_xorwow_draw(uint32_t state[6], int count, uint32_t* out) {
    oracle::XorwowState st;
    memcpy(st.v, state, 5 * sizeof(uint32_t));
    st.d = state[5];
    for (int i = 0; i < count; ++i) out[i] = oracle::xorwow_next(st);
    memcpy(state, st.v, 5 * sizeof(uint32_t));
    state[5] = st.d;
}

// Replay (invariant I1; the reference's MATLAB replay, visualizationKGMT_Single.m:79-116):
// re-propagate parent state p[i][0..3] with the stored controls u[i] = (a, steering, duration)
// for numDisc steps; out[i] = (x, y, theta, v), valid[i] = motion validity.
void oracle_replay(const oracle_params* prm, const float* obstacles, int nObs, const float* parents,
                   const float* controls, int n, float* out, uint8_t* valid) {
    ObsSoA soa;
    soa.assign(obstacles, nObs);
    PropCfg pc{prm->numDisc, prm->agentLength, prm->width, prm->height, obstacles, nObs,
               nObs >= kSoAMinObs ? &soa : nullptr};
#pragma omp parallel for schedule(static) num_threads(prm->threads > 0 ? prm->threads : 1)
    for (int i = 0; i < n; ++i) {
        const float* p = &parents[4 * i];
        const float* u = &controls[3 * i];
        const float dt = u[2] / (float)pc.numDisc;
        float x = p[0], y = p[1], theta = p[2], v = p[3];
        bool ok = true;
        const float tan_steering = prm->agent == 1 ? 0.0f : sbmp::tanf_d(u[1]);
        for (int k = 0; k < pc.numDisc; ++k) {
            const float v_state[WS_DIM] = {x, y};
            if (prm->agent == 1) {
                x = fmaf(u[0], dt, x);
                y = fmaf(u[1], dt, y);
            } else {
                float st, ct;
                sbmp::sincosf_d(theta, &st, &ct);
                x = fmaf(v * ct, dt, x);
                y = fmaf(v * st, dt, y);
            }
            if (x <= 0.0f || x >= pc.width || y <= 0.0f || y >= pc.height) {
                ok = false;
                break;
            }
            if (prm->agent != 1) {
                theta = fmaf((v / pc.agentLength) * tan_steering, dt, theta);
                v = fmaf(u[0], dt, v);
            }
            const float w_state[WS_DIM] = {x, y};
            float bbMin[WS_DIM], bbMax[WS_DIM];
            segment_aabb(v_state, w_state, bbMin, bbMax);
            if (!motion_valid(bbMin, bbMax, pc)) {
                ok = false;
                break;
            }
        }
        out[4 * i] = x;
        out[4 * i + 1] = y;
        out[4 * i + 2] = prm->agent == 1 ? 0.0f : theta;
        out[4 * i + 3] = prm->agent == 1 ? 0.0f : v;
        valid[i] = ok ? 1 : 0;
    }
}

// Legacy random-tree generators (reference include/planners/Planner.cuh:6-12,
// not built by the reference's CMake).  kind 0: NaivePlanner.cu:25-74 (curand_init(outIndex, 0, 0)
// per sample); kind 1: CostPropPlanner.cu:25-81 (curand_init(gtid * rows, 0, 0) per thread).
// 20 Euler steps of the car with a in [-2.5, 2.5), steering in [-pi/2, pi/2), duration in [0, 0.3).
// D16: row r > 0 of a block grows from the block's first sample of row r - 1, the intent of
// both kernels (NaivePlanner.cu:71 reads it from `root`, out of bounds; CostPropPlanner.cu:78
// from the tree).  Contractions as D10/D11: x = fmaf(v*cos, dt, x); theta in double, as the
// reference's `length` is the double literal 1.0.
// out: rows x (blocks * tpb) samples of 7 floats, row-major (tree[row * tWidth + col]).
void oracle_random_tree(int kind, const float* root, int rows, int blocks, int tpb, float* out) {
    const int width = blocks * tpb;
    const size_t tWidth = (size_t)width * 7;
    std::vector<oracle::XorwowState> st(kind == 1 ? width : 0);
    for (int g = 0; g < (int)st.size(); ++g) st[g] = oracle::xorwow_seed((uint64_t)(long long)(g * rows));
    std::vector<float> x0((size_t)blocks * 4);
    for (int b = 0; b < blocks; ++b)
        for (int k = 0; k < 4; ++k) x0[(size_t)b * 4 + k] = root[k];
    for (int row = 0; row < rows; ++row) {
        for (int g = 0; g < width; ++g) {
            const size_t outIndex = (size_t)row * tWidth + (size_t)g * 7;
            oracle::XorwowState fresh = oracle::xorwow_seed((uint64_t)(long long)(int)outIndex);
            oracle::XorwowState& rs = kind == 1 ? st[g] : fresh;
            const float a = fmaf(oracle::xorwow_uniform(rs), 5.0f, -2.5f);
            const float steering = (float)std::fma((double)oracle::xorwow_uniform(rs), M_PI, -M_PI / 2);
            const float duration = oracle::xorwow_uniform(rs) * 0.3f;
            const float dt = duration / 20.0f;
            const float* p = &x0[(size_t)(g / tpb) * 4];
            float x = p[0], y = p[1], theta = p[2], v = p[3];
            const float tn = sbmp::tanf_d(steering);
            for (int i = 0; i < 20; ++i) {
                float sn, cs;
                sbmp::sincosf_d(theta, &sn, &cs);
                x = fmaf(v * cs, dt, x);
                y = fmaf(v * sn, dt, y);
                theta = (float)std::fma((double)v * (double)tn, (double)dt, (double)theta);
                v = fmaf(a, dt, v);
            }
            float* o = &out[outIndex];
            o[0] = x; o[1] = y; o[2] = theta; o[3] = v; o[4] = a; o[5] = steering; o[6] = duration;
        }
        for (int b = 0; b < blocks; ++b)
            for (int k = 0; k < 4; ++k) x0[(size_t)b * 4 + k] = out[(size_t)row * tWidth + (size_t)b * tpb * 7 + k];
    }
}

// One batch of propagateG's per-child work (KGMT.cu:386-411, statePropagator.cu:5-76):
// child i expands parents[7 i ..] with RNG state rng[6 i ..] (advanced in place), then
// getR1 / getR2 and, when scores are given, the accept test against R1Score /
// R2Avail (KGMT.cu:394-400; D3: a valid child outside the grid is rejected).  The
// checker of sbmp_expand_batch.
void oracle_expand_batch(const oracle_params* prm, const float* obstacles, int nObs, const float* parents,
                         uint32_t* rng, int n, const float* R1Score, const int* R2Avail, float* children,
                         uint8_t* valid, int* r1, int* r2, uint8_t* accept) {
    ObsSoA soa;
    soa.assign(obstacles, nObs);
    PropCfg pc{prm->numDisc, prm->agentLength, prm->width, prm->height, obstacles, nObs,
               nObs >= kSoAMinObs ? &soa : nullptr};
    const float R1Size = prm->width / (float)prm->N;
    const float R2Size = prm->width / (float)(prm->n * prm->N);
#pragma omp parallel for schedule(static) num_threads(prm->threads > 0 ? prm->threads : 1)
    for (int i = 0; i < n; ++i) {
        oracle::XorwowState rs;
        memcpy(rs.v, &rng[6 * (size_t)i], 5 * sizeof(uint32_t));
        rs.d = rng[6 * (size_t)i + 5];
        float* x1 = &children[(size_t)i * SAMPLE_DIM];
        const float* x0 = &parents[(size_t)i * SAMPLE_DIM];
        const bool ok = prm->agent == 1 ? propagate_point(x0, x1, rs, pc) : propagate_car(x0, x1, rs, pc);
        const int c1 = getR1(x1[0], x1[1], R1Size, prm->N);
        const int c2 = getR2(x1[0], x1[1], c1, R1Size, prm->N, R2Size, prm->n);
        uint8_t acc = 0;
        if (ok && R1Score) {
            const float u = oracle::xorwow_uniform(rs);   // KGMT.cu:395
            acc = (c1 >= 0 && c2 >= 0 && (u <= R1Score[c1] || R2Avail[c2] == 0)) ? 1 : 0;
        }
        valid[i] = ok ? 1 : 0;
        r1[i] = c1;
        r2[i] = c2;
        accept[i] = acc;
        memcpy(&rng[6 * (size_t)i], rs.v, 5 * sizeof(uint32_t));
        rng[6 * (size_t)i + 5] = rs.d;
    }
}

void oracle_sincosf(const float* x, int n, float* s, float* c) {
    for (int i = 0; i < n; ++i) sbmp::sincosf_d(x[i], &s[i], &c[i]);
}

void oracle_tanf(const float* x, int n, float* t) {
    for (int i = 0; i < n; ++i) t[i] = sbmp::tanf_d(x[i]);
}

}  // extern "C"
