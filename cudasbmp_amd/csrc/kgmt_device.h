// kgmt_device.h — data layout and device functions of the MI355X KGMT hot path.
//
// HBM layout:
//   tree rows      treeState  float4[M]  (x, y, theta, v)
//                  treeCtrl   float4[M]  (a, steering, duration, cost)
//                  treeParent int[M]
//   child slots    uState     float4[slots] (x, y, theta, v) of the child in that slot
//                  uCtrl      float4[slots] (a, steering, duration, parent-row bits)
//                  rngA/rngB  uint4/uint2[slots]: XORWOW {v0..v3}, {v4, d}
//                  gnew       u64[slots/64]: accept flags (GNew), one bit per slot
// Every per-slot access is a 16-B (or 8-B) coalesced load/store; the region
// tables (~200 KB) and the obstacle list stay L2-resident.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sbmp/sbmp_math.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace sbmp {

constexpr int kBlock = 256;          // threads per expand block = slots per ownership block
constexpr int kWave = 64;
constexpr int kNoGoal = 0x7fffffff;
constexpr int kN = 16;               // R1 grid side: N must be 16 (reference KGMT.cu:8,501,520)
constexpr int kMaxR1 = kN * kN;
constexpr int kMaxR2Words = 2048;    // n <= 16: 256*16*16 cells / 32

// Per-iteration control block, written once by the plan kernel of that iteration.
struct IterCtrl {
    int run;        // iteration t is scheduled (the expand kernel also checks the goal status)
    int executed;   // expand t really ran (written by the next plan kernel)
    int treeSize;   // rows at the start of iteration t
    int gLo;        // frontier = rows [gLo, treeSize)  (G is always a contiguous range)
    int nG, k, nExp, S;
    int H;          // slot high-water mark including this iteration (stale GNew bits live below it)
    int A;          // accepted children (GNew popcount) at the end of iteration t
    int scoreBuf;   // R1Score buffer used by iteration t
    int pad[5];
};
static_assert(sizeof(IterCtrl) == 64, "IterCtrl is one 64-B line");

struct PlannerStatus {
    int goalIdx;    // lowest tree row inside the goal radius (kNoGoal if none), D4
    int pad[15];
};

constexpr int kMaxLdsObs = 2048;     // obstacle lists up to 32 KB are staged in LDS per block

// Everything a kernel needs, passed by value.
struct KgmtDev {
    int M, nSlots, nWords, nBlocks, numIterations, numDisc, N, n, nR1, nR2, nObs, cap, fixGNewClear;
    int batchRule;        // 0 = reference rule (+ cap), 1 = fill the cap (D14)
    int nranks, rank;
    float width, height, agentLength, invAgentLength, goalThreshold, R1Size, R2Size, goalX, goalY;
    float4* treeState;
    float4* treeCtrl;
    int* treeParent;
    float4* uState;
    float4* uCtrl;
    uint4* rngA;
    uint2* rngB;
    unsigned long long* gnew;
    int* blockCount;      // GNew popcount per 256-slot block (written by k_expand)
    int* blockOffsets;    // exclusive prefix of blockCount (written by k_plan)
    int* R1;
    int* R1Avail;
    int* R1Valid;
    int* R1Invalid;
    int* R1Cov;           // available R2 cells per R1 cell (covR numerator, kept incrementally)
    uint32_t* R2Avail;    // live availability bits
    uint32_t* R2Snap;     // availability bits at the iteration start (D2)
    uint32_t* R2New;      // cells seen valid this iteration while unavailable in the snapshot
    int* R2Valid;
    int* R2Invalid;
    float* R1Score;       // [2][nR1]
    unsigned long long* delta;   // [nR1]: this iteration's valid (bits 0-31) / invalid (32-63) children per R1 cell
    const float4* obstacles;
    IterCtrl* ctrl;
    PlannerStatus* status;
};

// ---------------------------------------------------------------- grid binning
// reference KGMT.cu:602-609 / 610-629.  Float->int truncates toward zero; an
// out-of-int-range or NaN quotient maps to -1 (D3).
SBMP_HD int cell_of(float q, bool* ok) {
    *ok = (q > -2147483648.0f && q < 2147483648.0f);
    return *ok ? (int)q : 0;
}

SBMP_HD int getR1(float x, float y, float R1Size, int N) {
    bool okx, oky;
    const int cx = cell_of(x / R1Size, &okx);
    const int cy = cell_of(y / R1Size, &oky);
    return (okx && oky && cx >= 0 && cx < N && cy >= 0 && cy < N) ? cy * N + cx : -1;
}

SBMP_HD int getR2(float x, float y, int r1, float R1Size, int N, float R2Size, int n) {
    if (r1 < 0) return -1;
    const int cyR1 = r1 / N;
    const int cxR1 = r1 % N;
    const float lx = x - (float)cxR1 * R1Size;
    const float ly = y - (float)cyR1 * R1Size;
    bool okx, oky;
    const int cx = cell_of(lx / R2Size, &okx);
    const int cy = cell_of(ly / R2Size, &oky);
    return (okx && oky && cx >= 0 && cx < n && cy >= 0 && cy < n) ? r1 * (n * n) + cy * n + cx : -1;
}

// ---------------------------------------------------------------- cuRAND XORWOW
struct Xorwow {
    uint32_t v0, v1, v2, v3, v4, d;
};

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

// curand_uniform: x * 2^-32 + 2^-33 (product exact, one rounding).
SBMP_HD float xorwow_uniform(Xorwow& s) {
    return (float)xorwow_next(s) * 2.3283064365386963e-10f + 1.1641532182693481e-10f;
}

// ---------------------------------------------------------------- collision
// reference collisionCheck.cu:6-28: a segment AABB is free of an obstacle box
// iff separated on some axis; the motion is valid iff free of every box.
// OBS > 0: the list is staged in LDS and every box is tested without early
// exit (independent broadcast reads, no load->compare->branch chain; the result
// is an order-independent OR, so identical to the reference's early return).
// Otherwise the list is read from global memory with the reference's early exit.
__device__ __forceinline__ int box_overlap(float minx, float miny, float maxx, float maxy, float4 o) {
    // (xmin, ymin, xmax, ymax).  !(a <= b), not (a > b): identical to the reference's
    // predicate for NaN too.  Bitwise, not short-circuit: one 16-B read, four compares.
    return (int)!(maxx <= o.x) & (int)!(o.z <= minx) & (int)!(maxy <= o.y) & (int)!(o.w <= miny);
}

// OBS: 0 = global list, reference early exit; 1 = LDS list, rolled loop;
//      2 = LDS list, 4-way unrolled (reads batched, more VGPRs).
template <int OBS>
__device__ __forceinline__ bool motion_valid(float minx, float miny, float maxx, float maxy,
                                             const float4* __restrict__ obs, int nObs) {
    if (OBS == 1) {
        int hit = 0;
#pragma unroll 1
        for (int i = 0; i < nObs; ++i) hit |= box_overlap(minx, miny, maxx, maxy, obs[i]);
        return hit == 0;
    }
    if (OBS == 2) {
        int hit = 0;
        int i = 0;
        for (; i + 4 <= nObs; i += 4) {
            const float4 a = obs[i], b = obs[i + 1], c = obs[i + 2], e = obs[i + 3];
            hit |= box_overlap(minx, miny, maxx, maxy, a) | box_overlap(minx, miny, maxx, maxy, b) |
                   box_overlap(minx, miny, maxx, maxy, c) | box_overlap(minx, miny, maxx, maxy, e);
        }
#pragma unroll 1
        for (; i < nObs; ++i) hit |= box_overlap(minx, miny, maxx, maxy, obs[i]);
        return hit == 0;
    }
    for (int i = 0; i < nObs; ++i) {
        const float4 o = obs[i];
        const bool free_ = (maxx <= o.x) || (o.z <= minx) || (maxy <= o.y) || (o.w <= miny);
        if (!free_) return false;
    }
    return true;
}

struct ChildOut {
    float4 state;   // x, y, theta, v
    float a, steer, dur;
};

// reference statePropagator.cu:5-76 (car).  Same operation sequence as the oracle
// (D9-D11): fmaf where nvcc would contract, steering via one double fma.
// v / agentLength: when agentLength is a power of two, v * (1/agentLength) is the
// same correctly rounded value (both are the exact product scaled by 2^-k), so the
// host passes invAgentLength != 0 and the per-step division disappears.
template <int OBS>
__device__ __forceinline__ bool propagate_car(float4 p, Xorwow& rs, const KgmtDev& d, const float4* obs,
                                              ChildOut& out) {
    const float a = __builtin_fmaf(xorwow_uniform(rs), 10.0f, -5.0f);
    const float u2 = xorwow_uniform(rs);
    const float steering = (float)__builtin_fma((double)(u2 * 2.0f), 3.141592653589793, -3.141592653589793);
    const float duration = __builtin_fmaf(xorwow_uniform(rs), 1.0f, 0.05f);
    const float dt = duration / (float)d.numDisc;
    float x = p.x, y = p.y, theta = p.z, v = p.w;
    const float tan_steering = tanf_d(steering);
    bool valid = true;
    for (int i = 0; i < d.numDisc; ++i) {
        const float px = x, py = y;
        float st, ct;
        sincosf_d(theta, &st, &ct);
        x = __builtin_fmaf(v * ct, dt, x);
        y = __builtin_fmaf(v * st, dt, y);
        if (x <= 0.0f || x >= d.width || y <= 0.0f || y >= d.height) {
            valid = false;
            break;
        }
        const float vl = (d.invAgentLength != 0.0f) ? v * d.invAgentLength : v / d.agentLength;
        theta = __builtin_fmaf(vl * tan_steering, dt, theta);
        v = __builtin_fmaf(a, dt, v);
        const float minx = (px > x) ? x : px, maxx = (px > x) ? px : x;
        const float miny = (py > y) ? y : py, maxy = (py > y) ? py : y;
        if (!motion_valid<OBS>(minx, miny, maxx, maxy, obs, d.nObs)) {
            valid = false;
            break;
        }
    }
    out.state = make_float4(x, y, theta, v);
    out.a = a;
    out.steer = steering;
    out.dur = duration;
    return valid;
}

// Holonomic R2 point (build extension).
template <int OBS>
__device__ __forceinline__ bool propagate_point(float4 p, Xorwow& rs, const KgmtDev& d, const float4* obs,
                                                ChildOut& out) {
    const float vx = __builtin_fmaf(xorwow_uniform(rs), 2.0f, -1.0f);
    const float vy = __builtin_fmaf(xorwow_uniform(rs), 2.0f, -1.0f);
    const float duration = __builtin_fmaf(xorwow_uniform(rs), 1.0f, 0.05f);
    const float dt = duration / (float)d.numDisc;
    float x = p.x, y = p.y;
    bool valid = true;
    for (int i = 0; i < d.numDisc; ++i) {
        const float px = x, py = y;
        x = __builtin_fmaf(vx, dt, x);
        y = __builtin_fmaf(vy, dt, y);
        if (x <= 0.0f || x >= d.width || y <= 0.0f || y >= d.height) {
            valid = false;
            break;
        }
        const float minx = (px > x) ? x : px, maxx = (px > x) ? px : x;
        const float miny = (py > y) ? y : py, maxy = (py > y) ? py : y;
        if (!motion_valid<OBS>(minx, miny, maxx, maxy, obs, d.nObs)) {
            valid = false;
            break;
        }
    }
    out.state = make_float4(x, y, 0.0f, 0.0f);
    out.a = vx;
    out.steer = vy;
    out.dur = duration;
    return valid;
}

}  // namespace sbmp
