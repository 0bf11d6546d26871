// grid.h — the two-level region grid and the cost / goal helpers of KGMT, for host
// and device code, with the reference's signatures:
//   __host__ __device__ int getR1(float x, float y, float R1Size, int N);           KGMT.cuh:207
//   __host__ __device__ int getR2(float x, float y, int r1, float R1Size, int N,
//                                 float R2Size, int n);                             KGMT.cuh:208
//   __device__ float getCost(float* x0, float* x1);                                 KGMT.cuh:209
//   __device__ bool inGoalRegion(float* x, float* goal, float r);                   KGMT.cuh:210
// (bodies KGMT.cu:602-638).  The planner's kernels use these for the root and the
// two-launch form; their hot loop uses forms with the divisions by R1Size / R2Size as
// a host-verified reciprocal multiply (kgmt_device.h getR1_k / getR2_k) that give the
// same cells.  Decisions: D3 -- a float -> int conversion out of int
// range or of NaN (undefined in C++) maps to -1; D10 -- x - c * R1Size is contracted
// to fmaf(-c, R1Size, x) as nvcc (-fmad=true) does.
#pragma once

#include "sbmp/sbmp_math.h"

namespace sbmp {

// static_cast<int>(q) where it is defined (truncation toward zero); *ok = false else.
SBMP_HD int cell_of(float q, bool* ok) {
    *ok = (q > -2147483648.0f && q < 2147483648.0f);
    return *ok ? (int)q : 0;
}

// reference KGMT.cu:602-609
SBMP_HD int getR1(float x, float y, float R1Size, int N) {
    bool okx, oky;
    const int cx = cell_of(x / R1Size, &okx);
    const int cy = cell_of(y / R1Size, &oky);
    return (okx && oky && cx >= 0 && cx < N && cy >= 0 && cy < N) ? cy * N + cx : -1;
}

// reference KGMT.cu:610-629
SBMP_HD int getR2(float x, float y, int r1, float R1Size, int N, float R2Size, int n) {
    if (r1 < 0) return -1;
    const int cyR1 = r1 / N;
    const int cxR1 = r1 % N;
    const float lx = __builtin_fmaf(-(float)cxR1, R1Size, x);   // nvcc's contraction of KGMT.cu:620 (D10)
    const float ly = __builtin_fmaf(-(float)cyR1, R1Size, y);
    bool okx, oky;
    const int cx = cell_of(lx / R2Size, &okx);
    const int cy = cell_of(ly / R2Size, &oky);
    return (okx && oky && cx >= 0 && cx < n && cy >= 0 && cy < n) ? r1 * (n * n) + cy * n + cx : -1;
}

// reference KGMT.cu:631-633: the cost of an edge is its duration, x1[6].
SBMP_HD float getCost(const float* x0, const float* x1) {
    (void)x0;
    return x1[6];
}

// reference KGMT.cu:635-638, in float: sqrt(dx^2 + dy^2) < r (pow(d, 2) is d * d).
SBMP_HD bool inGoalRegion(const float* x, const float* goal, float r) {
    const float dx = x[0] - goal[0], dy = x[1] - goal[1];
    return __builtin_sqrtf(dx * dx + dy * dy) < r;
}

}  // namespace sbmp
