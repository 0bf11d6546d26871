// collision.h — the reference's AABB broad phase for host and device code, with
// its signatures (reference include/collisionCheck/collisionCheck.cuh:4-8):
//   __device__ bool isBroadPhaseValid(float* bbMin, float* bbMax, float* obs);
//   __device__ bool isMotionValid(float* x0, float* x1, float* bbMin, float* bbMax,
//                                 float* obstacles, int obstaclesCount);
// Bodies: collisionCheck.cu:6-28.  A box is [xmin, ymin, xmax, ymax]; a segment's
// bounding box is free of it iff they are separated on some axis (touching edges
// count as free).  isMotionValid keeps the reference's early exit; x0 / x1 (the
// segment ends) are passed through unused, as in the reference.  The planner's
// kernels test the same predicate in specialised forms (obstacles in registers,
// LDS, or the uniform-grid index; kgmt_device.h box_overlap / motion_valid).
#pragma once

#include "sbmp/sbmp_math.h"

namespace sbmp {

constexpr int kWorkspaceDim = 2;   // collisionCheck.cu:3 DIM_WORKSPACE

// reference collisionCheck.cu:6-14
SBMP_HD bool isBroadPhaseValid(const float* bbMin, const float* bbMax, const float* obs) {
    for (int d = 0; d < kWorkspaceDim; ++d)
        if (bbMax[d] <= obs[d] || obs[kWorkspaceDim + d] <= bbMin[d]) return true;
    return false;
}

// reference collisionCheck.cu:16-28
SBMP_HD bool isMotionValid(const float* x0, const float* x1, const float* bbMin, const float* bbMax,
                           const float* obstacles, int obstaclesCount) {
    (void)x0;
    (void)x1;
    for (int i = 0; i < obstaclesCount; ++i)
        if (!isBroadPhaseValid(bbMin, bbMax, obstacles + i * 2 * kWorkspaceDim)) return false;
    return true;
}

}  // namespace sbmp
