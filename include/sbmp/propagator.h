// propagator.h — the car's state propagator for host and device code, with the
// reference's signature (include/statePropagator/statePropagator.cuh:5-14):
//   __device__ bool propagateAndCheck(float* x0, float* x1, int numDisc, float agentLength,
//                                     curandState* state, float* obstacles, int obstaclesCount,
//                                     float width, float height);
// Body: statePropagator.cu:5-76.  The RNG is the cuRAND-compatible Xorwow of
// xorwow.h in place of curandState.  It draws (a, steering, duration), runs numDisc
// explicit-Euler steps of the kinematic bicycle with a bounds check and a segment
// AABB collision check per step, writes x1 = [x, y, theta, v, a, steering, duration]
// and returns whether the motion is valid.  Float semantics as the planner's
// kernels and the CPU oracle: D9 -- sincosf_d / tanf_d (sbmp_math.h)
// for cosf / sinf / tanf; D10 -- a = fmaf(u, 10, -5), x = fmaf(v * cos, dt, x),
// y likewise, theta = fmaf((v / L) * tan, dt, theta), v = fmaf(a, dt, v); D11 --
// steering = (float)fma((double)(2u), pi, -pi).  tanf(steering) is loop-invariant
// and evaluated once (the same bits as per step).  The planner's kernels run the
// same sequence in exec-masked form with culled obstacle tests (kgmt_device.h
// propagate_car); a parity test checks this function against them
// (tests/test_gpu_batch.py).
#pragma once

#include "sbmp/collision.h"
#include "sbmp/sbmp_math.h"
#include "sbmp/xorwow.h"

namespace sbmp {

// reference statePropagator.cu:5-76
SBMP_HD bool propagateAndCheck(const float* x0, float* x1, int numDisc, float agentLength, Xorwow* state,
                               const float* obstacles, int obstaclesCount, float width, float height) {
    const float a = __builtin_fmaf(xorwow_uniform(*state), 10.0f, -5.0f);
    const float u2 = xorwow_uniform(*state);
    const float steering = (float)__builtin_fma((double)(u2 * 2.0f), 3.141592653589793, -3.141592653589793);
    const float duration = __builtin_fmaf(xorwow_uniform(*state), 1.0f, 0.05f);
    const float dt = duration / (float)numDisc;
    float x = x0[0], y = x0[1], theta = x0[2], v = x0[3];
    const float tan_steering = tanf_d(steering);
    bool motionValid = true;
    for (int i = 0; i < numDisc; ++i) {
        const float vs[kWorkspaceDim] = {x, y};
        float sin_theta, cos_theta;
        sincosf_d(theta, &sin_theta, &cos_theta);
        x = __builtin_fmaf(v * cos_theta, dt, x);
        y = __builtin_fmaf(v * sin_theta, dt, y);
        if (x <= 0.0f || x >= width || y <= 0.0f || y >= height) {
            motionValid = false;
            break;
        }
        theta = __builtin_fmaf((v / agentLength) * tan_steering, dt, theta);
        v = __builtin_fmaf(a, dt, v);
        const float ws[kWorkspaceDim] = {x, y};
        float bbMin[kWorkspaceDim], bbMax[kWorkspaceDim];
        for (int d = 0; d < kWorkspaceDim; ++d) {   // statePropagator.cu:52-60
            bbMin[d] = vs[d] > ws[d] ? ws[d] : vs[d];
            bbMax[d] = vs[d] > ws[d] ? vs[d] : ws[d];
        }
        motionValid = motionValid && isMotionValid(vs, ws, bbMin, bbMax, obstacles, obstaclesCount);
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

// Build extension, no reference counterpart: a
// holonomic R2 point in the same skeleton.  Controls (vx, vy) in (-1, 1]^2, the
// duration as the car's; x += vx dt, y += vy dt with the same per-step bounds and
// collision checks; x1 = [x, y, 0, 0, vx, vy, duration].
SBMP_HD bool propagatePoint(const float* x0, float* x1, int numDisc, Xorwow* state, const float* obstacles,
                            int obstaclesCount, float width, float height) {
    const float vx = __builtin_fmaf(xorwow_uniform(*state), 2.0f, -1.0f);
    const float vy = __builtin_fmaf(xorwow_uniform(*state), 2.0f, -1.0f);
    const float duration = __builtin_fmaf(xorwow_uniform(*state), 1.0f, 0.05f);
    const float dt = duration / (float)numDisc;
    float x = x0[0], y = x0[1];
    bool motionValid = true;
    for (int i = 0; i < numDisc; ++i) {
        const float vs[kWorkspaceDim] = {x, y};
        x = __builtin_fmaf(vx, dt, x);
        y = __builtin_fmaf(vy, dt, y);
        if (x <= 0.0f || x >= width || y <= 0.0f || y >= height) {
            motionValid = false;
            break;
        }
        const float ws[kWorkspaceDim] = {x, y};
        float bbMin[kWorkspaceDim], bbMax[kWorkspaceDim];
        for (int d = 0; d < kWorkspaceDim; ++d) {
            bbMin[d] = vs[d] > ws[d] ? ws[d] : vs[d];
            bbMax[d] = vs[d] > ws[d] ? vs[d] : ws[d];
        }
        motionValid = motionValid && isMotionValid(vs, ws, bbMin, bbMax, obstacles, obstaclesCount);
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

}  // namespace sbmp
