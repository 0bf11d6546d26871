// random_tree.hip — the reference's legacy random-tree generators:
// NaivePlanner (src/planners/NaivePlanner.cu:25-140) and CostPropPlanner
// (src/planners/CostPropPlanner.cu:25-139) behind the Planner interface
// (include/planners/Planner.cuh:6-12).  The reference's CMake does not build them.
//
// One thread per column: rows x (blocks * threadsPerBlock) children of a shared
// per-block parent, 20 Euler steps of the car each, controls a in [-2.5, 2.5),
// steering in [-pi/2, pi/2), duration in [0, 0.3).  RNG: naive seeds a fresh
// XORWOW per sample with its output index (curand_init(outIndex, 0, 0)); costprop
// one per thread (curand_init(gtid * rows, 0, 0)).  D16: row r > 0 grows from the
// block's first sample of row r - 1 (both kernels' intent; the naive kernel reads it
// from `root` out of bounds, NaivePlanner.cu:68-72).  Arithmetic as
// oracle/kgmt_oracle.cpp oracle_random_tree (D9-D11), bit-exact against it.
#include <hip/hip_runtime.h>

#include "kgmt_device.h"
#include "kgmt_planner.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace sbmp {

__global__ void k_random_tree(int kind, float4 root, int rows, float* tree) {
    __shared__ float4 x0;
    const int gtid = (int)(blockIdx.x * blockDim.x + threadIdx.x);
    const size_t tWidth = (size_t)gridDim.x * blockDim.x * 7;
    if (threadIdx.x == 0) x0 = root;
    __syncthreads();
    Xorwow st = xorwow_seed((uint64_t)(long long)(gtid * rows));
    for (int row = 0; row < rows; ++row) {
        const size_t outIndex = (size_t)row * tWidth + (size_t)gtid * 7;
        Xorwow fresh = xorwow_seed((uint64_t)(long long)(int)outIndex);
        Xorwow& rs = kind == 1 ? st : fresh;
        const float a = __builtin_fmaf(xorwow_uniform(rs), 5.0f, -2.5f);
        const float steering = (float)__builtin_fma((double)xorwow_uniform(rs), 3.141592653589793,
                                                    -3.141592653589793 / 2);
        const float duration = xorwow_uniform(rs) * 0.3f;
        const float dt = duration / 20.0f;
        const float4 p = x0;
        float x = p.x, y = p.y, theta = p.z, v = p.w;
        const float tn = tanf_d(steering);
        for (int i = 0; i < 20; ++i) {
            float sn, cs;
            sincosf_d(theta, &sn, &cs);
            x = __builtin_fmaf(v * cs, dt, x);
            y = __builtin_fmaf(v * sn, dt, y);
            theta = (float)__builtin_fma((double)v * (double)tn, (double)dt, (double)theta);
            v = __builtin_fmaf(a, dt, v);
        }
        float* o = tree + outIndex;
        o[0] = x; o[1] = y; o[2] = theta; o[3] = v; o[4] = a; o[5] = steering; o[6] = duration;
        __syncthreads();   // every thread has read this row's parent
        if (threadIdx.x == 0) x0 = make_float4(x, y, theta, v);
        __syncthreads();
    }
}

void random_tree(int device, int kind, const float* root, int rows, int blocks, int tpb, float* samples,
                 float* kernelMs) {
    SBMP_HIP(hipSetDevice(device));
    const size_t n = (size_t)rows * blocks * tpb * 7;
    float* d = nullptr;
    hipEvent_t e0 = nullptr, e1 = nullptr;
    SBMP_HIP(hipMalloc(&d, sizeof(float) * n));
    try {
        SBMP_HIP(hipEventCreate(&e0));
        SBMP_HIP(hipEventCreate(&e1));
        SBMP_HIP(hipEventRecord(e0, nullptr));
        hipLaunchKernelGGL(k_random_tree, dim3(blocks), dim3(tpb), 0, nullptr, kind,
                           make_float4(root[0], root[1], root[2], root[3]), rows, d);
        SBMP_HIP(hipGetLastError());
        SBMP_HIP(hipEventRecord(e1, nullptr));
        SBMP_HIP(hipEventSynchronize(e1));
        float ms = 0.0f;
        SBMP_HIP(hipEventElapsedTime(&ms, e0, e1));
        if (kernelMs) *kernelMs = ms;
        SBMP_HIP(hipMemcpy(samples, d, sizeof(float) * n, hipMemcpyDeviceToHost));
    } catch (...) {
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        (void)hipFree(d);
        throw;
    }
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    (void)hipFree(d);
}

}  // namespace sbmp
