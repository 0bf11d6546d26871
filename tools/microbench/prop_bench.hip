// Cost split of the Euler loop of k_expand (kgmt_device.h propagate_car) on
// synthetic inputs where every lane runs all steps: parents mid-workspace at v = 0,
// boxes in the corners (tested every step, never hit).  Variants switch parts of
// the step off so their cost can be read as differences.  Timing only; the
// production kernels are checked for parity by tests/test_gpu_parity.py.
//   hipcc -O3 -std=c++17 -ffp-contract=off -fno-slp-vectorize --offload-arch=gfx950 \
//     -Iinclude -Icudasbmp_amd/csrc tools/microbench/prop_bench.hip -o /tmp/prop_bench
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "kgmt_device.h"

using namespace sbmp;

// SC: 1 = sincos_pred, 0 = a cheap stand-in; NB: boxes tested; BND: bounds test on.
template <int SC, int NB, int BND>
__device__ __forceinline__ bool prop(float4 p, Xorwow& rs, const float4* obs, float W, float H, int D, float4& o) {
    const float a = __builtin_fmaf(xorwow_uniform(rs), 10.0f, -5.0f);
    const float u2 = xorwow_uniform(rs);
    const float steering = (float)__builtin_fma((double)(u2 * 2.0f), 3.141592653589793, -3.141592653589793);
    const float duration = __builtin_fmaf(xorwow_uniform(rs), 1.0f, 0.05f);
    const float dt = duration / (float)D;
    float x = p.x, y = p.y, theta = p.z, v = p.w;
    const float tan_steering = tanf_d(steering);
    bool alive = true;
    for (int i = 0; i < D; ++i) {
        float st, ct;
        if (SC) sincos_pred(theta, &st, &ct);
        else { st = theta * 0.5f; ct = 1.0f - theta; }
        const float nx = __builtin_fmaf(v * ct, dt, x);
        const float ny = __builtin_fmaf(v * st, dt, y);
        const bool oob = BND ? ((nx <= 0.0f) | (nx >= W) | (ny <= 0.0f) | (ny >= H)) : false;
        const float nth = __builtin_fmaf(v * tan_steering, dt, theta);
        const float nv = __builtin_fmaf(a, dt, v);
        const float minx = seg_min(x, nx), maxx = seg_max(x, nx);
        const float miny = seg_min(y, ny), maxy = seg_max(y, ny);
        bool hit = false;
#pragma unroll
        for (int k = 0; k < NB; ++k) hit |= box_overlap(minx, miny, maxx, maxy, obs[k]);
        const bool adv = alive & !oob;
        x = alive ? nx : x;
        y = alive ? ny : y;
        theta = adv ? nth : theta;
        v = adv ? nv : v;
        alive = adv & !hit;
        if (__ballot(alive) == 0ull) break;
    }
    o = make_float4(x, y, theta, v);
    return alive;
}

template <int SC, int NB, int BND>
__global__ __launch_bounds__(256) void k_prop(const float4* __restrict__ parents, uint4* rngA, uint2* rngB,
                                             float4* out, const float4* __restrict__ obsG, int D) {
    float4 ob[NB > 0 ? NB : 1];
#pragma unroll
    for (int k = 0; k < NB; ++k) ob[k] = obsG[k];
    const int s = blockIdx.x * 256 + threadIdx.x;
    const uint4 ra = rngA[s];
    const uint2 rb = rngB[s];
    Xorwow rs{ra.x, ra.y, ra.z, ra.w, rb.x, rb.y};
    float4 o;
    const bool valid = prop<SC, NB, BND>(parents[s >> 8], rs, ob, 20.0f, 20.0f, D, o);
    out[s] = o;
    rngA[s] = make_uint4(rs.v0, rs.v1, rs.v2, rs.v3);
    rngB[s] = make_uint2(rs.v4, rs.d | (valid ? 0u : 0u));
}

template <int SC, int NB, int BND>
static float run(const char* name, const float4* P, uint4* A, uint2* B, float4* O, const float4* ob, int n) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 5; ++w) hipLaunchKernelGGL((k_prop<SC, NB, BND>), dim3(n / 256), dim3(256), 0, 0, P, A, B, O, ob, 10);
    const int R = 50;
    hipEventRecord(e0);
    for (int r = 0; r < R; ++r) hipLaunchKernelGGL((k_prop<SC, NB, BND>), dim3(n / 256), dim3(256), 0, 0, P, A, B, O, ob, 10);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    printf("%-34s %8.2f us/launch\n", name, 1e3f * ms / R);
    return 1e3f * ms / R;
}

int main() {
    const int n = 262144;
    std::vector<float4> par(n / 256);
    unsigned seed = 12345;
    auto rnd = [&]() { seed = seed * 1664525u + 1013904223u; return (seed >> 8) * (1.0f / 16777216.0f); };
    for (auto& p : par) p = make_float4(8.0f + 4.0f * rnd(), 8.0f + 4.0f * rnd(), 6.2831853f * rnd() - 3.14159f, 0.0f);
    std::vector<uint4> ra(n);
    std::vector<uint2> rb(n);
    for (int i = 0; i < n; ++i) {
        ra[i] = make_uint4(seed = seed * 747796405u + 1u, seed = seed * 747796405u + 1u, seed * 3u + 7u, seed ^ 0x9e37u);
        rb[i] = make_uint2(seed * 5u + 11u, 6615241u + i);
    }
    std::vector<float4> obs = {{0.1f, 0.1f, 0.6f, 0.6f}, {19.4f, 0.1f, 19.9f, 0.6f}, {0.1f, 19.4f, 0.6f, 19.9f},
                               {19.4f, 19.4f, 19.9f, 19.9f}, {0.1f, 9.0f, 0.5f, 11.0f}, {19.5f, 9.0f, 19.9f, 11.0f},
                               {9.0f, 0.1f, 11.0f, 0.5f}, {9.0f, 19.5f, 11.0f, 19.9f}};
    float4 *P, *O, *ob;
    uint4* A;
    uint2* B;
    hipMalloc(&P, sizeof(float4) * par.size());
    hipMalloc(&O, sizeof(float4) * n);
    hipMalloc(&ob, sizeof(float4) * obs.size());
    hipMalloc(&A, sizeof(uint4) * n);
    hipMalloc(&B, sizeof(uint2) * n);
    hipMemcpy(P, par.data(), sizeof(float4) * par.size(), hipMemcpyHostToDevice);
    hipMemcpy(ob, obs.data(), sizeof(float4) * obs.size(), hipMemcpyHostToDevice);
    hipMemcpy(A, ra.data(), sizeof(uint4) * n, hipMemcpyHostToDevice);
    hipMemcpy(B, rb.data(), sizeof(uint2) * n, hipMemcpyHostToDevice);
    run<1, 5, 1>("full (sincos, 5 boxes, bounds)", P, A, B, O, ob, n);
    run<1, 0, 1>("no boxes", P, A, B, O, ob, n);
    run<1, 8, 1>("8 boxes", P, A, B, O, ob, n);
    run<0, 5, 1>("no sincos", P, A, B, O, ob, n);
    run<1, 5, 0>("no bounds", P, A, B, O, ob, n);
    run<0, 0, 0>("none (loop skeleton + RNG + I/O)", P, A, B, O, ob, n);
    return 0;
}
