// Exhaustive check of k_step's odd-quadrant tangent reciprocal (kgmt_device.h tan_steer):
// for every float x in [-pi, pi] (a superset of the steering angles (float)fma(2u, pi, -pi)
// that statePropagator.cu:18 can produce), the Cody-Waite reduction and tan_poly of
// tan_steer give t; where the quadrant is odd, -1/t is formed two ways:
//   IEEE    -1.0f / t                      (correctly rounded division: what tanf_d and the
//                                            oracle compute)
//   Newton  -fma(fma(-t, y, 1), y, y), y = v_rcp_f32(t)
// and every mismatch is counted, with the range of |t| seen.  Zero mismatches is what lets
// tan_steer use the second form (3 VALU instead of ~11) with the same bits.
//   hipcc -O3 --offload-arch=gfx950 -I include tools/microbench/tan_rcp_check.hip -o /tmp/tan_rcp_check
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "sbmp/sbmp_math.h"

__device__ __forceinline__ float neg_rcp_newton(float t) {
    const float y = __builtin_amdgcn_rcpf(t);
    const float e = __builtin_fmaf(-t, y, 1.0f);
    return -__builtin_fmaf(e, y, y);
}

__global__ void k_check(uint32_t lo, uint32_t n, unsigned long long* out) {
    // out: [mismatches, odd-quadrant arguments, min |t| bits, max |t| bits, first mismatch x bits]
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint32_t bitsx = lo + i;
    const float x = sbmp::u2f(bitsx);
    if (!(__builtin_fabsf(x) <= 3.14159274f)) return;   // float(pi) rounds up: keep it in
    const float j = __builtin_rintf(x * 0.636619772f);
    float r = __builtin_fmaf(j, -1.57079601e+00f, x);
    r = __builtin_fmaf(j, -3.13916473e-07f, r);
    r = __builtin_fmaf(j, -5.39030253e-15f, r);
    if (!((int)j & 1)) return;
    const float t = sbmp::tan_poly(r);
    const float a = -1.0f / t, b = neg_rcp_newton(t);
    atomicAdd(&out[1], 1ull);
    const unsigned long long at = sbmp::f2u(__builtin_fabsf(t));
    atomicMin(&out[2], at);
    atomicMax(&out[3], at);
    if (sbmp::f2u(a) != sbmp::f2u(b)) {
        if (atomicAdd(&out[0], 1ull) == 0ull) out[4] = bitsx;
    }
}

int main() {
    unsigned long long* d = nullptr;
    (void)hipMalloc(&d, 5 * sizeof(unsigned long long));
    const unsigned long long init[5] = {0, 0, ~0ull, 0, 0};
    (void)hipMemcpy(d, init, sizeof(init), hipMemcpyHostToDevice);
    // every float with |x| <= pi: bit patterns [0, f2u(pi)] and their negatives
    const uint32_t piBits = sbmp::f2u(3.14159274f);
    for (int sign = 0; sign < 2; ++sign) {
        const uint32_t lo = sign ? 0x80000000u : 0u, n = piBits + 1;
        const uint32_t blocks = (n + 255) / 256;
        hipLaunchKernelGGL(k_check, dim3(blocks), dim3(256), 0, 0, lo, n, d);
    }
    unsigned long long h[5];
    (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    printf("odd-quadrant arguments %llu, mismatches %llu, |t| in [%.9g, %.9g]%s\n", h[1], h[0],
           sbmp::u2f((uint32_t)h[2]), sbmp::u2f((uint32_t)h[3]), h[0] ? "" : " -- the Newton form is exact here");
    if (h[0]) printf("first mismatch at x bits 0x%08llx\n", h[4]);
    return h[0] ? 1 : 0;
}
