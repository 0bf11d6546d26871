// VALU issue rate on one SIMD: wave64 v_fma_f32 vs v_pk_fma_f32 (two floats per lane),
// at 1..8 waves per SIMD, 8 independent chains per wave.  Answers whether two children
// per lane in packed f32 raise the Euler loop's throughput.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/valu_bench.hip -o tools/microbench/valu_bench
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int PK>
__global__ __launch_bounds__(256) void k_valu(float* out, int iters) {
    float a[8];
    f2 p[8];
    for (int i = 0; i < 8; ++i) {
        a[i] = threadIdx.x * 1e-3f + i;
        p[i] = f2{a[i], a[i] + 0.5f};
    }
    const float b = 0.999f, c = 1e-4f;
    const f2 pb = {b, b}, pc = {c, c};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            if (PK) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(p[i]) : "v"(pb), "v"(pc));
            else asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c));
        }
    }
    float s = 0.f;
    for (int i = 0; i < 8; ++i) s += PK ? p[i].x + p[i].y : a[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    printf("start\n");
    float* out;
    hipMalloc(&out, 1024 * sizeof(float));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 32768;   // ~0.5 ms per launch at 1 wave per SIMD: launch overhead < 1%
    for (int variant = 0; variant < 2; ++variant) {
        for (int w = 1; w <= 8; w *= 2) {
            const dim3 grid(256 * w);   // 256-thread workgroups: one wave per SIMD per workgroup
            for (int rep = 0; rep < 3; ++rep) {
                hipEventRecord(e0);
                if (variant == 0) hipLaunchKernelGGL(k_valu<0>, grid, dim3(256), 0, 0, out, iters);
                else hipLaunchKernelGGL(k_valu<1>, grid, dim3(256), 0, 0, out, iters);
                hipEventRecord(e1);
                hipEventSynchronize(e1);
            }
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr = (double)iters * 8 * w;   // VALU instructions per SIMD
            const char* name = variant == 0 ? "v_fma_f32" : "v_pk_fma_f32";
            printf("%-22s waves/SIMD %d: %.3f ms, %.2f ns per VALU instr per SIMD (%.2f cycles @2.4GHz)\n", name, w, ms,
                   ms * 1e6 / instr, ms * 1e6 / instr * 2.4);
        }
    }
    return 0;
}
