// SALU issue rate per CU: 8 independent s_add_u32 chains per wave (each asm declares its SCC write,
// alone, so the loop's own compare survives the asm), at 1..4 waves per SIMD (4..16 per
// CU); and SALU + VALU interleaved (one s_add_u32 per v_fma_f32) to see whether the
// scalar unit issues beside the vector units.  Answers how much of k_step's ~875 SALU per
// wave (16 waves per CU) is a serial cost of its own.
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/salu_bench.hip -o tools/microbench/salu_bench
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MIX>
__global__ __launch_bounds__(256) void k_salu(float* out, int iters, int seed) {
    int s0 = seed, s1 = seed + 1, s2 = seed + 2, s3 = seed + 3, s4 = seed + 4, s5 = seed + 5, s6 = seed + 6,
        s7 = seed + 7;
    float a[8];
    for (int i = 0; i < 8; ++i) a[i] = threadIdx.x * 1e-3f + i;
    const float b = 0.999f, c = 1e-4f;
    for (int it = 0; it < iters; ++it) {
#define SM(x) asm volatile("s_add_u32 %0, %0, 3" : "+s"(x) : : "scc")
#define VF(i) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(a[i]) : "v"(b), "v"(c))
        SM(s0); if (MIX) VF(0);
        SM(s1); if (MIX) VF(1);
        SM(s2); if (MIX) VF(2);
        SM(s3); if (MIX) VF(3);
        SM(s4); if (MIX) VF(4);
        SM(s5); if (MIX) VF(5);
        SM(s6); if (MIX) VF(6);
        SM(s7); if (MIX) VF(7);
#undef SM
#undef VF
    }
    float s = (float)(s0 ^ s1 ^ s2 ^ s3 ^ s4 ^ s5 ^ s6 ^ s7);
    for (int i = 0; i < 8; ++i) s += a[i];
    if (s == 12345.f) out[threadIdx.x] = s;
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    float* out;
    if (hipMalloc(&out, 1024 * sizeof(float)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 16384;
    for (int mix = 0; mix < 2; ++mix) {
        for (int w = 1; w <= 4; w *= 2) {
            const dim3 grid(256 * w);   // 256-thread workgroups: w waves per SIMD, 4w per CU
            float ms = 0.f;
            for (int rep = 0; rep < 3; ++rep) {
                (void)hipEventRecord(e0);
                if (mix) hipLaunchKernelGGL(k_salu<1>, grid, dim3(256), 0, 0, out, iters, rep);
                else hipLaunchKernelGGL(k_salu<0>, grid, dim3(256), 0, 0, out, iters, rep);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            const double perCu = (double)iters * 8 * 4 * w;   // SALU instructions per CU
            printf("%-26s waves/CU %2d: %.3f ms, %.3f ns per SALU instr per CU%s\n",
                   mix ? "s_add_u32 + v_fma_f32" : "s_add_u32", 4 * w, ms, ms * 1e6 / perCu,
                   mix ? " (one v_fma_f32 per SALU instr)" : "");
        }
    }
    return 0;
}
