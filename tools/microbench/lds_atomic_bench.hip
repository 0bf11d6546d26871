// LDS add rate per CU (ds_add_u32, no return) for the address patterns a histogram meets,
// beside ds_write_b32 on the same addresses.  One 1024-thread workgroup per CU (256
// workgroups, 16 waves per CU), 16,384-word table: the k_fold_r2 shape.
// Patterns (per wave-instruction, lane L):
//   distinct  consecutive words (L + 64 j): no bank conflict
//   random    a hash of (L, j, wave) over the table
//   bank      words L * 32: every lane of a 32-lane group on one bank, distinct words
//   same8     8 lanes per word (L / 8 + 64 j)
//   same64    one word for the whole wave
//   hot16     random over 16 words (a few hot cells)
//   hdist     a hash over the table, each lane's 8 adds in one u32 key chunk of 8 keys
//   hipcc -O3 --offload-arch=gfx950 tools/microbench/lds_atomic_bench.hip -o tools/microbench/lds_atomic_bench
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kWords = 16384;
constexpr int kAddrs = 16;   // addresses per lane, cycled

__device__ __forceinline__ unsigned hash32(unsigned x) {
    x ^= x >> 16;
    x *= 0x7feb352du;
    x ^= x >> 15;
    x *= 0x846ca68bu;
    x ^= x >> 16;
    return x;
}

template <int PAT>
__device__ __forceinline__ unsigned pattern(int lane, int j, int wave) {
    switch (PAT) {
        case 0: return (unsigned)(lane + 64 * (j + kAddrs * wave)) % kWords;
        case 1: return hash32((unsigned)(lane * 7919 + j * 104729 + wave * 1299709)) % kWords;
        case 2: return (unsigned)((lane & 31) * 32 + (lane >> 5) + j * 2 + wave * 64) % kWords;
        case 3: return (unsigned)(lane / 8 + 64 * (j + kAddrs * wave)) % kWords;
        case 4: return (unsigned)(j + kAddrs * wave) % kWords;
        default: return hash32((unsigned)(lane * 7919 + j * 104729 + wave * 1299709)) % 16u;
    }
}

template <int PAT, bool WRITE>
__global__ __launch_bounds__(1024) void k_lds(unsigned* out, int iters) {
    __shared__ unsigned s[kWords];
    for (int i = threadIdx.x; i < kWords; i += 1024) s[i] = 0u;
    __syncthreads();
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    unsigned a[kAddrs];
#pragma unroll
    for (int j = 0; j < kAddrs; ++j) a[j] = pattern<PAT>(lane, j, wave) * 4u;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int j = 0; j < kAddrs; ++j) {
            if (WRITE) asm volatile("ds_write_b32 %0, %1" : : "v"(a[j]), "v"(it) : "memory");
            else asm volatile("ds_add_u32 %0, %1" : : "v"(a[j]), "v"(1u) : "memory");
        }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __syncthreads();
    unsigned v = 0;
    for (int i = threadIdx.x; i < kWords; i += 1024) v += s[i];
    if (v == 0xdeadbeefu) out[blockIdx.x] = v;
}

template <int PAT, bool WRITE>
static void run(const char* name, unsigned* out) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    const int iters = 256;
    float ms = 0.f;
    for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        hipLaunchKernelGGL((k_lds<PAT, WRITE>), dim3(256), dim3(1024), 0, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        (void)hipEventElapsedTime(&ms, e0, e1);
    }
    const double perCu = (double)iters * kAddrs * 16;   // wave-instructions per CU
    printf("%-14s %-9s %.3f ms  %.2f ns per wave-instruction per CU  (%.1f lane-ops per ns per CU)\n",
           WRITE ? "ds_write_b32" : "ds_add_u32", name, ms, ms * 1e6 / perCu, perCu * 64 / (ms * 1e6));
}

int main() {
    setvbuf(stdout, nullptr, _IONBF, 0);
    unsigned* out;
    if (hipMalloc(&out, 1024 * sizeof(unsigned)) != hipSuccess) return 1;
    run<0, false>("distinct", out);
    run<1, false>("random", out);
    run<2, false>("bank", out);
    run<3, false>("same8", out);
    run<4, false>("same64", out);
    run<5, false>("hot16", out);
    run<0, true>("distinct", out);
    run<1, true>("random", out);
    run<2, true>("bank", out);
    run<4, true>("same64", out);
    (void)hipFree(out);
    return 0;
}
