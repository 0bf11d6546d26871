// Overlapped consecutive launches vs a kernel boundary, on a synthetic
// k_step-shaped grid: 1,025 workgroups of 256 threads, 5 waves per SIMD, a VALU body of
// about the k_step's length.  Forms:
//   serial      one stream, one dependent launch after another (a kernel boundary each)
//   ovl-top     two streams alternating, launch t waits in-kernel for launch t-1: every
//               workgroup adds to its shard (blockIdx % 8), the shard's last arrival adds
//               to a top counter that one lane of every workgroup polls (k_step's form)
//   ovl-shards  the same, but the pollers read the 8 shard counters (one lane each) and
//               sum them: one atomic fewer on the hand-off chain
// Each form with and without a memory phase (64 B written through and 64 B read per
// thread, sc1), since kernel-start/end cache maintenance of a launch can land in the
// middle of the other one.
//
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/overlap_bench.hip -o tools/microbench/overlap_bench
//   tools/microbench/overlap_bench [iters]
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                   \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                \
            exit(1);                                                               \
        }                                                                          \
    } while (0)


constexpr int kBlock = 256, kStride = 32;
constexpr int kOvl = 1, kShards = 2, kMem = 4;

struct Args {
    unsigned* cnt;   // [9][kStride]: 8 shards, top
    float4* a;
    float4* b;
    int* err;
    int iters, mode, groups;
};

__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) void k_body(Args a, int t) {
    const bool ovl = a.mode & kOvl;
    if (ovl && t > 1) {
        if (a.mode & kShards) {
            if (threadIdx.x < 8) {   // lanes 0-7 of wave 0: one shard each, summed with a ballot loop
                const unsigned per = (unsigned)((a.groups - (int)threadIdx.x + 7) >> 3);
                const unsigned want = (unsigned)(t - 1) * per;
                const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
                while (true) {
                    const unsigned v = __hip_atomic_load(a.cnt + threadIdx.x * kStride, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_AGENT);
                    if (__ballot((int)(v - want) < 0) == 0ull) break;
                    if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > 100000000ll) {
                        *a.err = 1;
                        break;
                    }
                    __builtin_amdgcn_s_sleep(2);
                }
            }
        } else if (threadIdx.x == 0) {
            const unsigned want = (unsigned)(t - 1) * 8u;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while ((int)(__hip_atomic_load(a.cnt + 8 * kStride, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) - want) < 0) {
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > 100000000ll) {
                    *a.err = 1;
                    break;
                }
                __builtin_amdgcn_s_sleep(2);
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __syncthreads();
    }
    const int gid = blockIdx.x * kBlock + threadIdx.x;
    float x = (float)threadIdx.x * 1e-3f, y = (float)blockIdx.x;
    if (a.mode & kMem) {   // the previous launch's output, read past L1
        const float4* src = (t & 1) ? a.a : a.b;
        unsigned long long* q = reinterpret_cast<unsigned long long*>(const_cast<float4*>(src + 4 * gid));
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            const unsigned long long w = __hip_atomic_load(q + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            x += __uint_as_float((unsigned)w) * 1e-30f;
        }
    }
    for (int i = 0; i < a.iters; ++i) {
        x = __builtin_fmaf(x, 1.0000001f, 0.25f);
        y = __builtin_fmaf(y, 0.9999f, x);
    }
    float4* dst = ((t & 1) ? a.b : a.a) + 4 * gid;
    unsigned long long* q = reinterpret_cast<unsigned long long*>(dst);
    const int nst = (a.mode & kMem) ? 8 : 2;
    for (int k = 0; k < nst; ++k)
        __hip_atomic_store(q + k, ((unsigned long long)__float_as_uint(y) << 32) | __float_as_uint(x), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    if (ovl) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            const int s = blockIdx.x & 7;
            if (a.mode & kShards) {
                __hip_atomic_fetch_add(a.cnt + s * kStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                const unsigned per = (unsigned)((a.groups - s + 7) >> 3);
                const unsigned old = __hip_atomic_fetch_add(a.cnt + s * kStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (old + 1u == (unsigned)t * per)
                    __hip_atomic_fetch_add(a.cnt + 8 * kStride, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
}

static double run(const Args& base, int mode, int n, hipStream_t s1, hipStream_t s2) {
    Args a = base;
    a.mode = mode;
    CHECK(hipMemset(a.cnt, 0, sizeof(unsigned) * 9 * kStride));
    CHECK(hipDeviceSynchronize());
    hipEvent_t e0, e1, ef, ej;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    CHECK(hipEventCreateWithFlags(&ef, hipEventDisableTiming));
    CHECK(hipEventCreateWithFlags(&ej, hipEventDisableTiming));
    CHECK(hipEventRecord(e0, s1));
    const bool ovl = mode & kOvl;
    if (ovl) {
        CHECK(hipEventRecord(ef, s1));
        CHECK(hipStreamWaitEvent(s2, ef, 0));
    }
    for (int t = 1; t <= n; ++t) {
        hipStream_t s = (ovl && (t & 1) == 0) ? s2 : s1;
        hipLaunchKernelGGL(k_body, dim3(a.groups), dim3(kBlock), 0, s, a, t);
    }
    if (ovl) {
        CHECK(hipEventRecord(ej, s2));
        CHECK(hipStreamWaitEvent(s1, ej, 0));
    }
    CHECK(hipEventRecord(e1, s1));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    int err = 0;
    CHECK(hipMemcpy(&err, a.err, sizeof(int), hipMemcpyDeviceToHost));
    if (err) printf("  (a wait timed out)\n");
    for (hipEvent_t e : {e0, e1, ef, ej}) CHECK(hipEventDestroy(e));
    return 1e3 * ms / n;
}

static double one_launch(const Args& base, int mode, hipStream_t s) {   // a single launch's span
    Args a = base;
    a.mode = mode & ~kOvl;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    double best = 1e30;
    for (int r = 0; r < 20; ++r) {
        hipExtLaunchKernelGGL(k_body, dim3(a.groups), dim3(kBlock), 0, s, e0, e1, 0u, a, 1);
        CHECK(hipEventSynchronize(e1));
        float ms = 0;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        if (ms * 1e3 < best) best = ms * 1e3;
    }
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return best;
}

int main(int argc, char** argv) {
    const int iters = argc > 1 ? atoi(argv[1]) : 1500;
    Args a{};
    CHECK(hipMalloc(&a.cnt, sizeof(unsigned) * 9 * kStride));
    CHECK(hipMalloc(&a.a, sizeof(float4) * 4 * 1025 * kBlock));
    CHECK(hipMalloc(&a.b, sizeof(float4) * 4 * 1025 * kBlock));
    CHECK(hipMalloc(&a.err, sizeof(int)));
    CHECK(hipMemset(a.err, 0, sizeof(int)));
    CHECK(hipMemset(a.a, 0, sizeof(float4) * 4 * 1025 * kBlock));
    CHECK(hipMemset(a.b, 0, sizeof(float4) * 4 * 1025 * kBlock));
    a.iters = iters;
    a.groups = argc > 2 ? atoi(argv[2]) : 1025;
    hipStream_t s1, s2;
    CHECK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CHECK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    const int n = 400;
    printf("iters %d, %d workgroups x %d threads, %d launches per run (us per launch, best of 3 runs)\n", iters,
           a.groups, kBlock, n);
    const struct {
        const char* name;
        int mode;
    } forms[] = {{"serial", 0},       {"ovl-top", kOvl},          {"ovl-shards", kOvl | kShards},
                 {"serial+mem", kMem}, {"ovl-top+mem", kOvl | kMem}, {"ovl-shards+mem", kOvl | kShards | kMem}};
    for (const auto& f : forms) {
        run(a, f.mode, 40, s1, s2);   // warm-up
        double best = 1e30;
        for (int r = 0; r < 3; ++r) {
            const double us = run(a, f.mode, n, s1, s2);
            if (us < best) best = us;
        }
        printf("%-16s %7.2f us per launch   (one launch alone: %6.2f us)\n", f.name, best, one_launch(a, f.mode, s1));
    }
    return 0;
}
