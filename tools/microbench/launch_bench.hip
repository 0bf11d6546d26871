// Per-launch cost of back-to-back dependent launches on one stream, by what the
// kernel stores: nothing, or 58 B per thread of a 262,144-thread grid (k_expand's
// slot outputs: 16 + 16 + 16 + 8 + 2 B) as plain, nt or sc1 (write-through) stores.
// Separates the end-of-kernel release (dirty L2 write-back) from launch overhead.
//
//   hipcc --offload-arch=gfx950 -O3 tools/microbench/launch_bench.hip -o tools/microbench/launch_bench
//   tools/microbench/launch_bench
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

constexpr int kThreads = 262144, kBlock = 256;

struct Bufs {
    float4* a;
    float4* b;
    uint4* c;
    uint2* e;
    unsigned short* f;
};

__global__ __launch_bounds__(kBlock) void k_empty(Bufs, int) {}
__global__ __launch_bounds__(1024) void k_empty1024(Bufs, int) {}

template <int MODE>   // 0 plain, 1 nt, 2 sc1 (agent-scope relaxed atomic stores are sc1)
__device__ __forceinline__ void st16(float4* p, float4 v) {
    if (MODE == 0) *p = v;
    else if (MODE == 1) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        __builtin_nontemporal_store(f4{v.x, v.y, v.z, v.w}, reinterpret_cast<f4*>(p));
    }
    else {
        unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
        __hip_atomic_store(q, ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x), __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 1, ((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int MODE>
__global__ __launch_bounds__(kBlock) void k_store(Bufs b, int t) {
    const int i = blockIdx.x * kBlock + threadIdx.x;
    const float v = (float)(i + t);
    st16<MODE>(&b.a[i], make_float4(v, v, v, v));
    st16<MODE>(&b.b[i], make_float4(v, v, v, v));
    st16<MODE>(reinterpret_cast<float4*>(&b.c[i]), make_float4(v, v, v, v));
    if (MODE == 1) {
        typedef unsigned u2 __attribute__((ext_vector_type(2)));
        __builtin_nontemporal_store(u2{(unsigned)i, (unsigned)t}, reinterpret_cast<u2*>(&b.e[i]));
        __builtin_nontemporal_store((unsigned short)i, &b.f[i]);
    } else {
        b.e[i] = make_uint2(i, t);
        b.f[i] = (unsigned short)i;
    }
}

template <typename K>
static float time_launches(K kernel, const Bufs& b, int n, hipStream_t s, int grid = kThreads / kBlock,
                           int block = kBlock) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, s, b, i);
    CHECK(hipEventRecord(e0, s));
    for (int i = 0; i < n; ++i) hipLaunchKernelGGL(kernel, dim3(grid), dim3(block), 0, s, b, i);
    CHECK(hipEventRecord(e1, s));
    CHECK(hipEventSynchronize(e1));
    float ms = 0;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.0f / n;
}

int main() {
    Bufs b;
    CHECK(hipMalloc(&b.a, sizeof(float4) * kThreads));
    CHECK(hipMalloc(&b.b, sizeof(float4) * kThreads));
    CHECK(hipMalloc(&b.c, sizeof(uint4) * kThreads));
    CHECK(hipMalloc(&b.e, sizeof(uint2) * kThreads));
    CHECK(hipMalloc(&b.f, sizeof(unsigned short) * kThreads));
    hipStream_t s;
    CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    const int n = 2000;
    for (int g : {1, 8, 64, 256, 512, 1024, 2048, 4096})
        printf("empty grid %5d x 256   %.2f us/launch\n", g, time_launches(k_empty, b, n, s, g, 256));
    for (int g : {256, 512})
        printf("empty grid %5d x 1024  %.2f us/launch\n", g, time_launches(k_empty1024, b, n, s, g, 1024));
    for (int work = 0; work < 2; ++work)
        for (int per : {2, 8, 16, 32, 64, 200}) {   // the same dependent launches replayed from a captured graph
            hipGraph_t g;
            hipGraphExec_t ge;
            CHECK(hipStreamBeginCapture(s, hipStreamCaptureModeGlobal));
            for (int i = 0; i < per; ++i) {
                if (work) hipLaunchKernelGGL(k_store<0>, dim3(1024), dim3(256), 0, s, b, i);
                else hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, b, i);
            }
            CHECK(hipStreamEndCapture(s, &g));
            CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
            hipEvent_t e0, e1;
            CHECK(hipEventCreate(&e0));
            CHECK(hipEventCreate(&e1));
            CHECK(hipGraphLaunch(ge, s));
            const int reps = 3200 / per;
            CHECK(hipEventRecord(e0, s));
            for (int r = 0; r < reps; ++r) CHECK(hipGraphLaunch(ge, s));
            CHECK(hipEventRecord(e1, s));
            CHECK(hipEventSynchronize(e1));
            float ms = 0;
            CHECK(hipEventElapsedTime(&ms, e0, e1));
            printf("graph of %3d nodes: %s  %.2f us/kernel\n", per, work ? "plain 58B" : "empty    ",
                   ms * 1000.0f / (reps * per));
        }
    for (int rep = 0; rep < 2; ++rep) {
        printf("empty      %.2f us/launch\n", time_launches(k_empty, b, n, s));
        printf("plain 58B  %.2f us/launch\n", time_launches(k_store<0>, b, n, s));
        printf("nt    58B  %.2f us/launch\n", time_launches(k_store<1>, b, n, s));
        printf("sc1   56B  %.2f us/launch\n", time_launches(k_store<2>, b, n, s));
    }
    return 0;
}
