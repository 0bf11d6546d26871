// Copy / read bandwidth sweep for the choice of sbmp_hbm_copy_bandwidth's kernel shape
// (cudasbmp_amd/csrc/measure.hip).  Build + run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 -o tools/microbench/copy_bench tools/microbench/copy_bench.hip
//   tools/microbench/copy_bench
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

typedef float v4f __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy(const v4f* __restrict__ src, v4f* __restrict__ dst, long long n) {
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long base = (long long)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
        v4f v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = base + (long long)u * 256;
            if (i < n) v[u] = NT ? __builtin_nontemporal_load(src + i) : src[i];
        }
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = base + (long long)u * 256;
            if (i < n) {
                if (NT) __builtin_nontemporal_store(v[u], dst + i);
                else dst[i] = v[u];
            }
        }
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const v4f* __restrict__ src, float* out, long long n) {
    const long long stride = (long long)gridDim.x * 256 * U;
    v4f acc = {0.f, 0.f, 0.f, 0.f};
    for (long long base = (long long)blockIdx.x * 256 * U + threadIdx.x; base < n; base += stride) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const long long i = base + (long long)u * 256;
            if (i < n) acc += __builtin_nontemporal_load(src + i);
        }
    }
    if (acc.x + acc.y + acc.z + acc.w == 12345.0f) out[0] = 1.0f;
}

#define CK(x)                                                              \
    do {                                                                   \
        hipError_t e = (x);                                                \
        if (e != hipSuccess) {                                             \
            std::printf("%s: %s\n", #x, hipGetErrorString(e));             \
            return 1;                                                      \
        }                                                                  \
    } while (0)

template <typename F>
static double best_ms(F launch, hipEvent_t e0, hipEvent_t e1) {
    double best = 1e30;
    for (int r = 0; r < 6; ++r) {
        (void)hipEventRecord(e0, 0);
        launch();
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (r > 0) best = std::min(best, (double)ms);
    }
    return best;
}

int main() {
    const size_t bytes = (size_t)4 << 30;
    const long long n = (long long)(bytes / 16);
    v4f *a, *b;
    float* o;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMalloc(&o, 16));
    CK(hipMemset(a, 0, bytes));
    CK(hipMemset(b, 0, bytes));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int cus = 256;
    for (int mult : {4, 8, 16, 32}) {
        const int g = cus * mult;
        double ms;
        ms = best_ms([&] { hipLaunchKernelGGL((k_copy<4, true>), dim3(g), dim3(256), 0, 0, a, b, n); }, e0, e1);
        std::printf("copy U4 nt   grid %5d: %7.1f GB/s\n", g, 2.0 * bytes / (ms * 1e-3) / 1e9);
        ms = best_ms([&] { hipLaunchKernelGGL((k_copy<4, false>), dim3(g), dim3(256), 0, 0, a, b, n); }, e0, e1);
        std::printf("copy U4 plain grid %5d: %7.1f GB/s\n", g, 2.0 * bytes / (ms * 1e-3) / 1e9);
        ms = best_ms([&] { hipLaunchKernelGGL((k_copy<8, true>), dim3(g), dim3(256), 0, 0, a, b, n); }, e0, e1);
        std::printf("copy U8 nt   grid %5d: %7.1f GB/s\n", g, 2.0 * bytes / (ms * 1e-3) / 1e9);
        ms = best_ms([&] { hipLaunchKernelGGL((k_copy<1, true>), dim3(g), dim3(256), 0, 0, a, b, n); }, e0, e1);
        std::printf("copy U1 nt   grid %5d: %7.1f GB/s\n", g, 2.0 * bytes / (ms * 1e-3) / 1e9);
        ms = best_ms([&] { hipLaunchKernelGGL((k_read<4>), dim3(g), dim3(256), 0, 0, a, o, n); }, e0, e1);
        std::printf("read U4 nt   grid %5d: %7.1f GB/s\n", g, 1.0 * bytes / (ms * 1e-3) / 1e9);
    }
    double ms = best_ms([&] { (void)hipMemcpyAsync(b, a, bytes, hipMemcpyDeviceToDevice, 0); }, e0, e1);
    std::printf("hipMemcpy D2D        : %7.1f GB/s\n", 2.0 * bytes / (ms * 1e-3) / 1e9);
    return 0;
}
