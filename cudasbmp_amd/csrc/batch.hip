// batch.hip — the step-level entry points (include/sbmp/sbmp.h):
// one stage of the KGMT iteration over caller buffers, built on the public
// device-function headers (propagateAndCheck, getR1 / getR2, inGoalRegion) so that
// those headers are exercised exactly as a user kernel would call them.
//   sbmp_expand_batch   propagateG's per-child work (KGMT.cu:386-411)
//   sbmp_insert_batch   exclusive_scan(GNew) + findInd + updateG (KGMT.cu:221-249, 540-593)
// The planner's own kernels (kgmt_kernels.hip) fuse these stages; the parity tests
// hold both to the same CPU oracle.
#include <hip/hip_runtime.h>

#include <climits>
#include <string>

#include "kgmt_planner.h"
#include "sbmp/grid.h"
#include "sbmp/propagator.h"
#include "sbmp/sbmp.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace sbmp {

// One child of propagateG (KGMT.cu:386-411), for the kernel and the host loop alike.
SBMP_HD void expand_one(const sbmp_expand_batch_args& a, int i) {
    Xorwow rs{a.rng[6 * i], a.rng[6 * i + 1], a.rng[6 * i + 2], a.rng[6 * i + 3], a.rng[6 * i + 4], a.rng[6 * i + 5]};
    float x1[7];
    const float* x0 = a.parents + 7 * (size_t)i;
    const bool ok = (a.agent == SBMP_AGENT_POINT)
                        ? propagatePoint(x0, x1, a.numDisc, &rs, a.obstacles, a.obstaclesCount, a.width, a.height)
                        : propagateAndCheck(x0, x1, a.numDisc, a.agentLength, &rs, a.obstacles, a.obstaclesCount,
                                            a.width, a.height);
    const float R1Size = a.width / (float)a.N;          // KGMT.cu:13
    const float R2Size = a.width / (float)(a.n * a.N);  // KGMT.cu:14
    const int c1 = getR1(x1[0], x1[1], R1Size, a.N);
    const int c2 = getR2(x1[0], x1[1], c1, R1Size, a.N, R2Size, a.n);
    uint8_t acc = 0;
    if (ok && a.R1Score) {   // KGMT.cu:394-400 (D3: a child outside the grid is rejected)
        const float u = xorwow_uniform(rs);
        acc = (c1 >= 0 && c2 >= 0 && (u <= a.R1Score[c1] || a.R2Avail[c2] == 0)) ? 1 : 0;
    }
    for (int k = 0; k < 7; ++k) a.children[7 * (size_t)i + k] = x1[k];
    if (a.valid) a.valid[i] = ok ? 1 : 0;
    if (a.r1) a.r1[i] = c1;
    if (a.r2) a.r2[i] = c2;
    if (a.accept) a.accept[i] = acc;
    a.rng[6 * i] = rs.v0;
    a.rng[6 * i + 1] = rs.v1;
    a.rng[6 * i + 2] = rs.v2;
    a.rng[6 * i + 3] = rs.v3;
    a.rng[6 * i + 4] = rs.v4;
    a.rng[6 * i + 5] = rs.d;
}

__global__ __launch_bounds__(256) void k_expand_batch(sbmp_expand_batch_args a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i < a.count) expand_one(a, i);
}

// insert, pass 1: flagged slots per 256-slot block.
__global__ __launch_bounds__(256) void k_insert_count(sbmp_insert_batch_args a, int* blockCount) {
    __shared__ int sWave[4];
    const int s = blockIdx.x * 256 + threadIdx.x;
    const bool f = s < a.slots && a.gnew[s];
    const unsigned long long m = __ballot(f);
    if ((threadIdx.x & 63) == 0) sWave[threadIdx.x >> 6] = __popcll(m);
    __syncthreads();
    if (threadIdx.x == 0) blockCount[blockIdx.x] = sWave[0] + sWave[1] + sWave[2] + sWave[3];
}

// insert, pass 2 (one workgroup): exclusive prefix of the block counts in place,
// total into blockCount[nBlocks] and *inserted.
__global__ __launch_bounds__(256) void k_insert_scan(int* blockCount, int nBlocks, int* inserted, int* goalIndex) {
    __shared__ int sPart[256];
    __shared__ int sCarry;
    if (threadIdx.x == 0) sCarry = 0;
    __syncthreads();
    for (int base = 0; base < nBlocks; base += 256) {
        const int i = base + threadIdx.x;
        const int v = i < nBlocks ? blockCount[i] : 0;
        sPart[threadIdx.x] = v;
        __syncthreads();
        for (int off = 1; off < 256; off <<= 1) {   // Hillis-Steele inclusive scan
            const int add = threadIdx.x >= off ? sPart[threadIdx.x - off] : 0;
            __syncthreads();
            sPart[threadIdx.x] += add;
            __syncthreads();
        }
        if (i < nBlocks) blockCount[i] = sCarry + sPart[threadIdx.x] - v;
        __syncthreads();
        if (threadIdx.x == 0) sCarry += sPart[255];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        blockCount[nBlocks] = sCarry;
        *inserted = sCarry;
        *goalIndex = INT_MAX;
    }
}

// insert, pass 3: row treeSize + j for the j-th flagged slot (updateG, KGMT.cu:540-593).
__global__ __launch_bounds__(256) void k_insert_rows(sbmp_insert_batch_args a, const int* blockPrefix, int nBlocks) {
    __shared__ int sWave[4];
    const int s = blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool f = s < a.slots && a.gnew[s];
    const unsigned long long m = __ballot(f);
    if (lane == 0) sWave[wave] = __popcll(m);
    __syncthreads();
    const int A = blockPrefix[nBlocks];
    const int M = a.maxTreeSize;
    const int grid = min(A, M / 32);        // updateG launch: min(|GNew|, M/32) blocks of 32 (KGMT.cu:231)
    const int nIns = min(A, 32 * grid);
    if (f) {
        int j = blockPrefix[blockIdx.x] + __popcll(m & ((1ull << lane) - 1ull));
        for (int w = 0; w < wave; ++w) j += sWave[w];
        const int dst = a.treeSize + j;
        if (j < nIns && dst < M) {          // D13: the reference writes past M here
            const float* u = a.unexplored + 7 * (size_t)s;
            const int par = a.uParent[s];
            for (int k = 0; k < 7; ++k) a.samples[7 * (size_t)dst + k] = u[k];
            a.parent[dst] = par;
            a.costs[dst] = a.costs[par] + getCost(nullptr, u);   // getCost, KGMT.cu:631-633
            const float goal[2] = {a.goalX, a.goalY};
            if (inGoalRegion(u, goal, a.goalThreshold)) atomicMin(a.goalIndex, dst);   // D4: lowest row
        }
    }
    // D6: GNew[0 .. 32 * grid) is cleared (all of it with fixGNewClear)
    if (s < a.slots && (a.fixGNewClear || s < 32 * grid)) a.gnew[s] = 0;
}

__global__ void k_insert_goal_fixup(int* goalIndex) {
    if (*goalIndex == INT_MAX) *goalIndex = -1;
}

}  // namespace sbmp

namespace sbmp {

static void check_expand(const sbmp_expand_batch_args* a) {
    if (!a) throw Error(SBMP_ERR_INVALID_ARGUMENT, "NULL args");
    if (a->count < 0 || a->numDisc < 1 || a->N < 1 || a->n < 1 || a->obstaclesCount < 0)
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "bad batch sizes");
    if (a->count > 0 && (!a->parents || !a->rng || !a->children))
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "parents, rng and children are required");
    if (a->obstaclesCount > 0 && !a->obstacles) throw Error(SBMP_ERR_INVALID_ARGUMENT, "NULL obstacles");
    if ((a->R1Score == nullptr) != (a->R2Avail == nullptr))
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "R1Score and R2Avail go together");
    if (a->agent != SBMP_AGENT_CAR && a->agent != SBMP_AGENT_POINT) throw Error(SBMP_ERR_INVALID_ARGUMENT, "agent");
}

void expand_batch(const sbmp_expand_batch_args* args, void* stream) {
    check_expand(args);
    if (args->count == 0) return;
    const hipStream_t s = static_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_expand_batch, dim3((args->count + 255) / 256), dim3(256), 0, s, *args);
    SBMP_HIP(hipGetLastError());
    SBMP_HIP(hipStreamSynchronize(s));
}

void expand_batch_host(const sbmp_expand_batch_args* args) {
    check_expand(args);
    for (int i = 0; i < args->count; ++i) expand_one(*args, i);
}

void insert_batch(const sbmp_insert_batch_args* a, void* stream) {
    if (!a || a->slots < 0 || a->maxTreeSize < 1 || a->treeSize < 0)
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "bad insert batch sizes");
    if (!a->gnew || !a->unexplored || !a->uParent || !a->samples || !a->parent || !a->costs || !a->inserted ||
        !a->goalIndex)
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "NULL buffer");
    const hipStream_t s = static_cast<hipStream_t>(stream);
    const int nBlocks = (a->slots + 255) / 256;
    int* counts = nullptr;
    SBMP_HIP(hipMalloc(reinterpret_cast<void**>(&counts), sizeof(int) * ((size_t)nBlocks + 1)));
    if (nBlocks > 0) hipLaunchKernelGGL(k_insert_count, dim3(nBlocks), dim3(256), 0, s, *a, counts);
    hipLaunchKernelGGL(k_insert_scan, dim3(1), dim3(256), 0, s, counts, nBlocks, a->inserted, a->goalIndex);
    if (nBlocks > 0) hipLaunchKernelGGL(k_insert_rows, dim3(nBlocks), dim3(256), 0, s, *a, counts, nBlocks);
    hipLaunchKernelGGL(k_insert_goal_fixup, dim3(1), dim3(1), 0, s, a->goalIndex);
    const hipError_t e = hipGetLastError();
    const hipError_t e2 = hipStreamSynchronize(s);
    (void)hipFree(counts);
    SBMP_HIP(e);
    SBMP_HIP(e2);
}

}  // namespace sbmp
