// kgmt_kernels.hip — hand-written gfx950 kernels of the KGMT iteration.
//
// One reference iteration (reference src/planners/KGMT.cu:118-292) becomes three
// kernels on one stream, with no host round trip:
//   k_expand(t)  : propagateG / propagateGV2 (KGMT.cu:341-482) fused with
//                  propagateAndCheck + isMotionValid (statePropagator.cu:5-76,
//                  collisionCheck.cu:6-28), region binning and the accept test.
//                  One thread per child slot, wave64 ballot -> GNew bitmask.
//   k_plan(t+1)  : exclusive_scan(GNew) (KGMT.cu:222-224) as a popcount scan of
//                  the bitmask, application of this iteration's region deltas,
//                  the next iteration's frontier/batch decision (KGMT.cu:139-188)
//                  and updateR1 (KGMT.cu:485-538).  One 1024-thread workgroup.
//   k_insert(t)  : findInd + updateG (KGMT.cu:225-245,540-593): append accepted
//                  children in slot order, goal test, partial GNew clear (D6).
// The reference's O(M) G scan + findInd disappears: every frontier node is
// expanded each iteration and new rows are appended contiguously, so G is
// always the row range [gLo, treeSize) (parity-tested against the oracle,
// which keeps the literal boolean scans).
#include <hip/hip_runtime.h>

#include "kgmt_device.h"
#include "kgmt_launch.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace sbmp {

// ------------------------------------------------------------------ expand
template <int AGENT>
__global__ __launch_bounds__(kBlock) void k_expand(KgmtDev d, int t) {
    __shared__ float sScore[kMaxR1];
    __shared__ int sCnt[4][kMaxR1];   // R1, R1Valid, R1Invalid, R1AvailSet (block-private)

    const IterCtrl c = d.ctrl[t];
    if (!c.run || d.status->goalIdx != kNoGoal) return;   // grid-uniform
    const int gblock = d.rank + d.nranks * (int)blockIdx.x;  // block-cyclic slot ownership
    const int slotBase = gblock * kBlock;
    if (slotBase >= c.S) return;                           // block-uniform

    const int tid = threadIdx.x;
    const float* score = d.R1Score + c.scoreBuf * d.nR1;
    for (int i = tid; i < d.nR1; i += kBlock) {
        sScore[i] = score[i];
        sCnt[0][i] = 0;
        sCnt[1][i] = 0;
        sCnt[2][i] = 0;
        sCnt[3][i] = 0;
    }
    __syncthreads();

    const int slot = slotBase + tid;
    bool accept = false;
    if (slot < c.S) {
        const int g = (c.k == 32) ? (slot >> 5) : (slot / c.k);   // slot = g*k + i
        const int parent = c.gLo + g;
        const float4 p = d.treeState[parent];
        const uint4 ra = d.rngA[slot];
        const uint2 rb = d.rngB[slot];
        Xorwow rs{ra.x, ra.y, ra.z, ra.w, rb.x, rb.y};
        ChildOut ch;
        const bool valid = (AGENT == 0) ? propagate_car(p, rs, d, ch) : propagate_point(p, rs, d, ch);
        const int r1 = getR1(ch.state.x, ch.state.y, d.R1Size, d.N);
        const int r2 = getR2(ch.state.x, ch.state.y, r1, d.R1Size, d.N, d.R2Size, d.n);
        if (valid) {
            const float u = xorwow_uniform(rs);   // KGMT.cu:395
            if (r1 >= 0 && r2 >= 0) {
                const bool r2Avail = (d.R2Snap[r2 >> 5] >> (r2 & 31)) & 1u;
                accept = (u <= sScore[r1]) || !r2Avail;
                if (!r2Avail) d.delta[4 * d.nR1 + r2] = 1;   // idempotent plain store
            }
        }
        // Region counters (KGMT.cu:392-411; D3: in-grid cells only).
        if (r1 >= 0) {
            atomicAdd(&sCnt[0][r1], 1);
            if (valid) {
                atomicAdd(&sCnt[1][r1], 1);
                sCnt[3][r1] = 1;
            } else {
                atomicAdd(&sCnt[2][r1], 1);
            }
        }
        if (r2 >= 0) atomicAdd(valid ? &d.R2Valid[r2] : &d.R2Invalid[r2], 1);

        d.uState[slot] = ch.state;
        d.uCtrl[slot] = make_float4(ch.a, ch.steer, ch.dur, __int_as_float(parent));
        d.rngA[slot] = make_uint4(rs.v0, rs.v1, rs.v2, rs.v3);
        d.rngB[slot] = make_uint2(rs.v4, rs.d);
    }
    // GNew |= accept (stale bits survive, D6).  A wave covers one 64-bit word.
    const unsigned long long mask = __ballot(accept);
    if ((tid & (kWave - 1)) == 0 && mask) d.gnew[slot >> 6] |= mask;

    __syncthreads();
    for (int i = tid; i < d.nR1; i += kBlock) {
        if (sCnt[0][i]) atomicAdd(&d.delta[i], sCnt[0][i]);
        if (sCnt[1][i]) atomicAdd(&d.delta[d.nR1 + i], sCnt[1][i]);
        if (sCnt[2][i]) atomicAdd(&d.delta[2 * d.nR1 + i], sCnt[2][i]);
        if (sCnt[3][i]) d.delta[3 * d.nR1 + i] = 1;
    }
}

// ------------------------------------------------------------------ plan
// Block-wide exclusive scan of one int per thread (1024 threads = 16 waves).
__device__ __forceinline__ int block_exclusive_scan(int v, int* sWave, int* total) {
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int off = 1; off < kWave; off <<= 1) {
        const int y = __shfl_up(x, off, kWave);
        if (lane >= off) x += y;
    }
    if (lane == kWave - 1) sWave[wave] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int run = 0;
        for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
            const int s = sWave[w];
            sWave[w] = run;
            run += s;
        }
        sWave[16] = run;
    }
    __syncthreads();
    *total = sWave[16];
    return sWave[wave] + x - v;
}

__global__ __launch_bounds__(1024) void k_plan(KgmtDev d, int t) {
    __shared__ int sWave[17];
    __shared__ int sCovInc[kMaxR1];
    __shared__ float sScore[kMaxR1];
    __shared__ float sPart[8];

    const int tid = threadIdx.x;
    bool ranPrev = false;
    if (t > 1) ranPrev = d.ctrl[t - 1].run && d.status->goalIdx == kNoGoal;
    if (t > 1 && !ranPrev) {
        if (tid == 0) d.ctrl[t].run = 0;
        return;
    }

    int treeSize = 1, gLo = 0, H = 0, A = 0;
    IterCtrl pc;
    if (ranPrev) {
        pc = d.ctrl[t - 1];
        H = pc.H;
        // (1) exclusive_scan(GNew) over [0, H): popcounts of the bitmask words.
        const int nw = (H + 63) >> 6;
        const int per = (nw + (int)blockDim.x - 1) / (int)blockDim.x;
        const int w0 = min(nw, tid * per), w1 = min(nw, w0 + per);
        int cnt = 0;
        for (int w = w0; w < w1; ++w) cnt += __popcll(d.gnew[w]);
        int run = block_exclusive_scan(cnt, sWave, &A);
        for (int w = w0; w < w1; ++w) {
            d.wordOffsets[w] = run;
            run += __popcll(d.gnew[w]);
        }
    }
    {
        // (2) fold the previous expansion's region deltas into the tables and take
        // the availability snapshot for iteration t (t == 1: deltas are zero).
        if (tid < kMaxR1) sCovInc[tid] = 0;
        for (int i = tid; i < d.nR1; i += blockDim.x) {
            int* dl = d.delta;
            const int a0 = dl[i], a1 = dl[d.nR1 + i], a2 = dl[2 * d.nR1 + i], a3 = dl[3 * d.nR1 + i];
            if (a0) { d.R1[i] += a0; dl[i] = 0; }
            if (a1) { d.R1Valid[i] += a1; dl[d.nR1 + i] = 0; }
            if (a2) { d.R1Invalid[i] += a2; dl[2 * d.nR1 + i] = 0; }
            if (a3) { d.R1Avail[i] = 1; dl[3 * d.nR1 + i] = 0; }
        }
        __syncthreads();
        const int nn = d.n * d.n;
        const int nR2w = d.nR2 >> 5;
        for (int w = tid; w < nR2w; w += blockDim.x) {   // one thread owns one availability word
            int4* dl = reinterpret_cast<int4*>(d.delta + 4 * d.nR1 + 32 * w);
            uint32_t bits = d.R2Avail[w];
            const uint32_t old = bits;
#pragma unroll
            for (int q = 0; q < 8; ++q) {
                const int4 v = dl[q];
                if (v.x | v.y | v.z | v.w) {
                    const int c0 = 32 * w + 4 * q;
                    const int vv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        const uint32_t b = 1u << (4 * q + e);
                        if (vv[e] && !(bits & b)) {
                            bits |= b;
                            atomicAdd(&sCovInc[(c0 + e) / nn], 1);
                        }
                    }
                    dl[q] = make_int4(0, 0, 0, 0);
                }
            }
            if (bits != old) d.R2Avail[w] = bits;
            d.R2Snap[w] = bits;   // snapshot for the next expand (D2)
        }
        __syncthreads();
        if (tid < d.nR1 && sCovInc[tid]) d.R1Cov[tid] += sCovInc[tid];
    }
    if (ranPrev) {
        treeSize = pc.treeSize + A;
        gLo = pc.gLo + pc.nExp;
        if (tid == 0) {
            d.ctrl[t - 1].executed = 1;
            d.ctrl[t - 1].A = A;
        }
    }

    // (3) next iteration's frontier / batch decision (KGMT.cu:151-158 + capped extension).
    const int run_t = (t <= d.numIterations) && (treeSize < d.M);
    int nG = 0, k = 0, nExp = 0;
    if (run_t) {
        nG = treeSize - gLo;
        if (nG > 0) {
            long long remaining = (long long)d.M - treeSize;
            if (d.cap > 0 && remaining > d.cap) remaining = d.cap;
            if (32ll * nG <= remaining) {
                k = 32;
                nExp = nG;
            } else {
                k = (int)((float)remaining / (float)nG);   // KGMT.cu:157
                nExp = nG;
                if (d.cap > 0 && k == 0) {
                    k = 1;
                    nExp = (int)remaining;
                }
            }
        }
    }
    const int S = k * nExp;
    const int buf = t & 1;

    // (4) updateR1 (KGMT.cu:485-538) for iteration t.
    if (run_t) {
        __syncthreads();
        if (tid < d.nR1) {
            float s = 0.0f;
            if (d.R1Avail[tid] != 0) {
                const int nValid = d.R1Valid[tid];
                const float covR = (float)d.R1Cov[tid] / (float)(d.n * d.n);
                const float freeVol = (0.01f + (float)nValid) / (0.01f + (float)nValid + (float)d.R1Invalid[tid]);
                const float fv2 = freeVol * freeVol;
                const float fv4 = fv2 * fv2;
                const double r = (double)d.R1[tid];
                const double den = (double)(1.0f + covR) * (1.0 + r * r);
                s = (float)((double)fv4 / den);
            }
            sScore[tid] = s;
        }
        __syncthreads();
        if (tid < 8) {   // CUB BlockReduce order (D8): balanced tree per 32 group ...
            float tt[32];
#pragma unroll
            for (int i = 0; i < 32; ++i) tt[i] = sScore[tid * 32 + i];
#pragma unroll
            for (int off = 1; off < 32; off <<= 1) {
#pragma unroll
                for (int i = 0; i + off < 32; i += 2 * off) tt[i] = tt[i] + tt[i + off];
            }
            sPart[tid] = tt[0];
        }
        __syncthreads();
        if (tid == 0) {   // ... then the warp aggregates in order
            float total = sPart[0];
            for (int w = 1; w < 8; ++w) total = total + sPart[w];
            sPart[0] = total;
        }
        __syncthreads();
        if (tid < d.nR1) {
            const float total = sPart[0];
            d.R1Score[buf * d.nR1 + tid] = (d.R1Avail[tid] == 0) ? 1.0f : sScore[tid] / total;
        }
    }
    if (tid == 0) {
        IterCtrl c;
        c.run = run_t;
        c.executed = 0;
        c.treeSize = treeSize;
        c.gLo = gLo;
        c.nG = nG;
        c.k = k;
        c.nExp = nExp;
        c.S = S;
        c.H = max(H, S);
        c.A = 0;
        c.scoreBuf = buf;
        for (int i = 0; i < 5; ++i) c.pad[i] = 0;
        d.ctrl[t] = c;
    }
}

// ------------------------------------------------------------------ insert
__global__ __launch_bounds__(kBlock) void k_insert(KgmtDev d, int t) {
    const IterCtrl c = d.ctrl[t];
    if (!c.executed) return;
    const int lane = threadIdx.x & (kWave - 1);
    const int w = blockIdx.x * (kBlock / kWave) + (threadIdx.x >> 6);
    const int nw = (c.H + 63) >> 6;
    if (w >= nw) return;
    const unsigned long long word = d.gnew[w];
    if (word == 0ull) return;

    const int m32 = d.M / 32;
    const int grid = min(c.A, m32);   // updateG launch: min(|GNew|, M/32) blocks of 32 (KGMT.cu:231)
    const int nIns = 32 * grid < c.A ? 32 * grid : c.A;
    if ((word >> lane) & 1ull) {
        const int j = d.wordOffsets[w] + __popcll(word & ((1ull << lane) - 1ull));
        const int dst = c.treeSize + j;
        if (j < nIns && dst < d.M) {   // D13: the reference writes past M here
            const int slot = w * kWave + lane;
            const float4 s = d.uState[slot];
            const float4 u = d.uCtrl[slot];
            const int parent = __float_as_int(u.w);
            const float cost = d.treeCtrl[parent].w + u.z;   // getCost = duration (KGMT.cu:631-633)
            d.treeState[dst] = s;
            d.treeCtrl[dst] = make_float4(u.x, u.y, u.z, cost);
            d.treeParent[dst] = parent;
            const float dx = s.x - d.goalX, dy = s.y - d.goalY;   // inGoalRegion, KGMT.cu:635-638
            const float d2 = dx * dx + dy * dy;
            if (__builtin_sqrtf(d2) < d.goalThreshold) atomicMin(&d.status->goalIdx, dst);
        }
    }
    if (lane == 0) {   // D6: only GNew[0 .. 32*grid) is cleared
        const long long cleared = d.fixGNewClear ? (1ll << 62) : 32ll * grid;
        const long long base = (long long)w * kWave;
        unsigned long long nw_ = word;
        if (base + kWave <= cleared) nw_ = 0ull;
        else if (base < cleared) nw_ = word & ~((1ull << (cleared - base)) - 1ull);
        if (nw_ != word) d.gnew[w] = nw_;
    }
}

// ------------------------------------------------------------------ init
__global__ void k_fill_i32(int* p, int v, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        p[i] = v;
}

__global__ void k_fill_f32(float* p, float v, long long n) {
    for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
        p[i] = v;
}

// curand_init(seed, subsequence = slot, 0) for every owned slot (KGMT.cu:595-600):
// base state from the seed, then the subsequence jump A^(2^67 * slot) as a product
// of the precomputed GF(2) matrices J[b] = A^(2^(67+b)) (160 columns x 5 words).
__global__ __launch_bounds__(kBlock) void k_init_slots(KgmtDev d, Xorwow base, const uint32_t* __restrict__ jumps,
                                                      int nbits) {
    const int gblock = d.rank + d.nranks * (int)blockIdx.x;
    const int slot = gblock * kBlock + threadIdx.x;
    if (slot >= d.nSlots) return;
    uint32_t v[5] = {base.v0, base.v1, base.v2, base.v3, base.v4};
    for (int b = 0; b < nbits; ++b) {
        if (!((slot >> b) & 1)) continue;
        const uint32_t* J = jumps + (size_t)b * 800;
        uint32_t r[5] = {0u, 0u, 0u, 0u, 0u};
#pragma unroll
        for (int w = 0; w < 5; ++w) {
            const uint32_t vw = v[w];
            for (int k = 0; k < 32; ++k) {
                const uint32_t m = 0u - ((vw >> k) & 1u);
                const uint32_t* col = J + (w * 32 + k) * 5;
#pragma unroll
                for (int q = 0; q < 5; ++q) r[q] ^= col[q] & m;
            }
        }
#pragma unroll
        for (int q = 0; q < 5; ++q) v[q] = r[q];
    }
    d.rngA[slot] = make_uint4(v[0], v[1], v[2], v[3]);
    d.rngB[slot] = make_uint2(v[4], base.d);
    d.uState[slot] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    d.uCtrl[slot] = make_float4(0.0f, 0.0f, 0.0f, __int_as_float(-1));
}

// Root row and root region seeds (KGMT.cu:85-97).
__global__ void k_seed_root(KgmtDev d, float4 rootState, float4 rootCtrl, int r1, int r2) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    d.treeState[0] = rootState;
    d.treeCtrl[0] = rootCtrl;
    if (r1 >= 0) {
        d.R1[r1] = 1;
        d.R1Avail[r1] = 1;
        d.R1Valid[r1] = 1;
    }
    if (r2 >= 0) {
        d.R2Avail[r2 >> 5] |= 1u << (r2 & 31);
        d.R1Cov[r2 / (d.n * d.n)] += 1;
    }
    d.status->goalIdx = kNoGoal;
}

// Export helpers: reference AoS layout.
__global__ void k_export_tree(KgmtDev d, float* samples, float* costs) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < d.M; i += gridDim.x * blockDim.x) {
        const float4 s = d.treeState[i];
        const float4 c = d.treeCtrl[i];
        float* o = samples + (size_t)i * 7;
        o[0] = s.x; o[1] = s.y; o[2] = s.z; o[3] = s.w;
        o[4] = c.x; o[5] = c.y; o[6] = c.z;
        costs[i] = c.w;
    }
}

__global__ void k_export_unexplored(KgmtDev d, float* samples, int* uParent) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < d.nSlots; i += gridDim.x * blockDim.x) {
        const float4 s = d.uState[i];
        const float4 c = d.uCtrl[i];
        float* o = samples + (size_t)i * 7;
        o[0] = s.x; o[1] = s.y; o[2] = s.z; o[3] = s.w;
        o[4] = c.x; o[5] = c.y; o[6] = c.z;
        uParent[i] = __float_as_int(c.w);
    }
}

// ------------------------------------------------------------------ launchers
void launch_expand(const KgmtDev& d, int t, int agent, int blocks, hipStream_t s) {
    if (agent == 0)
        hipLaunchKernelGGL(k_expand<0>, dim3(blocks), dim3(kBlock), 0, s, d, t);
    else
        hipLaunchKernelGGL(k_expand<1>, dim3(blocks), dim3(kBlock), 0, s, d, t);
}

void launch_plan(const KgmtDev& d, int t, hipStream_t s) {
    hipLaunchKernelGGL(k_plan, dim3(1), dim3(1024), 0, s, d, t);
}

void launch_insert(const KgmtDev& d, int t, int blocks, hipStream_t s) {
    hipLaunchKernelGGL(k_insert, dim3(blocks), dim3(kBlock), 0, s, d, t);
}

void launch_fill_i32(int* p, int v, long long n, hipStream_t s) {
    if (n <= 0) return;
    const int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill_i32, dim3(blocks), dim3(256), 0, s, p, v, n);
}

void launch_fill_f32(float* p, float v, long long n, hipStream_t s) {
    if (n <= 0) return;
    const int blocks = (int)std::min<long long>((n + 255) / 256, 4096);
    hipLaunchKernelGGL(k_fill_f32, dim3(blocks), dim3(256), 0, s, p, v, n);
}

void launch_init_slots(const KgmtDev& d, const Xorwow& base, const uint32_t* jumps, int nbits, int blocks,
                       hipStream_t s) {
    hipLaunchKernelGGL(k_init_slots, dim3(blocks), dim3(kBlock), 0, s, d, base, jumps, nbits);
}

void launch_seed_root(const KgmtDev& d, float4 rs, float4 rc, int r1, int r2, hipStream_t s) {
    hipLaunchKernelGGL(k_seed_root, dim3(1), dim3(64), 0, s, d, rs, rc, r1, r2);
}

void launch_export_tree(const KgmtDev& d, float* samples, float* costs, hipStream_t s) {
    hipLaunchKernelGGL(k_export_tree, dim3(1024), dim3(256), 0, s, d, samples, costs);
}

void launch_export_unexplored(const KgmtDev& d, float* samples, int* uParent, hipStream_t s) {
    hipLaunchKernelGGL(k_export_unexplored, dim3(1024), dim3(256), 0, s, d, samples, uParent);
}

}  // namespace sbmp
