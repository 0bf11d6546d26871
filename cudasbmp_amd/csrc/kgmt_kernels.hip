// kgmt_kernels.hip — hand-written gfx950 kernels of the KGMT iteration.
//
// One reference iteration (reference src/planners/KGMT.cu:118-292) becomes two
// kernels on one stream, with no host round trip:
//   k_expand(t)  : propagateG / propagateGV2 (KGMT.cu:341-482) fused with
//                  propagateAndCheck + isMotionValid (statePropagator.cu:5-76,
//                  collisionCheck.cu:6-28), region binning and the accept test.
//                  One thread per child slot, wave64 ballot -> GNew bitmask and a
//                  GNew popcount per 256-slot block.
//   k_finish(t)  : blocks 1..: exclusive_scan(GNew) + findInd + updateG
//                  (KGMT.cu:222-245,540-593) — each block sums the popcounts of
//                  the blocks before it, appends its accepted children in slot
//                  order, tests the goal and applies the partial GNew clear (D6);
//                  block 0, concurrently: folds the region deltas and prepares
//                  iteration t+1 (frontier/batch decision KGMT.cu:139-188,
//                  updateR1 KGMT.cu:485-538).
// The reference's O(M) G scan + findInd disappears: every frontier node is
// expanded each iteration and new rows are appended contiguously, so G is
// always the row range [gLo, treeSize) (parity-tested against the oracle,
// which keeps the literal boolean scans).
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include "kgmt_device.h"
#include "kgmt_launch.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace sbmp {

// ------------------------------------------------------------------ helpers
// a / b for 0 <= a < 2^24 (kFastDivMax), 1 <= b: float estimate (relative error
// < 2^-21, so off by at most 1 for a < 2^24) + exact integer correction of up to 2
// steps (tests/test_fast_division.py checks the bound on the host).  Larger slot
// counts take the exact integer division (slot_div, a uniform branch).
__device__ __forceinline__ int div_small(int a, int b) {
    int q = (int)((float)a * __builtin_amdgcn_rcpf((float)b));
    int r = a - q * b;
    if (r < 0) { --q; r += b; }
    if (r < 0) { --q; r += b; }
    if (r >= b) { ++q; r -= b; }
    if (r >= b) { ++q; }
    return q;
}

// slot = g * k + i -> g.  nSlots is a per-plan constant, so the branch is uniform.
__device__ __forceinline__ int slot_div(const KgmtDev& d, int slot, int k) {
    if (k == 32) return slot >> 5;
    return (d.nSlots <= kFastDivMax) ? div_small(slot, k) : slot / k;
}

// The 64-B control block of one iteration with ONE scalar load: a read through the
// constant address space (4), which the compiler lowers to s_load_dwordx16.  A
// vector load would wait with vmcnt(0) behind every older vector load (XORWOW
// states, snapshot words), which serialised the prologue; a scalar load waits on
// lgkmcnt only.  The fields read here are written by the previous launch; this
// launch writes only .executed, which it never reads.  The goal status (written by
// earlier launches only) comes with it.
typedef int sbmp_i32x16 __attribute__((ext_vector_type(16)));
typedef const __attribute__((address_space(4))) sbmp_i32x16 sbmp_const_i32x16;
typedef const __attribute__((address_space(4))) int sbmp_const_i32;
__device__ __forceinline__ IterCtrl load_ctrl(const IterCtrl* p, const PlannerStatus* st, int* goalIdx) {
    const sbmp_i32x16 v = *(sbmp_const_i32x16*)p;   // C cast: address-space casts are not reinterpret_casts
    *goalIdx = *(sbmp_const_i32*)st;
    IterCtrl c;
    c.run = v[0];
    c.executed = v[1];
    c.treeSize = v[2];
    c.gLo = v[3];
    c.nG = v[4];
    c.k = v[5];
    c.nExp = v[6];
    c.S = v[7];
    c.H = v[8];
    c.A = v[9];
    c.scoreBuf = v[10];
    return c;
}

__device__ __forceinline__ int wave_sum(int v) {
#pragma unroll
    for (int off = kWave / 2; off > 0; off >>= 1) v += __shfl_xor(v, off, kWave);
    return v;
}

// A record of a peer rank (or of this device, same code): system-scope loads bypass
// this GPU's caches, which may hold lines of the same parity buffer from two
// iterations ago.
__device__ __forceinline__ float4 load_record(const float4* p) {
    unsigned long long* q = const_cast<unsigned long long*>(reinterpret_cast<const unsigned long long*>(p));
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return make_float4(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)),
                       __uint_as_float((uint32_t)b), __uint_as_float((uint32_t)(b >> 32)));
}

// The same two forms for a global-address-space pointer (sharded k_step lists).
__device__ __forceinline__ float4 load_record_g(const SBMP_GAS float4* p) {
    const SBMP_GAS unsigned long long* q = reinterpret_cast<const SBMP_GAS unsigned long long*>(p);
    const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const unsigned long long b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    return make_float4(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)),
                       __uint_as_float((uint32_t)b), __uint_as_float((uint32_t)(b >> 32)));
}
__device__ __forceinline__ void store_record_g(SBMP_GAS float4* p, float4 v) {
    SBMP_GAS unsigned long long* q = reinterpret_cast<SBMP_GAS unsigned long long*>(p);
    __hip_atomic_store(q, ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + 1, ((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// ------------------------------------------------------------------ expand
// A sharded record word pair, stored through to memory (peers read it over xGMI).
__device__ __forceinline__ void store_record(float4* p, float4 v) {
    unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
    __hip_atomic_store(q, ((unsigned long long)__float_as_uint(v.y) << 32) | __float_as_uint(v.x), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + 1, ((unsigned long long)__float_as_uint(v.w) << 32) | __float_as_uint(v.z),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// One thread per child slot, 256-slot workgroups.  Outputs: child state/controls/
// parent (2 x 16 B), XORWOW state (16 + 8 B), GNew bits (one 8-B word per wave),
// the GNew popcount of the workgroup, and the region bookkeeping of
// KGMT.cu:392-411 (D3: in-grid cells only):
//   R1 counts   workgroup-private packed LDS counters (valid | invalid << 16), one
//               64-bit device atomic per touched cell;
//   R2New       availability bits of cells seen valid while unavailable in the
//               snapshot: an LDS bitmask, one device atomicOr per nonzero word;
//   R2 counts   one 16-bit key (r2 | valid << 15) per child into the key log, folded
//               into R2Valid / R2Invalid every kFoldEvery iterations (k_fold_r2).
//               Siblings scatter over ~150 distinct R2 cells per workgroup, and
//               scattered device atomics run ~17x below the contiguous rate
//               (MI355X_MICROARCH.md, global atomics); nothing reads these two
//               arrays during the run (KGMT.cu:405,410 are write-only).
template <int AGENT, int OBS>
__global__ __launch_bounds__(kBlock) void k_expand(KgmtDev d, int t) {
    extern __shared__ float4 sObs[];
    __shared__ float sScore[kMaxR1];
    __shared__ int sR1P[kMaxR1];
    __shared__ uint32_t sSnap[kMaxR2Words];   // R2 availability at the iteration start (D2)
    __shared__ uint32_t sNew[kMaxR2Words];
    __shared__ int sWaveCnt[kBlock / kWave];

    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid >> 6;
    long long* const tl = (d.timeline && t == d.timelineIter)
                              ? d.timeline + ((size_t)blockIdx.x * (kBlock / kWave) + wave) * kTimelineStamps
                              : nullptr;
    // Stamps stay in registers and are stored once at the exit: a store in the middle
    // would add vmcnt waits of its own (and alias every later load).
    long long stamp[kTimelineStamps] = {0, 0, 0, 0, 0, 0, 0, 0};
#define SBMP_STAMP(i)                                                                  \
    do {                                                                               \
        if (tl) stamp[i] = (long long)__builtin_amdgcn_s_memrealtime();                \
    } while (0)
    SBMP_STAMP(0);
    constexpr bool kLdsObs = (OBS == kObsLds || OBS == kObsLds4);
    constexpr int kRegObs = obs_in_registers(OBS);
    float4 ro[kRegObs > 0 ? kRegObs : 1];   // register-resident obstacle list
#pragma unroll
    for (int i = 0; i < kRegObs; ++i) ro[i] = d.obstacles[i];
    const int gblock = d.rank + d.nranks * (int)blockIdx.x;   // block-cyclic slot ownership
    const int slot = gblock * kBlock + tid;
    const int nW = d.nR2 >> 5;

    // Latency: every load that does not depend on the control block is issued
    // before it (slot arrays are allocated to a whole number of workgroups; the
    // score buffer of iteration t is t & 1); the control block is one scalar load;
    // the parent-row load and the active slots' XORWOW states follow it directly
    // (both are needed only when propagation starts; slots in [S, H) read nothing).
    const unsigned long long oldWord = (lane == 0) ? d.gnewOut[slot >> 6] : 0ull;   // this rank's own words
    const float scoreReg = (tid < d.nR1) ? d.R1Score[(t & 1) * d.nR1 + tid] : 0.0f;
    const float4 obsReg = (kLdsObs && tid < d.nObs) ? d.obstacles[tid] : make_float4(0.f, 0.f, 0.f, 0.f);
    uint32_t snapReg[kMaxR2Words / kBlock];
#pragma unroll
    for (int j = 0; j < kMaxR2Words / kBlock; ++j) snapReg[j] = (tid + j * kBlock < nW) ? d.R2Snap[tid + j * kBlock] : 0u;

    int goalIdx;
    const IterCtrl c = load_ctrl(d.ctrl + t, d.status, &goalIdx);
    if (!c.run || goalIdx != kNoGoal) return;   // grid-uniform
    if (blockIdx.x == 0 && threadIdx.x == 0) d.ctrl[t].executed = 1;
    if (gblock * kBlock >= c.H) return;   // past every batch and every stale bit (workgroup-uniform)

    // Parent row, unconditional (inactive slots read row 0, which always exists): a
    // load inside a branch makes the compiler wait with vmcnt(0) at the join, i.e.
    // for this load too before the LDS set-up below.
    const bool act = slot < c.S;
    const int g = !act ? 0 : slot_div(d, slot, c.k);   // slot = g*k + i
    const int parent = act ? c.gLo + g : 0;
    const float4 p = d.treeState[parent];
    const uint4 ra = load_rng_a(d.rngA, slot, c.S);   // act == slot < S
    const uint2 rb = load_rng_b(d.rngB, slot, c.S);

    if (tid < d.nR1) sScore[tid] = scoreReg;
    sR1P[tid] = 0;   // nR1 == kBlock
#pragma unroll
    for (int j = 0; j < kMaxR2Words / kBlock; ++j) {
        if (tid + j * kBlock < nW) {
            sSnap[tid + j * kBlock] = snapReg[j];
            sNew[tid + j * kBlock] = 0u;
        }
    }
    if (kLdsObs) {
        if (tid < d.nObs) sObs[tid] = obsReg;
        for (int i = tid + kBlock; i < d.nObs; i += kBlock) sObs[i] = d.obstacles[i];
    }
    __syncthreads();
    SBMP_STAMP(1);
    const float4* obs = (kRegObs > 0) ? ro : kLdsObs ? sObs : d.obstacles;

    bool accept = false;
    float4 cs = make_float4(0.f, 0.f, 0.f, 0.f), cc = cs;   // this slot's child (state, ctrl): the packed record
    // Register lists, car: k_step's fast loop (round 6; the per-step box schedule, the
    // separation-metric box tests, Cody-Waite alone where theta stays in range,
    // DESIGN.md §5.5), on every lane outside any divergent branch: lanes past S propagate
    // row 0 with the zero state the exact-size buffer gave them, and their result is
    // dropped (nothing of theirs is stored).  Other forms: the exec-masked car_euler.
    Xorwow rs{ra.x, ra.y, ra.z, ra.w, rb.x, rb.y};
    ChildOut out;
    bool valid = false, fast = false;
    if constexpr (AGENT == 0 && kRegObs > 0) {
        fast = car_fast_ok(d);   // per plan (uniform)
        if (fast) {
            const ChildCtl ctl = draw_controls<0>(rs, d);
            // box (lane % n) for the schedule: a load of its own (indexing ro[] by lane would put
            // the register list in scratch)
            const float4 oLane = G(d.obstacles)[lane % kRegObs];
            const StepSched sched = car_schedule<OBS>(p, parent, act, d, oLane);
            WaveCull cull{~0u, true};   // the schedule covers the whole reach
            if (!sched.valid) cull = car_cull<OBS>(p, ctl, d, obs);
            if (__ballot(!car_theta_bounded(p, ctl, d)) != 0ull)   // rare: Payne-Hanek per lane
                valid = car_euler_fast<OBS, true>(p, ctl, d, obs, cull, sched, out) && act;
            else if (d.invAgentLength == 1.0f)
                valid = car_euler_fast<OBS, false, true>(p, ctl, d, obs, cull, sched, out) && act;
            else
                valid = car_euler_fast<OBS, false>(p, ctl, d, obs, cull, sched, out) && act;
        }
    }
    if (act) {
        if (!fast)
            valid = (AGENT == 0) ? propagate_car<OBS>(p, rs, d, obs, out) : propagate_point<OBS>(p, rs, d, obs, out);
        SBMP_STAMP(2);
        int r1, r2;
        bins_k(out.state.x, out.state.y, d, &r1, &r2);   // getR1 / getR2 (KGMT.cu:390-391), N = 16
        if (valid) {
            const float u = xorwow_uniform(rs);   // KGMT.cu:395
            if (r2 >= 0) {                        // r2 >= 0 implies r1 >= 0
                const uint32_t bit = 1u << (r2 & 31);
                const bool r2Avail = sSnap[r2 >> 5] & bit;
                accept = (u <= sScore[r1]) || !r2Avail;
                if (!r2Avail) atomicOr(&sNew[r2 >> 5], bit);
            }
        }
        cs = out.state;
        cc = make_float4(out.a, out.steer, out.dur, __int_as_float(parent));
        store_wt(d.uState, slot, cs);   // write-through: fewer dirty lines at the boundary
        store_wt(d.uCtrl, slot, cc);
        store_wt(d.rngA, slot, make_uint4(rs.v0, rs.v1, rs.v2, rs.v3));
        store_wt(d.rngB, slot, make_uint2(rs.v4, rs.d));
        if (r1 >= 0) atomicAdd(&sR1P[r1], valid ? 1 : 0x10000);
        if (d.r2log) {
            d.r2log[(size_t)(t % kFoldEvery) * d.logSlots + (int)blockIdx.x * kBlock + tid] =
                (r2 >= 0) ? (uint16_t)(r2 | (valid ? 0x8000 : 0)) : kNoKey;
        } else if (r2 >= 0) {   // more than kLogMaxR2 R2 cells: direct device atomics
            atomicAdd(valid ? &d.R2Valid[r2] : &d.R2Invalid[r2], 1);
        }
    }
    SBMP_STAMP(3);
    // GNew |= accept (stale bits survive, D6).  A wave covers one 64-bit word; it is
    // always written (a sharded rank's Out word must carry its stale bits too).
    const unsigned long long mask = __ballot(accept);
    if (lane == 0) {
        const unsigned long long now = oldWord | mask;
        d.gnewOut[slot >> 6] = now;
        sWaveCnt[wave] = __popcll(now);   // slots past S: the stale bits' count
    }
    SBMP_STAMP(4);
    __syncthreads();
    SBMP_STAMP(5);
    const int cntB = sWaveCnt[0] + sWaveCnt[1] + sWaveCnt[2] + sWaveCnt[3];
    if (tid == 0) d.blockCountOut[gblock] = cntB;
    {   // one 64-bit atomic per touched cell, into this workgroup's replica
        unsigned long long* const rep = d.deltaOut + (size_t)(blockIdx.x % kDeltaReps) * d.nR1;
        const int v = sR1P[tid];   // nR1 == kBlock
        if (v) atomicAdd(&rep[tid], (unsigned long long)(v & 0xffff) | ((unsigned long long)(v >> 16) << 32));
    }
    for (int i = tid; i < nW; i += kBlock) {   // R2New as one byte per cell (sums merge ranks)
        uint32_t w = sNew[i];
        while (w) {
            const int b = __builtin_ctz(w);
            w &= w - 1u;
            d.r2newOut[32 * i + b] = 1;
        }
    }
    SBMP_STAMP(6);
    if (tl) {   // placement: XCC id << 32 | HW_ID (wave, SIMD, CU, SE fields)
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        stamp[7] = ((long long)xcc << 32) | hw;
    }
    if (tl && lane == 0)
        for (int i = 0; i < kTimelineStamps; ++i) tl[i] = stamp[i];
#undef SBMP_STAMP
}

// R2Valid / R2Invalid (KGMT.cu:405,410) from the key log of iteration
// tFirst + blockIdx.y: a dense LDS histogram per workgroup (packed valid |
// invalid << 16; a workgroup takes at most kFoldKeys < 2^16 keys, so neither half
// overflows), flushed with one atomic per nonzero half, consecutive lanes on
// consecutive cells.  Keys of slots >= S of that iteration are stale and skipped;
// iterations that did not execute are skipped whole.
// Where the time goes (round 5, -DSBMP_TIMELINE stamps, tools/fold_timeline.py): the
// adds are VALU-bound, not LDS-bound (64 keys per thread, 16 waves per CU; at ~10 VALU
// per key the adds took 3-4.5 us, against ~1 us of LDS time at the random-word rate of
// tools/microbench/lds_atomic_bench), so each key is now 5 VALU: the cell and the
// increment by shifts, masks and one multiply-add, and the skipped keys (kNoKey, or a
// slot >= S, which the rare piece that straddles S turns into kNoKey) sent by one min
// to a per-lane sink word past the histogram: no branch, no compare per key.  All of a
// thread's key loads issue at entry (one round trip, not one per 16 B) and the
// histogram is cleared while the control block's scalar load is in flight.
constexpr int kFoldThreads = 1024;
constexpr int kFoldLoads = (kFoldKeys + 8 * kFoldThreads - 1) / (8 * kFoldThreads);   // 16-B pieces per thread
// The histogram is the kernel's only LDS (dynamic, so at LDS address 0): the add takes
// the byte offset itself (the compiler added the base, 0, in one more VALU per key).
// Its completion is waited for explicitly before the barrier that ends the adds.
__device__ __forceinline__ void fold_add(uint32_t key, uint32_t sinkB) {
    // byte offset of cell (key & 0x7fff), or the sink for kNoKey (cell 0x7fff >= nR2)
    const uint32_t a = __builtin_elementwise_min((key & 0x7fffu) << 2, sinkB);
    const uint32_t valid = key >> 15;   // 0 or 1
    const uint32_t inc = 0x10000u - valid * 0xffffu;   // valid: 1, invalid: 1 << 16
    asm volatile("ds_add_u32 %0, %1" : : "v"(a), "v"(inc) : "memory");
}
__global__ __launch_bounds__(kFoldThreads) void k_fold_r2(KgmtDev d, int tFirst, int keysPerGroup) {
    extern __shared__ uint32_t sCnt[];   // nR2 cells, then kWave sink words
    const int tid = (int)threadIdx.x;
    const int t = tFirst + (int)blockIdx.y;
    const uint16_t* row = d.r2log + (size_t)(t % kFoldEvery) * d.logSlots;
    const int begin = (int)blockIdx.x * keysPerGroup;
    const int end = min(begin + keysPerGroup, d.logSlots);
    uint4 w[kFoldLoads];
#pragma unroll
    for (int u = 0; u < kFoldLoads; ++u) {
        const int i = begin + (tid + u * kFoldThreads) * 8;
        w[u] = (i < end) ? *reinterpret_cast<const uint4*>(row + i) : make_uint4(~0u, ~0u, ~0u, ~0u);
    }
#ifdef SBMP_TIMELINE   // diagnostics (tools/fold_timeline.py): the fold of iteration timelineIter, wave by wave
    // rows 9.. of the k_step stamp rows (0: planner, 1-8: exchange workers), where they fit
    const int ftlRow = 9 + (int)blockIdx.x * (kFoldThreads / kWave) + (tid >> 6);
    long long* const ftl = (d.timelineFin && t == d.timelineIter && (tid & (kWave - 1)) == 0 && ftlRow < 1 + d.nBlocks)
                               ? d.timelineFin + (size_t)ftlRow * kTimelineStamps : nullptr;
#define SBMP_FSTAMP(k) do { if (ftl) ftl[k] = (long long)__builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define SBMP_FSTAMP(k) do { } while (0)
#endif
    SBMP_FSTAMP(0);
    const IterCtrl c = d.ctrl[t];   // (the clear below overlaps its round trip)
    const int nR2 = d.nR2;
    for (int i = tid; i < nR2 + kWave; i += kFoldThreads) sCnt[i] = 0u;
    if (!c.executed) return;   // uniform
    SBMP_FSTAMP(1);
    __syncthreads();
    SBMP_FSTAMP(2);
#ifdef SBMP_TIMELINE
    if (ftl) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        SBMP_FSTAMP(3);
    }
#endif
    const uint32_t sinkB = (uint32_t)(nR2 + (tid & (kWave - 1))) * 4u;
#pragma unroll
    for (int u = 0; u < kFoldLoads; ++u) {
        const int i = begin + (tid + u * kFoldThreads) * 8;
        const int live = c.S - (d.rank + d.nranks * (i >> 8)) * kBlock - (i & (kBlock - 1));   // keys of slots < S
        uint32_t kw[4] = {w[u].x, w[u].y, w[u].z, w[u].w};
        if (live < 8) {   // the piece that straddles S (or lies past it): its stale keys become kNoKey
#pragma unroll
            for (int k = 0; k < 4; ++k)
                kw[k] |= (2 * k >= live ? 0xffffu : 0u) | (2 * k + 1 >= live ? 0xffff0000u : 0u);
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            fold_add(kw[k] & 0xffffu, sinkB);
            fold_add(kw[k] >> 16, sinkB);
        }
    }
    SBMP_FSTAMP(4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // the adds (inline asm: not tracked)
    __syncthreads();
    SBMP_FSTAMP(5);
    for (int i0 = tid; i0 < nR2; i0 += 8 * kFoldThreads) {   // 8 cells read, then their atomics
        uint32_t v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = (i0 + q * kFoldThreads < nR2) ? sCnt[i0 + q * kFoldThreads] : 0u;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            if (v[q] & 0xffffu) atomicAdd(&d.R2Valid[i0 + q * kFoldThreads], (int)(v[q] & 0xffffu));
            if (v[q] >> 16) atomicAdd(&d.R2Invalid[i0 + q * kFoldThreads], (int)(v[q] >> 16));
        }
    }
#ifdef SBMP_TIMELINE
    if (ftl) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        SBMP_FSTAMP(6);
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        ftl[7] = ((long long)xcc << 32) | hw;
    }
#endif
#undef SBMP_FSTAMP
}

// ------------------------------------------------------------------ finish
// Batch decision for iteration t (KGMT.cu:151-158 + the capped / fill extensions).
__device__ __forceinline__ void batch_rule(const KgmtDev& d, int treeSize, int nG, int* k, int* nExp) {
    *k = 0;
    *nExp = 0;
    if (nG <= 0) return;   // D7: a zero-block launch is a no-op
    // Both callers run it only while treeSize < M (KGMT.cu:255), so the room left is in
    // [1, M - 1] and everything below is 32-bit scalar arithmetic (gfx9's scalar unit has
    // no 64-bit ordered compare: the 64-bit form went through VALU compares and moves on
    // the plan's critical path, which every expanding wave waits for).
    int remaining = d.M - treeSize;
    if (d.cap > 0 && remaining > d.cap) remaining = d.cap;
    if (d.cap > 0 && d.batchRule == 1) {   // D14: fill the batch
        if (nG <= remaining) {
            *k = (remaining < kFastDivMax) ? div_small(remaining, nG) : remaining / nG;
            *nExp = nG;
        } else {
            *k = 1;
            *nExp = remaining;
        }
    } else if (nG <= (remaining >> 5)) {   // 32 nG <= remaining, exactly (remaining >= 0)
        *k = 32;
        *nExp = nG;
    } else {
        *k = (int)((float)remaining / (float)nG);   // KGMT.cu:157
        *nExp = nG;
        if (d.cap > 0 && *k == 0) {
            *k = 1;
            *nExp = (int)remaining;
        }
    }
}

#define SBMP_FIN_STAMP(i)                                                    \
    do {                                                                     \
        if (st) st[i] = (long long)__builtin_amdgcn_s_memrealtime();         \
    } while (0)

// Close iteration t-1 (accepted count, region deltas) and prepare iteration t:
// frontier range, batch, updateR1 (KGMT.cu:485-538), availability snapshot.
// Runs in block 0 of k_finish(t-1), concurrently with that launch's insert blocks
// (it reads only what k_expand(t-1) wrote and nothing the insert blocks write).
// It is the critical path of k_finish, so every load (all of them independent:
// one R1 cell and up to kMaxR2Words / kBlock availability words per thread) is
// issued at entry and the tables are updated in registers: one memory round trip
// instead of six.  Block counts at or past the high-water block are zero (H never
// decreases), so the accepted count is the sum over all blocks.
__device__ void plan_iteration(const KgmtDev& d, int t, long long* st) {
    __shared__ int sRed[3][kBlock / kWave];
    __shared__ int sCovInc[kMaxR1];
    __shared__ float sPart[8];
    constexpr int kW = kMaxR2Words / kBlock;

    const int tid = threadIdx.x;
    const int cell = min(tid, d.nR1 - 1);   // nR1 <= kMaxR1 == kBlock: one R1 cell per thread
    const bool own = tid < d.nR1;
    const int nn = d.n * d.n;
    const int nR2w = d.nR2 >> 5;
    // ---- loads
    const IterCtrl pc = d.ctrl[t > 1 ? t - 1 : 0];
    int cnt = 0;
    const int pfxTotal = d.pfxIn ? d.pfxIn[d.nBlocks] : 0;   // sharded: the exchange carries the total
    if (!d.pfxIn) {
        for (int i = tid * 4; i < d.nBlocks; i += kBlock * 4) {   // counts are int4-readable
            const int4 v = *reinterpret_cast<const int4*>(d.blockCountIn + i);
            cnt += v.x + v.y + v.z + v.w;
        }
    }
    unsigned long long dv[kDeltaReps];
#pragma unroll
    for (int r = 0; r < kDeltaReps; ++r) dv[r] = d.deltaIn[(size_t)r * d.nR1 + cell];
    int r1 = d.R1[cell], r1v = d.R1Valid[cell], r1i = d.R1Invalid[cell], r1a = d.R1Avail[cell], r1c = d.R1Cov[cell];
    uint32_t bits[kW];
    uint4 nb0[kW], nb1[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) {
        const int w = min(tid + j * kBlock, nR2w - 1);
        if (j * kBlock < nR2w) {   // uniform
            bits[j] = d.R2Avail[w];
            const uint4* nb = reinterpret_cast<const uint4*>(d.r2newIn + 32 * w);   // 32 cells, one byte each
            nb0[j] = nb[0];
            nb1[j] = nb[1];
        }
    }

    const bool ranPrev = (t > 1) && pc.executed;
    if (t > 1 && !ranPrev) {
        if (tid == 0) d.ctrl[t].run = 0;
        return;
    }
    sCovInc[tid] = 0;
    int A = 0;
    if (ranPrev && !d.pfxIn) {   // accepted children of iteration t-1
        const int wsum = wave_sum(cnt);
        if ((tid & (kWave - 1)) == 0) sRed[0][tid >> 6] = wsum;
    }
    __syncthreads();
    if (ranPrev) A = d.pfxIn ? pfxTotal : sRed[0][0] + sRed[0][1] + sRed[0][2] + sRed[0][3];
    SBMP_FIN_STAMP(1);

    // ---- fold the previous expansion's region deltas (t == 1: all zero)
    unsigned long long dl = 0ull;   // replicas: carry-free sums
#pragma unroll
    for (int r = 0; r < kDeltaReps; ++r) dl += dv[r];
    const int nv = (int)(dl & 0xffffffffull), ni = (int)(dl >> 32);
    r1 += nv + ni;      // every in-grid child (KGMT.cu:392)
    r1v += nv;          // KGMT.cu:406
    r1i += ni;          // KGMT.cu:409
    if (nv) r1a = 1;    // KGMT.cu:399-401
    // ---- R2 availability: cells seen valid while unavailable (KGMT.cu:396-402).
    // All words are decided before any is stored: a store ahead of a later word's
    // loaded data would make that use wait for the store as well (vmcnt is in order).
    uint32_t nws[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) {
        const int w = tid + j * kBlock;
        nws[j] = 0u;
        if (j * kBlock < nR2w && w < nR2w) {
            const uint32_t q[8] = {nb0[j].x, nb0[j].y, nb0[j].z, nb0[j].w, nb1[j].x, nb1[j].y, nb1[j].z, nb1[j].w};
            uint32_t nw = 0u;
#pragma unroll
            for (int k = 0; k < 8; ++k) {   // nonzero bytes -> 4 bits (byte sums <= nranks never carry)
                const uint32_t hi = (((q[k] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | q[k]) & 0x80808080u;
                nw |= ((((hi >> 7) * 0x00204081u) >> 21) & 0xfu) << (4 * k);
            }
            nws[j] = nw;
            uint32_t fresh = nw & ~bits[j];
            if (fresh && nn % 32 == 0) {   // the 32 cells of a word lie in one R1 cell
                atomicAdd(&sCovInc[(32 * w) / nn], __popc(fresh));
            } else {
                while (fresh) {
                    const int k = __builtin_ctz(fresh);
                    fresh &= fresh - 1u;
                    atomicAdd(&sCovInc[(32 * w + k) / nn], 1);
                }
            }
        }
    }
#pragma unroll
    for (int j = 0; j < kW; ++j) {
        const int w = tid + j * kBlock;
        if (j * kBlock < nR2w && w < nR2w) {
            const uint32_t nw = nws[j], b = bits[j];
            if (nw) {
                uint4* ob = reinterpret_cast<uint4*>(d.r2newOut + 32 * w);
                ob[0] = make_uint4(0u, 0u, 0u, 0u);
                ob[1] = make_uint4(0u, 0u, 0u, 0u);
                if (nw & ~b) d.R2Avail[w] = b | nw;
            }
            d.R2Snap[w] = b | nw;   // snapshot for the next expand (D2)
        }
    }
    __syncthreads();
    r1c += sCovInc[cell];
    if (own) {
#pragma unroll
        for (int r = 0; r < kDeltaReps; ++r) d.deltaOut[(size_t)r * d.nR1 + cell] = 0ull;
        if (dl) {
            d.R1[cell] = r1;
            d.R1Valid[cell] = r1v;
            d.R1Invalid[cell] = r1i;
            d.R1Avail[cell] = r1a;
        }
        if (sCovInc[cell]) d.R1Cov[cell] = r1c;
    }
    SBMP_FIN_STAMP(2);

    int treeSize = 1, gLo = 0, H = 0;
    if (ranPrev) {
        H = pc.H;
        treeSize = pc.treeSize + A;   // KGMT.cu:249
        gLo = pc.gLo + pc.nExp;
        if (tid == 0) d.ctrl[t - 1].A = A;
    }
    const int run_t = (t <= d.numIterations) && (treeSize < d.M);   // KGMT.cu:118,255
    int nG = 0, k = 0, nExp = 0;
    if (run_t) {
        nG = treeSize - gLo;
        batch_rule(d, treeSize, nG, &k, &nExp);
    }
    const int S = k * nExp;
    const int buf = t & 1;
    if (run_t) {   // updateR1 for iteration t
        float sc = 0.0f;
        if (r1a != 0) {
            const float covR = (float)r1c / (float)nn;
            const float freeVol = (0.01f + (float)r1v) / (0.01f + (float)r1v + (float)r1i);
            const float fv2 = freeVol * freeVol;
            const float fv4 = fv2 * fv2;
            const double r = (double)r1;
            const double den = (double)(1.0f + covR) * (1.0 + r * r);
            sc = (float)((double)fv4 / den);
        }
        // CUB BlockReduce order (D8): a shuffle-down tree (offsets 1, 2, 4, 8, 16) per
        // 32-lane group, then the 8 group sums in order.
        float v = own ? sc : 0.0f;
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) {
            const float o = __shfl_down(v, off, 32);
            v = v + o;
        }
        if ((tid & 31) == 0) sPart[tid >> 5] = v;
        __syncthreads();
        float tsum = sPart[0];
#pragma unroll
        for (int w = 1; w < 8; ++w) tsum = tsum + sPart[w];
        const float total = tsum;
        SBMP_FIN_STAMP(3);
        if (own) d.R1Score[buf * d.nR1 + cell] = (r1a == 0) ? 1.0f : sc / total;
    }
    SBMP_FIN_STAMP(4);
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

// One 256-slot block of iteration t: the j-th accepted slot (global slot order)
// becomes row treeSize + j (findInd + updateG, KGMT.cu:225-245,540-593), goal test,
// partial GNew clear (D6).  The block's j offset is the sum of the GNew counts of
// the blocks before it (counts written by k_expand(t)).
__device__ void insert_block(const KgmtDev& d, int t, int gblock, long long* st) {
    __shared__ int sRed[2][kBlock / kWave];
    __shared__ int sWaveCnt[kBlock / kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x >> 6;
    const int w = gblock * (kBlock / kWave) + wave;
    const int slot = w * kWave + lane;
    // Every load that depends on nothing else is issued first: the flag word, the
    // block counts (the first 1,024 as one int4 per thread; counts at or past the
    // high-water block were never written and are zero) and the control block.
    const unsigned long long word = d.gnewIn[w];
    const int myCount = d.blockCountIn[gblock];
    const int nb4 = (d.nBlocks + 3) & ~3;
    const int i0 = min((int)threadIdx.x * 4, nb4 - 4);
    const int4 c0 = *reinterpret_cast<const int4*>(d.blockCountIn + i0);
    const IterCtrl c = d.ctrl[t];
    if (!c.executed) return;
    if (gblock * kBlock >= c.H) return;
    if (myCount == 0) return;   // no accepted (or stale) slot: nothing to insert or clear
    SBMP_FIN_STAMP(1);
    // The flagged lanes' children (this XCD wrote them, see k_finish), in flight
    // while the prefix is reduced.
    const bool flagged = (word >> lane) & 1ull;
    float4 us = make_float4(0.f, 0.f, 0.f, 0.f), uc = us;
    if (flagged) {
        us = d.uState[slot];
        uc = d.uCtrl[slot];
    }
    // exclusive prefix of this block and the total, over the block counts
    int p = 0, tot = 0;
    if ((int)threadIdx.x * 4 < nb4) {
        const int e[4] = {c0.x, c0.y, c0.z, c0.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            tot += e[k];
            p += (i0 + k < gblock) ? e[k] : 0;
        }
    }
    for (int i = (int)threadIdx.x * 4 + kBlock * 4; i < nb4; i += kBlock * 4) {   // more than 1,024 blocks
        const int4 v = *reinterpret_cast<const int4*>(d.blockCountIn + i);
        const int e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            tot += e[k];
            p += (i + k < gblock) ? e[k] : 0;
        }
    }
    p = wave_sum(p);
    tot = wave_sum(tot);
    if (lane == 0) {
        sRed[0][wave] = p;
        sRed[1][wave] = tot;
        sWaveCnt[wave] = __popcll(word);
    }
    __syncthreads();
    const int pre = sRed[0][0] + sRed[0][1] + sRed[0][2] + sRed[0][3];
    const int A = sRed[1][0] + sRed[1][1] + sRed[1][2] + sRed[1][3];
    SBMP_FIN_STAMP(2);
    int waveOff = pre;
    for (int i = 0; i < wave; ++i) waveOff += sWaveCnt[i];
    if (word == 0ull) return;

    const int m32 = d.M / 32;
    const int grid = min(A, m32);   // updateG launch: min(|GNew|, M/32) blocks of 32 (KGMT.cu:231)
    const int nIns = 32 * grid < A ? 32 * grid : A;
    if (flagged) {
        const int j = waveOff + __popcll(word & ((1ull << lane) - 1ull));
        const int dst = c.treeSize + j;
        if (j < nIns && dst < d.M) {   // D13: the reference writes past M here
            const int parent = __float_as_int(uc.w);
            const float cost = d.treeCtrl[parent].w + uc.z;   // getCost = duration (KGMT.cu:631-633)
            d.treeState[dst] = us;
            d.treeCtrl[dst] = make_float4(uc.x, uc.y, uc.z, cost);
            d.treeParent[dst] = parent;
            const float dx = us.x - d.goalX, dy = us.y - d.goalY;   // inGoalRegion, KGMT.cu:635-638
            const float d2 = dx * dx + dy * dy;
            if (__builtin_sqrtf(d2) < d.goalThreshold) atomicMin(&d.status->goalIdx, dst);
        }
    }
    SBMP_FIN_STAMP(3);
    if (lane == 0) {   // D6: only GNew[0 .. 32*grid) is cleared
        const long long cleared = d.fixGNewClear ? (1ll << 62) : 32ll * grid;
        const long long base = (long long)w * kWave;
        unsigned long long nw_ = word;
        if (base + kWave <= cleared) nw_ = 0ull;
        else if (base < cleared) nw_ = word & ~((1ull << (cleared - base)) - 1ull);
        if (nw_ != word) d.gnewIn[w] = nw_;
    }
}

// The same for iterations of more than 1,024 blocks (the two-launch form at c4 / c5's
// 1,048,576 children): insert workgroup w0 takes blocks w0 + r G (r < kInsertMaxR; G a
// multiple of 8, so every one of them ran on this workgroup's XCD in k_expand, whose
// L2 holds its slots) and reduces the block counts once for all of them.  One workgroup
// per block (insert_block) dispatched 4,096 workgroups that each re-read the 16-KB
// count array: k_finish 12.4 us at c4's 1,048,576 children, its insert workgroups
// entering over 8 us (profiles/r05/workloads/k_finish_c4_1M_iter20.txt).
#ifndef SBMP_INSERT_R
#define SBMP_INSERT_R 4
#endif
constexpr int kInsertMaxR = SBMP_INSERT_R;
__device__ void insert_blocks(const KgmtDev& d, int t, int w0, int G, long long* st) {
    __shared__ int sRed[kInsertMaxR + 1][kBlock / kWave];
    __shared__ int sWaveCnt[kInsertMaxR][kBlock / kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x >> 6;
    // every load that depends on nothing else first: the flag words, the control
    // block, the block counts
    int gb[kInsertMaxR];
    unsigned long long word[kInsertMaxR];
#pragma unroll
    for (int r = 0; r < kInsertMaxR; ++r) {
        gb[r] = w0 + r * G;
        word[r] = (gb[r] < d.nBlocks) ? d.gnewIn[gb[r] * (kBlock / kWave) + wave] : 0ull;
    }
    const IterCtrl c = d.ctrl[t];
    const int nb4 = (d.nBlocks + 3) & ~3;
    int p[kInsertMaxR] = {}, tot = 0;
#pragma unroll 4
    for (int i = (int)threadIdx.x * 4; i < nb4; i += kBlock * 4) {
        const int4 v = *reinterpret_cast<const int4*>(d.blockCountIn + i);
        const int e[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            tot += e[k];
#pragma unroll
            for (int r = 0; r < kInsertMaxR; ++r) p[r] += (i + k < gb[r]) ? e[k] : 0;
        }
    }
    if (!c.executed) return;   // uniform
    SBMP_FIN_STAMP(1);
    // the flagged lanes' children, in flight while the prefixes are reduced
    float4 us[kInsertMaxR], uc[kInsertMaxR];
    bool flagged[kInsertMaxR];
#pragma unroll
    for (int r = 0; r < kInsertMaxR; ++r) {
        if (gb[r] >= d.nBlocks || gb[r] * kBlock >= c.H) word[r] = 0ull;   // uniform: never ran
        flagged[r] = (word[r] >> lane) & 1ull;
        us[r] = uc[r] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (flagged[r]) {
            const int slot = gb[r] * kBlock + (int)threadIdx.x;
            us[r] = d.uState[slot];
            uc[r] = d.uCtrl[slot];
        }
    }
    tot = wave_sum(tot);
#pragma unroll
    for (int r = 0; r < kInsertMaxR; ++r) p[r] = wave_sum(p[r]);
    if (lane == 0) {
#pragma unroll
        for (int r = 0; r < kInsertMaxR; ++r) {
            sRed[r][wave] = p[r];
            sWaveCnt[r][wave] = __popcll(word[r]);
        }
        sRed[kInsertMaxR][wave] = tot;
    }
    __syncthreads();
    const int A = sRed[kInsertMaxR][0] + sRed[kInsertMaxR][1] + sRed[kInsertMaxR][2] + sRed[kInsertMaxR][3];
    SBMP_FIN_STAMP(2);
    const int m32 = d.M / 32;
    const int grid = min(A, m32);   // updateG launch: min(|GNew|, M/32) blocks of 32 (KGMT.cu:231)
    const int nIns = 32 * grid < A ? 32 * grid : A;
    const long long cleared = d.fixGNewClear ? (1ll << 62) : 32ll * grid;
#pragma unroll
    for (int r = 0; r < kInsertMaxR; ++r) {
        if (word[r] == 0ull) continue;   // uniform
        int waveOff = sRed[r][0] + sRed[r][1] + sRed[r][2] + sRed[r][3];
        for (int i = 0; i < wave; ++i) waveOff += sWaveCnt[r][i];
        if (flagged[r]) {
            const int j = waveOff + __popcll(word[r] & ((1ull << lane) - 1ull));
            const int dst = c.treeSize + j;
            if (j < nIns && dst < d.M) {   // D13: the reference writes past M here
                const int parent = __float_as_int(uc[r].w);
                const float cost = d.treeCtrl[parent].w + uc[r].z;   // getCost = duration (KGMT.cu:631-633)
                d.treeState[dst] = us[r];
                d.treeCtrl[dst] = make_float4(uc[r].x, uc[r].y, uc[r].z, cost);
                d.treeParent[dst] = parent;
                const float dx = us[r].x - d.goalX, dy = us[r].y - d.goalY;   // inGoalRegion, KGMT.cu:635-638
                const float d2 = dx * dx + dy * dy;
                if (__builtin_sqrtf(d2) < d.goalThreshold) atomicMin(&d.status->goalIdx, dst);
            }
        }
        if (lane == 0) {   // D6: only GNew[0 .. 32*grid) is cleared
            const int w = gb[r] * (kBlock / kWave) + wave;
            const long long base = (long long)w * kWave;
            unsigned long long nw_ = word[r];
            if (base + kWave <= cleared) nw_ = 0ull;
            else if (base < cleared) nw_ = word[r] & ~((1ull << (cleared - base)) - 1ull);
            if (nw_ != word[r]) d.gnewIn[w] = nw_;
        }
    }
    SBMP_FIN_STAMP(3);
}

// k_finish's insert workgroups for an iteration of nBlocks 256-slot blocks: one per
// block up to 1,024 blocks, else the fewest (a multiple of 8) that give each at most
// kInsertMaxR.
int finish_insert_groups(int nBlocks) {
    if (nBlocks <= 1024) return nBlocks;
    const int g = (nBlocks + kInsertMaxR - 1) / kInsertMaxR;
    return (g + 7) & ~7;
}

// Sharded ranks: iteration t's accepted (and stale, D6) children of
// every rank, record-driven.  The owners' record lists, concatenated in rank order,
// are walked with a grid-stride loop; record (block g, index i) becomes row
// treeSize + pfx[g] + i, its rank in global slot order.  The work is proportional
// to the accepted count, not to the number of slots or ranks.
__device__ void insert_records(const KgmtDev& d, int t, int wg, int nWG, long long* st) {
    const IterCtrl c = d.ctrl[t];
    if (!c.executed) return;
    int start[kMaxRanks + 1];
    start[0] = 0;
    for (int q = 0; q < d.nranks; ++q) start[q + 1] = start[q] + d.totIn[q];
    const int A = start[d.nranks];
    SBMP_FIN_STAMP(1);
    const int m32 = d.M / 32;
    const int grid = min(A, m32);   // updateG launch: min(|GNew|, M/32) blocks of 32 (KGMT.cu:231)
    const int nIns = 32 * grid < A ? 32 * grid : A;
    for (int i = wg * kBlock + (int)threadIdx.x; i < A; i += nWG * kBlock) {
        int q = 0;
        while (q + 1 < d.nranks && i >= start[q + 1]) ++q;
        const float4* rec = d.recPeer[q] + ((size_t)(t & 1) * d.recCap + (i - start[q])) * kRecordF4;
        const float4 s = load_record(rec);
        const float4 u = load_record(rec + 1);
        const float4 m = load_record(rec + 2);
        const int j = d.pfxIn[__float_as_int(m.x)] + __float_as_int(m.y);
        const int dst = c.treeSize + j;
        if (j < nIns && dst < d.M) {   // D13
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
    SBMP_FIN_STAMP(3);
}

// Sharded ranks: the D6 clear of GNew[0 .. 32*grid) on this rank's own words (owned
// block lb; no other rank keeps them).
__device__ void owner_clear(const KgmtDev& d, int t, int lb) {
    const int gblock = d.rank + d.nranks * lb;
    const IterCtrl c = d.ctrl[t];
    if (!c.executed || gblock * kBlock >= c.H) return;
    const int w = gblock * (kBlock / kWave) + (int)(threadIdx.x >> 6);
    if ((threadIdx.x & (kWave - 1)) != 0) return;
    const unsigned long long word = d.gnewOut[w];
    if (word == 0ull) return;
    const int A = d.pfxIn[d.nBlocks];
    const int grid = min(A, d.M / 32);
    const long long cleared = d.fixGNewClear ? (1ll << 62) : 32ll * grid;
    const long long base = (long long)w * kWave;
    unsigned long long nw_ = word;
    if (base + kWave <= cleared) nw_ = 0ull;
    else if (base < cleared) nw_ = word & ~((1ull << (cleared - base)) - 1ull);
    if (nw_ != word) d.gnewOut[w] = nw_;
}

// Sharded ranks: this rank's accepted (and stale, D6) children of iteration t in
// owned-slot order into record buffer t & 1, for the insert kernels of every rank.
// A block's position is the count over this rank's earlier blocks (local counts).
// The records are written through to memory (system-scope stores): peers read them
// over xGMI after the all-reduce that follows this kernel in stream order.  The
// block also fills its part of the exchange's prefix fields (KgmtDev::pfx / opfx):
// its owner-local offset, and this rank's share of the global prefix of every block
// up to its next owned block (the last active block: up to the total), so the
// all-reduce's sum hands every insert block its offset and the total in O(1).

__device__ __forceinline__ void pack_block(const KgmtDev& d, int t) {
    __shared__ int sRed[3][kBlock / kWave];
    __shared__ int sWaveCnt[kBlock / kWave];
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x >> 6;
    const int lb = (int)blockIdx.x;
    const int gblock = d.rank + d.nranks * lb;
    const IterCtrl c = d.ctrl[t];
    if (!c.executed || gblock * kBlock >= c.H) return;   // workgroup-uniform
    const int w = gblock * (kBlock / kWave) + wave;
    const unsigned long long word = d.gnewOut[w];
    int pre = 0;
    for (int i = threadIdx.x; i < lb; i += kBlock) pre += d.blockCountOut[d.rank + d.nranks * i];
    pre = wave_sum(pre);
    if (lane == 0) {
        sRed[0][wave] = pre;
        sWaveCnt[wave] = __popcll(word);
    }
    __syncthreads();
    const int preLocal = sRed[0][0] + sRed[0][1] + sRed[0][2] + sRed[0][3];
    int inBlock = 0;
    for (int i = 0; i < wave; ++i) inBlock += sWaveCnt[i];
    if ((word >> lane) & 1ull) {
        const int slot = w * kWave + lane;
        const int idx = inBlock + __popcll(word & ((1ull << lane) - 1ull));   // index within the block
        float4* rec = d.recOut + ((size_t)(t & 1) * d.recCap + preLocal + idx) * kRecordF4;
        store_record(rec, d.uState[slot]);
        store_record(rec + 1, d.uCtrl[slot]);
        store_record(rec + 2, make_float4(__int_as_float(gblock), __int_as_float(idx), 0.0f, 0.0f));
    }
    const int cnt = sWaveCnt[0] + sWaveCnt[1] + sWaveCnt[2] + sWaveCnt[3];
    const int next = gblock + d.nranks;   // H never decreases: blocks >= H never ran, entries past them are unused
    const bool last = (long long)next * kBlock >= c.H;
    const int hi = last ? d.nBlocks : min(next, d.nBlocks);
    for (int g = gblock + 1 + (int)threadIdx.x; g <= hi; g += kBlock)
        __hip_atomic_store(d.pfxOut + g, preLocal + cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (last && threadIdx.x == 0)
        __hip_atomic_store(d.totOut + d.rank, preLocal + cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__global__ __launch_bounds__(kBlock) void k_pack(KgmtDev d, int t) { pack_block(d, t); }

// Local shard group (P ranks on one device, one stream): the all-reduce of the
// exchange buffers as a sum kernel.
struct XsumArgs {
    const unsigned long long* send[kMaxRanks];
    unsigned long long* recv[kMaxRanks];
};
__global__ void k_xsum(XsumArgs a, int nranks, long long n) {
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
        unsigned long long v = 0ull;
        for (int q = 0; q < nranks; ++q) v += a.send[q][i];
        for (int q = 0; q < nranks; ++q) a.recv[q][i] = v;
    }
}

// k_finish(t): block 0 prepares iteration t+1, the others insert iteration t.  On a
// single rank, 256-slot block g is inserted by workgroup kInsertBase + g: workgroups
// are dealt to the 8 XCDs round-robin, so that is the XCD whose k_expand workgroup g
// just wrote the slots (its L2 holds them).
__global__ __launch_bounds__(kBlock) void k_finish(KgmtDev d, int t) {
    // Diagnostics (tools/timeline.py --finish): stamps of wave 0, kept in registers.
    const bool tl = d.timelineFin && t == d.timelineIter && threadIdx.x < kWave;
    long long st[kTimelineStamps] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (tl) st[0] = (long long)__builtin_amdgcn_s_memrealtime();
    if (blockIdx.x == 0) {
        plan_iteration(d, t + 1, tl ? st : nullptr);
    } else if (d.sharded) {   // every rank inserts every rank's children (replicated tree)
        insert_records(d, t, (int)blockIdx.x - 1, (int)gridDim.x - 1, tl ? st : nullptr);
        owner_clear(d, t, (int)blockIdx.x - 1);
    } else if (blockIdx.x >= kInsertBase) {   // blocks 1 .. kInsertBase-1 are idle
        const int G = (int)gridDim.x - kInsertBase;
        if (G >= d.nBlocks) insert_block(d, t, (int)blockIdx.x - kInsertBase, tl ? st : nullptr);
        else insert_blocks(d, t, (int)blockIdx.x - kInsertBase, G, tl ? st : nullptr);
    }
    if (tl) {
        st[7] = (long long)__builtin_amdgcn_s_memrealtime();
        if (threadIdx.x == 0)
            for (int i = 0; i < kTimelineStamps; ++i) d.timelineFin[(size_t)blockIdx.x * kTimelineStamps + i] = st[i];
    }
}

// ------------------------------------------------------------------ one-shot exchange
// recv = sum over ranks of send, through inboxes mapped with HIP IPC, in place of the
// RCCL all-reduce of the exchange buffer.  Every rank's inbox is
// [2 parities][nranks slots][n words] followed by flags[nranks][kOneshotChunks].
// Workgroup c owns chunk c of the words: it stores the chunk into slot `rank` of every
// peer's inbox (parity seq & 1) with system-scope stores, fences, raises its flag
// (seq) at every peer, waits for every peer's flag of chunk c in its own inbox, and
// combines the chunk's slots with its own words (read again from send, not stored).  seq counts the exchanges of the plan's lifetime and is
// the same on every rank; a rank is at most one exchange ahead of another (it waits for
// the other's flags), so it writes parity seq & 1 only after every reader of exchange
// seq - 2 has combined it.
//
// Sharded k_step (OneshotArgs::compact): the words on the wire are a compact form of the
// send buffer, 5x fewer at 8 ranks, since every word is stored once per rank over xGMI:
//   [nR1]          R1 deltas, this rank's kDeltaReps replicas summed      (summed)
//   [rows / 2]     this rank's part of every row word, 2 ints per word    (summed)
//   [owned / 2]    this rank's block words only (owned block lb -> global
//                  block rank + P lb), 2 ints per word                    (placed)
//   [nR2 / 64]     R2New as bits instead of bytes                         (or-ed)
// and the receiver writes recv in the send layout k_step reads (delta replica 0, the
// row words, every rank's block words, R2New bytes 0/1); recv's other delta replicas
// stay zero (begin() clears recv).
constexpr int kOneshotChunks = 32;   // workgroups: each thread holds about one word or list entry
struct OneshotArgs {
    unsigned long long* inbox[kMaxRanks];
    int compactOn;
    OneshotCompact cx;
    long long* tl;   // diagnostics: 8 stamps per workgroup (SBMP_TIMELINE_ITER), or null
};

// Compact word i of this rank (see above).
// SC1: every load of send is an agent-scope (sc1) load, for the fused exchange, which
// reads what other workgroups of the same launch wrote through (k_step's tail).
template <bool SC1 = false>
__device__ __forceinline__ unsigned long long send_u64(const unsigned long long* p) {
    if constexpr (SC1) return __hip_atomic_load(G(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool SC1 = false>
__device__ __forceinline__ unsigned send_u32(const int* p) {
    if constexpr (SC1) return (unsigned)__hip_atomic_load(G(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return (unsigned)*p;
}
template <bool SC1 = false>
__device__ __forceinline__ unsigned long long oneshot_pack(const OneshotCompact& x, const unsigned long long* send,
                                                           int i, int rank, int nranks) {
    if (i < x.cR) {
        unsigned long long v = 0ull;
#pragma unroll
        for (int r = 0; r < kDeltaReps; ++r) v += send_u64<SC1>(send + (size_t)r * x.nR1 + i);
        return v;
    }
    if (i < x.cB) return send_u64<SC1>(send + x.rowOff + (i - x.cR));
    if (i < x.cN) {
        const int* cnt = reinterpret_cast<const int*>(send + x.cntOff);
        const int lb = 2 * (i - x.cB);
        const int g0 = rank + nranks * lb, g1 = g0 + nranks;
        const unsigned lo = (lb < x.owned && g0 < x.nBlocks) ? send_u32<SC1>(cnt + g0) : 0u;
        const unsigned hi = (lb + 1 < x.owned && g1 < x.nBlocks) ? send_u32<SC1>(cnt + g1) : 0u;
        return ((unsigned long long)hi << 32) | lo;
    }
    const int w = i - x.cN;
    unsigned long long bits = 0ull;
#pragma unroll
    for (int m = 0; m < 8; ++m) {   // 8 bytes -> 8 bits (bytes are 0 or 1; a nonzero byte is a set bit)
        const int k = 8 * w + m;
        const unsigned long long q = (k < x.newWords) ? send_u64<SC1>(send + x.newOff + k) : 0ull;
        const unsigned long long hi = (((q & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | q) & 0x8080808080808080ull;
        bits |= (((hi >> 7) * 0x0102040810204080ull) >> 56) << (8 * m);
    }
    return bits;
}

// Combine compact word i over the ranks' slots into recv (send layout).
__device__ __forceinline__ void oneshot_unpack(const OneshotCompact& x, const unsigned long long* inbox, size_t slotStride,
                                               unsigned long long* recv, int i, int nranks, int rank,
                                               unsigned long long mine) {
    unsigned long long v[kMaxRanks];
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
        v[r] = (r == rank) ? mine
               : (r < nranks) ? __hip_atomic_load(inbox + (size_t)r * slotStride + i, __ATOMIC_RELAXED,
                                                  __HIP_MEMORY_SCOPE_SYSTEM)
                              : 0ull;
    if (i < x.cB) {   // deltas, rows: sums
        unsigned long long s = 0ull;
#pragma unroll
        for (int r = 0; r < kMaxRanks; ++r) s += v[r];
        recv[i < x.cR ? i : x.rowOff + (i - x.cR)] = s;
    } else if (i < x.cN) {   // rank r's owned blocks lb, lb + 1 -> global blocks r + P lb
        int* cnt = reinterpret_cast<int*>(recv + x.cntOff);
        uint16_t* c16 = reinterpret_cast<uint16_t*>(recv + x.c16Off);   // and the counts alone (k_step's LDS table)
        const int lb = 2 * (i - x.cB);
        for (int r = 0; r < nranks; ++r) {
            const int g0 = r + nranks * lb, g1 = g0 + nranks;
            if (lb < x.owned && g0 < x.nBlocks) {
                cnt[g0] = (int)(unsigned)v[r];
                c16[g0] = (uint16_t)(v[r] & 0xffffu);
            }
            if (lb + 1 < x.owned && g1 < x.nBlocks) {
                cnt[g1] = (int)(unsigned)(v[r] >> 32);
                c16[g1] = (uint16_t)((v[r] >> 32) & 0xffffu);
            }
        }
    } else {   // R2New: or of the bits, back to bytes
        unsigned long long bits = 0ull;
#pragma unroll
        for (int r = 0; r < kMaxRanks; ++r) bits |= v[r];
        const int w = i - x.cN;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int k = 8 * w + m;
            if (k < x.newWords) {
                const unsigned long long b8 = (bits >> (8 * m)) & 0xffull;   // bit b -> byte b (0 or 1)
                const unsigned long long s = (b8 * 0x0101010101010101ull) & 0x8040201008040201ull;
                recv[x.newOff + k] =
                    ((((s & 0x7f7f7f7f7f7f7f7full) + 0x7f7f7f7f7f7f7f7full) | s) & 0x8080808080808080ull) >> 7;
            }
        }
    }
}

// Chunk c of the exchange.
__device__ __forceinline__ void oneshot_chunk(const OneshotArgs& a, const unsigned long long* __restrict__ send,
                                              unsigned long long* __restrict__ recv, long long n, int nranks,
                                              int rank, unsigned long long seq, int* error, int c) {
    const int tid = (int)threadIdx.x;
    long long* const tl = (a.tl && tid == 0 && c < 8) ? a.tl + (size_t)c * 8 : nullptr;   // chunks 0-7
    if (tl) tl[0] = (long long)__builtin_amdgcn_s_memrealtime();
    const long long nw = a.compactOn ? a.cx.total : n;   // words on the wire
    const long long per = (nw + kOneshotChunks - 1) / kOneshotChunks;
    const long long lo = c * per, hi = min(nw, lo + per);
    const size_t par = (size_t)(seq & 1ull) * nranks * n;   // slots stay n words apart
    const size_t flags = (size_t)2 * nranks * n;
    // this rank's own slot is not stored: its words are recomputed from send below
    for (long long i = lo + tid; i < hi; i += kBlock) {
        const unsigned long long v = a.compactOn ? oneshot_pack(a.cx, send, (int)i, rank, nranks) : send[i];
        for (int q = 0; q < nranks; ++q)
            if (q != rank)
                __hip_atomic_store(a.inbox[q] + par + (size_t)rank * n + i, v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (tl) tl[1] = (long long)__builtin_amdgcn_s_memrealtime();
    if (tl) tl[2] = (long long)__builtin_amdgcn_s_memrealtime();
    if (nranks > 1) {
        __threadfence_system();   // this thread's stores reach every rank before the flag
        __syncthreads();
        if (tl) tl[3] = (long long)__builtin_amdgcn_s_memrealtime();
        if (tid < nranks && tid != rank) {   // raise flag (rank, c) at peer q, wait for (q, c) here
            const int q = tid;
            __hip_atomic_store(a.inbox[q] + flags + (size_t)rank * kOneshotChunks + c, seq, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            unsigned long long* f = a.inbox[rank] + flags + (size_t)q * kOneshotChunks + c;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kExchangeWaitTicks) {   // report, do not hang
                    atomicExch(error, kErrExchange);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __threadfence_system();
        __syncthreads();
    }
    if (tl) tl[4] = (long long)__builtin_amdgcn_s_memrealtime();
    for (long long i = lo + tid; i < hi; i += kBlock) {
        const unsigned long long mine = a.compactOn ? oneshot_pack(a.cx, send, (int)i, rank, nranks) : send[i];
        if (a.compactOn) {
            oneshot_unpack(a.cx, a.inbox[rank] + par, (size_t)n, recv, (int)i, nranks, rank, mine);
        } else {
            unsigned long long sum = mine;
            for (int r = 0; r < nranks; ++r)
                if (r != rank)
                    sum += __hip_atomic_load(a.inbox[rank] + par + (size_t)r * n + i, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_SYSTEM);
            recv[i] = sum;
        }
    }
    if (tl) tl[5] = (long long)__builtin_amdgcn_s_memrealtime();
}

__global__ __launch_bounds__(kBlock) void k_oneshot(OneshotArgs a, const unsigned long long* __restrict__ send,
                                                    unsigned long long* __restrict__ recv, long long n, int nranks,
                                                    int rank, unsigned long long seq, int* error) {
    oneshot_chunk(a, send, recv, n, nranks, rank, seq, error, (int)blockIdx.x);
}
// ------------------------------------------------------------------ fused exchange
// Sharded k_step with the one-shot exchange and the list mirror (d.fusedX): the exchange
// of t runs at the end of k_step(t) itself, so an iteration is one launch per rank and
// not two (a dependent launch costs 1.5-1.9 us, and k_oneshot's own start ~2.5 us more).
// Every expanding workgroup calls this at its exit.  Its stores that the exchange reads
// (R1 deltas: agent atomics; row and block words, R2New bytes: sc1 stores) and its list
// pushes into the mirrors (system scope) have completed (s_waitcnt vmcnt(0) in every
// wave, then a barrier); then one wave instruction with 8 active lanes adds one to each
// of 8 arrival replicas, each sharded 8 ways (the workgroup's shard: owned block mod 8;
// every counter on a 128-B line of its own, so a line takes ~128 arrivals, not 1,025; the
// planner workgroup adds too, step_planner_arrive), and the workgroup leaves unless it is
// a worker.  The workers are the workgroups of owned blocks 0..7: worker c polls the 8
// shard counters of replica c (one load per lane) until every workgroup of the launch has
// added (the guide's replicated, sharded counter hand-off: MI355X_MICROARCH.md, inter-
// workgroup visibility), so the last arrival's one atomic instruction releases all eight
// workers.  (Round 4 let each shard's last arrival add to a top counter that the workers
// polled: one more dependent atomic after the last wave.)
// Every byte the workers need is then in memory, and worker c reads chunk c of the
// compact words with sc1 loads (past both caches; per-XCD L2s are not coherent), sends
// it into the peers' inboxes, raises its flag and waits for theirs (chunk c of
// k_oneshot's flags, the same sequence numbers), and writes its part of recv, which the
// next launch reads after the kernel boundary.
constexpr int kFxRegs = 4;   // compact words a thread keeps between its send and its combine
// Arrival of one workgroup (shard = its owned block mod 8; the planner counts in shard 0):
// one instruction, lane r adding to replica r's counter of that shard.
__device__ __forceinline__ void fx_arrive(const KgmtDev& d, int t, int shard) {
    SBMP_GAS unsigned* const arr = G(d.xArrive) + (size_t)(t & 1) * kFxCounters * kFxStride;
    if (threadIdx.x < kFxReplicas)
        __hip_atomic_fetch_add(arr + (threadIdx.x * kFxShards + shard) * kFxStride, 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void k_step_exchange(const KgmtDev& d, int nranks, int rank, int nRows, int t) {
    const int tid = (int)threadIdx.x;
    const int nW = min(kFxReplicas, nRows);   // workers: owned blocks 0 .. nW - 1
    const int c = (int)blockIdx.x - 1;        // this workgroup's owned block: worker c if c < nW
    fx_arrive(d, t, c & (kFxShards - 1));
    if (c >= nW) return;
    if (tid < kFxShards) {   // lanes 0-7: replica c's shard counters, until every workgroup is in
        const SBMP_GAS unsigned* const rep = G(d.xArrive) + ((size_t)(t & 1) * kFxCounters + c * kFxShards + tid) * kFxStride;
        const unsigned want = (unsigned)((nRows - tid + kFxShards - 1) / kFxShards) + (tid == 0 ? 1u : 0u);   // + the planner
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        while (true) {
            const bool in = __hip_atomic_load(rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
            if (__ballot(!in) == 0ull) break;   // (lanes 8-63 are inactive here)
            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kExchangeWaitTicks) {   // report, do not hang
                if (tid == 0) atomicExch(&d.status->error, kErrExchange);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");   // no instruction: the loads below stay below
    __syncthreads();
    // diagnostics: worker 0's stamps in k_oneshot's rows of the timeline (tools/timeline.py --step)
    long long* const fxTl =
        (d.timelineFin && t == d.timelineIter && tid == 0) ? d.timelineFin + (size_t)(1 + c) * kTimelineStamps : nullptr;
    if (fxTl) fxTl[0] = (long long)__builtin_amdgcn_s_memrealtime();
    const OneshotCompact& x = d.xc;
    const unsigned long long seq = d.xSeqBase + (unsigned long long)t;
    const long long n = d.xInboxWords;
    const size_t par = (size_t)(seq & 1ull) * nranks * n;
    const size_t flags = (size_t)2 * nranks * n;
    const unsigned long long* const send = d.stepXs[t & 1];
    const int per = (x.total + nW - 1) / nW;
    const int lo = c * per, hi = min(x.total, lo + per);
    unsigned long long mine[kFxRegs];
#pragma unroll
    for (int u = 0; u < kFxRegs; ++u) {
        const int i = lo + tid + u * kBlock;
        mine[u] = (i < hi) ? oneshot_pack<true>(x, send, i, rank, nranks) : 0ull;
    }
#pragma unroll
    for (int u = 0; u < kFxRegs; ++u) {
        const int i = lo + tid + u * kBlock;
        if (i < hi)
            for (int q = 0; q < nranks; ++q)
                if (q != rank)
                    __hip_atomic_store(G(d.xInbox[q]) + par + (size_t)rank * n + i, mine[u], __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_SYSTEM);
    }
    for (int i = lo + tid + kFxRegs * kBlock; i < hi; i += kBlock) {   // chunks past kFxRegs words per thread
        const unsigned long long v = oneshot_pack<true>(x, send, i, rank, nranks);
        for (int q = 0; q < nranks; ++q)
            if (q != rank)
                __hip_atomic_store(G(d.xInbox[q]) + par + (size_t)rank * n + i, v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_SYSTEM);
    }
    if (fxTl) fxTl[1] = fxTl[2] = fxTl[3] = (long long)__builtin_amdgcn_s_memrealtime();
    if (nranks > 1) {
        __threadfence_system();   // this thread's stores reach every rank before the flag
        __syncthreads();
        if (fxTl) fxTl[3] = (long long)__builtin_amdgcn_s_memrealtime();
        if (tid < nranks && tid != rank) {   // flag (rank, chunk c) at peer q; wait for (q, chunk c) here
            const int q = tid;
            __hip_atomic_store(d.xInbox[q] + flags + (size_t)rank * kOneshotChunks + c, seq, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            unsigned long long* f = d.xInbox[rank] + flags + (size_t)q * kOneshotChunks + c;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < seq) {
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kExchangeWaitTicks) {   // report, do not hang
                    atomicExch(&d.status->error, kErrExchange);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __threadfence_system();
        __syncthreads();
    }
    if (fxTl) fxTl[4] = (long long)__builtin_amdgcn_s_memrealtime();
    unsigned long long* const recv = const_cast<unsigned long long*>(d.stepXr);
#pragma unroll
    for (int u = 0; u < kFxRegs; ++u) {
        const int i = lo + tid + u * kBlock;
        if (i < hi) oneshot_unpack(x, d.xInbox[rank] + par, (size_t)n, recv, i, nranks, rank, mine[u]);
    }
    for (int i = lo + tid + kFxRegs * kBlock; i < hi; i += kBlock)
        oneshot_unpack(x, d.xInbox[rank] + par, (size_t)n, recv, i, nranks, rank,
                       oneshot_pack<true>(x, send, i, rank, nranks));
    if (fxTl) fxTl[5] = (long long)__builtin_amdgcn_s_memrealtime();
}

// The planner workgroup of a fused-exchange k_step(t) reads t-1's recv (row, block and
// delta words, R2New bytes) at entry and, while it inserts t-1's rows, the block words of
// their rows; the workers of exchange t rewrite recv.  So it arrives too, once its loads
// have returned (every wave's vmcnt(0), then a barrier): it adds to the arrival replicas
// like an expanding workgroup, and the workers wait for it too.
__device__ __forceinline__ void step_planner_arrive(const KgmtDev& d, int t) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    fx_arrive(d, t, 0);
}

size_t oneshot_inbox_words(long long n, int nranks) { return (size_t)2 * nranks * n + (size_t)nranks * kOneshotChunks; }

// ------------------------------------------------------------------ list-mirror check
// The start-up check of the list mirror (KgmtPlanner::mirror_self_test):
// every rank's k_step stores its flagged children's entries into every peer's mirror with
// system-scope stores, and each rank reads its own mirror in its next k_step with plain
// loads, relying on the kernel boundary in between to drop lines its L2 still holds from
// two iterations back.  The check reproduces exactly that: touch (plain loads of the probed
// entries, so they sit in this GPU's caches), a host barrier, push (every rank stores a
// pass-specific pattern into the entries of its own global blocks in every rank's mirror,
// as k_step does), a host barrier, check (a new launch reads them with plain loads and
// compares).  Two passes, so that pass 1 finds pass 0's lines cached.
__device__ __forceinline__ float4 probe_entry(int writer, int g, int i, int k, int pass) {
    const uint32_t h = (uint32_t)(writer * 0x9E3779B1u) ^ (uint32_t)(g * 0x85EBCA77u) ^ (uint32_t)(i * 0xC2B2AE3Du) ^
                       (uint32_t)(k * 0x27D4EB2Fu) ^ (uint32_t)((pass + 1) * 0x165667B1u);
    return make_float4(__uint_as_float(h & 0x7f7fffffu), __uint_as_float((h * 3u) & 0x7f7fffffu),
                       __uint_as_float((h ^ 0x5bd1e995u) & 0x7f7fffffu), __uint_as_float((h + 0x68e31da4u) & 0x7f7fffffu));
}
// entry (parity, global block g, index i) of the probed set: parity-major, one thread each
__device__ __forceinline__ size_t probe_index(const MirrorProbe& a, int e, int* g, int* i) {
    const int par = e / (a.blocks * a.entries), r = e % (a.blocks * a.entries);
    *g = r / a.entries;
    *i = r % a.entries;
    return ((size_t)par * a.nBlocks + *g) * kBlock * kStepEntry + (size_t)*i * kStepEntry;
}
__global__ void k_mirror_touch(MirrorProbe a, float* sink) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 2 * a.blocks * a.entries) return;
    int g, i;
    const size_t o = probe_index(a, e, &g, &i);
    float acc = 0.0f;
    for (int k = 0; k < kStepEntry; ++k) acc += G(a.own)[o + k].x;   // plain loads, as k_step's
    if (acc == 1.2345f) sink[0] = acc;   // keeps the loads
}
__global__ void k_mirror_push(MirrorProbe a, int pass) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 2 * a.blocks * a.entries) return;
    int g, i;
    const size_t o = probe_index(a, e, &g, &i);
    if (g % a.nranks != a.rank) return;   // this rank's global blocks only, as k_step
    for (int q = 0; q < a.nranks; ++q)
        for (int k = 0; k < kStepEntry; ++k) store_record_g(G(a.peer[q]) + o + k, probe_entry(a.rank, g, i, k, pass));
}
__global__ void k_mirror_check(MirrorProbe a, int pass) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 2 * a.blocks * a.entries) return;
    int g, i;
    const size_t o = probe_index(a, e, &g, &i);
    int bad = 0;
    for (int k = 0; k < kStepEntry; ++k) {
        const float4 v = G(a.own)[o + k];   // plain loads, as k_step's
        const float4 w = probe_entry(g % a.nranks, g, i, k, pass);
        bad += (__float_as_uint(v.x) != __float_as_uint(w.x)) | (__float_as_uint(v.y) != __float_as_uint(w.y)) |
               (__float_as_uint(v.z) != __float_as_uint(w.z)) | (__float_as_uint(v.w) != __float_as_uint(w.w));
    }
    if (bad) atomicAdd(a.bad, bad);
}
// ------------------------------------------------------------------ fused-exchange check
// The fused exchange's in-kernel order (k_step_exchange), reproduced once at start-up on
// this machine (KgmtPlanner::fused_self_test): every workgroup pushes its
// entries into every rank's list mirror with the system-scope stores k_step uses, drains
// them (s_waitcnt vmcnt(0), barrier) and arrives with one relaxed agent-scope add on the
// replicated, sharded counters; the workers (owned blocks 0..7) wait for every arrival,
// fence (which orders only their own stores) and raise their flags at the peers, then
// wait for the peers' flags; the next launch on each rank (k_mirror_check) reads its
// mirror with plain loads.  No host barrier and no kernel boundary sits between a peer's
// pushes and its flags: the order the fused exchange relies on, which the list-mirror
// check (pushes in a launch of their own, then a host barrier) does not probe.
__global__ __launch_bounds__(kBlock) void k_fx_probe(FxProbe a, int pass) {
    const int tid = (int)threadIdx.x;
    const int b = (int)blockIdx.x;              // owned block
    const int g = a.rank + a.nranks * b;        // its global block
    if (tid < 2 * a.entries) {   // entry (parity, g, i) in every rank's mirror, as k_step pushes
        const int par = tid / a.entries, i = tid % a.entries;
        const size_t o = ((size_t)par * a.nBlocks + g) * kBlock * kStepEntry + (size_t)i * kStepEntry;
        for (int q = 0; q < a.nranks; ++q)
            for (int k = 0; k < kStepEntry; ++k) store_record_g(G(a.peer[q]) + o + k, probe_entry(a.rank, g, i, k, pass));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's pushes have completed
    __syncthreads();
    const int shard = b & (kFxShards - 1);
    if (tid < kFxReplicas)   // the arrival: one instruction, lane r adding to replica r's shard counter
        __hip_atomic_fetch_add(G(a.arrive) + (tid * kFxShards + shard) * kFxStride, 1u, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
    const int nW = min(kFxReplicas, a.owned);
    if (b >= nW) return;
    if (tid < kFxShards) {   // worker b: replica b's shard counters, until every workgroup is in
        const SBMP_GAS unsigned* const rep = G(a.arrive) + (b * kFxShards + tid) * kFxStride;
        const unsigned want = (unsigned)((a.owned - tid + kFxShards - 1) / kFxShards);
        const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
        while (true) {
            const bool in = __hip_atomic_load(rep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= want;
            if (__ballot(!in) == 0ull) break;
            if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kExchangeWaitTicks) {
                if (tid == 0) atomicExch(a.error, kErrExchange);
                break;
            }
            __builtin_amdgcn_s_sleep(1);
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __syncthreads();
    if (a.nranks > 1) {
        __threadfence_system();
        __syncthreads();
        if (tid < a.nranks && tid != a.rank) {   // flag (rank, chunk b) at peer q; wait for (q, chunk b) here
            const int q = tid;
            __hip_atomic_store(a.inbox[q] + a.flagsOff + (size_t)a.rank * kOneshotChunks + b, a.seq, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
            unsigned long long* f = a.inbox[a.rank] + a.flagsOff + (size_t)q * kOneshotChunks + b;
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < a.seq) {
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kExchangeWaitTicks) {
                    atomicExch(a.error, kErrExchange);
                    break;
                }
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __threadfence_system();
        __syncthreads();
    }
}
void launch_fx_probe(const FxProbe& a, int pass, hipStream_t s) {
    hipLaunchKernelGGL(k_fx_probe, dim3(a.owned), dim3(kBlock), 0, s, a, pass);
}

void launch_mirror_probe(const MirrorProbe& a, int phase, int pass, float* sink, hipStream_t s) {
    const int n = 2 * a.blocks * a.entries;
    const dim3 grid((n + kBlock - 1) / kBlock), block(kBlock);
    if (phase == 0) hipLaunchKernelGGL(k_mirror_touch, grid, block, 0, s, a, sink);
    else if (phase == 1) hipLaunchKernelGGL(k_mirror_push, grid, block, 0, s, a, pass);
    else hipLaunchKernelGGL(k_mirror_check, grid, block, 0, s, a, pass);
}


// ------------------------------------------------------------------ step
// k_step(t): one launch per iteration on a single rank, doing what
// k_finish(t-1) and k_expand(t) do without the launch between them.
//   Workgroup 0 (dispatched first, never waits) is the planner: it folds t-1's
//   region deltas into the tables of parity t & 1, computes the R2 snapshot and
//   the scores (updateR1), persists ctrl[t], and publishes scores and snapshot as
//   8-B words tagged with t.
//   Workgroups 1..nBlocks (block b = blockIdx - 1) each scan t-1's packed block
//   counts into LDS and derive the same plan scalars; expand their 256 slots -- a
//   parent row inserted by t-1 is read from t-1's compacted list of the block that
//   produced it (binary search of the LDS prefix), any older row from the tree --
//   then take the published scores and snapshot (re-reading until every tag is t,
//   bounded), run the accept test and write their outputs for t+1: the packed count
//   and goal index and the compacted list (parity t & 1), R1 deltas and R2New bits
//   (ring t % 3).  Each also inserts its own block's flagged children of t-1 (rows
//   treeSize(t-1) + prefix + index) and applies the D6 clear to its words.
// expand == 0 is the flush pass run before a read-back (no expansion; the same
// values are rewritten by k_step(t) proper, so it is idempotent).
// OR of word w over the kNewReps R2New replicas ([rep][nW] layout: one line per replica)
__device__ __forceinline__ uint32_t merge_new(const SBMP_GAS uint32_t* p, int nW, int w) {
    uint32_t v = 0u;
#pragma unroll
    for (int r = 0; r < kNewReps; ++r) v |= p[(size_t)r * nW + w];
    return v;
}

// ctrl[t] written through (lane-uniform value, one thread stores)
__device__ __forceinline__ void st_ctrl(IterCtrl* base, int t, const IterCtrl& c) {
    uint4* const q = reinterpret_cast<uint4*>(base + t);
    store_wt(q, 0, make_uint4(c.run, c.executed, c.treeSize, c.gLo));
    store_wt(q, 1, make_uint4(c.nG, c.k, c.nExp, c.S));
    store_wt(q, 2, make_uint4(c.H, c.A, c.scoreBuf, c.pad[0]));
    store_wt(q, 3, make_uint4(c.pad[1], c.pad[2], c.pad[3], c.pad[4]));
}

__device__ __forceinline__ void step_unpack(int v, int* cnt, int* goal) {
    *cnt = v & 0xffff;
    *goal = (v >> 16) - 1;
}

// Scan of iteration t-1's packed block counts (4 per thread, kMaxStepBlocks = 4 x
// kBlock) with one barrier: sPfx[g] = flagged children of the blocks before g (g <=
// nBlocks), *A the total, *jGoal the lowest global index of a flagged child in the
// goal region.  Each wave publishes its total and its lowest goal index relative to
// its own start before the barrier, so A and jGoal are known right after it; sPfx is
// written after it and needs the caller's next barrier before other waves read it.
__device__ __forceinline__ void step_scan(const KgmtDev& d, int4 pk, int* sPfx, int (*sRed)[kBlock / kWave], int* A,
                                          int* jGoal) {
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform: scalar selects below
    int loc[4];
    int run = 0;
    const int v4[4] = {pk.x, pk.y, pk.z, pk.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        loc[e] = run;
        run += v4[e] & 0xffff;
    }
    const int incl = wave_incl_sum(run);
    const int excl = incl - run;   // this thread's start within its wave
    // Prefixes grow with g and a goal child's in-block index is below its block's
    // count, so the lowest g holding a goal child has the lowest global index.  Only a
    // wave that holds a goal flag looks (none while the goal is out of reach or disabled).
    int gl = kNoGoalIdx;
    if (__ballot(((pk.x | pk.y | pk.z | pk.w) >> 16) != 0) != 0ull) {
#pragma unroll
        for (int e = 3; e >= 0; --e) {
            int c, g;
            step_unpack(v4[e], &c, &g);
            if (g >= 0) gl = excl + loc[e] + g;
        }
        gl = first_lane_value(gl != kNoGoalIdx, gl, kNoGoalIdx);
    }
    if (lane == kWave - 1) sRed[0][wave] = incl;
    if (lane == 0) sRed[1][wave] = gl;
    __syncthreads();
    // uniform by construction; readfirstlane so that A, jGoal and the plan that follows
    // are scalar code
    const int w0 = __builtin_amdgcn_readfirstlane(sRed[0][0]), w1 = __builtin_amdgcn_readfirstlane(sRed[0][1]),
              w2 = __builtin_amdgcn_readfirstlane(sRed[0][2]), w3 = __builtin_amdgcn_readfirstlane(sRed[0][3]);
    *A = w0 + w1 + w2 + w3;
    const int g0 = __builtin_amdgcn_readfirstlane(sRed[1][0]), g1 = __builtin_amdgcn_readfirstlane(sRed[1][1]),
              g2 = __builtin_amdgcn_readfirstlane(sRed[1][2]), g3 = __builtin_amdgcn_readfirstlane(sRed[1][3]);
    int jg = kNoGoalIdx;   // the lowest wave holding one has the lowest index
    if (g3 != kNoGoalIdx) jg = w0 + w1 + w2 + g3;
    if (g2 != kNoGoalIdx) jg = w0 + w1 + g2;
    if (g1 != kNoGoalIdx) jg = w0 + g1;
    if (g0 != kNoGoalIdx) jg = g0;
    *jGoal = jg;
    const int base = excl + (wave > 0 ? w0 : 0) + (wave > 1 ? w1 : 0) + (wave > 2 ? w2 : 0);
    if (tid * 4 + 3 <= d.nBlocks) {   // one 16-B LDS store (sPfx is 16-B aligned)
        *reinterpret_cast<int4*>(sPfx + tid * 4) = make_int4(base, base + loc[1], base + loc[2], base + loc[3]);
    } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
            if (tid * 4 + e <= d.nBlocks) sPfx[tid * 4 + e] = base + loc[e];
    }
    if (tid == kBlock - 1 && d.nBlocks == kMaxStepBlocks) sPfx[kMaxStepBlocks] = *A;
}

// Sharded k_step: the scan runs over rows (block b of every rank), so its size is the
// rank's block count however many ranks there are.  sPfx[r] = children of the rows
// before r, *A the total, *gRow the lowest row holding a goal child (kNoGoalIdx if none).
// One barrier, as step_scan: sPfx is written after it and needs the caller's next one.
// A sharded rank's geometry for k_step, from kernel arguments: they arrive with the
// first batch of argument loads, where the same fields of the plan struct took two more
// dependent scalar round trips in front of the prologue's loads.
struct ShardView {
    int nranks, rank, nRows;    // ranks, this rank, rows (owned blocks)
    const SBMP_GAS int* bw;     // the exchange's block words (stepXr + xCntOff)
};

__device__ __forceinline__ void step_scan_rows(const ShardView& sv, int4 pk, int* sPfx, int (*sRed)[kBlock / kWave],
                                               int* A, int* gRow) {
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid >> 6;
    const int nRows = sv.nRows;
    int loc[4];
    int run = 0, grow = kNoGoalIdx;
    const int v4[4] = {pk.x, pk.y, pk.z, pk.w};
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        loc[e] = run;
        run += v4[e] & 0xffff;
        if ((v4[e] >> 16) != 0 && grow == kNoGoalIdx) grow = tid * 4 + e;
    }
    const int incl = wave_incl_sum(run);
    grow = first_lane_value(grow != kNoGoalIdx, grow, kNoGoalIdx);   // rows grow with the lane
    if (lane == kWave - 1) sRed[0][wave] = incl;
    if (lane == 0) sRed[1][wave] = grow;
    __syncthreads();
    const int w0 = __builtin_amdgcn_readfirstlane(sRed[0][0]), w1 = __builtin_amdgcn_readfirstlane(sRed[0][1]),
              w2 = __builtin_amdgcn_readfirstlane(sRed[0][2]), w3 = __builtin_amdgcn_readfirstlane(sRed[0][3]);
    *A = w0 + w1 + w2 + w3;
    *gRow = __builtin_amdgcn_readfirstlane(min(min(sRed[1][0], sRed[1][1]), min(sRed[1][2], sRed[1][3])));
    const int base = incl - run + (wave > 0 ? w0 : 0) + (wave > 1 ? w1 : 0) + (wave > 2 ? w2 : 0);
#pragma unroll
    for (int e = 0; e < 4; ++e)
        if (tid * 4 + e <= nRows) sPfx[tid * 4 + e] = base + loc[e];
    if (tid == kBlock - 1 && nRows == kMaxStepBlocks) sPfx[kMaxStepBlocks] = *A;
}

// The P block words of row r (counts | (1 + goal index) << 16), in block order.  All
// kMaxRanks words are loaded unconditionally (one batch, no load behind a branch: the
// conditional form became a chain of scalar loads, each waited for before the next);
// the ones past row r's P lie inside the exchange buffer (the block words of row r + 1,
// or the R2New bytes after them) and are masked.
__device__ __forceinline__ void row_words(const ShardView& sv, int r, int* w) {
    const SBMP_GAS int* blk = sv.bw + (size_t)r * sv.nranks;
    int v[kMaxRanks];
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q) v[q] = blk[q];
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q) w[q] = (q < sv.nranks) ? v[q] : 0;
}

// Position off inside row r -> (global block, index in it), from the row's words.
__device__ __forceinline__ void row_locate(const ShardView& sv, const int* w, int r, int off, int* block, int* idx) {
    int q = 0;
#pragma unroll
    for (int k = 0; k < kMaxRanks - 1; ++k) {
        const int c = w[k] & 0xffff;
        if (k == q && k + 1 < sv.nranks && off >= c) {
            off -= c;
            q = k + 1;
        }
    }
    *block = r * sv.nranks + q;
    *idx = off;
}

// The same from the LDS table of u16 block counts (global block order, all rows): a
// position inside a row without a dependent load of the row's block words.
__device__ __forceinline__ void row_locate_lds(const ShardView& sv, const uint16_t* sC16, int r, int off, int* block,
                                               int* idx) {
    const uint16_t* w = sC16 + (size_t)r * sv.nranks;
    int q = 0;
#pragma unroll
    for (int k = 0; k < kMaxRanks - 1; ++k) {
        if (k == q && k + 1 < sv.nranks) {
            const int c = w[k];
            if (off >= c) {
                off -= c;
                q = k + 1;
            }
        }
    }
    *block = r * sv.nranks + q;
    *idx = off;
}
// A position inside row r: from the LDS table when the launch staged it (d.c16Lds, the
// default), else from the row's block words (one dependent L2 round trip, round 4's form;
// begin() picks it when the table's LDS would leave too few workgroups resident).
__device__ __forceinline__ void row_locate_any(const KgmtDev& d, const ShardView& sv, const uint16_t* sC16, int r,
                                               int off, int* block, int* idx) {
    if (d.c16Lds) {   // uniform
        row_locate_lds(sv, sC16, r, off, block, idx);
    } else {
        int w[kMaxRanks];
        row_words(sv, r, w);
        row_locate(sv, w, r, off, block, idx);
    }
}
// Sharded prologue: the exchange's u16 block counts (nBlocks of them, 16-B padded) into
// LDS, loaded with the first batch (issue) and stored once the scan has waited for it
// (none when d.c16Lds is 0: the exact-size buffer is then empty).
struct C16Load {
    uint4 v[kMaxRanks / 2];   // 1,024 rows x P u16 over 256 threads: at most 4 x 16 B each
};
__device__ __forceinline__ C16Load c16_issue(const KgmtDev& d) {
    C16Load c;
    // an exact-size buffer: loads past the table return 0 without a memory access, so every
    // load is issued unconditionally (no branch, one batch)
    const int n16 = d.c16Lds ? (d.nBlocks + 7) >> 3 : 0;
    const __amdgpu_buffer_rsrc_t r =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<unsigned long long*>(d.stepXr + d.xC16Off), (short)0, n16 * 16,
                                          kBufferDword3);
#pragma unroll
    for (int u = 0; u < kMaxRanks / 2; ++u) {
        const sbmp_u32x4 x = __builtin_amdgcn_raw_buffer_load_b128(r, ((int)threadIdx.x + u * kBlock) * 16, 0, 0);
        c.v[u] = make_uint4(x[0], x[1], x[2], x[3]);
    }
    return c;
}
__device__ __forceinline__ void c16_store(const KgmtDev& d, const C16Load& c, uint16_t* sC16) {
    const int n16 = d.c16Lds ? (d.nBlocks + 7) >> 3 : 0;
#pragma unroll
    for (int u = 0; u < kMaxRanks / 2; ++u) {
        const int i = (int)threadIdx.x + u * kBlock;
        if (i < n16) reinterpret_cast<uint4*>(sC16)[i] = c.v[u];
    }
}

// jGoal of a sharded scan: the lowest global index of a goal child, in row gRow.
__device__ __forceinline__ int row_goal(const ShardView& sv, const int* sPfx, int gRow) {
    if (gRow == kNoGoalIdx) return kNoGoalIdx;
    int w[kMaxRanks];
    row_words(sv, gRow, w);
    int pre = sPfx[gRow], j = kNoGoalIdx;
#pragma unroll
    for (int q = 0; q < kMaxRanks; ++q) {
        if (q < sv.nranks && j == kNoGoalIdx && (w[q] >> 16) != 0) j = pre + (w[q] >> 16) - 1;
        pre += w[q] & 0xffff;
    }
    return __builtin_amdgcn_readfirstlane(j);
}

// The list entry (state, ctrl, cost) of row j of t-1's flagged children, given the
// block lo holding it: a single rank's own compacted list, or on a sharded rank the
// owner's (rank lo mod P, owned block lo / P) through its record buffer.
template <bool SH>
__device__ __forceinline__ const SBMP_GAS float4* list_entry(const KgmtDev& d, int pp, int lo, int i) {
    if constexpr (SH) {
        if (d.stepMirror)   // every rank's k_step pushed its lists here (uniform branch)
            return G(d.stepMirror) + ((size_t)pp * d.nBlocks * kBlock + (size_t)lo * kBlock + i) * kStepEntry;
        return G(d.recPeer[lo % d.nranks]) +
               ((size_t)pp * d.recCap + (size_t)(lo / d.nranks) * kBlock + i) * kStepEntry;
    } else {
        return G(d.stepList) + ((size_t)pp * d.nBlocks * kBlock + (size_t)lo * kBlock + i) * kStepEntry;
    }
}
// Sharded lists in a peer's memory (mapped, no list mirror) take system-scope loads: this
// GPU's L2 may hold their lines from two iterations ago.  The list mirror and a local
// shard group's buffers are this GPU's memory written before this launch: plain loads.
template <bool SH>
__device__ __forceinline__ float4 list_load(const KgmtDev& d, const SBMP_GAS float4* p) {
    if (SH && !d.listPlain) return load_record_g(p);
    return *p;
}

// Plan scalars of iteration t from t-1's control block and the scan (KGMT.cu:118,
// 139-188,249-259); every workgroup derives the same values.
struct StepPlan {
    bool ranPrev;
    int tsPrev, treeSize, gLo, H, grid, nIns, newGoal, runT, nG, k, nExp, S;
    bool executes;
};
// A plan read back from LDS, made wave-uniform (scalar registers).
__device__ __forceinline__ StepPlan uniform_plan(const StepPlan& s) {
    StepPlan q;
    q.ranPrev = __builtin_amdgcn_readfirstlane((int)s.ranPrev) != 0;
    q.tsPrev = __builtin_amdgcn_readfirstlane(s.tsPrev);
    q.treeSize = __builtin_amdgcn_readfirstlane(s.treeSize);
    q.gLo = __builtin_amdgcn_readfirstlane(s.gLo);
    q.H = __builtin_amdgcn_readfirstlane(s.H);
    q.grid = __builtin_amdgcn_readfirstlane(s.grid);
    q.nIns = __builtin_amdgcn_readfirstlane(s.nIns);
    q.newGoal = __builtin_amdgcn_readfirstlane(s.newGoal);
    q.runT = __builtin_amdgcn_readfirstlane(s.runT);
    q.nG = __builtin_amdgcn_readfirstlane(s.nG);
    q.k = __builtin_amdgcn_readfirstlane(s.k);
    q.nExp = __builtin_amdgcn_readfirstlane(s.nExp);
    q.S = __builtin_amdgcn_readfirstlane(s.S);
    q.executes = __builtin_amdgcn_readfirstlane((int)s.executes) != 0;
    return q;
}
__device__ __forceinline__ StepPlan step_plan(const KgmtDev& d, int t, int expand, const IterCtrl& pc, int goalIdx,
                                              int A, int jGoal) {
    StepPlan q;
    q.ranPrev = (t == 1) || pc.executed;
    q.tsPrev = (t == 1) ? 1 : pc.treeSize;
    q.treeSize = (t == 1) ? 1 : pc.treeSize + A;   // KGMT.cu:249
    q.gLo = (t == 1) ? 0 : pc.gLo + pc.nExp;
    const int Hprev = (t == 1) ? 0 : pc.H;
    q.grid = min(A, d.M / 32);   // updateG launch: min(|GNew|, M/32) blocks of 32 (KGMT.cu:231)
    q.nIns = 32 * q.grid < A ? 32 * q.grid : A;
    // The lowest inserted row of t-1 inside the goal radius (D4): rows grow with j,
    // so if the lowest candidate is not inserted (D13) none is.
    q.newGoal = goalIdx;
    if (jGoal < q.nIns && jGoal < d.M - q.tsPrev) q.newGoal = min(q.newGoal, q.tsPrev + jGoal);   // tsPrev <= M: no overflow
    q.runT = (t <= d.numIterations) && (q.treeSize < d.M);   // KGMT.cu:118,255
    q.nG = 0;
    q.k = 0;
    q.nExp = 0;
    if (q.runT) {
        q.nG = q.treeSize - q.gLo;
        batch_rule(d, q.treeSize, q.nG, &q.k, &q.nExp);
    }
    q.S = q.k * q.nExp;
    q.H = max(Hprev, q.S);
    q.executes = expand && q.runT && q.newGoal == kNoGoal;
    return q;
}

// Workgroup 0 of k_step(t): tables of t (R1 deltas folded, R2New merged into R2Avail
// = the snapshot, R1Cov), scores (updateR1, KGMT.cu:485-538, CUB order D8), ctrl[t];
// scores and snapshot published as 8-B words tagged with t.
template <bool SH>
__device__ __forceinline__ void step_planner(const KgmtDev& d, const ShardView& sv, int t, int expand, int* sPfx,
                                             int (*sRed)[kBlock / kWave], int* sCovInc, float* sPart, uint16_t* sC16) {
    constexpr int kW = kMaxR2Words / kBlock;
    const int tid = threadIdx.x;
    const int nW = d.nR2 >> 5;
    const int nn = d.n * d.n;
    const int pp = (t - 1) & 1, cp = t & 1;
    const int cell = min(tid, d.nR1 - 1);
    const bool own = tid < d.nR1;
    const bool tl = d.timelineFin && t == d.timelineIter && tid == 0;   // diagnostics: entry, publish
    if (tl) G(d.timelineFin)[0] = (long long)__builtin_amdgcn_s_memrealtime();
    // every input at entry
    // t-1's packed counts: blocks, or (sharded) rows of the exchange
    const int4 pk = SH ? reinterpret_cast<const SBMP_GAS int4*>(G(d.stepXr) + d.xRowOff)[tid]
                       : *reinterpret_cast<const SBMP_GAS int4*>(G(d.stepCnt) + (size_t)pp * kMaxStepBlocks + tid * 4);
    const IterCtrl pc = G(d.ctrl)[t - 1];
    const int goalIdx = G(d.status)->goalIdx;
    // a bounded wait of an earlier launch gave up: the host's plan loop stops (hostPoll's
    // "ended" bit) and raises it (KgmtPlanner::run_to_goal)
    const int errPrev = G(d.status)->error;
    const SBMP_GAS int* tabPrev = G(d.R1) + (size_t)pp * 5 * d.nR1;
    int r1 = tabPrev[cell], r1a = tabPrev[d.nR1 + cell], r1v = tabPrev[2 * d.nR1 + cell],
        r1i = tabPrev[3 * d.nR1 + cell], r1c = tabPrev[4 * d.nR1 + cell];
    // sharded: the exchange's sum over ranks; else ring (t - 1) % 3
    const SBMP_GAS unsigned long long* deltaPrev =
        SH ? G(d.stepXr) : G(d.stepDelta) + (size_t)((t - 1) % 3) * kDeltaReps * d.nR1;
    unsigned long long dl = 0ull;   // replicas: carry-free sums
#pragma unroll
    for (int r = 0; r < kDeltaReps; ++r) dl += deltaPrev[(size_t)r * d.nR1 + cell];
    const SBMP_GAS uint32_t* availPrev = G(d.R2Avail) + (size_t)pp * nW;
    const SBMP_GAS uint32_t* newPrev = G(d.stepR2New) + (size_t)((t - 1) % 3) * kNewReps * nW;
    uint32_t availW[kW], newW[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) {
        const int w = min(tid + j * kBlock, nW - 1);
        availW[j] = availPrev[w];
        newW[j] = 0u;
    }
    // the R2New replicas: n <= 8 (two words per thread) with all 16 loads in flight;
    // larger grids one word at a time (8 VGPRs live: all 64 at once would spill).
    // Sharded: the exchange's bytes (a sum over ranks of 0/1 per cell), 32 per word.
    if constexpr (SH) {
        const SBMP_GAS uint8_t* nbp = reinterpret_cast<const SBMP_GAS uint8_t*>(G(d.stepXr) + d.xNewOff);
#pragma unroll
        for (int j = 0; j < kW; ++j) {
            if (j * kBlock < nW) {   // uniform
                const int w = min(tid + j * kBlock, nW - 1);
                const uint4 b0 = reinterpret_cast<const SBMP_GAS uint4*>(nbp + 32 * (size_t)w)[0];
                const uint4 b1 = reinterpret_cast<const SBMP_GAS uint4*>(nbp + 32 * (size_t)w)[1];
                const uint32_t qv[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
                uint32_t nw = 0u;
#pragma unroll
                for (int k = 0; k < 8; ++k) {   // nonzero bytes -> 4 bits (sums <= nranks never carry)
                    const uint32_t hi = (((qv[k] & 0x7f7f7f7fu) + 0x7f7f7f7fu) | qv[k]) & 0x80808080u;
                    nw |= ((((hi >> 7) * 0x00204081u) >> 21) & 0xfu) << (4 * k);
                }
                newW[j] = nw;
            }
        }
    } else if (nW <= 2 * kBlock) {
        newW[0] = merge_new(newPrev, nW, min(tid, nW - 1));
        newW[1] = merge_new(newPrev, nW, min(tid + kBlock, nW - 1));
    } else {
#pragma unroll
        for (int j = 0; j < kW; ++j)
            if (j * kBlock < nW) newW[j] = merge_new(newPrev, nW, min(tid + j * kBlock, nW - 1));
    }
    for (int i = tid; i < d.nR1; i += kBlock) sCovInc[i] = 0;
    int A, jGoal;
    if constexpr (SH) {
        const C16Load c16 = c16_issue(d);
        int gRow;
        step_scan_rows(sv, pk, sPfx, sRed, &A, &gRow);
        c16_store(d, c16, sC16);   // read by the inserts, behind the barrier before the scores
        if (gRow != kNoGoalIdx) __syncthreads();   // uniform (rare): row_goal reads sPfx[gRow]
        jGoal = row_goal(sv, sPfx, gRow);
    } else {
        step_scan(d, pk, sPfx, sRed, &A, &jGoal);
    }
    const StepPlan q = step_plan(d, t, expand, pc, goalIdx, A, jGoal);
    int* const tabCur = d.R1 + (size_t)cp * 5 * d.nR1;   // written through, like everything below
    if (!q.ranPrev) {   // t-1 did not run: the loop has ended; carry the tables forward
        for (int i = tid; i < 5 * d.nR1; i += kBlock) store_wt(tabCur, i, (int)tabPrev[i]);
        for (int i = tid; i < nW; i += kBlock) store_wt(d.R2Avail + (size_t)cp * nW, i, (uint32_t)availPrev[i]);
        if (tid == 0) {
            IterCtrl c{};
            c.run = 0;
            c.H = pc.H;
            st_ctrl(d.ctrl, t, c);
            if (d.hostPoll)   // the loop has ended (goal, limit or tree full in t-1): say so as well
                __hip_atomic_store(G(d.hostPoll), ((unsigned long long)t << 2) | 2ull | (goalIdx != kNoGoal ? 1ull : 0ull),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
        return;
    }
    const int nv = (int)(dl & 0xffffffffull), ni = (int)(dl >> 32);
    r1 += nv + ni;      // KGMT.cu:392
    r1v += nv;          // KGMT.cu:406
    r1i += ni;          // KGMT.cu:409
    if (nv) r1a = 1;    // KGMT.cu:399-401
    uint32_t snapW[kW];
#pragma unroll
    for (int j = 0; j < kW; ++j) {
        const int w = tid + j * kBlock;
        snapW[j] = 0u;
        if (j * kBlock < nW && w < nW) {
            const uint32_t fresh = newW[j] & ~availW[j];
            snapW[j] = availW[j] | newW[j];   // R2Avail of t = the snapshot (D2)
            if (fresh && nn % 32 == 0) {
                atomicAdd(&sCovInc[(32 * w) / nn], __popc(fresh));
            } else {
                uint32_t f = fresh;
                while (f) {
                    const int b = __builtin_ctz(f);
                    f &= f - 1u;
                    atomicAdd(&sCovInc[(32 * w + b) / nn], 1);
                }
            }
        }
    }
    __syncthreads();
    r1c += sCovInc[cell];
    float scv = 1.0f;
    if (q.runT) {
        float sc = 0.0f;
        if (r1a != 0) {
            const float covR = (float)r1c / (float)nn;
            const float freeVol = (0.01f + (float)r1v) / (0.01f + (float)r1v + (float)r1i);
            const float fv2 = freeVol * freeVol;
            const float fv4 = fv2 * fv2;
            const double rr = (double)r1;
            const double den = (double)(1.0f + covR) * (1.0 + rr * rr);
            sc = (float)((double)fv4 / den);
        }
        float v = own ? sc : 0.0f;
#pragma unroll
        for (int off = 1; off < 32; off <<= 1) {
            const float o = __shfl_down(v, off, 32);
            v = v + o;
        }
        if ((tid & 31) == 0) sPart[tid >> 5] = v;
        __syncthreads();
        float total = sPart[0];
#pragma unroll
        for (int w = 1; w < 8; ++w) total = total + sPart[w];
        scv = (r1a == 0) ? 1.0f : sc / total;
    }
    // publish first (tagged 8-B words, written through)
    SBMP_GAS unsigned long long* const pub = G(d.stepPub) + (size_t)cp * (d.nR1 + nW);
    const unsigned long long tag = (unsigned long long)(unsigned)t << 32;
    if (q.executes) {
        if (own) __hip_atomic_store(pub + cell, tag | __float_as_uint(scv), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
        for (int j = 0; j < kW; ++j) {
            const int w = tid + j * kBlock;
            if (j * kBlock < nW && w < nW)
                __hip_atomic_store(pub + d.nR1 + w, tag | snapW[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    if (tl) G(d.timelineFin)[1] = (long long)__builtin_amdgcn_s_memrealtime();
    if (own) {
        store_wt(tabCur, cell, r1);
        store_wt(tabCur, d.nR1 + cell, r1a);
        store_wt(tabCur, 2 * d.nR1 + cell, r1v);
        store_wt(tabCur, 3 * d.nR1 + cell, r1i);
        store_wt(tabCur, 4 * d.nR1 + cell, r1c);
        if (q.runT) store_wt(d.R1Score, cp * d.nR1 + cell, scv);
    }
#pragma unroll
    for (int j = 0; j < kW; ++j) {
        const int w = tid + j * kBlock;
        if (j * kBlock < nW && w < nW) store_wt(d.R2Avail + (size_t)cp * nW, w, snapW[j]);
    }
    if constexpr (SH) {   // send parity (t+1) & 1, last read by exchange t-1: zero for k_step(t+1)
        if (d.fusedX && tid < kFxCounters)   // and the fused exchange's arrival counters of t+1
            __hip_atomic_store(G(d.xArrive) + ((size_t)((t + 1) & 1) * kFxCounters + tid) * kFxStride, 0u,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        SBMP_GAS unsigned long long* zx = G(d.stepXs[(t + 1) & 1]);
        for (int i = tid; i < kDeltaReps * d.nR1; i += kBlock) zx[i] = 0ull;
        for (int i = tid; i < d.nR2 / 8; i += kBlock) zx[d.xNewOff + i] = 0ull;   // R2New bytes (count words: owner-written)
    } else {   // ring (t+1) % 3, last read by k_step(t-1): zero for k_step(t+1)
        unsigned long long* const zd = d.stepDelta + (size_t)((t + 1) % 3) * kDeltaReps * d.nR1;   // written through
        for (int i = tid; i < kDeltaReps * d.nR1; i += kBlock) store_wt(zd, i, 0ull);
        int* const zn = reinterpret_cast<int*>(d.stepR2New + (size_t)((t + 1) % 3) * kNewReps * nW);
        for (int i = tid; i < kNewReps * nW; i += kBlock) store_wt(zn, i, 0);
    }
    if (tid == 0) {
        IterCtrl c;
        c.run = q.runT;
        c.executed = q.executes ? 1 : 0;
        c.treeSize = q.treeSize;
        c.gLo = q.gLo;
        c.nG = q.nG;
        c.k = q.k;
        c.nExp = q.nExp;
        c.S = q.S;
        c.H = q.H;
        c.A = 0;
        c.scoreBuf = cp;
        for (int i = 0; i < 5; ++i) c.pad[i] = 0;
        st_ctrl(d.ctrl, t, c);
        if (t > 1) store_wt(reinterpret_cast<int*>(d.ctrl + (t - 1)), 9, A);   // .A
        if (q.newGoal != goalIdx) store_wt(reinterpret_cast<int*>(d.status), 0, q.newGoal);   // .goalIdx
        if (d.hostPoll)   // the host's plan loop: this launch planned t (a vector store over PCIe)
            __hip_atomic_store(G(d.hostPoll),
                               ((unsigned long long)t << 2) | (q.runT && !errPrev ? 0ull : 2ull) |
                                   (q.newGoal != kNoGoal ? 1ull : 0ull),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    // Insert t-1's flagged children (rows tsPrev + j, KGMT.cu:540-593) when they are
    // few: everything above is what the expanders wait for, and from here on this
    // workgroup is idle.
    if (t > 1 && A <= kPlannerInsertMax) {
        const int n = min(q.nIns, d.M - q.tsPrev);   // D13: the reference writes past M
        // list entry of row j: block (sharded: row) lo with sPfx[lo] <= j < sPfx[lo + 1]
        const int nS = SH ? sv.nRows : d.nBlocks;
        auto entry = [&](int j) {
            int lo = 0;
            for (int step = kMaxStepBlocks / 2; step > 0; step >>= 1)
                if (lo + step < nS && sPfx[lo + step] <= j) lo += step;
            if constexpr (SH) {
                int blk, idx;
                row_locate_any(d, sv, sC16, lo, j - sPfx[lo], &blk, &idx);
                return list_entry<SH>(d, pp, blk, idx);
            } else {
                return list_entry<SH>(d, pp, lo, j - sPfx[lo]);
            }
        };
        auto put = [&](int j, float4 s4, float4 u4, float c) {   // row tsPrev + j, written through
            store_wt(d.treeState + q.tsPrev, j, s4);
            store_wt(d.treeCtrl + q.tsPrev, j, make_float4(u4.x, u4.y, u4.z, c));   // cost = parent's + duration (KGMT.cu:631-633)
            store_wt(d.treeParent + q.tsPrev, j, __float_as_int(u4.w));
        };
        for (int j0 = tid; j0 < n; j0 += 2 * kBlock) {   // two rows per thread per round, loads first
            const int j1 = j0 + kBlock;
            const SBMP_GAS float4* e0 = entry(j0);
            const SBMP_GAS float4* e1 = entry(min(j1, n - 1));
            const float4 s0 = list_load<SH>(d, e0), u0 = list_load<SH>(d, e0 + 1), s1 = list_load<SH>(d, e1),
                         u1 = list_load<SH>(d, e1 + 1);
            const float c0 = list_load<SH>(d, e0 + 2).x, c1 = list_load<SH>(d, e1 + 2).x;
            put(j0, s0, u0, c0);
            if (j1 < n) put(j1, s1, u1, c1);
        }
    }
}

#ifndef SBMP_VALU_DUP
#define SBMP_VALU_DUP 0   // diagnostics: 1-4 run one part of the expanding wave twice (VALU attribution by PMC A/B)
#endif
// 5 waves per SIMD: the 1 + nBlocks workgroups (1,025 at 262,144 slots) fit the chip at once.
// The expanding workgroups:
//   prologue   RNG / count / control-block loads; the count scan; the plan scalars
//              (wave 0) while waves 1-3 draw the child's controls (they need the slot's
//              stream only; wave 0 draws after the plan's barrier); the D6 clear, the
//              parent (list search);
//   propagate  the Euler loop (statePropagator.cu:23-65);
//   accept     each lane reads the two published words it needs (score of its R1 cell,
//              snapshot word of its R2 cell, tagged with t) straight from L2, with no
//              LDS staging and no barrier; stores overlap that round trip;
//   epilogue   one barrier: wave counts -> list positions, the R1 / R2New flushes and
//              the block's packed count.
// SH: a sharded rank: workgroup b expands owned block rank + P b; the
// counts, R1 deltas and R2New of t-1 come from the exchange (stepXr), this launch's
// go to stepXs[t & 1]; the flagged children's lists are the record buffers, and
// workgroup b inserts t-1's children of blocks b P .. b P + P - 1 (one of each rank).
// The arguments the prologue's first loads need come first: the build preloads the
// first 16 argument dwords into SGPRs (-amdgpu-kernarg-preload-count, build.py), so
// those loads issue at wave start instead of behind two dependent scalar loads
// (kernel argument -> plan struct -> pointer).
// (14 dwords: the kernel-argument segment pointer takes two of the 16 user SGPRs)
//   cnt4     t-1's packed counts (parity (t-1) & 1 of stepCnt; sharded: the exchange's rows)
//   ctrlPrev ctrl[t-1]
template <int AGENT, int OBS, bool SH>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(5))) void k_step(
    const KgmtDev* __restrict__ dp, int tx, int shRR, const int4* __restrict__ cnt4,
    const IterCtrl* __restrict__ ctrlPrev, const uint4* __restrict__ rngAArg, const uint2* __restrict__ rngBArg,
    const unsigned long long* __restrict__ gnewArg, const PlannerStatus* __restrict__ statusArg, long long* tlBase,
    int shRows, const int* __restrict__ shBw) {
    // tx = t | expand << 31 and shRR = rank | ranks << 8 share the preloaded argument
    // dwords with the prologue's first pointers (a sharded slot index needs the rank
    // before its first load)
    const int t = tx & 0x7fffffff, expand = (int)((unsigned)tx >> 31);
    const KgmtDev& d = *dp;
    const ShardView sv{SH ? (shRR >> 8) : 1, SH ? (shRR & 0xff) : 0, SH ? shRows : 0, G(shBw)};
    extern __shared__ float4 sDyn[];   // [LDS obstacles][prefix: nBlocks + 1 ints][R2New bits: nR2 / 32]
    __shared__ int sR1P[kMaxR1];
    __shared__ StepPlan sPlan;
    __shared__ int sWaveCnt[kBlock / kWave];
    __shared__ int sWaveGoal[kBlock / kWave];
    __shared__ int sRed[2][kBlock / kWave];
    __shared__ float sPart[8];
    __shared__ int sCovInc[kMaxR1];

    constexpr bool kLdsObs = (OBS == kObsLds || OBS == kObsLds4);
    constexpr int kRegObs = obs_in_registers(OBS);
    int* const sPfx = reinterpret_cast<int*>(sDyn + (kLdsObs ? d.nObs : 0));
    uint32_t* const sNew = reinterpret_cast<uint32_t*>(sPfx + (SH ? sv.nRows : d.nBlocks) + 1);
    // sharded: the u16 block counts of every row, 16-B aligned after the R2New bits (step_lds_bytes)
    uint16_t* const sC16 = reinterpret_cast<uint16_t*>(sPfx + ((((SH ? sv.nRows : d.nBlocks) + 1 + (d.nR2 >> 5)) + 3) & ~3));
    if (blockIdx.x == 0) {
        step_planner<SH>(d, sv, t, expand, sPfx, sRed, sCovInc, sPart, sC16);
        if constexpr (SH) {
            if (expand && d.fusedX) step_planner_arrive(d, t);
        }
        return;
    }
    float4* const sObs = sDyn;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);   // uniform
    __shared__ int2 sWaveDiv[kBlock / kWave];   // (frontier position, remainder) of each wave's first slot
    const int b = (int)blockIdx.x - 1;                // this workgroup's 256-slot block (owned index)
    const int gb = SH ? sv.rank + sv.nranks * b : b;   // global block
    const int slot = gb * kBlock + tid;
    const int nW = d.nR2 >> 5;
    const int pp = (t - 1) & 1, cp = t & 1;
    const SBMP_GAS unsigned long long* const pubCur = G(d.stepPub) + (size_t)cp * (d.nR1 + nW);
    // d.timeline if this launch is the traced one (decided on the host: no dependent
    // loads of the plan struct before the prologue's own).  Only a diagnostic build
    // (SBMP_HIPCC_FLAGS=-DSBMP_TIMELINE, tools/mk_variant.sh tl) stamps: held in registers, the
    // eight 64-bit stamps cost every wave ~30 VALU of zeroing and moves.
#ifdef SBMP_TIMELINE
    long long* const tl = tlBase ? tlBase + ((size_t)b * (kBlock / kWave) + wave) * kTimelineStamps : nullptr;
#else
    long long* const tl = nullptr;
    (void)tlBase;
#endif
    long long stamp[kTimelineStamps] = {0, 0, 0, 0, 0, 0, 0, 0};
#define SBMP_STAMP(i)                                                                  \
    do {                                                                               \
        if (tl) stamp[i] = (long long)__builtin_amdgcn_s_memrealtime();                \
    } while (0)
    // The first loads' pointers are preloaded arguments; the plan's scalars and the
    // next pointers in one batch of scalar loads from the struct (one round trip, in
    // flight with the vector loads below)
    const SBMP_GAS IterCtrl* const ctrlP = G(ctrlPrev);
    const SBMP_GAS PlannerStatus* const statusP = G(statusArg);
    const SBMP_GAS uint4* const rngAP = G(rngAArg);
    const SBMP_GAS uint2* const rngBP = G(rngBArg);
    const SBMP_GAS unsigned long long* const gnewP = G(gnewArg);
    SBMP_STAMP(0);

    // ---- loads that depend on nothing else (the control block as a plain load: a
    // waiting scalar load would serialise behind the scan)
    const int4 pk = G(cnt4)[tid];
    const IterCtrl pc = *ctrlP;
    C16Load c16;   // sharded: the u16 block counts of every row (row positions, inserts)
    if constexpr (SH) c16 = c16_issue(d);
    const int goalIdx = statusP->goalIdx;
    const uint4 ra = rngAP[slot];
    const uint2 rb = rngBP[slot];
    const unsigned long long oldWord = (lane == 0) ? gnewP[slot >> 6] : 0ull;
    asm volatile("" ::"s"(d.M), "s"(d.nBlocks), "s"(d.numIterations), "s"(d.numDisc), "s"(d.nR1), "s"(d.nR2),
                 "s"(d.cap), "s"(d.fixGNewClear), "s"(d.batchRule), "s"(d.rcpNumDisc), "s"(d.treeState),
                 "s"(d.treeCtrl), "s"(d.stepList));
    float4 obsReg = make_float4(0.f, 0.f, 0.f, 0.f);
    if (kLdsObs && tid < d.nObs) obsReg = G(d.obstacles)[tid];
    // register lists: box (lane % n) for the per-step schedule (car_schedule)
    float4 oLane = make_float4(0.f, 0.f, 0.f, 0.f);
    if (AGENT == 0 && kRegObs > 0) oLane = G(d.obstacles)[lane % (kRegObs > 0 ? kRegObs : 1)];
    sR1P[tid] = 0;   // nR1 == kBlock
    if (nW <= 2 * kBlock) {   // n <= 8 (uniform): two fixed stores, no loop
        if (tid < nW) sNew[tid] = 0u;
        if (tid + kBlock < nW) sNew[tid + kBlock] = 0u;
    } else {
        for (int i = tid; i < nW; i += kBlock) sNew[i] = 0u;
    }
    // ---- the child's controls (statePropagator.cu:17-21) depend on the slot's stream
    // alone.  Drawn after the count scan (round 6): waves 1-3 while wave 0 plans, wave 0
    // right after the plan's barrier.  Drawn before the scan (rounds 3-5) they held the
    // scan behind the XORWOW states' arrival, the launch's 6.3 MB burst, although the
    // 4-KB counts arrive first: count scan done 2.02 -> 1.32 us p50, every later phase
    // ~0.55 us earlier (profiles/r06/prologue/).
    Xorwow rs{ra.x, ra.y, ra.z, ra.w, rb.x, rb.y};
    ChildCtl ctl;
    auto draw = [&]() __attribute__((always_inline)) {
        ctl = draw_controls<AGENT>(rs, d);
        asm volatile("" : "+v"(ctl.a), "+v"(ctl.steer), "+v"(ctl.dur), "+v"(ctl.dt), "+v"(ctl.tanS));
    };
#if SBMP_VALU_DUP == 1   // diagnostics (VALU by part): the draw once more, on an opaque copy
    {
        Xorwow r2{ra.x, ra.y, ra.z, ra.w, rb.x, rb.y};
        asm volatile("" : "+v"(r2.v0), "+v"(r2.v1), "+v"(r2.v2), "+v"(r2.v3), "+v"(r2.v4), "+v"(r2.d));
        const ChildCtl c2 = draw_controls<AGENT>(r2, d);
        asm volatile("" ::"v"(c2.a), "v"(c2.steer), "v"(c2.dur), "v"(c2.dt), "v"(c2.tanS), "v"(r2.v4), "v"(r2.d));
    }
#endif
    int A, jGoal;
    // the control block and the goal index were loaded per lane (vector loads do not
    // wait behind the scan's scalar work); the plan is wave-uniform, so scalar code
    auto plan = [&]() {
        IterCtrl pcu = pc;
        pcu.executed = __builtin_amdgcn_readfirstlane(pc.executed);
        pcu.treeSize = __builtin_amdgcn_readfirstlane(pc.treeSize);
        pcu.gLo = __builtin_amdgcn_readfirstlane(pc.gLo);
        pcu.nExp = __builtin_amdgcn_readfirstlane(pc.nExp);
        pcu.H = __builtin_amdgcn_readfirstlane(pc.H);
        return step_plan(d, t, expand, pcu, __builtin_amdgcn_readfirstlane(goalIdx), A, jGoal);
    };
    StepPlan q;
    {
        if constexpr (SH) {
            int gRow;
            step_scan_rows(sv, pk, sPfx, sRed, &A, &gRow);
            c16_store(d, c16, sC16);   // published by the plan's barrier below
            if (gRow != kNoGoalIdx) __syncthreads();   // uniform (rare): row_goal reads sPfx[gRow]
            jGoal = row_goal(sv, sPfx, gRow);
        } else {
            step_scan(d, pk, sPfx, sRed, &A, &jGoal);
        }
        SBMP_STAMP(1);
        // One wave per workgroup computes the plan while the others write their prefix
        // entries; the barrier that publishes sPfx publishes the plan.  (Every wave
        // computing it kept the CU's one scalar unit busy for 16 waves at once.)
        if (wave == 0) {
            const StepPlan q0 = plan();
            if (lane == 0) sPlan = q0;
            // slot = g k + i for the first slot of each wave, one division for all four
            // (k >= 64: a wave's slots then span at most two frontier positions)
            if (lane < kBlock / kWave && q0.k >= kWave) {
                const int s0 = gb * kBlock + lane * kWave;
                const int g0 = slot_div(d, s0, q0.k);
                sWaveDiv[lane] = make_int2(g0, s0 - g0 * q0.k);
            }
        }
        else {   // waves 1-3 draw their controls while wave 0 plans
            draw();
        }
        __syncthreads();
        if (wave == 0) draw();
        q = uniform_plan(sPlan);
#ifdef SBMP_TL_PROLOGUE   // diagnostics: stamp 4 = after the plan's barrier (instead of the hand-off)
        SBMP_STAMP(4);
#endif
    }
    // the fused exchange's arrival (every exit of an expanding workgroup)
    auto fx_exit = [&]() {
        if constexpr (SH) {
            if (expand && d.fusedX) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's stores have completed
                __syncthreads();
                k_step_exchange(d, sv.nranks, sv.rank, sv.nRows, t);
            }
        }
    };
    // the workgroup's work; every exit of it then passes the fused exchange's arrival once
    auto body = [&]() __attribute__((always_inline)) {
    if (!q.ranPrev) return;

    // ---- D6 clear of this block's words of t-1 (KGMT.cu:231,556)
    const long long cleared = d.fixGNewClear ? (1ll << 62) : 32ll * q.grid;
    unsigned long long word = oldWord;
    if (d.fixGNewClear) {   // the complete clear: every word (uniform branch)
        word = 0ull;
    } else if (lane == 0) {
        const long long wbase = (long long)(slot >> 6) * kWave;
        if (wbase + kWave <= cleared) word = 0ull;
        else if (wbase < cleared) word = oldWord & ~((1ull << (cleared - wbase)) - 1ull);
    }
    const bool doExpand = q.executes && gb * kBlock < q.H;
    // ---- insert t-1: this block's flagged children (rows treeSize(t-1) + prefix +
    // index).  Each entry carries its cost, so this is one load and three stores; an
    // expanding block issues it right behind its parent loads (one round trip).
    const bool selfInsert = A > kPlannerInsertMax;   // else the planner workgroup inserts
    auto insert_block = [&](int lo, int j0, int cnt) {   // t-1's flagged children of global block lo: rows j0 ..
        if (tid < cnt) {
            const int j = j0 + tid;
            const int dst = q.tsPrev + j;
            if (j < q.nIns && dst < d.M) {   // D13: the reference writes past M here
                const SBMP_GAS float4* e = list_entry<SH>(d, pp, lo, tid);
                const float4 s4 = list_load<SH>(d, e);
                const float4 u4 = list_load<SH>(d, e + 1);
                const float4 m4 = list_load<SH>(d, e + 2);
                // written through (fewer dirty lines at the boundary); the V# based at row tsPrev keeps
                // the byte offset j * 16 far below 2^31 whatever M is
                store_wt(d.treeState + q.tsPrev, j, s4);
                store_wt(d.treeCtrl + q.tsPrev, j, make_float4(u4.x, u4.y, u4.z, m4.x));   // cost = parent's + duration (KGMT.cu:631-633)
                store_wt(d.treeParent + q.tsPrev, j, __float_as_int(u4.w));
            }
        }
    };
    auto insert_prev = [&]() {
        if (t > 1 && selfInsert) {
            if constexpr (SH) {   // every rank holds the whole tree: row b = blocks b P .. b P + P - 1
                // the row's entries over the workgroup's lanes (one round of loads for up to
                // 256 entries, whichever of the P blocks holds them)
                const int j0 = sPfx[b], tot = sPfx[b + 1] - j0;
                for (int o = tid; o < tot; o += kBlock) {
                    const int j = j0 + o, dst = q.tsPrev + j;
                    if (j < q.nIns && dst < d.M) {   // D13: the reference writes past M here
                        int blk, idx;
                        row_locate_any(d, sv, sC16, b, o, &blk, &idx);
                        const SBMP_GAS float4* e = list_entry<SH>(d, pp, blk, idx);
                        const float4 s4 = list_load<SH>(d, e);
                        const float4 u4 = list_load<SH>(d, e + 1);
                        const float4 m4 = list_load<SH>(d, e + 2);
                        store_wt(d.treeState + q.tsPrev, j, s4);
                        store_wt(d.treeCtrl + q.tsPrev, j, make_float4(u4.x, u4.y, u4.z, m4.x));
                        store_wt(d.treeParent + q.tsPrev, j, __float_as_int(u4.w));
                    }
                }
            } else {
                insert_block(b, sPfx[b], sPfx[b + 1] - sPfx[b]);
            }
        }
    };
    if (!doExpand) {
        insert_prev();
        if (lane == 0 && word != oldWord) store_wt(d.gnewOut, slot >> 6, word);
        return;
    }

    // ---- expand t
    const bool act = slot < q.S;
    int g;   // slot = g*k + i
    if (q.k >= kWave) {
        const int2 gr = sWaveDiv[wave];
        g = gr.x + ((gr.y + lane >= q.k) ? 1 : 0);
    } else {
        g = slot_div(d, slot, q.k);
    }
    g = act ? g : 0;
    const int parent = act ? q.gLo + g : 0;
    const SBMP_GAS float4* src = G(d.treeState) + parent;   // the parent's state, and its cost
    const SBMP_GAS float* srcCost = &G(d.treeCtrl)[parent].w;
    // A parent inserted by t-1 is read from its block's compacted list: block lo with
    // sPfx[lo] <= j < sPfx[lo + 1].  j grows with the lane; when a wave's parents are
    // at most two consecutive list positions jA, jB (k >= 32 children per parent) both
    // are found by a two-level 32-ary ballot search (lanes 0-31 for jA, 32-63 for jB):
    // two dependent LDS reads instead of log2(nBlocks).
    const bool fromList = parent >= q.tsPrev;
    const int j = parent - q.tsPrev;
    const unsigned long long need = __ballot(fromList);
    const int nS = SH ? sv.nRows : d.nBlocks;   // scan entries: blocks, or (sharded) rows
    // the list block lo of this lane's position j (the wave's positions: `need`)
    auto find_lo = [&](const int j, const bool fromList, const unsigned long long need) __attribute__((always_inline)) {
        const int jA = __builtin_amdgcn_readlane(j, (int)__builtin_ctzll(need));
        const int jB = __builtin_amdgcn_readlane(j, 63 - (int)__builtin_clzll(need));
        int lo = 0;
        if (jB - jA <= 1) {
            const int jj = (lane < 32) ? jA : jB;
            const int sub = lane & 31;
            int idx = sub * 32;
            unsigned long long m = __ballot((idx < nS ? sPfx[idx] : INT_MAX) <= jj);
            const int cA = __popcll(m & 0xffffffffull) - 1, cB = __popcll(m >> 32) - 1;
            idx = ((lane < 32) ? cA : cB) * 32 + sub;
            m = __ballot((idx < nS ? sPfx[idx] : INT_MAX) <= jj);
            lo = (j == jA) ? cA * 32 + __popcll(m & 0xffffffffull) - 1 : cB * 32 + __popcll(m >> 32) - 1;
        } else {
            // k < 64: the wave's positions jA .. jB are consecutive and span a couple of
            // blocks (a block holds A / nBlocks > 4 of them on average), so the block of jA
            // by the same 32-ary ballot search, then each lane steps forward (was a
            // 10-step binary search per lane: iterations 2-10 of the c3 window)
            const int sub = lane & 31;
            int idx = sub * 32;
            unsigned long long m = __ballot((idx < nS ? sPfx[idx] : INT_MAX) <= jA);
            const int c = __popcll(m & 0xffffffffull) - 1;
            idx = c * 32 + sub;
            m = __ballot((idx < nS ? sPfx[idx] : INT_MAX) <= jA);
            lo = c * 32 + __popcll(m & 0xffffffffull) - 1;
            if (fromList)
                while (lo + 1 < nS && sPfx[lo + 1] <= j) ++lo;
        }
        return lo;
    };
    if (need) {
        const int lo = find_lo(j, fromList, need);
#if SBMP_VALU_DUP == 2   // diagnostics (VALU by part): the search once more, on opaque copies
        {
            int j2 = j;
            asm volatile("" : "+v"(j2));
            asm volatile("" ::"v"(find_lo(j2, fromList, need)));
        }
#endif
        if (fromList) {
            if constexpr (SH) {   // the row's blocks: from the LDS table (round 4: one more L2 round trip)
                int blk, idx;
                row_locate_any(d, sv, sC16, lo, j - sPfx[lo], &blk, &idx);
                src = list_entry<SH>(d, pp, blk, idx);
            } else {
                src = list_entry<SH>(d, pp, lo, j - sPfx[lo]);
            }
            srcCost = reinterpret_cast<const SBMP_GAS float*>(src + 2);
        }
    }
#ifdef SBMP_TL_PROLOGUE   // stamp 5 = parent located (instead of the epilogue barrier)
    SBMP_STAMP(5);
#endif
    // Parent and obstacles are issued back to back and waited for together.
    float4 p;
    float parentCost;
    if (SH && fromList && !d.listPlain) {   // the owner's list over the mapping: system-scope loads
        p = load_record_g(src);
        parentCost = load_record_g(src + 2).x;
    } else {
        p = *src;
        parentCost = *srcCost;
    }
    float4 ro[kRegObs > 0 ? kRegObs : 1];
#pragma unroll
    for (int i = 0; i < kRegObs; ++i) ro[i] = G(d.obstacles)[i];
    insert_prev();
    if (kLdsObs) {
        if (tid < d.nObs) sObs[tid] = obsReg;
        for (int i = tid + kBlock; i < d.nObs; i += kBlock) sObs[i] = G(d.obstacles)[i];
        __syncthreads();
    }
    // the grid index's cell-start table into LDS: every row lookup of the Euler loop is
    // then an LDS read instead of an L2 round trip (the boxes stay in global memory)
    int* const sGridStart =
        SH ? reinterpret_cast<int*>(sC16 + (d.c16Lds ? ((d.nBlocks + 7) & ~7) : 0)) : reinterpret_cast<int*>(sNew + nW);
    if constexpr (OBS == kObsGrid) {
        const int nStart = d.gridG * d.gridG + 1;
        const SBMP_GAS int* const gs = G(d.gridStart);
        for (int i = tid; i < nStart; i += 4 * kBlock) {
            int v[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) v[u] = (i + u * kBlock < nStart) ? gs[i + u * kBlock] : 0;
#pragma unroll
            for (int u = 0; u < 4; ++u)
                if (i + u * kBlock < nStart) sGridStart[i + u * kBlock] = v[u];
        }
        __syncthreads();
    }
    SBMP_STAMP(2);
    const float4* obs = (kRegObs > 0) ? ro : kLdsObs ? sObs : d.obstacles;
    ChildOut out;
    bool valid = false;
    // The fast loop runs on every lane, outside any divergent branch, so its lane masks
    // need no merging with exec: inactive lanes (slots >= S) propagate row 0 with
    // controls from their unused stream, and their result is dropped.
    bool fast = false;
    if constexpr (AGENT == 0 && kRegObs > 0) {
        fast = car_fast_ok(d);   // per plan (uniform)
        if (fast) {
            // a huge steering tan can drive theta past Cody-Waite's range within a child
            const StepSched sched = car_schedule<OBS>(p, parent, act, d, oLane);
#if SBMP_VALU_DUP == 3   // diagnostics: the schedule and the theta bound once more, on opaque copies
            {
                float4 p2 = p;
                asm volatile("" : "+v"(p2.x), "+v"(p2.y), "+v"(p2.z), "+v"(p2.w));
                const StepSched s2 = car_schedule<OBS>(p2, parent, act, d, oLane);
                const unsigned long long tb = __ballot(!car_theta_bounded(p2, ctl, d));
                asm volatile("" ::"s"(s2.boxes), "s"(s2.bounds), "s"(tb));
            }
#endif
            WaveCull cull{~0u, true};   // the schedule covers the whole reach
            if (!sched.valid) cull = car_cull<OBS>(p, ctl, d, obs);
            if (__ballot(!car_theta_bounded(p, ctl, d)) != 0ull)   // rare: Payne-Hanek per lane
                valid = car_euler_fast<OBS, true>(p, ctl, d, obs, cull, sched, out) && act;
            else if (d.invAgentLength == 1.0f)   // per plan (uniform): L = 1, one multiply less per step
                valid = car_euler_fast<OBS, false, true>(p, ctl, d, obs, cull, sched, out) && act;
            else
                valid = car_euler_fast<OBS, false>(p, ctl, d, obs, cull, sched, out) && act;
        }
    }
    if (!fast) {
        out = ChildOut{};   // inactive lanes: defined values (the fast loop writes every lane)
        if (act)
            valid = (AGENT == 0)
                        ? car_euler<OBS, NoMidHook, OBS == kObsGrid>(p, ctl, d, obs, out, NoMidHook(), sGridStart)
                        : point_euler<OBS, NoMidHook, OBS == kObsGrid>(p, ctl, d, obs, out, NoMidHook(), sGridStart);
    }
    SBMP_STAMP(3);

    // ---- bins (KGMT.cu:390-391) and the accept test (KGMT.cu:394-411, D2)
    int q1 = -1, q2 = -1;
    if (act) bins_k(out.state.x, out.state.y, d, &q1, &q2);   // N = 16 (KGMT.cu:8)
#if SBMP_VALU_DUP == 4   // diagnostics: the binning once more, on opaque copies
    if (act) {
        float x2 = out.state.x, y2 = out.state.y;
        asm volatile("" : "+v"(x2), "+v"(y2));
        int a2, b2;
        bins_k(x2, y2, d, &a2, &b2);
        asm volatile("" ::"v"(a2), "v"(b2));
    }
#endif
    // The planner workgroup publishes iteration t's scores and snapshot as 8-B words
    // tagged with t (step_planner); each lane that takes the test reads its two words
    // from L2 now, and the stores below overlap that round trip.  q2 >= 0 implies q1 >= 0.
    const bool look = act && valid && q2 >= 0;
    unsigned long long sw = 0ull, aw = 0ull;
    if (look) {
        // Plain loads (the first try; agent-scope loads measured 0.1-0.3 us slower per
        // launch): the first wave of an XCD to load a line after the planner published
        // brings it into that XCD's L2 and later waves hit there instead of each going
        // to memory; a line loaded before publication carries an older tag, and the
        // re-read below (agent scope, past this CU's caches) corrects it.
        // (relaxed atomic loads at workgroup scope: the same plain, cacheable global_load,
        // without the data race a plain load of a word another workgroup stores would be)
        sw = __hip_atomic_load(pubCur + q1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        aw = __hip_atomic_load(pubCur + d.nR1 + (q2 >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
    float u = 0.0f;
    if (valid) u = xorwow_uniform(rs);   // KGMT.cu:395 (valid implies act)
    // this slot's child (state, ctrl); meaningless on inactive lanes, which store nothing
    // (a stale flag past S re-reads its child below)
    float4 cs = out.state;
    float4 cc = make_float4(out.a, out.steer, out.dur, __int_as_float(parent));
    float cost = parentCost + out.dur;   // getCost (KGMT.cu:631-633), as the insert computes it
    if (act) {
        store_wt(d.uState, slot, cs);   // write-through: fewer dirty lines at the boundary
        store_wt(d.uCtrl, slot, cc);
        store_wt(d.rngA, slot, make_uint4(rs.v0, rs.v1, rs.v2, rs.v3));
        store_wt(d.rngB, slot, make_uint2(rs.v4, rs.d));
        if (q1 >= 0) atomicAdd(&sR1P[q1], valid ? 1 : 0x10000);
        if (d.r2log) {
            store_wt(d.r2log, (t % kFoldEvery) * d.logSlots + b * kBlock + tid,
                     (q2 >= 0) ? (uint16_t)(q2 | (valid ? 0x8000 : 0)) : kNoKey);
        } else if (q2 >= 0) {
            __hip_atomic_fetch_add(G(valid ? d.R2Valid : d.R2Invalid) + q2, 1, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
    }
    {   // tags must read t; a word read before the planner published it is re-read (bounded)
        const unsigned want = (unsigned)t;
        bool stale = look && (((unsigned)(sw >> 32) != want) | ((unsigned)(aw >> 32) != want));
        if (__ballot(stale) != 0ull) {
            const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
            for (;;) {
                __builtin_amdgcn_s_sleep(8);
                if (stale) {
                    sw = __hip_atomic_load(pubCur + q1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    aw = __hip_atomic_load(pubCur + d.nR1 + (q2 >> 5), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    stale = ((unsigned)(sw >> 32) != want) | ((unsigned)(aw >> 32) != want);
                }
                if (__ballot(stale) == 0ull) break;
                if ((long long)__builtin_amdgcn_s_memrealtime() - t0 > kStepWaitTicks) {   // give up, report
                    if (stale)
                        __hip_atomic_exchange(&G(d.status)->error, kErrStepHandoff, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT);
                    break;
                }
            }
        }
    }
    bool accept = false;
    if (look) {
        const uint32_t bit = 1u << (q2 & 31);
        const bool r2Avail = (uint32_t)aw & bit;
        accept = (u <= __uint_as_float((uint32_t)sw)) || !r2Avail;
        if (!r2Avail) atomicOr(&sNew[q2 >> 5], bit);
    }
#ifndef SBMP_TL_PROLOGUE
    SBMP_STAMP(4);
#endif
    const unsigned long long mask = __ballot(accept);
    const unsigned long long word0 =   // lane 0's word
        ((unsigned long long)(uint32_t)__builtin_amdgcn_readlane((int)(word >> 32), 0) << 32) |
        (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)word, 0);
    const unsigned long long wordAll = word0 | mask;   // GNew |= accept (stale bits survive)
    const bool flagged = __builtin_amdgcn_inverse_ballot_w64(wordAll);   // this lane's bit of wordAll (a lane mask)
    if ((wordAll & ~__ballot(act)) != 0ull) {   // rare; keeps the wait below off the common path
        if (flagged && !act) {   // a stale flag on a slot past S: the child last written there
            cs = G(d.uState)[slot];
            cc = G(d.uCtrl)[slot];
            cost = G(d.treeCtrl)[__float_as_int(cc.w)].w + cc.z;
        }
    }
    bool inGoal = false;
    if (flagged && d.goalThreshold > 0.0f) {   // sqrtf(.) < r is false for every r <= 0 (and NaN)
        const float dx = cs.x - d.goalX, dy = cs.y - d.goalY;   // inGoalRegion, KGMT.cu:635-638
        inGoal = __builtin_sqrtf(dx * dx + dy * dy) < d.goalThreshold;
    }
    // index among the wave's flagged slots; the first goal child is the wave's lowest
    const int idxW = __builtin_amdgcn_mbcnt_hi((uint32_t)(wordAll >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)wordAll, 0u));
    const int glW = first_lane_value(flagged && inGoal, idxW, kNoGoalIdx);
    if (lane == 0) {
        store_wt(d.gnewOut, slot >> 6, wordAll);
        sWaveCnt[wave] = __popcll(wordAll);
        sWaveGoal[wave] = glW;
    }
    __syncthreads();
#ifndef SBMP_TL_PROLOGUE
    SBMP_STAMP(5);
#endif
    const int c0 = sWaveCnt[0], c1 = sWaveCnt[1], c2 = sWaveCnt[2], c3 = sWaveCnt[3];
    const int waveOff = (wave > 0 ? c0 : 0) + (wave > 1 ? c1 : 0) + (wave > 2 ? c2 : 0);
    if (flagged) {
        if constexpr (SH) {   // this rank's list of owned block b
            SBMP_GAS float4* e = G(d.recOut) + ((size_t)cp * d.recCap + (size_t)b * kBlock + waveOff + idxW) * kStepEntry;
            if (d.stepMirror) {   // into every rank's list mirror (global block gb), over xGMI for peers
                const size_t m = ((size_t)cp * d.nBlocks * kBlock + (size_t)gb * kBlock + waveOff + idxW) * kStepEntry;
                for (int q = 0; q < sv.nranks; ++q) {
                    SBMP_GAS float4* mq = G(d.mirrorPeer[q]) + m;
                    store_record_g(mq, cs);
                    store_record_g(mq + 1, cc);
                    store_record_g(mq + 2, make_float4(cost, 0.0f, 0.0f, 0.0f));
                }
            } else if (d.listPlain) {   // read on this GPU after this launch (a local group)
                e[0] = cs;
                e[1] = cc;
                e[2] = make_float4(cost, 0.0f, 0.0f, 0.0f);
            } else {             // read by the peers over the mapping: written through
                store_record_g(e, cs);
                store_record_g(e + 1, cc);
                store_record_g(e + 2, make_float4(cost, 0.0f, 0.0f, 0.0f));
            }
        } else {
#ifdef SBMP_SOFFSET_DEMO   // the round-3 form of these stores (kgmt_device.h, SBMP_WT_OFF)
            const __amdgpu_buffer_rsrc_t rl = wt_rsrc(d.stepList);
            const int so = __builtin_amdgcn_readfirstlane(((cp * d.nBlocks + b) * kBlock) * kStepEntry * 16);
            const int vo = (waveOff + idxW) * kStepEntry * 16;
            __builtin_amdgcn_raw_buffer_store_b128(sbmp_u32x4{__float_as_uint(cs.x), __float_as_uint(cs.y), __float_as_uint(cs.z), __float_as_uint(cs.w)}, rl, vo, so, 0);
            __builtin_amdgcn_raw_buffer_store_b128(sbmp_u32x4{__float_as_uint(cc.x), __float_as_uint(cc.y), __float_as_uint(cc.z), __float_as_uint(cc.w)}, rl, vo + 16, so, 0);
            __builtin_amdgcn_raw_buffer_store_b128(sbmp_u32x4{__float_as_uint(cost), 0u, 0u, 0u}, rl, vo + 32, so, 0);
#else
            // < 2^27 entries; the row part is uniform, the lane part a 24-bit multiply (full rate)
            const int e = (cp * d.nBlocks + b) * kBlock * kStepEntry + (int)__umul24((unsigned)(waveOff + idxW), (unsigned)kStepEntry);
            store_wt(d.stepList, e, cs);
            store_wt(d.stepList, e + 1, cc);
            store_wt(d.stepList, e + 2, make_float4(cost, 0.0f, 0.0f, 0.0f));
#endif
        }
    }
    {   // one 64-bit atomic per touched cell, into this workgroup's replica
        SBMP_GAS unsigned long long* const rep =
            (SH ? G(d.stepXs[cp]) : G(d.stepDelta) + (size_t)(t % 3) * kDeltaReps * d.nR1) + (size_t)(b % kDeltaReps) * d.nR1;
        const int v = sR1P[tid];   // nR1 == kBlock
        if (v)
            __hip_atomic_fetch_add(rep + tid, (unsigned long long)(v & 0xffff) | ((unsigned long long)(v >> 16) << 32),
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if constexpr (SH) {   // R2New as bytes of the exchange (a sum over ranks), one store per cell the block saw
        SBMP_GAS uint8_t* const nb = reinterpret_cast<SBMP_GAS uint8_t*>(G(d.stepXs[cp]) + d.xNewOff);
        for (int i = tid; i < nW; i += kBlock) {
            uint32_t w = sNew[i];
            while (w) {   // written through (sc1): the fused exchange reads them in this launch
                __hip_atomic_store(nb + 32 * i + __builtin_ctz(w), (uint8_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                w &= w - 1u;
            }
        }
    } else {
        // replicas: a device atomic on one word serialises (~11 ns each); in the early
        // iterations most blocks set the same few words, so each replica sees 1/kNewReps
        SBMP_GAS uint32_t* const newCur = G(d.stepR2New) + ((size_t)(t % 3) * kNewReps + (size_t)(b % kNewReps)) * nW;
        if (nW <= 2 * kBlock) {   // n <= 8 (uniform): both words' LDS reads, then their atomics
            const uint32_t w0 = tid < nW ? sNew[tid] : 0u, w1 = tid + kBlock < nW ? sNew[tid + kBlock] : 0u;
            if (w0) __hip_atomic_fetch_or(newCur + tid, w0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (w1) __hip_atomic_fetch_or(newCur + tid + kBlock, w1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        } else {
            for (int i = tid; i < nW; i += kBlock) {
                const uint32_t w = sNew[i];
                if (w) __hip_atomic_fetch_or(newCur + i, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        }
    }
    if (tid == 0) {   // the block's flagged count and its lowest goal child (in-block index)
        const int g0 = sWaveGoal[0], g1 = sWaveGoal[1], g2 = sWaveGoal[2], g3 = sWaveGoal[3];
        int gmin = kNoGoalIdx;
        if (g3 != kNoGoalIdx) gmin = c0 + c1 + c2 + g3;
        if (g2 != kNoGoalIdx) gmin = c0 + c1 + g2;
        if (g1 != kNoGoalIdx) gmin = c0 + g1;
        if (g0 != kNoGoalIdx) gmin = g0;
        const int cw = (c0 + c1 + c2 + c3) | ((gmin == kNoGoalIdx ? 0 : gmin + 1) << 16);
        if constexpr (SH) {   // the block word, and this rank's part of row b (the exchange sums the row); sc1
            __hip_atomic_store(reinterpret_cast<SBMP_GAS int*>(G(d.stepXs[cp]) + d.xCntOff) + gb, cw, __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_store(reinterpret_cast<SBMP_GAS int*>(G(d.stepXs[cp]) + d.xRowOff) + b,
                               (c0 + c1 + c2 + c3) | ((gmin == kNoGoalIdx ? 0 : 1) << 16), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_AGENT);
            // the count again as u16 (the summed exchange forms carry it; the compact one rebuilds it)
            store_wt(reinterpret_cast<uint16_t*>(d.stepXs[cp] + d.xC16Off), gb, (uint16_t)(c0 + c1 + c2 + c3));
        }
        else store_wt(d.stepCnt, cp * kMaxStepBlocks + b, cw);
    }
    SBMP_STAMP(6);
    if (tl) {
        unsigned hw, xcc;
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
        asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
        stamp[7] = ((long long)xcc << 32) | hw;
    }
    if (tl && lane == 0)
        for (int i = 0; i < kTimelineStamps; ++i) G(tl)[i] = stamp[i];
    };
    body();
    fx_exit();
#undef SBMP_STAMP
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

// Holds the stream for `ticks` of the 100 MHz constant clock (bounded by
// construction), so launches queued behind it run back to back.
__global__ void k_delay(long long ticks) {
    if (threadIdx.x != 0) return;
    const long long t0 = (long long)__builtin_amdgcn_s_memrealtime();
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(127);
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
    d.status->error = 0;
}

// A 64-bit digest of the replicated planning state (bench.py --gpus N checks that every
// rank's is the same): tree rows [0, rows) (state, controls + cost,
// parent), the five R1 tables and the R2 availability bits of parity tp, and the
// iteration control blocks [1, iters].  Order-independent: the sum (mod 2^64) of a
// splitmix64 of (array tag, index, 32-bit word) over every word, so grid shape and
// atomic order do not matter.
__device__ __forceinline__ unsigned long long hash_word(unsigned long long tag, unsigned long long i, uint32_t w) {
    unsigned long long z = (tag << 56) ^ (i << 24) ^ (unsigned long long)w ^ (i >> 40);
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}
__global__ void k_state_hash(KgmtDev d, int rows, int tp, int iters, unsigned long long* out) {
    unsigned long long acc = 0ull;
    const long long stride = (long long)gridDim.x * blockDim.x;
    const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    for (long long i = tid; i < rows; i += stride) {
        const float4 s4 = d.treeState[i], c4 = d.treeCtrl[i];
        const uint32_t w[9] = {__float_as_uint(s4.x), __float_as_uint(s4.y), __float_as_uint(s4.z),
                               __float_as_uint(s4.w), __float_as_uint(c4.x), __float_as_uint(c4.y),
                               __float_as_uint(c4.z), __float_as_uint(c4.w), (uint32_t)d.treeParent[i]};
        for (int k = 0; k < 9; ++k) acc += hash_word(1 + k, (unsigned long long)i, w[k]);
    }
    const int* tab = d.R1 + (size_t)tp * 5 * d.nR1;
    for (long long i = tid; i < 5 * d.nR1; i += stride) acc += hash_word(16, (unsigned long long)i, (uint32_t)tab[i]);
    const uint32_t* av = d.R2Avail + (size_t)tp * (d.nR2 / 32);
    for (long long i = tid; i < d.nR2 / 32; i += stride) acc += hash_word(17, (unsigned long long)i, av[i]);
    const int* cw = reinterpret_cast<const int*>(d.ctrl);
    for (long long i = tid; i < (long long)iters * 16; i += stride)   // IterCtrl = 16 words; entries 1 .. iters
        if ((i & 15) < 11) acc += hash_word(18, (unsigned long long)i, (uint32_t)cw[16 + i]);
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off, 64);
    if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}
void launch_state_hash(const KgmtDev& d, int rows, int tp, int iters, unsigned long long* out, hipStream_t s) {
    hipLaunchKernelGGL(k_state_hash, dim3(1024), dim3(256), 0, s, d, rows, tp, iters, out);
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

// Solution path: rows root .. node by walking treeParent, root
// first.  One thread; the depth is bounded by maxDepth (parent[j] < j, and every
// iteration adds at most one level); out[0] = length, or -1 if the walk did not
// reach the root within maxDepth rows.  rows/samples/costs hold maxDepth rows.
__global__ void k_solution_path(KgmtDev d, int node, int maxDepth, int* out, int* rows, float* samples,
                                float* costs) {
    if (threadIdx.x != 0 || blockIdx.x != 0) return;
    int depth = 0;
    for (int j = node; j >= 0; j = d.treeParent[j]) {
        if (++depth > maxDepth) {
            out[0] = -1;
            return;
        }
    }
    out[0] = depth;
    int k = depth - 1;
    for (int j = node; j >= 0; j = d.treeParent[j], --k) {
        const float4 st = d.treeState[j];
        const float4 c = d.treeCtrl[j];
        rows[k] = j;
        float* o = samples + (size_t)k * 7;
        o[0] = st.x; o[1] = st.y; o[2] = st.z; o[3] = st.w;
        o[4] = c.x; o[5] = c.y; o[6] = c.z;
        costs[k] = c.w;
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
// With timing events, hipExtLaunchKernelGGL stamps them from the kernel's own
// dispatch packet (start/end of execution, as rocprofv3's kernel trace does);
// events recorded as separate stream packets would add the dispatch latency.
template <typename K, typename... Args>
static void launch(K kernel, dim3 grid, dim3 block, size_t shm, hipStream_t s, const KernelTiming& tm,
                   Args... args) {
    if (tm.start)
        hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)shm, s, tm.start, tm.stop, 0u, args...);
    else
        hipLaunchKernelGGL(kernel, grid, block, shm, s, args...);
}

template <int AGENT>
static void launch_expand_reg(const KgmtDev& d, int t, dim3 grid, dim3 block, hipStream_t s, const KernelTiming& tm) {
    switch (d.nObs) {   // the box count is a compile-time constant of the register path
        case 0: launch(k_expand<AGENT, kObsReg + 0>, grid, block, 0, s, tm, d, t); break;
        case 1: launch(k_expand<AGENT, kObsReg + 1>, grid, block, 0, s, tm, d, t); break;
        case 2: launch(k_expand<AGENT, kObsReg + 2>, grid, block, 0, s, tm, d, t); break;
        case 3: launch(k_expand<AGENT, kObsReg + 3>, grid, block, 0, s, tm, d, t); break;
        case 4: launch(k_expand<AGENT, kObsReg + 4>, grid, block, 0, s, tm, d, t); break;
        case 5: launch(k_expand<AGENT, kObsReg + 5>, grid, block, 0, s, tm, d, t); break;
        case 6: launch(k_expand<AGENT, kObsReg + 6>, grid, block, 0, s, tm, d, t); break;
        case 7: launch(k_expand<AGENT, kObsReg + 7>, grid, block, 0, s, tm, d, t); break;
        default: launch(k_expand<AGENT, kObsReg + 8>, grid, block, 0, s, tm, d, t); break;
    }
}

template <int AGENT>
static void launch_expand_agent(const KgmtDev& d, int t, int blocks, int variant, hipStream_t s,
                                const KernelTiming& tm) {
    const size_t shm = sizeof(float4) * (size_t)d.nObs;
    const dim3 grid(blocks), block(kBlock);
    if (d.gridStart) {   // the planner built the grid index (large lists, or variant 4)
        launch(k_expand<AGENT, kObsGrid>, grid, block, 0, s, tm, d, t);
    } else if (d.nObs > kMaxLdsObs) {
        launch(k_expand<AGENT, kObsGlobal>, grid, block, 0, s, tm, d, t);
    } else if (d.nObs <= kMaxRegObs && (variant == 0 || variant == 3)) {
        launch_expand_reg<AGENT>(d, t, grid, block, s, tm);
    } else if (variant == 2) {
        launch(k_expand<AGENT, kObsLds4>, grid, block, shm, s, tm, d, t);
    } else {
        launch(k_expand<AGENT, kObsLds>, grid, block, shm, s, tm, d, t);
    }
}

void launch_expand(const KgmtDev& d, int t, int agent, int blocks, int variant, hipStream_t s,
                   const KernelTiming& tm) {
    if (agent == 0) launch_expand_agent<0>(d, t, blocks, variant, s, tm);
    else launch_expand_agent<1>(d, t, blocks, variant, s, tm);
}

// k_step's dynamic LDS past the obstacle list: the block (row) prefix and the R2New bits;
// on a sharded rank also the u16 block counts of every row, 16-B aligned (the kernel's
// sC16 / sGridStart layout).
static size_t step_lds_bytes(const KgmtDev& d, bool sh) {
    const size_t nS = sh ? d.nBlocks / d.nranks : d.nBlocks;   // scan entries: blocks, or rows
    size_t b = sizeof(int) * (nS + 1) + sizeof(uint32_t) * (size_t)(d.nR2 / 32);
    if (sh) b = ((b + 15) & ~(size_t)15) + (d.c16Lds ? sizeof(uint16_t) * (((size_t)d.nBlocks + 7) & ~(size_t)7) : 0);
    return b;
}

template <int AGENT, bool SH>
static void launch_step_form(const KgmtDev& d, int t, int expand, int variant, hipStream_t s,
                             const KernelTiming& tm) {
    // dynamic LDS: [LDS obstacles][block prefix: nBlocks + 1 ints][R2New bits: nR2 / 32 words]
    // (sharded: [16-B aligned u16 block counts]) [grid cell starts]
    const size_t pfx = step_lds_bytes(d, SH);
    const size_t shm = sizeof(float4) * (size_t)d.nObs + pfx;   // LDS obstacle forms
    const size_t gridLds = d.gridStart ? sizeof(int) * ((size_t)d.gridG * d.gridG + 1) : 0;   // + the cell starts
    const int blocks = SH ? d.nBlocks / d.nranks : d.nBlocks;
    const dim3 grid(1 + blocks), block(kBlock);   // workgroup 0 plans, 1.. expand
    long long* const tlBase = (d.timeline && t == d.timelineIter && expand) ? d.timeline : nullptr;
    const int4* const cnt4 = SH ? reinterpret_cast<const int4*>(d.stepXr + d.xRowOff)
                                : reinterpret_cast<const int4*>(d.stepCnt + (size_t)((t - 1) & 1) * kMaxStepBlocks);
#define SBMP_STEP_ARGS                                                                                        \
    d.devSelf, (int)((unsigned)t | ((unsigned)(expand != 0) << 31)), SH ? (d.rank | (d.nranks << 8)) : (1 << 8),  \
        cnt4, d.ctrl + (t - 1), d.rngA, d.rngB, d.gnewOut, d.status, tlBase, SH ? d.nBlocks / d.nranks : d.nBlocks, \
        SH ? reinterpret_cast<const int*>(d.stepXr + d.xCntOff) : nullptr
    if (d.gridStart) {
        launch(k_step<AGENT, kObsGrid, SH>, grid, block, pfx + gridLds, s, tm, SBMP_STEP_ARGS);
    } else if (d.nObs > kMaxLdsObs) {
        launch(k_step<AGENT, kObsGlobal, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS);
    } else if (d.nObs <= kMaxRegObs && (variant == 0 || variant == 3)) {
        switch (d.nObs) {
            case 0: launch(k_step<AGENT, kObsReg + 0, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
            case 1: launch(k_step<AGENT, kObsReg + 1, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
            case 2: launch(k_step<AGENT, kObsReg + 2, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
            case 3: launch(k_step<AGENT, kObsReg + 3, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
            case 4: launch(k_step<AGENT, kObsReg + 4, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
            case 5: launch(k_step<AGENT, kObsReg + 5, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
            case 6: launch(k_step<AGENT, kObsReg + 6, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
            case 7: launch(k_step<AGENT, kObsReg + 7, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
            default: launch(k_step<AGENT, kObsReg + 8, SH>, grid, block, pfx, s, tm, SBMP_STEP_ARGS); break;
        }
    } else if (variant == 2) {
        launch(k_step<AGENT, kObsLds4, SH>, grid, block, shm, s, tm, SBMP_STEP_ARGS);
    } else {
        launch(k_step<AGENT, kObsLds, SH>, grid, block, shm, s, tm, SBMP_STEP_ARGS);
    }
#undef SBMP_STEP_ARGS
}

// The k_step instantiation launch_step_form picks, and its dynamic LDS, for the
// residency check (step_resident_groups).
using StepFn = void (*)(const KgmtDev*, int, int, const int4*, const IterCtrl*, const uint4*, const uint2*,
                        const unsigned long long*, const PlannerStatus*, long long*, int, const int*);
template <int AGENT, bool SH>
static StepFn step_fn(const KgmtDev& d, int variant, size_t* shm) {
    const size_t pfx = step_lds_bytes(d, SH);
    *shm = pfx;
    if (d.gridStart) {
        *shm = pfx + sizeof(int) * ((size_t)d.gridG * d.gridG + 1);   // + the cell-start table (k_step stages it)
        return k_step<AGENT, kObsGrid, SH>;
    }
    if (d.nObs > kMaxLdsObs) return k_step<AGENT, kObsGlobal, SH>;
    if (d.nObs <= kMaxRegObs && (variant == 0 || variant == 3)) {
        switch (d.nObs) {
            case 0: return k_step<AGENT, kObsReg + 0, SH>;
            case 1: return k_step<AGENT, kObsReg + 1, SH>;
            case 2: return k_step<AGENT, kObsReg + 2, SH>;
            case 3: return k_step<AGENT, kObsReg + 3, SH>;
            case 4: return k_step<AGENT, kObsReg + 4, SH>;
            case 5: return k_step<AGENT, kObsReg + 5, SH>;
            case 6: return k_step<AGENT, kObsReg + 6, SH>;
            case 7: return k_step<AGENT, kObsReg + 7, SH>;
            default: return k_step<AGENT, kObsReg + 8, SH>;
        }
    }
    *shm = sizeof(float4) * (size_t)d.nObs + pfx;   // LDS obstacle forms
    return (variant == 2) ? k_step<AGENT, kObsLds4, SH> : k_step<AGENT, kObsLds, SH>;
}

int step_resident_groups(const KgmtDev& d, int agent, int variant, StepResidency* why) {
    size_t shm = 0;
    StepFn fn;
    if (agent == 0) fn = d.sharded ? step_fn<0, true>(d, variant, &shm) : step_fn<0, false>(d, variant, &shm);
    else fn = d.sharded ? step_fn<1, true>(d, variant, &shm) : step_fn<1, false>(d, variant, &shm);
    int dev = 0, cus = 0, perCU = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
    if (shm > 65536)   // LDS above 64 KB needs the opt-in (not reached by k_step's forms, kept for safety)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(fn), hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)shm);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, reinterpret_cast<const void*>(fn), kBlock, shm) !=
        hipSuccess)
        return 0;
    if (why) {
        why->perCU = perCU;
        why->cus = cus;
        why->dynLds = (long long)shm;
    }
    return perCU * cus;
}

template <int AGENT>
static void launch_step_agent(const KgmtDev& d, int t, int expand, int variant, hipStream_t s,
                              const KernelTiming& tm) {
    if (d.sharded) launch_step_form<AGENT, true>(d, t, expand, variant, s, tm);
    else launch_step_form<AGENT, false>(d, t, expand, variant, s, tm);
}

void launch_step(const KgmtDev& d, int t, int expand, int agent, int variant, hipStream_t s,
                 const KernelTiming& tm) {
    if (agent == 0) launch_step_agent<0>(d, t, expand, variant, s, tm);
    else launch_step_agent<1>(d, t, expand, variant, s, tm);
}

void launch_fold_r2(const KgmtDev& d, int tFirst, int tLast, hipStream_t s, const KernelTiming& tm) {
    if (!d.r2log || tLast < tFirst) return;
    const size_t shm = sizeof(uint32_t) * ((size_t)d.nR2 + kWave);
    if (shm > 65536)   // dynamic LDS above 64 KB needs the opt-in; per device, so every time
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_fold_r2),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)shm);
    // the iteration's keys split evenly (whole 8-key loads) over the fewest workgroups of
    // at most kFoldKeys each
    const int groups = (d.logSlots + kFoldKeys - 1) / kFoldKeys;
    const int per = (((d.logSlots + groups - 1) / groups) + 7) & ~7;
    const dim3 grid(groups, tLast - tFirst + 1);
    launch(k_fold_r2, grid, dim3(kFoldThreads), shm, s, tm, d, tFirst, per);
}

OneshotCompact oneshot_compact(const OneshotLayout& l) {
    OneshotCompact x{};
    x.nR1 = l.nR1;
    x.rowOff = l.rowOff;
    x.rowWords = (l.rows + 1) / 2;
    x.cntOff = l.cntOff;
    x.owned = l.owned;
    x.nBlocks = l.nBlocks;
    x.newOff = l.newOff;
    x.c16Off = l.c16Off;
    x.newWords = l.newWords;
    x.cR = x.nR1;
    x.cB = x.cR + x.rowWords;
    x.cN = x.cB + (x.owned + 1) / 2;
    x.total = x.cN + (x.newWords + 7) / 8;
    return x;
}

void launch_oneshot(unsigned long long* const* inbox, const unsigned long long* send, unsigned long long* recv,
                    long long n, int nranks, int rank, unsigned long long seq, int* error, hipStream_t s,
                    const KernelTiming& tm, const OneshotLayout* compact,
                    long long* tl) {
    OneshotArgs a{};
    for (int q = 0; q < nranks; ++q) a.inbox[q] = inbox[q];
    if (compact && compact->on) {
        a.cx = oneshot_compact(*compact);
        a.compactOn = (a.cx.total <= n) ? 1 : 0;   // always (the compact form is smaller); the full sum is exact too
    }
    a.tl = tl;
    launch(k_oneshot, dim3(kOneshotChunks), dim3(kBlock), 0, s, tm, a, send, recv, n, nranks, rank, seq, error);
}

void launch_finish(const KgmtDev& d, int t, int insertBlocks, hipStream_t s, const KernelTiming& tm) {
    launch(k_finish, dim3(1 + insertBlocks), dim3(kBlock), 0, s, tm, d, t);
}

void launch_pack(const KgmtDev& d, int t, int blocks, hipStream_t s, const KernelTiming& tm) {
    launch(k_pack, dim3(blocks), dim3(kBlock), 0, s, tm, d, t);
}

void launch_xsum(const unsigned long long* const* send, unsigned long long* const* recv, int nranks, long long n,
                 hipStream_t s) {
    XsumArgs a{};
    for (int q = 0; q < nranks; ++q) {
        a.send[q] = send[q];
        a.recv[q] = recv[q];
    }
    const int blocks = (int)std::min<long long>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(k_xsum, dim3(blocks), dim3(256), 0, s, a, nranks, n);
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

void launch_delay(double microseconds, hipStream_t s) {
    const long long ticks = (long long)(microseconds * 100.0);   // s_memrealtime runs at 100 MHz
    hipLaunchKernelGGL(k_delay, dim3(1), dim3(64), 0, s, ticks);
}

void launch_seed_root(const KgmtDev& d, float4 rs, float4 rc, int r1, int r2, hipStream_t s) {
    hipLaunchKernelGGL(k_seed_root, dim3(1), dim3(64), 0, s, d, rs, rc, r1, r2);
}

void launch_export_tree(const KgmtDev& d, float* samples, float* costs, hipStream_t s) {
    hipLaunchKernelGGL(k_export_tree, dim3(1024), dim3(256), 0, s, d, samples, costs);
}

void launch_solution_path(const KgmtDev& d, int node, int maxDepth, int* out, int* rows, float* samples, float* costs,
                          hipStream_t s) {
    hipLaunchKernelGGL(k_solution_path, dim3(1), dim3(64), 0, s, d, node, maxDepth, out, rows, samples, costs);
}

void launch_export_unexplored(const KgmtDev& d, float* samples, int* uParent, hipStream_t s) {
    hipLaunchKernelGGL(k_export_unexplored, dim3(1024), dim3(256), 0, s, d, samples, uParent);
}

}  // namespace sbmp
