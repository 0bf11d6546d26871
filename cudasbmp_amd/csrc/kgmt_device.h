// kgmt_device.h — data layout and device functions of the MI355X KGMT hot path.
//
// HBM layout:
//   tree rows      treeState  float4[M]  (x, y, theta, v)
//                  treeCtrl   float4[M]  (a, steering, duration, cost)
//                  treeParent int[M]
//   child slots    uState     float4[slots] (x, y, theta, v) of the child in that slot
//                  uCtrl      float4[slots] (a, steering, duration, parent-row bits)
//                  rngA/rngB  uint4/uint2[slots]: XORWOW {v0..v3}, {v4, d}
//                  gnew       u64[slots/64]: accept flags (GNew), one bit per slot
// Every per-slot access is a 16-B (or 8-B) coalesced load/store; the region
// tables (~200 KB) and the obstacle list stay L2-resident.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sbmp/collision.h"
#include "sbmp/grid.h"
#include "sbmp/obstacle_grid.h"
#include "sbmp/sbmp_math.h"
#include "sbmp/xorwow.h"

#if defined(__clang__)
#pragma clang fp contract(off)
#endif

namespace sbmp {

constexpr int kBlock = 256;          // threads per expand block = slots per ownership block
constexpr int kWave = 64;
constexpr int kNoGoal = 0x7fffffff;
constexpr int kN = 16;               // R1 grid side: N must be 16 (reference KGMT.cu:8,501,520)
constexpr int kMaxR1 = kN * kN;
constexpr int kMaxR2Words = 2048;    // n <= 16: 256*16*16 cells / 32

// Per-iteration control block, written once by the plan kernel of that iteration.
struct IterCtrl {
    int run;        // iteration t is scheduled (the expand kernel also checks the goal status)
    int executed;   // expand t really ran (written by the next plan kernel)
    int treeSize;   // rows at the start of iteration t
    int gLo;        // frontier = rows [gLo, treeSize)  (G is always a contiguous range)
    int nG, k, nExp, S;
    int H;          // slot high-water mark including this iteration (stale GNew bits live below it)
    int A;          // accepted children (GNew popcount) at the end of iteration t
    int scoreBuf;   // R1Score buffer used by iteration t
    int pad[5];
};
static_assert(sizeof(IterCtrl) == 64, "IterCtrl is one 64-B line");

struct PlannerStatus {
    int goalIdx;    // lowest tree row inside the goal radius (kNoGoal if none), D4
    int error;      // nonzero: a bounded in-kernel wait gave up (kErr*; the host raises it)
    int pad[14];
};
// PlannerStatus::error: which bounded wait gave up.
constexpr int kErrStepHandoff = 1;   // k_step: the planner workgroup's tagged scores/snapshot never arrived
constexpr int kErrExchange = 2;      // k_oneshot: a peer rank's inbox flag never arrived
// Bounds of those waits, in ticks of the 100 MHz s_memrealtime clock.  The in-launch
// hand-off waits for a workgroup of the same launch (1 s); the exchange waits for
// other processes, whose kernels may start seconds apart (startup, code loading,
// per-iteration dumps), so it waits 20 s before it reports.
constexpr long long kStepWaitTicks = 100000000ll;
constexpr long long kExchangeWaitTicks = 2000000000ll;

constexpr int kMaxLdsObs = 2048;     // obstacle lists up to 32 KB are staged in LDS per block
// Obstacle-list forms of k_expand (template parameter OBS):
constexpr int kObsGlobal = 0;        // read from global memory, reference early exit (> kMaxLdsObs boxes)
constexpr int kObsLds = 1;           // staged in LDS, rolled loop
constexpr int kObsLds4 = 2;          // staged in LDS, 4-way batched reads
constexpr int kObsGrid = 3;          // uniform-grid index (include/sbmp/obstacle_grid.h), large obstacle lists
constexpr int kMaxLdsGridG = 90;     // k_step stages the grid's (G^2 + 1)-int cell-start table in LDS: G <= 90 (32 KB)
constexpr int kObsReg = 16;          // kObsReg + n: exactly n <= kMaxRegObs boxes held in registers
constexpr int kMaxRegObs = 8;
constexpr int kMaxRanks = 8;         // ranks of one sharded planning problem (one node)
constexpr int obs_in_registers(int obs) { return obs >= kObsReg ? obs - kObsReg : 0; }
constexpr int kTimelineStamps = 8;   // s_memrealtime stamps per k_expand wave (diagnostics)
constexpr int kFoldEvery = 64;       // iterations per R2 key-log fold (k_fold_r2 at c3, round 5: 24.3-24.8 us per 64, 12.2-12.6 per 20)
#ifndef SBMP_FOLD_KEYS
#define SBMP_FOLD_KEYS 65280
#endif
constexpr int kFoldKeys = SBMP_FOLD_KEYS;   // keys per fold workgroup (< 2^16: packed 16-bit LDS counters; a multiple of 8)
static_assert(kFoldKeys % 8 == 0 && kFoldKeys < 65536, "fold: whole 8-key loads, 16-bit counters");
constexpr int kLogMaxR2 = 32767;     // the 16-bit key (r2 | valid << 15) holds r2 < 32767
constexpr uint16_t kNoKey = 0xffff;  // child outside the R2 grid (D3)
// R1 delta replicas [kDeltaReps][nR1]: workgroup b adds to replica b % kDeltaReps.
// Device atomics execute at the memory side; 1024 workgroups adding into one 2-KB
// table serialise there and back up the stores of the CUs behind them (k_expand
// 18.7 -> 14.6 us at 8 replicas).
constexpr int kDeltaReps = 8;
constexpr int kNewReps = 8;     // k_step R2New replicas (merged by the next planner)
constexpr int kMaxStepBlocks = 1024;   // k_step: one int4 of block (or row) counts per thread (<= 262,144 slots per rank)
constexpr int kNoGoalIdx = 0x7fffffff;
constexpr int kFastDivMax = 1 << 24;   // slot counts up to this use the float-estimate division
constexpr int kStepEntry = 3;       // k_step list entry: state, (a, steer, dur, parent), (cost, -, -, -)
// k_step: when iteration t-1 accepted at most this many children, the planner
// workgroup (idle once it has published) writes all of them into the tree, and the
// expanding workgroups issue no insert loads or stores ahead of their propagation.
// 1024 rather than 4096: the planner inserts 2 rows per thread per round behind a
// binary search, so between 1,024 and 4,096 rows it became the launch's tail; the
// driver's window measured +2.7% (13.58 vs 13.22 G samples/s mean, 5 run triples),
// 300-step lines equal.
constexpr int kPlannerInsertMax = 1024;
static_assert(kBlock / kWave == 4 && kMaxR1 == kBlock, "the flush and prefix code assumes 4 waves and 256 R1 cells");
constexpr int kInsertBase = 8;   // k_finish workgroup of insert block 0 (one per XCD ahead of it)
constexpr int kRecordF4 = 3;   // sharded record: state, ctrl (a, steer, dur, parent), (block, index in block, -, -)

// Everything a kernel needs, passed by value.
// The compact form of the sharded k_step's exchange (k_oneshot, and k_step's own tail
// when the exchange is fused; kgmt_kernels.hip): u64 offsets and counts of the send
// buffer, then the compact layout's region starts and total.
constexpr int kFxReplicas = 8;   // fused exchange: arrival counter replicas (one per worker) ...
constexpr int kFxShards = 8;     // ... each sharded by owned block mod 8
constexpr int kFxCounters = kFxReplicas * kFxShards;
constexpr int kFxStride = 32;    // u32 words between counters (128 B)
struct OneshotCompact {
    int nR1, rowOff, rowWords, cntOff, owned, nBlocks, newOff, newWords;
    int c16Off;   // u64 offset of the block counts as u16 (the receiver writes them from the block words)
    int cR, cB, cN, total;
};

struct KgmtDev {
    int M, nSlots, nWords, nBlocks, numIterations, numDisc, N, n, nR1, nR2, nObs, cap, fixGNewClear;
    int batchRule;        // 0 = reference rule (+ cap), 1 = fill the cap (D14)
    int nranks, rank;
    float width, height, agentLength, invAgentLength, goalThreshold, R1Size, R2Size, goalX, goalY;
    // RN(1/b) for div_by when the host verified it for this b (planner.cpp markstein_rcp), else 0
    float rcpR1Size, rcpR2Size, rcpNumDisc, rcpAgentLength;
    float reachStep;   // 1.06 / numDisc: a bound on dt (duration <= 1.05) for car_schedule
    float4* treeState;
    float4* treeCtrl;
    int* treeParent;
    float4* uState;
    float4* uCtrl;
    uint4* rngA;
    uint2* rngB;
    // Per-iteration exchange, one fused u64 buffer per direction.
    // *Out is what this rank produced, *In the sum over ranks (RCCL all-reduce, or
    // the local group's sum kernel); on a single rank Out and In are the same memory.
    // Every exchanged field is either disjoint per rank (rank totals) or a carry-free
    // counter (R1 deltas, block prefixes, R2New bytes), so a sum merges them.
    // GNew words and block counts are never exchanged: In and Out are the same
    // (the owner's) memory, and a sharded rank holds only its owned slots' entries.
    unsigned long long* gnewOut;        // accept flags (GNew), one bit per slot; cleared by k_finish (D6)
    unsigned long long* gnewIn;
    int* blockCountOut;                 // accepted (+ stale) children per 256-slot block
    const int* blockCountIn;
    // Sharded ranks only (null otherwise), filled by k_pack: pfx[g] = accepted (+ stale)
    // children of the blocks before g, pfx[nBlocks] = the total (each rank adds the
    // part of its own blocks, so the sum is global); tot[q] = rank q's record count.
    int* pfxOut;
    const int* pfxIn;
    int* totOut;
    const int* totIn;
    unsigned long long* deltaOut;       // this iteration's valid (bits 0-31) / invalid (32-63) children per R1 cell
    const unsigned long long* deltaIn;
    uint8_t* r2newOut;                  // 1 = cell seen valid while unavailable in the snapshot
    const uint8_t* r2newIn;
    // Sharded ranks: accepted children packed in owned-slot order by k_pack into a
    // record buffer [2 parities][recCap][state, ctrl, (block, index in block)]; the
    // insert kernels of every rank read them from the owner's buffer (peer memory
    // over xGMI).  Block counts and GNew words stay with their owner.
    int sharded;
    int recCap;
    float4* recOut;
    const float4* recPeer[kMaxRanks];
    // Region tables: R1, R1Avail, R1Valid, R1Invalid, R1Cov are the parity-0 slices
    // of one int array [2][5][nR1], R2Avail of [2][nR2/32].  k_finish updates parity
    // 0 in place; k_step (below) reads iteration t-1's parity and writes t's.
    int* R1;
    int* R1Avail;
    int* R1Valid;
    int* R1Invalid;
    int* R1Cov;           // available R2 cells per R1 cell (covR numerator, kept incrementally)
    uint32_t* R2Avail;    // live availability bits
    // k_step (single rank, one launch per iteration): parity [t & 1]
    // or ring [t % 3] buffers of what iteration t hands to t + 1.
    int stepMode;
    int* stepCnt;         // [2][kMaxStepBlocks] per 256-slot block: flagged children | (1 + lowest
                          // in-block index of a flagged child in the goal region, 0 if none) << 16
    float4* stepList;     // [2][nBlocks * kBlock][kStepEntry] flagged children compacted per block
    unsigned long long* stepDelta;   // [3][kDeltaReps * nR1] packed R1 deltas
    uint32_t* stepR2New;  // [3][kNewReps][nR2 / 32] R2New bits, replica b % kNewReps per block
    unsigned long long* stepPub;     // [2][nR1 + nR2 / 32] scores and snapshot words, each tagged with t
    uint32_t* R2Snap;     // availability bits at the iteration start (D2)
    int* R2Valid;
    int* R2Invalid;
    float* R1Score;       // [2][nR1]
    uint16_t* r2log;      // [kFoldEvery][logSlots] per-child R2 keys (null when nR2 > kLogMaxR2)
    int logSlots;         // this rank's slots per log row
    const float4* obstacles;
    // Uniform-grid obstacle index (kObsGrid; null otherwise): gridG x gridG cells, CSR.
    int gridG;
    float gridInvW, gridInvH;
    const int* gridStart;
    const float4* gridBoxes;
    IterCtrl* ctrl;
    PlannerStatus* status;
    // Diagnostics (tools/timeline.py): when non-null, lane 0 of every k_expand wave of
    // iteration timelineIter stores s_memrealtime stamps at its phase boundaries.
    long long* timeline;
    long long* timelineFin;   // k_finish(timelineIter): [1 + nBlocks][kTimelineStamps], wave 0 of each workgroup
    int timelineIter;
    int obsNaN;   // an obstacle has a NaN coordinate: wave_cull keeps every box, the grid tests by compares
    // Sharded k_step: per-iteration exchange [R1 delta replicas | row
    // words | block words | R2New bytes].  Row b is block b of every rank (global
    // blocks b P .. b P + P - 1); every rank adds its block's count | goal flag << 16
    // into row word b, so the sum is the row's; block words are owner-written (count |
    // (1 + in-block goal index) << 16).  This rank's part of iteration t goes to
    // stepXs[t & 1], stepXr holds the sum over ranks of t - 1.  The flagged children's
    // lists are the record buffers (recOut / recPeer), one 256-entry list per owned
    // block, read by every rank with system-scope loads.
    unsigned long long* stepXs[2];
    const unsigned long long* stepXr;
    // [2][nBlocks][kBlock][kStepEntry]: every rank's lists of the last iteration, pushed
    // here by every rank's k_step (null with the collective exchange or in a local group:
    // the lists are read from the owners' record buffers)
    float4* stepMirror;
    float4* mirrorPeer[kMaxRanks];   // every rank's stepMirror, mapped here
    // Fused exchange (sharded k_step + one-shot exchange + list mirror): the last
    // expanding workgroup of k_step(t) runs the exchange of t itself (k_step_exchange),
    // instead of a k_oneshot launch.  xInbox: every rank's inbox, mapped here;
    // xArrive: [2 parities][kFxReplicas][kFxShards][kFxStride] arrival counters (replica r
    // polled by worker r, shard = owned block mod 8, each on a 128-B line); exchange t has
    // sequence number xSeqBase + t.
    int fusedX;
    int xInboxWords;   // n of the inbox layout (slot stride)
    unsigned long long* xInbox[kMaxRanks];
    unsigned* xArrive;
    unsigned long long xSeqBase;
    OneshotCompact xc;
    int listPlain;   // sharded lists readable with plain loads (the mirror, or a local shard group)
    int xRowOff, xCntOff, xNewOff;   // u64 offsets of the row words, block words and R2New bytes
    int xC16Off;   // u64 offset of the block counts as u16 (global block order; 16-B aligned): k_step's LDS row table
    int c16Lds;    // sharded k_step stages that table in LDS (else: a row's block words from the exchange, one
                   // more L2 round trip per lookup; chosen by begin() when the table would cost residency)
    // k_step reads this struct from device memory (a copy the host refreshes before a
    // launch when it changed): as a 600-B kernel argument its fields were loaded at
    // entry, spilled to VGPR lanes and reloaded, four serial scalar round trips
    // Single rank: pinned host word the planner workgroup of every k_step stores
    // t << 2 | (loop ended) << 1 | (goal found) into (KgmtPlanner::run_to_goal), else null.
    unsigned long long* hostPoll;
    const KgmtDev* devSelf;
};

// Global-address-space view of a device pointer.  A pointer loaded from the plan
// struct in device memory (k_step reads it there) is generic to the compiler: its
// accesses become flat_* instructions, which take no scalar base, count against
// lgkmcnt (so every LDS / scalar wait also waits for them) and check the apertures.
// (The qualifier exists only in the device pass: hipcc also parses kernel bodies for
// the host, where address-space-qualified vector copies do not compile.)
#if defined(__HIP_DEVICE_COMPILE__)
#define SBMP_GAS __attribute__((address_space(1)))
#else
#define SBMP_GAS
#endif
template <class T>
__device__ __forceinline__ SBMP_GAS T* G(T* p) {
    return (SBMP_GAS T*)p;
}

// 16-B / 8-B stores with sc1: written through to memory during the kernel, so the
// dependent kernel boundary has fewer dirty L2 lines to write back (MI355X_MICROARCH.md,
// "boundary": + dirty bytes / 6 TB/s).  Raw buffer stores carry the cache policy as a
// builtin operand, so the compiler schedules them and pads their hazards itself (an
// inline-asm global_store needed a hand-placed s_nop for the >8-B store-data hazard).
// One V# per array (base, no stride, byte bound 2^31 - 1: every per-slot array here is
// far smaller); `i` is the element index.
typedef uint32_t sbmp_u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t sbmp_u32x2 __attribute__((ext_vector_type(2)));
constexpr int kCpolSc1 = 16;            // gfx94x / gfx950 cache policy: SC1 (write through)
constexpr int kBufferDword3 = 0x00020000;   // raw-buffer V# word 3 for gfx9 (ck.hpp CK_BUFFER_RESOURCE_3RD_DWORD)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t wt_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7fffffff, kBufferDword3);
}
// Offsets as (voffset, soffset).  soffset stays 0: ROCm 7.2's hazard recognizer does not pad
// a MUBUF store whose soffset is an SGPR (tools/isa_hazards.py scans the
// built library).  SBMP_SOFFSET_DEMO is that form (the slot's uniform block part in an
// SGPR, valid for i = block * kBlock + threadIdx.x), kept only so tests/test_isa_hazards.py
// can show that the scan catches it.
#ifdef SBMP_SOFFSET_DEMO
#define SBMP_WT_OFF(i, sz) ((i) & (kBlock - 1)) * (sz), __builtin_amdgcn_readfirstlane(((i) / kBlock) * kBlock * (sz))
#else
#define SBMP_WT_OFF(i, sz) (i) * (sz), 0
#endif
__device__ __forceinline__ void store_wt(float4* base, int i, float4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(
        sbmp_u32x4{__float_as_uint(v.x), __float_as_uint(v.y), __float_as_uint(v.z), __float_as_uint(v.w)},
        wt_rsrc(base), SBMP_WT_OFF(i, 16), kCpolSc1);
}
__device__ __forceinline__ void store_wt(uint4* base, int i, uint4 v) {
    __builtin_amdgcn_raw_buffer_store_b128(sbmp_u32x4{v.x, v.y, v.z, v.w}, wt_rsrc(base), SBMP_WT_OFF(i, 16), kCpolSc1);
}
__device__ __forceinline__ void store_wt(uint2* base, int i, uint2 v) {
    __builtin_amdgcn_raw_buffer_store_b64(sbmp_u32x2{v.x, v.y}, wt_rsrc(base), SBMP_WT_OFF(i, 8), kCpolSc1);
}
__device__ __forceinline__ void store_wt(unsigned long long* base, int i, unsigned long long v) {
    __builtin_amdgcn_raw_buffer_store_b64(sbmp_u32x2{(uint32_t)v, (uint32_t)(v >> 32)}, wt_rsrc(base), SBMP_WT_OFF(i, 8),
                                          kCpolSc1);
}
__device__ __forceinline__ void store_wt(int* base, int i, int v) {
    __builtin_amdgcn_raw_buffer_store_b32((uint32_t)v, wt_rsrc(base), SBMP_WT_OFF(i, 4), kCpolSc1);
}
__device__ __forceinline__ void store_wt(uint16_t* base, int i, uint16_t v) {
    __builtin_amdgcn_raw_buffer_store_b16(v, wt_rsrc(base), SBMP_WT_OFF(i, 2), kCpolSc1);
}
__device__ __forceinline__ void store_wt(float* base, int i, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), wt_rsrc(base), SBMP_WT_OFF(i, 4), kCpolSc1);
}
__device__ __forceinline__ void store_wt(uint32_t* base, int i, uint32_t v) {
    __builtin_amdgcn_raw_buffer_store_b32(v, wt_rsrc(base), SBMP_WT_OFF(i, 4), kCpolSc1);
}

// Slot i's XORWOW state for i < n, zeros with no memory access for i >= n: the
// buffer's num_records is the n slots' bytes, and a raw buffer load whose offset is
// at or past num_records returns 0 (k_expand: slots in [S, H) of a launch whose batch
// is below its high-water mark read nothing).  Offsets of the other lanes also get
// bit 31 set (CK's invalid-element form), past any num_records below 2 GiB.
__device__ __forceinline__ uint4 load_rng_a(const uint4* base, int i, int n) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(base), (short)0, n * 16, kBufferDword3);
    const sbmp_u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, (i < n ? 0 : (int)0x80000000) + i * 16, 0, 0);
    return make_uint4(v[0], v[1], v[2], v[3]);
}
__device__ __forceinline__ uint2 load_rng_b(const uint2* base, int i, int n) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint2*>(base), (short)0, n * 8, kBufferDword3);
    const sbmp_u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(r, (i < n ? 0 : (int)0x80000000) + i * 8, 0, 0);
    return make_uint2(v[0], v[1]);
}

// Inclusive prefix sum over the 64 lanes of a wave with DPP: shifts by 1, 2, 4, 8
// inside each 16-lane row, then the row totals by row_bcast:15 / row_bcast:31.  Every
// lane must be active.  (__shfl_up compiles to ds_bpermute, one LDS round trip per step.)
__device__ __forceinline__ int wave_incl_sum(int v) {
    v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, false);   // row_shr:1
    v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, false);   // row_shr:2
    v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, false);   // row_shr:4
    v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, false);   // row_shr:8
    v += __builtin_amdgcn_update_dpp(0, v, 0x142, 0xa, 0xf, false);   // row_bcast:15 -> rows 1, 3
    v += __builtin_amdgcn_update_dpp(0, v, 0x143, 0xc, 0xf, false);   // row_bcast:31 -> rows 2, 3
    return v;
}

// Value of v in the lowest lane where `pick` holds (`fallback` if none); uniform.
__device__ __forceinline__ int first_lane_value(bool pick, int v, int fallback) {
    const unsigned long long m = __ballot(pick);
    return m ? __builtin_amdgcn_readlane(v, (int)__builtin_ctzll(m)) : fallback;
}

// ---------------------------------------------------------------- grid binning
// getR1 / getR2 with the reference's signatures: include/sbmp/grid.h.

// a / b for a per-plan constant b, given y = RN(1/b) computed on the host (Markstein):
// q0 = RN(a y), r = a - q0 b exactly by FMA, RN(q0 + r y) = RN(a / b) while r stays
// normal.  tools/check_fast_division.c checks every float a for the divisors the
// tests and the bench use: bit-exact for |a| >= 2^-100, and the truncation to a grid
// cell agrees for every a.  3 VALU instead of the ~11 of an IEEE division.
__device__ __forceinline__ float div_by(float a, float b, float y) {
    const float q0 = a * y;
    const float r = __builtin_fmaf(-q0, b, a);
    return __builtin_fmaf(r, y, q0);
}

// y == 0: the host could not verify div_by for this b; the branch is uniform.
__device__ __forceinline__ float div_or_ieee(float a, float b, float y) {
    if (y != 0.0f) return div_by(a, b, y);
    return a / b;
}

// getR1 / getR2 of the kernels: the same cells as the SBMP_HD forms above (they only
// truncate the quotients), with the divisions by R1Size / R2Size as div_by.
__device__ __forceinline__ int getR1_k(float x, float y, float R1Size, float rcpR1, int N) {
    bool okx, oky;
    const int cx = cell_of(div_or_ieee(x, R1Size, rcpR1), &okx);
    const int cy = cell_of(div_or_ieee(y, R1Size, rcpR1), &oky);
    return (okx && oky && cx >= 0 && cx < N && cy >= 0 && cy < N) ? cy * N + cx : -1;
}

__device__ __forceinline__ int getR2_k(float x, float y, int r1, float R1Size, int N, float R2Size, float rcpR2,
                                       int n) {
    if (r1 < 0) return -1;
    const int cyR1 = r1 / N;
    const int cxR1 = r1 % N;
    const float lx = __builtin_fmaf(-(float)cxR1, R1Size, x);   // nvcc's contraction of KGMT.cu:620 (D10)
    const float ly = __builtin_fmaf(-(float)cyR1, R1Size, y);
    bool okx, oky;
    const int cx = cell_of(div_or_ieee(lx, R2Size, rcpR2), &okx);
    const int cy = cell_of(div_or_ieee(ly, R2Size, rcpR2), &oky);
    return (okx && oky && cx >= 0 && cx < n && cy >= 0 && cy < n) ? r1 * (n * n) + cy * n + cx : -1;
}

// getR1 and getR2 of one state in one pass (what getR1_k then getR2_k return).  The
// range tests of cell_of and of getR1 / getR2 fold into one pair of comparisons per
// axis: cell_of(q) is defined and in [0, N) iff -1 < q < N (the conversion truncates
// toward zero; a NaN fails both), and the R1 cell's (cx, cy) are the ones getR2
// re-derives from r1.  One uniform branch picks the reciprocal or the IEEE quotients.
__device__ __forceinline__ void bins_k(float x, float y, const KgmtDev& d, int* r1, int* r2) {
    float qx, qy;
    const bool fast = (d.rcpR1Size != 0.0f) & (d.rcpR2Size != 0.0f);
    if (fast) {
        qx = div_by(x, d.R1Size, d.rcpR1Size);
        qy = div_by(y, d.R1Size, d.rcpR1Size);
    } else {
        qx = x / d.R1Size;
        qy = y / d.R1Size;
    }
    const float fN = (float)kN, fn = (float)d.n;
    const bool in1 = (qx > -1.0f) & (qx < fN) & (qy > -1.0f) & (qy < fN);
    const int cx = in1 ? (int)qx : 0, cy = in1 ? (int)qy : 0;
    const float lx = __builtin_fmaf(-(float)cx, d.R1Size, x);   // nvcc's contraction of KGMT.cu:620 (D10)
    const float ly = __builtin_fmaf(-(float)cy, d.R1Size, y);
    float px, py;
    if (fast) {
        px = div_by(lx, d.R2Size, d.rcpR2Size);
        py = div_by(ly, d.R2Size, d.rcpR2Size);
    } else {
        px = lx / d.R2Size;
        py = ly / d.R2Size;
    }
    const bool in2 = in1 & (px > -1.0f) & (px < fn) & (py > -1.0f) & (py < fn);
    const int c = cy * kN + cx;
    *r1 = in1 ? c : -1;
    *r2 = in2 ? (c * d.n + (int)py) * d.n + (int)px : -1;
}

// ---------------------------------------------------------------- cuRAND XORWOW
// Xorwow, xorwow_next / xorwow_seed / xorwow_uniform: include/sbmp/xorwow.h.

// ---------------------------------------------------------------- collision
// reference collisionCheck.cu:6-28 (isBroadPhaseValid / isMotionValid with the
// reference's signatures: include/sbmp/collision.h): a segment AABB is free of an
// obstacle box iff separated on some axis; the motion is valid iff free of every box.
// Register and LDS forms test every box without early exit (no load->compare->
// branch chain; the result is an order-independent OR, so identical to the
// reference's early return); the global form keeps the reference's early exit.
__device__ __forceinline__ bool box_overlap(float minx, float miny, float maxx, float maxy, float4 o) {
    // (xmin, ymin, xmax, ymax).  !(a <= b), not (a > b): identical to the reference's
    // predicate for NaN too.  Bitwise, not short-circuit: four compares whose lane
    // masks are combined with scalar ANDs.
    return !(maxx <= o.x) & !(o.z <= minx) & !(maxy <= o.y) & !(o.w <= miny);
}

// OBS: kObsGlobal, kObsLds, kObsLds4, or kObsReg + n (obs points at a kernel-local
// array of exactly n boxes: the loop is unrolled with no per-box guard, so the hit
// mask is combined with plain scalar ANDs/ORs).
template <int OBS>
__device__ __forceinline__ bool motion_valid(float minx, float miny, float maxx, float maxy,
                                             const float4* __restrict__ obs, int nObs) {
    if (OBS >= kObsReg) {
        bool hit = false;
#pragma unroll
        for (int i = 0; i < obs_in_registers(OBS); ++i) hit |= box_overlap(minx, miny, maxx, maxy, obs[i]);
        return !hit;
    }
    if (OBS == kObsLds) {
        bool hit = false;
#pragma unroll 1
        for (int i = 0; i < nObs; ++i) hit |= box_overlap(minx, miny, maxx, maxy, obs[i]);
        return !hit;
    }
    if (OBS == kObsLds4) {
        bool hit = false;
        int i = 0;
        for (; i + 4 <= nObs; i += 4) {
            const float4 a = obs[i], b = obs[i + 1], c = obs[i + 2], e = obs[i + 3];
            hit |= box_overlap(minx, miny, maxx, maxy, a) | box_overlap(minx, miny, maxx, maxy, b) |
                   box_overlap(minx, miny, maxx, maxy, c) | box_overlap(minx, miny, maxx, maxy, e);
        }
#pragma unroll 1
        for (; i < nObs; ++i) hit |= box_overlap(minx, miny, maxx, maxy, obs[i]);
        return !hit;
    }
    for (int i = 0; i < nObs; ++i) {
        const float4 o = obs[i];
        const bool free_ = (maxx <= o.x) || (o.z <= minx) || (maxy <= o.y) || (o.w <= miny);
        if (!free_) return false;
    }
    return true;
}

// One v_min_f32 / v_max_f32: fminf / fmaxf (and fmed3 against +-inf, which the
// compiler folds into them) add a canonicalising v_max per operand in IEEE mode.
__device__ __forceinline__ float seg_min(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ float seg_max(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

struct ChildOut {
    float4 state;   // x, y, theta, v
    float a, steer, dur;
};

// sincosf_d (sbmp_math.h) for the device loop: the Cody-Waite reduction, both
// polynomials and the quadrant fix-up run on every lane; only if some lane has
// |x| > 105615, inf or NaN does the wave enter the branch that recomputes those
// lanes (Payne-Hanek reduction, or x - x).  Bitwise equal to sincosf_d for every x.
// sin_poly and cos_poly (sbmp_math.h) evaluated as one float2 chain: every
// component sees the same fused operations in the same order (so the same bits),
// and the pair issues as packed v_pk_fma_f32 / v_pk_mul_f32.
typedef float sbmp_f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void sincos_poly2(float r, float* sp, float* cp) {
    const float z = r * r;
    const sbmp_f32x2 zz = {z, z};
    sbmp_f32x2 p = __builtin_elementwise_fma(sbmp_f32x2{-1.9515295891e-4f, 2.443315711809948e-5f}, zz,
                                             sbmp_f32x2{8.3321608736e-3f, -1.388731625493765e-3f});
    p = __builtin_elementwise_fma(p, zz, sbmp_f32x2{-1.6666654611e-1f, 4.166664568298827e-2f});
    const sbmp_f32x2 pz = p * zz;
    const sbmp_f32x2 res = __builtin_elementwise_fma(pz, sbmp_f32x2{r, z},
                                                     sbmp_f32x2{r, __builtin_fmaf(-0.5f, z, 1.0f)});
    *sp = res.x;
    *cp = res.y;
}

__device__ __forceinline__ void sincos_quadrant(float r, int q, float* s, float* c) {
    float sp, cp;
    sincos_poly2(r, &sp, &cp);
    const bool odd = (q & 1) != 0;
    const float s0 = odd ? cp : sp;
    const float c0 = odd ? sp : cp;
    *s = u2f(f2u(s0) ^ ((uint32_t)(q & 2) << 30));
    *c = u2f(f2u(c0) ^ ((uint32_t)((q + 1) & 2) << 30));
}

// sincos_pred's Cody-Waite branch with the same operations (hence bits) as
// sincos_quadrant(sincos_poly2): the polynomial pairs packed, the last two FMAs scalar
// (the packed form needed two register copies to pair its operands).
__device__ __forceinline__ void sincos_cw(float x, float* s, float* c) {
    const float j = __builtin_rintf(x * 0.636619772f);
    float r = __builtin_fmaf(j, -1.57079601e+00f, x);
    r = __builtin_fmaf(j, -3.13916473e-07f, r);
    r = __builtin_fmaf(j, -5.39030253e-15f, r);
    const int q = (int)j;
    const float z = r * r;
    const sbmp_f32x2 zz = {z, z};
    sbmp_f32x2 p = __builtin_elementwise_fma(sbmp_f32x2{-1.9515295891e-4f, 2.443315711809948e-5f}, zz,
                                             sbmp_f32x2{8.3321608736e-3f, -1.388731625493765e-3f});
    p = __builtin_elementwise_fma(p, zz, sbmp_f32x2{-1.6666654611e-1f, 4.166664568298827e-2f});
    const sbmp_f32x2 pz = p * zz;
    const float sp = __builtin_fmaf(pz.x, r, r);
    const float cp = __builtin_fmaf(pz.y, z, __builtin_fmaf(-0.5f, z, 1.0f));
    const bool odd = (q & 1) != 0;
    const float s0 = odd ? cp : sp;
    const float c0 = odd ? sp : cp;
    *s = u2f(f2u(s0) ^ ((uint32_t)(q & 2) << 30));
    *c = u2f(f2u(c0) ^ ((uint32_t)((q + 1) & 2) << 30));
}

__device__ __forceinline__ void sincos_pred(float x, float* s, float* c) {
    sincos_cw(x, s, c);
    if (!(__builtin_fabsf(x) <= 105615.0f)) {   // rare: huge, inf or NaN argument
        if (finitef(x)) {
            int q;
            const float rh = reduce_payne_hanek(x, &q);
            sincos_quadrant(rh, q, s, c);
        } else {
            *s = x - x;
            *c = x - x;
        }
    }
}

// tanf_d for a steering angle: (float)fma(2u, pi, -pi) with u in (0, 1] lies in
// (-pi, pi], so reduce_pio2 always takes its Cody-Waite branch and the argument is
// finite: the non-finite and Payne-Hanek paths of tanf_d are dead here, and the
// result is bitwise tanf_d's (same operations on the same reduced value).
// The odd quadrants' -1/t as v_rcp_f32 and one Newton step instead of the IEEE division
// (3 VALU instead of ~11): the same bits for every t this function can see.  An odd
// quadrant means |x| in [pi/4, 3pi/4], where |r| >= |float(pi/2) - pi/2| = 4.4e-8 and
// |t| <= 1, far from the range ends where the Newton form loses correct rounding;
// tools/microbench/tan_rcp_check.hip compares both forms on every float in [-pi, pi]
// (profiles/r06/tan_rcp_check.txt: no mismatch).  -DSBMP_TAN_IEEE keeps the division.
__device__ __forceinline__ float tan_steer(float x) {
    const float j = __builtin_rintf(x * 0.636619772f);
    float r = __builtin_fmaf(j, -1.57079601e+00f, x);
    r = __builtin_fmaf(j, -3.13916473e-07f, r);
    r = __builtin_fmaf(j, -5.39030253e-15f, r);
    const float t = tan_poly(r);
#ifdef SBMP_TAN_IEEE
    return ((int)j & 1) ? -1.0f / t : t;
#else
    const float y = __builtin_amdgcn_rcpf(t);
    const float e = __builtin_fmaf(-t, y, 1.0f);
    return ((int)j & 1) ? -__builtin_fmaf(e, y, y) : t;
#endif
}

// Wave-level culling of the per-step tests (register obstacle lists).  Every
// segment box of a child lies inside the square of half-width R around its start
// (sup |displacement| over the steps, plus a margin far above the rounding of the
// update chain), so an obstacle no lane's square overlaps, under the same predicate,
// can never be hit by the wave, and a wave whose squares all lie strictly inside
// the workspace can never leave it.  Skipping those tests does not change a result.
struct WaveCull {
    unsigned boxes;    // bit i: some lane may overlap box i (wave-uniform)
    bool bounds;       // some lane may leave the workspace (wave-uniform)
};

// The square test as vector arithmetic: a box (minx, miny)-(maxx, maxy) meets obstacle
// o under isBroadPhaseValid's predicate iff max(o.x - maxx, minx - o.z, o.y - maxy,
// miny - o.w) < 0 (for finite operands a - b < 0 <=> a < b exactly: IEEE subtraction
// with gradual underflow, .amdhsa_float_denorm_mode_32 3).  maxnum ignores a NaN
// operand, so a list with a NaN coordinate keeps every box (KgmtDev::obsNaN).
__device__ __forceinline__ float vmax3(float a, float b, float c) { return __builtin_fmaxf(__builtin_fmaxf(a, b), c); }
__device__ __forceinline__ float vmin3(float a, float b, float c) { return __builtin_fminf(__builtin_fminf(a, b), c); }

template <int OBS>
__device__ __forceinline__ WaveCull wave_cull(float x0, float y0, float rx, float ry, const float4* obs,
                                              const KgmtDev& d) {
    WaveCull w;
    rx = rx * 1.0001f + 1e-3f;
    ry = ry * 1.0001f + 1e-3f;
    const sbmp_f32x2 c = {x0, y0}, rr = {rx, ry};
    const sbmp_f32x2 mn = c - rr, mx = c + rr;
    const sbmp_f32x2 far = sbmp_f32x2{d.width, d.height} - mx;
    // (minx > 0) & (maxx < W) & (miny > 0) & (maxy < H), as min(...) > 0 (see above)
    const bool inside = __builtin_fminf(vmin3(mn.x, mn.y, far.x), far.y) > 0.0f;
    w.bounds = __ballot(!inside) != 0ull;
    w.boxes = 0u;
#pragma unroll
    for (int i = 0; i < obs_in_registers(OBS); ++i) {
        const float4 o = obs[i];
        const sbmp_f32x2 lo = sbmp_f32x2{o.x, o.y} - mx;
        const sbmp_f32x2 hi = mn - sbmp_f32x2{o.z, o.w};
        const float sep = __builtin_fmaxf(vmax3(lo.x, lo.y, hi.x), hi.y);
        // the flag from the ballot on the scalar unit (written as a select, the compiler
        // kept the flags as lane booleans and merged them with vector ORs)
        const unsigned long long m = __ballot(sep < 0.0f);
        unsigned bit;
        asm("s_cmp_lg_u64 %1, 0\n\ts_cselect_b32 %0, %2, 0" : "=s"(bit) : "s"(m), "s"(1u << i) : "scc");
        w.boxes |= bit;
    }
    if (d.obsNaN) w.boxes = ~0u;
    return w;
}

template <int OBS>
__device__ __forceinline__ bool motion_valid_culled(float minx, float miny, float maxx, float maxy,
                                                    const float4* __restrict__ obs, unsigned boxes) {
    if (boxes == 0u) return true;   // uniform: the common case skips every test
    bool hit = false;
#pragma unroll
    for (int i = 0; i < obs_in_registers(OBS); ++i)
        if ((boxes >> i) & 1u) hit |= box_overlap(minx, miny, maxx, maxy, obs[i]);   // uniform branch
    return !hit;
}

// grid_motion_valid_batched (include/sbmp/obstacle_grid.h) for the kernels: the same
// boolean from the same listed boxes, in fewer and cheaper instructions.
//   - The CSR arrays through global-address-space pointers: loaded from the plan struct
//     the pointers are generic, and flat loads count against lgkmcnt, so every box
//     batch waited with vmcnt(0) lgkmcnt(0) behind the scalar and LDS traffic as well.
//   - isBroadPhaseValid (collisionCheck.cu:6-14) as wave_cull's separation metric,
//     max(o.xmin - maxx, minx - o.xmax, o.ymin - maxy, miny - o.ymax) < 0 iff the boxes
//     overlap (exact for finite segments, D15, and any box without NaN; begin() sends a
//     list with a NaN coordinate to the reference form), folded with min: VALU only,
//     where the four compares and their mask ANDs / ORs ran on the SALU and the
//     short-circuit OR had become branches.
//   - A batch loads kGridBatch consecutive rows unconditionally (the box array holds
//     kGridBatch never-met padding rows past its end) at immediate offsets from one
//     address, and tests them all: rows past the cell run are other cells' boxes, which
//     cannot change the answer (grid_run_sep), instead of clamping each index.
//   - Cells by fmed3 (segments are finite: grid_cell's NaN case cannot arise).
#ifndef SBMP_GRID_BATCH
#define SBMP_GRID_BATCH 8
#endif
constexpr int kGridBatch = SBMP_GRID_BATCH;   // boxes loaded per round trip; also the padding rows of gridBoxes
// k_expand (the global cell-start table, 4-5 waves per SIMD) tests 4 rows per batch: fewer
// rows past the cell run for the VALU, where its occupancy hides the extra round trips
// (c5 at 1,048,576 children: k_expand 95.5 -> 85.3 us); k_step (the LDS table, 2 waves per
// SIMD at c5's per-rank shape, latency-bound) keeps 8 (4 cost it 1%; 16 spills).
// profiles/r06/workloads/grid_batch/.
#ifndef SBMP_GRID_BATCH_GLOBAL
#define SBMP_GRID_BATCH_GLOBAL 4
#endif
constexpr int kGridBatchGlobal = SBMP_GRID_BATCH_GLOBAL;
static_assert(kGridBatchGlobal <= kGridBatch, "the padding rows cover the larger batch");

// The segment's cell span and the start offsets of its first two cell rows (grid_run_sep
// tests their boxes).
struct GridRun {
    int cx0, cx1, cy0, cy1;
    int b0, e0, b1, e1;   // runs of rows cy0 and cy0 + 1 (e1 = b1 for a one-row span)
};

// The cell-start table: in global memory (G(d.gridStart)), or staged in LDS by k_step
// (SP = const SBMP_LDS int*, one LDS read per row lookup instead of an L2 round trip).
#define SBMP_LDS __attribute__((address_space(3)))
template <class SP>
__device__ __forceinline__ GridRun grid_run(float minx, float miny, float maxx, float maxy, const KgmtDev& d,
                                            SP start) {
    const int g = d.gridG;
    const float top = (float)(g - 1);
    auto cell = [&](float v, float inv) { return (int)__builtin_amdgcn_fmed3f(__builtin_floorf(v * inv), 0.0f, top); };
    GridRun q;
    q.cx0 = cell(minx, d.gridInvW);
    q.cx1 = cell(maxx, d.gridInvW);
    q.cy0 = cell(miny, d.gridInvH);
    q.cy1 = cell(maxy, d.gridInvH);
    const int c1 = min(q.cy0 + 1, q.cy1);
    q.b0 = start[q.cy0 * g + q.cx0];
    q.e0 = start[q.cy0 * g + q.cx1 + 1];
    q.b1 = start[c1 * g + q.cx0];
    q.e1 = (q.cy0 + 1 <= q.cy1) ? start[c1 * g + q.cx1 + 1] : q.b1;
    return q;
}

// min over the span's boxes of the separation metric (< 0: a box overlaps the segment box).
template <int B, class SP>
__device__ __forceinline__ float grid_run_sep(GridRun q, float minx, float miny, float maxx, float maxy,
                                              const KgmtDev& d, SP start) {
    const SBMP_GAS float4* const boxes = G(d.gridBoxes);
    const int g = d.gridG;
    const sbmp_f32x2 mn = {minx, miny}, mx = {maxx, maxy};
    float sep = 1.0f;
    for (int cy = q.cy0; cy <= q.cy1 && !(sep < 0.0f); cy += 2) {
        if (cy > q.cy0) {   // a span of three or more rows: the next two rows' runs
            const int c1 = min(cy + 1, q.cy1);
            q.b0 = start[cy * g + q.cx0];
            q.e0 = start[cy * g + q.cx1 + 1];
            q.b1 = start[c1 * g + q.cx0];
            q.e1 = (cy + 1 <= q.cy1) ? start[c1 * g + q.cx1 + 1] : q.b1;
        }
#pragma unroll
        for (int r = 0; r < 2; ++r) {
            const int b = r ? q.b1 : q.b0, e = r ? q.e1 : q.e0;
            for (int i = b; i < e && !(sep < 0.0f); i += B) {
                const SBMP_GAS float4* const row = boxes + i;
                float4 o[B];
#pragma unroll
                for (int k = 0; k < B; ++k) o[k] = row[k];
#pragma unroll
                for (int k = 0; k < B; ++k) {
                    const sbmp_f32x2 lo = sbmp_f32x2{o[k].x, o[k].y} - mx;
                    const sbmp_f32x2 hi = mn - sbmp_f32x2{o[k].z, o[k].w};
                    const float sk = __builtin_fmaxf(vmax3(lo.x, lo.y, hi.x), hi.y);
                    // Rows past the run are tested too, unmasked: they are other cells' boxes (or the
                    // never-met padding rows), and a box that meets the segment is listed in one of
                    // the segment's cells (obstacle_grid.h), so the answer (some box meets it) is the
                    // same; the mask cost a ballot and a select per row.
                    sep = seg_min(sep, sk);
                }
            }
        }
    }
    return sep;
}

template <int B, class SP>
__device__ __forceinline__ bool grid_free_fast(float minx, float miny, float maxx, float maxy, const KgmtDev& d,
                                               SP start) {
    return !(grid_run_sep<B>(grid_run(minx, miny, maxx, maxy, d, start), minx, miny, maxx, maxy, d, start) < 0.0f);
}
// the table the grid query reads: LDS when the caller staged it (sStart != nullptr is
// decided at compile time by LDSG), else global memory
template <bool LDSG>
__device__ __forceinline__ bool grid_free_at(float minx, float miny, float maxx, float maxy, const KgmtDev& d,
                                             const int* sStart) {
    if constexpr (LDSG) return grid_free_fast<kGridBatch>(minx, miny, maxx, maxy, d, (const SBMP_LDS int*)sStart);
    else return grid_free_fast<kGridBatchGlobal>(minx, miny, maxx, maxy, d, G(d.gridStart));
}

// reference statePropagator.cu:5-76 (car).  Same operation sequence as the oracle
// (D9-D11): fmaf where nvcc would contract, steering via one double fma.
// v / agentLength: when agentLength is a power of two, v * (1/agentLength) is the
// same correctly rounded value (both are the exact product scaled by 2^-k), so the
// host passes invAgentLength != 0 and the per-step division disappears.
// Exec-masked instead of the reference's per-lane break: a dead lane skips the
// step body (the wave keeps iterating while any lane is alive); a lane that fails
// the bounds test keeps its new (x, y) and its old (theta, v), a lane that fails the
// collision test keeps the step's new (x, y, theta, v) -- exactly the state at the
// reference's break (statePropagator.cu:42-45, 61-64).
// Loop-invariant divisions by numDisc / agentLength use div_by when the host
// verified the reciprocal (bit-exact; tools/check_fast_division.c).
struct NoMidHook {
    __device__ void operator()() const {}
};

// The controls of one child (statePropagator.cu:17-21): they depend on the slot's
// XORWOW stream only, not on the parent, so k_step draws them while its block counts
// are still in flight.  car: (a, steering, duration, dt, tan(steering));
// point: (vx, vy, duration, dt).
struct ChildCtl {
    float a, steer, dur, dt, tanS;
};

template <int AGENT>
__device__ __forceinline__ ChildCtl draw_controls(Xorwow& rs, const KgmtDev& d) {
    ChildCtl c;
    if (AGENT == 0) {
        c.a = __builtin_fmaf(xorwow_uniform(rs), 10.0f, -5.0f);
        const float u2 = xorwow_uniform(rs);
        c.steer = (float)__builtin_fma((double)(u2 * 2.0f), 3.141592653589793, -3.141592653589793);
        c.dur = __builtin_fmaf(xorwow_uniform(rs), 1.0f, 0.05f);
        c.dt = div_or_ieee(c.dur, (float)d.numDisc, d.rcpNumDisc);
        c.tanS = tan_steer(c.steer);
    } else {
        c.a = __builtin_fmaf(xorwow_uniform(rs), 2.0f, -1.0f);      // vx
        c.steer = __builtin_fmaf(xorwow_uniform(rs), 2.0f, -1.0f);  // vy
        c.dur = __builtin_fmaf(xorwow_uniform(rs), 1.0f, 0.05f);
        c.dt = div_or_ieee(c.dur, (float)d.numDisc, d.rcpNumDisc);
        c.tanS = 0.0f;
    }
    return c;
}

// midHook() runs once, before Euler step numDisc / 2, on every lane that entered (k_step
// issues the planner-publication loads there: late enough to see them, early enough
// that they have landed when propagation ends).
template <int OBS, typename MidHook = NoMidHook, bool LDSG = false>
__device__ __forceinline__ bool car_euler(float4 p, const ChildCtl& ctl, const KgmtDev& d, const float4* obs,
                                          ChildOut& out, MidHook midHook = MidHook(), const int* sStart = nullptr) {
    const float a = ctl.a, duration = ctl.dur, dt = ctl.dt, tan_steering = ctl.tanS;
    // (x, y) and (theta, v) as float pairs: each pair update is one v_pk_mul_f32 /
    // v_pk_fma_f32 doing the same IEEE operation per component (same bits).
    sbmp_f32x2 xy = {p.x, p.y}, tv = {p.z, p.w};
    const sbmp_f32x2 dt2 = {dt, dt};
    // |v| <= |v0| + |a| t, so the displacement stays below T |v0| + |a| T^2 / 2.
    WaveCull cull{~0u, true};
    if (OBS >= kObsReg) {
        const float r = duration * __builtin_fabsf(p.w) + 0.5f * __builtin_fabsf(a) * duration * duration;
        cull = wave_cull<OBS>(p.x, p.y, r, r, obs, d);
    }
    bool alive = true;
    // v / L: one multiply when L is a power of two (invAgentLength != 0), else div_by
    // with an IEEE fallback.  The choice is per plan, so the loop is unswitched on it.
    auto step = [&](auto invL) {
        if (!alive) return;
        float st, ct;
        sincos_pred(tv.x, &st, &ct);
        const sbmp_f32x2 nxy = __builtin_elementwise_fma(sbmp_f32x2{tv.y, tv.y} * sbmp_f32x2{ct, st}, dt2, xy);
        const float nx = nxy.x, ny = nxy.y;
        // min(nx, ny) <= 0 is (nx <= 0) | (ny <= 0) for finite operands (D15)
        const bool oob = cull.bounds && ((seg_min(nx, ny) <= 0.0f) | (nx >= d.width) | (ny >= d.height));
        const float v = tv.y;
        float vl;
        if (decltype(invL)::value) {
            vl = v * d.invAgentLength;
        } else {
            vl = div_by(v, d.agentLength, d.rcpAgentLength);
            const bool slow = (d.rcpAgentLength == 0.0f) | !(__builtin_fabsf(v) >= 0x1p-100f) |
                              !(__builtin_fabsf(v) <= 0x1p100f);
            if (__ballot(slow) != 0ull && slow) vl = v / d.agentLength;
        }
        // (theta + vl tan dt, v + a dt): KGMT statePropagator.cu's two updates as one pair
        const sbmp_f32x2 ntv = __builtin_elementwise_fma(sbmp_f32x2{vl * tan_steering, a}, dt2, tv);
        // (x > nx ? nx : x) etc. as one v_min / v_max.  They differ from the ternaries
        // only for NaN operands, which need a non-finite theta or v: begin() rejects a
        // non-finite root, and finite states stay finite.
        const float minx = seg_min(xy.x, nx), maxx = seg_max(xy.x, nx);
        const float miny = seg_min(xy.y, ny), maxy = seg_max(xy.y, ny);
        bool freeSeg;
        if (OBS >= kObsReg) freeSeg = motion_valid_culled<OBS>(minx, miny, maxx, maxy, obs, cull.boxes);
        else if (OBS == kObsGrid)   // only lanes whose result counts walk their cells
            freeSeg = oob || (d.obsNaN ? grid_motion_valid_batched(minx, miny, maxx, maxy, d.gridG, d.gridInvW,
                                                                   d.gridInvH, d.gridStart, d.gridBoxes)
                                       : grid_free_at<LDSG>(minx, miny, maxx, maxy, d, sStart));
        else freeSeg = motion_valid<OBS>(minx, miny, maxx, maxy, obs, d.nObs);
        xy = nxy;
        if (!oob) tv = ntv;
        alive = !oob & freeSeg;
    };
    // two loops around the hook: no per-step test of the step index
    const int nSteps = __builtin_amdgcn_readfirstlane(d.numDisc), midStep = nSteps >> 1;
    if (d.invAgentLength != 0.0f) {
        for (int i = 0; i < midStep; ++i) step(std::true_type());
        midHook();
        for (int i = midStep; i < nSteps; ++i) step(std::true_type());
    } else {
        for (int i = 0; i < midStep; ++i) step(std::false_type());
        midHook();
        for (int i = midStep; i < nSteps; ++i) step(std::false_type());
    }
    out.state = make_float4(xy.x, xy.y, tv.x, tv.y);
    out.a = a;
    out.steer = ctl.steer;
    out.dur = duration;
    return alive;
}

// Holonomic R2 point (build extension), predicated like car_euler.
template <int OBS, typename MidHook = NoMidHook, bool LDSG = false>
__device__ __forceinline__ bool point_euler(float4 p, const ChildCtl& ctl, const KgmtDev& d, const float4* obs,
                                            ChildOut& out, MidHook midHook = MidHook(), const int* sStart = nullptr) {
    const float vx = ctl.a, vy = ctl.steer, duration = ctl.dur, dt = ctl.dt;
    float x = p.x, y = p.y;
    WaveCull cull{~0u, true};
    if (OBS >= kObsReg)
        cull = wave_cull<OBS>(p.x, p.y, duration * __builtin_fabsf(vx), duration * __builtin_fabsf(vy), obs, d);
    bool alive = true;
    auto step = [&]() {
        if (!alive) return;
        const float nx = __builtin_fmaf(vx, dt, x);
        const float ny = __builtin_fmaf(vy, dt, y);
        const bool oob = cull.bounds && ((seg_min(nx, ny) <= 0.0f) | (nx >= d.width) | (ny >= d.height));
        const float minx = seg_min(x, nx), maxx = seg_max(x, nx);   // see car_euler
        const float miny = seg_min(y, ny), maxy = seg_max(y, ny);
        bool freeSeg;
        if (OBS >= kObsReg) freeSeg = motion_valid_culled<OBS>(minx, miny, maxx, maxy, obs, cull.boxes);
        else if (OBS == kObsGrid)
            freeSeg = oob || (d.obsNaN ? grid_motion_valid_batched(minx, miny, maxx, maxy, d.gridG, d.gridInvW,
                                                                   d.gridInvH, d.gridStart, d.gridBoxes)
                                       : grid_free_at<LDSG>(minx, miny, maxx, maxy, d, sStart));
        else freeSeg = motion_valid<OBS>(minx, miny, maxx, maxy, obs, d.nObs);
        x = nx;
        y = ny;
        alive = !oob & freeSeg;
    };
    const int nSteps = __builtin_amdgcn_readfirstlane(d.numDisc), midStep = nSteps >> 1;
    for (int i = 0; i < midStep; ++i) step();
    midHook();
    for (int i = midStep; i < nSteps; ++i) step();
    out.state = make_float4(x, y, 0.0f, 0.0f);
    out.a = vx;
    out.steer = vy;
    out.dur = duration;
    return alive;
}

// ---------------------------------------------------------------- fast car loop
// The Euler loop of a car child for register obstacle lists, written for k_step's
// budget of vector AND scalar instructions (both ran near their limits: 1,141 VALU
// and 875 SALU per wave, 16 waves per CU sharing one scalar unit):
//   - no per-lane branches: a lane whose child ended keeps its state by selects, as
//     at the reference's break (statePropagator.cu:42-45, 61-64), so no exec-mask
//     save / restore / merge per step;
//   - the workspace test (statePropagator.cu:42-45) as min(x, y, W - x, H - y) > 0;
//   - isBroadPhaseValid (collisionCheck.cu:6-14) as the separation metric of wave_cull
//     (exact for finite operands; a NaN box list never takes this loop), one uniform
//     branch per box the wave's cull kept, the metric a float (no lane-mask merge);
//   - sincos: Cody-Waite alone when car_theta_bounded holds on every lane (nearly
//     every wave), else sincos_pred: Cody-Waite on every lane and Payne-Hanek only for
//     a lane past 105615 (a steering angle near +-pi/2 makes theta grow that far).
// The results are those of car_euler bit for bit (the same operations on the same
// values; the tests only replace comparisons by exact equivalents).

// min(a, b, c, e) without the canonicalising v_max that minnum adds in IEEE mode for
// operands the compiler cannot prove canonical (packed-FMA results).
__device__ __forceinline__ float min4_asm(float a, float b, float c, float e) {
    float r;
    asm("v_min3_f32 %0, %1, %2, %3\n\tv_min_f32 %0, %0, %4" : "=&v"(r) : "v"(a), "v"(b), "v"(c), "v"(e));
    return r;
}

// >= 0: the box (mn, mx) is separated from obstacle o (wave_cull's metric).
__device__ __forceinline__ float box_sep(sbmp_f32x2 mn, sbmp_f32x2 mx, float4 o) {
    const sbmp_f32x2 lo = sbmp_f32x2{o.x, o.y} - mx;
    const sbmp_f32x2 hi = mn - sbmp_f32x2{o.z, o.w};
    return __builtin_fmaxf(vmax3(lo.x, lo.y, hi.x), hi.y);
}

// true if this wave may take car_euler_fast: L a power of two (v / L is one multiply)
// and no NaN box (the separation metric ignores NaN).  Per plan, so wave-uniform.
__device__ __forceinline__ bool car_fast_ok(const KgmtDev& d) { return d.invAgentLength != 0.0f && !d.obsNaN; }

// true if no Euler step of this child can take theta past 100000 (so Cody-Waite
// alone reduces it): |theta_k| <= |theta_0| + T / L |tan steer| (|v_0| + |a| T), with
// a 5% margin below 105615 for the float rounding of the steps and of this bound.
// NaN / inf inputs fail it.
__device__ __forceinline__ bool car_theta_bounded(float4 p, const ChildCtl& ctl, const KgmtDev& d) {
    const float T = ctl.dur;
    const float B = __builtin_fabsf(p.z) +
                    T * d.invAgentLength * __builtin_fabsf(ctl.tanS) * (__builtin_fabsf(p.w) + __builtin_fabsf(ctl.a) * T);
    return B < 100000.0f;
}

// PH: some lane of the wave may pass 105615 (car_theta_bounded failed): sincos_pred's
// per-step check and Payne-Hanek branch; otherwise Cody-Waite alone.
// The wave's cull for car_euler_fast, taken once before the caller picks the PH form
// (inside each form the compiler kept the box flags as lane booleans across the branch).
template <int OBS>
__device__ __forceinline__ WaveCull car_cull(float4 p, const ChildCtl& ctl, const KgmtDev& d, const float4* obs) {
    const float T = ctl.dur;
    const float r = T * __builtin_fabsf(p.w) + 0.5f * __builtin_fabsf(ctl.a) * T * T;
    return wave_cull<OBS>(p.x, p.y, r, r, obs, d);
}

// Per-step cull of car_euler_fast, in place of wave_cull for most waves.  wave_cull
// bounds a child's whole reach; the segment of Euler step i ends within r(t) = t |v0| +
// |a| t^2 / 2 of the parent at t = (i + 1) dt, and the controls bound dt <= 1.05 / numDisc
// and |a| <= 5 (statePropagator.cu:17-21: a = 10 u - 5, duration = u + 0.05, u in (0, 1]).
// When the wave's active lanes expand at most two parents (consecutive rows: k >= 64,
// where a steady-state wave holds one or two), box k cannot be met at step i by any lane
// if its L-inf distance from the parents' bounding box is at least that bound for t =
// (i + 1) reachStep (reachStep = 1.06 / numDisc, with wave_cull's margins), and the
// workspace test of step i cannot fail if the square of that half-width around the box
// lies inside the workspace.  One ballot decides every (step, box) pair and every step's
// workspace test: lane L < NOBS D is the pair (L / NOBS, L % NOBS), lane NOBS D + i the
// workspace test of step i.  Early steps of a long reach then skip the tests the whole-
// child cull keeps (the parents move fast: a wave's reach spans half the workspace).
// At the last step the bound covers every lane's whole reach (T <= 1.05), so the
// schedule subsumes wave_cull, which runs only for waves it does not cover.
// Inactive lanes' results are dropped, so only active lanes' parents count.
struct StepSched {
    unsigned long long boxes;    // bit i NOBS + k: box k may be met at step i
    unsigned long long bounds;   // bit i: the workspace test of step i may fail
    int shBoxes, shBounds;       // shift per step (0: no schedule, every step keeps the cull's set)
    bool valid;                  // the schedule covers this wave (else wave_cull's set at every step)
};

__device__ __forceinline__ float lanef(float v, int l) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}

// oLane: box (lane % NOBS) of the register list.
template <int OBS>
__device__ __forceinline__ StepSched car_schedule(float4 p, int parent, bool act, const KgmtDev& d, float4 oLane) {
    constexpr int NOBS = obs_in_registers(OBS);
    StepSched s{~0ull, ~0ull, 0, 0, false};
    const int D = d.numDisc;
    const unsigned long long am = __ballot(act);
    if (am == 0ull || (NOBS + 1) * D > 64) return s;   // uniform
    const int l0 = (int)__builtin_ctzll(am), l1 = 63 - (int)__builtin_clzll(am);
    if (__builtin_amdgcn_readlane(parent, l1) - __builtin_amdgcn_readlane(parent, l0) > 1) return s;
    const float x0 = lanef(p.x, l0), y0 = lanef(p.y, l0), x1 = lanef(p.x, l1), y1 = lanef(p.y, l1);
    // (seg_min / seg_max: no canonicalising v_max per operand; finite states, D15)
    const float v = seg_max(__builtin_fabsf(lanef(p.w, l0)), __builtin_fabsf(lanef(p.w, l1)));
    const float xlo = seg_min(x0, x1), xhi = seg_max(x0, x1);
    const float ylo = seg_min(y0, y1), yhi = seg_max(y0, y1);
    const int L = (int)(threadIdx.x & (kWave - 1));
    const int nb = NOBS * D;
    const int i = (L < nb) ? L / (NOBS > 0 ? NOBS : 1) : L - nb;   // this lane's step
    const float t = (float)(i + 1) * d.reachStep;
    const float r = __builtin_fmaf(__builtin_fmaf(t, v, 2.5f * t * t), 1.0001f, 1e-3f);
    // box item: L-inf distance of the lane's box from the parents' bounding box (the four
    // differences as two packed subtractions, as in box_sep)
    const sbmp_f32x2 dlo = sbmp_f32x2{oLane.x, oLane.y} - sbmp_f32x2{xhi, yhi};
    const sbmp_f32x2 dhi = sbmp_f32x2{xlo, ylo} - sbmp_f32x2{oLane.z, oLane.w};
    const float db = __builtin_fmaxf(vmax3(dlo.x, dlo.y, dhi.x), dhi.y);
    // workspace item: the box's distance to the workspace's edges (uniform)
    const float dw = __builtin_fminf(__builtin_fminf(xlo, ylo), __builtin_fminf(d.width - xhi, d.height - yhi));
    const bool isBox = L < nb;   // bitwise, no branch: both items are computed on every lane
    const bool may = (isBox & !(db >= r)) | (!isBox & (L < nb + D) & !(dw > r));
    const unsigned long long m = __ballot(may);
    s.boxes = m;
    s.bounds = m >> nb;
    s.shBoxes = NOBS;
    s.shBounds = 1;
    s.valid = true;
    return s;
}

// UNIT_L: agentLength == 1 (invAgentLength == 1, the reference demo's and every bench
// workload's): v / L is v itself (finite states, D15), so the heading rate is one multiply,
// v tan(steering), with the same bits as (v * 1) tan(steering).
template <int OBS, bool PH, bool UNIT_L = false>
__device__ __forceinline__ bool car_euler_fast(float4 p, const ChildCtl& ctl, const KgmtDev& d, const float4* obs,
                                               const WaveCull& cull, const StepSched& sched, ChildOut& out) {
    constexpr int NOBS = obs_in_registers(OBS);
    const float a = ctl.a, T = ctl.dur, dt = ctl.dt;
    // (v, theta): v in the low half, so the packed products broadcast it without a copy
    sbmp_f32x2 xy = {p.x, p.y}, vt = {p.w, p.z};
    const sbmp_f32x2 dt2 = {dt, dt}, wh = {d.width, d.height};
    const float invL = d.invAgentLength;
    const unsigned kept = __builtin_amdgcn_readfirstlane(cull.boxes);   // wave-uniform (a ballot)
    unsigned long long sb = sched.boxes, sw = cull.bounds ? sched.bounds : 0ull;   // uniform
    float aliveF = 1.0f;   // 1 alive, 0 ended: a float, so no lane mask is carried across steps
    // the step count in a register: read through d in the loop condition, it was re-loaded
    // (s_load + lgkmcnt wait) every step, the inline asm below being opaque to alias analysis
    const int nSteps = __builtin_amdgcn_readfirstlane(d.numDisc);
    for (int i = 0; i < nSteps; ++i) {
        // re-tested every step (s_bitcmp1 + branch): hoisted, each kept flag would hold
        // a 64-bit lane mask in scalar registers for the whole loop
        unsigned keptNow = kept & (unsigned)sb;
        if (NOBS > 1) asm volatile("" : "+s"(keptNow));   // (one box: a single flag either way)
        const bool bnd = (sw & 1ull) != 0ull;
        sb >>= sched.shBoxes;
        sw >>= sched.shBounds;
        float st, ct;
        if constexpr (PH) sincos_pred(vt.y, &st, &ct);   // Payne-Hanek for the rare lane past 105615
        else sincos_cw(vt.y, &st, &ct);
        const sbmp_f32x2 nxy = __builtin_elementwise_fma(sbmp_f32x2{vt.x, vt.x} * sbmp_f32x2{ct, st}, dt2, xy);
        const sbmp_f32x2 far = wh - nxy;   // W - x, H - y
        const float vl = UNIT_L ? vt.x : vt.x * invL;     // v / L, exact for a power-of-two L
        const sbmp_f32x2 nvt = __builtin_elementwise_fma(sbmp_f32x2{a, vl * ctl.tanS}, dt2, vt);
        float sep = 1.0f;   // >= 0: free of every kept box
        if (keptNow) {
            const sbmp_f32x2 mn = {seg_min(xy.x, nxy.x), seg_min(xy.y, nxy.y)};
            const sbmp_f32x2 mx = {seg_max(xy.x, nxy.x), seg_max(xy.y, nxy.y)};
#pragma unroll
            for (int k = 0; k < NOBS; ++k)
                if ((keptNow >> k) & 1u) sep = seg_min(sep, box_sep(mn, mx, obs[k]));   // uniform branch
        }
        // the reference's break: out of bounds keeps the new (x, y) and the old
        // (theta, v); a collision keeps the new (x, y, theta, v) and ends the child
        const bool live = aliveF > 0.0f;
        const float in4 = bnd ? min4_asm(aliveF, nxy.x, nxy.y, __builtin_fminf(far.x, far.y)) : aliveF;
        const bool upd = in4 > 0.0f;   // alive & inside
        xy = live ? nxy : xy;
        vt = upd ? nvt : vt;
        // > 0 iff upd and sep >= 0: sep + 2^-149 > 0 iff sep >= 0 (f32 denormals on;
        // sep is never NaN, a min from 1), and no lane mask is combined on the SALU
        aliveF = seg_min(in4, sep + 0x1p-149f);
    }
    asm volatile("" : "+v"(aliveF));   // keep the last step's masks from living across the loop
    out.state = make_float4(xy.x, xy.y, vt.y, vt.x);
    out.a = a;
    out.steer = ctl.steer;
    out.dur = T;
    return aliveF > 0.0f;
}

// reference statePropagator.cu:5-76: controls, then the Euler loop (k_expand's form).
template <int OBS, typename MidHook = NoMidHook>
__device__ __forceinline__ bool propagate_car(float4 p, Xorwow& rs, const KgmtDev& d, const float4* obs,
                                              ChildOut& out, MidHook midHook = MidHook()) {
    const ChildCtl c = draw_controls<0>(rs, d);
    return car_euler<OBS>(p, c, d, obs, out, midHook);
}

template <int OBS, typename MidHook = NoMidHook>
__device__ __forceinline__ bool propagate_point(float4 p, Xorwow& rs, const KgmtDev& d, const float4* obs,
                                                ChildOut& out, MidHook midHook = MidHook()) {
    const ChildCtl c = draw_controls<1>(rs, d);
    return point_euler<OBS>(p, c, d, obs, out, midHook);
}

}  // namespace sbmp
