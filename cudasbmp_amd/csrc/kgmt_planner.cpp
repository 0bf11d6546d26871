// kgmt_planner.cpp — host driver of the device-resident KGMT loop.
//
// Reference: KGMT::KGMT (src/planners/KGMT.cu:10-78) allocates ~25 thrust vectors;
// KGMT::plan (KGMT.cu:80-317) runs a host loop with >= 6 blocking device->host
// reads per iteration.  Here every iteration is two kernels (expand, finish; plus
// pack + one all-reduce on a sharded rank) whose sizes live in device memory
// (IterCtrl), so the host only enqueues; it synchronises once per `pollEvery`
// iterations to learn whether the loop has ended.
#include "kgmt_planner.h"

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iomanip>
#include <mutex>
#include <string>
#include <unordered_map>
#include <sys/stat.h>

#include "kgmt_launch.h"
#include "obstacle_grid.h"

namespace sbmp {

double now_ms() {
    using namespace std::chrono;
    return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

template <typename T>
T* KgmtPlanner::alloc(size_t n) {
    void* p = nullptr;
    const size_t bytes = std::max<size_t>(n, 1) * sizeof(T);
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess)
        throw Error(e == hipErrorOutOfMemory ? SBMP_ERR_OUT_OF_MEMORY : SBMP_ERR_HIP,
                    "hipMalloc(" + std::to_string(bytes) + "): " + hipGetErrorString(e));
    allocs_.push_back(p);
    return static_cast<T*>(p);
}

// RN(1/b) when the kernels' div_by (q0 = a y, r = fma(-q0, b, a), q = fma(r, y, q0))
// returns RN(a / b) bit for bit for every float a with |a| in [2^-100, 2^100]; else 0,
// and the kernels divide.  Quotient and residual scale exactly with a's exponent
// there (b is limited to [2^-20, 2^20], so both stay normal), so checking the 2^23
// mantissas of one binade covers the range (tools/check_fast_division.c checks all
// 2^32 inputs for the bench's divisors).  Cached per divisor: ~20 ms each.
static float markstein_rcp(float b) {
    static std::mutex mu;
    static std::unordered_map<uint32_t, float> cache;
    uint32_t key;
    std::memcpy(&key, &b, 4);
    {
        std::lock_guard<std::mutex> g(mu);
        auto it = cache.find(key);
        if (it != cache.end()) return it->second;
    }
    float y = 0.0f;
    if (std::isfinite(b) && std::fabs(b) >= 0x1p-20f && std::fabs(b) <= 0x1p20f) {
        const volatile float vb = b;
        y = 1.0f / vb;
        for (uint32_t m = 0; m < (1u << 23); ++m) {
            float a;
            const uint32_t bits = 0x3f800000u | m;   // [1, 2)
            std::memcpy(&a, &bits, 4);
            const volatile float ref = a / vb;
            const volatile float q0 = a * y;
            const float r = std::fma(-q0, b, a);
            const float q = std::fma(r, y, (float)q0);
            if (q != ref) {
                y = 0.0f;
                break;
            }
        }
    }
    std::lock_guard<std::mutex> g(mu);
    cache[key] = y;
    return y;
}

// PlannerStatus::error -> the bounded wait that gave up (kgmt_device.h kErr*).
[[noreturn]] static void throw_wait_error(int e) {
    if (e == kErrExchange)
        throw Error(SBMP_ERR_COMM, "k_oneshot: a peer rank's exchange flag did not arrive within 20 s");
    if (e == kErrStepHandoff)
        throw Error(SBMP_ERR_HIP, "k_step: the planner workgroup's hand-off did not arrive within 1 s");
    throw Error(SBMP_ERR_HIP, "in-kernel wait failed (status " + std::to_string(e) + ")");
}

static int round_up(long long x, long long m) { return (int)(((x + m - 1) / m) * m); }

KgmtPlanner::KgmtPlanner(const sbmp_kgmt_params& p, int nranks, int rank, Exchange* ex, hipStream_t shared)
    : p_(p), ex_(ex) {
    if (p.N * p.N != kMaxR1) throw Error(SBMP_ERR_INVALID_ARGUMENT, "N must be 16 (reference KGMT.cu:8 NUM_R1)");
    if (p.n < 1 || p.n > 16) throw Error(SBMP_ERR_INVALID_ARGUMENT, "n must be in [1, 16]");
    if (p.maxTreeSize < 1) throw Error(SBMP_ERR_INVALID_ARGUMENT, "maxTreeSize must be >= 1");
    if (p.numDisc < 1) throw Error(SBMP_ERR_INVALID_ARGUMENT, "numDisc must be >= 1");
    if (p.numIterations < 0) throw Error(SBMP_ERR_INVALID_ARGUMENT, "numIterations must be >= 0");
    if (p.samplesPerIteration < 0) throw Error(SBMP_ERR_INVALID_ARGUMENT, "samplesPerIteration must be >= 0");
    if (p.batchRule != SBMP_BATCH_REFERENCE && p.batchRule != SBMP_BATCH_FILL)
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "unknown batchRule");
    if (p.batchRule == SBMP_BATCH_FILL && p.samplesPerIteration <= 0)
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "batchRule FILL needs samplesPerIteration > 0");
    if (p.agent != SBMP_AGENT_CAR && p.agent != SBMP_AGENT_POINT) throw Error(SBMP_ERR_INVALID_ARGUMENT, "unknown agent");
    if (!(p.width > 0.0f) || !(p.height > 0.0f)) throw Error(SBMP_ERR_INVALID_ARGUMENT, "width/height must be > 0");
    if (nranks < 1 || nranks > kMaxRanks || rank < 0 || rank >= nranks)
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "bad rank/nranks (at most 8 ranks)");
    int ndev = 0;
    SBMP_HIP(hipGetDeviceCount(&ndev));
    if (p.device < 0 || p.device >= ndev) throw Error(SBMP_ERR_INVALID_ARGUMENT, "no such HIP device");
    SBMP_HIP(hipSetDevice(p.device));
    if (shared) {
        stream_ = shared;
        ownStream_ = false;
    } else {
        SBMP_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    }
    // Obstacle-list form of k_expand (diagnostics / A-B): 0 auto, 1 LDS, 2 LDS x4,
    // 3 registers, 4 grid index at any count, 5 global list without the grid.
    if (const char* v = getenv("SBMP_EXPAND_VARIANT")) expandVariant_ = std::min(5, std::max(0, atoi(v)));

    const int M = p.maxTreeSize;
    const int nSlots = p.samplesPerIteration > 0 ? std::min(M, p.samplesPerIteration) : M;
    slotsPadded_ = round_up(nSlots, (long long)kBlock * nranks);   // whole workgroups on every rank
    expandBlocks_ = slotsPadded_ / kBlock / nranks;
    const int nWords = slotsPadded_ / kWave;
    while ((1ll << nbits_) < nSlots) ++nbits_;

    KgmtDev& d = d_;
    d.M = M;
    d.nSlots = nSlots;
    d.nWords = nWords;
    d.nBlocks = slotsPadded_ / kBlock;
    d.batchRule = p.batchRule;
    d.numIterations = p.numIterations;
    d.numDisc = p.numDisc;
    d.N = p.N;
    d.n = p.n;
    d.nR1 = p.N * p.N;
    d.nR2 = d.nR1 * p.n * p.n;
    d.cap = p.samplesPerIteration;
    d.fixGNewClear = p.fixGNewClear;
    d.nranks = nranks;
    d.rank = rank;
    d.width = p.width;
    d.height = p.height;
    d.agentLength = p.agentLength;
    {   // exact reciprocal only for powers of two (then v * (1/L) == v / L bitwise)
        int e = 0;
        const float m = std::frexp(p.agentLength, &e);
        d.invAgentLength = (m == 0.5f) ? 1.0f / p.agentLength : 0.0f;
    }
    d.goalThreshold = p.goalThreshold;
    d.R1Size = p.width / (float)p.N;          // KGMT.cu:13
    d.R2Size = p.width / (float)(p.n * p.N);  // KGMT.cu:14
    d.rcpR1Size = markstein_rcp(d.R1Size);
    d.rcpR2Size = markstein_rcp(d.R2Size);
    d.rcpNumDisc = markstein_rcp((float)p.numDisc);
    d.rcpAgentLength = markstein_rcp(p.agentLength);
    // dt = duration / numDisc <= 1.05 / numDisc (statePropagator.cu:19-21); 1% above it
    d.reachStep = p.numDisc > 0 ? 1.06f / (float)p.numDisc : 0.0f;

    d.treeState = alloc<float4>(M);
    d.treeCtrl = alloc<float4>(M);
    d.treeParent = alloc<int>(M);
    d.uState = alloc<float4>(slotsPadded_);
    d.uCtrl = alloc<float4>(slotsPadded_);
    d.rngA = alloc<uint4>(slotsPadded_);
    d.rngB = alloc<uint2>(slotsPadded_);
    {   // region tables [2 parities][R1, R1Avail, R1Valid, R1Invalid, R1Cov][nR1] (kgmt_device.h)
        int* tab = alloc<int>((size_t)2 * 5 * d.nR1);
        d.R1 = tab;
        d.R1Avail = tab + d.nR1;
        d.R1Valid = tab + 2 * d.nR1;
        d.R1Invalid = tab + 3 * d.nR1;
        d.R1Cov = tab + 4 * d.nR1;
    }
    d.R2Avail = alloc<uint32_t>((size_t)2 * (d.nR2 / 32));
    d.R2Snap = alloc<uint32_t>(d.nR2 / 32);
    d.R2Valid = alloc<int>(d.nR2);
    d.R2Invalid = alloc<int>(d.nR2);
    d.R1Score = alloc<float>(2 * d.nR1);
    {   // Exchange buffer, one u64 array per direction (16-B aligned fields).
        // Single rank: [R1 delta replicas | block counts (int4-readable) | GNew words |
        //               R2New bytes], Out == In.
        // Sharded: [R1 delta replicas | block prefixes pfx | rank totals | R2New bytes]
        //          is all-reduced; block counts and GNew words are the owner's alone
        //          (a separate local buffer), since the inserts are record-driven.
        // Sharded k_step (one launch per iteration): [R1 delta replicas | row words
        //          (kMaxStepBlocks, summed over ranks) | block words (nBlocks, owner-
        //          written) | R2New bytes], two send parities.
        const bool sharded = nranks > 1 || ex;
        const char* sv = std::getenv("SBMP_STEP");
        shStep_ = sharded && d.nBlocks / nranks <= kMaxStepBlocks && !(sv && atoi(sv) == 0);
        const size_t rowWords = shStep_ ? kMaxStepBlocks / 2 : 0;
        const size_t dWords = round_up((long long)kDeltaReps * d.nR1, 2);
        const size_t bcWords = round_up(d.nBlocks, 4) / 2, r2Words = round_up(d.nR2, 16) / 8;
        const size_t pfxWords = round_up(d.nBlocks + 1, 4) / 2, totWords = kMaxRanks / 2;
        // sharded k_step: the block counts again as u16 (owner-written like the block words), so
        // that every workgroup holds the whole table in LDS and locates a position inside a row
        // without a dependent load
        const size_t c16Words = shStep_ ? round_up(d.nBlocks, 8) / 4 : 0;
        unsigned long long* local = nullptr;
        if (shStep_) {
            xWords_ = dWords + rowWords + bcWords + c16Words + r2Words;
            local = alloc<unsigned long long>(bcWords + (size_t)nWords);
            localWords_ = bcWords + (size_t)nWords;
            local_ = local;
        } else if (sharded) {
            xWords_ = dWords + pfxWords + totWords + r2Words;
            local = alloc<unsigned long long>(bcWords + (size_t)nWords);
            localWords_ = bcWords + (size_t)nWords;
            local_ = local;
        } else {
            xWords_ = dWords + bcWords + (size_t)nWords + r2Words;
        }
        xSend_ = alloc<unsigned long long>(xWords_);
        xSendOdd_ = shStep_ ? alloc<unsigned long long>(xWords_) : xSend_;
        xRecv_ = sharded ? alloc<unsigned long long>(xWords_) : xSend_;
        d.stepXs[0] = shStep_ ? xSend_ : nullptr;
        d.stepXs[1] = shStep_ ? xSendOdd_ : nullptr;
        d.stepXr = shStep_ ? xRecv_ : nullptr;
        d.stepMirror = nullptr;   // set below once the one-shot exchange is confirmed
        d.listPlain = (sharded && !ex) ? 1 : 0;   // a local group: every rank's buffers are this GPU's
        d.xRowOff = (int)dWords;
        d.xCntOff = (int)(dWords + rowWords);
        d.xC16Off = (int)(dWords + rowWords + bcWords);
        d.xNewOff = (int)(dWords + rowWords + bcWords + c16Words);
        int* bc = reinterpret_cast<int*>(sharded ? local : xSend_ + dWords);
        unsigned long long* gn = sharded ? local + bcWords : xSend_ + dWords + bcWords;
        d.blockCountOut = bc;
        d.blockCountIn = bc;
        d.gnewOut = gn;
        d.gnewIn = gn;
        auto views = [&](unsigned long long* x, bool out) {
            int* pfx = sharded ? reinterpret_cast<int*>(x + dWords) : nullptr;
            int* tot = sharded ? reinterpret_cast<int*>(x + dWords + pfxWords) : nullptr;
            uint8_t* r2 = reinterpret_cast<uint8_t*>(sharded ? x + dWords + pfxWords + totWords
                                                             : x + dWords + bcWords + nWords);
            if (out) {
                d.deltaOut = x;
                d.pfxOut = pfx;
                d.totOut = tot;
                d.r2newOut = r2;
            } else {
                d.deltaIn = x;
                d.pfxIn = pfx;
                d.totIn = tot;
                d.r2newIn = r2;
            }
        };
        views(xSend_, true);
        views(xRecv_, false);
    }
    d.sharded = nranks > 1 || ex != nullptr;   // one RCCL rank still takes the sharded path
    // One launch per iteration (k_step) on a single rank whose block prefix fits LDS;
    // SBMP_STEP=0 keeps the two-kernel form (k_expand + k_finish).
    // begin() confirms it per plan: all 1 + blocks workgroups must be resident at once
    // for the obstacle form the plan's list picks (step_resident_groups).
    {
        const char* v = getenv("SBMP_STEP");
        stepCapable_ = (!d.sharded && d.nBlocks <= kMaxStepBlocks && !(v && atoi(v) == 0)) || shStep_;
    }
    d.stepMode = stepCapable_ ? 1 : 0;
    d.stepCnt = nullptr;
    d.stepPub = nullptr;
    d.stepList = nullptr;
    d.stepDelta = nullptr;
    d.stepR2New = nullptr;
    if (stepCapable_) {
        d.stepPub = alloc<unsigned long long>((size_t)2 * (d.nR1 + d.nR2 / 32));
        if (!d.sharded) {   // a sharded rank's counts, deltas and R2New travel in the exchange, its lists in recOut
            d.stepCnt = alloc<int>((size_t)2 * kMaxStepBlocks);
            d.stepList = alloc<float4>((size_t)2 * d.nBlocks * kBlock * kStepEntry);
            d.stepDelta = alloc<unsigned long long>((size_t)3 * kDeltaReps * d.nR1);
            d.stepR2New = alloc<uint32_t>((size_t)3 * kNewReps * (d.nR2 / 32));
        }
        dDev_ = alloc<KgmtDev>(1);
        SBMP_HIP(hipHostMalloc(reinterpret_cast<void**>(&dStage_), sizeof(KgmtDev), hipHostMallocDefault));
    }
    d.devSelf = dDev_;
    d.recCap = expandBlocks_ * kBlock;   // a rank never holds more flagged slots than it owns
    d.recOut = d.sharded ? alloc<float4>((size_t)2 * kRecordF4 * d.recCap) : nullptr;
    for (int q = 0; q < kMaxRanks; ++q) d.recPeer[q] = nullptr;
    d.recPeer[rank] = d.recOut;
    d.logSlots = expandBlocks_ * kBlock;
    d.r2log = (d.nR2 <= kLogMaxR2) ? alloc<uint16_t>((size_t)kFoldEvery * d.logSlots) : nullptr;
    d.ctrl = alloc<IterCtrl>(p.numIterations + 2);
    d.status = alloc<PlannerStatus>(1);
    SBMP_HIP(hipHostMalloc(reinterpret_cast<void**>(&poll_), sizeof(PollBuf), hipHostMallocDefault));
    poll_->word = 0;
    d.hostPoll = nullptr;   // a single rank's plan loop watches it (run_to_goal)
    if (!d.sharded) SBMP_HIP(hipHostGetDevicePointer(reinterpret_cast<void**>(&d.hostPoll), &poll_->word, 0));
    d.timeline = nullptr;
    d.timelineFin = nullptr;
    d.timelineIter = -1;
    if (const char* v = getenv("SBMP_TIMELINE_ITER")) {   // diagnostics: tools/timeline.py
#ifndef SBMP_TIMELINE
        fprintf(stderr, "sbmp: SBMP_TIMELINE_ITER set, but k_step stamps only in a build with "
                        "SBMP_HIPCC_FLAGS=-DSBMP_TIMELINE (tools/_tl.sh); its expanding waves' stamps stay 0\n");
#endif
        d.timelineIter = atoi(v);
        const size_t n = (size_t)expandBlocks_ * (kBlock / kWave) * kTimelineStamps;
        const size_t nf = (size_t)(1 + d.nBlocks) * kTimelineStamps;
        d.timeline = alloc<long long>(n + nf);
        d.timelineFin = d.timeline + n;
        SBMP_HIP(hipMemsetAsync(d.timeline, 0, sizeof(long long) * (n + nf), stream_));
    }
    jumps_ = alloc<uint32_t>((size_t)nbits_ * 800);
    const std::vector<uint32_t>& J = subsequence_jump_matrices(nbits_);
    SBMP_HIP(hipMemcpyAsync(jumps_, J.data(), (size_t)nbits_ * 800 * sizeof(uint32_t), hipMemcpyHostToDevice,
                            stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    if (d.sharded && ex_) {   // map every rank's record buffer (IPC over xGMI)
        void* peers[kMaxRanks] = {nullptr};
        ex_->share_buffer(d.recOut, sizeof(float4) * 2 * kRecordF4 * (size_t)d.recCap, peers);
        for (int q = 0; q < nranks; ++q) d.recPeer[q] = static_cast<const float4*>(peers[q]);
        // The per-iteration exchange: a one-shot sum through IPC-mapped inboxes (the
        // default), or SBMP_EXCHANGE=collective for the Exchange's all-reduce (RCCL).
        // Peers write the inboxes over xGMI while the owner's kernel polls them, so they
        // are uncached device memory: a coarse-grained (hipMalloc) page may keep a stale
        // line in the owner's L2, which only a kernel boundary refreshes.
        const char* v = getenv("SBMP_EXCHANGE");
        if (!(v && std::string(v) == "collective")) {
            const size_t words = oneshot_inbox_words((long long)xWords_, nranks);
            void* own = nullptr;
            SBMP_HIP(hipExtMallocWithFlags(&own, sizeof(unsigned long long) * words, hipDeviceMallocUncached));
            allocs_.push_back(own);
            SBMP_HIP(hipMemset(own, 0, sizeof(unsigned long long) * words));
            SBMP_HIP(hipDeviceSynchronize());   // zeroed before any peer can see it
            void* ib[kMaxRanks] = {nullptr};
            ex_->share_buffer(own, sizeof(unsigned long long) * words, ib);
            for (int q = 0; q < nranks; ++q) inbox_[q] = static_cast<unsigned long long*>(ib[q]);
            oneshot_ = true;
            oneshotCheck_ = oneshot_self_test() ? 1 : -1;
            if (oneshotCheck_ < 0) {
                oneshot_ = false;   // on every rank: the verdict is all-reduced
                fprintf(stderr, "sbmp: rank %d: the one-shot exchange failed its start-up check on this machine; "
                                "the per-iteration exchange is the communicator's all-reduce\n", rank);
            }
        }
        // Sharded k_step + one-shot exchange: k_step pushes this rank's flagged-children
        // lists into every rank's mirror (system-scope stores, over xGMI for the peers) and
        // reads its parents from its own, in its own HBM, instead of the owners' record
        // buffers over xGMI (SBMP_MIRROR=0: the remote reads).  A peer's stores are complete
        // at the end of its k_step, before its k_oneshot raises the flags this rank's
        // k_oneshot waits for; this rank's next k_step reads them after that kernel boundary,
        // which refreshes this GPU's L2.  Parity t & 1 is rewritten in t + 2, after every
        // rank's k_step(t + 1), the last reader, has ended (the exchange of t + 1 waits for it).
        const char* cv = getenv("SBMP_ONESHOT_COMPACT");   // 0: the full send buffer on the wire
        compactX_ = !(cv && atoi(cv) == 0);
        const char* mv = getenv("SBMP_MIRROR");
        if (oneshot_ && shStep_ && !(mv && atoi(mv) == 0)) {
            const size_t bytes = sizeof(float4) * 2 * (size_t)d.nBlocks * kBlock * kStepEntry;
            float4* own = alloc<float4>(bytes / sizeof(float4));
            void* mp[kMaxRanks] = {nullptr};
            ex_->share_buffer(own, bytes, mp);
            for (int q = 0; q < nranks; ++q) d.mirrorPeer[q] = static_cast<float4*>(mp[q]);
            d.stepMirror = own;
            d.listPlain = 1;
            // The mirror relies on the kernel boundary dropping this GPU's cached lines of
            // entries a peer rewrote over xGMI: checked once here, on this machine (every
            // rank gets the same all-reduced verdict); on failure every rank reads the lists
            // from the owners' record buffers with system-scope loads instead (SBMP_MIRROR=0).
            mirrorCheck_ = mirror_self_test() ? 1 : -1;
            if (mirrorCheck_ < 0) {
                d.stepMirror = nullptr;
                for (int q = 0; q < kMaxRanks; ++q) d.mirrorPeer[q] = nullptr;
                d.listPlain = 0;
                fprintf(stderr, "sbmp: rank %d: the list mirror failed its start-up check on this machine; k_step "
                                "reads the peers' lists over the mapping (system-scope loads)\n", rank);
            }
        }
        // The fused exchange (k_step_exchange, kgmt_kernels.hip): with the mirror and the
        // compact form, the last expanding workgroup of k_step runs the exchange, and no
        // k_oneshot is launched (SBMP_FUSED_EXCHANGE=0: the separate kernel; DESIGN.md §7
        // has the measurements).  The same on every rank: it depends on the all-reduced
        // one-shot verdict and the switches.
        const char* fv = getenv("SBMP_FUSED_EXCHANGE");
        if (d.stepMirror && compactX_ && !(fv && atoi(fv) == 0)) {
            d.fusedX = 1;
            for (int q = 0; q < nranks; ++q) d.xInbox[q] = inbox_[q];
            d.xInboxWords = (int)xWords_;
            d.xArrive = alloc<unsigned>((size_t)2 * kFxCounters * kFxStride);
            SBMP_HIP(hipMemset(d.xArrive, 0, sizeof(unsigned) * 2 * kFxCounters * kFxStride));
            OneshotLayout l{};
            l.on = 1;
            l.nR1 = d.nR1;
            l.rowOff = d.xRowOff;
            l.rows = expandBlocks_;
            l.cntOff = d.xCntOff;
            l.owned = expandBlocks_;
            l.nBlocks = d.nBlocks;
            l.newOff = d.xNewOff;
            l.newWords = (int)xWords_ - d.xNewOff;
            l.c16Off = d.xC16Off;
            d.xc = oneshot_compact(l);
            if (d.xc.total > (int)xWords_) d.fusedX = 0;   // cannot happen (compact is smaller)
        }
        // The fused exchange orders a peer's mirror pushes before its flags inside one
        // launch (drained stores, relaxed arrivals, the workers' fence and flags), with no
        // kernel boundary between them: checked once here, on this machine; on failure
        // every rank (the verdict is all-reduced) runs the exchange as its own k_oneshot,
        // whose launch boundary follows the pushes (SBMP_FUSED_EXCHANGE=0's form).
        if (d.fusedX) {
            fusedCheck_ = fused_self_test() ? 1 : -1;
            if (fusedCheck_ < 0) {
                d.fusedX = 0;
                fprintf(stderr, "sbmp: rank %d: the fused exchange failed its start-up check on this machine; "
                                "the exchange runs as its own k_oneshot launch\n", rank);
            }
        }
    }
}

// The one-shot exchange checked once on this machine before an iteration relies on it:
// two exchanges (both inbox parities) of rank-specific words through k_oneshot, the sums
// compared on the host.  A wrong word or a timed-out peer flag on any rank (the verdicts
// are summed with the communicator's all-reduce) makes every rank use that all-reduce
// instead, so a fabric on which the inboxes' system-scope stores and flags misbehave costs
// speed, not a wrong or stalled run.  Runs in the constructor, where the collective IPC
// handle exchange has just lined the ranks up.
static unsigned long long oneshot_pattern(int rank, size_t i, int pass) {
    return ((unsigned long long)(rank + 1) * 0x9E3779B97F4A7C15ull) ^ ((unsigned long long)i * 0x100000001ull + pass);
}

bool KgmtPlanner::oneshot_self_test() {
    const size_t n = xWords_;
    const int P = d_.nranks;
    std::vector<unsigned long long> h(n), got(n);
    unsigned long long* send = alloc<unsigned long long>(n);
    unsigned long long* verdict = alloc<unsigned long long>(2);
    int error = 0;
    SBMP_HIP(hipMemsetAsync(&d_.status->error, 0, sizeof(int), stream_));
    bool ok = true;
    for (int pass = 0; pass < 2; ++pass) {
        for (size_t i = 0; i < n; ++i) h[i] = oneshot_pattern(d_.rank, i, pass);
        SBMP_HIP(hipMemcpyAsync(send, h.data(), sizeof(unsigned long long) * n, hipMemcpyHostToDevice, stream_));
        ++xSeq_;
        launch_oneshot(inbox_, send, xRecv_, (long long)n, P, d_.rank, xSeq_, &d_.status->error, stream_,
                       KernelTiming{});
        SBMP_HIP(hipMemcpyAsync(got.data(), xRecv_, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost, stream_));
        SBMP_HIP(hipMemcpyAsync(&error, &d_.status->error, sizeof(int), hipMemcpyDeviceToHost, stream_));
        SBMP_HIP(hipStreamSynchronize(stream_));
        if (error) ok = false;
        for (size_t i = 0; i < n && ok; ++i) {
            unsigned long long want = 0;
            for (int q = 0; q < P; ++q) want += oneshot_pattern(q, i, pass);
            if (got[i] != want) ok = false;
        }
    }
    SBMP_HIP(hipMemsetAsync(&d_.status->error, 0, sizeof(int), stream_));
    if (const char* f = getenv("SBMP_ONESHOT_SELFTEST"))   // tests: this rank reports a failure
        if (std::string(f) == "fail") ok = false;
    const unsigned long long bad = ok ? 0ull : 1ull;
    SBMP_HIP(hipMemcpyAsync(verdict, &bad, sizeof(bad), hipMemcpyHostToDevice, stream_));
    ex_->allreduce_u64(verdict, verdict + 1, 1, stream_);
    unsigned long long anyBad = 0;
    SBMP_HIP(hipMemcpyAsync(&anyBad, verdict + 1, sizeof(anyBad), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    return anyBad == 0;
}

// The list mirror checked once on this machine (the kernels and their
// sequence: k_mirror_touch / push / check, kgmt_kernels.hip).  Probed: both parities, the
// first 64 entries of the first min(nBlocks, 64) global blocks (every rank's among them),
// two passes.  SBMP_MIRROR_SELFTEST=fail makes this rank report a failure (tests).
bool KgmtPlanner::mirror_self_test() {
    MirrorProbe a{};
    for (int q = 0; q < d_.nranks; ++q) a.peer[q] = d_.mirrorPeer[q];
    a.own = d_.stepMirror;
    a.nranks = d_.nranks;
    a.rank = d_.rank;
    a.nBlocks = d_.nBlocks;
    a.blocks = std::min(d_.nBlocks, 64);
    a.entries = 64;
    int* dev = alloc<int>(2);   // [bad, sink]
    a.bad = dev;
    unsigned long long* verdict = alloc<unsigned long long>(2);
    SBMP_HIP(hipMemsetAsync(dev, 0, sizeof(int) * 2, stream_));
    for (int pass = 0; pass < 2; ++pass) {
        launch_mirror_probe(a, 0, pass, reinterpret_cast<float*>(dev + 1), stream_);   // lines of the old values cached
        ex_->barrier(stream_);
        launch_mirror_probe(a, 1, pass, nullptr, stream_);   // every rank pushes into every mirror
        ex_->barrier(stream_);                                // every push has completed (stream drained)
        launch_mirror_probe(a, 2, pass, nullptr, stream_);   // a new launch reads them with plain loads
    }
    SBMP_HIP(hipGetLastError());
    int bad = 0;
    SBMP_HIP(hipMemcpyAsync(&bad, dev, sizeof(int), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    bool ok = bad == 0;
    if (!ok) fprintf(stderr, "sbmp: rank %d: list mirror check: %d stale or wrong words\n", d_.rank, bad);
    if (const char* f = getenv("SBMP_MIRROR_SELFTEST"))   // tests: this rank reports a failure
        if (std::string(f) == "fail") ok = false;
    const unsigned long long badv = ok ? 0ull : 1ull;
    SBMP_HIP(hipMemcpyAsync(verdict, &badv, sizeof(badv), hipMemcpyHostToDevice, stream_));
    ex_->allreduce_u64(verdict, verdict + 1, 1, stream_);
    unsigned long long anyBad = 0;
    SBMP_HIP(hipMemcpyAsync(&anyBad, verdict + 1, sizeof(anyBad), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    return anyBad == 0;
}

// The fused exchange's in-kernel order checked once on this machine (k_fx_probe,
// kgmt_kernels.hip): per pass, every rank's plain loads cache the probed
// mirror lines (k_mirror_touch), a host barrier, then one launch in which every owned
// workgroup pushes its entries into every rank's mirror, drains, arrives, and the workers
// exchange flags with the peers, then a new launch reads the mirror with plain loads
// (k_mirror_check).  Probed: both parities, the first 64 entries of every global block,
// two passes (patterns 2 and 3: the list-mirror check used 0 and 1).  The verdicts and
// any timed-out wait are all-reduced.  SBMP_FUSED_SELFTEST=fail: this rank reports a
// failure (tests).
bool KgmtPlanner::fused_self_test() {
    const int P = d_.nranks;
    MirrorProbe m{};
    FxProbe a{};
    for (int q = 0; q < P; ++q) {
        m.peer[q] = a.peer[q] = d_.mirrorPeer[q];
        a.inbox[q] = d_.xInbox[q];
    }
    m.own = d_.stepMirror;
    m.nranks = a.nranks = P;
    m.rank = a.rank = d_.rank;
    m.nBlocks = a.nBlocks = d_.nBlocks;
    m.blocks = d_.nBlocks;
    m.entries = a.entries = 64;
    a.owned = expandBlocks_;
    a.flagsOff = (size_t)2 * P * xWords_;
    a.arrive = alloc<unsigned>((size_t)kFxCounters * kFxStride);
    a.error = &d_.status->error;
    int* dev = alloc<int>(2);   // [bad, sink]
    m.bad = dev;
    unsigned long long* verdict = alloc<unsigned long long>(2);
    SBMP_HIP(hipMemsetAsync(dev, 0, sizeof(int) * 2, stream_));
    SBMP_HIP(hipMemsetAsync(&d_.status->error, 0, sizeof(int), stream_));
    for (int pass = 2; pass < 4; ++pass) {
        launch_mirror_probe(m, 0, pass, reinterpret_cast<float*>(dev + 1), stream_);   // old lines cached
        SBMP_HIP(hipMemsetAsync(a.arrive, 0, sizeof(unsigned) * kFxCounters * kFxStride, stream_));
        ex_->barrier(stream_);   // every rank's touch before any push
        a.seq = ++xSeq_;         // the same count on every rank (the fused exchange's base follows it)
        launch_fx_probe(a, pass, stream_);
        launch_mirror_probe(m, 2, pass, nullptr, stream_);   // the next launch: plain loads, compared
    }
    SBMP_HIP(hipGetLastError());
    int bad = 0, error = 0;
    SBMP_HIP(hipMemcpyAsync(&bad, dev, sizeof(int), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipMemcpyAsync(&error, &d_.status->error, sizeof(int), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    SBMP_HIP(hipMemsetAsync(&d_.status->error, 0, sizeof(int), stream_));
    bool ok = bad == 0 && error == 0;
    if (!ok) fprintf(stderr, "sbmp: rank %d: fused exchange check: %d stale or wrong words, wait error %d\n", d_.rank,
                     bad, error);
    if (const char* f = getenv("SBMP_FUSED_SELFTEST"))   // tests: this rank reports a failure
        if (std::string(f) == "fail") ok = false;
    const unsigned long long badv = ok ? 0ull : 1ull;
    SBMP_HIP(hipMemcpyAsync(verdict, &badv, sizeof(badv), hipMemcpyHostToDevice, stream_));
    ex_->allreduce_u64(verdict, verdict + 1, 1, stream_);
    unsigned long long anyBad = 0;
    SBMP_HIP(hipMemcpyAsync(&anyBad, verdict + 1, sizeof(anyBad), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    return anyBad == 0;
}

KgmtPlanner::~KgmtPlanner() {
    if (stream_) {
        (void)hipSetDevice(p_.device);
        (void)hipStreamSynchronize(stream_);
    }
    for (auto& q : pending_) {
        (void)hipEventDestroy(q.a);
        (void)hipEventDestroy(q.b);
    }
    for (hipEvent_t e : eventPool_) (void)hipEventDestroy(e);
    for (void* ptr : allocs_) (void)hipFree(ptr);
    if (poll_) (void)hipHostFree(poll_);
    if (obs_) (void)hipFree(obs_);
    if (dStage_) (void)hipHostFree(dStage_);
    if (gridStart_) (void)hipFree(gridStart_);
    if (gridBoxes_) (void)hipFree(gridBoxes_);
    if (stream_ && ownStream_) (void)hipStreamDestroy(stream_);
}

void KgmtPlanner::begin(const float* initial, const float* goal, const float* d_obstacles, int nObs, uint64_t seed) {
    if (!initial || !goal) throw Error(SBMP_ERR_INVALID_ARGUMENT, "initial/goal must be non-NULL");
    if (nObs < 0 || (nObs > 0 && !d_obstacles)) throw Error(SBMP_ERR_INVALID_ARGUMENT, "bad obstacles");
    // D15: a non-finite root (x, y, theta, v) would only propagate NaN children; the
    // kernels' min/max segment bounds rely on finite states (kgmt_device.h).
    for (int i = 0; i < 4; ++i)
        if (!std::isfinite(initial[i]))
            throw Error(SBMP_ERR_INVALID_ARGUMENT, "initial state (x, y, theta, v) must be finite");
    SBMP_HIP(hipSetDevice(p_.device));
    KgmtDev& d = d_;
    hipStream_t s = stream_;
    // Constructor state (KGMT.cu:16-72): zero-filled vectors, parents -1, R1Score 1.0.
    SBMP_HIP(hipMemsetAsync(d.treeState, 0, sizeof(float4) * d.M, s));
    SBMP_HIP(hipMemsetAsync(d.treeCtrl, 0, sizeof(float4) * d.M, s));
    launch_fill_i32(d.treeParent, -1, d.M, s);
    SBMP_HIP(hipMemsetAsync(xSend_, 0, sizeof(unsigned long long) * xWords_, s));
    if (xSendOdd_ != xSend_) SBMP_HIP(hipMemsetAsync(xSendOdd_, 0, sizeof(unsigned long long) * xWords_, s));
    if (local_) SBMP_HIP(hipMemsetAsync(local_, 0, sizeof(unsigned long long) * localWords_, s));
    if (xRecv_ != xSend_) SBMP_HIP(hipMemsetAsync(xRecv_, 0, sizeof(unsigned long long) * xWords_, s));
    if (d.fusedX) {   // exchange t of this plan has sequence number xSeqBase + t
        SBMP_HIP(hipMemsetAsync(d.xArrive, 0, sizeof(unsigned) * 2 * kFxCounters * kFxStride, s));
        d.xSeqBase = xSeq_;
    }
    SBMP_HIP(hipMemsetAsync(d.R1, 0, sizeof(int) * 2 * 5 * d.nR1, s));   // both parities
    SBMP_HIP(hipMemsetAsync(d.R2Avail, 0, sizeof(uint32_t) * 2 * (d.nR2 / 32), s));
    if (stepCapable_) SBMP_HIP(hipMemsetAsync(d.stepPub, 0, sizeof(unsigned long long) * 2 * (d.nR1 + d.nR2 / 32), s));
    if (stepCapable_ && !d.sharded) {
        SBMP_HIP(hipMemsetAsync(d.stepCnt, 0, sizeof(int) * 2 * kMaxStepBlocks, s));
        SBMP_HIP(hipMemsetAsync(d.stepDelta, 0, sizeof(unsigned long long) * 3 * kDeltaReps * d.nR1, s));
        SBMP_HIP(hipMemsetAsync(d.stepR2New, 0, sizeof(uint32_t) * 3 * kNewReps * (d.nR2 / 32), s));
    }
    SBMP_HIP(hipMemsetAsync(d.R2Snap, 0, sizeof(uint32_t) * (d.nR2 / 32), s));
    SBMP_HIP(hipMemsetAsync(d.R2Valid, 0, sizeof(int) * d.nR2, s));
    SBMP_HIP(hipMemsetAsync(d.R2Invalid, 0, sizeof(int) * d.nR2, s));
    launch_fill_f32(d.R1Score, 1.0f, 2 * d.nR1, s);
    SBMP_HIP(hipMemsetAsync(d.ctrl, 0, sizeof(IterCtrl) * (p_.numIterations + 2), s));

    // Obstacles: a private float4 copy of the caller's device array (KGMT.cu:80 takes
    // d_obstacles by pointer; copying keeps the row layout 16-B aligned).
    if (nObs > obsCap_) {
        if (obs_) SBMP_HIP(hipFree(obs_));
        obs_ = nullptr;
        SBMP_HIP(hipMalloc(&obs_, sizeof(float4) * nObs));
        obsCap_ = nObs;
    }
    if (nObs > 0)
        SBMP_HIP(hipMemcpyAsync(obs_, d_obstacles, sizeof(float4) * nObs, hipMemcpyDeviceToDevice, s));
    d.obstacles = obs_;
    d.nObs = nObs;
    d.obsNaN = 0;
    if (nObs > 0 && nObs <= kMaxRegObs) {   // register lists: wave_cull's separation metric ignores NaN
        float h[4 * kMaxRegObs];
        SBMP_HIP(hipMemcpyAsync(h, d_obstacles, sizeof(float) * 4 * nObs, hipMemcpyDeviceToHost, s));
        SBMP_HIP(hipStreamSynchronize(s));
        for (int i = 0; i < 4 * nObs; ++i)
            if (std::isnan(h[i])) d.obsNaN = 1;
    }
    // Large obstacle lists: the uniform-grid index (include/sbmp/obstacle_grid.h),
    // built on the host from the caller's boxes; the global all-boxes loop remains
    // as variant 5.
    d.gridG = 0;
    d.gridInvW = d.gridInvH = 0.0f;
    d.gridStart = nullptr;
    d.gridBoxes = nullptr;
    if (nObs > 0 && ((nObs > kMaxLdsObs && expandVariant_ != 5) || expandVariant_ == 4)) build_grid(d_obstacles, nObs);
    choose_form(d_obstacles, nObs);
    d.goalX = goal[0];
    d.goalY = goal[1];

    // Root (KGMT.cu:85-97).
    const int r1 = getR1(initial[0], initial[1], d.R1Size, d.N);
    const int r2 = getR2(initial[0], initial[1], r1, d.R1Size, d.N, d.R2Size, d.n);
    launch_seed_root(d, make_float4(initial[0], initial[1], initial[2], initial[3]),
                     make_float4(initial[4], initial[5], initial[6], 0.0f), r1, r2, s);
    // curand_init(seed, slot, 0) for every slot (KGMT.cu:109-111, D1).
    launch_init_slots(d, curand_seed_state(seed), jumps_, nbits_, expandBlocks_, s);
    SBMP_HIP(hipGetLastError());
    // tests: SBMP_INJECT_WAIT_ERROR=<kErr*> starts the plan as if a bounded in-kernel wait
    // had already given up, so the host's error paths can be exercised without a hang
    if (const char* inj = getenv("SBMP_INJECT_WAIT_ERROR")) {
        const int code = atoi(inj);
        SBMP_HIP(hipStreamSynchronize(s));   // after k_seed_root's reset
        SBMP_HIP(hipMemcpy(&d.status->error, &code, sizeof(int), hipMemcpyHostToDevice));
    }

    t_next_ = 1;
    lastFolded_ = 0;
    begun_ = true;
    wallMs_ = 0.0;
    wallFixed_ = false;
    SBMP_HIP(hipStreamSynchronize(s));
    poll_->word = 0;   // no k_step of this plan has run (the stream is idle)
    if (ex_) ex_->barrier(s);   // every rank set up before the first (time-bounded) exchange
    t0_ = now_ms();
    if (d.stepMode) flushed_ = false;   // k_step(1) plans iteration 1 itself
    else launch_finish(d, 0, 0, s, timing(K_FINISH));   // prepares iteration 1
    SBMP_HIP(hipGetLastError());
}

void KgmtPlanner::choose_form(const float* d_obstacles, int nObs) {
    KgmtDev& d = d_;
    // k_step's expanders wait for workgroup 0, so every workgroup of the launch must be
    // resident at once; the dispatch order is not defined.  A list that leaves too few
    // workgroups per CU (LDS near kMaxLdsObs boxes at 262,144 slots per rank) takes the
    // two-launch form on one rank, and the grid index on a sharded rank (whose exchange
    // layout is k_step's); both are bit-exact for every list.
    d.stepMode = stepCapable_ ? 1 : 0;
    neededGroups_ = 1 + (d.sharded ? d.nBlocks / d.nranks : d.nBlocks);
    // a sharded rank stages the exchange's u16 block counts in LDS (2 B per global block)
    // unless that costs residency (below) or SBMP_C16_LDS=0
    const char* cv = getenv("SBMP_C16_LDS");
    d.c16Lds = (d.sharded && !(cv && atoi(cv) == 0)) ? 1 : 0;
    StepResidency why;
    residentGroups_ = stepCapable_ ? step_resident_groups(d, p_.agent, expandVariant_, &why) : 0;
    // SBMP_STEP_RESIDENCY=warn: sharded ranks that share one GPU (a rehearsal on one
    // device), where the query answers for the device the other processes hold too
    const char* rv = getenv("SBMP_STEP_RESIDENCY");
    const bool warnOnly = d.sharded && rv && std::string(rv) == "warn";
    if (stepCapable_ && residentGroups_ < neededGroups_ && warnOnly) {
        if (!formLogged_)
            fprintf(stderr, "sbmp: rank %d: k_step needs %d resident workgroups, the occupancy query gives %d "
                            "(%d per CU x %d CUs); SBMP_STEP_RESIDENCY=warn: launching it as is\n",
                    d.rank, neededGroups_, residentGroups_, why.perCU, why.cus);
        formLogged_ = true;
    } else if (stepCapable_ && residentGroups_ < neededGroups_) {
        const int before = residentGroups_;
        const char* how = "two launches per iteration";
        auto fits = [&]() {
            residentGroups_ = step_resident_groups(d, p_.agent, expandVariant_, &why);
            return residentGroups_ >= neededGroups_;
        };
        if (!d.sharded) {
            d.stepMode = 0;
        } else if (d.c16Lds && (d.c16Lds = 0, fits())) {   // row positions from the block words instead
            how = "this rank reads row positions from the exchange's block words (no LDS row table)";
        } else if (!d.gridStart && nObs > 0) {
            build_grid(d_obstacles, nObs);
            how = "this rank indexes the obstacles with the uniform grid";
            d.c16Lds = (cv && atoi(cv) == 0) ? 0 : 1;
            if (!fits() && d.c16Lds) {
                d.c16Lds = 0;
                (void)fits();
                how = "this rank indexes the obstacles with the uniform grid, without the LDS row table";
            }
        }
        if (d.sharded && residentGroups_ < neededGroups_)
            throw Error(SBMP_ERR_INVALID_ARGUMENT,
                        "k_step needs " + std::to_string(neededGroups_) + " resident workgroups per rank; the device holds " +
                            std::to_string(residentGroups_) + " (" + std::to_string(why.perCU) + " per CU x " +
                            std::to_string(why.cus) + " CUs at " + std::to_string(why.dynLds) + " B of dynamic LDS)");
        if (!formLogged_) {
            fprintf(stderr, "sbmp: %d obstacles: k_step needs %d workgroups resident, the device holds %d; %s\n", nObs,
                    neededGroups_, before, how);
            formLogged_ = true;
        }
    }
}

void KgmtPlanner::path_info(sbmp_path_info* out) {
    const KgmtDev& d = d_;
    out->stepForm = d.stepMode ? 1 : 0;
    out->obstacleForm = d.gridStart                    ? SBMP_OBS_GRID
                        : d.nObs > kMaxLdsObs           ? SBMP_OBS_GLOBAL
                        : (d.nObs <= kMaxRegObs && (expandVariant_ == 0 || expandVariant_ == 3)) ? SBMP_OBS_REGISTERS
                                                        : SBMP_OBS_LDS;
    out->residentGroups = residentGroups_;
    out->neededGroups = neededGroups_;
    out->exchange = !d.sharded ? SBMP_EXCHANGE_NONE : (oneshot_ ? SBMP_EXCHANGE_ONESHOT : SBMP_EXCHANGE_COLLECTIVE);
    out->nranks = d.nranks;
    out->rank = d.rank;
    out->commRanks = ex_ ? ex_->comm_ranks() : 0;
    out->listMirror = d.stepMirror ? 1 : 0;
    out->fusedExchange = d.fusedX ? 1 : 0;
    out->oneshotCheck = oneshotCheck_;
    out->mirrorCheck = mirrorCheck_;
    out->fusedCheck = fusedCheck_;
    out->rowTableLds = d.c16Lds;
}

void KgmtPlanner::build_grid(const float* d_obstacles, int nObs) {
    KgmtDev& d = d_;
    {
        std::vector<float> h((size_t)4 * nObs);
        SBMP_HIP(hipMemcpy(h.data(), d_obstacles, sizeof(float) * h.size(), hipMemcpyDeviceToHost));
        // k_step stages the cell-start table in LDS (G^2 + 1 ints): at most kMaxLdsGridG
        // cells a side (32 KB); any G gives the same answers, a coarser one more boxes per cell
        const HostObstacleGrid g =
            build_obstacle_grid(h.data(), nObs, d.width, d.height, std::min(grid_resolution(nObs), kMaxLdsGridG));
        // kGridBatch rows past the end that no segment meets ((+inf, +inf) - (-inf, -inf): the
        // separation metric is +inf): grid_free_fast loads and tests whole batches
        const size_t nStart = g.start.size(), nBoxes = g.boxes.size() + kGridBatch;
        if (nStart > gridStartCap_) {
            if (gridStart_) SBMP_HIP(hipFree(gridStart_));
            gridStart_ = nullptr;
            SBMP_HIP(hipMalloc(&gridStart_, sizeof(int) * nStart));
            gridStartCap_ = nStart;
        }
        if (nBoxes > gridBoxesCap_) {
            if (gridBoxes_) SBMP_HIP(hipFree(gridBoxes_));
            gridBoxes_ = nullptr;
            SBMP_HIP(hipMalloc(&gridBoxes_, sizeof(float4) * nBoxes));
            gridBoxesCap_ = nBoxes;
        }
        SBMP_HIP(hipMemcpy(gridStart_, g.start.data(), sizeof(int) * nStart, hipMemcpyHostToDevice));
        std::vector<float4> rows(nBoxes, make_float4(INFINITY, INFINITY, -INFINITY, -INFINITY));
        if (!g.boxes.empty()) std::memcpy(rows.data(), g.boxes.data(), sizeof(float4) * g.boxes.size());
        SBMP_HIP(hipMemcpy(gridBoxes_, rows.data(), sizeof(float4) * nBoxes, hipMemcpyHostToDevice));
        for (float v : h)   // grid_free_fast's separation metric needs boxes without NaN
            if (std::isnan(v)) d.obsNaN = 1;
        d.gridG = g.g;
        d.gridInvW = g.invW;
        d.gridInvH = g.invH;
        d.gridStart = gridStart_;
        d.gridBoxes = gridBoxes_;
    }
}

void KgmtPlanner::enqueue(int iterations) {
    if (!begun_) throw Error(SBMP_ERR_STATE, "begin() has not been called");
    if (d_.sharded && !ex_) throw Error(SBMP_ERR_STATE, "a local-group rank is driven by its group");
    for (int i = 0; i < iterations; ++i) {
        const int t = take_iteration();
        if (t == 0) break;
        if (d_.stepMode) {
            stage_step(t);
            if (d_.sharded) stage_exchange(t);
            stage_fold(t);
            continue;
        }
        stage_expand(t);
        if (d_.sharded) {
            stage_pack(t);
            stage_exchange(t);
        }
        stage_finish(t);
        stage_fold(t);
    }
    SBMP_HIP(hipGetLastError());
}

int KgmtPlanner::take_iteration() {
    if (!begun_ || t_next_ > p_.numIterations) return 0;
    return t_next_++;
}

void KgmtPlanner::stage_expand(int t) {
    launch_expand(d_, t, p_.agent, expandBlocks_, expandVariant_, stream_, timing(K_EXPAND));
}

void KgmtPlanner::stage_pack(int t) {
    launch_pack(d_, t, expandBlocks_, stream_, timing(K_PACK));
}

void KgmtPlanner::stage_step(int t) {
    upload_dev();
    launch_step(d_, t, 1, p_.agent, expandVariant_, stream_, timing(K_STEP));
    flushed_ = false;
}

void KgmtPlanner::stage_exchange(int t) {
    if (!ex_) return;
    if (d_.fusedX) {   // k_step(t) ran the exchange itself
        ++xSeq_;
        if (xSeq_ != d_.xSeqBase + (unsigned long long)t)
            throw Error(SBMP_ERR_STATE, "fused exchange: sequence " + std::to_string(xSeq_) + " at iteration " +
                                            std::to_string(t));
        return;
    }
    const unsigned long long* send = exchange_send(t);
    if (oneshot_) {
        ++xSeq_;
        OneshotLayout cx{};
        if (shStep_ && compactX_) {   // the sharded k_step layout, compact on the wire
            cx.on = 1;
            cx.nR1 = d_.nR1;
            cx.rowOff = d_.xRowOff;
            cx.rows = expandBlocks_;
            cx.cntOff = d_.xCntOff;
            cx.owned = expandBlocks_;
            cx.nBlocks = d_.nBlocks;
            cx.newOff = d_.xNewOff;
            cx.newWords = (int)xWords_ - d_.xNewOff;
            cx.c16Off = d_.xC16Off;
        }
        long long* tl = (d_.timelineFin && t == d_.timelineIter) ? d_.timelineFin + kTimelineStamps : nullptr;
        launch_oneshot(inbox_, send, xRecv_, (long long)xWords_, d_.nranks, d_.rank, xSeq_, &d_.status->error,
                       stream_, timing(K_XCHG), &cx, tl);
    } else {
        ex_->allreduce_u64(send, xRecv_, xWords_, stream_);
    }
}

// k_step mode: complete the last enqueued iteration (insert it, plan t_next) before a read-back
void KgmtPlanner::flush() {
    if (d_.stepMode && begun_ && !flushed_) {
        upload_dev();
        launch_step(d_, t_next_, 0, p_.agent, expandVariant_, stream_, KernelTiming());
        flushed_ = true;
    }
}

void KgmtPlanner::stage_finish(int t) {
    // single rank: one insert workgroup per 256-slot block up to 1,024 blocks, then up to
    // kInsertMaxR blocks each (insert_blocks); sharded: the record-driven insert and the
    // owner's GNew clear, one workgroup per owned block
    launch_finish(d_, t, d_.sharded ? expandBlocks_ : kInsertBase - 1 + finish_insert_groups(d_.nBlocks), stream_,
                  timing(K_FINISH));
}

void KgmtPlanner::stage_fold(int t) {
    if (t - lastFolded_ >= kFoldEvery) fold_to(t);
}

// Bring R2Valid / R2Invalid up to iteration tLast (k_fold_r2 over the key log).
void KgmtPlanner::fold_to(int tLast) {
    if (tLast <= lastFolded_) return;
    if (d_.r2log) launch_fold_r2(d_, lastFolded_ + 1, tLast, stream_, timing(K_FOLD));
    lastFolded_ = tLast;
}

// k_step reads the plan struct at d_.devSelf: refresh that copy when d_ changed (at
// begin(), or a diagnostics switch), from pinned memory not touched while a copy is queued.
void KgmtPlanner::upload_dev() {
    if (!dDev_) throw Error(SBMP_ERR_STATE, "k_step: the plan struct has no device copy");
    if (uploaded_ && std::memcmp(&d_, dStage_, sizeof(KgmtDev)) == 0) return;
    if (uploaded_) SBMP_HIP(hipStreamSynchronize(stream_));   // the previous copy has been read
    std::memcpy(dStage_, &d_, sizeof(KgmtDev));
    SBMP_HIP(hipMemcpyAsync(dDev_, dStage_, sizeof(KgmtDev), hipMemcpyHostToDevice, stream_));
    uploaded_ = true;
}

void KgmtPlanner::sync() {
    flush();
    SBMP_HIP(hipStreamSynchronize(stream_));
    if (!wallFixed_) wallMs_ = now_ms() - t0_;
    if (d_.timeline && !timelineDumped_ && t_next_ > d_.timelineIter) {
        const size_t n = (size_t)expandBlocks_ * (kBlock / kWave) * kTimelineStamps;
        const size_t nf = (size_t)(1 + d_.nBlocks) * kTimelineStamps;
        std::vector<long long> h(n + nf);
        SBMP_HIP(hipMemcpy(h.data(), d_.timeline, sizeof(long long) * (n + nf), hipMemcpyDeviceToHost));
        std::string path = getenv("SBMP_TIMELINE_OUT") ? getenv("SBMP_TIMELINE_OUT") : "sbmp_timeline.bin";
        if (d_.nranks > 1) path += ".r" + std::to_string(d_.rank);   // a local group's ranks share the process
        if (FILE* f = fopen(path.c_str(), "wb")) {
            fwrite(h.data(), sizeof(long long), n, f);
            fclose(f);
        }
        if (FILE* f = fopen((path + ".fin").c_str(), "wb")) {   // k_finish stamps
            fwrite(h.data() + n, sizeof(long long), nf, f);
            fclose(f);
        }
        timelineDumped_ = true;
    }
}

void KgmtPlanner::read_ctrl(std::vector<IterCtrl>& c, PlannerStatus& st) {
    c.resize(p_.numIterations + 2);
    SBMP_HIP(hipMemcpyAsync(c.data(), d_.ctrl, sizeof(IterCtrl) * c.size(), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipMemcpyAsync(&st, d_.status, sizeof(PlannerStatus), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
}

int KgmtPlanner::last_executed(const std::vector<IterCtrl>& c) const {
    int itr = 0;
    for (int t = 1; t < t_next_ && t < (int)c.size(); ++t) {
        if (c[t].executed) itr = t;
        else break;
    }
    return itr;
}

bool KgmtPlanner::active() {
    if (!begun_) return false;
    flush();   // k_step mode: the flush pass writes ctrl[t_next] and the goal of t_next - 1
    // ctrl has numIterations + 2 entries, so t_next <= numIterations + 1 is in range
    SBMP_HIP(hipMemcpyAsync(&poll_->ctrl, d_.ctrl + t_next_, sizeof(IterCtrl), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipMemcpyAsync(&poll_->status, d_.status, sizeof(PlannerStatus), hipMemcpyDeviceToHost, stream_));
    sync();
    if (t_next_ > p_.numIterations) return false;
    const IterCtrl c = poll_->ctrl;
    const PlannerStatus st = poll_->status;
    if (st.error) throw_wait_error(st.error);
    // ctrl[t_next] was written by the last enqueued plan kernel: it says whether the
    // next iteration would run (tree not full, limit not reached); the goal ends it too.
    return c.run && st.goalIdx == kNoGoal;
}

void Planner::run(int pollEvery) {
    if (!dumpDir_.empty()) {   // one iteration at a time, dumping each (KGMT.cu:263-290)
        int done = 0;
        while (true) {
            enqueue(1);
            sync();
            const std::vector<sbmp_iter_record> log = iter_log();
            for (const sbmp_iter_record& e : log)
                if (e.itr > done) dump_iteration(dumpDir_, e.itr);
            if (!log.empty()) done = log.back().itr;
            rank_barrier();   // the dump's host time must not count against a peer's exchange wait
            if (!active()) break;
        }
        sync();
        return;
    }
    if (pollEvery < 1) pollEvery = 1;
    while (true) {
        enqueue(pollEvery);
        if (!active()) break;
    }
    sync();
}

// plan(): a single k_step rank keeps kAhead iterations in flight and watches the pinned
// word its planner workgroups store (KgmtDev::hostPoll) instead of polling with stream
// synchronisations (run(8): a flush launch, two copies and a synchronisation every 8
// iterations).  The planner of launch t inserts t-1's children and checks them for the
// goal, so when its word says "goal" (or "loop ended"), the plan ends with launch t:
// wallMs is taken when launch t has ended (the next launch's planner has stored its word:
// a planner whose loop has ended stores it too; or the stream is idle), before the
// launches already queued behind it (no-ops: a found goal or an ended loop stops every
// later iteration) drain.  A planner that finds status.error set (an earlier launch's
// bounded wait gave up) reports the loop as ended, and the error is raised after sync().
// Time-to-first-solution is then the end of the iteration that inserts the goal node
// (BASELINE.md), without the polls.  The result is the same as run(8)'s.
void KgmtPlanner::run_plan() {
    if (d_.stepMode && !d_.sharded && d_.hostPoll && dumpDir_.empty()) run_to_goal();
    else run(8);
}

void KgmtPlanner::run_to_goal() {
#ifndef SBMP_PLAN_AHEAD
#define SBMP_PLAN_AHEAD 3
#endif
    constexpr int kAhead = SBMP_PLAN_AHEAD;   // iterations in flight (2, 3, 4 within noise; 6 slower: profiles/r05/ttfs/)
    const volatile unsigned long long* w = &poll_->word;
    int issued = t_next_ - 1;   // iterations launched
    int goalSeen = -1;          // the launch whose planner first reported the goal (or the loop's end)
    while (true) {
        const unsigned long long v = *w;
        const int seen = (int)(v >> 2);   // the last launch whose planner has run
        if (goalSeen < 0 && (v & 3ull)) goalSeen = seen;
        // launch goalSeen has ended once a later launch's planner has run (stream order), or
        // once the stream is idle; no event per launch (their marker packets cost ~2 us each)
        if (goalSeen >= 0) {
            const hipError_t q = (seen > goalSeen) ? hipSuccess : hipStreamQuery(stream_);
            if (seen > goalSeen || q != hipErrorNotReady) {
                wallMs_ = now_ms() - t0_;
                wallFixed_ = true;
                break;
            }
        } else if (t_next_ <= p_.numIterations && issued - seen < kAhead) {
            enqueue(1);
            ++issued;
            continue;
        } else if (t_next_ > p_.numIterations) {
            break;   // every iteration launched: sync() ends it
        } else {   // the stream drained (or failed) without the word this loop waits for: sync() decides
            const hipError_t q = hipStreamQuery(stream_);
            if (q != hipErrorNotReady && (q != hipSuccess || (int)((*w) >> 2) < issued)) break;
        }
        __builtin_ia32_pause();
    }
    sync();
    // a bounded in-kernel wait that gave up (its planner's word ended the loop above):
    // raised here, as run(8) raises it from active(), whether or not a result is read
    SBMP_HIP(hipMemcpyAsync(&poll_->status, d_.status, sizeof(PlannerStatus), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    if (poll_->status.error) throw_wait_error(poll_->status.error);
}

void KgmtPlanner::result(sbmp_plan_result* r) {
    sync();
    std::vector<IterCtrl> c;
    PlannerStatus st;
    read_ctrl(c, st);
    if (st.error) throw_wait_error(st.error);
    const int itr = last_executed(c);
    memset(r, 0, sizeof(*r));
    r->iterations = itr;
    r->treeSize = itr > 0 ? c[itr].treeSize + c[itr].A : 1;
    for (int t = 1; t <= itr; ++t) {
        r->samplesGenerated += c[t].S;
        r->accepted += c[t].A;
    }
    r->goalIndex = (st.goalIdx == kNoGoal) ? -1 : st.goalIdx;
    r->costToGoal = 0.0f;
    if (r->goalIndex >= 0) {
        float4 gc;
        SBMP_HIP(hipMemcpy(&gc, d_.treeCtrl + r->goalIndex, sizeof(float4), hipMemcpyDeviceToHost));
        r->costToGoal = gc.w;
    }
    r->wallMs = wallMs_;
    r->stalled = (itr > 0 && c[itr].nG == 0) ? 1 : 0;
}

std::vector<sbmp_iter_record> KgmtPlanner::iter_log() {
    sync();
    std::vector<IterCtrl> c;
    PlannerStatus st;
    read_ctrl(c, st);
    const int itr = last_executed(c);
    std::vector<sbmp_iter_record> out;
    for (int t = 1; t <= itr; ++t) {
        sbmp_iter_record e;
        e.itr = t;
        e.treeSizeBefore = c[t].treeSize;
        e.nG = c[t].nG;
        e.k = c[t].k;
        e.nExp = c[t].nExp;
        e.S = c[t].S;
        e.A = c[t].A;
        e.treeSizeAfter = c[t].treeSize + c[t].A;
        e.goalIdx = (t == itr && st.goalIdx != kNoGoal) ? st.goalIdx : -1;
        out.push_back(e);
    }
    return out;
}

void KgmtPlanner::copy_tree(float* samples, int* parent, float* costs) {
    sync();
    const size_t M = d_.M;
    float* dS = nullptr;
    float* dC = nullptr;
    SBMP_HIP(hipMalloc(&dS, sizeof(float) * M * 7));
    SBMP_HIP(hipMalloc(&dC, sizeof(float) * M));
    launch_export_tree(d_, dS, dC, stream_);
    if (samples) SBMP_HIP(hipMemcpyAsync(samples, dS, sizeof(float) * M * 7, hipMemcpyDeviceToHost, stream_));
    if (costs) SBMP_HIP(hipMemcpyAsync(costs, dC, sizeof(float) * M, hipMemcpyDeviceToHost, stream_));
    if (parent) SBMP_HIP(hipMemcpyAsync(parent, d_.treeParent, sizeof(int) * M, hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    (void)hipFree(dS);
    (void)hipFree(dC);
}

// The replicated state's digest (k_state_hash): every rank of a sharded run holds the same
// tree, tables and control blocks, so every rank's digest must be the same.
unsigned long long KgmtPlanner::state_hash() {
    sbmp_plan_result r;
    result(&r);   // syncs (the flush pass has inserted the last iteration)
    unsigned long long* dev = alloc_scratch_u64();
    SBMP_HIP(hipMemsetAsync(dev, 0, sizeof(unsigned long long), stream_));
    const int rows = std::min(std::max(r.treeSize, 1), d_.M);
    const int tp = d_.stepMode ? (t_next_ & 1) : 0;   // the tables of iteration t_next (copy_regions' parity)
    launch_state_hash(d_, rows, tp, r.iterations, dev, stream_);
    unsigned long long h = 0;
    SBMP_HIP(hipMemcpyAsync(&h, dev, sizeof(h), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    return h;
}

unsigned long long* KgmtPlanner::alloc_scratch_u64() {
    if (!scratch_) scratch_ = alloc<unsigned long long>(8);
    return scratch_;
}

int KgmtPlanner::solution_path(int node, int* rows, float* samples, float* costs, int capacity) {
    sbmp_plan_result r;
    result(&r);   // syncs
    if (node < 0) {
        if (r.goalIndex < 0) return 0;
        node = r.goalIndex;
    }
    const int rowsInTree = std::min(r.treeSize, d_.M);
    if (node >= rowsInTree) throw Error(SBMP_ERR_INVALID_ARGUMENT, "node is not a tree row");
    const int maxDepth = p_.numIterations + 2;   // one level per iteration, plus the root
    int* dI = nullptr;
    float* dF = nullptr;
    SBMP_HIP(hipMalloc(&dI, sizeof(int) * (1 + (size_t)maxDepth)));
    SBMP_HIP(hipMalloc(&dF, sizeof(float) * 8 * (size_t)maxDepth));
    launch_solution_path(d_, node, maxDepth, dI, dI + 1, dF, dF + 7 * (size_t)maxDepth, stream_);
    std::vector<int> hi(1 + (size_t)maxDepth);
    std::vector<float> hf(8 * (size_t)maxDepth);
    SBMP_HIP(hipMemcpyAsync(hi.data(), dI, sizeof(int) * hi.size(), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipMemcpyAsync(hf.data(), dF, sizeof(float) * hf.size(), hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    (void)hipFree(dI);
    (void)hipFree(dF);
    const int len = hi[0];
    if (len < 0) throw Error(SBMP_ERR_STATE, "parent chain longer than numIterations + 2 rows");
    if ((rows || samples || costs) && capacity < len)
        throw Error(SBMP_ERR_INVALID_ARGUMENT, "capacity " + std::to_string(capacity) + " < path length " +
                                                   std::to_string(len));
    if (rows) memcpy(rows, hi.data() + 1, sizeof(int) * len);
    if (samples) memcpy(samples, hf.data(), sizeof(float) * 7 * len);
    if (costs) memcpy(costs, hf.data() + 7 * (size_t)maxDepth, sizeof(float) * len);
    return len;
}

void KgmtPlanner::copy_unexplored(float* samples, int* uParent) {
    sync();
    const size_t M = d_.M, n = d_.nSlots;
    float* dS = nullptr;
    int* dP = nullptr;
    SBMP_HIP(hipMalloc(&dS, sizeof(float) * n * 7));
    SBMP_HIP(hipMalloc(&dP, sizeof(int) * n));
    launch_export_unexplored(d_, dS, dP, stream_);
    // The reference's unexplored buffer has M rows; slots never used stay 0 / -1.
    std::vector<float> hs(n * 7);
    std::vector<int> hp(n);
    SBMP_HIP(hipMemcpyAsync(hs.data(), dS, sizeof(float) * n * 7, hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipMemcpyAsync(hp.data(), dP, sizeof(int) * n, hipMemcpyDeviceToHost, stream_));
    SBMP_HIP(hipStreamSynchronize(stream_));
    (void)hipFree(dS);
    (void)hipFree(dP);
    if (d_.nranks > 1) {   // rows of slots owned by other ranks are not held here
        for (size_t i = 0; i < n; ++i) {
            if ((int)((i / kBlock) % d_.nranks) != d_.rank) {
                for (int q = 0; q < 7; ++q) hs[i * 7 + q] = 0.0f;
                hp[i] = -1;
            }
        }
    }
    if (samples) {
        memcpy(samples, hs.data(), sizeof(float) * n * 7);
        memset(samples + n * 7, 0, sizeof(float) * (M - n) * 7);
    }
    if (uParent) {
        memcpy(uParent, hp.data(), sizeof(int) * n);
        for (size_t i = n; i < M; ++i) uParent[i] = -1;
    }
}

void KgmtPlanner::copy_flags(uint8_t* G, uint8_t* GNew) {
    sync();
    std::vector<IterCtrl> c;
    PlannerStatus st;
    read_ctrl(c, st);
    const int itr = last_executed(c);
    const int M = d_.M;
    if (G) {
        memset(G, 0, M);
        int lo = 0, hi = 1;
        if (itr > 0) {
            lo = c[itr].gLo + c[itr].nExp;
            hi = c[itr].treeSize + c[itr].A;
        }
        for (int i = lo; i < std::min(hi, M); ++i) G[i] = 1;
    }
    if (GNew) {
        std::vector<unsigned long long> w(d_.nWords);
        if (ex_ && d_.nranks > 1) {   // each rank holds its owned words (zero elsewhere): the sum merges
            unsigned long long* tmp = nullptr;
            SBMP_HIP(hipMalloc(&tmp, sizeof(unsigned long long) * d_.nWords));
            ex_->allreduce_u64(d_.gnewOut, tmp, d_.nWords, stream_);
            SBMP_HIP(hipStreamSynchronize(stream_));
            SBMP_HIP(hipMemcpy(w.data(), tmp, sizeof(unsigned long long) * d_.nWords, hipMemcpyDeviceToHost));
            (void)hipFree(tmp);
        } else {
            SBMP_HIP(hipMemcpy(w.data(), d_.gnewOut, sizeof(unsigned long long) * d_.nWords, hipMemcpyDeviceToHost));
        }
        memset(GNew, 0, M);
        for (int s = 0; s < d_.nSlots; ++s) GNew[s] = (w[s >> 6] >> (s & 63)) & 1ull;
    }
}

void KgmtPlanner::copy_regions(int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score, int* R2Avail,
                               int* R2Valid, int* R2Invalid) {
    if (begun_) fold_to(t_next_ - 1);
    sync();
    std::vector<IterCtrl> c;
    PlannerStatus st;
    read_ctrl(c, st);
    const int itr = last_executed(c);
    const size_t n1 = d_.nR1, n2 = d_.nR2;
    auto cp = [&](void* dst, const void* src, size_t bytes) {
        if (dst) SBMP_HIP(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToHost));
    };
    // k_step keeps the tables of iteration t_next (its flush pass planned it) at parity t_next & 1
    const size_t tp = d_.stepMode ? (size_t)(t_next_ & 1) : 0;
    cp(R1, d_.R1 + tp * 5 * n1, sizeof(int) * n1);
    cp(R1Avail, d_.R1Avail + tp * 5 * n1, sizeof(int) * n1);
    cp(R1Valid, d_.R1Valid + tp * 5 * n1, sizeof(int) * n1);
    cp(R1Invalid, d_.R1Invalid + tp * 5 * n1, sizeof(int) * n1);
    cp(R1Score, d_.R1Score + (itr & 1) * n1, sizeof(float) * n1);
    if (ex_ && (R2Valid || R2Invalid)) {   // sharded: each rank folded its own children
        int* tmp = nullptr;
        SBMP_HIP(hipMalloc(&tmp, sizeof(int) * 2 * n2));
        ex_->allreduce_i32(d_.R2Valid, tmp, n2, stream_);
        ex_->allreduce_i32(d_.R2Invalid, tmp + n2, n2, stream_);
        SBMP_HIP(hipStreamSynchronize(stream_));
        cp(R2Valid, tmp, sizeof(int) * n2);
        cp(R2Invalid, tmp + n2, sizeof(int) * n2);
        (void)hipFree(tmp);
    } else {
        cp(R2Valid, d_.R2Valid, sizeof(int) * n2);
        cp(R2Invalid, d_.R2Invalid, sizeof(int) * n2);
    }
    if (R2Avail) {
        std::vector<uint32_t> bits(n2 / 32);
        SBMP_HIP(hipMemcpy(bits.data(), d_.R2Avail + tp * (n2 / 32), sizeof(uint32_t) * bits.size(),
                           hipMemcpyDeviceToHost));
        for (size_t i = 0; i < n2; ++i) R2Avail[i] = (bits[i >> 5] >> (i & 31)) & 1u;
    }
}

void KgmtPlanner::copy_rng(uint32_t* states) {
    sync();
    const size_t n = d_.nSlots;
    std::vector<uint4> a(n);
    std::vector<uint2> b(n);
    SBMP_HIP(hipMemcpy(a.data(), d_.rngA, sizeof(uint4) * n, hipMemcpyDeviceToHost));
    SBMP_HIP(hipMemcpy(b.data(), d_.rngB, sizeof(uint2) * n, hipMemcpyDeviceToHost));
    for (size_t i = 0; i < n; ++i) {
        uint32_t* o = states + 6 * i;
        o[0] = a[i].x;
        o[1] = a[i].y;
        o[2] = a[i].z;
        o[3] = a[i].w;
        o[4] = b[i].x;
        o[5] = b[i].y;
    }
}

// KGMT.cu:299-311 with helper.cuh:53-79 formatting.
template <typename T>
static void write_csv(const std::string& path, const T* v, size_t rows, size_t cols) {
    std::ofstream f(path);
    if (!f.is_open()) throw Error(SBMP_ERR_IO, "cannot open " + path);
    f << std::fixed << std::setprecision(10);
    for (size_t i = 0; i < rows; ++i) {
        for (size_t j = 0; j < cols; ++j) {
            f << v[i * cols + j];
            if (j < cols - 1) f << ",";
        }
        f << std::endl;
    }
}

void KgmtPlanner::copy_r2_partial(int* R2Valid, int* R2Invalid) {
    if (begun_) fold_to(t_next_ - 1);
    sync();
    SBMP_HIP(hipMemcpy(R2Valid, d_.R2Valid, sizeof(int) * d_.nR2, hipMemcpyDeviceToHost));
    SBMP_HIP(hipMemcpy(R2Invalid, d_.R2Invalid, sizeof(int) * d_.nR2, hipMemcpyDeviceToHost));
}

// The per-iteration dumps of KGMT.cu:263-290 (the reference creates Data/G and
// Data/GNew as well but writes nothing there).  State as at the end of iteration itr:
// tree, parents and the unexplored buffer after its insertion, R1 / R1Avail with its
// children counted, the R1Score its accept test used.
void Planner::dump_iteration(const std::string& dir, int itr) {
    const sbmp_kgmt_params& p = params();
    const size_t M = p.maxTreeSize, n1 = (size_t)p.N * p.N, n2 = n1 * p.n * p.n;
    const std::string base = (dir.empty() ? std::string(".") : dir) + "/Data";
    mkdir((dir.empty() ? std::string(".") : dir).c_str(), 0755);
    mkdir(base.c_str(), 0755);
    for (const char* k : {"Samples", "UnexploredSamples", "Parents", "R1Scores", "R1Avail", "R1", "G", "GNew"})
        mkdir((base + "/" + k).c_str(), 0755);
    std::vector<float> samples(M * 7), costs(M), uS(M * 7), score(n1);
    std::vector<int> parent(M), uP(M), R1(n1), R1A(n1);
    copy_tree(samples.data(), parent.data(), costs.data());
    copy_unexplored(uS.data(), uP.data());
    copy_regions(R1.data(), R1A.data(), nullptr, nullptr, score.data(), nullptr, nullptr, nullptr);
    const std::string i = std::to_string(itr);
    write_csv(base + "/Samples/samples" + i + ".csv", samples.data(), M, 7);
    write_csv(base + "/Parents/parents" + i + ".csv", parent.data(), M, 1);
    write_csv(base + "/R1Scores/R1Scores" + i + ".csv", score.data(), n1, 1);
    write_csv(base + "/R1Avail/R1Avail" + i + ".csv", R1A.data(), n1, 1);
    write_csv(base + "/R1/R1" + i + ".csv", R1.data(), n1, 1);
    write_csv(base + "/UnexploredSamples/unexploredSamples" + i + ".csv", uS.data(), M, 7);
    (void)n2;
}

void Planner::export_csv(const std::string& dir) {
    const sbmp_kgmt_params& p = params();
    const size_t M = p.maxTreeSize, n1 = (size_t)p.N * p.N, n2 = n1 * p.n * p.n;
    mkdir(dir.c_str(), 0755);
    const std::string pre = dir.empty() ? "" : dir + "/";
    std::vector<float> samples(M * 7), costs(M), uS(M * 7), score(n1);
    std::vector<int> parent(M), uP(M), R1(n1), R1A(n1), R1V(n1), R1I(n1), R2A(n2), R2V(n2), R2I(n2);
    std::vector<uint8_t> G(M), GN(M);
    copy_tree(samples.data(), parent.data(), costs.data());
    copy_unexplored(uS.data(), uP.data());
    copy_flags(G.data(), GN.data());
    copy_regions(R1.data(), R1A.data(), R1V.data(), R1I.data(), score.data(), R2A.data(), R2V.data(), R2I.data());
    std::vector<int> Gi(G.begin(), G.end());
    write_csv(pre + "samples.csv", samples.data(), M, 7);
    write_csv(pre + "unexploredSamples.csv", uS.data(), M, 7);
    write_csv(pre + "parentRelations.csv", parent.data(), M, 1);
    write_csv(pre + "uParentIdx.csv", uP.data(), M, 1);
    write_csv(pre + "G.csv", Gi.data(), M, 1);
    write_csv(pre + "R2Avail.csv", R2A.data(), n2, 1);
    write_csv(pre + "R1Avail.csv", R1A.data(), n1, 1);
    write_csv(pre + "R1Valid.csv", R1V.data(), n1, 1);
    write_csv(pre + "R2Valid.csv", R2V.data(), n2, 1);
    write_csv(pre + "R1Invalid.csv", R1I.data(), n1, 1);
    write_csv(pre + "R2Invalid.csv", R2I.data(), n2, 1);
    write_csv(pre + "R1Score.csv", score.data(), n1, 1);
    write_csv(pre + "R1.csv", R1.data(), n1, 1);
}

// ---------------------------------------------------------------- profiling
// Events for one launch (null pair when profiling is off).  They are handed to
// hipExtLaunchKernelGGL, which stamps them with the kernel's own start/end.
KernelTiming KgmtPlanner::timing(int id) {
    KernelTiming tm;
    if (!p_.profileKernels) return tm;
    for (hipEvent_t* e : {&tm.start, &tm.stop}) {
        if (!eventPool_.empty()) {
            *e = eventPool_.back();
            eventPool_.pop_back();
        } else {
            SBMP_HIP(hipEventCreate(e));
        }
    }
    pending_.push_back({id, tm.start, tm.stop});
    return tm;
}

void KgmtPlanner::collect_events() {
    for (auto& q : pending_) {
        SBMP_HIP(hipEventSynchronize(q.b));
        float ms = 0.0f;
        SBMP_HIP(hipEventElapsedTime(&ms, q.a, q.b));
        launches_[q.id] += 1;
        totalMs_[q.id] += ms;
        samples_[q.id].push_back(ms);
        eventPool_.push_back(q.a);
        eventPool_.push_back(q.b);
    }
    pending_.clear();
}

static const char* kKernelNames[] = {"k_expand", "k_finish", "k_fold_r2", "k_pack", "k_step", "k_oneshot"};

std::vector<float> KgmtPlanner::kernel_samples(const std::string& name) {
    collect_events();
    for (int i = 0; i < K_COUNT; ++i)
        if (name == kKernelNames[i]) return samples_[i];
    throw Error(SBMP_ERR_INVALID_ARGUMENT, "unknown kernel " + name);
}

std::vector<sbmp_kernel_stat> KgmtPlanner::kernel_stats() {
    collect_events();
    const char* const* names = kKernelNames;
    std::vector<sbmp_kernel_stat> out;
    for (int i = 0; i < K_COUNT; ++i) {
        sbmp_kernel_stat s;
        memset(&s, 0, sizeof(s));
        strncpy(s.name, names[i], sizeof(s.name) - 1);
        s.launches = launches_[i];
        s.totalMs = totalMs_[i];
        out.push_back(s);
    }
    return out;
}

void KgmtPlanner::reset_kernel_stats() {
    collect_events();
    for (int i = 0; i < K_COUNT; ++i) {
        launches_[i] = 0;
        totalMs_[i] = 0.0;
        samples_[i].clear();
    }
}

}  // namespace sbmp
