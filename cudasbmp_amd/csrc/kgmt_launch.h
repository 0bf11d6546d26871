// kgmt_launch.h — host-side launch entry points of kgmt_kernels.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

#include "kgmt_device.h"

namespace sbmp {

// Optional start/stop events stamped by the kernel's dispatch packet.
struct KernelTiming {
    hipEvent_t start = nullptr;
    hipEvent_t stop = nullptr;
};

// variant: obstacle form: 0 = auto, 1 = LDS rolled, 2 = LDS 4-way batched, 3 = registers
// (lists of at most kMaxRegObs boxes; auto picks it there, else 1); lists longer
// than kMaxLdsObs always use the global early-exit form.
void launch_expand(const KgmtDev& d, int t, int agent, int blocks, int variant, hipStream_t s,
                   const KernelTiming& tm = KernelTiming());
// k_fold_r2: add the key log of iterations [tFirst, tLast] (at most kFoldEvery) to R2Valid / R2Invalid.
// k_step(t): one launch per iteration on a single rank; expand == 0: flush pass.
void launch_step(const KgmtDev& d, int t, int expand, int agent, int variant, hipStream_t s,
                 const KernelTiming& tm = KernelTiming());
// Workgroups of the k_step form launch_step would pick for d that the device holds at
// once (occupancy per CU x CUs); k_step needs all of its 1 + blocks resident, since
// its expanders wait for workgroup 0.  0 if the query fails.
struct StepResidency {   // the query's terms, for the message when k_step does not fit
    int perCU = 0, cus = 0;
    long long dynLds = 0;
};
int step_resident_groups(const KgmtDev& d, int agent, int variant, StepResidency* why = nullptr);
void launch_fold_r2(const KgmtDev& d, int tFirst, int tLast, hipStream_t s, const KernelTiming& tm = KernelTiming());
// k_finish(t): insert iteration t (insertBlocks = every global 256-slot block) +
// prepare iteration t+1.  t = 0 prepares iteration 1 only (insertBlocks = 0).
int finish_insert_groups(int nBlocks);   // k_finish's insert workgroups for nBlocks 256-slot blocks
void launch_finish(const KgmtDev& d, int t, int insertBlocks, hipStream_t s,
                   const KernelTiming& tm = KernelTiming());
// Sharded ranks: pack this rank's accepted children of iteration t (blocks = owned blocks).
void launch_pack(const KgmtDev& d, int t, int blocks, hipStream_t s, const KernelTiming& tm = KernelTiming());
// Sharded ranks: recv = sum over ranks of send through IPC-mapped inboxes (inbox[q] =
// rank q's, oneshot_inbox_words() u64 each, zeroed once); seq = this exchange's number
// in the plan's lifetime (1, 2, ...), the same on every rank.
size_t oneshot_inbox_words(long long n, int nranks);
// The list mirror's start-up check (kgmt_kernels.hip, KgmtPlanner::mirror_self_test):
// phase 0 touches this rank's probed entries with plain loads, 1 pushes this rank's
// pattern of `pass` into every rank's mirror (system scope), 2 checks them (plain loads;
// mismatching float4 words are added to *bad).
struct MirrorProbe {
    float4* peer[kMaxRanks];   // every rank's mirror, mapped here
    const float4* own;         // this rank's
    int nranks, rank, nBlocks;   // mirror layout [2][nBlocks][kBlock][kStepEntry]
    int blocks, entries;       // probed: global blocks < blocks, entries < entries, both parities
    int* bad;
};
void launch_mirror_probe(const MirrorProbe& a, int phase, int pass, float* sink, hipStream_t s);
// The fused exchange's order at start-up (KgmtPlanner::fused_self_test): `owned` workgroups
// push entries (both parities, entries < entries, their global block) into every rank's
// mirror, drain, arrive on the replicated sharded counters; the workers flag the peers and
// wait for theirs.  k_mirror_check (phase 2 of launch_mirror_probe) reads the mirror next.
struct FxProbe {
    float4* peer[kMaxRanks];                 // every rank's mirror, mapped here
    unsigned long long* inbox[kMaxRanks];    // every rank's one-shot inbox (flags at flagsOff)
    size_t flagsOff;
    int nranks, rank, nBlocks, owned, entries;
    unsigned* arrive;                        // [kFxReplicas][kFxShards][kFxStride], zeroed per pass
    unsigned long long seq;
    int* error;
};
void launch_fx_probe(const FxProbe& a, int pass, hipStream_t s);
// error: the planner's status word (set to kErrExchange when a peer never arrives).
// compact (sharded k_step): the send layout, sent in compact form (kgmt_kernels.hip).
struct OneshotLayout {
    int on;
    int nR1;                  // R1 cells (kDeltaReps replicas of nR1 words at offset 0)
    int rowOff, rows;         // u64 offset of the row words, rows (ints)
    int cntOff, owned, nBlocks;   // u64 offset of the block words (ints), owned blocks, global blocks
    int newOff, newWords;     // u64 offset and words of the R2New bytes
    int c16Off;               // u64 offset of the u16 block counts (written by the receiver)
};
OneshotCompact oneshot_compact(const OneshotLayout& l);   // the compact layout of l
// tl: diagnostics, 8 stamps per workgroup, or null.
void launch_oneshot(unsigned long long* const* inbox, const unsigned long long* send, unsigned long long* recv,
                    long long n, int nranks, int rank, unsigned long long seq, int* error, hipStream_t s,
                    const KernelTiming& tm = KernelTiming(), const OneshotLayout* compact = nullptr,
                    long long* tl = nullptr);
// Local shard group: recv[q][i] = sum over ranks of send[r][i], for every rank q.
void launch_xsum(const unsigned long long* const* send, unsigned long long* const* recv, int nranks, long long n,
                 hipStream_t s);
void launch_delay(double microseconds, hipStream_t s);
void launch_fill_i32(int* p, int v, long long n, hipStream_t s);
void launch_fill_f32(float* p, float v, long long n, hipStream_t s);
void launch_init_slots(const KgmtDev& d, const Xorwow& base, const uint32_t* jumps, int nbits, int blocks,
                       hipStream_t s);
void launch_solution_path(const KgmtDev& d, int node, int maxDepth, int* out, int* rows, float* samples, float* costs,
                          hipStream_t s);
void launch_seed_root(const KgmtDev& d, float4 rs, float4 rc, int r1, int r2, hipStream_t s);
void launch_export_tree(const KgmtDev& d, float* samples, float* costs, hipStream_t s);
// *out += the digest of tree rows [0, rows), the tables of parity tp and ctrl[1 .. iters]
// (k_state_hash; *out zeroed by the caller).
void launch_state_hash(const KgmtDev& d, int rows, int tp, int iters, unsigned long long* out, hipStream_t s);
void launch_export_unexplored(const KgmtDev& d, float* samples, int* uParent, hipStream_t s);

// xorwow_jump.cpp: cuRAND seeding and the subsequence jump matrices.
Xorwow curand_seed_state(uint64_t seed);
// J[b] = A^(2^(67+b)), b < nbits, each 160 columns x 5 words, concatenated.
const std::vector<uint32_t>& subsequence_jump_matrices(int nbits);

}  // namespace sbmp
