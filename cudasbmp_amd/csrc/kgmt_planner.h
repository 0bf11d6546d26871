// kgmt_planner.h — host side of the MI355X KGMT planner (behind the C ABI).
#pragma once

#include <hip/hip_runtime.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "kgmt_device.h"
#include "kgmt_launch.h"
#include "sbmp/sbmp.h"

namespace sbmp {

struct Error : std::runtime_error {
    sbmp_status status;
    Error(sbmp_status s, const std::string& m) : std::runtime_error(m), status(s) {}
};

#define SBMP_HIP(expr)                                                                                   \
    do {                                                                                                 \
        hipError_t e_ = (expr);                                                                          \
        if (e_ != hipSuccess)                                                                            \
            throw ::sbmp::Error(SBMP_ERR_HIP, std::string(#expr) + ": " + hipGetErrorString(e_));      \
    } while (0)

// Collectives of one rank of a sharded planning problem (kgmt_sharded.cpp: RCCL
// over xGMI, one process per GPU).
class Exchange {
public:
    virtual ~Exchange() = default;
    // recv[i] = sum over ranks of send[i] (stream-ordered, also the per-iteration fence).
    virtual void allreduce_u64(const unsigned long long* send, unsigned long long* recv, size_t n, hipStream_t s) = 0;
    virtual void allreduce_i32(const int* send, int* recv, size_t n, hipStream_t s) = 0;
    // Every rank's device buffer of the same size, mapped into this process (IPC).
    virtual void share_buffer(void* own, size_t bytes, void* peers[kMaxRanks]) = 0;
    // Returns once every rank has called it (host-side; `s` is drained first).  The
    // one-shot exchange waits for its peers in-kernel with a time bound, so ranks are
    // lined up here before their first exchange and after host-side pauses (dumps).
    virtual void barrier(hipStream_t s) = 0;
    virtual int comm_ranks() const { return 0; }   // ranks of the RCCL communicator, 0 if none
};

// What the C ABI drives: one rank (single GPU or one rank of an RCCL group) or a
// local shard group (several ranks on one GPU, used to test the sharded data flow).
class Planner {
public:
    virtual ~Planner() = default;
    virtual void begin(const float* initial, const float* goal, const float* d_obstacles, int nObs, uint64_t seed) = 0;
    virtual void enqueue(int iterations) = 0;
    virtual void sync() = 0;
    virtual void fold_pending() = 0;   // enqueue k_fold_r2 up to the last enqueued iteration
    virtual bool active() = 0;   // syncs; false once the loop has ended
    virtual void rank_barrier() {}   // sharded ranks: all ranks reach this point (Exchange::barrier)
    virtual void result(sbmp_plan_result* r) = 0;
    void run(int pollEvery);     // enqueue until the loop ends
    // plan(): run() with the planner's own loop control (a single k_step rank: the host
    // watches a pinned word instead of polling with stream synchronisations)
    virtual void run_plan() { run(8); }
    // Per-iteration dumps (reference KGMT.cu:263-290, commented out there; read by
    // visualization/visualizationKGMT_Steps.m): with a directory set, run() steps one
    // iteration at a time and writes <dir>/Data/<Kind>/<kind><itr>.csv after each.
    void set_iteration_dump(const std::string& dir) { dumpDir_ = dir; }
    void dump_iteration(const std::string& dir, int itr);

    virtual hipStream_t stream() const = 0;
    virtual int num_slots() const = 0;
    virtual const sbmp_kgmt_params& params() const = 0;

    // exports (reference layouts)
    virtual void copy_tree(float* samples, int* parent, float* costs) = 0;
    virtual void copy_unexplored(float* samples, int* uParent) = 0;
    virtual void copy_flags(uint8_t* G, uint8_t* GNew) = 0;
    virtual void copy_regions(int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score, int* R2Avail,
                              int* R2Valid, int* R2Invalid) = 0;
    virtual void copy_rng(uint32_t* states) = 0;
    virtual std::vector<sbmp_iter_record> iter_log() = 0;
    // Rows root .. node (node < 0: the solution node); returns the length (0: no
    // solution).  Outputs may be null; capacity in rows (too small: SBMP_ERR_INVALID_ARGUMENT).
    virtual int solution_path(int node, int* rows, float* samples, float* costs, int capacity) = 0;
    // Digest of the replicated state (tree rows, region tables, control blocks): the same on
    // every rank of a sharded run (k_state_hash).
    virtual unsigned long long state_hash() = 0;
    void export_csv(const std::string& dir);

    virtual std::vector<sbmp_kernel_stat> kernel_stats() = 0;
    virtual void path_info(sbmp_path_info* out) = 0;
    virtual void reset_kernel_stats() = 0;
    virtual void set_profiling(bool on) = 0;
    virtual void enqueue_delay(double us) = 0;
    virtual std::vector<float> kernel_samples(const std::string& name) = 0;

protected:
    std::string dumpDir_;
};

// Legacy random-tree generators (random_tree.hip): rows x (blocks * tpb) samples
// of 7 floats into host memory.
void random_tree(int device, int kind, const float* root, int rows, int blocks, int tpb, float* samples,
                 float* kernelMs);

class KgmtPlanner : public Planner {
public:
    // nranks > 1: rank `rank` of a sharded problem.  ex = its RCCL collectives, or
    // nullptr inside a LocalShardGroup (which then drives the stages itself);
    // shared = a stream owned by the caller (the group), else the planner makes one.
    KgmtPlanner(const sbmp_kgmt_params& p, int nranks = 1, int rank = 0, Exchange* ex = nullptr,
                hipStream_t shared = nullptr);
    ~KgmtPlanner() override;
    KgmtPlanner(const KgmtPlanner&) = delete;
    KgmtPlanner& operator=(const KgmtPlanner&) = delete;

    void begin(const float* initial, const float* goal, const float* d_obstacles, int nObs, uint64_t seed) override;
    void enqueue(int iterations) override;
    void sync() override;
    void fold_pending() override {
        if (begun_) fold_to(t_next_ - 1);
    }
    bool active() override;
    void rank_barrier() override {
        if (ex_) ex_->barrier(stream_);
    }
    void result(sbmp_plan_result* r) override;
    void run_plan() override;

    hipStream_t stream() const override { return stream_; }
    int num_slots() const override { return d_.nSlots; }
    const sbmp_kgmt_params& params() const override { return p_; }

    void copy_tree(float* samples, int* parent, float* costs) override;
    void copy_unexplored(float* samples, int* uParent) override;
    void copy_flags(uint8_t* G, uint8_t* GNew) override;
    void copy_regions(int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score, int* R2Avail,
                      int* R2Valid, int* R2Invalid) override;
    void copy_rng(uint32_t* states) override;
    std::vector<sbmp_iter_record> iter_log() override;
    int solution_path(int node, int* rows, float* samples, float* costs, int capacity) override;
    unsigned long long state_hash() override;

    std::vector<sbmp_kernel_stat> kernel_stats() override;
    void path_info(sbmp_path_info* out) override;
    void reset_kernel_stats() override;
    void set_profiling(bool on) override { p_.profileKernels = on ? 1 : 0; }
    void enqueue_delay(double us) override { launch_delay(us, stream_); }
    std::vector<float> kernel_samples(const std::string& name) override;

    // ---- stages of one iteration (enqueue() composes them; a LocalShardGroup
    // interleaves them across its ranks)
    int take_iteration();                 // next iteration number, 0 past numIterations
    void stage_expand(int t);
    void stage_pack(int t);               // sharded ranks only
    void stage_exchange(int t);           // sharded ranks with an Exchange: the all-reduce of t
    void stage_finish(int t);
    void stage_fold(int t);               // every kFoldEvery iterations
    void stage_step(int t);               // k_step mode: the iteration's one launch
    void flush();                         // k_step mode: insert the last iteration, plan the next
    bool step_mode() const { return d_.stepMode != 0; }
    // what iteration t sends (sharded k_step alternates two buffers by parity)
    unsigned long long* exchange_send(int t = 0) const { return (t & 1) ? xSendOdd_ : xSend_; }
    unsigned long long* exchange_recv() const { return xRecv_; }
    size_t exchange_words() const { return xWords_; }
    float4* record_buffer() const { return d_.recOut; }
    void set_peer_records(int q, const float4* p) { d_.recPeer[q] = p; }
    void copy_r2_partial(int* R2Valid, int* R2Invalid);   // this rank's folded R2 counters
    int rank() const { return d_.rank; }

private:
    enum KernelId { K_EXPAND = 0, K_FINISH, K_FOLD, K_PACK, K_STEP, K_XCHG, K_COUNT };
    KernelTiming timing(int id);
    void collect_events();
    void read_ctrl(std::vector<IterCtrl>& c, PlannerStatus& st);
    int last_executed(const std::vector<IterCtrl>& c) const;
    void fold_to(int tLast);
    template <typename T>
    T* alloc(size_t n);

    sbmp_kgmt_params p_;
    KgmtDev d_{};
    KgmtDev* dDev_ = nullptr;      // the copy k_step reads (d_.devSelf)
    KgmtDev* dStage_ = nullptr;    // pinned: what was last copied there
    bool uploaded_ = false;
    void upload_dev();
    hipStream_t stream_ = nullptr;
    bool ownStream_ = true;
    Exchange* ex_ = nullptr;
    int t_next_ = 1;
    bool begun_ = false;
    int slotsPadded_ = 0, expandBlocks_ = 0, nbits_ = 1;
    int expandVariant_ = 0;   // SBMP_EXPAND_VARIANT: obstacle form, 0 = auto (3 if <= kMaxRegObs boxes, else 1)
    bool timelineDumped_ = false;
    // Pinned host copy of (ctrl[t_next], status) for active(): both land with one
    // stream synchronisation instead of two blocking copies per poll.
    struct PollBuf {
        IterCtrl ctrl;
        PlannerStatus status;
        unsigned long long word;   // KgmtDev::hostPoll (single rank)
    };
    PollBuf* poll_ = nullptr;
    void run_to_goal();                   // run_plan() for a single k_step rank
    bool wallFixed_ = false;              // wallMs_ was taken at the goal iteration's end
    bool flushed_ = true;     // k_step mode: the last enqueued iteration has been inserted
    int lastFolded_ = 0;      // iterations <= lastFolded_ are in R2Valid / R2Invalid
    unsigned long long* local_ = nullptr;   // sharded: the owner's block counts + GNew words
    size_t localWords_ = 0;
    unsigned long long* xSend_ = nullptr;
    unsigned long long* xSendOdd_ = nullptr;   // sharded k_step: the send buffer of odd iterations
    bool shStep_ = false;                      // sharded rank in k_step mode
    bool stepCapable_ = false;                 // k_step buffers exist; begin() decides per plan (d_.stepMode)
    int residentGroups_ = 0, neededGroups_ = 0;   // k_step residency at the last begin()
    bool formLogged_ = false;
    void choose_form(const float* d_obstacles, int nObs);
    void build_grid(const float* d_obstacles, int nObs);
    unsigned long long* xRecv_ = nullptr;
    size_t xWords_ = 0;
    bool oneshot_ = false;                   // sharded: the exchange is k_oneshot over IPC-mapped inboxes
    bool oneshot_self_test();                // k_oneshot checked once at construction (all ranks agree)
    bool mirror_self_test();                 // the list mirror checked once at construction (all ranks agree)
    bool fused_self_test();                  // the fused exchange's in-kernel order, likewise
    int oneshotCheck_ = 0, mirrorCheck_ = 0, fusedCheck_ = 0;   // start-up checks: 0 not run, 1 passed, -1 failed (fell back)
    unsigned long long* inbox_[kMaxRanks] = {nullptr};
    bool compactX_ = true;   // sharded k_step: k_oneshot sends the compact form of the exchange
    unsigned long long xSeq_ = 0;            // exchanges so far (the same count on every rank)
    uint32_t* jumps_ = nullptr;
    float4* obs_ = nullptr;
    int obsCap_ = 0;
    int* gridStart_ = nullptr;       // obstacle grid index (kObsGrid)
    size_t gridStartCap_ = 0;
    float4* gridBoxes_ = nullptr;
    size_t gridBoxesCap_ = 0;
    std::vector<void*> allocs_;
    unsigned long long* scratch_ = nullptr;   // 8 device words for small results (state_hash)
    unsigned long long* alloc_scratch_u64();
    double wallMs_ = 0.0;
    double t0_ = 0.0;

    struct Pending {
        int id;
        hipEvent_t a, b;
    };
    std::vector<Pending> pending_;
    std::vector<hipEvent_t> eventPool_;
    long long launches_[K_COUNT] = {0};
    double totalMs_[K_COUNT] = {0};
    std::vector<float> samples_[K_COUNT];
};

// Several ranks of one sharded problem on ONE device and one stream, exchanging
// through a sum kernel instead of RCCL and reading each other's record buffers
// directly.  Same data flow as the RCCL ranks, so the GPU parity tests can prove
// the sharded planner equal to the single-rank one on a one-GPU machine.
class LocalShardGroup : public Planner {
public:
    LocalShardGroup(const sbmp_kgmt_params& p, int nranks);
    ~LocalShardGroup() override;

    void begin(const float* initial, const float* goal, const float* d_obstacles, int nObs, uint64_t seed) override;
    void enqueue(int iterations) override;
    void sync() override {
        for (KgmtPlanner* k : ranks_) k->flush();   // every rank's flush pass (GNew words live with their owner)
        r0().sync();
    }
    void fold_pending() override {
        for (KgmtPlanner* k : ranks_) k->fold_pending();
    }
    bool active() override {
        for (KgmtPlanner* k : ranks_) k->flush();
        return r0().active();
    }
    void result(sbmp_plan_result* r) override { r0().result(r); }

    hipStream_t stream() const override { return stream_; }
    int num_slots() const override { return ranks_[0]->num_slots(); }
    const sbmp_kgmt_params& params() const override { return ranks_[0]->params(); }

    void copy_tree(float* samples, int* parent, float* costs) override { r0().copy_tree(samples, parent, costs); }
    void copy_unexplored(float* samples, int* uParent) override;
    void copy_flags(uint8_t* G, uint8_t* GNew) override;   // GNew words live with their owner
    void copy_regions(int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score, int* R2Avail,
                      int* R2Valid, int* R2Invalid) override;
    void copy_rng(uint32_t* states) override;
    std::vector<sbmp_iter_record> iter_log() override { return r0().iter_log(); }
    int solution_path(int node, int* rows, float* samples, float* costs, int capacity) override {
        return r0().solution_path(node, rows, samples, costs, capacity);   // every rank holds the whole tree
    }
    unsigned long long state_hash() override;   // every rank's digest; throws if they differ

    std::vector<sbmp_kernel_stat> kernel_stats() override { return r0().kernel_stats(); }
    void path_info(sbmp_path_info* out) override { r0().path_info(out); }
    void reset_kernel_stats() override;
    void set_profiling(bool on) override;
    void enqueue_delay(double us) override { r0().enqueue_delay(us); }
    std::vector<float> kernel_samples(const std::string& name) override { return r0().kernel_samples(name); }

private:
    KgmtPlanner& r0() { return *ranks_[0]; }
    hipStream_t stream_ = nullptr;
    std::vector<KgmtPlanner*> ranks_;
};

double now_ms();

}  // namespace sbmp
