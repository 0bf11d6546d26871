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

// Collective layer for the sharded planner (RCCL over xGMI, or an in-process
// stand-in used by tests); see kgmt_sharded.cpp.
class Exchange;

class KgmtPlanner {
public:
    KgmtPlanner(const sbmp_kgmt_params& p, int nranks = 1, int rank = 0, Exchange* ex = nullptr);
    ~KgmtPlanner();
    KgmtPlanner(const KgmtPlanner&) = delete;
    KgmtPlanner& operator=(const KgmtPlanner&) = delete;

    void begin(const float* initial, const float* goal, const float* d_obstacles, int nObs, uint64_t seed);
    void enqueue(int iterations);
    void sync();
    bool active();                    // syncs; false once the loop has ended
    void result(sbmp_plan_result* r);
    void run(int pollEvery);          // enqueue until the loop ends

    hipStream_t stream() const { return stream_; }
    int num_slots() const { return d_.nSlots; }
    const sbmp_kgmt_params& params() const { return p_; }

    // exports (reference layouts)
    void copy_tree(float* samples, int* parent, float* costs);
    void copy_unexplored(float* samples, int* uParent);
    void copy_flags(uint8_t* G, uint8_t* GNew);
    void copy_regions(int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score, int* R2Avail,
                      int* R2Valid, int* R2Invalid);
    void copy_rng(uint32_t* states);
    std::vector<sbmp_iter_record> iter_log();
    void export_csv(const std::string& dir);

    std::vector<sbmp_kernel_stat> kernel_stats();
    void reset_kernel_stats();
    void set_profiling(bool on) { p_.profileKernels = on ? 1 : 0; }
    void enqueue_delay(double us) { launch_delay(us, stream_); }
    std::vector<float> kernel_samples(const std::string& name);

    // sharded pieces (kgmt_sharded.cpp)
    void enqueue_sharded_iteration(int t);

private:
    enum KernelId { K_EXPAND = 0, K_FINISH, K_FOLD, K_PACK, K_MERGE, K_COUNT };
    KernelTiming timing(int id);
    void collect_events();
    void read_ctrl(std::vector<IterCtrl>& c, PlannerStatus& st);
    int last_executed(const std::vector<IterCtrl>& c) const;
    template <typename T>
    T* alloc(size_t n);

    sbmp_kgmt_params p_;
    KgmtDev d_{};
    hipStream_t stream_ = nullptr;
    Exchange* ex_ = nullptr;
    int t_next_ = 1;
    bool begun_ = false;
    int slotsPadded_ = 0, expandBlocks_ = 0, nbits_ = 1;
    int expandVariant_ = 0;   // SBMP_EXPAND_VARIANT: obstacle form, 0 = auto (3 if <= kMaxRegObs boxes, else 1)
    bool timelineDumped_ = false;
    int lastFolded_ = 0;      // iterations <= lastFolded_ are in R2Valid / R2Invalid
    void fold_to(int tLast);
    uint32_t* jumps_ = nullptr;
    float4* obs_ = nullptr;
    int obsCap_ = 0;
    std::vector<void*> allocs_;
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

    friend class ShardedDriver;
};

double now_ms();

}  // namespace sbmp
