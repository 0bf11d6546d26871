// kgmt_sharded.cpp — one planning problem sharded over ranks.
//
// Slots are owned block-cyclically (256-slot block b -> rank b mod P); every rank
// keeps a full replica of the tree, frontier and region tables.  Per iteration a
// rank expands its own slots (k_expand), packs its accepted children in slot order
// (k_pack), and all ranks all-reduce one fused exchange buffer (R1 deltas, block
// counts, GNew words, R2New bytes; every field disjoint per rank or a carry-free
// counter, so a sum merges them).  Then every rank inserts every block (k_finish),
// reading other ranks' accepted children from their record buffers over xGMI.
// The all-reduce is also the fence: rank q's record buffer of parity t & 1 is
// rewritten only in iteration t + 2, after the all-reduce of t + 1, which waits
// for every rank's inserts of t.
//
// RcclExchange: RCCL over xGMI, one process per GPU, record buffers mapped with
// HIP IPC.  LocalShardGroup: P ranks on one GPU and one stream (a sum kernel for
// the all-reduce, direct pointers for the records), so the sharded data flow can be
// parity-tested against the single-rank planner on a one-GPU machine.
#include <rccl/rccl.h>

#include <cstring>

#include "kgmt_planner.h"

namespace sbmp {

#define SBMP_NCCL(expr)                                                                                  \
    do {                                                                                                 \
        ncclResult_t r_ = (expr);                                                                        \
        if (r_ != ncclSuccess)                                                                           \
            throw ::sbmp::Error(SBMP_ERR_COMM, std::string(#expr) + ": " + ncclGetErrorString(r_));     \
    } while (0)

static_assert(sizeof(ncclUniqueId) == SBMP_COMM_ID_BYTES, "RCCL unique id size");

class RcclExchange : public Exchange {
public:
    RcclExchange(const uint8_t* id, int nranks, int rank, int device) : nranks_(nranks), rank_(rank) {
        SBMP_HIP(hipSetDevice(device));
        ncclUniqueId uid;
        memcpy(&uid, id, sizeof(uid));
        SBMP_NCCL(ncclCommInitRank(&comm_, nranks, uid, rank));
        SBMP_HIP(hipStreamCreateWithFlags(&setup_, hipStreamNonBlocking));
        SBMP_HIP(hipMalloc(&token_, sizeof(int)));
    }
    ~RcclExchange() override {
        if (token_) (void)hipFree(token_);
        for (void* p : mapped_) (void)hipIpcCloseMemHandle(p);
        if (setup_) (void)hipStreamDestroy(setup_);
        if (comm_) (void)ncclCommDestroy(comm_);
    }
    int comm_ranks() const override {
        int n = 0;
        return (comm_ && ncclCommCount(comm_, &n) == ncclSuccess) ? n : 0;
    }

    void allreduce_u64(const unsigned long long* send, unsigned long long* recv, size_t n, hipStream_t s) override {
        SBMP_NCCL(ncclAllReduce(send, recv, n, ncclUint64, ncclSum, comm_, s));
    }
    void allreduce_i32(const int* send, int* recv, size_t n, hipStream_t s) override {
        SBMP_NCCL(ncclAllReduce(send, recv, n, ncclInt32, ncclSum, comm_, s));
    }
    void barrier(hipStream_t s) override {   // a one-word all-reduce, waited for on the host
        SBMP_HIP(hipStreamSynchronize(s));
        SBMP_NCCL(ncclAllReduce(token_, token_, 1, ncclInt32, ncclSum, comm_, setup_));
        SBMP_HIP(hipStreamSynchronize(setup_));
    }
    void share_buffer(void* own, size_t bytes, void* peers[kMaxRanks]) override {
        (void)bytes;
        hipIpcMemHandle_t h;
        SBMP_HIP(hipIpcGetMemHandle(&h, own));
        uint8_t* dev = nullptr;
        SBMP_HIP(hipMalloc(&dev, sizeof(h) * (nranks_ + 1)));
        SBMP_HIP(hipMemcpy(dev, &h, sizeof(h), hipMemcpyHostToDevice));
        SBMP_NCCL(ncclAllGather(dev, dev + sizeof(h), sizeof(h), ncclUint8, comm_, setup_));
        std::vector<hipIpcMemHandle_t> all(nranks_);
        SBMP_HIP(hipStreamSynchronize(setup_));
        SBMP_HIP(hipMemcpy(all.data(), dev + sizeof(h), sizeof(h) * nranks_, hipMemcpyDeviceToHost));
        (void)hipFree(dev);
        for (int q = 0; q < nranks_; ++q) {
            if (q == rank_) {
                peers[q] = own;
                continue;
            }
            void* p = nullptr;
            SBMP_HIP(hipIpcOpenMemHandle(&p, all[q], hipIpcMemLazyEnablePeerAccess));
            mapped_.push_back(p);
            peers[q] = p;
        }
    }

private:
    int nranks_, rank_;
    ncclComm_t comm_ = nullptr;
    hipStream_t setup_ = nullptr;
    int* token_ = nullptr;
    std::vector<void*> mapped_;
};

// HostExchange: the same protocol with the collectives done by host callbacks
// (sbmp_host_collectives): the stream is synchronised, the buffer copied to pinned
// host memory, reduced by the callback, copied back.  The synchronisation makes it
// the fence RcclExchange's stream order is (every rank's k_pack records are written
// before any rank returns from the all-reduce).  Record buffers are mapped with HIP
// IPC as with RCCL, the handles exchanged by the allgather callback.
class HostExchange : public Exchange {
public:
    HostExchange(const sbmp_host_collectives& c, int nranks, int rank, int device)
        : c_(c), nranks_(nranks), rank_(rank), device_(device) {}
    ~HostExchange() override {
        for (void* p : mapped_) (void)hipIpcCloseMemHandle(p);
        if (host_) (void)hipHostFree(host_);
    }

    void allreduce_u64(const unsigned long long* send, unsigned long long* recv, size_t n, hipStream_t s) override {
        reduce(send, recv, n * sizeof(uint64_t), s, [&](void* hs, void* hr) {
            return c_.allreduce_u64(c_.ctx, static_cast<const uint64_t*>(hs), static_cast<uint64_t*>(hr), n);
        });
    }
    void allreduce_i32(const int* send, int* recv, size_t n, hipStream_t s) override {
        reduce(send, recv, n * sizeof(int32_t), s, [&](void* hs, void* hr) {
            return c_.allreduce_i32(c_.ctx, static_cast<const int32_t*>(hs), static_cast<int32_t*>(hr), n);
        });
    }
    void barrier(hipStream_t s) override {   // a one-int all-reduce through the callbacks
        SBMP_HIP(hipSetDevice(device_));
        SBMP_HIP(hipStreamSynchronize(s));
        const int32_t one = 1;
        int32_t sum = 0;
        if (c_.allreduce_i32(c_.ctx, &one, &sum, 1) != 0 || sum != nranks_)
            throw Error(SBMP_ERR_COMM, "host barrier (all-reduce callback) failed");
    }
    void share_buffer(void* own, size_t bytes, void* peers[kMaxRanks]) override {
        (void)bytes;
        hipIpcMemHandle_t h;
        SBMP_HIP(hipIpcGetMemHandle(&h, own));
        std::vector<hipIpcMemHandle_t> all(nranks_);
        if (c_.allgather(c_.ctx, &h, sizeof(h), all.data()) != 0)
            throw Error(SBMP_ERR_COMM, "host allgather of the record-buffer handles failed");
        for (int q = 0; q < nranks_; ++q) {
            if (q == rank_) {
                peers[q] = own;
                continue;
            }
            void* p = nullptr;
            SBMP_HIP(hipIpcOpenMemHandle(&p, all[q], hipIpcMemLazyEnablePeerAccess));
            mapped_.push_back(p);
            peers[q] = p;
        }
    }

private:
    template <typename F>
    void reduce(const void* send, void* recv, size_t bytes, hipStream_t s, F&& call) {
        SBMP_HIP(hipSetDevice(device_));
        if (2 * bytes > hostBytes_) {
            void* old = host_;
            host_ = nullptr;   // cleared first: a throw below leaves nothing to free twice
            hostBytes_ = 0;
            if (old) (void)hipHostFree(old);
            SBMP_HIP(hipHostMalloc(&host_, 2 * bytes));
            hostBytes_ = 2 * bytes;
        }
        char* hs = static_cast<char*>(host_);
        char* hr = hs + bytes;
        SBMP_HIP(hipMemcpyAsync(hs, send, bytes, hipMemcpyDeviceToHost, s));
        SBMP_HIP(hipStreamSynchronize(s));
        if (call(hs, hr) != 0) throw Error(SBMP_ERR_COMM, "host all-reduce callback failed");
        SBMP_HIP(hipMemcpyAsync(recv, hr, bytes, hipMemcpyHostToDevice, s));
        SBMP_HIP(hipStreamSynchronize(s));
    }

    sbmp_host_collectives c_;
    int nranks_, rank_, device_;
    void* host_ = nullptr;
    size_t hostBytes_ = 0;
    std::vector<void*> mapped_;
};

Exchange* sharded_create_comm(const uint8_t* id, int nranks, int rank, int device) {
    return new RcclExchange(id, nranks, rank, device);
}
Exchange* sharded_create_host_comm(const sbmp_host_collectives& c, int nranks, int rank, int device) {
    return new HostExchange(c, nranks, rank, device);
}

void comm_get_unique_id(uint8_t* id) {
    ncclUniqueId uid;
    SBMP_NCCL(ncclGetUniqueId(&uid));
    memcpy(id, &uid, sizeof(uid));
}

// ---------------------------------------------------------------- local group
LocalShardGroup::LocalShardGroup(const sbmp_kgmt_params& p, int nranks) {
    if (nranks < 2 || nranks > kMaxRanks) throw Error(SBMP_ERR_INVALID_ARGUMENT, "local group needs 2..8 ranks");
    SBMP_HIP(hipSetDevice(p.device));
    SBMP_HIP(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    try {
        for (int r = 0; r < nranks; ++r) ranks_.push_back(new KgmtPlanner(p, nranks, r, nullptr, stream_));
    } catch (...) {
        for (KgmtPlanner* k : ranks_) delete k;
        (void)hipStreamDestroy(stream_);
        throw;
    }
    for (KgmtPlanner* k : ranks_)
        for (KgmtPlanner* q : ranks_) k->set_peer_records(q->rank(), q->record_buffer());
}

LocalShardGroup::~LocalShardGroup() {
    for (KgmtPlanner* k : ranks_) delete k;
    if (stream_) (void)hipStreamDestroy(stream_);
}

void LocalShardGroup::begin(const float* initial, const float* goal, const float* d_obstacles, int nObs,
                            uint64_t seed) {
    for (KgmtPlanner* k : ranks_) k->begin(initial, goal, d_obstacles, nObs, seed);
}

void LocalShardGroup::enqueue(int iterations) {
    const int P = (int)ranks_.size();
    const unsigned long long* send[kMaxRanks];
    unsigned long long* recv[kMaxRanks];
    for (int q = 0; q < P; ++q) {
        send[q] = ranks_[q]->exchange_send();
        recv[q] = ranks_[q]->exchange_recv();
    }
    for (int i = 0; i < iterations; ++i) {
        int t = 0;
        for (KgmtPlanner* k : ranks_) t = k->take_iteration();   // all ranks advance together
        if (t == 0) break;
        if (r0().step_mode()) {   // one k_step per rank, then the exchange of t
            for (KgmtPlanner* k : ranks_) k->stage_step(t);
            for (int q = 0; q < P; ++q) send[q] = ranks_[q]->exchange_send(t);
            launch_xsum(send, recv, P, (long long)ranks_[0]->exchange_words(), stream_);
            for (KgmtPlanner* k : ranks_) k->stage_fold(t);
            continue;
        }
        for (KgmtPlanner* k : ranks_) k->stage_expand(t);
        for (KgmtPlanner* k : ranks_) k->stage_pack(t);
        launch_xsum(send, recv, P, (long long)ranks_[0]->exchange_words(), stream_);
        for (KgmtPlanner* k : ranks_) k->stage_finish(t);
        for (KgmtPlanner* k : ranks_) k->stage_fold(t);
    }
    SBMP_HIP(hipGetLastError());
}

// Slot rows live on their owning rank.
void LocalShardGroup::copy_unexplored(float* samples, int* uParent) {
    const int M = params().maxTreeSize, n = num_slots(), P = (int)ranks_.size();
    std::vector<float> s((size_t)M * 7);
    std::vector<int> u(M);
    for (int q = 0; q < P; ++q) {
        ranks_[q]->copy_unexplored(s.data(), u.data());
        for (int i = 0; i < n; ++i) {
            if ((i / kBlock) % P != q) continue;
            if (samples) memcpy(samples + (size_t)i * 7, &s[(size_t)i * 7], sizeof(float) * 7);
            if (uParent) uParent[i] = u[i];
        }
    }
    for (int i = n; i < M; ++i) {
        if (samples) memset(samples + (size_t)i * 7, 0, sizeof(float) * 7);
        if (uParent) uParent[i] = -1;
    }
}

unsigned long long LocalShardGroup::state_hash() {
    sync();
    const unsigned long long h = ranks_[0]->state_hash();
    for (size_t q = 1; q < ranks_.size(); ++q)
        if (ranks_[q]->state_hash() != h)
            throw Error(SBMP_ERR_STATE, "local shard group: rank " + std::to_string(q) + "'s replicated state differs");
    return h;
}

void LocalShardGroup::copy_rng(uint32_t* states) {
    const int n = num_slots(), P = (int)ranks_.size();
    std::vector<uint32_t> st((size_t)n * 6);
    for (int q = 0; q < P; ++q) {
        ranks_[q]->copy_rng(st.data());
        for (int i = 0; i < n; ++i)
            if ((i / kBlock) % P == q) memcpy(states + (size_t)i * 6, &st[(size_t)i * 6], sizeof(uint32_t) * 6);
    }
}

void LocalShardGroup::copy_flags(uint8_t* G, uint8_t* GNew) {
    r0().copy_flags(G, GNew);
    if (!GNew) return;
    std::vector<uint8_t> f(params().maxTreeSize);
    for (size_t q = 1; q < ranks_.size(); ++q) {   // non-owned words are zero on every rank
        ranks_[q]->copy_flags(nullptr, f.data());
        for (size_t i = 0; i < f.size(); ++i) GNew[i] |= f[i];
    }
}

// R2Valid / R2Invalid: each rank folded the children of its own slots.
void LocalShardGroup::copy_regions(int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score, int* R2Avail,
                                   int* R2Valid, int* R2Invalid) {
    r0().copy_regions(R1, R1Avail, R1Valid, R1Invalid, R1Score, R2Avail, nullptr, nullptr);
    if (!R2Valid && !R2Invalid) return;
    const size_t n2 = (size_t)params().N * params().N * params().n * params().n;
    std::vector<int> v(n2), iv(n2), sv(n2, 0), si(n2, 0);
    for (KgmtPlanner* k : ranks_) {
        k->copy_r2_partial(v.data(), iv.data());
        for (size_t i = 0; i < n2; ++i) {
            sv[i] += v[i];
            si[i] += iv[i];
        }
    }
    if (R2Valid) memcpy(R2Valid, sv.data(), sizeof(int) * n2);
    if (R2Invalid) memcpy(R2Invalid, si.data(), sizeof(int) * n2);
}

void LocalShardGroup::reset_kernel_stats() {
    for (KgmtPlanner* k : ranks_) k->reset_kernel_stats();
}

void LocalShardGroup::set_profiling(bool on) {
    for (KgmtPlanner* k : ranks_) k->set_profiling(on);
}

}  // namespace sbmp
