// sbmp_abi.cpp — extern "C" boundary of libsbmp.so (declared in include/sbmp/sbmp.h).
// Every entry point converts exceptions into sbmp_status + a thread-local message.
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "kgmt_planner.h"
#include "obstacle_grid.h"
#include "sbmp/sbmp.h"

using sbmp::Error;
using sbmp::KgmtPlanner;
using sbmp::Planner;

struct sbmp_kgmt {
    Planner* planner = nullptr;
    sbmp::Exchange* comm = nullptr;   // sharded: owned collectives (kgmt_sharded.cpp)
};

namespace sbmp {
Exchange* sharded_create_comm(const uint8_t* id, int nranks, int rank, int device);
Exchange* sharded_create_host_comm(const sbmp_host_collectives& c, int nranks, int rank, int device);
void comm_get_unique_id(uint8_t* id);
void expand_batch(const sbmp_expand_batch_args* args, void* stream);   // batch.hip
void expand_batch_host(const sbmp_expand_batch_args* args);
void insert_batch(const sbmp_insert_batch_args* args, void* stream);
double hbm_copy_bandwidth(size_t bytes, int reps);
void load_system_config(const char* path, sbmp_system_config* out);   // config.cpp
}  // namespace sbmp

static thread_local std::string g_last_error;

template <typename F>
static sbmp_status guarded(F&& f) {
    try {
        f();
        return SBMP_OK;
    } catch (const Error& e) {
        g_last_error = e.what();
        return e.status;
    } catch (const std::bad_alloc&) {
        g_last_error = "host out of memory";
        return SBMP_ERR_OUT_OF_MEMORY;
    } catch (const std::exception& e) {
        g_last_error = e.what();
        return SBMP_ERR_STATE;
    }
}

#define REQUIRE(cond, msg)                                                   \
    do {                                                                     \
        if (!(cond)) throw Error(SBMP_ERR_INVALID_ARGUMENT, msg);            \
    } while (0)

extern "C" {

int sbmp_abi_version(void) { return SBMP_ABI_VERSION; }

const char* sbmp_status_string(sbmp_status s) {
    switch (s) {
        case SBMP_OK: return "ok";
        case SBMP_ERR_INVALID_ARGUMENT: return "invalid argument";
        case SBMP_ERR_HIP: return "HIP runtime error";
        case SBMP_ERR_IO: return "I/O error";
        case SBMP_ERR_OUT_OF_MEMORY: return "out of memory";
        case SBMP_ERR_STATE: return "invalid state";
        case SBMP_ERR_UNSUPPORTED: return "unsupported";
        case SBMP_ERR_COMM: return "communication error";
        default: return "unknown status";
    }
}

const char* sbmp_last_error(void) { return g_last_error.c_str(); }

sbmp_status sbmp_kgmt_default_params(sbmp_kgmt_params* p) {
    return guarded([&] {
        REQUIRE(p, "params is NULL");
        memset(p, 0, sizeof(*p));
        // reference demos/main.cu:19-28
        p->width = 20.0f;
        p->height = 20.0f;
        p->N = 16;
        p->n = 8;
        p->numIterations = 100;
        p->maxTreeSize = 30000;
        p->numDisc = 10;
        p->agentLength = 1.0f;
        p->goalThreshold = 0.5f;
        p->samplesPerIteration = 0;
        p->agent = SBMP_AGENT_CAR;
        p->fixGNewClear = 0;
        p->device = 0;
        p->profileKernels = 0;
    });
}

sbmp_status sbmp_load_system_config(const char* path, sbmp_system_config* out) {
    return guarded([&] { sbmp::load_system_config(path, out); });
}

sbmp_status sbmp_kgmt_create(const sbmp_kgmt_params* p, sbmp_kgmt** out) {
    return guarded([&] {
        REQUIRE(p && out, "NULL argument");
        *out = nullptr;
        sbmp_kgmt* h = new sbmp_kgmt;
        try {
            h->planner = new KgmtPlanner(*p);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

sbmp_status sbmp_kgmt_create_sharded(const sbmp_kgmt_params* p, const uint8_t id[SBMP_COMM_ID_BYTES], int nranks,
                                     int rank, sbmp_kgmt** out) {
    return guarded([&] {
        REQUIRE(p && id && out, "NULL argument");
        REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
        *out = nullptr;
        sbmp_kgmt* h = new sbmp_kgmt;
        try {
            h->comm = sbmp::sharded_create_comm(id, nranks, rank, p->device);
            h->planner = new KgmtPlanner(*p, nranks, rank, h->comm);
        } catch (...) {
            delete h->planner;
            delete h->comm;
            delete h;
            throw;
        }
        *out = h;
    });
}

sbmp_status sbmp_kgmt_create_sharded_host(const sbmp_kgmt_params* p, const sbmp_host_collectives* coll, int nranks,
                                          int rank, sbmp_kgmt** out) {
    return guarded([&] {
        REQUIRE(p && coll && out, "NULL argument");
        REQUIRE(coll->allreduce_u64 && coll->allreduce_i32 && coll->allgather, "NULL collective callback");
        REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
        *out = nullptr;
        sbmp_kgmt* h = new sbmp_kgmt;
        try {
            h->comm = sbmp::sharded_create_host_comm(*coll, nranks, rank, p->device);
            h->planner = new KgmtPlanner(*p, nranks, rank, h->comm);
        } catch (...) {
            delete h->planner;
            delete h->comm;
            delete h;
            throw;
        }
        *out = h;
    });
}

sbmp_status sbmp_kgmt_create_local_group(const sbmp_kgmt_params* p, int nranks, sbmp_kgmt** out) {
    return guarded([&] {
        REQUIRE(p && out, "NULL argument");
        *out = nullptr;
        sbmp_kgmt* h = new sbmp_kgmt;
        try {
            h->planner = (nranks == 1) ? static_cast<Planner*>(new KgmtPlanner(*p))
                                       : static_cast<Planner*>(new sbmp::LocalShardGroup(*p, nranks));
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

sbmp_status sbmp_expand_batch(const sbmp_expand_batch_args* args, void* stream) {
    return guarded([&] { sbmp::expand_batch(args, stream); });
}

sbmp_status sbmp_expand_batch_host(const sbmp_expand_batch_args* args) {
    return guarded([&] { sbmp::expand_batch_host(args); });
}

sbmp_status sbmp_insert_batch(const sbmp_insert_batch_args* args, void* stream) {
    return guarded([&] { sbmp::insert_batch(args, stream); });
}

sbmp_status sbmp_comm_get_unique_id(uint8_t id[SBMP_COMM_ID_BYTES]) {
    return guarded([&] {
        REQUIRE(id, "NULL id");
        sbmp::comm_get_unique_id(id);
    });
}

sbmp_status sbmp_kgmt_destroy(sbmp_kgmt* h) {
    return guarded([&] {
        if (!h) return;
        delete h->planner;
        delete h->comm;
        delete h;
    });
}

#define PLANNER(h)                                                     \
    REQUIRE((h) && (h)->planner, "NULL planner handle");               \
    Planner& P = *(h)->planner

sbmp_status sbmp_kgmt_begin(sbmp_kgmt* h, const float initial[7], const float goal[7], const float* d_obstacles,
                            int obstaclesCount, uint64_t seed) {
    return guarded([&] {
        PLANNER(h);
        P.begin(initial, goal, d_obstacles, obstaclesCount, seed);
    });
}

sbmp_status sbmp_kgmt_plan(sbmp_kgmt* h, const float initial[7], const float goal[7], const float* d_obstacles,
                           int obstaclesCount, uint64_t seed, sbmp_plan_result* result) {
    return guarded([&] {
        PLANNER(h);
        P.begin(initial, goal, d_obstacles, obstaclesCount, seed);
        // The planner's loop control (KgmtPlanner::run_plan): over-enqueued iterations of a
        // finished loop are no-ops, so they cost a few microseconds, not correctness.
        P.run_plan();
        if (result) P.result(result);
    });
}

sbmp_status sbmp_kgmt_step(sbmp_kgmt* h, int iterations, int* active) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(iterations >= 0, "iterations must be >= 0");
        P.enqueue(iterations);
        const bool a = P.active();
        if (active) *active = a ? 1 : 0;
    });
}

sbmp_status sbmp_kgmt_enqueue(sbmp_kgmt* h, int iterations) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(iterations >= 0, "iterations must be >= 0");
        P.enqueue(iterations);
    });
}

sbmp_status sbmp_kgmt_sync(sbmp_kgmt* h) {
    return guarded([&] {
        PLANNER(h);
        P.sync();
    });
}

sbmp_status sbmp_kgmt_set_iteration_dump(sbmp_kgmt* h, const char* dir) {
    return guarded([&] {
        PLANNER(h);
        P.set_iteration_dump(dir ? std::string(dir) : std::string());
    });
}

sbmp_status sbmp_kgmt_fold(sbmp_kgmt* h) {
    return guarded([&] {
        PLANNER(h);
        P.fold_pending();
    });
}

sbmp_status sbmp_kgmt_result(sbmp_kgmt* h, sbmp_plan_result* result) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(result, "NULL result");
        P.result(result);
    });
}

sbmp_status sbmp_kgmt_stream(sbmp_kgmt* h, void** stream) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(stream, "NULL stream");
        *stream = (void*)P.stream();
    });
}

sbmp_status sbmp_kgmt_copy_tree(sbmp_kgmt* h, float* samples, int* parent, float* costs, int capacity) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(capacity >= P.params().maxTreeSize, "capacity < maxTreeSize");
        P.copy_tree(samples, parent, costs);
    });
}

sbmp_status sbmp_kgmt_copy_unexplored(sbmp_kgmt* h, float* samples, int* uParent, int capacity) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(capacity >= P.params().maxTreeSize, "capacity < maxTreeSize");
        P.copy_unexplored(samples, uParent);
    });
}

sbmp_status sbmp_kgmt_copy_flags(sbmp_kgmt* h, uint8_t* G, uint8_t* GNew, int capacity) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(capacity >= P.params().maxTreeSize, "capacity < maxTreeSize");
        P.copy_flags(G, GNew);
    });
}

sbmp_status sbmp_kgmt_copy_regions(sbmp_kgmt* h, int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score,
                                   int* R2Avail, int* R2Valid, int* R2Invalid) {
    return guarded([&] {
        PLANNER(h);
        P.copy_regions(R1, R1Avail, R1Valid, R1Invalid, R1Score, R2Avail, R2Valid, R2Invalid);
    });
}

sbmp_status sbmp_kgmt_num_slots(sbmp_kgmt* h, int* slots) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(slots, "NULL slots");
        *slots = P.num_slots();
    });
}

sbmp_status sbmp_kgmt_copy_rng(sbmp_kgmt* h, uint32_t* states, int capacity) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(states && capacity >= P.num_slots(), "capacity < num_slots");
        P.copy_rng(states);
    });
}

sbmp_status sbmp_kgmt_iter_log(sbmp_kgmt* h, sbmp_iter_record* out, int capacity, int* count) {
    return guarded([&] {
        PLANNER(h);
        std::vector<sbmp_iter_record> log = P.iter_log();
        const int n = std::min<int>(capacity, (int)log.size());
        if (out && n > 0) memcpy(out, log.data(), sizeof(sbmp_iter_record) * n);
        if (count) *count = (int)log.size();
    });
}

sbmp_status sbmp_kgmt_export_csv(sbmp_kgmt* h, const char* dir) {
    return guarded([&] {
        PLANNER(h);
        P.export_csv(dir ? dir : "");
    });
}

sbmp_status sbmp_kgmt_solution_path(sbmp_kgmt* h, int node, int* rows, float* samples, float* costs, int capacity,
                                    int* length) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(length, "length must be non-NULL");
        const int len = P.solution_path(node, nullptr, nullptr, nullptr, 0);
        *length = len;
        if (!rows && !samples && !costs) return;
        REQUIRE(capacity >= len, "capacity smaller than the path length");
        P.solution_path(node, rows, samples, costs, capacity);
    });
}

sbmp_status sbmp_kgmt_kernel_stats(sbmp_kgmt* h, sbmp_kernel_stat* out, int capacity, int* count) {
    return guarded([&] {
        PLANNER(h);
        std::vector<sbmp_kernel_stat> st = P.kernel_stats();
        const int n = std::min<int>(capacity, (int)st.size());
        if (out && n > 0) memcpy(out, st.data(), sizeof(sbmp_kernel_stat) * n);
        if (count) *count = (int)st.size();
    });
}

sbmp_status sbmp_kgmt_path_info(sbmp_kgmt* h, sbmp_path_info* out) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(out, "out must be non-NULL");
        P.path_info(out);
    });
}

sbmp_status sbmp_kgmt_reset_kernel_stats(sbmp_kgmt* h) {
    return guarded([&] {
        PLANNER(h);
        P.reset_kernel_stats();
    });
}

sbmp_status sbmp_kgmt_enqueue_delay(sbmp_kgmt* h, double microseconds) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(microseconds >= 0.0 && microseconds <= 1e6, "delay must be in [0, 1 s]");
        P.enqueue_delay(microseconds);
    });
}

sbmp_status sbmp_kgmt_kernel_samples(sbmp_kgmt* h, const char* name, float* out, int capacity, int* count) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(name, "NULL name");
        std::vector<float> v = P.kernel_samples(name);
        const int n = std::min<int>(capacity, (int)v.size());
        if (out && n > 0) memcpy(out, v.data(), sizeof(float) * n);
        if (count) *count = (int)v.size();
    });
}

sbmp_status sbmp_kgmt_set_profiling(sbmp_kgmt* h, int enabled) {
    return guarded([&] {
        PLANNER(h);
        P.set_profiling(enabled != 0);
    });
}

sbmp_status sbmp_kgmt_state_hash(sbmp_kgmt* h, uint64_t* out) {
    return guarded([&] {
        PLANNER(h);
        REQUIRE(out, "out must be non-NULL");
        *out = (uint64_t)P.state_hash();
    });
}


// readObstaclesFromCSV (reference src/helper/helper.cu:11-34): values separated
// by whitespace or single commas, read line by line with operator>>.
sbmp_status sbmp_read_obstacles_csv(const char* path, int workspaceDim, float* out, int capacity,
                                    int* numObstacles) {
    return guarded([&] {
        REQUIRE(path && numObstacles && workspaceDim > 0, "bad argument");
        std::ifstream file(path);
        if (!file.is_open()) throw Error(SBMP_ERR_IO, std::string("Error opening file: ") + path);
        std::vector<float> v;
        std::string line;
        while (std::getline(file, line)) {
            std::stringstream ss(line);
            float value;
            while (ss >> value) {
                v.push_back(value);
                if (ss.peek() == ',') ss.ignore();
            }
        }
        const int n = (int)(v.size() / (2 * workspaceDim));
        *numObstacles = n;
        if (out) {
            REQUIRE(capacity >= (int)v.size(), "capacity smaller than the file's float count");
            memcpy(out, v.data(), sizeof(float) * v.size());
        }
    });
}

sbmp_status sbmp_random_tree(int device, int kind, const float* root, int rows, int blocks, int threadsPerBlock,
                             float* samples, long long capacity, float* kernelMs) {
    return guarded([&] {
        REQUIRE(root && samples, "root and samples must be non-NULL");
        REQUIRE(kind == SBMP_RANDOM_TREE_NAIVE || kind == SBMP_RANDOM_TREE_COSTPROP, "unknown generator kind");
        const bool naive = kind == SBMP_RANDOM_TREE_NAIVE;
        if (rows <= 0) rows = naive ? 10 : 1;                       // NaivePlanner.cu:80 / CostPropPlanner.cu:87
        if (blocks <= 0) blocks = naive ? 32 : 512;                 // :79 / :86
        if (threadsPerBlock <= 0) threadsPerBlock = naive ? 32 : 1024;   // :78 / :85
        REQUIRE(threadsPerBlock <= 1024, "threadsPerBlock must be <= 1024");
        const long long n = (long long)rows * blocks * threadsPerBlock * 7;
        REQUIRE(n < (1ll << 31), "tree larger than 2^31 floats (the reference indexes it with int)");
        REQUIRE(capacity >= n, "capacity smaller than rows * blocks * threadsPerBlock * 7");
        int ndev = 0;
        SBMP_HIP(hipGetDeviceCount(&ndev));
        REQUIRE(device >= 0 && device < ndev, "no such HIP device");
        sbmp::random_tree(device, kind, root, rows, blocks, threadsPerBlock, samples, kernelMs);
    });
}

sbmp_status sbmp_obstacle_grid_query(const float* obstacles, int nObs, float width, float height, int gridSize,
                                     const float* segments, int nSegments, uint8_t* freeOut, int* gridUsed) {
    return guarded([&] {
        REQUIRE(nObs >= 0 && nSegments >= 0 && (nObs == 0 || obstacles) && (nSegments == 0 || (segments && freeOut)),
                "bad argument");
        REQUIRE(width > 0.0f && height > 0.0f, "width and height must be positive");
        const sbmp::HostObstacleGrid g = sbmp::build_obstacle_grid(obstacles, nObs, width, height, gridSize);
        for (int i = 0; i < nSegments; ++i) {
            const float* q = segments + 4 * i;
            freeOut[i] = sbmp::grid_motion_valid(q[0], q[1], q[2], q[3], g.g, g.invW, g.invH, g.start.data(),
                                                 g.boxes.data())
                             ? 1
                             : 0;
        }
        if (gridUsed) *gridUsed = g.g;
    });
}

sbmp_status sbmp_device_upload_f32(const float* host, size_t count, float** d_out) {
    return guarded([&] {
        REQUIRE(d_out && (host || count == 0), "bad argument");
        void* p = nullptr;
        SBMP_HIP(hipMalloc(&p, std::max<size_t>(count, 1) * sizeof(float)));
        if (count) {
            hipError_t e = hipMemcpy(p, host, count * sizeof(float), hipMemcpyHostToDevice);
            if (e != hipSuccess) {
                hipFree(p);
                SBMP_HIP(e);
            }
        }
        *d_out = static_cast<float*>(p);
    });
}

sbmp_status sbmp_device_free(void* d_ptr) {
    return guarded([&] {
        if (d_ptr) SBMP_HIP(hipFree(d_ptr));
    });
}

sbmp_status sbmp_device_alloc(size_t bytes, void** d_out) {
    return guarded([&] {
        REQUIRE(d_out, "NULL output pointer");
        *d_out = nullptr;
        SBMP_HIP(hipMalloc(d_out, bytes > 0 ? bytes : 1));
    });
}

sbmp_status sbmp_device_copy_to(void* d_dst, const void* host, size_t bytes) {
    return guarded([&] {
        REQUIRE(bytes == 0 || (d_dst && host), "NULL pointer");
        if (bytes) SBMP_HIP(hipMemcpy(d_dst, host, bytes, hipMemcpyHostToDevice));
    });
}

sbmp_status sbmp_device_copy_from(void* host, const void* d_src, size_t bytes) {
    return guarded([&] {
        REQUIRE(bytes == 0 || (d_src && host), "NULL pointer");
        if (bytes) SBMP_HIP(hipMemcpy(host, d_src, bytes, hipMemcpyDeviceToHost));
    });
}

sbmp_status sbmp_device_count(int* count) {
    return guarded([&] {
        REQUIRE(count, "NULL count");
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        *count = (e == hipSuccess) ? n : 0;
    });
}

sbmp_status sbmp_hbm_copy_bandwidth(size_t bytes, int reps, double* gbs) {
    return guarded([&] {
        REQUIRE(gbs, "NULL output");
        *gbs = 0.0;
        *gbs = sbmp::hbm_copy_bandwidth(bytes, reps);
    });
}

}  // extern "C"
