/* sbmp.h — C ABI of the MI355X-native KGMT planner (libsbmp.so).
 *
 * The reference (nipe1783/cudaSBMP) exposes one planner, the C++ class KGMT
 * (reference include/planners/KGMT.cuh:23-109), driven by demos/main.cu.  This
 * ABI is the thin, plain-pointer boundary that replaces it; the C++ facade in
 * include/planners/KGMT.h rebuilds the reference's class on top of it, so
 * demos/main.cpp stays a drop-in for demos/main.cu.
 *
 * Conventions
 *   - Every call returns sbmp_status (0 = SBMP_OK).  On failure
 *     sbmp_last_error() describes the cause.  (The reference has no error
 *     codes: CUDA_ERROR_CHECK prints and exit(1)s, include/helper/helper.cuh:19-27,
 *     and the KGMT kernel launches are unchecked.)
 *   - Host arrays are plain C arrays; device arrays are HIP device pointers
 *     (d_ prefix), exactly as the reference's plan() takes d_obstacles.
 *   - One planner handle = one HIP stream on one device; a handle is not
 *     thread-safe.  plan()/begin() may be called repeatedly on one handle
 *     (the reference's plan() is single-shot: it frees ctor-owned buffers,
 *     KGMT.cu:314-316).
 */
#ifndef SBMP_H
#define SBMP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SBMP_ABI_VERSION 1

typedef int sbmp_status;
#define SBMP_OK 0
#define SBMP_ERR_INVALID_ARGUMENT 1
#define SBMP_ERR_HIP 2
#define SBMP_ERR_IO 3
#define SBMP_ERR_OUT_OF_MEMORY 4
#define SBMP_ERR_STATE 5
#define SBMP_ERR_UNSUPPORTED 6
#define SBMP_ERR_COMM 7

#define SBMP_AGENT_CAR 0   /* kinematic bicycle, reference src/statePropagator/statePropagator.cu:5-76 */
#define SBMP_AGENT_POINT 1 /* holonomic R2 point (build extension, no reference counterpart) */

#define SBMP_SAMPLE_DIM 7  /* [x, y, theta, v, a, steering, duration], reference KGMT.cu:5, State.h:6-20 */

/* Constructor arguments of KGMT::KGMT (reference KGMT.cuh:28, KGMT.cu:10-78)
 * plus the build's knobs. */
typedef struct sbmp_kgmt_params {
    float width, height;      /* workspace extent */
    int N, n;                 /* R1 grid N x N (N must be 16, KGMT.cu:8); R2 sub-grid n x n per R1 cell (1..16) */
    int numIterations;        /* loop bound, KGMT.cu:118 */
    int maxTreeSize;          /* tree capacity M */
    int numDisc;              /* Euler sub-steps per child, statePropagator.cu:33 */
    float agentLength;        /* bicycle wheelbase, statePropagator.cu:58 */
    float goalThreshold;      /* goal radius, KGMT.cu:635-638 (0 disables the goal) */
    int samplesPerIteration;  /* 0 = reference batch rule (KGMT.cu:151-219); S > 0 = capped extension */
    int agent;                /* SBMP_AGENT_* */
    int fixGNewClear;         /* 0 = reproduce the reference's partial GNew clear */
    int device;               /* HIP device ordinal */
    int profileKernels;       /* 1 = time every kernel launch with HIP events (sbmp_kgmt_kernel_stats) */
    int batchRule;            /* SBMP_BATCH_REFERENCE or SBMP_BATCH_FILL (needs samplesPerIteration > 0) */
} sbmp_kgmt_params;

/* Children per frontier node.  REFERENCE: 32, or floor(remaining/|G|) once 32|G|
 * exceeds the remaining capacity (KGMT.cu:151-158), with remaining additionally
 * capped at samplesPerIteration when that is > 0.  FILL (build extension D14):
 * floor(samplesPerIteration/|G|) children per frontier node, so every iteration
 * generates (almost exactly) samplesPerIteration children. */
#define SBMP_BATCH_REFERENCE 0
#define SBMP_BATCH_FILL 1

/* Outcome of a plan (the reference's public fields treeSize_/costToGoal_, KGMT.cuh:37,40,
 * plus what its prints report, KGMT.cu:295-296). */
typedef struct sbmp_plan_result {
    int iterations;           /* loop iterations executed */
    int treeSize;             /* treeSize_ (may exceed maxTreeSize on the final iteration, as in the reference) */
    float costToGoal;         /* costToGoal_: cost of the first goal node, 0 if none */
    int goalIndex;            /* tree row of that node, -1 if none (D4: lowest row of the first goal iteration) */
    long long samplesGenerated; /* children propagated and collision-checked, all iterations */
    long long accepted;       /* nodes appended to the tree, all iterations */
    double wallMs;            /* device-synchronised wall time of the iteration loop */
    int stalled;              /* 1 if the loop ended with an empty frontier (D7) */
} sbmp_plan_result;

/* Per-iteration bookkeeping (same fields as the oracle's log). */
typedef struct sbmp_iter_record {
    int itr, treeSizeBefore, nG, k, nExp, S, A, treeSizeAfter, goalIdx;
} sbmp_iter_record;

typedef struct sbmp_kernel_stat {
    char name[32];
    long long launches;
    double totalMs;           /* sum of HIP-event durations on the planner's stream */
} sbmp_kernel_stat;

/* Which form of the hot path a planner runs (sbmp_kgmt_path_info): no reference
 * counterpart (the reference has one form, KGMT.cu:118-292); for logs and bench lines. */
#define SBMP_OBS_REGISTERS 0  /* <= 8 boxes held in registers (wave cull + per-step schedule) */
#define SBMP_OBS_LDS 1        /* <= 2,048 boxes staged in LDS per workgroup */
#define SBMP_OBS_GRID 2       /* uniform-grid obstacle index (include/sbmp/obstacle_grid.h) */
#define SBMP_OBS_GLOBAL 3     /* the all-boxes loop from global memory (diagnostics) */
#define SBMP_EXCHANGE_NONE 0      /* one rank */
#define SBMP_EXCHANGE_ONESHOT 1   /* k_oneshot through IPC-mapped inboxes (sharded default) */
#define SBMP_EXCHANGE_COLLECTIVE 2 /* the communicator's all-reduce (RCCL, or host callbacks) */
typedef struct sbmp_path_info {
    int stepForm;             /* 1: one k_step launch per iteration; 0: k_expand + k_finish (+ k_pack) */
    int obstacleForm;         /* SBMP_OBS_* of the last begin() */
    int residentGroups;       /* k_step workgroups the device holds at once (occupancy x CUs), 0 if not k_step-capable */
    int neededGroups;         /* 1 + blocks per rank: k_step needs them all resident */
    int exchange;             /* SBMP_EXCHANGE_* */
    int nranks, rank;
    int commRanks;            /* ranks of the RCCL communicator (0: none) */
    int listMirror;           /* 1: the one-shot exchange copies the flagged-children lists into each
                                 rank's mirror, and k_step reads its parents from local HBM */
    int fusedExchange;        /* 1: the last expanding workgroup of k_step runs the one-shot exchange
                                 (no k_oneshot launch) */
    int oneshotCheck;         /* start-up check of the one-shot exchange: 0 not run, 1 passed,
                                 -1 failed on some rank (every rank then uses the all-reduce) */
    int mirrorCheck;          /* start-up check of the list mirror (stores into peers' mirrors
                                 seen after a kernel boundary): 0 not run, 1 passed, -1 failed
                                 on some rank (every rank then reads the lists over the mapping) */
    int fusedCheck;           /* start-up check of the fused exchange's in-kernel order (pushes
                                 drained, relaxed arrivals, the workers' flags, the peers' next
                                 launch reading the mirror): 0 not run, 1 passed, -1 failed on some
                                 rank (every rank then runs the exchange as its own k_oneshot) */
    int rowTableLds;          /* sharded k_step: 1 stages the exchange's u16 block counts in LDS
                                 (row positions without a dependent load); 0 reads a row's block
                                 words (chosen when the table's LDS would cost residency) */
} sbmp_path_info;

typedef struct sbmp_kgmt sbmp_kgmt;

int sbmp_abi_version(void);
const char* sbmp_status_string(sbmp_status s);
const char* sbmp_last_error(void);

/* The demo configuration, reference demos/main.cu:19-28. */
sbmp_status sbmp_kgmt_default_params(sbmp_kgmt_params* p);

/* A system / workspace file (systems/NAME.yaml): the reference hardcodes
 * this in demos/main.cu:19-46 and leaves systems/car.yaml empty.  Flat "key: value"
 * lines over the demo defaults: agent, width, height, N, n, numIterations, maxTreeSize,
 * numDisc, agentLength, goalThreshold, samplesPerIteration, batchRule (reference | fill),
 * fixGNewClear, device, initial / goal ([7 values] or a CSV file such as
 * configurations/init/init.csv), obstacles (a CSV path, resolved against the file's
 * directory).  Numeric keys may name a file holding the number.  Unknown keys fail. */
typedef struct sbmp_system_config {
    sbmp_kgmt_params params;
    float initial[7];
    float goal[7];
    char obstacles[1024];     /* resolved path, "" if the file names none */
} sbmp_system_config;
sbmp_status sbmp_load_system_config(const char* path, sbmp_system_config* out);

/* KGMT::KGMT (KGMT.cu:10-78): allocates every planner buffer on p->device. */
sbmp_status sbmp_kgmt_create(const sbmp_kgmt_params* p, sbmp_kgmt** out);
sbmp_status sbmp_kgmt_destroy(sbmp_kgmt* h);

/* KGMT::plan (KGMT.cu:80-317): root init, RNG init (curand_init(seed, slot, 0),
 * KGMT.cu:111 — the reference seeds with time(NULL); here the seed is explicit),
 * iterate until goal / full tree / numIterations.  initial and goal are host
 * arrays of 7 floats; d_obstacles is a device array of obstaclesCount boxes
 * [xmin, ymin, xmax, ymax] (reference collisionCheck.cu:7-14).  Blocking. */
sbmp_status sbmp_kgmt_plan(sbmp_kgmt* h, const float initial[7], const float goal[7], const float* d_obstacles,
                           int obstaclesCount, uint64_t seed, sbmp_plan_result* result);

/* Stepwise form of plan: begin = prologue (KGMT.cu:84-116); step enqueues up to
 * `iterations` more loop iterations and waits for them (*active = 0 once the
 * loop has ended); result reads the outcome. */
sbmp_status sbmp_kgmt_begin(sbmp_kgmt* h, const float initial[7], const float goal[7], const float* d_obstacles,
                            int obstaclesCount, uint64_t seed);
sbmp_status sbmp_kgmt_step(sbmp_kgmt* h, int iterations, int* active);
/* Enqueue iterations without waiting (device-resident loop; kernels become
 * no-ops once the loop has ended).  sbmp_kgmt_sync waits for the stream. */
sbmp_status sbmp_kgmt_enqueue(sbmp_kgmt* h, int iterations);
sbmp_status sbmp_kgmt_sync(sbmp_kgmt* h);
/* Enqueue, without waiting, the fold of R2Valid / R2Invalid (KGMT.cu:405,410) over
 * every iteration enqueued so far.  The loop folds its per-child key log every 32
 * iterations; exports fold the rest themselves.  A timed window calls this before
 * its closing sync so the deferred work of its own iterations is inside it. */
sbmp_status sbmp_kgmt_fold(sbmp_kgmt* h);
sbmp_status sbmp_kgmt_result(sbmp_kgmt* h, sbmp_plan_result* result);
/* The HIP stream (hipStream_t) every kernel of this planner runs on. */
sbmp_status sbmp_kgmt_stream(sbmp_kgmt* h, void** stream);

/* State export in the reference's layouts (thrust vectors of KGMT.cuh:44-68):
 * samples M x 7 AoS, parents M, costs M, bools as bytes.  capacity = rows of
 * the caller's arrays (must be >= maxTreeSize).  Any pointer may be NULL. */
sbmp_status sbmp_kgmt_copy_tree(sbmp_kgmt* h, float* samples, int* parent, float* costs, int capacity);
sbmp_status sbmp_kgmt_copy_unexplored(sbmp_kgmt* h, float* samples, int* uParent, int capacity);
sbmp_status sbmp_kgmt_copy_flags(sbmp_kgmt* h, uint8_t* G, uint8_t* GNew, int capacity);
/* R1* arrays have N*N entries, R2* arrays N*N*n*n. */
sbmp_status sbmp_kgmt_copy_regions(sbmp_kgmt* h, int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score,
                                   int* R2Avail, int* R2Valid, int* R2Invalid);
/* XORWOW state per slot: 6 words {v0..v4, d}.  Slots = sbmp_kgmt_num_slots. */
sbmp_status sbmp_kgmt_num_slots(sbmp_kgmt* h, int* slots);
sbmp_status sbmp_kgmt_copy_rng(sbmp_kgmt* h, uint32_t* states, int capacity);
sbmp_status sbmp_kgmt_iter_log(sbmp_kgmt* h, sbmp_iter_record* out, int capacity, int* count);
/* The 13 CSV dumps of KGMT.cu:299-311 (std::fixed, 10 decimals, helper.cuh:53-72) into dir. */
sbmp_status sbmp_kgmt_export_csv(sbmp_kgmt* h, const char* dir);
/* The per-iteration dumps the reference has commented out (KGMT.cu:263-290), read by
 * visualization/visualizationKGMT_Steps.m: with dir set, sbmp_kgmt_plan runs one
 * iteration at a time (one host sync each) and after iteration itr writes
 * dir/Data/{Samples/samples, Parents/parents, R1Scores/R1Scores, R1Avail/R1Avail,
 * R1/R1, UnexploredSamples/unexploredSamples}<itr>.csv in the export format.
 * dir NULL or "": off (the default). */
sbmp_status sbmp_kgmt_set_iteration_dump(sbmp_kgmt* h, const char* dir);

/* Solution path (the reference keeps only the goal node's cost,
 * KGMT.cu:586-591): the tree rows from the root to `node` (node < 0: the
 * solution node, result goalIndex), root first, found by walking treeParent.
 * rows (ints), samples (7 floats per row, the samples.csv layout of
 * KGMT.cu:299) and costs may each be NULL; capacity = their length in rows.
 * *length = the path length (0 if node < 0 and there is no solution); with
 * capacity < *length the call fails with SBMP_ERR_INVALID_ARGUMENT (and still sets
 * *length), so a NULL/0 call returns the size to allocate. */
sbmp_status sbmp_kgmt_solution_path(sbmp_kgmt* h, int node, int* rows, float* samples, float* costs, int capacity,
                                    int* length);

sbmp_status sbmp_kgmt_kernel_stats(sbmp_kgmt* h, sbmp_kernel_stat* out, int capacity, int* count);
/* The form of the hot path chosen at the last begin() (sbmp_path_info). */
sbmp_status sbmp_kgmt_path_info(sbmp_kgmt* h, sbmp_path_info* out);
sbmp_status sbmp_kgmt_reset_kernel_stats(sbmp_kgmt* h);
/* Turn per-launch HIP-event timing on/off for subsequently enqueued iterations. */
sbmp_status sbmp_kgmt_set_profiling(sbmp_kgmt* h, int enabled);
/* A 64-bit digest of the replicated planning state after the last enqueued iteration
 * (waits for it): tree rows, region tables of the next iteration, per-iteration control
 * blocks (no reference counterpart).  Every rank of a sharded run holds the same replica,
 * so every rank's digest must be equal: bench.py --gpus N checks it (replicas_agree). */
sbmp_status sbmp_kgmt_state_hash(sbmp_kgmt* h, uint64_t* out);
/* Queue a device-side delay (bounded spin on the GPU clock) so that the
 * launches enqueued after it execute back to back, as in an un-instrumented run. */
sbmp_status sbmp_kgmt_enqueue_delay(sbmp_kgmt* h, double microseconds);
/* Individual launch durations (ms, launch order) of kernel `name` since the last reset. */
sbmp_status sbmp_kgmt_kernel_samples(sbmp_kgmt* h, const char* name, float* out, int capacity, int* count);

/* readObstaclesFromCSV (reference src/helper/helper.cu:11-34): whitespace or
 * comma separated floats, numObstacles = floats / (2*workspaceDim).  Returns
 * SBMP_ERR_IO instead of exit(1) when the file cannot be opened.  capacity is
 * the length of out in floats (>= 2*workspaceDim*numObstacles).  With out == NULL
 * only *numObstacles is computed. */
sbmp_status sbmp_read_obstacles_csv(const char* path, int workspaceDim, float* out, int capacity, int* numObstacles);

/* Legacy random-tree generators behind the reference's Planner interface
 * (include/planners/Planner.cuh:6-12; the reference's CMake does not
 * build them): SBMP_RANDOM_TREE_NAIVE = NaivePlanner::generateRandomTree
 * (NaivePlanner.cu:76-140), SBMP_RANDOM_TREE_COSTPROP = CostPropPlanner
 * (CostPropPlanner.cu:83-139).  rows / blocks / threadsPerBlock <= 0 take the
 * reference's sizes (naive 10 x 32 x 32, costprop 1 x 512 x 1024).  samples: host
 * array of capacity floats >= rows * blocks * threadsPerBlock * 7, row-major like the
 * reference's tree; kernelMs (optional) receives the kernel time.  Semantics and the
 * one deviation (D16): DESIGN.md. */
#define SBMP_RANDOM_TREE_NAIVE 0
#define SBMP_RANDOM_TREE_COSTPROP 1
sbmp_status sbmp_random_tree(int device, int kind, const float* root, int rows, int blocks, int threadsPerBlock,
                             float* samples, long long capacity, float* kernelMs);

/* The uniform-grid obstacle index the planner uses for large obstacle lists
 * (include/sbmp/obstacle_grid.h; replaces the all-boxes loop of isMotionValid,
 * reference src/collisionCheck/collisionCheck.cu:16-28), evaluated on the host:
 * freeOut[i] = isMotionValid(segment i) for nSegments boxes (minx, miny, maxx, maxy).
 * gridSize <= 0 picks the planner's resolution; *gridUsed (optional) receives it.
 * Host-only, no device needed (test entry point). */
sbmp_status sbmp_obstacle_grid_query(const float* obstacles, int nObs, float width, float height, int gridSize,
                                     const float* segments, int nSegments, uint8_t* freeOut, int* gridUsed);

/* ---- Step-level entry points (one stage of the iteration over caller buffers, so each
 * can be parity-tested alone) ----
 *
 * sbmp_expand_batch: propagateG's per-child work (KGMT.cu:386-411): child i expands
 * the parent state parents[7 i .. 7 i + 3] with the XORWOW state rng[6 i .. 6 i + 5]
 * (advanced in place) through propagateAndCheck (include/sbmp/propagator.h, the car;
 * propagatePoint for agent = SBMP_AGENT_POINT), then getR1 / getR2
 * (include/sbmp/grid.h) and, if R1Score and R2Avail are given, the accept test
 * (u <= R1Score[r1] || !R2Avail[r2], one more draw for a valid child; KGMT.cu:394-400).
 * Every pointer is device memory; valid / r1 / r2 / accept may be NULL.
 * sbmp_expand_batch_host runs the same code on the CPU over host buffers. */
typedef struct sbmp_expand_batch_args {
    int count;                       /* children */
    const float* parents;            /* count x 7 */
    uint32_t* rng;                   /* count x 6: v0..v4, d */
    const float* obstacles;          /* obstaclesCount x [xmin, ymin, xmax, ymax] */
    int obstaclesCount;
    int agent;                       /* SBMP_AGENT_CAR / SBMP_AGENT_POINT */
    int numDisc;
    float agentLength, width, height;
    int N, n;                        /* region grid: R1Size = width / N, R2Size = width / (N n) */
    const float* R1Score;            /* N*N, or NULL: no accept test */
    const int* R2Avail;              /* N*N*n*n 0/1 */
    float* children;                 /* count x 7 out: [x, y, theta, v, a, steering, duration] */
    uint8_t* valid;                  /* count out */
    int* r1;                         /* count out (-1: outside the grid) */
    int* r2;                         /* count out */
    uint8_t* accept;                 /* count out */
} sbmp_expand_batch_args;
sbmp_status sbmp_expand_batch(const sbmp_expand_batch_args* args, void* stream /* hipStream_t; NULL: default */);
sbmp_status sbmp_expand_batch_host(const sbmp_expand_batch_args* args);

/* sbmp_insert_batch: exclusive_scan(GNew) + findInd + updateG (KGMT.cu:221-249,
 * 540-593): the flagged slots, in slot order, become tree rows treeSize + j with
 * parent uParent[slot] and cost = costs[parent] + duration (getCost, KGMT.cu:631-633);
 * min(A, 32 floor(M/32)) rows are written (the updateG grid, KGMT.cu:231), none at or
 * past maxTreeSize (D13); then GNew[0 .. 32 min(A, M/32)) is cleared (D6), all of it
 * with fixGNewClear.  *inserted = A, *goalIndex = the lowest new row within
 * goalThreshold of (goalX, goalY) or -1 (D4).  Device buffers; inserted / goalIndex
 * are device ints. */
typedef struct sbmp_insert_batch_args {
    int slots;
    uint8_t* gnew;                   /* slots: accept flags (cleared as above) */
    const float* unexplored;         /* slots x 7 */
    const int* uParent;              /* slots */
    float* samples;                  /* maxTreeSize x 7 */
    int* parent;                     /* maxTreeSize */
    float* costs;                    /* maxTreeSize */
    int treeSize, maxTreeSize;
    float goalX, goalY, goalThreshold;
    int fixGNewClear;
    int* inserted;                   /* 1 */
    int* goalIndex;                  /* 1 */
} sbmp_insert_batch_args;
sbmp_status sbmp_insert_batch(const sbmp_insert_batch_args* args, void* stream);

/* Device memory helpers replacing demos/main.cu:60-61,64 (cudaMalloc/cudaMemcpy/cudaFree). */
sbmp_status sbmp_device_upload_f32(const float* host, size_t count, float** d_out);
sbmp_status sbmp_device_free(void* d_ptr);
/* Raw device buffers for the step-level entry points: allocate, copy in, copy out. */
sbmp_status sbmp_device_alloc(size_t bytes, void** d_out);
sbmp_status sbmp_device_copy_to(void* d_dst, const void* host, size_t bytes);
sbmp_status sbmp_device_copy_from(void* host, const void* d_src, size_t bytes);
sbmp_status sbmp_device_count(int* count);
/* Measured HBM copy bandwidth of the current device (the STREAM-copy
 * figure quoted next to the 8 TB/s spec): a 16-B-per-lane copy of `bytes` (>= 1 MiB)
 * into a second buffer, best of `reps` passes, GB/s = 2 x bytes / time. */
sbmp_status sbmp_hbm_copy_bandwidth(size_t bytes, int reps, double* gbs);

/* ---- Multi-GPU: one planning problem sharded over ranks (one process per GPU) ----
 * Slots are owned block-cyclically (slot s -> rank (s/256) mod nranks); every
 * rank keeps a full replica of the tree; per iteration the ranks all-reduce one
 * fused exchange buffer over RCCL (region deltas, accept flags and counts) and
 * read each other's accepted children over xGMI (IPC-mapped record buffers), so
 * every rank builds the same tree as a 1-GPU run with the same seed. */
#define SBMP_COMM_ID_BYTES 128
sbmp_status sbmp_comm_get_unique_id(uint8_t id[SBMP_COMM_ID_BYTES]);
sbmp_status sbmp_kgmt_create_sharded(const sbmp_kgmt_params* p, const uint8_t id[SBMP_COMM_ID_BYTES], int nranks,
                                     int rank, sbmp_kgmt** out);
/* The same sharded data flow with nranks ranks on ONE device (p->device) and one
 * stream: the all-reduce is a sum kernel, peer records are read directly.  For
 * testing the sharding on a one-GPU machine; the handle behaves like one planner
 * (exports merge the ranks).  nranks = 1 gives a plain planner. */
sbmp_status sbmp_kgmt_create_local_group(const sbmp_kgmt_params* p, int nranks, sbmp_kgmt** out);

/* Host collectives for ranks that do not share an RCCL communicator (several
 * processes on one GPU, or a host program that already runs MPI / gloo).  Each
 * callback is collective over the nranks ranks and blocking, on host buffers, and
 * returns 0 on success.  allreduce_*: recv[i] = sum over ranks of send[i];
 * allgather: recv[q * bytes ..] = rank q's `bytes` bytes of send. */
typedef struct sbmp_host_collectives {
    void* ctx;
    int (*allreduce_u64)(void* ctx, const uint64_t* send, uint64_t* recv, size_t count);
    int (*allreduce_i32)(void* ctx, const int32_t* send, int32_t* recv, size_t count);
    int (*allgather)(void* ctx, const void* send, size_t bytes, void* recv);
} sbmp_host_collectives;
/* The sharded planner of sbmp_kgmt_create_sharded (same kernels, k_pack records
 * read over HIP IPC) with its per-iteration all-reduce and the record-buffer
 * handle exchange done by `coll` on the host: the stream is synchronised, the
 * fused buffer copied out, reduced, copied back.  *coll is copied; its callbacks
 * must stay valid until sbmp_kgmt_destroy. */
sbmp_status sbmp_kgmt_create_sharded_host(const sbmp_kgmt_params* p, const sbmp_host_collectives* coll, int nranks,
                                          int rank, sbmp_kgmt** out);

#ifdef __cplusplus
}
#endif

#endif /* SBMP_H */
