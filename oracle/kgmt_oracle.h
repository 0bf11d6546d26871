/* oracle/kgmt_oracle.h — TEST INFRASTRUCTURE ONLY.
 *
 * C API of the CPU restatement of the reference KGMT planner
 * (reference src/planners/KGMT.cu:80-638, src/statePropagator/statePropagator.cu:5-76,
 * src/collisionCheck/collisionCheck.cu:6-28).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg load this library, as the checker or as the
 * timed CPU baseline; the product library never links it.
 */
#ifndef KGMT_ORACLE_H
#define KGMT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct oracle_params {
    float width, height;        /* workspace (main.cu:20-21) */
    int N, n;                   /* R1 grid N x N, R2 sub-grid n x n per R1 cell (main.cu:22-23) */
    int numIterations;          /* main.cu:24 */
    int maxTreeSize;            /* main.cu:25 */
    int numDisc;                /* main.cu:26 */
    float agentLength;          /* main.cu:27 */
    float goalThreshold;        /* main.cu:28 */
    int samplesPerIteration;    /* 0 = reference batch rule (KGMT.cu:151-219); >0 = capped extension */
    int agent;                  /* 0 = car (statePropagator.cu), 1 = R2 point (build extension) */
    int fixGNewClear;           /* 0 = reproduce the partial GNew clear (D6) */
    int threads;                /* OpenMP threads for the expansion loop (<=0: 1) */
    int nranks, rank;           /* slot-ownership sharding (1, 0 = unsharded) */
    int batchRule;              /* 0 = reference rule + cap, 1 = fill the cap (D14) */
} oracle_params;

/* One accepted child as exchanged between ranks: slot id, 7 sample floats, parent. */
typedef struct oracle_record {
    int32_t slot;
    float sample[7];
    int32_t parent;
} oracle_record;

/* Per-iteration bookkeeping. */
typedef struct oracle_iter_log {
    int itr, treeSizeBefore, nG, k, nExp, S, A, treeSizeAfter, goalIdx;
} oracle_iter_log;

#define ORACLE_DELTA_R1_FIELDS 4  /* R1, R1Valid, R1Invalid, R1AvailSet */
#define ORACLE_DELTA_R2_FIELDS 3  /* R2AvailSet, R2Valid, R2Invalid */

void* oracle_create(const oracle_params* p);
void oracle_destroy(void* h);

/* Equivalent of KGMT::plan's prologue (KGMT.cu:84-116) with an explicit curand seed. */
int oracle_begin(void* h, const float initial[7], const float goal[7], const float* obstacles,
                 int obstaclesCount, uint64_t seed);
/* One loop iteration (KGMT.cu:118-292).  Returns 1 if it ran, 0 if the loop had already ended. */
int oracle_step(void* h);
/* begin + step until the loop ends.  Returns the number of iterations run. */
int oracle_plan(void* h, const float initial[7], const float goal[7], const float* obstacles,
                int obstaclesCount, uint64_t seed);

/* Sharded form of oracle_step, for the multi-rank protocol tests:
 * expand_local runs score + frontier + expansion of the slots this rank owns and
 * returns the number of local accepted records (copied out with
 * oracle_local_records) and the region deltas (oracle_local_deltas, int32
 * [4*N*N + 3*N*N*n*n]); finish applies the summed deltas and the gathered
 * records (any order: sorted by slot inside) and does insertion/termination. */
int oracle_expand_local(void* h);
int oracle_local_records(void* h, oracle_record* out, int capacity);
int oracle_delta_size(void* h);
int oracle_local_deltas(void* h, int32_t* out);
int oracle_finish(void* h, const oracle_record* records, int count, const int32_t* summedDeltas);

/* State accessors (reference layouts: AoS samples M x 7, bools as bytes). */
int oracle_info(void* h, int* itr, int* treeSize, int* goalIdx, float* costToGoal, int* terminated);
int oracle_num_slots(void* h);
int oracle_tree(void* h, float* samples, int* parent, float* costs);
int oracle_unexplored(void* h, float* samples, int* uParent);
int oracle_flags(void* h, uint8_t* G, uint8_t* GNew);
int oracle_regions(void* h, int* R1, int* R1Avail, int* R1Valid, int* R1Invalid, float* R1Score,
                   int* R2Avail, int* R2Valid, int* R2Invalid);
int oracle_rng(void* h, uint32_t* states /* num_slots x 6: v0..v4, d */);
int oracle_iter_logs(void* h, oracle_iter_log* out, int capacity);
long long oracle_samples_generated(void* h);

/* cuRAND XORWOW restatement exposed for the RNG known-answer tests.
 * seeding: 0 = cuRAND constants, 1 = rocRAND constants. */
void oracle_xorwow_init(uint64_t seed, uint64_t subsequence, int seeding, uint32_t state[6]);
void oracle_xorwow_draw(uint32_t state[6], int count, uint32_t* out);

/* Invariant I1: re-propagate parents (n x 4) with stored controls (n x 3: a, steering,
 * duration) -> out (n x 4), valid (n).  Uses prm's agent, numDisc, agentLength, workspace. */
void oracle_expand_batch(const oracle_params* prm, const float* obstacles, int nObs, const float* parents,
                         uint32_t* rng, int n, const float* R1Score, const int* R2Avail, float* children,
                         uint8_t* valid, int* r1, int* r2, uint8_t* accept);
void oracle_replay(const oracle_params* prm, const float* obstacles, int nObs, const float* parents,
                   const float* controls, int n, float* out, uint8_t* valid);

/* Deterministic math exposed for tests. */
void oracle_sincosf(const float* x, int n, float* s, float* c);
void oracle_tanf(const float* x, int n, float* t);

#ifdef __cplusplus
}
#endif

#endif
