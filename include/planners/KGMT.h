// KGMT.h — drop-in C++ facade of the reference planner class on top of the C ABI.
//
// Replaces reference include/planners/KGMT.cuh:23-109 for callers such as
// demos/main.cu:30,51,60-64: same constructor
//   KGMT(width, height, N, n, numIterations, maxTreeSize, numDisc, agentLength, goalThreshold)
// (KGMT.cuh:28, KGMT.cu:10-78), same void plan(float* initial, float* goal,
// float* d_obstacles, int obstaclesCount) (KGMT.cuh:31, KGMT.cu:80-317), same
// public result fields treeSize_ / costToGoal_ (KGMT.cuh:36,40) and the same prints
// and CSV dumps (KGMT.cu:100,256-257,295-311).  Header-only, plain C++: the caller
// compiles it with any C++ compiler and links libsbmp.so.
//
// Differences, all deliberate:
//   - errors: every ABI failure prints the cause and exit(1)s, matching the
//     reference's CUDA_ERROR_CHECK (helper.cuh:19-27); the reference's own kernel
//     launches are unchecked;
//   - the RNG seed is time(NULL) converted to unsigned long long exactly as the
//     reference's initCurandStates(..., int seed) (KGMT.cu:111, D1); setSeed() makes
//     it explicit for reproducible runs;
//   - plan() may be called more than once (the reference frees ctor-owned buffers
//     at the end of plan, KGMT.cu:314-316);
//   - "time inside KGMT" is wall time of the device-resident loop, not std::clock
//     CPU time (KGMT.cu:294-295).
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <ctime>
#include <iostream>
#include <vector>

#include "sbmp/sbmp.h"

#define SBMP_CHECK(call)                                                                               \
    do {                                                                                               \
        const sbmp_status s_ = (call);                                                                 \
        if (s_ != SBMP_OK) {                                                                           \
            fprintf(stderr, "%s failed: %s: %s\n", #call, sbmp_status_string(s_), sbmp_last_error());  \
            exit(1);                                                                                   \
        }                                                                                              \
    } while (0)

class KGMT {
public:
    KGMT() = default;
    KGMT(float width, float height, int N, int n, int numIterations, int maxTreeSize, int numDisc, float agentLength,
         float goalThreshold)
        : numIterations_(numIterations), maxTreeSize_(maxTreeSize), numDisc_(numDisc), treeSize_(0), width_(width),
          height_(height), costToGoal_(0.0f), agentLength_(agentLength), R1Threshold_(0.0f),
          goalThreshold_(goalThreshold) {
        SBMP_CHECK(sbmp_kgmt_default_params(&params_));
        params_.width = width;
        params_.height = height;
        params_.N = N;
        params_.n = n;
        params_.numIterations = numIterations;
        params_.maxTreeSize = maxTreeSize;
        params_.numDisc = numDisc;
        params_.agentLength = agentLength;
        params_.goalThreshold = goalThreshold;
        SBMP_CHECK(sbmp_kgmt_create(&params_, &h_));
    }
    // Build extension: every planner parameter, e.g. from a system file (loadConfig).
    explicit KGMT(const sbmp_kgmt_params& p)
        : numIterations_(p.numIterations), maxTreeSize_(p.maxTreeSize), numDisc_(p.numDisc), treeSize_(0),
          width_(p.width), height_(p.height), costToGoal_(0.0f), agentLength_(p.agentLength), R1Threshold_(0.0f),
          goalThreshold_(p.goalThreshold), params_(p) {
        SBMP_CHECK(sbmp_kgmt_create(&params_, &h_));
    }
    ~KGMT() {
        if (h_) sbmp_kgmt_destroy(h_);
    }
    // systems/*.yaml (the reference hardcodes these in main.cu:19-46).
    static sbmp_system_config loadConfig(const char* path) {
        sbmp_system_config c;
        SBMP_CHECK(sbmp_load_system_config(path, &c));
        return c;
    }
    KGMT(const KGMT&) = delete;
    KGMT& operator=(const KGMT&) = delete;

    // KGMT.cu:80-317.  initial / goal: 7 host floats; d_obstacles: device array of
    // obstaclesCount boxes [xmin, ymin, xmax, ymax].
    void plan(float* initial, float* goal, float* d_obstacles, int obstaclesCount) {
        printf("Goal: %f, %f\n", goal[0], goal[1]);   // KGMT.cu:100
        const uint64_t seed = explicitSeed_ ? seed_ : (uint64_t)(long long)(int)time(NULL);
        SBMP_CHECK(sbmp_kgmt_plan(h_, initial, goal, d_obstacles, obstaclesCount, seed, &result_));
        treeSize_ = result_.treeSize;
        costToGoal_ = result_.costToGoal;
        if (costToGoal_ == 0.0f && treeSize_ >= maxTreeSize_) {   // KGMT.cu:256-257
            printf("Iteration %d, Tree size %d\n", result_.iterations, treeSize_);
            printf("Tree size exceeded maxTreeSize\n");
        }
        std::cout << "time inside KGMT is " << result_.wallMs / 1e3 << std::endl;   // KGMT.cu:294-295
        printf("Iteration %d, Tree size %d\n", result_.iterations, treeSize_);       // KGMT.cu:296
        if (writeCsv_) SBMP_CHECK(sbmp_kgmt_export_csv(h_, "."));                   // KGMT.cu:299-311
    }

    // Build extensions.
    void setSeed(uint64_t seed) {
        seed_ = seed;
        explicitSeed_ = true;
    }
    void setWriteCsv(bool on) { writeCsv_ = on; }
    // The per-iteration Data/<Kind>/<kind><itr>.csv dumps of KGMT.cu:263-290 (commented
    // out in the reference); nullptr: off.
    void dumpIterations(const char* dir) { SBMP_CHECK(sbmp_kgmt_set_iteration_dump(h_, dir)); }
    const sbmp_plan_result& result() const { return result_; }
    // Path root .. solution node: tree rows and their 7-float
    // samples; empty if plan() found no solution.
    void solutionPath(std::vector<int>& rows, std::vector<float>& samples) const {
        int n = 0;
        SBMP_CHECK(sbmp_kgmt_solution_path(h_, -1, nullptr, nullptr, nullptr, 0, &n));
        rows.assign(n, 0);
        samples.assign(7 * (size_t)n, 0.0f);
        if (n) SBMP_CHECK(sbmp_kgmt_solution_path(h_, -1, rows.data(), samples.data(), nullptr, n, &n));
    }
    sbmp_kgmt* handle() const { return h_; }

    // Public fields of KGMT.cuh:33-43 that carry meaning outside the class.
    int numIterations_ = 0;
    int maxTreeSize_ = 0;
    int numDisc_ = 0;
    int treeSize_ = 0;
    float width_ = 0.0f;
    float height_ = 0.0f;
    float costToGoal_ = 0.0f;
    float agentLength_ = 0.0f;
    float R1Threshold_ = 0.0f;   // dead in the reference (D12)
    float goalThreshold_ = 0.0f;

private:
    sbmp_kgmt_params params_{};
    sbmp_kgmt* h_ = nullptr;
    uint64_t seed_ = 0;
    bool explicitSeed_ = false;
    bool writeCsv_ = true;
    sbmp_plan_result result_{};
};
