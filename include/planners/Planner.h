// Planner.h — the reference's legacy planner interface and its two random-tree
// generators (include/planners/Planner.cuh:6-12, NaivePlanner.cuh, CostPropPlanner.cuh;
// src/planners/NaivePlanner.cu, CostPropPlanner.cu), header-only over the C ABI
// (sbmp_random_tree).  The reference's CMake does not build these.
//
// Kept from the reference: the interface (plan, generateRandomTree), plan() calling
// generateRandomTree(start, 100, &samples), the hard-coded sizes (naive 10 rows of
// 32 x 32 threads, costprop 1 row of 512 x 1024), the prints, and the naive
// planner's samples.csv ("%f," per value, one tree row per line, NaivePlanner.cu:133-140).
// Differences: errors exit(1) like the reference's CUDA_ERROR_CHECK;
// generateRandomTree hands the tree back through *samples (new[]; the reference never
// assigns it, so callers of the reference pass it and ignore it); D16:
// the naive planner's next-row parent is the block's first sample of the previous row
// (the reference reads it out of bounds of `root`).
#pragma once

#include <cstdio>
#include <cstdlib>

#include "sbmp/sbmp.h"

#ifndef SBMP_CHECK
#define SBMP_CHECK(call)                                                                               \
    do {                                                                                               \
        const sbmp_status s_ = (call);                                                                 \
        if (s_ != SBMP_OK) {                                                                           \
            fprintf(stderr, "%s failed: %s: %s\n", #call, sbmp_status_string(s_), sbmp_last_error());  \
            exit(1);                                                                                   \
        }                                                                                              \
    } while (0)
#endif

class Planner {
public:
    virtual ~Planner() = default;
    virtual void plan(float* root, float* goal) = 0;
    virtual void generateRandomTree(const float* root, const int numSamples, float** samples) = 0;
};

namespace sbmp_legacy {

// rows x (blocks * threads) samples of 7 floats; prints like the reference.
inline float* random_tree(int kind, const float* root, int rows, int blocks, int threads, bool writeCsv) {
    const long long n = (long long)rows * blocks * threads * 7;
    float* tree = new float[n];
    float ms = 0.0f;
    SBMP_CHECK(sbmp_random_tree(0, kind, root, rows, blocks, threads, tree, n, &ms));
    printf("Kernel execution time: %f milliseconds\n", ms);
    printf("Tree size: %d\n", (int)n);   // rowsTree * colsTree floats, as the reference prints
    if (writeCsv) {
        FILE* fp = fopen("samples.csv", "w");
        if (!fp) {
            fprintf(stderr, "cannot open samples.csv\n");
            exit(1);
        }
        const long long cols = (long long)blocks * threads * 7;
        for (int i = 0; i < rows; ++i) {
            for (long long j = 0; j < cols; ++j) fprintf(fp, "%f,", tree[(long long)i * cols + j]);
            fprintf(fp, "\n");
        }
        fclose(fp);
    }
    return tree;
}

}  // namespace sbmp_legacy

class NaivePlanner : public Planner {
public:
    NaivePlanner() = default;
    void plan(float* start, float* goal) override {   // NaivePlanner.cu:18-23
        (void)goal;
        float* samples = nullptr;
        generateRandomTree(start, 100, &samples);
        delete[] samples;
    }
    void generateRandomTree(const float* root, const int numSamples, float** samples) override {
        (void)numSamples;   // ignored, as in the reference (sizes hard-coded, NaivePlanner.cu:78-81)
        float* t = sbmp_legacy::random_tree(SBMP_RANDOM_TREE_NAIVE, root, 10, 32, 32, true);
        if (samples) *samples = t;
        else delete[] t;
    }
};

class CostPropPlanner : public Planner {
public:
    CostPropPlanner() = default;
    void plan(float* start, float* goal) override {   // CostPropPlanner.cu:18-23
        (void)goal;
        float* samples = nullptr;
        generateRandomTree(start, 100, &samples);
        delete[] samples;
    }
    void generateRandomTree(const float* root, const int numSamples, float** samples) override {
        (void)numSamples;   // ignored, as in the reference (CostPropPlanner.cu:85-87)
        float* t = sbmp_legacy::random_tree(SBMP_RANDOM_TREE_COSTPROP, root, 1, 512, 1024, false);
        if (samples) *samples = t;
        else delete[] t;
    }
};
