// The reference's legacy planners (include/planners/Planner.cuh) on MI355X: runs
// NaivePlanner::plan / CostPropPlanner::generateRandomTree from a root given on the
// command line.  Usage: random_tree [naive|costprop] [x y theta v]
#include <cstring>
#include <iostream>

#include "planners/Planner.h"

int main(int argc, char** argv) {
    const bool naive = argc < 2 || strcmp(argv[1], "costprop") != 0;
    float root[7] = {5.0f, 5.0f, 0.0f, 1.0f, 0.0f, 0.0f, 0.0f};
    for (int i = 0; i < 4 && 2 + i < argc; ++i) root[i] = (float)atof(argv[2 + i]);
    float goal[7] = {2.0f, 18.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
    Planner* p = naive ? static_cast<Planner*>(new NaivePlanner()) : static_cast<Planner*>(new CostPropPlanner());
    if (naive) {
        p->plan(root, goal);   // NaivePlanner.cu:18-23: writes samples.csv
    } else {
        float* samples = nullptr;
        p->generateRandomTree(root, 100, &samples);
        std::cout << "first sample: " << samples[0] << " " << samples[1] << std::endl;
        delete[] samples;
    }
    delete p;
    return 0;
}
