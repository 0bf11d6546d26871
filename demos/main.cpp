// demos/main.cpp — the reference's demos/main.cu (lines 17-68) on the MI355X planner.
//
// Same workspace, planner arguments, start and goal; the CUDA calls become the C
// ABI's device helpers (cudaMalloc/cudaMemcpy -> sbmp_device_upload_f32,
// cudaFree -> sbmp_device_free) and readObstaclesFromCSV becomes
// sbmp_read_obstacles_csv (helper.cu:11-34).  Build: make -C demos; run from
// demos/ (the reference runs from build/, hence the ../configurations path).
//   ./main [obstacles.csv] [seed]
//   ./main --config ../systems/car.yaml [seed] [--dump-iterations DIR]
// --config takes every constant below from a system file instead;
// --dump-iterations writes the per-iteration CSVs of KGMT.cu:263-290.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "planners/KGMT.h"

#define WORKSPACE_DIM 2

int main(int argc, char** argv) {
    std::vector<const char*> args;
    const char* configPath = nullptr;
    const char* dumpDir = nullptr;
    for (int i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "--config") && i + 1 < argc) configPath = argv[++i];
        else if (!strcmp(argv[i], "--dump-iterations") && i + 1 < argc) dumpDir = argv[++i];
        else args.push_back(argv[i]);
    }
    int sampleDim = 7;
    float width = 20.0;
    float height = 20.0;
    int N = 16;
    int n = 8;
    int numIterations = 100;
    int maxTreeSize = 30000;
    int numDisc = 10;
    float agentLength = 1.0;
    float goalThreshold = 0.5;

    sbmp_system_config cfg{};
    if (configPath) cfg = KGMT::loadConfig(configPath);
    std::unique_ptr<KGMT> planner(configPath ? new KGMT(cfg.params)
                                             : new KGMT(width, height, N, n, numIterations, maxTreeSize, numDisc,
                                                        agentLength, goalThreshold));
    KGMT& kgmt = *planner;
    const char* seedArg = configPath ? (args.size() > 0 ? args[0] : nullptr) : (args.size() > 1 ? args[1] : nullptr);
    if (seedArg) kgmt.setSeed(strtoull(seedArg, nullptr, 10));
    if (dumpDir) kgmt.dumpIterations(dumpDir);
    float* initial = new float[sampleDim];
    float* goal = new float[sampleDim];
    initial[0] = 5;
    initial[1] = 5;
    initial[2] = 0;
    initial[3] = 0;
    initial[4] = 0;
    initial[5] = 0;
    initial[6] = 0;
    goal[0] = 2;
    goal[1] = 18;
    goal[2] = 0;
    goal[3] = 0;
    goal[4] = 0;
    goal[5] = 0;
    goal[6] = 0;

    if (configPath) {
        for (int i = 0; i < sampleDim; ++i) {
            initial[i] = cfg.initial[i];
            goal[i] = cfg.goal[i];
        }
    }
    const char* path = configPath ? cfg.obstacles
                                  : (args.size() > 0 ? args[0] : "../configurations/obstacles/obstacles.csv");
    int numObstacles = 0;
    SBMP_CHECK(sbmp_read_obstacles_csv(path, WORKSPACE_DIM, nullptr, 0, &numObstacles));
    std::vector<float> obstacles(2 * WORKSPACE_DIM * (size_t)numObstacles);
    SBMP_CHECK(sbmp_read_obstacles_csv(path, WORKSPACE_DIM, obstacles.data(), (int)obstacles.size(), &numObstacles));
    printf("Obstacles: \n");
    for (int i = 0; i < numObstacles; i++) {
        for (int j = 0; j < 2 * WORKSPACE_DIM; j++) printf("%f ", obstacles[i * 2 * WORKSPACE_DIM + j]);
        printf("\n");
    }
    printf("numObstacles: %d\n", numObstacles);
    float* d_obstacles = nullptr;
    SBMP_CHECK(sbmp_device_upload_f32(obstacles.data(), obstacles.size(), &d_obstacles));
    kgmt.plan(initial, goal, d_obstacles, numObstacles);

    SBMP_CHECK(sbmp_device_free(d_obstacles));
    delete[] initial;
    delete[] goal;
    return 0;
}
