// Host side of the uniform-grid obstacle index (include/sbmp/obstacle_grid.h).
#pragma once

#include <vector>

#include "sbmp/obstacle_grid.h"

namespace sbmp {

struct HostObstacleGrid {
    int g = 0;
    float invW = 0.0f, invH = 0.0f;
    std::vector<int> start;        // g*g + 1
    std::vector<GridBox> boxes;    // start[g*g] rows
};

// n boxes (xmin, ymin, xmax, ymax) over [0, width) x [0, height).  g <= 0: from
// grid_resolution(n), halved while the copies would exceed maxEntries.
HostObstacleGrid build_obstacle_grid(const float* obs, int n, float width, float height, int g,
                                     long long maxEntries = 1ll << 25);

}  // namespace sbmp
