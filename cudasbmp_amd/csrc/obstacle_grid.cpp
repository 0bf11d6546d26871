// obstacle_grid.cpp — CSR build of the uniform-grid obstacle index (see
// include/sbmp/obstacle_grid.h for the layout and why the lookup is exact).
#include "obstacle_grid.h"

#include <algorithm>
#include <cmath>

namespace sbmp {

namespace {

struct CellRange {
    int x0, x1, y0, y1;
};

CellRange cells_of(const float* b, int g, float invW, float invH) {
    if (std::isnan(b[0]) || std::isnan(b[1]) || std::isnan(b[2]) || std::isnan(b[3])) return {0, g - 1, 0, g - 1};
    const int a = grid_cell(b[0], invW, g), c = grid_cell(b[2], invW, g);
    const int e = grid_cell(b[1], invH, g), f = grid_cell(b[3], invH, g);
    return {std::min(a, c), std::max(a, c), std::min(e, f), std::max(e, f)};
}

long long count_entries(const float* obs, int n, int g, float invW, float invH) {
    long long total = 0;
    for (int i = 0; i < n; ++i) {
        const CellRange r = cells_of(obs + 4 * i, g, invW, invH);
        total += (long long)(r.x1 - r.x0 + 1) * (r.y1 - r.y0 + 1);
    }
    return total;
}

}  // namespace

HostObstacleGrid build_obstacle_grid(const float* obs, int n, float width, float height, int g,
                                     long long maxEntries) {
    HostObstacleGrid G;
    if (g <= 0) g = grid_resolution(n);
    float invW = (float)g / width, invH = (float)g / height;
    while (g > 1 && count_entries(obs, n, g, invW, invH) > maxEntries) {
        g /= 2;
        invW = (float)g / width;
        invH = (float)g / height;
    }
    G.g = g;
    G.invW = invW;
    G.invH = invH;
    std::vector<int> cnt((size_t)g * g + 1, 0);
    for (int i = 0; i < n; ++i) {
        const CellRange r = cells_of(obs + 4 * i, g, invW, invH);
        for (int y = r.y0; y <= r.y1; ++y)
            for (int x = r.x0; x <= r.x1; ++x) ++cnt[(size_t)y * g + x];
    }
    G.start.assign((size_t)g * g + 1, 0);
    for (size_t c = 0; c < (size_t)g * g; ++c) G.start[c + 1] = G.start[c] + cnt[c];
    G.boxes.resize((size_t)G.start[(size_t)g * g]);
    std::vector<int> fill(G.start.begin(), G.start.end() - 1);
    for (int i = 0; i < n; ++i) {   // ascending box index within every cell
        const float* b = obs + 4 * i;
        const CellRange r = cells_of(b, g, invW, invH);
        for (int y = r.y0; y <= r.y1; ++y)
            for (int x = r.x0; x <= r.x1; ++x) G.boxes[(size_t)fill[(size_t)y * g + x]++] = {b[0], b[1], b[2], b[3]};
    }
    return G;
}

}  // namespace sbmp
