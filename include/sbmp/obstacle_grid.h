// obstacle_grid.h — uniform-grid obstacle index.
//
// The reference tests every step segment against every obstacle
// (collisionCheck.cu:16-28, isMotionValid: a loop over all boxes, first hit ends
// it).  With 10,000 boxes that loop is the whole cost.  The grid replaces it with
// the boxes of the cells the segment's box covers; the answer is the same boolean,
// bit for bit, for every input:
//
//   cell(v) = clamp(floor(v * inv), 0, G - 1) is monotone non-decreasing in v, and
//   the same function bins the boxes (host) and locates the segments (device).
//   The reference calls a segment box S and obstacle O disjoint iff
//   S.maxx <= O.xmin || O.xmax <= S.minx || (same in y)  (isBroadPhaseValid,
//   collisionCheck.cu:6-14).  If they are not disjoint, S.minx < O.xmax and
//   O.xmin < S.maxx, so cell(S.minx) <= cell(O.xmax) and cell(O.xmin) <=
//   cell(S.maxx): the cell ranges [cell(S.minx), cell(S.maxx)] and
//   [min, max of cell(O.xmin), cell(O.xmax)] intersect, in x and in y alike, and
//   O is listed in a cell the query visits.  (Taking min/max keeps inverted boxes,
//   xmin > xmax, which the reference can still hit.)  A box with a NaN coordinate
//   compares unpredictably and is listed in every cell.
//
// Layout (CSR, row-major cells): start[G*G + 1], boxes[start[G*G]] as float4
// (xmin, ymin, xmax, ymax), each box copied into every cell of its range, so a
// query reads contiguous 16-B rows: for cell row cy, the cells cx0..cx1 are the
// entries start[cy*G + cx0] .. start[cy*G + cx1 + 1].
#pragma once

#include "sbmp/sbmp_math.h"

namespace sbmp {

// Cell of coordinate v; NaN maps to 0 (segments are finite, D15; NaN boxes are
// listed everywhere and never located).
SBMP_HD int grid_cell(float v, float inv, int g) {
    float f = __builtin_floorf(v * inv);
    if (!(f >= 0.0f)) f = 0.0f;
    if (f > (float)(g - 1)) f = (float)(g - 1);
    return (int)f;
}

// Grid resolution for n boxes: about two boxes per cell.
SBMP_HD int grid_resolution(int n) {
    int g = 1;
    while (g < 256 && 2 * g * g < n) ++g;
    return g;
}

struct GridBox {   // host mirror of the float4 row: xmin, ymin, xmax, ymax
    float x, y, z, w;
};

// Free iff no listed box overlaps (minx, miny, maxx, maxy) under the reference
// predicate; Box is float4 (device) or GridBox (host).
template <class Box>
SBMP_HD bool grid_motion_valid(float minx, float miny, float maxx, float maxy, int g, float invW, float invH,
                               const int* start, const Box* boxes) {
    const int cx0 = grid_cell(minx, invW, g), cx1 = grid_cell(maxx, invW, g);
    const int cy0 = grid_cell(miny, invH, g), cy1 = grid_cell(maxy, invH, g);
    for (int cy = cy0; cy <= cy1; ++cy) {
        const int e = start[cy * g + cx1 + 1];
        for (int i = start[cy * g + cx0]; i < e; ++i) {
            const Box o = boxes[i];
            if (!((maxx <= o.x) || (o.z <= minx) || (maxy <= o.y) || (o.w <= miny))) return false;
        }
    }
    return true;
}

#if defined(__HIPCC__)
// Device form of grid_motion_valid with the same answer (an OR over the listed
// boxes, so the order of the tests does not matter): the start offsets of the
// segment's cell rows are loaded together, and the boxes of a row in groups of
// eight, all eight loads issued before any test, instead of one dependent global
// load per box with an early exit after each (a chain of L2 round trips per Euler
// step, which bounded the dense c5 field).
__device__ __forceinline__ bool grid_motion_valid_batched(float minx, float miny, float maxx, float maxy, int g,
                                                          float invW, float invH, const int* __restrict__ start,
                                                          const float4* __restrict__ boxes) {
    const int cx0 = grid_cell(minx, invW, g), cx1 = grid_cell(maxx, invW, g);
    const int cy0 = grid_cell(miny, invH, g), cy1 = grid_cell(maxy, invH, g);
    constexpr int kRows = 2;   // a step's segment spans one or two cell rows almost always
    constexpr int kBatch = 8;  // boxes loaded per round trip (a row of a few cells lists ~4-14 at c5's density)
    int b[kRows], e[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
        const int cy = min(cy0 + r, cy1);
        b[r] = start[cy * g + cx0];
        e[r] = start[cy * g + cx1 + 1];
        if (cy0 + r > cy1) e[r] = b[r];
    }
    bool hit = false;
    for (int cy = cy0; cy <= cy1 && !hit; cy += kRows) {
        if (cy > cy0) {   // rows beyond the first pair (a long segment): reload
#pragma unroll
            for (int r = 0; r < kRows; ++r) {
                const int c = min(cy + r, cy1);
                b[r] = start[c * g + cx0];
                e[r] = start[c * g + cx1 + 1];
                if (cy + r > cy1) e[r] = b[r];
            }
        }
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
            for (int i = b[r]; i < e[r] && !hit; i += kBatch) {
                const int last = e[r] - 1;
                float4 o[kBatch];
#pragma unroll
                for (int k = 0; k < kBatch; ++k) o[k] = boxes[min(i + k, last)];
                // a repeated last box (fewer than kBatch left in the row) is tested twice: same answer
#pragma unroll
                for (int k = 0; k < kBatch; ++k)
                    hit |= !((maxx <= o[k].x) || (o[k].z <= minx) || (maxy <= o[k].y) || (o[k].w <= miny));
            }
        }
    }
    return !hit;
}
#endif

}  // namespace sbmp
