// cg_grid.h — PCL VoxelGrid's lattice setup, shared by the device backend and the host-only
// halo plan (cg_host.cpp, built by hipcc and, for the host sanitizers, by g++).
#pragma once
#include <stdint.h>
#include <math.h>
#include "cg_internal.h"
#include "cg_math.h"

// bits needed for values below v (at least 1)
CG_HD uint32_t cg_bits_of(uint64_t v) { uint32_t b = 0; while (b < 64 && (1ull << b) <= v) b++; return b ? b : 1; }

// pcl::VoxelGrid::applyFilter setup (PCL 1.10, src/cone_detection.cpp:240-249) from the
// getMinMax3D bounds of the nfin finite points: the int64 overflow guard (pass = 1: output the
// input unchanged) and min_b / div_b of the idx computation.
CG_HD void voxel_grid_setup(uint32_t nfin, const float* bmn, const float* bmx,
                                                 const CgDevParams& P, uint32_t& pass, int* min_b,
                                                 int* div_b) {
    pass = 0;
    for (int a = 0; a < 3; a++) { min_b[a] = 0; div_b[a] = 1; }
    if (nfin == 0) return;
    double prod = 1.0;
    for (int a = 0; a < 3; a++) {
        const float span = (bmx[a] - bmn[a]) * P.inv_leaf[a];
        const double d = span >= 9.0e18f ? 9.0e18 : (double)((int64_t)span + 1);
        prod *= d;
    }
    if (prod > 2147483647.0) pass = 1;
    for (int a = 0; a < 3; a++) {
        min_b[a] = (int)floorf(bmn[a] * P.inv_leaf[a]);
        const int max_b = (int)floorf(bmx[a] * P.inv_leaf[a]);
        div_b[a] = max_b - min_b[a] + 1;
    }
}
