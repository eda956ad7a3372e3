// cg_back.hip — the backend launch of batch frames (built with CG_BLOCK = 256, build.py).
//
// cg_launch_batch runs a detector batch as two launches on one stream: the front
// (cg_frame_kernel<..., FRONT = true>: pass 1, thresholds, pass 2, the survivors gathered into
// the frame's HBM scratch slot with a front record) and this one, one 256-lane workgroup per
// frame: the survivors ranked by point index into LDS, then the backend of cg_backend.h
// (VoxelGrid in PCL's order, Euclidean clustering, cluster order, CSR, centroids;
// src/cone_detection.cpp:206-279). Sized to share a CU with two streaming front workgroups:
// ~29 KB of LDS for up to CG_BACK_CAP points and at most 128 VGPRs (one wave per SIMD beside
// their four); a frame with more detector points runs the same backend on its HBM slot.
// all-pairs clustering up to 128 voxels here (its adjacency rows overlay KEY: 32 B per voxel);
// C3's frames have V <= 143, so nearly all of them take it
#define CG_BRUTE_V 128
#include "cg_backend.h"

// CG_BACK_CAP (cg_internal.h): C3's synthetic frames have M <= 413, 97.7% of them <= 384
static_assert(CG_BLOCK == 256, "cg_back.hip is built with CG_BLOCK=256 (build.py)");
static_assert(CG_BACK_CAP <= 2 * CG_BLOCK, "LDS backend capacity within pcl_block_sort<2>");
static_assert(backend_lds_fits<CG_BACK_CAP, (CG_BACK_CAP + 32) / 32>(), "backend overlays fit the LDS arrays");
typedef BackLdsT<CG_BACK_CAP> BackLdsB;
#define BACK_SMEM (FRONT_BYTES + sizeof(BackLdsB))
// two front workgroups (FRONT_BYTES + 64 KiB of codes each) and this one on a 160 KiB CU
static_assert(2 * (FRONT_BYTES + CG_MAX_POINTS) + BACK_SMEM <= 163840, "LDS: two fronts and one backend per CU");

__global__ __launch_bounds__(CG_BLOCK, 4) void cg_back_kernel(CgLaunch L, CgDevParams P) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[BACK_SMEM];
    const uint32_t f = blockIdx.x;
    const uint32_t* const rec = (const uint32_t*)(L.scratch + (uint64_t)f * L.scratch_stride + cg_work_bytes(L.n_points));
    // up to CG_BACK_CAP detector points in LDS here; up to CG_MMAX the front listed the frame
    // for cg_back_big (the frame kernel's LDS capacity); beyond, the backend on the frame's HBM
    // slot here (dense scenes only)
    const uint32_t M = rec[CG_FREC_M];
    if (M <= CG_BACK_CAP) back_frame<CG_BACK_CAP>(L, P, f, (FrontShared*)smem, (BackLdsB*)(smem + FRONT_BYTES));
    else if (M > CG_MMAX) back_frame<0>(L, P, f, (FrontShared*)smem, nullptr);
    if (L.span && threadIdx.x == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

int cg_launch_back(const CgLaunch& L, const CgDevParams& P, hipStream_t s) {
    hipLaunchKernelGGL(cg_back_kernel, dim3(L.n_frames), dim3(CG_BLOCK), 0, s, L, P);
    return hipGetLastError();
}

// Served batches (cg_debug_route 8): the batch's backend launch runs beside its front launch
// (another stream) instead of after it: workgroup f waits for frame f's publish word (the
// front's survivors and record are in the slot, written device-coherently), then runs
// back_frame on it: in LDS up to CG_BACK_CAP detector points, else on the frame's slot. So a
// frame's backend starts as soon as its own front ends, with no launch boundary in between,
// and no launch follows (a large-LDS follow-up launch would wait for CU room behind the fronts).
// Workgroups start in frame order, as the fronts do; the fronts never wait on them, and a
// waiting workgroup leaves room for two fronts on its CU (BACK_SMEM beside two front
// workgroups, like cg_back_kernel). Every wait is bounded (SERVE_TIMEOUT: then L.serve[2] is
// set and the frame skipped).
#define SERVE_TIMEOUT 100000000ull   // s_memrealtime ticks (100 MHz): 1 s
__global__ __launch_bounds__(CG_BLOCK, 4) void cg_serve_kernel(CgLaunch L, CgDevParams P) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[BACK_SMEM];
    __shared__ uint32_t late_s;
    uint32_t* const sv = L.serve;
    const uint32_t f = blockIdx.x, tid = threadIdx.x;
    if (tid == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t late = 0;
        while (ld_rlx(&sv[4 + f]) != L.epoch) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > SERVE_TIMEOUT) {
                late = 1;
                st_rlx(&sv[2], 1u);
                break;
            }
        }
        late_s = late;
    }
    __syncthreads();
    if (late_s) return;
    const uint32_t* const rec =
        (const uint32_t*)(L.scratch + (uint64_t)f * L.scratch_stride + cg_work_bytes(L.n_points));
    if (ld_rlx((uint32_t*)&rec[CG_FREC_M]) <= CG_BACK_CAP)
        back_frame<CG_BACK_CAP, true>(L, P, f, (FrontShared*)smem, (BackLdsB*)(smem + FRONT_BYTES));
    else   // more detector points: the backend on the frame's slot
        back_frame<0, true>(L, P, f, (FrontShared*)smem, nullptr);
    if (L.span && tid == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

int cg_launch_serve(const CgLaunch& L, const CgDevParams& P, hipStream_t s) {
    if (L.n_frames == 0 || !L.serve) return hipSuccess;
    hipLaunchKernelGGL(cg_serve_kernel, dim3(L.n_frames), dim3(CG_BLOCK), 0, s, L, P);
    return hipGetLastError();
}

// Pair batches (cg_pair.hip): the listed frames of more than CG_MMAX detector points, the
// backend on their HBM slots (cg_back_big then takes the listed frames up to CG_MMAX and clears
// the list).
#define BACK_LIST_GRID 32
// 32 workgroups: registers for 2 waves per SIMD, no spills
__global__ __launch_bounds__(CG_BLOCK, 2) void cg_back_list_kernel(CgLaunch L, CgDevParams P) {
    __shared__ FrontShared fs;
    const uint32_t* const list = L.biglist;
    const uint32_t n = __hip_atomic_load(&list[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma clang loop unroll(disable)
    for (uint32_t i = blockIdx.x; i < n; i += gridDim.x) {
        const uint32_t f = list[2 + i];
        const uint32_t* const rec = (const uint32_t*)(L.scratch + (uint64_t)f * L.scratch_stride + cg_work_bytes(L.n_points));
        if (rec[CG_FREC_M] <= CG_MMAX) continue;
        back_frame<0>(L, P, f, &fs, nullptr);
        __syncthreads();
    }
    if (L.span && threadIdx.x == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

int cg_launch_back_list(const CgLaunch& L, const CgDevParams& P, hipStream_t s) {
    hipLaunchKernelGGL(cg_back_list_kernel, dim3(BACK_LIST_GRID), dim3(CG_BLOCK), 0, s, L, P);
    return hipGetLastError();
}
