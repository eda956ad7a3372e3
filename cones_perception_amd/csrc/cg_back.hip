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

#ifndef CG_BACK_CAP
#define CG_BACK_CAP 392   // C3's synthetic frames: M <= 413, 97.7% of them <= 384
#endif
static_assert(CG_BLOCK == 256, "cg_back.hip is built with CG_BLOCK=256 (build.py)");
static_assert(CG_BACK_CAP <= 2 * CG_BLOCK, "LDS backend capacity within pcl_block_sort<2>");
static_assert(CG_BACK_CAP <= CG_RANK_SORT_MAX, "survivors ranked by one rank sort (no bitonic sort over KEY)");
static_assert(backend_lds_fits<CG_BACK_CAP, (CG_BACK_CAP + 32) / 32>(), "backend overlays fit the LDS arrays");
typedef BackLdsT<CG_BACK_CAP> BackLdsB;
#define BACK_SMEM (FRONT_BYTES + sizeof(BackLdsB))
// two front workgroups (FRONT_BYTES + 64 KiB of codes each) and this one on a 160 KiB CU
static_assert(2 * (FRONT_BYTES + CG_MAX_POINTS) + BACK_SMEM <= 163840, "LDS: two fronts and one backend per CU");

__global__ __launch_bounds__(CG_BLOCK, 4) void cg_back_kernel(CgLaunch L, CgDevParams P) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[BACK_SMEM];
    FrontShared* fs = (FrontShared*)smem;
    BackLdsB* bl = (BackLdsB*)(smem + FRONT_BYTES);
    const uint32_t f = blockIdx.x, tid = threadIdx.x, N = L.n_points;
    uint8_t* const slot = L.scratch + (uint64_t)f * L.scratch_stride;
    const uint32_t* const rec = (const uint32_t*)(slot + cg_work_bytes(N));
    const Work Wg = global_work(slot, N);
    const uint32_t Ms = rec[CG_FREC_MS], M = rec[CG_FREC_M];
    if (tid < 64) {
        uint32_t v = 0;
        if (tid == S_MS) v = Ms;
        else if (tid == S_MF) v = rec[CG_FREC_NFIN];
        else if (tid >= S_BMIN0 && tid <= S_BMIN2) v = rec[CG_FREC_BMIN + (tid - S_BMIN0)];
        else if (tid >= S_BMAX0 && tid <= S_BMAX2) v = rec[CG_FREC_BMAX + (tid - S_BMAX0)];
        fs->scal[tid] = v;
    }
    if (M <= CG_BACK_CAP) {
        // the front appended survivors in wave order; ranked by point index they take their
        // rank as point index, so index_vector (cloud order) and the point-order ties are the
        // frame kernel's, and pcl_index_vector's bitmap spans Ms bits
        const Work W = lds_work(bl);
        uint64_t* const tmp = (uint64_t*)W.VOX;   // free until pcl_index_vector
        for (uint32_t j = tid; j < Ms; j += CG_BLOCK) tmp[j] = ((uint64_t)Wg.IDX[j] << 16) | j;
        __syncthreads();
        rank_sort(tmp, W.KEY, Ms);
        for (uint32_t r = tid; r < Ms; r += CG_BLOCK) {
            W.P[r] = Wg.P[(uint32_t)(W.KEY[r] & 0xffffu)];
            W.IDX[r] = r;
        }
        for (uint32_t j = Ms + tid; j < M; j += CG_BLOCK) {   // PointXYZI() pads after every kept point
            W.P[j] = make_float4(0.f, 0.f, 0.f, 0.f);
            W.IDX[j] = 0xffffu;
        }
        __syncthreads();
        backend(W, M, fs, L, P, f, 0u, (Ms + 32) / 32, CG_BACK_CAP);
    } else {
        __syncthreads();
        backend(Wg, M, fs, L, P, f, 0x2u, CG_MAX_POINTS / 32, 0);
    }
    if (L.span && tid == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

int cg_launch_back(const CgLaunch& L, const CgDevParams& P, hipStream_t s) {
    hipLaunchKernelGGL(cg_back_kernel, dim3(L.n_frames), dim3(CG_BLOCK), 0, s, L, P);
    return hipGetLastError();
}
