// cg_recrop.hip — cone re-crop, ConeDetector::get_reconstructed_cone (src/cone_detection.cpp:
// 222-238): for each cone centre, the points of the detector's whole input cloud inside an
// axis-aligned box of half-width 0.228f / 1.5 around it, in cloud order.
//
// The reference loops over the whole cloud once per cone (C x N box tests). Here one pass over
// the frame tests every point against every box (boxes in LDS), in two launches: count per
// (box, block), then write at the scanned offsets with a stable in-block order (k-major, then
// wave, then lane, which is point order). The double compares of the reference are exact float
// bounds (host, cg_api.cpp). For a fused pipeline call the whole cloud is the groundless cloud:
// a point belongs to it iff it is not ground, which is decided exactly (certified sector,
// threshold key) only for the few points that fall inside a box; the groundless cloud's zero
// pads are appended by the host.
#include "cg_device.h"

namespace {

constexpr int RC_LANES = 512;
constexpr int RC_WAVES = RC_LANES / 64;
constexpr int RC_PPT = 4;                       // points per lane per block

// cone_center.x + (CONE_WIDTH / 1.5) >= x && cone_center.x - (CONE_WIDTH / 1.5) <= x, same in y
// (src/cone_detection.cpp:228-229): exact as float bounds; NaN coordinates or bounds fail
__device__ __forceinline__ bool rc_in(const RcBox& b, const float4& p) {
    return (p.x >= b.lox) & (p.x <= b.hix) & (p.y >= b.loy) & (p.y <= b.hiy);
}

template <int LAYOUT, bool PIPE>
__device__ __forceinline__ bool rc_member(const CgLaunch& L, const CgDevParams& P, const uint32_t* tkey,
                                          const RcBox* box, uint32_t nb, uint32_t i, float4& p) {
    p = load_xyzi<LAYOUT>(L.in, i, L);
    bool any = false;
    for (uint32_t b = 0; b < nb; b++) any |= rc_in(box[b], p);
    if (!any) return false;
    if (PIPE) {   // in the groundless cloud iff !(z < T[sector]) (src/ground_removal.cpp:70-77)
        int s = 0;
        bool unused = false;
        classify_angle<true, false>(P, p.x, p.y, s, unused);
        if (cg_zkey(p.z) < tkey[s]) return false;
    }
    return true;
}

template <bool PIPE>
__device__ __forceinline__ void rc_setup(const CgDevParams& P, const uint32_t* seckeys, const RcBox* boxes,
                                         uint32_t nb, RcBox* sbox, uint32_t* tkey, float* thr, uint32_t* band) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t b = tid; b < nb; b += RC_LANES) sbox[b] = boxes[b];
    if (PIPE && tid < 64) sector_thresholds(seckeys, 0u, P, thr, tkey, &band[0], &band[1]);
    __syncthreads();
}

template <int LAYOUT, bool PIPE>
__global__ __launch_bounds__(RC_LANES) void rc_count(CgLaunch L, CgDevParams P, const uint32_t* seckeys,
                                                     const RcBox* boxes, uint32_t nb, uint32_t* cnt) {
    __shared__ RcBox sbox[CG_RECROP_MAX_BOXES];
    __shared__ uint32_t scnt[CG_RECROP_MAX_BOXES];
    __shared__ uint32_t tkey[CG_NUM_BINS + 1], band[2];
    __shared__ float thr[CG_NUM_BINS + 1];
    const uint32_t tid = threadIdx.x, l = lane_id();
    for (uint32_t b = tid; b < nb; b += RC_LANES) scnt[b] = 0;
    rc_setup<PIPE>(P, seckeys, boxes, nb, sbox, tkey, thr, band);
    const uint32_t N = L.n_points;
    for (int k = 0; k < RC_PPT; k++) {
        const uint32_t i = blockIdx.x * (RC_LANES * RC_PPT) + (uint32_t)k * RC_LANES + tid;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool v = i < N && rc_member<LAYOUT, PIPE>(L, P, tkey, sbox, nb, i, p);
        if (!__ballot(v)) continue;                            // wave-uniform
        for (uint32_t b = 0; b < nb; b++) {
            const uint64_t bal = __ballot(v && rc_in(sbox[b], p));
            if (l == 0 && bal) atomicAdd(&scnt[b], (uint32_t)__popcll(bal));
        }
    }
    __syncthreads();
    for (uint32_t b = tid; b < nb; b += RC_LANES) cnt[(uint64_t)b * gridDim.x + blockIdx.x] = scnt[b];
}

template <int LAYOUT, bool PIPE>
__global__ __launch_bounds__(RC_LANES) void rc_write(CgLaunch L, CgDevParams P, const uint32_t* seckeys,
                                                     const RcBox* boxes, uint32_t nb, const uint32_t* off,
                                                     float4* out) {
    __shared__ RcBox sbox[CG_RECROP_MAX_BOXES];
    __shared__ uint32_t run[CG_RECROP_MAX_BOXES];
    __shared__ uint32_t wcnt[CG_RECROP_MAX_BOXES * RC_WAVES];
    __shared__ uint32_t tkey[CG_NUM_BINS + 1], band[2];
    __shared__ float thr[CG_NUM_BINS + 1];
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    for (uint32_t b = tid; b < nb; b += RC_LANES) run[b] = off[(uint64_t)b * gridDim.x + blockIdx.x];
    rc_setup<PIPE>(P, seckeys, boxes, nb, sbox, tkey, thr, band);
    const uint32_t N = L.n_points;
    const uint64_t lt = (1ull << l) - 1ull;
    for (int k = 0; k < RC_PPT; k++) {
        const uint32_t i = blockIdx.x * (RC_LANES * RC_PPT) + (uint32_t)k * RC_LANES + tid;
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        const bool v = i < N && rc_member<LAYOUT, PIPE>(L, P, tkey, sbox, nb, i, p);
        const bool any = __syncthreads_or(v);                  // block-uniform
        if (!any) continue;
        for (uint32_t b = 0; b < nb; b++) {
            const uint64_t bal = __ballot(v && rc_in(sbox[b], p));
            if (l == 0) wcnt[b * RC_WAVES + w] = (uint32_t)__popcll(bal);
        }
        __syncthreads();
        for (uint32_t b = 0; b < nb; b++) {
            const bool in = v && rc_in(sbox[b], p);
            const uint64_t bal = __ballot(in);
            if (in) {
                uint32_t pre = run[b];
                for (uint32_t u = 0; u < w; u++) pre += wcnt[b * RC_WAVES + u];
                out[pre + (uint32_t)__popcll(bal & lt)] = p;
            }
        }
        __syncthreads();
        for (uint32_t b = tid; b < nb; b += RC_LANES) {
            uint32_t t = 0;
            for (uint32_t u = 0; u < RC_WAVES; u++) t += wcnt[b * RC_WAVES + u];
            run[b] += t;
        }
        __syncthreads();
    }
}

}  // namespace

uint32_t cg_recrop_blocks(uint32_t n_points) { return (n_points + RC_LANES * RC_PPT - 1) / (RC_LANES * RC_PPT); }

int cg_launch_recrop(const CgLaunch& L, const CgDevParams& P, bool pipeline, const uint32_t* d_seckeys,
                     const RcBox* d_boxes, uint32_t nb, uint32_t* d_cnt, const uint32_t* d_off, float4* d_out,
                     bool write, hipStream_t s) {
    const uint32_t nblk = cg_recrop_blocks(L.n_points);
    if (nblk == 0 || nb == 0) return hipSuccess;
    const bool xyzi16 = L.point_step == 16 && L.off_x == 0 && L.off_y == 4 && L.off_z == 8 && L.off_i == 12;
#define RC_GO(LAY, PIPE)                                                                                        \
    do {                                                                                                        \
        if (write)                                                                                              \
            hipLaunchKernelGGL((rc_write<LAY, PIPE>), dim3(nblk), dim3(RC_LANES), 0, s, L, P, d_seckeys, d_boxes, \
                               nb, d_off, d_out);                                                               \
        else                                                                                                    \
            hipLaunchKernelGGL((rc_count<LAY, PIPE>), dim3(nblk), dim3(RC_LANES), 0, s, L, P, d_seckeys, d_boxes, \
                               nb, d_cnt);                                                                      \
    } while (0)
    if (xyzi16) {
        if (pipeline) RC_GO(CG_LAYOUT_XYZI16, true); else RC_GO(CG_LAYOUT_XYZI16, false);
    } else {
        if (pipeline) RC_GO(CG_LAYOUT_GENERIC, true); else RC_GO(CG_LAYOUT_GENERIC, false);
    }
#undef RC_GO
    return hipGetLastError();
}
