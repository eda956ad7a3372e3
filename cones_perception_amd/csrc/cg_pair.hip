// cg_pair.hip — batch frames as pairs of half-frame workgroups (built with CG_BLOCK = 256).
//
// The fused frame kernel (cg_kernels.hip) holds a frame's 64 KiB of z codes in LDS, so two
// 8-wave workgroups share a CU, and whenever both are in their latency-bound tail (pass 2,
// gather, backend) the CU streams nothing. Here a frame is two 4-wave workgroups, one per
// half (32,768 points, 32 KiB of codes): four of them share a CU (~37 KB of LDS each, <= 128
// VGPRs), and a frame's tail occupies one of the four slots while the other three stream.
//  - both halves run pass 1 (cg_device.h stream_pass1) on their points, codes in LDS;
//  - each swaps the batch's epoch into the frame's ticket word. The first publishes its sector keys,
//    used bins, codes and filter bits into the frame's scratch slot with device-coherent
//    stores, then a ready word (the batch's epoch), and exits;
//  - the second waits for that word (its partner is running: it took the first ticket), merges
//    the sector keys, runs the thresholds and pass 2 over both halves (its own codes from LDS,
//    the partner's from the slot), the compaction and gather of both halves' survivors, and the
//    backend (cg_backend.h) on them in LDS for up to PAIR_CAP detector points, ranked by point
//    index (index_vector's cloud order). A frame with more keeps its survivors in its HBM slot
//    with a front record and is listed for the two launches after this one (cg_back.hip
//    cg_back_list_kernel past CG_MMAX, cg_kernels.hip cg_back_big_kernel up to it); C3's
//    synthetic frames have M <= 413.
// The two halves of frame f are workgroups 16 (f / 8) + f % 8 and that + 8: the same XCD, so
// the partner's data is one L2 away. Results are bit-identical to the fused kernel's.
#define CG_BRUTE_V 128   // all-pairs clustering up to 128 voxels (adjacency rows overlay KEY)
#include "cg_backend.h"

#define PAIR_HALF (CG_MAX_POINTS / 2)      // points per workgroup
#define PAIR_PPT (PAIR_HALF / CG_BLOCK)    // points per lane
#define PAIR_CAP 512                       // the LDS backend's capacity (detector points)
#define PAIR_TIMEOUT 10000000ull           // s_memrealtime ticks (100 MHz): 100 ms
static_assert(CG_BLOCK == 256, "cg_pair.hip is built with CG_BLOCK=256 (build.py)");
static_assert(PAIR_PPT == 128, "two 64-point bit words per lane");
static_assert(PAIR_CAP <= CG_RANK_SORT_MAX && PAIR_CAP <= 2 * CG_BLOCK, "one rank sort, pcl_block_sort<2>");
static_assert(backend_lds_fits<PAIR_CAP, (PAIR_CAP + 32) / 32>(), "backend overlays fit the LDS arrays");
typedef BackLdsT<PAIR_CAP> BackLdsP;
constexpr size_t PAIR_BODY = sizeof(BackLdsP) > (size_t)PAIR_HALF ? sizeof(BackLdsP) : (size_t)PAIR_HALF;
#define PAIR_SMEM (FRONT_BYTES + PAIR_BODY)
static_assert(4 * PAIR_SMEM <= 163840, "four pair workgroups per CU");
// the exchange area: the last CG_PAIR_X_BYTES of the frame's scratch slot
static_assert(CG_PAIR_X_BYTES >= 128 + PAIR_HALF + 2 * CG_BLOCK * 8 && CG_PAIR_X_BYTES % 256 == 0, "exchange area");

template <int LAYOUT>
__global__ __launch_bounds__(CG_BLOCK, 4) void cg_pair_kernel(CgLaunch L, CgDevParams P) {
    constexpr int PPT = PAIR_PPT, NW = PPT / 64;
    __shared__ __attribute__((aligned(16))) unsigned char smem[PAIR_SMEM];
    FrontShared* fs = (FrontShared*)smem;
    BackLdsP* bl = (BackLdsP*)(smem + FRONT_BYTES);
    uint2* const zq = (uint2*)(smem + FRONT_BYTES);   // the half's codes, [group][lane]
    const uint32_t id = blockIdx.x, tid = threadIdx.x, l = lane_id();
    const uint32_t f = (id >> 4) * 8 + (id & 7), h = (id >> 3) & 1u;
    if (f >= L.n_frames) return;
    const uint32_t N = L.n_points;
    const uint8_t* const fb = L.in + (uint64_t)f * L.frame_stride;
    const uint32_t h0 = h * PAIR_HALF, o0 = (h ^ 1u) * PAIR_HALF;
    const uint32_t Nh = N > h0 ? min((uint32_t)PAIR_HALF, N - h0) : 0u;
    const uint32_t No = N > o0 ? min((uint32_t)PAIR_HALF, N - o0) : 0u;
    uint8_t* const slot = L.scratch + (uint64_t)f * L.scratch_stride;
    uint8_t* const xb = slot + L.scratch_stride - CG_PAIR_X_BYTES;   // the slot's tail (cg_scratch_bytes)
    uint32_t* const xh = (uint32_t*)xb;                 // [0] tickets, [1] ready, [2] used bins, [4, 22) keys
    uint64_t* const xcodes = (uint64_t*)(xb + 128);     // [group][lane], PPT / 8 groups
    uint64_t* const xposm = xcodes + PAIR_HALF / 8;     // [word][lane]
    if (L.span && tid == 0) atomicMin(&L.span[0], (unsigned long long)__builtin_amdgcn_s_memrealtime());

    if (tid <= CG_NUM_BINS) fs->sec_key[tid] = cg_fkey(P.default_low);
    init_rays<true>(P, fs->rays, tid);
    if (tid < 64) fs->scal[tid] = (tid >= S_BMIN0 && tid <= S_BMIN2) ? 0xffffffffu : 0u;
    __syncthreads();

    // ---- pass 1 over this half ----
    LaneBits<NW> posm;
    uint32_t touched = 0;
    {
        const uint8_t* const hb = fb + (uint64_t)h0 * L.point_step;
        auto store = [&](int g, uint2 c) { zq[g * CG_BLOCK + tid] = c; };
        if (LAYOUT == CG_LAYOUT_XYZI16 && Nh == (uint32_t)PAIR_HALF)
            stream_pass1<PPT, LAYOUT, true, true, decltype(store), true>(hb, Nh, L, P, fs->sec_key, fs->rays, posm,
                                                                         touched, store);
        else
            stream_pass1<PPT, LAYOUT, true, true>(hb, Nh, L, P, fs->sec_key, fs->rays, posm, touched, store);
    }
    touched = wave_or(touched);
    if (l == 0 && touched) atomicOr(&fs->scal[S_TOUCHED], touched);
    __syncthreads();   // the half's sector keys, used bins and codes are final in LDS
    // the ticket: the first half to swap this batch's epoch in sees an older one (the words
    // start zeroed; epochs count from 1), the second sees its own
    if (tid == 0)
        fs->scal[S_TMP] = __hip_atomic_exchange(&xh[0], L.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != L.epoch;
    __syncthreads();
    if (fs->scal[S_TMP]) {
        // the first half done: its data for the partner (device-coherent: no L2 writeback),
        // every store complete before the ready word
#pragma unroll
        for (int g = 0; g < PPT / 8; g++) {
            const uint2 c = zq[g * CG_BLOCK + tid];
            st64(&xcodes[g * CG_BLOCK + tid], ((uint64_t)c.y << 32) | c.x);
        }
#pragma unroll
        for (int i = 0; i < NW; i++) st64(&xposm[i * CG_BLOCK + tid], posm.w[i]);
        if (tid <= CG_NUM_BINS) st_rlx(&xh[4 + tid], fs->sec_key[tid]);
        if (tid == 0) st_rlx(&xh[2], fs->scal[S_TOUCHED]);
        __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
        __syncthreads();
        if (tid == 0) {
            st_rlx(&xh[1], L.epoch);
            if (L.span) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
        }
        return;
    }
    // ---- the second half done: the frame's tail ----
    if (tid == 0) {
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        uint32_t late = 0;
        while (ld_rlx(&xh[1]) != L.epoch) {   // the partner holds the first ticket: it is running
            __builtin_amdgcn_s_sleep(1);
            if (__builtin_amdgcn_s_memrealtime() - t0 > PAIR_TIMEOUT) {
                late = CG_F_PAIR_TIMEOUT;     // never expected; reported in the frame's flags
                break;
            }
        }
        fs->scal[S_LAST] = late;
    }
    __syncthreads();
    const uint32_t late = fs->scal[S_LAST];
    // the partner's codes and filter bits into registers now: one round of device-coherent
    // loads in flight behind the thresholds and this half's pass 2
    uint64_t oc[PPT / 8];
    LaneBits<NW> posm_o;
#pragma unroll
    for (int g = 0; g < PPT / 8; g++) oc[g] = ld64(&xcodes[g * CG_BLOCK + tid]);
#pragma unroll
    for (int i = 0; i < NW; i++) posm_o.w[i] = ld64(&xposm[i * CG_BLOCK + tid]);
    if (tid <= CG_NUM_BINS) fs->sec_key[tid] = min(fs->sec_key[tid], ld_rlx(&xh[4 + tid]));
    if (tid == 0) fs->scal[S_TOUCHED] |= ld_rlx(&xh[2]);
    __syncthreads();
    if (tid < 64) {
        sector_thresholds(fs->sec_key, fs->scal[S_TOUCHED], P, fs->thr, fs->tkey, &fs->scal[S_TKMIN], &fs->scal[S_TKMAX]);
        if (L.seckeys && tid <= CG_NUM_BINS) L.seckeys[(uint64_t)f * (CG_NUM_BINS + 1) + tid] = fs->sec_key[tid];
    }
    __syncthreads();

    // ---- pass 2 over both halves (the partner's codes and filter bits from the slot) ----
    const uint32_t qlo = fs->scal[S_TKMIN], qhi = fs->scal[S_TKMAX];
    LaneBits<NW> keep_h, keep_o;
    pass2_keep<PPT, LAYOUT>(fb + (uint64_t)h0 * L.point_step, Nh, L, P, qlo, qhi, fs->tkey,
                            [&](int g) { return zq[g * CG_BLOCK + tid]; }, keep_h);
    pass2_keep<PPT, LAYOUT>(fb + (uint64_t)o0 * L.point_step, No, L, P, qlo, qhi, fs->tkey,
                            [&](int g) { return make_uint2((uint32_t)oc[g], (uint32_t)(oc[g] >> 32)); }, keep_o);
    {
        const uint32_t kc = wave_sum(keep_h.count() + keep_o.count());
        if (l == 0) atomicAdd(&fs->scal[S_K], kc);
    }
    // ---- compaction (per-wave atomic append; the survivors carry their point index) ----
#pragma unroll
    for (int i = 0; i < NW; i++) {
        keep_h.w[i] &= posm.w[i];
        keep_o.w[i] &= posm_o.w[i];
    }
    const uint32_t nsv = keep_h.count() + keep_o.count();
    const uint32_t incl = wave_incl_scan(nsv);
    uint32_t wbase = 0;
    if (l == 63) wbase = atomicAdd(&fs->scal[S_MS], incl);
    wbase = (uint32_t)__builtin_amdgcn_readlane((int)wbase, 63);
    uint32_t pos = wbase + incl - nsv;
    __syncthreads();   // counts complete; the codes in LDS are dead from here on
    const uint32_t Ms = fs->scal[S_MS], K = fs->scal[S_K];
    const uint32_t npad = P.zero_pass ? N - K : 0u;   // the groundless cloud's PointXYZI() pads
    const uint32_t M = Ms + npad;
    const bool use_lds = M <= PAIR_CAP;
    if (tid == 0) {
        uint32_t* hd = L.hdr + (uint64_t)f * 8;
        hd[0] = N;
        hd[1] = K;
    }
    const Work Wl = lds_work(bl);
    const Work Wg = global_work(slot, N);
    // LDS: survivors staged in VOX / ORD, ranked below; HBM: straight into the slot's P / IDX
    float4* const gp = use_lds ? Wl.VOX : Wg.P;
    uint32_t* const gi = use_lds ? Wl.ORD : Wg.IDX;
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t nfin = 0;
    auto bound = [&](const float4& p) {
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
            mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
            nfin++;
        }
    };
    auto gather = [&](const LaneBits<NW>& km, uint32_t base) {
#pragma unroll
        for (int wi = 0; wi < NW; wi++) {
            uint64_t m = km.w[wi];
            while (m) {
                int ks[4];
                float4 pt[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    ks[q] = m ? __builtin_ctzll(m) : -1;
                    if (m) m &= m - 1;
                }
#pragma unroll
                for (int q = 0; q < 4; q++)
                    if (ks[q] >= 0) pt[q] = load_xyzi<LAYOUT>(fb, base + (uint32_t)(64 * wi + ks[q]) * CG_BLOCK + tid, L);
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    if (ks[q] < 0) continue;
                    gp[pos] = pt[q];
                    gi[pos] = base + (uint32_t)(64 * wi + ks[q]) * CG_BLOCK + tid;   // point index in the frame
                    bound(pt[q]);
                    pos++;
                }
            }
        }
    };
    gather(keep_h, h0);
    gather(keep_o, o0);
    for (uint32_t j = tid; j < npad; j += CG_BLOCK) {
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        gp[Ms + j] = z4;
        gi[Ms + j] = 0xffffu;   // after every kept point
        bound(z4);
    }
    {
        float r[6];
#pragma unroll
        for (int a = 0; a < 3; a++) { r[a] = wave_min(mn[a]); r[3 + a] = wave_max(mx[a]); }
        const uint32_t nf = wave_sum(nfin);
        if (l == 0 && nf) {
#pragma unroll
            for (int a = 0; a < 3; a++) {
                atomicMin(&fs->scal[S_BMIN0 + a], cg_fkey(r[a]));
                atomicMax(&fs->scal[S_BMAX0 + a], cg_fkey(r[3 + a]));
            }
            atomicAdd(&fs->scal[S_MF], nf);
        }
    }
    __syncthreads();
    if (use_lds) {
        // ranked by point index: the rank becomes the point index (pcl_index_vector's bitmap
        // spans Ms bits), so index_vector's cloud order and the point-order ties are the fused
        // kernel's
        uint64_t* const tmp = (uint64_t*)Wl.P;   // free until the ranked copy below
        for (uint32_t j = tid; j < Ms; j += CG_BLOCK) tmp[j] = ((uint64_t)Wl.ORD[j] << 16) | j;
        __syncthreads();
        rank_sort(tmp, Wl.KEY, Ms);
        for (uint32_t r = tid; r < Ms; r += CG_BLOCK) {
            Wl.P[r] = Wl.VOX[(uint32_t)(Wl.KEY[r] & 0xffffu)];
            Wl.IDX[r] = r;
        }
        for (uint32_t j = Ms + tid; j < M; j += CG_BLOCK) {
            Wl.P[j] = Wl.VOX[j];
            Wl.IDX[j] = 0xffffu;
        }
        __syncthreads();
        backend(Wl, M, fs, L, P, f, late, (Ms + 32) / 32, PAIR_CAP);
    } else if (tid == 0) {
        // the survivors are in the slot: the front record, and the frame listed for the launches
        // after this one (cg_back_list_kernel: HBM backend past CG_MMAX; cg_back_big_kernel: LDS)
        uint32_t* const rec = (uint32_t*)(slot + cg_work_bytes(N));
        rec[CG_FREC_MS] = Ms;
        rec[CG_FREC_M] = M;
        rec[CG_FREC_NFIN] = fs->scal[S_MF];
#pragma unroll
        for (int a = 0; a < 3; a++) {
            rec[CG_FREC_BMIN + a] = fs->scal[S_BMIN0 + a];
            rec[CG_FREC_BMAX + a] = fs->scal[S_BMAX0 + a];
        }
        const uint32_t q = atomicAdd(&L.biglist[0], 1u);
        L.biglist[2 + q] = f;
    }
    if (L.span && tid == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// Pipeline batches of frames of <= CG_MAX_POINTS points; the grid covers frames in groups of 8.
int cg_launch_pair(const CgLaunch& L, const CgDevParams& P, hipStream_t s) {
    if (L.n_frames == 0) return hipSuccess;
    const dim3 grid(16 * ((L.n_frames + 7) / 8)), block(CG_BLOCK);
    const bool xyzi16 = L.point_step == 16 && L.off_x == 0 && L.off_y == 4 && L.off_z == 8 && L.off_i == 12;
    if (xyzi16) hipLaunchKernelGGL(cg_pair_kernel<CG_LAYOUT_XYZI16>, grid, block, 0, s, L, P);
    else hipLaunchKernelGGL(cg_pair_kernel<CG_LAYOUT_GENERIC>, grid, block, 0, s, L, P);
    if (hipError_t e = hipGetLastError()) return e;
#ifdef CG_PAIR_NO_FOLLOWUP   // (experiment: what the two listed-frame launches cost; C3 lists none)
    return hipSuccess;
#endif
    if (int e = cg_launch_back_list(L, P, s)) return e;
    return cg_launch_back_big(L, P, s);
}
