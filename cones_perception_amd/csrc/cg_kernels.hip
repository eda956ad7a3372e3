// cg_kernels.hip — gfx950 kernels for the LiDAR cone-detection hot path.
//
// One 512-lane workgroup (8 waves) owns one frame end to end, two workgroups per CU; a batch
// launch is a grid of n_frames workgroups (a single frame: cg_launch_split, below). Per frame:
//
//  frontend (HBM-streaming, ~all of the frame's bytes)
//    pass 1  coalesced point loads (lane t handles points k*512 + t, up to 128 per lane),
//            certified 22-degree sector (glibc-exact atan2f only near an edge), position-filter
//            bits in registers, z kept as an 8-bit monotone code in LDS (64 KiB, overlaying the
//            backend arrays); per-lane sector minimum flushed into 17 LDS bins with ds_min_u32
//            on order-preserving keys                 (src/ground_removal.cpp:58-68)
//    pass 2  sector thresholds; ground decisions from the codes against the band of used
//            thresholds (band codes are ambiguous)  (src/ground_removal.cpp:70-77, and
//                                                        src/cone_detection.cpp:189-204)
//    gather  one round of loads: the kept filter survivors and the ambiguous points (decided
//            exactly from the loaded x, y, z); per-wave atomic append of the survivors (x, y,
//            z, intensity, point index) into LDS (M <= CG_MMAX) or the frame's HBM scratch
//  backend (latency-bound; M ~ 1e2-1e3 points)
//    voxel   bounds, PCL idx key, std::sort's permutation of PCL's index_vector (cg_pcl.h; or a
//            rank sort in point order), run heads, centroid sums in that order
//                                                       (pcl::VoxelGrid, src/cone_detection.cpp:240-249)
//    cluster all pairs (V <= CG_BRUTE_V) or a neighbour grid (cell >= tolerance), exact float
//            L2_Simple predicate, lock-free union-find hooking larger roots under smaller
//            ones so a component's root is its lowest voxel index = PCL's seed
//                                                       (KdTree + ECE, src/cone_detection.cpp:206-220)
//    order   size filter, PCL's std::sort(rbegin, rend) order (restated, cg_sort.h),
//            counting sort into CSR, per-cluster centroid + radial push
//                                                       (src/cone_detection.cpp:261-279)
//
// Compiled with -ffp-contract=off: every float/double expression must round like the
// reference's non-FMA x86-64 build.
#include <hip/hip_runtime.h>
#include "cg_internal.h"
#include "../../include/cones_gpu.h"
#include "cg_math.h"
#include "cg_sort.h"
#include "cg_device.h"
#include "cg_pcl.h"

#include "cg_backend.h"

typedef BackLdsT<CG_MMAX> BackLds;
#define SMEM_BYTES (FRONT_BYTES + sizeof(BackLds))
static_assert(SMEM_BYTES <= 163840, "LDS budget");
// pcl_index_vector keeps a 2,048-word point bitmap and its 2,048-word prefix in VOX; the other
// overlays (cg_backend.h backend_lds_fits)
static_assert(backend_lds_fits<CG_MMAX, CG_MAX_POINTS / 32>(), "backend overlays fit the LDS arrays");
// the LDS PCL sort (pcl_sort<2, true>) covers at most two records per thread
static_assert(CG_MMAX <= 2 * CG_BLOCK, "LDS backend capacity within pcl_block_sort<2>");
static_assert(sizeof(BackLds) >= CG_MAX_POINTS * sizeof(uint8_t), "z-code overlay must fit");
// the ground-only mode's per-(k, wave) counts overlay the z codes once pass 2 is done
static_assert(CG_MAX_POINTS / 64 * sizeof(uint32_t) <= CG_MAX_POINTS, "ground counts fit the code area");

uint64_t cg_scratch_bytes(uint32_t n) { return cg_work_bytes(n); }

// ------------------------------------------------------------------------------------------
// Fused per-frame kernel: one 512-lane workgroup per frame, two workgroups per CU (launch
// bounds: 4 waves per SIMD, so <= 128 VGPRs) so that one
// frame's latency-bound backend overlaps another frame's HBM streaming. PPT points per lane;
// lane t owns points k*512 + t.
//
// z of every point stays on chip for the ground decision as an 8-bit monotone code (64 KiB at
// 64k points, overlaying the backend arrays). Pass 2 decides `z < T[s]` against the band
// [min_s T[s], max_s T[s]] of the used sector thresholds, so it needs no per-point sector:
// a code below q(min T) is ground in every sector, one above q(max T) is kept in every sector.
// Only points whose code equals a band code re-read x, y, z from HBM and recompute their
// sector (tens of points per frame on flat ground: the code step is 1/64 m).
__device__ __forceinline__ void pack_frame(const CgLaunch& L, uint32_t f, uint32_t* out);
//
// SPLIT (single frames, cg_launch_split): pass 1 runs in one workgroup per 4,096-point chunk
// (a frame alone on the GPU is VALU-bound on one CU), each writing its z codes and filter
// bits to HBM and merging its sector minima into the frame's keys with atomics; the last
// workgroup to finish (release/acquire on a counter) continues with the frame's thresholds,
// pass 2 and backend below, codes and bits read back from L2.
template <int PPT, int LAYOUT, int KMODE, bool SPLIT = false>
__device__ __forceinline__ void frame_body(const CgLaunch& L, const CgDevParams& P) {
    constexpr int G = 8;                          // points per load group (double-buffered)
    constexpr int NW = (PPT + 63) / 64;
    static_assert(PPT % (2 * G) == 0, "PPT must be a multiple of two load groups");
    constexpr bool GROUND = KMODE != CG_KMODE_DETECT;
    constexpr bool FILTER = KMODE != CG_KMODE_GROUND;
    // a split launch's 16 workgroups take a CU each: LDS past half a CU says so to the compiler,
    // which then sizes registers for 2 waves per SIMD (no SGPR spill reaches scratch)
    constexpr size_t SMEM = SPLIT && SMEM_BYTES <= 81920 ? 81920 + 256 : SMEM_BYTES;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM];
    FrontShared* fs = (FrontShared*)smem;
    BackLds* bl = (BackLds*)(smem + FRONT_BYTES);
    uint8_t* zq = (uint8_t*)bl;                   // z codes, [k/8][lane][k%8]

    const uint32_t f = SPLIT ? 0u : blockIdx.x, tid = threadIdx.x, l = lane_id(), w = wave_id();
    const uint8_t* fb = L.in + (uint64_t)f * L.frame_stride;
    const uint32_t N = L.n_points;
    STAMP(0);
    // launch spans (cg_debug_launch_spans, CG_SPAN_WORDS per launch): the first workgroup's
    // start, the last one's end, and every workgroup's shader cycles and real time, whose ratio
    // is the clock the CUs held (s_memtime counts shader cycles, s_memrealtime 100 MHz ticks)
    uint64_t span_c0 = 0, span_r0 = 0;
    if (L.span && tid == 0) {
        span_r0 = __builtin_amdgcn_s_memrealtime();
        span_c0 = __builtin_amdgcn_s_memtime();
        atomicMin(&L.span[0], (unsigned long long)span_r0);
    }

    if (tid <= CG_NUM_BINS) fs->sec_key[tid] = cg_fkey(P.default_low);
    init_rays<FILTER>(P, fs->rays, tid);
    if (tid < 64) fs->scal[tid] = (tid >= S_BMIN0 && tid <= S_BMIN2) ? 0xffffffffu : 0u;
    __syncthreads();

    // ---- pass 1: stream the frame ----
    LaneBits<NW> posm;
    uint32_t touched = 0;
    if constexpr (SPLIT) {
        static_assert(PPT * CG_BLOCK == CG_MAX_POINTS, "split frames use the 64k tail");
        static_assert(CG_SPLIT_CHUNK == 8 * CG_BLOCK, "a chunk's codes are one uint2 and its bits one byte per lane");
        const uint32_t c = blockIdx.x, c0 = c * CG_SPLIT_CHUNK;
        const uint32_t Nc = N > c0 ? min((uint32_t)CG_SPLIT_CHUNK, N - c0) : 0u;
        if (L.in_host) {   // the chunk over PCIe from pinned host memory into the device copy
            if (L.in_flags) {   // the host publishes the chunk after the launch (run_single)
                if (tid == 0) {
                    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
                    while (__hip_atomic_load(&L.in_flags[c], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != L.in_seq) {
                        __builtin_amdgcn_s_sleep(2);
                        if (__builtin_amdgcn_s_memrealtime() - t0 > CG_STAGE_TIMEOUT) {
                            __hip_atomic_store(&L.in_flags[CG_STAGE_ERR], L.in_seq, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_SYSTEM);
                            // in host memory before this chunk arrives (so before the done word)
                            __builtin_amdgcn_s_waitcnt(0x0070);
                            break;
                        }
                    }
                }
                __syncthreads();
            }
            STAMP(27);   // the chunk is published
            const uint64_t b0 = (uint64_t)c0 * L.point_step, nb = (uint64_t)Nc * L.point_step;
            uint8_t* dst = (uint8_t*)L.in + b0;
            const uint8_t* src = L.in_host + b0;
            const uint64_t n16 = nb / 16;
            // four 16-byte reads in flight per lane; named registers (an array with
            // conditional elements was kept in scratch)
            // The device copy is written device-coherently (the last workgroup, on any XCD,
            // re-reads survivors from it): the hand-off below then needs no L2 writeback
            const uint4* s4 = (const uint4*)src;
            uint64_t* d8 = (uint64_t*)dst;
            auto put16 = [&](uint64_t i, const uint4& v) {
                st64(d8 + 2 * i, ((uint64_t)v.y << 32) | v.x);
                st64(d8 + 2 * i + 1, ((uint64_t)v.w << 32) | v.z);
            };
            for (uint64_t i = tid; i < n16; i += CG_BLOCK * 4) {
                const uint64_t i1 = i + CG_BLOCK, i2 = i + 2 * CG_BLOCK, i3 = i + 3 * CG_BLOCK;
                const uint4 v0 = s4[i];
                const uint4 v1 = s4[i1 < n16 ? i1 : i];
                const uint4 v2 = s4[i2 < n16 ? i2 : i];
                const uint4 v3 = s4[i3 < n16 ? i3 : i];
                put16(i, v0);
                if (i1 < n16) put16(i1, v1);
                if (i2 < n16) put16(i2, v2);
                if (i3 < n16) put16(i3, v3);
            }
            for (uint64_t i = n16 * 16 + 4 * (uint64_t)tid; i < nb; i += 4 * CG_BLOCK)
                st_rlx((uint32_t*)(dst + i), *(const uint32_t*)(src + i));
            __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0): this lane's stores are done
            __syncthreads();
            STAMP(28);   // the chunk is on the device
        }
        LaneBits<1> pm;
        uint2 code = make_uint2(0u, 0u);
        stream_pass1<CG_SPLIT_CHUNK / CG_BLOCK, LAYOUT, GROUND, FILTER>(
            fb + (uint64_t)c0 * L.point_step, Nc, L, P, fs->sec_key, fs->rays, pm, touched,
            [&](int, uint2 cw) { code = cw; });
        // Every chunk decides its own points once all the frame's sector minima are merged: the
        // chunks publish their minima (atomics), count themselves (a relaxed count after their
        // atomics completed) and wait for the count; then each takes the thresholds from the
        // merged keys, runs pass 2 on its own codes (still in registers) and appends its
        // survivors, K and bounds to the frame's state with device-coherent stores and atomics.
        // The last chunk to count itself done gathers the survivors and runs the backend. No
        // release / acquire fences (their L2 writeback and invalidate cost ~5 us per workgroup);
        // every cross-workgroup word is an atomic or an sc1 (device-coherent) access.
        if (GROUND) {
            touched = wave_or(touched);
            if (l == 0 && touched) atomicOr(L.split + SP_TOUCHED, touched);
        }
        __syncthreads();   // the chunk's sector minima are final in LDS
        STAMP(29);
        if (GROUND && tid <= CG_NUM_BINS) atomicMin(L.split + SP_KEYS + tid, fs->sec_key[tid]);
        __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
        __syncthreads();
        if (tid == 0) {
            __hip_atomic_fetch_add(L.split + SP_ARRIVE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // bounded: all chunk workgroups are running unless other work holds the CUs; past
            // the bound the frame is flagged and the host runs it again in one workgroup
            const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
            uint32_t ok = 1;
            if (L.split_give_up && blockIdx.x == 0) {
                st_rlx(L.split + SP_ERR, 1u);
                ok = 0;
            }
            while (ok && ld_rlx(L.split + SP_ARRIVE) < gridDim.x) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t0 > CG_SPLIT_TIMEOUT) {
                    st_rlx(L.split + SP_ERR, 1u);
                    ok = 0;
                    break;
                }
            }
            fs->scal[S_LAST] = ok;
        }
        __syncthreads();
        STAMP(30);
        if (fs->scal[S_LAST]) {
            if (GROUND && tid <= CG_NUM_BINS) fs->sec_key[tid] = ld_rlx(L.split + SP_KEYS + tid);
            if (tid == 0) fs->scal[S_TOUCHED] = GROUND ? ld_rlx(L.split + SP_TOUCHED) : 0u;
            __syncthreads();
            if (GROUND && tid < 64)
                sector_thresholds(fs->sec_key, fs->scal[S_TOUCHED], P, fs->thr, fs->tkey, &fs->scal[S_TKMIN],
                                  &fs->scal[S_TKMAX]);
            __syncthreads();
            LaneBits<1> kp, am;
            if (GROUND) {
                pass2_codes<8>(Nc, fs->scal[S_TKMIN], fs->scal[S_TKMAX], [&](int) { return code; }, kp, am);
            } else {
                kp.clear();
                am.clear();
#pragma unroll
                for (int k = 0; k < 8; k++)
                    if ((uint32_t)k * CG_BLOCK + tid < Nc) kp.w[0] |= 1ull << k;
            }
            // the lane's points to load (at most 8): kept filter survivors and ambiguous points
            const uint32_t todo = (uint32_t)((kp.w[0] & pm.w[0]) | am.w[0]);
            float4 pt[8];
#pragma unroll
            for (int k = 0; k < 8; k++)
                if ((todo >> k) & 1u) pt[k] = load_xyzi<LAYOUT>(fb, c0 + (uint32_t)k * CG_BLOCK + tid, L);
            uint32_t sv = 0, kamb = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (!((todo >> k) & 1u)) continue;
                bool kept = true;
                if (GROUND && ((am.w[0] >> k) & 1ull)) {
                    kept = pass2_exact(P, fs->tkey, pt[k].x, pt[k].y, pt[k].z);
                    kamb += kept ? 1u : 0u;
                }
                if (kept && ((pm.w[0] >> k) & 1ull)) sv |= 1u << k;
            }
            const uint32_t ns = (uint32_t)__builtin_popcount(sv);
            const uint32_t incl = wave_incl_scan(ns);
            uint32_t wbase = 0;
            if (l == 63 && incl) wbase = __hip_atomic_fetch_add(L.split + SP_MS, incl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            wbase = (uint32_t)__builtin_amdgcn_readlane((int)wbase, 63);
            uint32_t pos = wbase + incl - ns;
            float4* const sp_p = (float4*)(L.split + SP_SURV);
            uint32_t* const sp_i = L.split + SP_SURV + 4 * CG_MAX_POINTS;
            float bmn[3] = {INFINITY, INFINITY, INFINITY}, bmx[3] = {-INFINITY, -INFINITY, -INFINITY};
            uint32_t nf = 0;
#pragma unroll
            for (int k = 0; k < 8; k++) {
                if (!((sv >> k) & 1u)) continue;
                st_f4(&sp_p[pos], pt[k]);
                st_rlx(&sp_i[pos], c0 + (uint32_t)k * CG_BLOCK + tid);
                pos++;
                if (isfinite(pt[k].x) && isfinite(pt[k].y) && isfinite(pt[k].z)) {
                    bmn[0] = fminf(bmn[0], pt[k].x); bmn[1] = fminf(bmn[1], pt[k].y); bmn[2] = fminf(bmn[2], pt[k].z);
                    bmx[0] = fmaxf(bmx[0], pt[k].x); bmx[1] = fmaxf(bmx[1], pt[k].y); bmx[2] = fmaxf(bmx[2], pt[k].z);
                    nf++;
                }
            }
            float r[6];
#pragma unroll
            for (int a = 0; a < 3; a++) { r[a] = wave_min(bmn[a]); r[3 + a] = wave_max(bmx[a]); }
            const uint32_t nfw = wave_sum(nf);
            const uint32_t kc = GROUND ? wave_sum((uint32_t)__popcll(kp.w[0]) + kamb) : 0u;
            if (l == 0) {
                if (nfw) {
#pragma unroll
                    for (int a = 0; a < 3; a++) {
                        atomicMin(L.split + SP_BMIN + a, cg_fkey(r[a]));
                        atomicMax(L.split + SP_BMAX + a, cg_fkey(r[3 + a]));
                    }
                    atomicAdd(L.split + SP_NFIN, nfw);
                }
                if (kc) atomicAdd(L.split + SP_K, kc);
            }
        }
        __builtin_amdgcn_s_waitcnt(0x0070);   // every lane's stores and atomics are complete
        __syncthreads();
        if (tid == 0)
            fs->scal[S_LAST] = __hip_atomic_fetch_add(L.split + SP_DONE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
                               gridDim.x - 1;
        __syncthreads();
        if (!fs->scal[S_LAST]) return;
        STAMP(31);
        // the last workgroup: the frame's counts and bounds (the state reset for the next frame:
        // every chunk has read the keys and added its counts), then the survivors
        if (tid == 0) {
            fs->scal[S_MS] = ld_rlx(L.split + SP_MS);
            fs->scal[S_K] = ld_rlx(L.split + SP_K);
            fs->scal[S_MF] = ld_rlx(L.split + SP_NFIN);
            fs->scal[S_ERR] = ld_rlx(L.split + SP_ERR);
#pragma unroll
            for (int a = 0; a < 3; a++) {
                fs->scal[S_BMIN0 + a] = ld_rlx(L.split + SP_BMIN + a);
                fs->scal[S_BMAX0 + a] = ld_rlx(L.split + SP_BMAX + a);
            }
        }
        __syncthreads();
        if (fs->scal[S_ERR]) {   // (the keys of chunks that gave up were never read here)
            if (GROUND && tid <= CG_NUM_BINS) fs->sec_key[tid] = ld_rlx(L.split + SP_KEYS + tid);
            if (tid == 0) { fs->scal[S_MS] = 0; fs->scal[S_MF] = 0; }
        }
        if (L.seckeys && GROUND && tid <= CG_NUM_BINS) L.seckeys[tid] = fs->sec_key[tid];
        if (tid < SP_STATE) {
            const bool keyw = (tid >= SP_KEYS && tid < SP_KEYS + CG_NUM_BINS + 1) || (tid >= SP_BMIN && tid < SP_BMIN + 3);
            st_rlx(L.split + tid, keyw ? 0xffffffffu : 0u);
        }
        {
            const uint32_t Ms = fs->scal[S_MS];
            const float4* const sp_p = (const float4*)(L.split + SP_SURV);
            uint32_t* const sp_i = L.split + SP_SURV + 4 * CG_MAX_POINTS;
            const Work Wl = lds_work(bl);
            const Work Wg = global_work(L.scratch, N);
            for (uint32_t j = tid; j < Ms; j += CG_BLOCK) {
                const float4 p = ld_f4(&sp_p[j]);
                const uint32_t ix = ld_rlx(&sp_i[j]);
                if (j < (uint32_t)CG_MMAX) { Wl.P[j] = p; Wl.IDX[j] = ix; }
                else { Wg.P[j] = p; Wg.IDX[j] = ix; }
            }
        }
        __syncthreads();
    } else {
        auto store = [&](int g, uint2 c) { ((uint2*)zq)[g * CG_BLOCK + tid] = c; };
        if (LAYOUT == CG_LAYOUT_XYZI16 && N == (uint32_t)(PPT * CG_BLOCK))   // whole groups only
            stream_pass1<PPT, LAYOUT, GROUND, FILTER, decltype(store), true>(fb, N, L, P, fs->sec_key, fs->rays,
                                                                          posm, touched, store);
        else
            stream_pass1<PPT, LAYOUT, GROUND, FILTER>(fb, N, L, P, fs->sec_key, fs->rays, posm, touched, store);
    }
    if (GROUND && !SPLIT) {
        touched = wave_or(touched);
        if (l == 0) atomicOr(&fs->scal[S_TOUCHED], touched);
    }
    __syncthreads();
    STAMP(1);

    CG_HOOK_FRAME_PHASE(1);
    const uint32_t lcap = CG_MMAX;
    const Work Wl = lds_work(bl);
    const Work Wg = global_work(L.scratch + (uint64_t)f * L.scratch_stride, N);
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t nfin = 0;
    auto bound = [&](const float4& p) {
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
            mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
            nfin++;
        }
    };
  if constexpr (!SPLIT) {   // (split frames: the chunks decided their points above)
    if (GROUND && tid < 64) {
        sector_thresholds(fs->sec_key, fs->scal[S_TOUCHED], P, fs->thr, fs->tkey, &fs->scal[S_TKMIN], &fs->scal[S_TKMAX]);
        if (L.seckeys && tid <= CG_NUM_BINS) L.seckeys[(uint64_t)f * (CG_NUM_BINS + 1) + tid] = fs->sec_key[tid];
    }
    __syncthreads();
    STAMP(2);

    // ---- pass 2: ground decisions from the codes ----
    auto codes_of = [&](int g) { return ((const uint2*)zq)[g * CG_BLOCK + tid]; };
    LaneBits<NW> keepgm, amb;
    keepgm.clear();
    amb.clear();
    if (KMODE == CG_KMODE_GROUND) {
        pass2_keep<PPT, LAYOUT>(fb, N, L, P, fs->scal[S_TKMIN], fs->scal[S_TKMAX], fs->tkey, codes_of, keepgm);
        const uint32_t kc = wave_sum(keepgm.count());
        if (l == 0) atomicAdd(&fs->scal[S_K], kc);
    } else if (GROUND) {
        // the ambiguous points are decided below, in the same round of loads as the survivors
        pass2_codes<PPT>(N, fs->scal[S_TKMIN], fs->scal[S_TKMAX], codes_of, keepgm, amb);
    } else {
#pragma unroll
        for (int k = 0; k < PPT; k++)
            if ((uint32_t)k * CG_BLOCK + tid < N) keepgm.w[k >> 6] |= 1ull << (k & 63);
    }
    STAMP(22);

    if (KMODE == CG_KMODE_GROUND) {
        // groundless cloud: K kept points in point order, then N-K PointXYZI()
        // (ground_removal.cpp:70-79); stable order comes from per-(k, wave) ballot counts,
        // which overlay the z codes once every wave is past pass 2
        uint32_t* const cnt = (uint32_t*)zq;
        __syncthreads();
#pragma unroll 8
        for (int k = 0; k < PPT; k++) {
            const uint64_t bb = __ballot(keepgm.get(k));
            if (l == 0) cnt[k * WAVES + w] = (uint32_t)__popcll(bb);
        }
        __syncthreads();
        STAMP(3);
        const uint32_t Kc = block_scan(
            PPT * WAVES, [&](uint32_t i) -> uint32_t { return cnt[i]; },
            [&](uint32_t i, uint32_t e) { cnt[i] = e; }, fs->red);
        STAMP(4);
        float4* out = (float4*)(L.ground + (uint64_t)f * N * 32);
#pragma unroll 4
        for (int k = 0; k < PPT; k++) {
            const bool kp = keepgm.get(k);
            const uint64_t bb = __ballot(kp);
            if (kp) {
                const uint32_t i = (uint32_t)k * CG_BLOCK + tid;
                const uint32_t dst = cnt[k * WAVES + w] + (uint32_t)__popcll(bb & ((1ull << l) - 1ull));
                const float4 pp = load_xyzi<LAYOUT>(fb, i, L);
                out[2 * dst] = make_float4(pp.x, pp.y, pp.z, 1.0f);
                out[2 * dst + 1] = make_float4(pp.w, 0.f, 0.f, 0.f);
            }
        }
        for (uint32_t j = Kc + tid; j < N; j += CG_BLOCK) {
            out[2 * j] = make_float4(0.f, 0.f, 0.f, 1.0f);
            out[2 * j + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
        }
        if (tid == 0) {
            uint32_t* h = L.hdr + (uint64_t)f * 8;
            h[0] = N; h[1] = Kc; h[2] = N; h[3] = 0; h[4] = 0; h[5] = 0;
        }
        return;
    }

    // ---- survivors: one round of loads gathers the kept filter survivors and decides the
    // ambiguous points (exactly, from the loaded x, y, z). The points are spread over the
    // wave's lanes: a lane with many (a near cone's column) would otherwise take one round of
    // loads per four of them while its wave waits. Each wave appends its survivors per round;
    // every survivor carries its point index and the voxel sort orders by (voxel idx, point
    // index), so append order does not matter. Slots below the LDS capacity go to LDS, the rest
    // to the frame's HBM slot (moved whole below when M does not fit) ----
    __syncthreads();   // every wave is past the codes: LDS survivor slots overlay them from here
    STAMP(3);
    auto put = [&](uint32_t pos, const float4& pt, uint32_t idx) {
        if (pos < lcap) {
            Wl.P[pos] = pt;
            Wl.IDX[pos] = idx;
        } else {
            Wg.P[pos] = pt;
            Wg.IDX[pos] = idx;
        }
        bound(pt);
    };
    // the points to load: kept filter survivors, and every ambiguous point (an ambiguous point
    // outside the filter only counts toward K)
    LaneBits<NW> todo;
#pragma unroll
    for (int i = 0; i < NW; i++) todo.w[i] = (FILTER ? (keepgm.w[i] & posm.w[i]) : keepgm.w[i]) | amb.w[i];
    // the rest listed in wave order, 256 per round, in the wave's stage (KEY: free until the
    // backend): k << 8 | lane << 2 | ambiguous << 1 | filter survivor (never 0)
    uint32_t* const stage = (uint32_t*)Wl.KEY + w * 256;
    const uint32_t cnt = todo.count();
    const uint32_t lincl = wave_incl_scan(cnt);
    const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)lincl, 63), lex = lincl - cnt;
    uint32_t kamb = 0;   // ambiguous points the exact test keeps
    uint32_t r0 = 0;
    do {   // wave-uniform rounds
        {
            uint32_t idx = lex;
#pragma unroll
            for (int wi = 0; wi < NW; wi++) {
                uint64_t m = todo.w[wi];
                while (m && idx < r0 + 256u) {
                    const uint32_t k = 64 * wi + (uint32_t)__builtin_ctzll(m);
                    m &= m - 1;
                    if (idx >= r0)
                        stage[idx - r0] = (k << 8) | (l << 2) | (amb.get(k) ? 2u : 0u) |
                                          ((!FILTER || posm.get(k)) ? 1u : 0u);
                    idx++;
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
        const uint32_t n = T > r0 ? min(256u, T - r0) : 0u;
        uint32_t e[4];
#pragma unroll
        for (int q = 0; q < 4; q++) e[q] = (uint32_t)(l + 64 * q) < n ? stage[l + 64 * q] : 0u;
        __builtin_amdgcn_wave_barrier();   // the stage read before the next round writes it
        float4 pt[4];
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (e[q]) pt[q] = load_xyzi<LAYOUT>(fb, (e[q] >> 8) * CG_BLOCK + w * 64 + ((e[q] >> 2) & 63u), L);
        bool sv[4];
        uint32_t ns = 0;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            sv[q] = false;
            if (!e[q]) continue;
            bool kept = true;
            if (GROUND && (e[q] & 2u)) {
                kept = pass2_exact(P, fs->tkey, pt[q].x, pt[q].y, pt[q].z);
                kamb += kept ? 1u : 0u;
            }
            sv[q] = kept && (e[q] & 1u);
            ns += sv[q] ? 1u : 0u;
        }
        const uint32_t incl = wave_incl_scan(ns);
        uint32_t wbase = 0;
        if (l == 63 && incl) wbase = atomicAdd(&fs->scal[S_MS], incl);
        wbase = (uint32_t)__builtin_amdgcn_readlane((int)wbase, 63);
        uint32_t pos = wbase + incl - ns;
#pragma unroll
        for (int q = 0; q < 4; q++)
            if (sv[q]) { put(pos, pt[q], (e[q] >> 8) * CG_BLOCK + w * 64 + ((e[q] >> 2) & 63u)); pos++; }
        r0 += 256u;
    } while (r0 < T);
    if (GROUND) {
        const uint32_t kc = wave_sum(keepgm.count() + kamb);
        if (l == 0) atomicAdd(&fs->scal[S_K], kc);
    }
    STAMP(25);
    __syncthreads();   // counts complete
  }
    STAMP(4);

    CG_HOOK_FRAME_PHASE(2);
    const uint32_t Ms = fs->scal[S_MS];
    const uint32_t K = GROUND ? fs->scal[S_K] : N;
    // pipeline: the detector input is the groundless cloud, whose N-K trailing
    // PointXYZI() points survive the filter iff P.zero_pass (src/cone_detection.cpp:195-201)
    const uint32_t npad = (KMODE == CG_KMODE_PIPELINE && P.zero_pass) ? N - K : 0u;
    const uint32_t M = Ms + npad;
    const bool use_lds = M <= CG_MMAX;
    const uint32_t flags = use_lds ? 0u : 0x2u;
    if (tid == 0) {
        uint32_t* h = L.hdr + (uint64_t)f * 8;
        h[0] = N;
        h[1] = K;
    }
    const Work W = use_lds ? Wl : Wg;
    if (!use_lds) {   // the slots below the LDS capacity to the frame's HBM slot
        const uint32_t nl = min(Ms, lcap);
        for (uint32_t j = tid; j < nl; j += CG_BLOCK) {
            Wg.P[j] = Wl.P[j];
            Wg.IDX[j] = Wl.IDX[j];
        }
    }
    for (uint32_t j = tid; j < npad; j += CG_BLOCK) {
        const float4 z4 = make_float4(0.f, 0.f, 0.f, 0.f);
        W.P[Ms + j] = z4;
        W.IDX[Ms + j] = 0xffffu;   // after every kept point; exact-zero terms are order-free
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
    STAMP(26);
    __syncthreads();
    STAMP(5);

    CG_HOOK_FRAME_PHASE(3);
    if (use_lds) {
        backend(lds_work(bl), M, fs, L, P, f, flags, CG_MAX_POINTS / 32, CG_MMAX);
    } else {
        backend(W, M, fs, L, P, f, flags, CG_MAX_POINTS / 32, 0);
    }
    if constexpr (SPLIT) {   // the results packed for the host's one copy (fetch_frame)
        // header word 7: a chunk gave up waiting for the others (the host runs the frame again)
        if (tid == 0) L.hdr[CG_HDR_ERR] = fs->scal[S_ERR];
        if (L.pack) {
            __threadfence();
            __syncthreads();
            pack_frame(L, f, L.pack);
            if (L.pack_seq) {
                // the done word after every packed word: every wave's stores complete
                // (vmcnt(0)), the barrier, then one system-scope release (the L2 write-back that
                // puts the packed words in host memory: plain stores alone were seen overtaken by
                // the done word, and a system-scope store per word cost ~80 us per call,
                // profiles/r4_chunk_batch_reverted.txt), then the word
                __builtin_amdgcn_s_waitcnt(0x0070);
                __syncthreads();
                if (tid == 0) {
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
                    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (the fence's wait, kept)
                    __hip_atomic_store(&L.pack[CG_PACK_DONE], L.pack_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
    if (L.span && tid == 0) {
        const uint64_t c1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        atomicMax(&L.span[1], (unsigned long long)r1);
        atomicAdd(&L.span[2], (unsigned long long)(c1 - span_c0));
        atomicAdd(&L.span[3], (unsigned long long)(r1 - span_r0));
    }
}

// The kernels: the batch frame kernel (two workgroups per CU: <= 128 VGPRs); the single-frame
// split kernel (its 16 workgroups have a CU each: 2 waves per SIMD, room to keep every spill out
// of scratch).
template <int PPT, int LAYOUT, int KMODE>
__global__ __launch_bounds__(CG_BLOCK, 4) void cg_frame_kernel(CgLaunch L, CgDevParams P) {
    frame_body<PPT, LAYOUT, KMODE>(L, P);
}
template <int PPT, int LAYOUT, int KMODE>
__global__ __launch_bounds__(CG_BLOCK, 2) void cg_split_kernel(CgLaunch L, CgDevParams P) {
    frame_body<PPT, LAYOUT, KMODE, true>(L, P);
}

// ------------------------------------------------------------------------------------------
// Large frames whose detector input fits the LDS path (M <= CG_MMAX): the survivors come from
// HBM in append order; sorted by frame index they get ranks as point indices, so the voxel
// keys order ties exactly as the frame kernel does. npad PointXYZI() pads follow.
// npad = CG_K_FROM_META (the backend sized on the device): npad and K from the meta words, and
// the launch returns unless the decisions' fold chose this backend (LG_SMALL).
__global__ __launch_bounds__(CG_BLOCK, 2) void cg_lg_back_small(CgLaunch L, CgDevParams P, LgScratch S,
                                                                uint32_t f, uint32_t npad, uint32_t K) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
    FrontShared* fs = (FrontShared*)smem;
    BackLds* bl = (BackLds*)(smem + FRONT_BYTES);
    const uint32_t tid = threadIdx.x;
    if (npad == CG_K_FROM_META) {
        if (!S.meta[LG_SMALL]) return;
        npad = S.meta[LG_NPAD];
        K = S.meta[LG_KHDR];
    }
    const uint32_t Ms = S.meta[LG_MS], M = Ms + npad;
    if (tid < 64) fs->scal[tid] = 0;
    __syncthreads();
    if (tid == 0) {
        const uint32_t zk = cg_fkey(0.0f);
        for (int a = 0; a < 3; a++) {
            uint32_t lo = S.meta[LG_BMIN + a], hi = S.meta[LG_BMAX + a];
            if (npad) { lo = min(lo, zk); hi = max(hi, zk); }
            fs->scal[S_BMIN0 + a] = lo;
            fs->scal[S_BMAX0 + a] = hi;
        }
        fs->scal[S_MF] = S.meta[LG_NFIN] + npad;
        uint32_t* h = L.hdr + (uint64_t)f * 8;
        h[0] = L.n_points;
        h[1] = K;
    }
    uint64_t* tmp = (uint64_t*)bl->VOX;
    for (uint32_t j = tid; j < Ms; j += CG_BLOCK) tmp[j] = ((uint64_t)S.surv_i[j] << 16) | j;
    __syncthreads();
    if (Ms <= CG_RANK_SORT_MAX) {
        rank_sort(tmp, bl->KEY, Ms);
    } else {
        uint32_t n2 = 1;
        while (n2 < Ms) n2 <<= 1;
        for (uint32_t j = tid; j < n2; j += CG_BLOCK) bl->KEY[j] = j < Ms ? tmp[j] : ~0ull;
        __syncthreads();
        bitonic_sort(bl->KEY, n2);
    }
    for (uint32_t r = tid; r < Ms; r += CG_BLOCK) {
        bl->P[r] = S.surv_p[(uint32_t)(bl->KEY[r] & 0xffffu)];
        bl->IDX[r] = r;
    }
    for (uint32_t j = tid; j < npad; j += CG_BLOCK) {
        bl->P[Ms + j] = make_float4(0.f, 0.f, 0.f, 0.f);
        bl->IDX[Ms + j] = 0xffffu;   // after every kept point
    }
    if (tid == 0) fs->scal[S_MS] = Ms;   // kept survivors (slots [0, Ms)); pads follow
    __syncthreads();
    Work W;
    W.P = bl->P; W.KEY = bl->KEY; W.VOX = bl->VOX; W.A = bl->A; W.PAR = bl->PAR; W.CNT = bl->CNT;
    W.UK = bl->UK; W.LAB = bl->LAB; W.ORD = bl->ORD; W.IDX = bl->IDX; W.OFF = bl->OFF;
    backend(W, M, fs, L, P, f, 0u, CG_MAX_POINTS / 32, CG_MMAX);
}
int cg_launch_lg_back_small(const CgLaunch& L, const CgDevParams& P, const LgScratch& S, uint32_t f,
                            uint32_t npad, uint32_t K, hipStream_t s) {
    hipLaunchKernelGGL(cg_lg_back_small, dim3(1), dim3(CG_BLOCK), 0, s, L, P, S, f, npad, K);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Launchers. Batches: one fused workgroup per frame.
template <int PPT, int LAYOUT>
static hipError_t launch3(const CgLaunch& L, const CgDevParams& P, int kmode, hipStream_t s) {
    const dim3 grid(L.n_frames), block(CG_BLOCK);
    switch (kmode) {
        case CG_KMODE_PIPELINE:
            hipLaunchKernelGGL((cg_frame_kernel<PPT, LAYOUT, CG_KMODE_PIPELINE>), grid, block, 0, s, L, P);
            break;
        case CG_KMODE_DETECT:
            hipLaunchKernelGGL((cg_frame_kernel<PPT, LAYOUT, CG_KMODE_DETECT>), grid, block, 0, s, L, P);
            break;
        default:
            hipLaunchKernelGGL((cg_frame_kernel<PPT, LAYOUT, CG_KMODE_GROUND>), grid, block, 0, s, L, P);
            break;
    }
    return hipGetLastError();
}

int cg_launch_split(const CgLaunch& L, const CgDevParams& P, int kmode, hipStream_t s) {
    constexpr int PPT = CG_MAX_POINTS / CG_BLOCK;
    const uint32_t nch = (L.n_points + CG_SPLIT_CHUNK - 1) / CG_SPLIT_CHUNK;
    const dim3 grid(nch ? nch : 1u), block(CG_BLOCK);
    const bool xyzi16 = L.point_step == 16 && L.off_x == 0 && L.off_y == 4 && L.off_z == 8 && L.off_i == 12;
    if (kmode == CG_KMODE_PIPELINE) {
        if (xyzi16) hipLaunchKernelGGL((cg_split_kernel<PPT, CG_LAYOUT_XYZI16, CG_KMODE_PIPELINE>), grid, block, 0, s, L, P);
        else hipLaunchKernelGGL((cg_split_kernel<PPT, CG_LAYOUT_GENERIC, CG_KMODE_PIPELINE>), grid, block, 0, s, L, P);
    } else {
        if (xyzi16) hipLaunchKernelGGL((cg_split_kernel<PPT, CG_LAYOUT_XYZI16, CG_KMODE_DETECT>), grid, block, 0, s, L, P);
        else hipLaunchKernelGGL((cg_split_kernel<PPT, CG_LAYOUT_GENERIC, CG_KMODE_DETECT>), grid, block, 0, s, L, P);
    }
    return hipGetLastError();
}

int cg_launch_batch(const CgLaunch& L, const CgDevParams& P, int kmode, hipStream_t s) {
    if (L.n_frames == 0) return hipSuccess;
    const bool xyzi16 = L.point_step == 16 && L.off_x == 0 && L.off_y == 4 && L.off_z == 8 &&
                        L.off_i == 12;
    if (L.n_points <= 32 * CG_BLOCK) {
        return xyzi16 ? launch3<32, CG_LAYOUT_XYZI16>(L, P, kmode, s)
                      : launch3<32, CG_LAYOUT_GENERIC>(L, P, kmode, s);
    }
    return xyzi16 ? launch3<CG_MAX_POINTS / CG_BLOCK, CG_LAYOUT_XYZI16>(L, P, kmode, s)
                  : launch3<CG_MAX_POINTS / CG_BLOCK, CG_LAYOUT_GENERIC>(L, P, kmode, s);
}

// ------------------------------------------------------------------------------------------
// Self-test kernels: the device restatements, evaluated element-wise for host comparison.
// Results of one frame packed for a single device-to-host copy (fetch_frame): the header, then
// up to CG_PACK_MAX entries of each result array at fixed offsets (cg_internal.h CG_PACK_*).
__device__ __forceinline__ void pack_frame(const CgLaunch& L, uint32_t f, uint32_t* out) {
    auto put = [](uint32_t* q, uint32_t v) { *q = v; };
    const uint32_t nt = blockDim.x;
    const uint32_t* hdr = L.hdr + (uint64_t)f * CG_HDR_WORDS;
    const uint32_t V = min(hdr[CG_HDR_V], (uint32_t)CG_PACK_MAX), C = min(hdr[CG_HDR_C], (uint32_t)CG_PACK_MAX);
    const int32_t* offs = L.offs + (uint64_t)f * (L.cap + 1);
    const uint32_t nidx = min(C ? (uint32_t)offs[C] : 0u, (uint32_t)CG_PACK_MAX);
    const float4* vox = L.vox + (uint64_t)f * L.cap;
    const int32_t* lab = L.lab + (uint64_t)f * L.cap;
    const int32_t* idx = L.idx + (uint64_t)f * L.cap;
    const float2* cen = L.cen + (uint64_t)f * L.cap;
    for (uint32_t i = threadIdx.x; i < CG_HDR_WORDS; i += nt) put(out + i, hdr[i]);
    for (uint32_t i = threadIdx.x; i < V; i += nt) {
        const float4 p = vox[i];
        uint32_t* q = out + CG_PACK_VOX + 4 * i;
        put(q, __float_as_uint(p.x)); put(q + 1, __float_as_uint(p.y));
        put(q + 2, __float_as_uint(p.z)); put(q + 3, __float_as_uint(p.w));
        put(out + CG_PACK_LAB + i, (uint32_t)lab[i]);
    }
    for (uint32_t i = threadIdx.x; i <= C; i += nt) put(out + CG_PACK_OFFS + i, (uint32_t)offs[i]);
    for (uint32_t i = threadIdx.x; i < nidx; i += nt) put(out + CG_PACK_IDX + i, (uint32_t)idx[i]);
    for (uint32_t i = threadIdx.x; i < C; i += nt) {
        put(out + CG_PACK_CEN + 2 * i, __float_as_uint(cen[i].x));
        put(out + CG_PACK_CEN + 2 * i + 1, __float_as_uint(cen[i].y));
    }
}
__global__ __launch_bounds__(256) void cg_pack_results(CgLaunch L, uint32_t f, uint32_t* out) {
    pack_frame(L, f, out);
}
int cg_launch_pack(const CgLaunch& L, uint32_t f, uint32_t* out, hipStream_t s) {
    hipLaunchKernelGGL(cg_pack_results, dim3(1), dim3(256), 0, s, L, f, out);
    return hipGetLastError();
}

__global__ void cg_selftest_atan2f_kernel(const float* y, const float* x, float* out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float a = cg_atan2f(y[i], x[i]);
        out[2 * i] = a;
        // sector and angle-filter decision (|a| >= 1.3) through the certified fast path (must
        // equal the exact ones): sector + 32 * removed
        CgDevParams P{};
        P.ang_lo = -1.3f; P.ang_hi = 1.3f;
        P.ang_cert_lo = 1.3f - 2.0f * CG_ANG_MARGIN;   // (the host derives these in prepare)
        P.ang_cert_hi = 1.3f + 2.0f * CG_ANG_MARGIN;
        int s = 0;
        bool rm = false;
        classify_angle<true, true>(P, x[i], y[i], s, rm);
        out[2 * i + 1] = (float)(s + (rm ? 32 : 0));
    }
}
__global__ void cg_selftest_sqrt_kernel(const double* in, double* out, uint32_t n) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = __builtin_sqrt(in[i]);
}
int cg_launch_selftest_atan2f(const float* y, const float* x, float* out, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(cg_selftest_atan2f_kernel, dim3((n + 255) / 256), dim3(256), 0, s, y, x, out, n);
    return hipGetLastError();
}
int cg_launch_selftest_sqrt(const double* in, double* out, uint32_t n, hipStream_t s) {
    hipLaunchKernelGGL(cg_selftest_sqrt_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, out, n);
    return hipGetLastError();
}
