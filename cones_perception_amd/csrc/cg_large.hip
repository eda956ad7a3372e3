// cg_large.hip — frames of more than 65,536 points (C5's 1M-point dense frame,
// and any LiDAR with more than 64 x 1024 returns). Same semantics as the frame kernel
// (cg_kernels.hip), spread over many workgroups per frame and HBM scratch:
//
//   lg_front    one 512-lane workgroup per 4,096-point chunk: pass 1 (stream_pass1), z codes
//               to HBM, per-chunk statistics (sector minima, used bins; detector mode: the
//               filter survivors' bits and count)
//   lg_reduce_chunks  one workgroup folds the chunk statistics into the frame's meta words
//   lg_decide   per chunk: thresholds, pass 2 over the chunk's codes (kept count K), survivor
//               bits = ground-kept & filter bits (ambiguous codes decided exactly)
//   lg_surv_write  survivors in frame-index order (chunk-count prefix, then (k, lane) order)
//               with their VoxelGrid bounds
//   lg_ground_* ground-only mode: stable per-chunk output offsets, kept points then zero pads
//   backend     M <= CG_MMAX: one workgroup from LDS (cg_kernels.hip, cg_launch_lg_back_small);
//               otherwise the global backend below: PCL's index_vector as (idx, slot) records
//               and std::sort's permutation of it (partition levels lg_pq_split / lg_pq_swap,
//               then lg_pcl_leaf and lg_pcl_mid; point order instead: a stable LSD
//               radix sort), voxel runs + centroids in that order, a dense neighbour grid, a
//               lowest-neighbour forest, pointer jumping and cross-tree unions (roots = lowest
//               voxel index = PCL's seed), size filter, PCL's cluster order, CSR by a sort of
//               the rank bits, per-cluster centroids.
//   cg_halo_*   C5 spatial tiling: the backend per voxel slab, cross-slab edges, merge (voxel
//               sums in point order there).
//
// Every sum keeps the order of the frame kernel's on the same input (PCL's std::sort order by
// default), so the results are bit-identical to it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>
#include "cg_internal.h"
#include "../../include/cones_gpu.h"
#include "cg_math.h"
#include "cg_sort.h"
#include "cg_device.h"
#include "cg_pcl.h"

#define LG_TILE 4096   // elements per scan / sort workgroup (512 threads x 8)

// ------------------------------------------------------------------------------------------
// Meta words (initialised by lg_init).
__device__ __forceinline__ void lg_init_meta(const LgScratch& S, const CgDevParams& P, uint32_t t) {
    if (t < LG_META_WORDS) {
        uint32_t v = 0;
        if (t <= CG_NUM_BINS) v = cg_fkey(P.default_low);
        if (t >= LG_BMIN && t < LG_BMIN + 3) v = 0xffffffffu;
        S.meta[t] = v;
    }
}
__global__ void lg_init(LgScratch S, CgDevParams P) { lg_init_meta(S, P, threadIdx.x); }

// The launch's last workgroup to arrive (thread 0, after every storing thread of its workgroup
// has waited for its stores), with the arrivals spread over eight counters: one word takes ~88
// atomics per us (MI355X_MICROARCH.md, "dequeue"), so a 1,024-workgroup launch would queue ~12
// us on one. A workgroup adds to counter blockIdx % 8, the last of each counter to the top one,
// and the last there is the launch's last: it resets the nine words (every other arrival has
// happened). Each arrival is an agent-scope atomic after the arriving workgroup's sc1 stores
// completed, so the last sees every workgroup's stores through sc1 loads.
__device__ __forceinline__ bool lg_last_arrival(uint32_t* cnt) {
    const uint32_t G = gridDim.x, sh = blockIdx.x & 7u;
    const uint32_t in_shard = (G - sh + 7u) / 8u, shards = min(G, 8u);
    if (__hip_atomic_fetch_add(&cnt[sh], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != in_shard - 1u) return false;
    if (__hip_atomic_fetch_add(&cnt[8], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != shards - 1u) return false;
    for (int i = 0; i < 9; i++) st_rlx(&cnt[i], 0u);
    return true;
}
// Arrival counters of the launches that hand over to their last workgroup (zeroed scratch, and
// left zeroed by their last arrival): 0 lg_surv_write
__device__ __forceinline__ uint32_t* lg_arrivals(const LgScratch& S, uint32_t k);

// Bounds of finite points, merged into the frame's meta words (order-preserving keys).
struct Bounds {
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t n = 0;
    __device__ __forceinline__ void add(const float4& p) {
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
            mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
            n++;
        }
    }
    // whole workgroup: wave partials through LDS (part: 7 * WAVES words), then one lane writes
    // the workgroup's bounds keys and finite count into its chunk statistics words cs
    // rlx: sc1 stores (a workgroup of the same launch folds them, lg_surv_write)
    __device__ __forceinline__ void merge_block(uint32_t* meta, uint32_t* part, bool rlx = false) {
        float r[6];
#pragma unroll
        for (int a = 0; a < 3; a++) { r[a] = wave_min(mn[a]); r[3 + a] = wave_max(mx[a]); }
        const uint32_t nf = wave_sum(n), w = wave_id();
        if (lane_id() == 0) {
#pragma unroll
            for (int a = 0; a < 6; a++) part[7 * w + a] = __float_as_uint(r[a]);
            part[7 * w + 6] = nf;
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            float q[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
            uint32_t t = 0;
            for (int v = 0; v < WAVES; v++) {
                for (int a = 0; a < 3; a++) {
                    q[a] = fminf(q[a], __uint_as_float(part[7 * v + a]));
                    q[3 + a] = fmaxf(q[3 + a], __uint_as_float(part[7 * v + 3 + a]));
                }
                t += part[7 * v + 6];
            }
            for (int a = 0; a < 3; a++) {   // (no finite point: keys that change no MIN / MAX)
                const uint32_t lo = t ? cg_fkey(q[a]) : 0xffffffffu, hi = t ? cg_fkey(q[3 + a]) : 0u;
                if (rlx) { st_rlx(meta + LG_CS_BMIN + a, lo); st_rlx(meta + LG_CS_BMAX + a, hi); }
                else { meta[LG_CS_BMIN + a] = lo; meta[LG_CS_BMAX + a] = hi; }
            }
            if (rlx) st_rlx(meta + LG_CS_NFIN, t);
            else meta[LG_CS_NFIN] = t;
        }
    }
    __device__ __forceinline__ void merge(uint32_t* meta) {   // every lane of the wave calls
        float r[6];
#pragma unroll
        for (int a = 0; a < 3; a++) { r[a] = wave_min(mn[a]); r[3 + a] = wave_max(mx[a]); }
        const uint32_t nf = wave_sum(n);
        if (lane_id() == 0 && nf) {
#pragma unroll
            for (int a = 0; a < 3; a++) {
                atomicMin(&meta[LG_BMIN + a], cg_fkey(r[a]));
                atomicMax(&meta[LG_BMAX + a], cg_fkey(r[3 + a]));
            }
            atomicAdd(&meta[LG_NFIN], nf);
        }
    }
};

// ------------------------------------------------------------------------------------------
// The chunk's survivor bits m (point k*CG_BLOCK + tid of the chunk, bit k of the lane) go to
// S.keep, their count to S.chunk_cnt[c]; lg_surv_write then writes the survivors in frame-index
// order (every workgroup of the launch calls this).
template <int NW>
__device__ __forceinline__ void lg_store_survivor_bits(LgScratch& S, uint32_t c, const LaneBits<NW>& m,
                                                       uint32_t* red) {
    const uint32_t tid = threadIdx.x;
#pragma unroll
    for (int wi = 0; wi < NW; wi++) S.keep[((uint64_t)c * CG_BLOCK + tid) * NW + wi] = m.w[wi];
    const uint32_t n = wave_sum(m.count());
    if (lane_id() == 0) red[wave_id()] = n;
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
        for (int w = 0; w < WAVES; w++) t += red[w];
        S.chunk_cnt[c] = t;
    }
}

// One workgroup folds the per-chunk statistics into the meta words: the sector keys (MIN) and
// used bins (OR) after the front; K, survivor count, finite count (SUM) and the VoxelGrid
// bounds (MIN / MAX keys) after the decisions. what: bit 0 keys, bit 1 K, bit 2 survivors,
// bit 3 (LG_FOLD_SIZE, with bit 2) the detector input's size and backend for the launches
// sized on the device (szfl: LG_SZ_*; N the frame's points).
#define LG_FOLD_SIZE 8u
#define LG_SZ_PIPE 1u     // K from the ground stage (detector mode: K = N)
#define LG_SZ_ZPAD 2u     // the N - K PointXYZI() pads survive the filter (P.zero_pass)
#define LG_SZ_GLOBAL 4u   // the global backend even when M fits the LDS one (diagnostics)
#define LG_SZ_ON 0x80000000u   // (host side: cg_large_front / cg_large_decide fold the sizes)
#define LG_WM_KEYS ((1u << (CG_NUM_BINS + 1)) - 1u)   // fold words: the sector keys,
#define LG_WM_TOUCHED (1u << LG_CS_TOUCHED)            // the used bins
// The fold itself, called by every thread of the block: thread w < LG_CS_WORDS returns word w
// folded over the nch chunks (words outside wmask: not loaded).
__device__ __forceinline__ uint32_t lg_fold_core(const LgScratch& S, uint32_t nch, uint32_t wmask,
                                                 uint32_t (*part)[LG_CS_WORDS], bool rlx = false) {
    const uint32_t tid = threadIdx.x, w = tid & 31, q = tid >> 5;   // word, one of 16 chunk strides
    const bool mn = (w <= CG_NUM_BINS) || (w >= LG_CS_BMIN && w < LG_CS_BMIN + 3);
    const bool mx = w >= LG_CS_BMAX && w < LG_CS_BMAX + 3;
    const bool orw = w == LG_CS_TOUCHED;
    uint32_t acc = mn ? 0xffffffffu : 0u;
    auto fold = [&](uint32_t a, uint32_t v) { return mn ? min(a, v) : mx ? max(a, v) : orw ? (a | v) : a + v; };
    // rlx: sc1 loads (words a workgroup of the same launch stored with sc1)
    auto ld = [&](uint32_t c) { uint32_t* a = S.cstat + (uint64_t)c * LG_CS_WORDS + w; return rlx ? ld_rlx(a) : *a; };
    if ((wmask >> w) & 1u) {
        for (uint32_t c0 = q; c0 < nch; c0 += 256) {   // sixteen independent loads per trip
            uint32_t v[16];
#pragma unroll
            for (int u = 0; u < 16; u++) v[u] = c0 + 16u * u < nch ? ld(c0 + 16u * u) : (mn ? 0xffffffffu : 0u);
#pragma unroll
            for (int u = 0; u < 16; u++) acc = fold(acc, v[u]);
        }
    }
    part[q][w] = acc;
    __syncthreads();
    uint32_t a = 0;
    if (tid < LG_CS_WORDS) {
        a = part[0][w];
        for (int k = 1; k < 16; k++) a = fold(a, part[k][w]);
    }
    return a;
}
// The detector input's size and backend from K (ground kept count) and Ms (survivors), into the
// meta words m (one thread)
__device__ __forceinline__ void lg_size_fold(const LgScratch& S, uint32_t* m, uint32_t k, uint32_t ms, uint32_t N,
                                             uint32_t szfl, bool hint = true) {
    const uint32_t K = (szfl & LG_SZ_PIPE) ? k : N;
    const uint32_t npad = (szfl & LG_SZ_ZPAD) ? N - K : 0u;
    const uint32_t Mt = ms + npad;
    const bool small = Mt <= CG_MMAX && !(szfl & LG_SZ_GLOBAL);
    m[LG_KHDR] = K;
    m[LG_NPAD] = npad;
    m[LG_MALL] = Mt;
    m[LG_MTOT] = small ? 0u : Mt;
    m[LG_SMALL] = small ? 1u : 0u;
    if (hint && S.hint) S.hint[LG_HINT_SMALL] = Mt <= CG_MMAX ? 2u : 1u;   // (forced global or not)
}
__device__ __forceinline__ void lg_fold_chunks(LgScratch S, uint32_t nch, uint32_t what, uint32_t N = 0,
                                               uint32_t szfl = 0, bool rlx = false) {
    __shared__ uint32_t part[16][LG_CS_WORDS];
    const uint32_t tid = threadIdx.x, w = tid & 31;
    const uint32_t a = lg_fold_core(S, nch, 0xffffffffu, part, rlx);
    if (tid >= LG_CS_WORDS) return;
    uint32_t* m = S.meta;
    if (what & LG_FOLD_SIZE) {   // (all 32 lanes of wave 0 are here)
        const uint32_t k = (uint32_t)__shfl((int)a, LG_CS_K, 64), ms = (uint32_t)__shfl((int)a, LG_CS_MS, 64);
        if (tid == 0) lg_size_fold(S, m, k, ms, N, szfl);
    }
    if ((what & 1u) && w <= CG_NUM_BINS) m[LG_SECKEY + w] = a;
    if ((what & 1u) && w == LG_CS_TOUCHED) m[LG_TOUCHED] = a;
    if ((what & 2u) && w == LG_CS_K) m[LG_K] = a;
    if (what & 4u) {
        if (w == LG_CS_MS) m[LG_MS] = a;
        if (w == LG_CS_NFIN) m[LG_NFIN] = a;
        if (w >= LG_CS_BMIN && w < LG_CS_BMIN + 3) m[LG_BMIN + (w - LG_CS_BMIN)] = a;
        if (w >= LG_CS_BMAX && w < LG_CS_BMAX + 3) m[LG_BMAX + (w - LG_CS_BMAX)] = a;
    }
}

__global__ __launch_bounds__(CG_BLOCK) void lg_reduce_chunks(LgScratch S, uint32_t nch, uint32_t what, uint32_t N,
                                                             uint32_t szfl) {
    lg_fold_chunks(S, nch, what, N, szfl);
}
// (Folding in the last workgroup of the chunk launch instead, behind a release/acquire counter,
// measured 7 -> 53 us per launch on a 256-chunk frame: every workgroup's agent-scope release
// writes back its XCD's L2.)

// ------------------------------------------------------------------------------------------
// Front: pass 1 per chunk.
template <int LAYOUT, int KMODE>
__global__ __launch_bounds__(CG_BLOCK, 4) void lg_front(CgLaunch L, CgDevParams P, LgScratch S, uint32_t f,
                                                       uint32_t init) {
    // init: workgroup 0 resets the frame's meta words (lg_init's work; nothing here reads them,
    // lg_reduce_chunks after this launch folds the chunks into them)
    if (init && blockIdx.x == 0) lg_init_meta(S, P, threadIdx.x);
    constexpr int PPT = LG_CHUNK / CG_BLOCK;
    constexpr int NW = (PPT + 63) / 64;
    constexpr bool GROUND = KMODE != CG_KMODE_DETECT;
    constexpr bool FILTER = KMODE != CG_KMODE_GROUND;
    __shared__ uint32_t sec_key[CG_NUM_BINS + 1];
    __shared__ float4 rays[CG_NUM_BINS];
    const uint32_t c = blockIdx.x, tid = threadIdx.x, l = lane_id();
    const uint64_t base = (uint64_t)c * LG_CHUNK;
    const uint32_t Nc = (uint32_t)min((uint64_t)LG_CHUNK, (uint64_t)L.n_points - base);
    const uint8_t* fb = L.in + (uint64_t)f * L.frame_stride + base * L.point_step;
    if (tid <= CG_NUM_BINS) sec_key[tid] = cg_fkey(P.default_low);
    init_rays<FILTER>(P, rays, tid);
    __syncthreads();
    LaneBits<NW> posm;
    uint32_t touched = 0;
    uint2* codes = (uint2*)S.codes + (uint64_t)c * (LG_CHUNK / 8);
    stream_pass1<PPT, LAYOUT, GROUND, FILTER>(fb, Nc, L, P, sec_key, rays, posm, touched,
                                             [&](int g, uint2 cw) { codes[g * CG_BLOCK + tid] = cw; });
    __shared__ uint32_t tw[WAVES];
    if (GROUND) {
        touched = wave_or(touched);
        if (l == 0) tw[wave_id()] = touched;
    }
    __syncthreads();
    uint32_t* const cs = S.cstat + (uint64_t)c * LG_CS_WORDS;
    if (GROUND && tid <= CG_NUM_BINS) cs[LG_CS_KEYS + tid] = sec_key[tid];
    if (GROUND && tid == 0) {
        uint32_t t = 0;
        for (int w = 0; w < WAVES; w++) t |= tw[w];
        cs[LG_CS_TOUCHED] = t;
    }
    if (GROUND) {
        if (FILTER) {   // pipeline: the filter bits wait for the ground decision (lg_decide)
#pragma unroll
            for (int wi = 0; wi < NW; wi++) S.keep[((uint64_t)c * CG_BLOCK + tid) * NW + wi] = posm.w[wi];
        }
        return;
    }
    // detector: the filter survivors themselves
    __shared__ uint32_t red[WAVES];
    lg_store_survivor_bits<NW>(S, c, posm, red);
}

// Decide: thresholds, pass 2 per chunk, survivors = ground-kept & filter bits (from lg_front).
// (The device-sized pipeline frame: lg_decide_write.)
template <int LAYOUT, int KMODE>
__global__ __launch_bounds__(CG_BLOCK, 4) void lg_decide(CgLaunch L, CgDevParams P, LgScratch S, uint32_t f) {
    constexpr int PPT = LG_CHUNK / CG_BLOCK;
    constexpr int NW = (PPT + 63) / 64;
    __shared__ float thr[CG_NUM_BINS + 1];
    __shared__ uint32_t tkey[CG_NUM_BINS + 1], band[2], kcount;
    const uint32_t c = blockIdx.x, tid = threadIdx.x, l = lane_id();
    const uint64_t base = (uint64_t)c * LG_CHUNK;
    const uint32_t Nc = (uint32_t)min((uint64_t)LG_CHUNK, (uint64_t)L.n_points - base);
    const uint8_t* fb = L.in + (uint64_t)f * L.frame_stride + base * L.point_step;
    const uint32_t* keys = S.meta + LG_SECKEY;
    const uint32_t touched = S.meta[LG_TOUCHED];
    if (tid < 64) sector_thresholds(keys, touched, P, thr, tkey, &band[0], &band[1]);
    // the frame's sector keys to the caller's per-frame output (the pipeline's re-crop reads them)
    if (KMODE == CG_KMODE_PIPELINE && c == 0 && tid <= CG_NUM_BINS && L.seckeys)
        L.seckeys[(uint64_t)f * (CG_NUM_BINS + 1) + tid] = keys[tid];
    if (tid == 0) kcount = 0;
    __syncthreads();
    const uint32_t qlo = band[0], qhi = band[1];
    const uint2* codes = (const uint2*)S.codes + (uint64_t)c * (LG_CHUNK / 8);
    LaneBits<NW> keep;
    pass2_keep<PPT, LAYOUT>(fb, Nc, L, P, qlo, qhi, tkey, [&](int g) { return codes[g * CG_BLOCK + tid]; }, keep);
    const uint32_t kc = wave_sum(keep.count());
    if (l == 0) atomicAdd(&kcount, kc);
    LaneBits<NW> surv;
#pragma unroll
    for (int wi = 0; wi < NW; wi++) {
        uint64_t* const kw = S.keep + ((uint64_t)c * CG_BLOCK + tid) * NW + wi;
        if (KMODE == CG_KMODE_GROUND) *kw = keep.w[wi];
        else surv.w[wi] = keep.w[wi] & *kw;   // kept by the ground filter and by the position filter
    }
    __syncthreads();
    if (tid == 0) {
        S.cstat[(uint64_t)c * LG_CS_WORDS + LG_CS_K] = kcount;
        if (KMODE == CG_KMODE_GROUND) S.chunk_cnt[c] = kcount;
    }
    if (KMODE == CG_KMODE_GROUND) return;
    __shared__ uint32_t red[WAVES];
    lg_store_survivor_bits<NW>(S, c, surv, red);
}

// Survivors of every chunk in frame-index order: the chunk's base is the count of the chunks
// before it, and within the chunk the order is (k, lane), i.e. the point index. VoxelGrid bounds
// of the finite survivors merged into the meta words.
// fold_what != 0 (the device-sized path): the launch's last workgroup to finish folds the chunk
// statistics (lg_reduce_chunks' work, what = fold_what) instead of a launch after it. The words
// this launch writes go out with sc1 stores, every thread waits for its stores, then one count
// per workgroup (lg_last_arrival); the last reads the
// words with sc1 loads (MI355X_MICROARCH.md's hand-off table, row 1).
template <int LAYOUT>
__global__ __launch_bounds__(CG_BLOCK) void lg_surv_write(CgLaunch L, LgScratch S, uint32_t f, uint32_t fold_what = 0,
                                                          uint32_t N = 0, uint32_t szfl = 0) {
    constexpr int PPT = LG_CHUNK / CG_BLOCK;
    constexpr int NW = (PPT + 63) / 64;
    __shared__ uint32_t cnt[PPT * WAVES];
    __shared__ uint32_t red[8 * WAVES];
    __shared__ uint32_t cbase;
    const uint32_t c = blockIdx.x, tid = threadIdx.x, l = lane_id(), w = wave_id();
    const uint64_t base = (uint64_t)c * LG_CHUNK;
    const uint8_t* fb = L.in + (uint64_t)f * L.frame_stride + base * L.point_step;
    __shared__ uint32_t pw[WAVES];
    uint32_t pre = 0;
    for (uint32_t t = tid; t < c; t += CG_BLOCK) pre += S.chunk_cnt[t];
    pre = wave_sum(pre);
    if (l == 0) pw[w] = pre;
    LaneBits<NW> m;
#pragma unroll
    for (int wi = 0; wi < NW; wi++) m.w[wi] = S.keep[((uint64_t)c * CG_BLOCK + tid) * NW + wi];
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        const uint64_t bb = __ballot(m.get(k));
        if (l == 0) cnt[k * WAVES + w] = (uint32_t)__popcll(bb);
    }
    __syncthreads();
    if (tid == 0) {
        uint32_t t = 0;
        for (int q = 0; q < WAVES; q++) t += pw[q];
        cbase = t;
    }
    const uint32_t tot = block_scan(PPT * WAVES, [&](uint32_t i) -> uint32_t { return cnt[i]; },
                                    [&](uint32_t i, uint32_t e) { cnt[i] = e; }, red);
    if (tid == 0) {
        if (fold_what) st_rlx(S.cstat + (uint64_t)c * LG_CS_WORDS + LG_CS_MS, tot);
        else S.cstat[(uint64_t)c * LG_CS_WORDS + LG_CS_MS] = tot;
    }
    const uint32_t b0 = cbase;
    const uint64_t lt = (1ull << l) - 1ull;
    const uint32_t pidx0 = S.pidx_base + (uint32_t)base;
    Bounds bd;
#pragma unroll
    for (int k0 = 0; k0 < PPT; k0 += 4) {   // four loads in flight
        bool has[4];
        uint32_t pos[4];
        float4 pt[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const int k = k0 + q;
            has[q] = m.get(k);
            const uint64_t bb = __ballot(has[q]);
            pos[q] = b0 + cnt[k * WAVES + w] + (uint32_t)__popcll(bb & lt);
            if (has[q]) pt[q] = load_xyzi<LAYOUT>(fb, (uint32_t)k * CG_BLOCK + tid, L);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (!has[q]) continue;
            S.surv_p[pos[q]] = pt[q];
            S.surv_i[pos[q]] = pidx0 + (uint32_t)(k0 + q) * CG_BLOCK + tid;
            bd.add(pt[q]);
        }
    }
    __shared__ uint32_t part[7 * WAVES];
    bd.merge_block(S.cstat + (uint64_t)c * LG_CS_WORDS, part, fold_what != 0);
    if (!fold_what) return;
    __shared__ uint32_t last;
    __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0): this thread's words are stored
    __syncthreads();
    if (tid == 0) last = lg_last_arrival(lg_arrivals(S, 0));
    __syncthreads();
    if (last) lg_fold_chunks(S, gridDim.x, fold_what, N, szfl, true);
}

// Ground-only output: each chunk's kept points at its stable offset, then the zero pads.
template <int LAYOUT>
__global__ __launch_bounds__(CG_BLOCK, 2) void lg_ground_out(CgLaunch L, CgDevParams P, LgScratch S, uint32_t f) {
    constexpr int PPT = LG_CHUNK / CG_BLOCK;
    constexpr int NW = (PPT + 63) / 64;
    __shared__ uint32_t cnt[PPT * WAVES];
    __shared__ uint32_t red[8 * WAVES];
    __shared__ uint32_t chunk_off;
    const uint32_t c = blockIdx.x, tid = threadIdx.x, l = lane_id(), w = wave_id();
    const uint64_t base = (uint64_t)c * LG_CHUNK;
    const uint32_t N = L.n_points;
    const uint8_t* fb = L.in + (uint64_t)f * L.frame_stride + base * L.point_step;
    LaneBits<NW> keep;
#pragma unroll
    for (int wi = 0; wi < NW; wi++) keep.w[wi] = S.keep[((uint64_t)c * CG_BLOCK + tid) * NW + wi];
    if (w == 0) {   // kept points of the chunks before this one
        uint32_t o = 0;
        for (uint32_t q = l; q < c; q += 64) o += S.chunk_cnt[q];
        o = wave_sum(o);
        if (l == 0) chunk_off = o;
    }
#pragma unroll 8
    for (int k = 0; k < PPT; k++) {
        const uint64_t bb = __ballot(keep.get(k));
        if (l == 0) cnt[k * WAVES + w] = (uint32_t)__popcll(bb);
    }
    __syncthreads();
    block_scan(PPT * WAVES, [&](uint32_t i) -> uint32_t { return cnt[i]; },
               [&](uint32_t i, uint32_t e) { cnt[i] = e; }, red);
    const uint32_t off = chunk_off;
    float4* out = (float4*)(L.ground + (uint64_t)f * N * 32);
#pragma unroll 4
    for (int k = 0; k < PPT; k++) {
        const bool kp = keep.get(k);
        const uint64_t bb = __ballot(kp);
        if (kp) {
            const uint32_t i = (uint32_t)k * CG_BLOCK + tid;
            const uint32_t dst = off + cnt[k * WAVES + w] + (uint32_t)__popcll(bb & ((1ull << l) - 1ull));
            const float4 pp = load_xyzi<LAYOUT>(fb, i, L);
            out[2 * dst] = make_float4(pp.x, pp.y, pp.z, 1.0f);
            out[2 * dst + 1] = make_float4(pp.w, 0.f, 0.f, 0.f);
        }
    }
    // zero pads (src/ground_removal.cpp:79): PointXYZI() after the K kept points
    const uint32_t K = S.meta[LG_K];
    for (uint64_t j = (uint64_t)K + (uint64_t)c * CG_BLOCK + tid; j < N; j += (uint64_t)gridDim.x * CG_BLOCK) {
        out[2 * j] = make_float4(0.f, 0.f, 0.f, 1.0f);
        out[2 * j + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
    }
    if (c == 0 && tid == 0) {
        uint32_t* h = L.hdr + (uint64_t)f * 8;
        h[0] = N; h[1] = K; h[2] = 0; h[3] = 0; h[4] = 0; h[5] = 0;
    }
}

// ------------------------------------------------------------------------------------------
// Single-pass device-wide scans (decoupled look-back). A tile takes a ticket when it starts,
// so it only ever waits on tiles already running; it publishes its count (LG_ST_A), sums the
// tiles before it (the nearest inclusive prefix, LG_ST_P, ends the walk) and publishes its own
// prefix. The last tile to finish zeroes the status words for the next launch (the scratch
// starts zeroed). st: [0] tickets, [1] finished tiles, [2 + t] tile t's status.
#define LG_ST_A 0x40000000u
#define LG_ST_P 0x80000000u
#define LG_ST_V 0x3fffffffu   // counts < 2^30 (frames of <= CG_MAX_FRAME_POINTS points)
__device__ __forceinline__ uint32_t lg_tile_ticket(uint32_t* st) {
    __shared__ uint32_t tk;
    if (threadIdx.x == 0) tk = __hip_atomic_fetch_add(&st[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
    return tk;
}
// Wave 0 of tile t: publish count, return the exclusive prefix of the tiles before t.
__device__ __forceinline__ uint32_t lg_lookback(uint32_t* st, uint32_t t, uint32_t count) {
    uint32_t* ts = st + 2;
    const uint32_t l = lane_id();
    if (t == 0) {
        if (l == 0) __hip_atomic_store(&ts[0], LG_ST_P | count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (l == 0) __hip_atomic_store(&ts[t], LG_ST_A | count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t base = 0;
    int32_t hi = (int32_t)t - 1;
    for (;;) {
        const int32_t j = hi - (int32_t)l;
        const uint32_t w = j >= 0 ? __hip_atomic_load(&ts[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : LG_ST_P;
        const uint64_t pm = __ballot((w & LG_ST_P) != 0u);
        const uint32_t first = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;
        if (__ballot(w == 0u && l < first)) {   // a tile before the nearest prefix not published yet
            __builtin_amdgcn_s_sleep(1);
            continue;
        }
        base += wave_sum(l <= first ? (w & LG_ST_V) : 0u);
        if (first < 64u) break;
        hi -= 64;
    }
    if (l == 0) __hip_atomic_store(&ts[t], LG_ST_P | (base + count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return base;
}
// Every thread of the block, after its look-back: the last tile resets the status words.
__device__ __forceinline__ void lg_tile_done(uint32_t* st, uint32_t active) {
    __shared__ uint32_t last;
    __syncthreads();
    // The status words are the only data the tiles exchange, and they are device-coherent
    // atomics, so nothing needs a release (an agent-scope release writes back the XCD's whole
    // L2). Only the zeroing must not overtake a tile's final status store: the thread that
    // made it (lane 0 of wave 0) waits for its stores to complete (vmcnt(0)) before counting
    // the tile done.
    if (threadIdx.x == 0) {
        __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
        last = __hip_atomic_fetch_add(&st[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == active - 1;
    }
    __syncthreads();
    if (last)
        for (uint32_t i = threadIdx.x; i < active + 2; i += CG_BLOCK) st[i] = 0;
}
// Block-wide: this tile's eight-per-thread counts c -> each thread's exclusive position;
// returns through tot_out the device-wide total when this is the last active tile.
__device__ __forceinline__ uint32_t lg_tile_scan(uint32_t* st, uint32_t t, uint32_t active, uint32_t c,
                                                 uint32_t* total) {
    __shared__ uint32_t red[WAVES];
    __shared__ uint32_t tbase;
    const uint32_t inc = wave_incl_scan(c);
    if (lane_id() == 63) red[wave_id()] = inc;
    __syncthreads();
    if (wave_id() == 0) {
        const uint32_t tot = wave_sum(lane_id() < WAVES ? red[lane_id()] : 0u);
        const uint32_t base = lg_lookback(st, t, tot);
        if (lane_id() == 0) {
            tbase = base;
            if (t == active - 1 && total) *total = base + tot;
        }
    }
    __syncthreads();
    uint32_t pos = tbase + inc - c;
    for (uint32_t w = 0; w < wave_id(); w++) pos += red[w];
    return pos;
}

// Exclusive scan of flag(i) over i < n (count from meta[n_word] when n_word >= 0), calling
// emit(i, position) for every flagged i; the total goes to meta[total_word]. One launch, tiles
// of PER * CG_BLOCK elements (fewer per tile spread a short scan's loads over more CUs).
template <class FLAG, class EMIT, int PER = 8>
__global__ __launch_bounds__(CG_BLOCK) void lg_scan_emit(uint32_t n, int n_word, uint32_t* meta, FLAG flag,
                                                         EMIT emit, uint32_t* st, int total_word) {
    constexpr uint32_t TILE = PER * CG_BLOCK;
    if (n_word >= 0) n = meta[n_word];
    const uint32_t active = n ? (n + TILE - 1) / TILE : 1u;
    if (blockIdx.x >= active) return;
    const uint32_t t = lg_tile_ticket(st);
    const uint64_t b0 = (uint64_t)t * TILE + (uint64_t)threadIdx.x * PER;
    uint32_t fl[PER], c = 0;
#pragma unroll
    for (int q = 0; q < PER; q++) { fl[q] = (b0 + q < n) ? flag((uint32_t)(b0 + q)) : 0u; c += fl[q]; }
    uint32_t pos = lg_tile_scan(st, t, active, c, meta + total_word);
#pragma unroll
    for (int q = 0; q < PER; q++)
        if (fl[q]) emit((uint32_t)(b0 + q), pos++);
    lg_tile_done(st, active);
}

// The device-sized pipeline frame's decisions and survivors in one launch (lg_decide with the
// front's keys folded, then lg_surv_write): a workgroup takes its chunk by ticket (so the chunk
// look-back below only waits on chunks already running), decides the chunk's points, and the
// chunk's survivor count goes through a decoupled look-back over the chunks (S.sstat) for its
// base in frame-index order, instead of a launch boundary and a prefix over the chunk counts.
// The chunk's K, survivor count and bounds leave with sc1 stores; the last workgroup to arrive
// (lg_last_arrival, after each workgroup's storing thread waited for its stores) resets the
// look-back words and folds the chunks into the meta words, sizing the backend.
template <int LAYOUT>
__global__ __launch_bounds__(CG_BLOCK, 2) void lg_decide_write(CgLaunch L, CgDevParams P, LgScratch S, uint32_t f,
                                                              uint32_t nch, uint32_t N, uint32_t szfl) {
    constexpr int PPT = LG_CHUNK / CG_BLOCK;
    constexpr int NW = (PPT + 63) / 64;
    __shared__ float thr[CG_NUM_BINS + 1];
    __shared__ uint32_t tkey[CG_NUM_BINS + 1], band[2], kw[WAVES], tk, cbase, last;
    __shared__ uint32_t fk[CG_NUM_BINS + 2];
    __shared__ uint32_t part[16][LG_CS_WORDS];
    __shared__ uint32_t cnt[PPT * WAVES];
    __shared__ uint32_t red[8 * WAVES];
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    // the ticket from the last wave, so that the other waves' fold loads overlap its latency
    if (tid == CG_BLOCK - 1) tk = __hip_atomic_fetch_add(&S.sstat[0], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x == 0) CG_HOOK_LG_STAMP(S, 0);
    {
        const uint32_t a = lg_fold_core(S, nch, LG_WM_KEYS | LG_WM_TOUCHED, part);   // (ends with a barrier)
        if (tid <= CG_NUM_BINS + 1) fk[tid] = a;   // (LG_CS_KEYS = 0, LG_CS_TOUCHED = CG_NUM_BINS + 1)
    }
    __syncthreads();
    const uint32_t c = tk;
    if (c == 0 && tid <= CG_NUM_BINS) S.meta[LG_SECKEY + tid] = fk[tid];
    if (c == 0 && tid == LG_CS_TOUCHED) S.meta[LG_TOUCHED] = fk[LG_CS_TOUCHED];
    if (tid < 64) sector_thresholds(fk, fk[LG_CS_TOUCHED], P, thr, tkey, &band[0], &band[1]);
    if (c == 0 && tid <= CG_NUM_BINS && L.seckeys) L.seckeys[(uint64_t)f * (CG_NUM_BINS + 1) + tid] = fk[tid];
    __syncthreads();
    if (blockIdx.x == 0) CG_HOOK_LG_STAMP(S, 13);
    const uint64_t base = (uint64_t)c * LG_CHUNK;
    const uint32_t Nc = (uint32_t)min((uint64_t)LG_CHUNK, (uint64_t)L.n_points - base);
    const uint8_t* fb = L.in + (uint64_t)f * L.frame_stride + base * L.point_step;
    const uint2* codes = (const uint2*)S.codes + (uint64_t)c * (LG_CHUNK / 8);
    LaneBits<NW> keep;
    pass2_keep<PPT, LAYOUT>(fb, Nc, L, P, band[0], band[1], tkey, [&](int g) { return codes[g * CG_BLOCK + tid]; },
                            keep);
    const uint32_t kc = wave_sum(keep.count());
    LaneBits<NW> m;   // kept by the ground filter and by the position filter
#pragma unroll
    for (int wi = 0; wi < NW; wi++) m.w[wi] = keep.w[wi] & S.keep[((uint64_t)c * CG_BLOCK + tid) * NW + wi];
    // the survivors' points: loaded now, so that their latency overlaps the scans below (only
    // their stores wait for the chunk's base), and their bounds taken before it
    float4 pt[PPT];
#pragma unroll
    for (int k = 0; k < PPT; k++)
        if (m.get(k)) pt[k] = load_xyzi<LAYOUT>(fb, (uint32_t)k * CG_BLOCK + tid, L);
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        const uint64_t bb = __ballot(m.get(k));
        if (l == 0) cnt[k * WAVES + w] = (uint32_t)__popcll(bb);
    }
    if (l == 0) kw[w] = kc;
    __syncthreads();
    const uint32_t tot = block_scan(PPT * WAVES, [&](uint32_t i) -> uint32_t { return cnt[i]; },
                                    [&](uint32_t i, uint32_t e) { cnt[i] = e; }, red);
    if (w == 0) {   // the chunks before this one (their survivor counts), then this chunk's words
        const uint32_t b = lg_lookback(S.sstat, c, tot);
        if (l == 0) {
            cbase = b;
            uint32_t k = 0;
            for (int q = 0; q < WAVES; q++) k += kw[q];
            st_rlx(S.cstat + (uint64_t)c * LG_CS_WORDS + LG_CS_K, k);
            st_rlx(S.cstat + (uint64_t)c * LG_CS_WORDS + LG_CS_MS, tot);
        }
    }
    Bounds bd;
#pragma unroll
    for (int k = 0; k < PPT; k++)
        if (m.get(k)) bd.add(pt[k]);
    __shared__ uint32_t bpart[7 * WAVES];
    bd.merge_block(S.cstat + (uint64_t)c * LG_CS_WORDS, bpart, true);   // (thread 0 stores; ends after a barrier)
    if (blockIdx.x == 0) CG_HOOK_LG_STAMP(S, 14);
    const uint32_t b0 = cbase;
    const uint64_t lt = (1ull << l) - 1ull;
    const uint32_t pidx0 = S.pidx_base + (uint32_t)base;
#pragma unroll
    for (int k = 0; k < PPT; k++) {
        const bool has = m.get(k);
        const uint64_t bb = __ballot(has);
        if (!has) continue;
        const uint32_t pos = b0 + cnt[k * WAVES + w] + (uint32_t)__popcll(bb & lt);
        S.surv_p[pos] = pt[k];
        S.surv_i[pos] = pidx0 + (uint32_t)k * CG_BLOCK + tid;
    }
    if (tid == 0) {
        __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0): its words and status are stored
        last = lg_last_arrival(lg_arrivals(S, 0));
    }
    __syncthreads();
    if (!last) return;
    for (uint32_t i = tid; i < nch + 2; i += CG_BLOCK) st_rlx(&S.sstat[i], 0u);   // (lg_tile_done's reset)
    lg_fold_chunks(S, nch, 2u | 4u | LG_FOLD_SIZE, N, szfl, true);
    CG_HOOK_LG_STAMP(S, 15);
}

// ------------------------------------------------------------------------------------------
// Stable LSD radix sort of (64-bit key, 32-bit value) pairs, 8 bits per pass, tiles of
// LG_RS_TILE elements (LG_RS_ROUNDS rounds of 512 per workgroup).
#define LG_RS_ROUNDS 2
#define LG_RS_TILE (LG_RS_ROUNDS * CG_BLOCK)
__global__ __launch_bounds__(CG_BLOCK) void lg_rs_hist(const uint64_t* key, uint32_t n, uint32_t shift,
                                                       uint32_t* hist, const uint32_t* n_dev, const uint32_t* lim) {
    __shared__ uint32_t h[256];
    if (n_dev) n = *n_dev;   // count known on the device only (grid sized for an upper bound)
    if (lim && shift >= *lim) return;   // key width known on the device only: an identity pass
    if ((uint64_t)blockIdx.x * LG_RS_TILE >= n) return;   // (read by the tiles below n only)
    if (threadIdx.x < 256) h[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * LG_RS_TILE;
    for (int q = 0; q < LG_RS_ROUNDS; q++) {
        const uint64_t i = b0 + (uint64_t)q * CG_BLOCK + threadIdx.x;
        if (i < n) atomicAdd(&h[(key[i] >> shift) & 255u], 1u);
    }
    __syncthreads();
    const uint32_t nt = (uint32_t)(((uint64_t)n + LG_RS_TILE - 1) / LG_RS_TILE);   // tiles holding elements
    if (threadIdx.x < 256) hist[threadIdx.x * nt + blockIdx.x] = h[threadIdx.x];
}
// hist (raw counts, digit-major) gives each (digit, tile) its output base. Within a tile the
// elements go in 8 rounds of 512 in index order; a round ranks equal digits per wave with
// eight ballots (the wave's lanes whose digit matches bit for bit) and offsets waves by the
// per-wave digit counts of the round, so equal keys keep their input order (stable).
// skip (with lim): a pass past the keys' width does nothing (the consumer reads the buffer the
// last real pass wrote, lg_rs_passes); without skip it is a copy.
__global__ __launch_bounds__(CG_BLOCK) void lg_rs_scatter(const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                                          uint32_t* vout, uint32_t n, uint32_t shift,
                                                          const uint32_t* hist, const uint32_t* n_dev,
                                                          const uint32_t* lim, uint32_t skip) {
    if (n_dev) n = *n_dev;
    if (lim && shift >= *lim && skip) return;
    if ((uint64_t)blockIdx.x * LG_RS_TILE >= n) return;
    if (lim && shift >= *lim) {   // digits past the keys' width: the pass is a copy
        for (int q = 0; q < LG_RS_ROUNDS; q++) {
            const uint64_t i = (uint64_t)blockIdx.x * LG_RS_TILE + (uint64_t)q * CG_BLOCK + threadIdx.x;
            if (i < n) { kout[i] = kin[i]; vout[i] = vin[i]; }
        }
        return;
    }
    __shared__ uint32_t run[256];
    __shared__ uint32_t wcnt[WAVES][256];
    __shared__ uint32_t red[8 * WAVES];
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    // this tile's base per digit from the raw (digit-major) counts: the digit's offset (all
    // tiles' counts of smaller digits) plus its count in the tiles before this one
    {
        // the tiles holding elements (the grid may be sized for an upper bound of n)
        const uint32_t nt = (uint32_t)(((uint64_t)n + LG_RS_TILE - 1) / LG_RS_TILE), b = blockIdx.x;
        uint32_t tot = 0, pre = 0;
        if (tid < 256) {   // eight count loads in flight (a dependent walk costs an L2 trip per tile)
            const uint32_t* h = hist + (uint64_t)tid * nt;
            uint32_t t = 0;
            for (; t + 8 <= nt; t += 8) {
                uint32_t c[8];
#pragma unroll
                for (int u = 0; u < 8; u++) c[u] = h[t + u];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    tot += c[u];
                    pre += t + u < b ? c[u] : 0u;
                }
            }
            for (; t < nt; t++) {
                const uint32_t c = h[t];
                tot += c;
                pre += t < b ? c : 0u;
            }
        }
        block_scan(256, [&](uint32_t i) -> uint32_t { return tot; },
                   [&](uint32_t i, uint32_t e) { run[i] = e + pre; }, red);
    }
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * LG_RS_TILE;
    const uint64_t lt = (1ull << l) - 1ull;
    for (int q = 0; q < LG_RS_ROUNDS; q++) {
        for (uint32_t x = tid; x < WAVES * 256; x += CG_BLOCK) (&wcnt[0][0])[x] = 0;
        __syncthreads();
        const uint64_t i = b0 + (uint64_t)q * CG_BLOCK + tid;
        const bool valid = i < n;
        uint64_t k = 0;
        uint32_t v = 0, d = 0;
        if (valid) { k = kin[i]; v = vin[i]; d = (uint32_t)(k >> shift) & 255u; }
        uint64_t m = __ballot(valid);
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const uint64_t bb = __ballot((d >> b) & 1u);
            m &= ((d >> b) & 1u) ? bb : ~bb;
        }
        const uint32_t rank = (uint32_t)__popcll(m & lt);
        if (valid && rank == 0) wcnt[w][d] = (uint32_t)__popcll(m);
        __syncthreads();
        if (valid) {
            uint32_t pos = run[d] + rank;
            for (uint32_t u = 0; u < w; u++) pos += wcnt[u][d];
            kout[pos] = k;
            vout[pos] = v;
        }
        __syncthreads();
        if (tid < 256) {
            uint32_t t = 0;
            for (int u = 0; u < WAVES; u++) t += wcnt[u][tid];
            run[tid] += t;
        }
        __syncthreads();
    }
}

namespace {

uint32_t tiles_of(uint64_t n) { return (uint32_t)((n + LG_TILE - 1) / LG_TILE); }
// wave-per-item launches whose count (V, C) is known on the device only: a grid-stride loop
// over at most 1024 workgroups (the chip's 8192 wave slots) instead of one wave per upper bound
uint32_t lg_wave_blocks(uint64_t n) {
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>((n + WAVES - 1) / WAVES, 1024));
}
uint32_t blocks_of(uint64_t n) { return (uint32_t)((n + CG_BLOCK - 1) / CG_BLOCK); }
uint32_t bits_of(uint64_t v) { return cg_bits_of(v); }

// Stable sort of n pairs in (k[0], v[0]) by key bits [lo, bits); returns the buffer index (0 or
// 1) that holds the result. The pairs are already in order of the bits below lo. With n_dev,
// the count is read on the device and n is only its upper bound.
// skip (with lim): passes past the device-side key width do nothing instead of copying; the
// result's buffer is then lg_rs_passes(lo, bits, *lim) & 1, known on the device only (returns -1).
int radix_sort(LgScratch& S, uint32_t n, uint32_t bits, hipStream_t s, uint32_t lo = 0,
               const uint32_t* n_dev = nullptr, const uint32_t* lim = nullptr, bool skip = false) {
    uint64_t* k[2] = {S.key0, S.key1};
    uint32_t* v[2] = {S.val0, S.val1};
    int cur = 0;
    if (n <= 1 && !n_dev) return cur;
    const uint32_t nt = std::max<uint32_t>(1, (uint32_t)(((uint64_t)n + LG_RS_TILE - 1) / LG_RS_TILE));
    for (uint32_t shift = lo; shift < bits; shift += 8) {
        hipLaunchKernelGGL(lg_rs_hist, dim3(nt), dim3(CG_BLOCK), 0, s, k[cur], n, shift, S.hist, n_dev, lim);
        hipLaunchKernelGGL(lg_rs_scatter, dim3(nt), dim3(CG_BLOCK), 0, s, k[cur], v[cur], k[cur ^ 1], v[cur ^ 1], n,
                           shift, S.hist, n_dev, lim, skip ? 1u : 0u);
        cur ^= 1;
    }
    return skip && lim ? -1 : cur;
}

}  // namespace

// The LSD passes at shifts [lo, hi) that the device-side key width (*lim) still needs, after the
// first pass of a sort whose data are now in buffer 1, by one workgroup (an identity launch for
// the usual key widths: the CSR's cluster ranks fit one 8-bit digit below 255 clusters). Stable:
// the tiles go in order, a tile's equal digits ranked in lane order by ballots as lg_rs_scatter.
__global__ __launch_bounds__(CG_BLOCK) void lg_rs_rest(LgScratch S, uint32_t lo, uint32_t hi, const uint32_t* n_dev,
                                                       const uint32_t* lim) {
    const uint32_t top = min(hi, *lim);
    if (lo >= top) return;
    __shared__ uint32_t base[256];
    __shared__ uint32_t wcnt[WAVES][256];
    __shared__ uint32_t red[8 * WAVES];
    const uint32_t n = *n_dev, tid = threadIdx.x, l = lane_id(), w = wave_id();
    const uint64_t lt = (1ull << l) - 1ull;
    int cur = 1;
    for (uint32_t shift = lo; shift < top; shift += 8, cur ^= 1) {
        const uint64_t* kin = cur ? S.key1 : S.key0;
        const uint32_t* vin = cur ? S.val1 : S.val0;
        uint64_t* kout = cur ? S.key0 : S.key1;
        uint32_t* vout = cur ? S.val0 : S.val1;
        if (tid < 256) base[tid] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < n; i += CG_BLOCK) atomicAdd(&base[(kin[i] >> shift) & 255u], 1u);
        __syncthreads();
        block_scan(256, [&](uint32_t d) -> uint32_t { return base[d]; }, [&](uint32_t d, uint32_t e) { base[d] = e; }, red);
        for (uint32_t t0 = 0; t0 < n; t0 += CG_BLOCK) {
            for (uint32_t x = tid; x < WAVES * 256; x += CG_BLOCK) (&wcnt[0][0])[x] = 0;
            __syncthreads();
            const uint32_t i = t0 + tid;
            const bool valid = i < n;
            uint64_t k = 0;
            uint32_t v = 0, d = 0;
            if (valid) { k = kin[i]; v = vin[i]; d = (uint32_t)(k >> shift) & 255u; }
            uint64_t m = __ballot(valid);
#pragma unroll
            for (int b = 0; b < 8; b++) {
                const uint64_t bb = __ballot((d >> b) & 1u);
                m &= ((d >> b) & 1u) ? bb : ~bb;
            }
            const uint32_t rank = (uint32_t)__popcll(m & lt);
            if (valid && rank == 0) wcnt[w][d] = (uint32_t)__popcll(m);
            __syncthreads();
            if (valid) {
                uint32_t pos = base[d] + rank;
                for (uint32_t u = 0; u < w; u++) pos += wcnt[u][d];
                kout[pos] = k;
                vout[pos] = v;
            }
            __syncthreads();
            if (tid < 256) {
                uint32_t t = 0;
                for (int u = 0; u < WAVES; u++) t += wcnt[u][tid];
                base[tid] += t;
            }
            __syncthreads();
        }
    }
}

namespace {
template <int PER = 8, class FLAG, class EMIT>
void scan_emit(LgScratch& S, uint32_t n_max, int n_word, FLAG flag, EMIT emit, int total_word, hipStream_t s) {
    const uint32_t nt = std::max<uint32_t>(1, (uint32_t)((n_max + PER * CG_BLOCK - 1) / (PER * CG_BLOCK)));
    hipLaunchKernelGGL((lg_scan_emit<FLAG, EMIT, PER>), dim3(nt), dim3(CG_BLOCK), 0, s, n_max, n_word, S.meta, flag,
                       emit, S.sstat, total_word);
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Global backend (M > CG_MMAX). The detector's input is the M = Ms + npad points: survivors
// (surv_p / surv_i, any order; frame index pidx) and npad PointXYZI() pads after every kept
// point (pidx = N + j). PB bits hold a pidx.
__device__ __forceinline__ float4 lg_point(const LgScratch& S, uint32_t j, uint32_t Ms) {
    return j < Ms ? S.surv_p[j] : make_float4(0.f, 0.f, 0.f, 0.f);
}

// pcl::VoxelGrid setup from the bounds (getMinMax3D + the int64 overflow guard)
// (one thread; reads the bounds words of in, writes the grid words of m)
__device__ void lg_grid_setup(const uint32_t* in, uint32_t* m, const CgDevParams& P, uint32_t npad, uint32_t Mtot) {
    float bmn[3], bmx[3];
    uint32_t nfin = in[LG_NFIN];
    for (int a = 0; a < 3; a++) {
        bmn[a] = nfin ? cg_fkey_inv(in[LG_BMIN + a]) : INFINITY;
        bmx[a] = nfin ? cg_fkey_inv(in[LG_BMAX + a]) : -INFINITY;
        if (npad) { bmn[a] = fminf(bmn[a], 0.f); bmx[a] = fmaxf(bmx[a], 0.f); }
    }
    nfin += npad;
    uint32_t pass = 0;
    int min_b[3] = {0, 0, 0}, div_b[3] = {1, 1, 1};
    voxel_grid_setup(nfin, bmn, bmx, P, pass, min_b, div_b);
    m[LG_NFIN_ALL] = nfin;
    m[LG_PASS] = pass;
    m[LG_SCAN_N] = pass ? Mtot : nfin;   // runs over the finite points, or every point
    for (int a = 0; a < 3; a++) m[LG_MINB + a] = (uint32_t)min_b[a];
    m[LG_MUL1] = (uint32_t)div_b[0];
    m[LG_MUL2] = (uint32_t)div_b[0] * (uint32_t)div_b[1];
    m[LG_ORG + 0] = __float_as_uint(nfin ? bmn[0] : 0.f);
    m[LG_ORG + 1] = __float_as_uint(nfin ? bmn[1] : 0.f);
    m[LG_ORG + 2] = __float_as_uint(nfin ? bmn[2] : 0.f);
    // dense neighbour grid over the bounds: cells of edge >= 1.0625 tol (so an edge joins
    // voxels in adjacent cells), widened where an axis would need more than LG_DGRID_AXIS
    uint32_t ncell = 1;
    for (int a = 0; a < 3; a++) {
        const float ext = nfin ? bmx[a] - bmn[a] : 0.f;
        const float q = floorf(ext * P.cell_inv);
        float inv = P.cell_inv;
        uint32_t n = 1;
        if (q >= (float)(LG_DGRID_AXIS - 1)) {          // ext / 127 > 1.0625 tol
            inv = (float)(LG_DGRID_AXIS - 1) / ext;     // an infinite extent: one cell (inv 0)
            n = LG_DGRID_AXIS;
        } else if (q >= 0.f) {
            n = (uint32_t)q + 1;
        }
        m[LG_DGINV + a] = __float_as_uint(inv);
        m[LG_DGN + a] = n;
        ncell *= n;
    }
    m[LG_NCELL] = ncell;
}

// PCL order's partition levels (lg_pq_*, below): sizes and the range lists' header words
#define LG_PCL_LEAF 4096       // the longest leaf sorted in LDS
#ifndef LG_PCL_CUT
// the levels cut ranges longer than this; the leaves take up to LG_PCL_LEAF, so a range an
// uneven last cut leaves between the two still sorts in LDS (4,096 against 2,048 on C5:
// 271 / 268 us per frame, profiles/r5_c5_cut_ab.txt; with the flow launch 3,072 / 4,096 /
// 2,048: 246-247 / 239-240 / 235-237 us, profiles/r6_c5_cut_ab.txt)
#define LG_PCL_CUT 2048
#endif
#define LG_PQ_HDR 8            // [0..2] level list counts, [3] leaf count, [4] [5] level-0 nL / nR,
                               // [6] (unused), [7] mid tasks (lg_pcl_mid)
#define PQ_MIDS 7
#define PQ_TILES 8             // S.ca: [0] a level's tile count; from word 8, eight words per tile
                               // (range, median, pivot, budget, range index, tile in range):
                               // lg_pq_split -> lg_pq_swap (<= 8 (N / 512 + 2048) + 8 words)
#define PQ_LEAFLIST 3
#define PQ_EW 5                // entry words: first, last, depth, then nL, nR (levels) / buffer (leaves)
#define PQ_T CG_BLOCK          // elements per tile
#define PQ_MAXR 2048           // ranges per level (levels <= 11)
#define LG_PQ_LEVELS_MAX 11
#define LG_PQ_CAP ((2u << LG_PQ_LEVELS_MAX) + 64)   // entries per list: a level pushes <= 2 per range

// keys: passthrough -> pidx; else (PCL idx << PB | pidx), non-finite idx = 0xffffffff (last)
// Every workgroup derives the grid words from the bounds (lg_grid_setup); workgroup 0 also
// stores them in the meta words for the kernels after it (a halo slab: with its own count of
// finite points, nfin_local, for the voxel runs).
// Mtot = CG_K_FROM_META (the backend sized on the device): Mtot and npad from the meta words
// (LG_MTOT, LG_NPAD; the grid sized for the frame's N); Mtot 0 (the LDS backend takes the frame)
// leaves every later global-backend launch without work.
__global__ __launch_bounds__(CG_BLOCK) void lg_voxel_keys(LgScratch S, CgDevParams P, uint32_t Mtot, uint32_t N,
                                                          uint32_t PB, uint32_t npad,
                                                          uint32_t nfin_local = 0xffffffffu) {
    __shared__ uint32_t m[LG_META_WORDS];
    const uint32_t j = blockIdx.x * CG_BLOCK + threadIdx.x;
    const bool dev = Mtot == CG_K_FROM_META;
    const uint32_t* in = S.meta;   // the counts and bounds words
    if (dev) {
        Mtot = in[LG_MTOT];
        npad = in[LG_NPAD];
    }
    if (threadIdx.x == 0) {
        lg_grid_setup(in, m, P, npad, Mtot);
        if (dev && Mtot == 0) m[LG_NCELL] = 0;
        if (blockIdx.x == 0) {
            lg_grid_setup(in, S.meta, P, npad, Mtot);
            if (nfin_local != 0xffffffffu) S.meta[LG_NFIN_ALL] = S.meta[LG_SCAN_N] = nfin_local;
            if (dev && Mtot == 0) S.meta[LG_NFIN_ALL] = S.meta[LG_SCAN_N] = S.meta[LG_NCELL] = 0;
        }
    }
    __syncthreads();
    {   // the dense neighbour grid's cell counts (lg_voxel_centroids), ncell from lg_grid_setup
        const uint32_t nc = m[LG_NCELL] + 1;
        for (uint32_t i = j; i < nc; i += gridDim.x * CG_BLOCK) S.cstart[i] = 0;
    }
    if (j >= Mtot) return;
    const uint32_t Ms = in[LG_MS];
    const float4 p = lg_point(S, j, Ms);
    const uint64_t pidx = j < Ms ? S.surv_i[j] : (uint64_t)N + (j - Ms);
    // PB = 0 (survivors in frame-index order): a stable sort by idx alone keeps each voxel's
    // points in frame-index order; otherwise the frame index is the key's low part
    uint64_t key;
    if (m[LG_PASS]) {
        key = PB ? pidx : 0ull;
    } else if (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) {
        key = (0xffffffffull << PB) | (PB ? pidx : 0ull);
    } else {
        const float mnb0 = (float)(int)m[LG_MINB], mnb1 = (float)(int)m[LG_MINB + 1], mnb2 = (float)(int)m[LG_MINB + 2];
        const int i0 = (int)(floorf(p.x * P.inv_leaf[0]) - mnb0);
        const int i1 = (int)(floorf(p.y * P.inv_leaf[1]) - mnb1);
        const int i2 = (int)(floorf(p.z * P.inv_leaf[2]) - mnb2);
        const uint32_t idx = (uint32_t)i0 + (uint32_t)i1 * m[LG_MUL1] + (uint32_t)i2 * m[LG_MUL2];
        key = ((uint64_t)idx << PB) | (PB ? pidx : 0ull);
    }
    S.key0[j] = key;
    S.val0[j] = j;
}

struct VoxelHead {   // start of a voxel run among the finite points (every point if passthrough)
    const uint64_t* key; const uint32_t* meta; uint32_t PB;
    __device__ uint32_t operator()(uint32_t r) const {
        if (meta[LG_PASS]) return 1u;
        return (r == 0 || (key[r] >> PB) != (key[r - 1] >> PB)) ? 1u : 0u;
    }
};
struct VoxelEmit {
    uint32_t* run;
    __device__ void operator()(uint32_t r, uint32_t v) const { run[v] = r; }
};

// The dense neighbour grid of the clustering (its words from lg_grid_setup, in meta).
__device__ __forceinline__ uint32_t lg_dcell(float c, float o, float inv, uint32_t n) {
    const float q = floorf((c - o) * inv);
    if (!(q >= 0.f)) return 0u;                      // NaN or below the origin
    return q >= (float)(n - 1) ? n - 1 : (uint32_t)q;   // clamped: a superset of neighbours
}
struct LgGrid {
    float o[3], inv[3];
    uint32_t n[3];
    __device__ explicit LgGrid(const uint32_t* m) {
#pragma unroll
        for (int a = 0; a < 3; a++) {
            o[a] = __uint_as_float(m[LG_ORG + a]);
            inv[a] = __uint_as_float(m[LG_DGINV + a]);
            n[a] = m[LG_DGN + a];
        }
    }
    __device__ void cell(const float4& q, uint32_t& cx, uint32_t& cy, uint32_t& cz) const {
        cx = lg_dcell(q.x, o[0], inv[0], n[0]);
        cy = lg_dcell(q.y, o[1], inv[1], n[1]);
        cz = lg_dcell(q.z, o[2], inv[2], n[2]);
    }
    __device__ uint32_t id(uint32_t cx, uint32_t cy, uint32_t cz) const { return cx + n[0] * (cy + n[1] * cz); }
};
// A voxel's neighbour-grid cell and its slot there (the cell counts; lg_voxel_keys zeroed
// them): written with the voxel's centroid, by the lane that computed it.
__device__ __forceinline__ void lg_dgrid_count_one(const LgScratch& S, uint32_t v, const float4& c) {
    const LgGrid g(S.meta);
    uint32_t cx, cy, cz;
    g.cell(c, cx, cy, cz);
    const uint32_t k = g.id(cx, cy, cz);
    S.uk[v] = k;
    S.ca[v] = atomicAdd(&S.cstart[k], 1u);
}
// Sequential float sums over lanes 0..n-1 of a wave (n wave-uniform), in lane order: blocks
// of eight lanes with immediate lane indices (no lane-select SGPR, no per-member branch);
// the lanes of the last block past n must hold +0.0f.
__device__ __forceinline__ void lg_sum_lanes(uint32_t n, float a, float b, float c, float d, float& sa, float& sb,
                                             float& sc, float& sd) {
#define LG_ACC(k)                                                                \
    sa += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(a), k));       \
    sb += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(b), k));       \
    sc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(c), k));       \
    sd += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(d), k));
#define LG_BLK(k0)                                                                                          \
    if (n > k0) {                                                                                           \
        LG_ACC(k0) LG_ACC(k0 + 1) LG_ACC(k0 + 2) LG_ACC(k0 + 3) LG_ACC(k0 + 4) LG_ACC(k0 + 5) LG_ACC(k0 + 6) \
        LG_ACC(k0 + 7)                                                                                      \
    }
    LG_BLK(0) LG_BLK(8) LG_BLK(16) LG_BLK(24) LG_BLK(32) LG_BLK(40) LG_BLK(48) LG_BLK(56)
#undef LG_BLK
#undef LG_ACC
}

// CentroidPoint: float sums in ascending frame index / float(n); passthrough copies the point.
// One wave per voxel: the lanes fetch 64 members at a time, the sums run through them in
// member order.
__device__ __forceinline__ void lg_voxel_centroids_one(const CgLaunch& L, const LgScratch& S, uint32_t f, int buf,
                                                       uint32_t v) {
    const uint32_t l = lane_id();
    const uint32_t* m = S.meta;
    const uint32_t V = m[LG_V], Ms = m[LG_MS];
    const uint32_t* val = buf ? S.val1 : S.val0;
    float4* vox_out = L.vox + (uint64_t)f * L.cap;
    if (l == 0) {
        S.par[v] = v;
        S.cnt[v] = 0;
        S.rk[v] = 0xffffffffu;
    }
    if (m[LG_PASS]) {
        if (l == 0) {
            const float4 p = lg_point(S, val[v], Ms);
            S.vox[v] = p;
            vox_out[v] = p;
            lg_dgrid_count_one(S, v, p);
        }
        return;
    }
    const uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.run[v]);
    const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)(v + 1 < V ? S.run[v + 1] : m[LG_NFIN_ALL]));
    float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
    for (uint32_t g0 = s; g0 < e; g0 += 64) {
        const uint32_t n = min(64u, e - g0);
        float4 p = make_float4(0.f, 0.f, 0.f, 0.f);
        if (l < n) p = lg_point(S, val[g0 + l], Ms);
        // lanes in blocks of eight with immediate lane indices; a block's lanes past n hold
        // +0.0f, and adding +0.0f to a sum that starts at +0.0f is exact (the sum is never -0.0
        // under round-to-nearest), so the sums are bit-identical to the member-by-member loop
        lg_sum_lanes(n, p.x, p.y, p.z, p.w, sx, sy, sz, si);
    }
    if (l != 0) return;
    const float nn = (float)(e - s);
    const float4 c = make_float4(sx / nn, sy / nn, sz / nn, si / nn);
    S.vox[v] = c;
    vox_out[v] = c;
    lg_dgrid_count_one(S, v, c);
}
__global__ __launch_bounds__(CG_BLOCK) void lg_voxel_centroids(CgLaunch L, LgScratch S, uint32_t f, uint32_t Mtot,
                                                               int buf) {
    for (uint32_t v = blockIdx.x * WAVES + wave_id(), V = S.meta[LG_V]; v < V; v += gridDim.x * WAVES)
        lg_voxel_centroids_one(L, S, f, buf, v);
}

// ------------------------------------------------------------------------------------------
// PCL's voxel order for the global backend (cg_pcl.h has the algorithm). index_vector is the
// finite detector-input points in frame-index order; lg_scan_emit lists them as records
// (idx << 32 | slot) (PclCompact*), then libstdc++'s introsort runs on them level by level.
// Each level of ranges longer than LG_PCL_LEAF is two launches, one workgroup per tile of
// PQ_T elements of a range:
//   lg_pq_split: every tile of a range computes the range's median of three (the swap with the
//     first is virtual: V(m) = E[first], V(first) = E[m]), compares its elements with the
//     pivot, and a decoupled look-back segmented by range (tickets: a tile only waits on tiles
//     already running) gives each element its index in the range's L list (>= pivot, from the
//     left) and in the ascending list of <= pivot elements; both lists are written, and each
//     element's two indices; the range's last tile notes both totals;
//   lg_pq_swap: the k-th swap pairs L_k with R_k (the k-th <= pivot element from the right)
//     while L_k < R_k; each element finds its partner with two list reads and writes V of it
//     (or itself) to the other buffer; the last swap (or L_0 when there is none) computes the
//     cut and queues both children: longer than LG_PCL_LEAF (budget left) for the next level,
//     else as leaves (with the buffer they are in).
// Median-of-three cuts are uneven (C5's index_vector of 49k records takes ~6 levels to reach
// 4096-element ranges), so the host launches three levels more than an even split needs; a
// level with no range returns at once. lg_pcl_leaf finishes each leaf with pcl_block_sort in
// LDS (up to 4096 records, 8 per thread, results straight to the outputs), with the depth
// budget left on its path; a range still longer (a degenerate split) in HBM.
struct PclCompactFlag {   // finite points (non-finite keys carry idx 0xffffffff)
    const uint64_t* key; uint32_t PB;
    const uint32_t* meta;   // (the device-sized path: a passthrough frame lists nothing, so its
                            // points keep lg_voxel_keys' frame-index order: PCL does not sort them)
    __device__ uint32_t operator()(uint32_t j) const {
        if (meta && meta[LG_PASS]) return 0u;
        return (uint32_t)(key[j] >> PB) != 0xffffffffu ? 1u : 0u;
    }
};
struct PclCompactEmit {
    const uint64_t* key; const uint32_t* val; uint64_t* E; uint32_t PB;
    __device__ void operator()(uint32_t j, uint32_t r) const {
        E[r] = ((uint64_t)(uint32_t)(key[j] >> PB) << 32) | val[j];
    }
};

// The device-sized path's index_vector in one launch (lg_voxel_keys + lg_scan_emit with
// PclCompact*): each tile of LG_IDX_TILE survivors computes its points' voxel keys, lists the finite
// ones in frame-index order through the decoupled look-back and writes their (idx << 32 | slot)
// records to Eout; the count goes to meta[LG_PCL_N]. The keys and slots also go to key0 / val0
// (a passthrough frame keeps them as its order). Workgroup 0 writes the grid words to the meta
// words and empties the partition lists; every workgroup zeroes its share of the neighbour
// grid's cell counts (lg_voxel_centroids counts into them). Survivors arrive in frame-index
// order (lg_surv_write), so the keys carry no frame-index bits (PB = 0).
#ifndef LG_IDX_PER
#define LG_IDX_PER 2   // records per thread of lg_pcl_index and the voxel-run scan after the sort
                       // (1, 4 and round 5's first 8 measured slower, profiles/r5_c5_idx_ab.txt)
#endif
#define LG_IDX_TILE (LG_IDX_PER * CG_BLOCK)
__global__ __launch_bounds__(CG_BLOCK) void lg_pcl_index(LgScratch S, CgDevParams P, uint64_t* Eout) {
    __shared__ uint32_t m[LG_META_WORDS];
    const uint32_t tid = threadIdx.x;
    const uint32_t* in = S.meta;
    if (blockIdx.x == 1) CG_HOOK_LG_STAMP(S, 58);
    const uint32_t Mtot = in[LG_MTOT], npad = in[LG_NPAD];
    if (tid == 0) {
        lg_grid_setup(in, m, P, npad, Mtot);
        if (Mtot == 0) m[LG_NCELL] = 0;
        if (blockIdx.x == 0) {
            S.pq[1] = 0; S.pq[2] = 0; S.pq[PQ_LEAFLIST] = 0; S.pq[PQ_MIDS] = 0;
            lg_grid_setup(in, S.meta, P, npad, Mtot);
            if (Mtot == 0) S.meta[LG_NFIN_ALL] = S.meta[LG_SCAN_N] = S.meta[LG_NCELL] = 0;
        }
    }
    __syncthreads();
    if (blockIdx.x == 1) CG_HOOK_LG_STAMP(S, 59);
    {
        const uint32_t nc = m[LG_NCELL] + 1;
        for (uint32_t i = blockIdx.x * CG_BLOCK + tid; i < nc; i += gridDim.x * CG_BLOCK) S.cstart[i] = 0;
    }
    const uint32_t active = Mtot ? (Mtot + LG_IDX_TILE - 1) / LG_IDX_TILE : 1u;
    if (blockIdx.x >= active) return;
    const uint32_t t = lg_tile_ticket(S.sstat);
    if (t == 1) CG_HOOK_LG_STAMP(S, 60);
    const uint64_t b0 = (uint64_t)t * LG_IDX_TILE + (uint64_t)tid * LG_IDX_PER;
    const uint32_t Ms = in[LG_MS];
    const bool pass = m[LG_PASS] != 0;
    const float mnb0 = (float)(int)m[LG_MINB], mnb1 = (float)(int)m[LG_MINB + 1], mnb2 = (float)(int)m[LG_MINB + 2];
    const uint32_t mul1 = m[LG_MUL1], mul2 = m[LG_MUL2];
    uint32_t idx[LG_IDX_PER], c = 0;
    float4 pt[LG_IDX_PER];
#pragma unroll
    for (int q = 0; q < LG_IDX_PER; q++) {   // the points' loads first (clamped: no branch between them)
        const uint32_t j = (uint32_t)min(b0 + q, (uint64_t)(Mtot ? Mtot - 1 : 0));
        pt[q] = j < Ms ? S.surv_p[j] : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int q = 0; q < LG_IDX_PER; q++) {
        const uint64_t j = b0 + q;
        idx[q] = 0xffffffffu;
        if (j < Mtot) {
            const float4 p = pt[q];
            uint64_t key = 0ull;   // passthrough: frame-index order (nothing listed)
            if (!pass) {
                if (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) {
                    key = 0xffffffffull;
                } else {   // lg_voxel_keys's arithmetic
                    const int i0 = (int)(floorf(p.x * P.inv_leaf[0]) - mnb0);
                    const int i1 = (int)(floorf(p.y * P.inv_leaf[1]) - mnb1);
                    const int i2 = (int)(floorf(p.z * P.inv_leaf[2]) - mnb2);
                    key = (uint64_t)((uint32_t)i0 + (uint32_t)i1 * mul1 + (uint32_t)i2 * mul2);
                    idx[q] = (uint32_t)key;
                }
            }
            S.key0[j] = key;
            S.val0[j] = (uint32_t)j;
            c += idx[q] != 0xffffffffu ? 1u : 0u;
        }
    }
    if (t == 1) CG_HOOK_LG_STAMP(S, 61);
    uint32_t pos = lg_tile_scan(S.sstat, t, active, c, S.meta + LG_PCL_N);
    if (t == 1) CG_HOOK_LG_STAMP(S, 62);
#pragma unroll
    for (int q = 0; q < LG_IDX_PER; q++)
        if (idx[q] != 0xffffffffu) Eout[pos++] = ((uint64_t)idx[q] << 32) | (uint32_t)(b0 + q);
    lg_tile_done(S.sstat, active);
    if (t == 1) CG_HOOK_LG_STAMP(S, 63);
}

__device__ __forceinline__ uint32_t pq_key(const uint64_t* E, uint32_t x) {
    return ((const uint32_t*)E)[2 * x + 1];
}
__device__ __forceinline__ uint32_t* pq_list(const LgScratch& S, uint32_t which) {
    return S.pq + LG_PQ_HDR + (uint64_t)which * PQ_EW * LG_PQ_CAP;
}
__device__ __forceinline__ void pq_push(const LgScratch& S, uint32_t which, uint32_t first, uint32_t last, uint32_t depth,
                                        uint32_t w3) {
    const uint32_t i = atomicAdd(&S.pq[which], 1u);
    if (i < LG_PQ_CAP) {
        uint32_t* e = pq_list(S, which) + PQ_EW * i;
        e[0] = first; e[1] = last; e[2] = depth; e[3] = w3;
    } else {
        S.meta[LG_PQ_TIMEOUT] = 1u;   // (a list overflowed: the frame's results are void, never expected)
    }
}
// The ranges of a level (level 0: the whole index_vector when it needs partitioning) and the
// tiles of each: tp[r] = first tile of range r (block-wide, ends with a barrier). Returns the
// number of tiles.
__device__ __forceinline__ uint32_t pq_tiles(const LgScratch& S, uint32_t level, uint32_t* tp, uint32_t* red,
                                             uint32_t& nr) {
    if (level == 0) {
        const uint32_t n = S.meta[LG_PCL_N];
        nr = n > LG_PCL_CUT ? 1u : 0u;
        const uint32_t nt = nr ? (n - 1 + PQ_T - 1) / PQ_T : 0u;
        if (threadIdx.x == 0) { tp[0] = 0; tp[1] = nt; }
        __syncthreads();
        return nt;
    }
    nr = min(S.pq[level % 3u], (uint32_t)PQ_MAXR);
    const uint32_t* L = pq_list(S, level % 3u);
    const uint32_t nt = block_scan(
        nr, [&](uint32_t r) -> uint32_t { return (L[PQ_EW * r + 1] - L[PQ_EW * r] - 1 + PQ_T - 1) / PQ_T; },
        [&](uint32_t r, uint32_t e) { tp[r] = e; }, red);
    if (threadIdx.x == 0) tp[nr] = nt;
    __syncthreads();
    return nt;
}
__device__ __forceinline__ void pq_range(const LgScratch& S, uint32_t level, uint32_t r, uint32_t& f, uint32_t& e,
                                         uint32_t& d) {
    if (level == 0) {
        f = 0; e = S.meta[LG_PCL_N]; d = (uint32_t)(2 * cg_lg((long)e));
        return;
    }
    const uint32_t* L = pq_list(S, level % 3u) + PQ_EW * r;
    f = L[0]; e = L[1]; d = L[2];
}
// range of tile t: the last r with tp[r] <= t
__device__ __forceinline__ uint32_t pq_find(const uint32_t* tp, uint32_t nr, uint32_t t) {
    uint32_t lo = 0, hi = nr - 1;
    while (lo < hi) {
        const uint32_t mid = (lo + hi + 1) / 2;
        if (tp[mid] <= t) lo = mid; else hi = mid - 1;
    }
    return lo;
}
#ifndef PQ_POLL_SLEEP
#define PQ_POLL_SLEEP 1   // s_sleep between the partition's polls (look-back, entries, range words); 0 measured
                          // no faster on C5 (236.1-236.3 against 234.3-236.7 us, profiles/r6_c5_poll_sleep_ab.txt)
#endif
// Decoupled look-back over tiles [lo, t) of one range, 64-bit status words: flags in bits
// 62 / 63, the >= count in bits 32..61, the <= count in bits 0..31 (counts < 2^30).
#define PQ_ST_A (1ull << 62)
#define PQ_ST_P (1ull << 63)
#define PQ_ST_V (~(PQ_ST_A | PQ_ST_P))
__device__ __forceinline__ uint64_t pq_lookback(uint64_t* ts, uint32_t lo, uint32_t t, uint64_t count,
                                                uint32_t* fail = nullptr) {
    const uint32_t l = lane_id();
    const uint64_t t_0 = __builtin_amdgcn_s_memrealtime();
    if (t == lo) {
        if (l == 0) __hip_atomic_store(&ts[t], PQ_ST_P | count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return 0;
    }
    if (l == 0) __hip_atomic_store(&ts[t], PQ_ST_A | count, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint64_t base = 0;
    int32_t hi = (int32_t)t - 1;
    for (;;) {
        const int32_t j = hi - (int32_t)l;
        const uint64_t w = j >= (int32_t)lo ? __hip_atomic_load(&ts[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                             : PQ_ST_P;
        const uint64_t pm = __ballot((w & PQ_ST_P) != 0ull);
        const uint32_t first = pm ? (uint32_t)__builtin_ctzll(pm) : 64u;
        if (__ballot(w == 0ull && l < first)) {   // a tile before the nearest prefix not published yet
            // (bounded: a tile that never publishes fails the frame, never the launch's end;
            // 200 ms, never expected)
            if (fail && __builtin_amdgcn_s_memrealtime() - t_0 > 20000000ull) {
                if (l == 0) *fail = 1u;
                break;
            }
            __builtin_amdgcn_s_sleep(PQ_POLL_SLEEP);
            continue;
        }
        const uint64_t v = l <= first ? (w & PQ_ST_V) : 0ull;
        base += ((uint64_t)wave_sum((uint32_t)(v >> 32)) << 32) | wave_sum((uint32_t)v);
        if (first < 64u) break;
        hi -= 64;
    }
    if (l == 0) __hip_atomic_store(&ts[t], PQ_ST_P | (base + count), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return base;
}

__global__ __launch_bounds__(CG_BLOCK) void lg_pq_split(LgScratch S, const uint64_t* E, uint32_t level) {
    __shared__ uint32_t tp[PQ_MAXR + 1];
    __shared__ uint32_t red[8 * WAVES];
    __shared__ uint32_t tk, cg[WAVES], cl[WAVES];
    __shared__ uint64_t tbase;
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    if (level == 0 && blockIdx.x == 0 && tid == 0) {
        S.pq[1] = 0; S.pq[2] = 0; S.pq[PQ_LEAFLIST] = 0; S.pq[PQ_MIDS] = 0;
        const uint32_t n = S.meta[LG_PCL_N];
        if (n <= LG_PCL_CUT) pq_push(S, PQ_LEAFLIST, 0, n, (uint32_t)(2 * cg_lg((long)n)), 0u);
    }
    {   // workgroups past the level's tiles return before their ticket (a grid sized from the
        // frame's N): the tiles number at most ceil(n / PQ_T) + one per range
        const uint32_t n = S.meta[LG_PCL_N];
        const uint32_t nr0 = level == 0 ? (n > LG_PCL_CUT ? 1u : 0u) : min(S.pq[level % 3u], (uint32_t)PQ_MAXR);
        if (blockIdx.x >= (n + PQ_T - 1) / PQ_T + nr0) {
            if (blockIdx.x == 0 && tid == 0) S.ca[0] = 0;   // no tile: lg_pq_swap reads the count
            return;
        }
    }
    uint64_t* st = S.pqst;   // [0] tickets, [2 + t] tile t's status; lg_pq_swap zeroes them
    // the ticket first (its latency overlaps the range lists' loads): tickets are handed out
    // in start order to every workgroup, and the one holding ticket t runs tile t, so a tile
    // still waits only on tiles already running; tickets past the tiles return
    if (tid == 0) tk = (uint32_t)__hip_atomic_fetch_add(&st[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    uint32_t nr;
    const uint32_t active = pq_tiles(S, level, tp, red, nr);   // ends with a barrier
    const uint32_t t = tk;
    if (t == 0 && tid == 0) S.ca[0] = active;   // for lg_pq_swap (PQ_TILES)
    if (t >= active) return;
    const uint32_t r = pq_find(tp, nr, t), q = t - tp[r];
    uint32_t f, e, d, m, p;
    pq_range(S, level, r, f, e, d);
    // the median of three and this element's key in one batch of loads: x > f, and x's
    // virtual record is E[f] when x is the median (__move_median_to_first's swap)
    const uint32_t x = f + 1 + q * PQ_T + tid;
    const bool valid = x < e;
    const uint32_t a = f + 1, b = f + (e - f) / 2, c = e - 1;
    const uint32_t ka = pq_key(E, a), kb = pq_key(E, b), kc = pq_key(E, c), kf = pq_key(E, f);
    const uint32_t kx = valid ? pq_key(E, x) : 0u;
    m = pb_median(a, b, c, ka, kb, kc);
    p = m == a ? ka : (m == b ? kb : kc);
    if (tid == 0) {   // the tile's range, median and pivot for lg_pq_swap: one load there
        uint32_t* tt = S.ca + PQ_TILES + 8u * t;
        tt[0] = f; tt[1] = e; tt[2] = m; tt[3] = p;
        tt[4] = d; tt[5] = r; tt[6] = q; tt[7] = 0u;
    }
    const uint32_t k = valid ? (x == m ? kf : kx) : 0u;
    const bool ge = valid && k >= p, le = valid && k <= p;
    const uint64_t gm = __ballot(ge), lm = __ballot(le);
    if (l == 0) { cg[w] = (uint32_t)__popcll(gm); cl[w] = (uint32_t)__popcll(lm); }
    __syncthreads();
    if (w == 0) {
        uint32_t tg = 0, tl = 0;
        for (uint32_t v = 0; v < WAVES; v++) { tg += cg[v]; tl += cl[v]; }
        const uint64_t b = pq_lookback(st + 2, tp[r], t, ((uint64_t)tg << 32) | tl);
        if (l == 0) {
            tbase = b;
            if (t == tp[r + 1] - 1) {   // the range's last tile: both totals
                uint32_t* tot = level == 0 ? S.pq + 4 : pq_list(S, level % 3u) + PQ_EW * r + 3;
                tot[0] = (uint32_t)(b >> 32) + tg;
                tot[1] = (uint32_t)b + tl;
            }
        }
    }
    __syncthreads();
    uint32_t gi = (uint32_t)(tbase >> 32) + mbcnt(gm), li = (uint32_t)tbase + mbcnt(lm);
    for (uint32_t v = 0; v < w; v++) { gi += cg[v]; li += cl[v]; }
    if (ge) S.par[f + 1 + gi] = x;
    if (le) S.cnt[f + 1 + li] = x;
    if (valid) ((uint64_t*)S.vox)[x] = ((uint64_t)gi << 32) | li;
}

__global__ __launch_bounds__(CG_BLOCK) void lg_pq_swap(LgScratch S, const uint64_t* E, uint64_t* Eo, uint32_t level,
                                                       uint32_t last_level, uint32_t out_buf) {
    const uint32_t tid = threadIdx.x;
    if (blockIdx.x == 0 && tid == 0 && level > 0) S.pq[(level + 2u) % 3u] = 0;   // the list level + 1 fills
    // lg_pq_split's ticket counter (every split workgroup takes a ticket) and status words of
    // this level, for the next level's split (the kernel boundary orders these stores after
    // every split tile's look-back, so its status words need no release)
    if (blockIdx.x == 0 && tid == 0) S.pqst[0] = 0;
    const uint32_t active = S.ca[0];   // the split's tile count
    if (blockIdx.x >= active) return;
    if (tid == 0) S.pqst[2 + blockIdx.x] = 0;
    // the tile's range, median and pivot as the split left them, then one batch of loads:
    // E[f], this element and its ranks (x > f), the range's totals
    const uint32_t t = blockIdx.x;
    const uint4 t0 = ((const uint4*)(S.ca + PQ_TILES))[2 * t], t1 = ((const uint4*)(S.ca + PQ_TILES))[2 * t + 1];
    const uint32_t f = t0.x, e = t0.y, m = t0.z, p = t0.w, d = t1.x, r = t1.y, q = t1.z;
    const uint32_t* tot = level == 0 ? S.pq + 4 : pq_list(S, level % 3u) + PQ_EW * r + 3;
    const uint32_t nL = tot[0], nR = tot[1];
    const uint32_t x = f + 1 + q * PQ_T + tid;
    const uint64_t rf = E[f];
    const uint64_t rx = x < e ? E[x] : 0ull;
    const uint64_t rk = x < e ? ((const uint64_t*)S.vox)[x] : 0ull;
    if (q == 0 && tid == 0) Eo[f] = E[m];
    if (x >= e) return;
    const uint64_t vx = x == m ? rf : rx;
    const uint32_t k = pcl_key(vx);
    const bool ge = k >= p, le = k <= p;
    const uint32_t gi = (uint32_t)(rk >> 32), li = (uint32_t)rk;
    uint32_t partner = x;
    bool cutter = false;
    uint32_t cut = 0;
    if (ge && gi < nR) {
        const uint32_t j = S.cnt[f + 1 + (nR - 1 - gi)];   // R_gi
        if (x < j) {
            partner = j;
            const bool nx = gi + 1 < min(nL, nR);
            const uint32_t l2 = nx ? S.par[f + 2 + gi] : 0xffffffffu;
            const uint32_t r2 = nx ? S.cnt[f + 1 + (nR - 2 - gi)] : 0u;
            if (!nx || !(l2 < r2)) {   // swap gi is the last: s = gi + 1
                cutter = true;
                cut = min(gi + 1 < nL ? S.par[f + 2 + gi] : 0xffffffffu, j);
            }
        } else if (gi == 0) {   // no swap at all: the left scan stops at L_0
            cutter = true;
            cut = x;
        }
    }
    if (le) {
        const uint32_t ri = nR - 1 - li;
        if (ri < nL) {
            const uint32_t i = S.par[f + 1 + ri];   // L_ri
            if (i < x) partner = i;
        }
    }
    Eo[x] = partner == x ? vx : (partner == m ? rf : E[partner]);
    if (cutter) {
        const uint32_t lo[2] = {f, cut}, hi[2] = {cut, e};
        for (int c = 0; c < 2; c++) {
            if (hi[c] - lo[c] > LG_PCL_CUT && d > 1 && level < last_level)
                pq_push(S, (level + 1u) % 3u, lo[c], hi[c], d - 1u, 0u);
            else
                pq_push(S, PQ_LEAFLIST, lo[c], hi[c], d - 1u, out_buf);
        }
    }
}

// ------------------------------------------------------------------------------------------
// One launch per partition level (the device-sized path): lg_pq_split's split and lg_pq_swap's
// swaps in one launch.
//   Split phase: workgroups take tiles by ticket and run each tile's split (median of three,
//   >= / <= counts, the look-back segmented by range, the L / R lists). A workgroup takes its
//   tickets (at most ceil(tiles / grid)) before it waits on anything, and a tile's look-back
//   only waits on tiles with smaller tickets, which are held by workgroups still in this phase:
//   every split finishes, whatever the grid and whatever else holds the CUs.
//   Swap phase: for each tile it holds, a workgroup waits until every tile of the tile's range
//   has written its lists, then runs the tile's swaps and, at the range's last swap, queues the
//   children. The wait is on one 64-bit word per range: every tile adds 1 << 46 | its >= count
//   << 23 | its <= count once its lists are stored, so the word that shows all the range's tiles
//   also holds the range's totals nL and nR (< 2^23: ranges of at most LG_DEV_MAX_POINTS).
// The lists cross workgroups (and XCDs) inside the launch: sc1 stores (st_rlx), every storing
// wave's vmcnt(0), a barrier, one agent-scope add per tile; the reader polls and loads with sc1
// (ld_rlx): MI355X_MICROARCH.md's hand-off table, row 1. No release fence (an agent-scope
// release writes back the XCD's whole L2).
// The ticket counter, look-back words and range words alternate between two sets by level
// parity; each level clears the set the next level uses (its last user, the level before, has
// ended), and lg_pcl_leaf clears the last level's set.
// A workgroup's first tile keeps its state in registers; further tiles (only when the level has
// more tiles than the grid) leave theirs in the tile table (S.ca) and their ranks in S.vox.
#define PQ_OWN 16   // tiles per workgroup and level beyond the first (the host sizes the grid)
#ifndef LG_PQ_GRID
// the levels' smallest grid (more when a workgroup would hold > PQ_OWN + 1 tiles); 128 and 256
// measured the same on C5, a level with no range included (4.6 us, profiles/r5_c5_grid_ab.txt)
#define LG_PQ_GRID 512
#endif
#define PQ_RW_TILE (1ull << 46)
#define PQ_RW_N ((1ull << 23) - 1ull)
static_assert(LG_DEV_MAX_POINTS < (1u << 23), "range totals fit 23 bits");
__device__ __forceinline__ uint64_t* pq_set(const LgScratch& S, uint32_t par) {
    return S.pqst + (uint64_t)par * (S.pq_tmax + 2u);
}
__device__ __forceinline__ uint64_t* pq_done(const LgScratch& S, uint32_t par) {
    return S.pqst + 2ull * (S.pq_tmax + 2u) + (uint64_t)par * PQ_MAXR;
}
__device__ __forceinline__ uint32_t* lg_arrivals(const LgScratch& S, uint32_t k) {
    return (uint32_t*)(S.pqst + 2ull * (S.pq_tmax + 2u) + 2ull * PQ_MAXR) + 16u * k;
}
// the set of parity par as no level has used it: ticket counter, look-back words of the tiles
// that took tickets, the range words of the nd ranges the set's level had (every thread of
// the block; nothing to clear when that level handed out no ticket)
__device__ __forceinline__ void pq_clear_set(const LgScratch& S, uint32_t par, uint32_t nd = PQ_MAXR) {
    uint64_t* const st = pq_set(S, par);
    const uint32_t used = (uint32_t)min(st[0], (uint64_t)S.pq_tmax);   // tickets handed out
    __syncthreads();
    if (used == 0) return;   // (uniform) no tile took a ticket: no word was written
    for (uint32_t i = threadIdx.x; i < used + 2u; i += CG_BLOCK) st[i] = 0ull;
    uint64_t* const dn = pq_done(S, par);
    for (uint32_t i = threadIdx.x; i < nd; i += CG_BLOCK) dn[i] = 0ull;
}
#define PQ_WAIT_TICKS 20000000ull   // s_memrealtime (100 MHz): 200 ms, then LG_PQ_TIMEOUT
__global__ __launch_bounds__(CG_BLOCK) void lg_pq_level(LgScratch S, const uint64_t* E, uint64_t* Eo, uint32_t level,
                                                        uint32_t last_level, uint32_t out_buf) {
    __shared__ uint32_t tp[PQ_MAXR + 1];
    __shared__ uint32_t rf_[CG_BLOCK], re_[CG_BLOCK], rd_[CG_BLOCK];   // the first CG_BLOCK ranges
    __shared__ uint32_t red[8 * WAVES];
    __shared__ uint32_t tk, cg[WAVES], cl[WAVES], nown;
    __shared__ uint32_t own[PQ_OWN];
    __shared__ uint64_t tbase, rword;
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    const uint32_t par = level & 1u;
    uint64_t* const st = pq_set(S, par);
    uint64_t* const done = pq_done(S, par);
    const uint32_t n = S.meta[LG_PCL_N];
    // range tid's entry (level > 0), loaded with the counts: entries past the count are stale
    // and unused
    uint32_t pf = 0, pe = 0, pd = 0;
    if (level > 0) {
        const uint32_t* Lr = pq_list(S, level % 3u) + PQ_EW * tid;
        pf = Lr[0]; pe = Lr[1]; pd = Lr[2];
    }
    if (blockIdx.x == 0) {
        // for level + 1: the set level - 1 used, with the ranges level - 1 had (level 0: the
        // whole index_vector; later levels: their list's count, read before the barrier in
        // pq_clear_set, and that list is emptied below). Level 0 finds both sets clean: the
        // levels and lg_pcl_leaf of the previous frame (or the allocation) left them so.
        const uint32_t nprev = level == 1 ? 1u : (level ? min(S.pq[(level + 2u) % 3u], (uint32_t)PQ_MAXR) : 0u);
        pq_clear_set(S, par ^ 1u, nprev);
        if (tid == 0) {
            if (level == 0) {   // (the lists' counts were zeroed by lg_pcl_index: this level pushes)
                if (n <= LG_PCL_CUT) pq_push(S, PQ_LEAFLIST, 0, n, (uint32_t)(2 * cg_lg((long)n)), 0u);
            } else {
                S.pq[(level + 2u) % 3u] = 0;   // the list level + 1 fills
            }
        }
    }
    {
        const uint32_t nr0 = level == 0 ? (n > LG_PCL_CUT ? 1u : 0u) : min(S.pq[level % 3u], (uint32_t)PQ_MAXR);
        if (nr0 == 0) return;   // nothing to cut at this level
        // workgroups past the level's tiles (at most one per PQ_T records plus one per range)
        // return before their ticket: 512 tickets on one word take ~6 us to hand out
        if (blockIdx.x >= (n + PQ_T - 1) / PQ_T + nr0) return;
    }
    // the first ticket before the range lists' loads (its latency overlaps them)
    if (tid == 0) {
        tk = (uint32_t)__hip_atomic_fetch_add(&st[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        nown = 0;
    }
    uint32_t nr, active;
    const bool pre = level > 0 && min(S.pq[level % 3u], (uint32_t)PQ_MAXR) <= CG_BLOCK;
    if (pre) {   // pq_tiles from the entries loaded above, kept in LDS for pq_range
        nr = min(S.pq[level % 3u], (uint32_t)PQ_MAXR);
        rf_[tid] = pf; re_[tid] = pe; rd_[tid] = pd;
        active = block_scan(nr, [&](uint32_t r) -> uint32_t { return (pe - pf - 1 + PQ_T - 1) / PQ_T; },
                            [&](uint32_t r, uint32_t e) { tp[r] = e; }, red);
        if (tid == 0) tp[nr] = active;
        __syncthreads();
    } else {
        active = pq_tiles(S, level, tp, red, nr);   // ends with a barrier
    }
    if (tk == 0 && level < 7) CG_HOOK_LG_STAMP(S, 16 + 6 * level);
    // tickets per workgroup: ceil(active / grid) of them take every tile
    const uint32_t kmax = min((active + gridDim.x - 1) / gridDim.x, (uint32_t)PQ_OWN + 1u);
    // the first tile's state (registers)
    uint32_t t0 = 0xffffffffu, f0 = 0, e0 = 0, m0 = 0, p0 = 0, d0 = 0, r0 = 0, q0 = 0, gi0 = 0, li0 = 0;
    uint64_t rx0 = 0, rf0 = 0;
    for (uint32_t it = 0; it < kmax; it++) {
        if (it > 0) {
            if (tid == 0) tk = (uint32_t)__hip_atomic_fetch_add(&st[0], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __syncthreads();
        }
        const uint32_t t = tk;
        if (t >= active) break;
        const uint32_t r = pq_find(tp, nr, t), q = t - tp[r];
        uint32_t f, e, d;
        if (pre) { f = rf_[r]; e = re_[r]; d = rd_[r]; }
        else pq_range(S, level, r, f, e, d);
        // the median of three and this element's record in one batch of loads: x > f, and x's
        // virtual record is E[f] when x is the median (__move_median_to_first's swap)
        const uint32_t x = f + 1 + q * PQ_T + tid;
        const bool valid = x < e;
        const uint32_t a = f + 1, b = f + (e - f) / 2, c = e - 1;
        const uint32_t ka = pq_key(E, a), kb = pq_key(E, b), kc = pq_key(E, c);
        const uint64_t rf = E[f];
        const uint64_t rx = E[valid ? x : f];   // (clamped: no branch between the loads)
        const uint32_t m = pb_median(a, b, c, ka, kb, kc);
        const uint32_t p = m == a ? ka : (m == b ? kb : kc);
        const uint32_t k = valid ? (x == m ? pcl_key(rf) : pcl_key(rx)) : 0u;
        const bool ge = valid && k >= p, le = valid && k <= p;
        const uint64_t gm = __ballot(ge), lm = __ballot(le);
        if (l == 0) { cg[w] = (uint32_t)__popcll(gm); cl[w] = (uint32_t)__popcll(lm); }
        __syncthreads();
        uint32_t tg = 0, tl = 0;
        for (uint32_t v = 0; v < WAVES; v++) { tg += cg[v]; tl += cl[v]; }
        if (w == 0) {
            const uint64_t bs = pq_lookback(st + 2, tp[r], t, ((uint64_t)tg << 32) | tl);
            if (l == 0) tbase = bs;
        }
        __syncthreads();
        if (t == 0 && level < 7) CG_HOOK_LG_STAMP(S, 17 + 6 * level);
        uint32_t gi = (uint32_t)(tbase >> 32) + mbcnt(gm), li = (uint32_t)tbase + mbcnt(lm);
        for (uint32_t v = 0; v < w; v++) { gi += cg[v]; li += cl[v]; }
        if (ge) st_rlx(S.par + f + 1 + gi, x);
        if (le) st_rlx(S.cnt + f + 1 + li, x);
        if (it == 0) {
            t0 = t; f0 = f; e0 = e; m0 = m; p0 = p; d0 = d; r0 = r; q0 = q; gi0 = gi; li0 = li; rx0 = rx; rf0 = rf;
        } else {   // (a level with more tiles than workgroups) the tile's state for its swaps
            if (valid) ((uint64_t*)S.vox)[x] = ((uint64_t)gi << 32) | li;
            if (tid == 0) {
                uint32_t* tt = S.ca + PQ_TILES + 8u * t;
                tt[0] = f; tt[1] = e; tt[2] = m; tt[3] = p; tt[4] = d; tt[5] = r; tt[6] = q; tt[7] = 0u;
                own[it - 1] = t;
                nown = it;
            }
        }
        // the tile's list stores done in every wave, then its counts into the range's word
        __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0)
        __syncthreads();
        if (t == 0 && level < 7) CG_HOOK_LG_STAMP(S, 18 + 6 * level);
        if (tid == 0)
            __hip_atomic_fetch_add(&done[r], PQ_RW_TILE | ((uint64_t)tg << 23) | tl, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        if (t == 0 && level < 7) CG_HOOK_LG_STAMP(S, 19 + 6 * level);
    }
    if (t0 == 0xffffffffu) return;   // (uniform) no tile for this workgroup
    const uint32_t extra = nown;
    for (uint32_t j = 0; j <= extra; j++) {
        uint32_t f, e, m, p, d, r, q, gi, li;
        uint64_t rx, rf;
        if (j == 0) {
            f = f0; e = e0; m = m0; p = p0; d = d0; r = r0; q = q0; gi = gi0; li = li0; rx = rx0; rf = rf0;
        } else {
            const uint32_t t = own[j - 1];
            const uint4 ta = ((const uint4*)(S.ca + PQ_TILES))[2 * t], tb = ((const uint4*)(S.ca + PQ_TILES))[2 * t + 1];
            f = ta.x; e = ta.y; m = ta.z; p = ta.w; d = tb.x; r = tb.y; q = tb.z;
            const uint32_t x = f + 1 + q * PQ_T + tid;
            rf = E[f];
            rx = x < e ? E[x] : 0ull;
            const uint64_t rk = x < e ? ((const uint64_t*)S.vox)[x] : 0ull;
            gi = (uint32_t)(rk >> 32); li = (uint32_t)rk;
        }
        // every tile of the range has stored its lists: the range's word counts them all, and
        // then holds the totals
        const uint64_t need = (uint64_t)(tp[r + 1] - tp[r]);
        if (tid == 0) {
            const uint64_t t_0 = __builtin_amdgcn_s_memrealtime();
            uint64_t wv = 0;
            // route 10 (tests) takes the expired path itself at level 0: no wait at all
            while (!(level == 0 && S.force_wait_fail) && ((wv = ld64(&done[r])) >> 46) < need) {
                __builtin_amdgcn_s_sleep(1);
                if (__builtin_amdgcn_s_memrealtime() - t_0 > PQ_WAIT_TICKS) break;   // (never expected)
            }
            if ((wv >> 46) < need) S.meta[LG_PQ_TIMEOUT] = 1u;   // (the frame's fetch fails on it)
            rword = wv;
        }
        if (t0 == 0 && j == 0 && level < 7) CG_HOOK_LG_STAMP(S, 20 + 6 * level);   // (the tile-0 holder)
        __syncthreads();
        const uint64_t rw = rword;
        const uint32_t x = f + 1 + q * PQ_T + tid;
        if ((rw >> 46) < need) {   // (uniform) the wait gave up: the range's totals and lists are
            // partial, so no list entry is read. The tile's records go out unchanged, and the
            // range's first tile queues the whole range as one leaf: every later index stays
            // inside [f, e). The frame's results are void (LG_PQ_TIMEOUT), never a wild access.
            if (x < e) Eo[x] = rx;
            if (q == 0 && tid == 0) {
                Eo[f] = rf;
                pq_push(S, PQ_LEAFLIST, f, e, d > 0 ? d - 1u : 0u, out_buf);
            }
            __syncthreads();
            continue;
        }
        const uint32_t nL = (uint32_t)(rw >> 23) & (uint32_t)PQ_RW_N, nR = (uint32_t)rw & (uint32_t)PQ_RW_N;
        if (q == 0 && tid == 0) Eo[f] = E[m];
        if (x < e) {
            const uint64_t vx = x == m ? rf : rx;
            const uint32_t k = pcl_key(vx);
            const bool ge = k >= p, le = k <= p;
            // the partners and the next pair in one batch of loads (indices clamped when unused)
            const bool hasL = ge && gi < nR;
            const bool nx = hasL && gi + 1 < min(nL, nR);
            const uint32_t ri = nR - 1 - li;
            const bool hasR = le && ri < nL;
            const uint32_t jj = ld_rlx(S.cnt + f + 1 + (hasL ? nR - 1 - gi : 0u));        // R_gi
            const uint32_t l2 = ld_rlx(S.par + f + 1 + (gi + 1 < nL ? gi + 1 : 0u));       // L_gi+1
            const uint32_t r2 = ld_rlx(S.cnt + f + 1 + (nx ? nR - 2 - gi : 0u));           // R_gi+1
            const uint32_t il = ld_rlx(S.par + f + 1 + (hasR ? ri : 0u));                  // L_ri
            uint32_t partner = x;
            bool cutter = false;
            uint32_t cut = 0;
            if (hasL) {
                if (x < jj) {
                    partner = jj;
                    if (!nx || !(l2 < r2)) {   // swap gi is the last: s = gi + 1
                        cutter = true;
                        cut = min(gi + 1 < nL ? l2 : 0xffffffffu, jj);
                    }
                } else if (gi == 0) {   // no swap at all: the left scan stops at L_0
                    cutter = true;
                    cut = x;
                }
            }
            if (hasR && il < x) partner = il;
            Eo[x] = partner == x ? vx : (partner == m ? rf : E[partner]);
            if (cutter) {
                const uint32_t lo[2] = {f, cut}, hi[2] = {cut, e};
                for (int c = 0; c < 2; c++) {
                    if (hi[c] - lo[c] > LG_PCL_CUT && d > 1 && level < last_level)
                        pq_push(S, (level + 1u) % 3u, lo[c], hi[c], d - 1u, 0u);
                    else
                        pq_push(S, PQ_LEAFLIST, lo[c], hi[c], d - 1u, out_buf);
                }
            }
        }
        __syncthreads();   // (rword is rewritten for the next tile)
    }
    if (t0 == 0 && level < 7) CG_HOOK_LG_STAMP(S, 21 + 6 * level);
}

// ------------------------------------------------------------------------------------------
// The device-sized frame's partition as ONE dataflow launch (lg_pq_flow), in place of one
// lg_pq_level launch per level. Each range's split and swaps are the level kernel's (the same
// median of three, >= / <= lists from a look-back segmented by range, swaps once a per-range
// word shows every tile's lists); what changes is how ranges reach workgroups:
//   - one queue of tickets for the whole sort. Tickets [0, T0) are the tiles of range 0 (the
//     whole index_vector, implicit); every later ticket's entry is published by the workgroup
//     that finished the range it belongs to, as soon as that range's swaps are stored. A range
//     starts when its parent ends, not when the slowest range of a level ends, and there are no
//     empty levels: the sort takes as many dependent range steps as its deepest range needs;
//   - a range's first tile reserves, as it starts, the block of T + 1 tickets its children will
//     take (their tiles number at most T + 1) and adds the block's base to the range's count
//     word; the range's last tile reads the base with the count and the cut in one atomic
//     (PQF_SD_BASE) and publishes every slot of the block: the children's tiles, then nops. The
//     end of a range costs no allocation;
//   - entries are 16 bytes, (first, last) and (budget | nop | kind | depth | tile, first ticket of
//     the range), both halves nonzero once written, stored by two sc1 stores and polled by two
//     sc1 loads (a half not yet written reads 0);
//   - the lists hold each element's record beside its position, so a swap loads its partner's
//     record with the partner's position: one round of loads;
//   - a tile's workgroup keeps its split state in registers and runs the tile's swaps itself
//     when every ticket of its range has been handed out (the ticket counter has passed them:
//     every tile of the range is held by a running workgroup, which never waits on a later
//     ticket). Otherwise it leaves its state in HBM (S.vox) and queues a swap entry for the
//     tile at the end of the queue, whose holder waits for the range word instead;
//   - the launch ends when every record is in a leaf: the tile that ends a range adds its leaf
//     children's records to PQF_DONE, and a workgroup whose ticket has no entry yet polls the
//     entry and that count together and leaves at n (a range still queued holds records that
//     are in no leaf, so no ordering with the entries is needed).
// Forward progress: a tile waits only on tickets below its own (look-back), or on a range all
// of whose tickets are held; a workgroup without an entry waits on workgroups with lower
// tickets. So the launch drains whatever the grid size and residency; every wait is bounded
// (200 ms, never expected: the frame then fails with CG_E_DEVICE, LG_PQ_TIMEOUT).
// Visibility: every cross-workgroup byte (records, lists, swap state, entries, words) is stored
// sc1 (st_rlx / st64 / agent-scope atomics) after which the storing waves wait vmcnt(0) before
// the barrier and the one signalling add or entry store, and loaded sc1 (ld_rlx / ld64):
// MI355X_MICROARCH.md's hand-off table, row 1. lg_pcl_leaf clears the used words and lg_pcl_mid
// the counters, so the next frame finds them zero. (tests/pqf_model.py models it tile by tile.)
#ifndef LG_FLOW_GRID
// workgroups of the launch: 192 measured best on C5 (235-238 us per frame against 237-241 at 128
// and 256, 266-270 at 512 before the counters had lines of their own, profiles/r6_c5_flow_ab.txt)
#define LG_FLOW_GRID 192
#endif
#define LG_CLEAR_FLOW 0x100u   // lg_pcl_leaf's clear_set for lg_pq_flow's words
#define PQF_HDR 48         // u64 words, the counters on lines of their own (they take every
                           // workgroup's atomics and polls): [PQF_TK] tickets handed out,
                           // [PQF_TAIL] tickets queued past range 0's, [PQF_DONE] records in leaves
#define PQF_TK 0
#define PQF_TAIL 16
#define PQF_DONE 32
#define PQF_KIND_SWAP (1u << 7)
#define PQF_NOP (1u << 6)  // an unused slot of a children block (budgets take bits 0-5)
struct PqfView {
    uint64_t* hdr; uint64_t* ent; uint64_t* lb; uint64_t* rw; uint64_t* sd; uint32_t cap;
};
__device__ __forceinline__ PqfView pqf_view(const LgScratch& S) {
    PqfView v;
    v.cap = S.pqf_cap;
    v.hdr = S.pqf;
    v.ent = S.pqf + PQF_HDR;      // two words per ticket
    v.lb = v.ent + 2ull * v.cap;  // look-back status per ticket
    v.rw = v.lb + v.cap;          // range word, by the range's first ticket
    v.sd = v.rw + v.cap;          // by first ticket: the range's count word (PQF_SD_BASE)
    return v;
}
__device__ __forceinline__ uint32_t pqf_tiles(uint32_t f, uint32_t e) { return (e - f - 1 + PQ_T - 1) / PQ_T; }
__device__ __forceinline__ uint32_t pqf_key(const uint64_t* E, uint32_t x) {
    return ld_rlx((uint32_t*)E + 2ull * x + 1);
}
__device__ __forceinline__ void pqf_entry(const PqfView& Q, uint64_t k, uint32_t f, uint32_t e, uint32_t w2, uint32_t tb) {
    st64(Q.ent + 2 * k, ((uint64_t)e << 32) | f);
    st64(Q.ent + 2 * k + 1, ((uint64_t)tb << 32) | w2);
}
// A leaf's results straight to the outputs: idx in the key array, slot in the value array.
struct PqLeafOut {
    uint64_t* k; uint32_t* v; uint32_t base;
    __device__ __forceinline__ void operator()(uint32_t i, uint64_t r) const {
        k[base + i] = r >> 32;
        v[base + i] = (uint32_t)r;
    }
};
// The ranges a leaf's levels leave (cg_pcl.h pcl_block_sort's wave tasks, 17-PQ_MID records):
//   17-64 records: the wave finishes the range itself (pw_range64 from LDS, results straight to
//   the outputs);
//   65-PQ_MID records (lg_pcl_leaf's): handed on to a chip-wide launch, lg_pcl_mid (one
//   workgroup each): the records go back to the HBM buffer the range was loaded from and onto
//   a task list in S.dsz (first, size | budget << 16 | buffer << 24; free until the
//   clustering). The leaf workgroups then only run the levels of their longer ranges, on a few
//   CUs; the tasks spread over the chip.
// (Round 5 handed the 17-64-record ranges on too, to a third launch of one wave each: 24.6 +
// 20.7 + 6.5 us against 26.4 + 21.2 us inline, profiles/r5_c5_waves_ab.txt.)
#ifndef PQ_MID
#define PQ_MID 512   // (256: 34.3 + 16.2 us, 1,024: 20.1 + 32.6 us against 26.6 + 21.4, profiles/r5_c5_mid_ab.txt)
#endif
struct PqDefer {
    uint64_t* Eh; uint32_t* list; uint32_t* count; uint32_t base, buf;
    template <class P64, class OUT>
    __device__ __forceinline__ void operator()(P64 E, uint32_t f, uint32_t m, uint32_t d, OUT out) const {
        if (m <= PW_MAX) {
            pw_range64(E, f, m, d, out);
            return;
        }
        const uint32_t l = lane_id();
        for (uint32_t i = l; i < m; i += 64) Eh[base + f + i] = E[f + i];
        if (l == 0) {
            const uint32_t q = atomicAdd(count, 1u);
            list[2 * q] = base + f;
            list[2 * q + 1] = m | (d << 16) | (buf << 24);
        }
    }
};
#define LG_PCL_LDS (8 * LG_PCL_LEAF + 4 * 4 * (LG_PCL_LEAF + 4))
// The rest of each leaf range (cg_pcl.h pcl_block_sort with the depth left on its path) from
// the buffer its last level wrote: in LDS (8 B of record and 16 B of scratch per element),
// else in HBM (ranges are disjoint, so each uses its own span of the scratch arrays).
__global__ __launch_bounds__(CG_BLOCK) void lg_pcl_leaf(LgScratch S, uint64_t* E0, uint64_t* E1, uint64_t* kout,
                                                        uint32_t* vout, uint32_t clear_set) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[LG_PCL_LDS];
    __shared__ uint32_t red[8 * WAVES];
    const uint32_t n = min(S.pq[PQ_LEAFLIST], (uint32_t)LG_PQ_CAP);
    const uint32_t tid = threadIdx.x;
    // the split's ticket counter, also when no level followed the level-0 split (no swap);
    // lg_pq_level's levels: the last level's set (clear_set = its parity + 1); lg_pq_flow
    // (clear_set = LG_CLEAR_FLOW): the words of every ticket it handed out, across the grid
    // (lg_pcl_mid clears its counters after this launch)
    if (blockIdx.x == 0 && tid == 0 && !clear_set) S.pqst[0] = 0;
    if (clear_set == LG_CLEAR_FLOW) {
        const PqfView Q = pqf_view(S);
        // every ticket handed out, and every slot allocated (nop slots published for a block
        // the workgroups never reached before the launch ended)
        const uint64_t n_ = S.meta[LG_PCL_N];
        const uint64_t alloc = n_ > LG_PCL_CUT ? 2ull * ((n_ - 1 + PQ_T - 1) / PQ_T) + Q.hdr[PQF_TAIL] : 0ull;
        const uint32_t used = (uint32_t)min(max(Q.hdr[PQF_TK], alloc), (uint64_t)Q.cap);
        for (uint32_t i = blockIdx.x * CG_BLOCK + tid; i < used; i += gridDim.x * CG_BLOCK) {
            Q.ent[2ull * i] = 0ull; Q.ent[2ull * i + 1] = 0ull;
            Q.lb[i] = 0ull; Q.rw[i] = 0ull; Q.sd[i] = 0ull;
        }
    } else if (blockIdx.x == 0 && clear_set) {
        pq_clear_set(S, clear_set - 1u);
        __syncthreads();
    }
    for (uint32_t b = blockIdx.x; b < n; b += gridDim.x) {
        const uint32_t* ent = pq_list(S, PQ_LEAFLIST) + PQ_EW * b;
        const uint32_t first = ent[0], last = ent[1], depth = ent[2], size = last - first;
        uint64_t* const E = ent[3] ? E1 : E0;
        if (size <= LG_PCL_LEAF) {
            lds_u64* const El = (lds_u64*)(uint64_t*)smem;
            lds_u32* const w0 = (lds_u32*)(uint32_t*)(smem + 8 * LG_PCL_LEAF);
            const PbScratch<PbLds> PS{w0, w0 + (LG_PCL_LEAF + 4), w0 + 2 * (LG_PCL_LEAF + 4), w0 + 3 * (LG_PCL_LEAF + 4)};
            lds_u32* const Rl = (lds_u32*)red;
            const PqLeafOut out{kout, vout, first};
            const PqDefer wt{E, S.dsz, S.pq + PQ_MIDS, first, ent[3]};
            for (uint32_t i = tid; i < size; i += CG_BLOCK) El[i] = E[first + i];
            __syncthreads();
            if (size <= CG_BLOCK)
                pcl_block_sort<1, PbLds, PqLeafOut, false, PqDefer, PQ_MID>(El, out, size, depth, PS, Rl, nullptr, wt);
            else if (size <= 2 * CG_BLOCK)
                pcl_block_sort<2, PbLds, PqLeafOut, false, PqDefer, PQ_MID>(El, out, size, depth, PS, Rl, nullptr, wt);
            else if (size <= 4 * CG_BLOCK)
                pcl_block_sort<4, PbLds, PqLeafOut, false, PqDefer, PQ_MID>(El, out, size, depth, PS, Rl, nullptr, wt);
            else pcl_block_sort<8, PbLds, PqLeafOut, false, PqDefer, PQ_MID>(El, out, size, depth, PS, Rl, nullptr, wt);
        } else {   // the range's own span of the HBM arrays
            Work W{};
            W.KEY = (uint64_t*)S.vox + 2ull * first;
            W.A = S.lab + first; W.PAR = S.par + first; W.CNT = S.cnt + first; W.UK = S.uk + first;
            W.ORD = S.ord + first; W.LAB = (int32_t*)S.rank + first; W.OFF = S.off + first;
            pcl_sort<2, false>(W, E + first, size, red, (int)depth);
            for (uint32_t i = tid; i < size; i += CG_BLOCK) {
                const uint64_t rr = W.KEY[i];
                kout[first + i] = rr >> 32;
                vout[first + i] = (uint32_t)rr;
            }
            __syncthreads();
        }
    }
}

// The leaves' ranges of 65-512 records (S.dsz), one workgroup each, in LDS (their ranges of
// 17-64 records one wave each, in LDS too).
#define LG_MID_LDS (8 * PQ_MID + 4 * 4 * (PQ_MID + 4))
__global__ __launch_bounds__(CG_BLOCK) void lg_pcl_mid(LgScratch S, uint64_t* E0, uint64_t* E1, uint64_t* kout,
                                                       uint32_t* vout, uint32_t clear_flow = 0u) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[LG_MID_LDS];
    __shared__ uint32_t red[8 * WAVES];
    const uint32_t n = S.pq[PQ_MIDS];
    if (clear_flow && blockIdx.x == 0 && threadIdx.x < PQF_HDR) S.pqf[threadIdx.x] = 0ull;   // (lg_pq_flow's counters)
    lds_u64* const El = (lds_u64*)(uint64_t*)smem;
    lds_u32* const w0 = (lds_u32*)(uint32_t*)(smem + 8 * PQ_MID);
    const PbScratch<PbLds> PS{w0, w0 + (PQ_MID + 4), w0 + 2 * (PQ_MID + 4), w0 + 3 * (PQ_MID + 4)};
    lds_u32* const Rl = (lds_u32*)red;
    for (uint32_t b = blockIdx.x; b < n; b += gridDim.x) {
        const uint32_t first = S.dsz[2 * b], w1 = S.dsz[2 * b + 1];
        const uint32_t size = w1 & 0xffffu, depth = (w1 >> 16) & 0xffu, buf = w1 >> 24;
        uint64_t* const E = buf ? E1 : E0;
        for (uint32_t i = threadIdx.x; i < size; i += CG_BLOCK) El[i] = E[first + i];
        __syncthreads();
        const PqDefer wt{E, nullptr, nullptr, first, buf};   // (every task here is <= 64 records)
        if constexpr (PQ_MID > CG_BLOCK) {
            if (size > CG_BLOCK) {
                pcl_block_sort<2, PbLds, PqLeafOut, false, PqDefer>(El, PqLeafOut{kout, vout, first}, size, depth, PS,
                                                                    Rl, nullptr, wt);
                continue;
            }
        }
        pcl_block_sort<1, PbLds, PqLeafOut, false, PqDefer>(El, PqLeafOut{kout, vout, first}, size, depth, PS, Rl,
                                                            nullptr, wt);
    }
}
#define PQF_WAIT_TICKS PQ_WAIT_TICKS
#define PQF_SD_BAD 0xffffffffu   // tcut of a tile whose range wait gave up
// the per-range count word (Q.sd): tiles whose swaps are stored (bits 0-15), the cut + 1 (16-38,
// from the cutter's tile), the children block's base ticket (39-62, from the first tile as it
// starts), a wait that gave up (63): one add per tile, the last one reads it all
#define PQF_SD_BASE 39
__global__ __launch_bounds__(CG_BLOCK) void lg_pq_flow(LgScratch S, uint64_t* E0, uint64_t* E1, uint32_t depth_cap) {
    __shared__ uint32_t cg[WAVES], cl[WAVES];
    __shared__ uint64_t tbase;
    __shared__ uint32_t es[8];   // the ticket's entry: ok, f, e, w2, tb, t; then the inline decision
    __shared__ uint32_t tcut;    // the tile's cut + 1 (its cutter), PQF_SD_BAD, or 0
    __shared__ uint32_t ch[9];   // children: [0] count, [1] block base, [2..5] their (first, last),
                                 // [6..7] their tiles, [8] this workgroup finished the range
    const PqfView Q = pqf_view(S);
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    const uint32_t n = S.meta[LG_PCL_N];
    if (n <= LG_PCL_CUT) {   // nothing to cut: index_vector is one leaf
        if (blockIdx.x == 0 && tid == 0) pq_push(S, PQ_LEAFLIST, 0, n, (uint32_t)(2 * cg_lg((long)n)), 0u);
        return;
    }
    const uint32_t T0 = pqf_tiles(0, n);
    const uint32_t d0 = (uint32_t)(2 * cg_lg((long)n));
    uint64_t* const vst = (uint64_t*)S.vox;   // a deferred tile's per-element state: gi << 32 | li
    uint64_t* const recL = S.pqr;             // the records of the L / R lists, beside their positions
    uint64_t* const recR = S.pqr + n;
    for (;;) {
        if (tid == 0) {   // the next ticket and its entry
            const uint32_t t = (uint32_t)__hip_atomic_fetch_add(&Q.hdr[PQF_TK], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            // (range 0: budget d0, depth 0, its swap slots at [T0, 2 T0))
            uint32_t ok = 1, f = 0, e = n, w2 = d0 | (T0 << 16), tb = 0;
            if (t >= T0) {
                if (t >= Q.cap) {
                    ok = 0;   // (past every ticket the sort can queue: nothing will be published here)
                } else {
                    const uint64_t t_0 = __builtin_amdgcn_s_memrealtime();
                    for (uint32_t it = 0;; it++) {
                        const uint64_t a = ld64(Q.ent + 2ull * t), b = ld64(Q.ent + 2ull * t + 1);
                        // (every fourth poll: one line that every waiting workgroup reads)
                        const uint64_t placed = (it & 3u) == 3u ? ld64(&Q.hdr[PQF_DONE]) : 0ull;
                        if (a && b) {
                            f = (uint32_t)a; e = (uint32_t)(a >> 32); w2 = (uint32_t)b; tb = (uint32_t)(b >> 32);
                            // (never expected) an entry that does not describe a range of this
                            // index_vector: the frame fails, no index is formed from it
                            if (!(f < e && e <= n && tb < Q.cap &&
                                  ((w2 & PQF_NOP) || ((w2 & PQF_KIND_SWAP) ? (w2 >> 16) : t - tb) < pqf_tiles(f, e)))) {
                                S.meta[LG_PQ_TIMEOUT] = 1u;
                                ok = 0;
                            }
                            break;
                        }
                        if (placed >= n) { ok = 0; break; }   // every record is in a leaf: the sort is done
                        if (__builtin_amdgcn_s_memrealtime() - t_0 > PQF_WAIT_TICKS) {   // (never expected)
                            S.meta[LG_PQ_TIMEOUT] = 1u;
                            ok = 0;
                            break;
                        }
                        __builtin_amdgcn_s_sleep(PQ_POLL_SLEEP);
                    }
                }
            }
            es[0] = ok; es[1] = f; es[2] = e; es[3] = w2; es[4] = tb; es[5] = t;
            if (ok) {
                CG_HOOK_PQF(S, t, 0, __builtin_amdgcn_s_memrealtime());
                CG_HOOK_PQF(S, t, 4, ((uint64_t)e << 32) | f);
                CG_HOOK_PQF(S, t, 5, ((uint64_t)tb << 32) | w2);
            }
        }
        __syncthreads();
        if (!es[0]) return;
        const uint32_t f = es[1], e = es[2], w2 = es[3], tb = es[4], t = es[5];
        if (w2 & PQF_NOP) continue;   // (uniform) an unused slot of a children block
        const uint32_t d = w2 & 0x3fu, depth = (w2 >> 8) & 0xffu;
        const bool swap_entry = (w2 & PQF_KIND_SWAP) != 0;
        const uint32_t q = swap_entry ? (w2 >> 16) : t - tb;
        const uint32_t off = swap_entry ? 0u : (w2 >> 16);   // a split entry: the range's swap slots at tb + off
        const uint32_t T = pqf_tiles(f, e);
        const uint64_t* const E = (depth & 1u) ? E1 : E0;
        uint64_t* const Eo = (depth & 1u) ? E0 : E1;
        // the range's first tile reserves the block its children will be queued in as it starts
        // (off the critical path; the base rides in the range's count word to the tile that ends
        // the range): T + 1 slots for the children's tiles (they number at most T + 1), then T + 1
        // for their swap slots
        if (!swap_entry && q == 0 && tid == 0) {
            const uint64_t base = 2ull * T0 + __hip_atomic_fetch_add(&Q.hdr[PQF_TAIL], 2ull * ((uint64_t)T + 1ull),
                                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            __hip_atomic_fetch_add(&Q.sd[tb], min(base, (uint64_t)Q.cap) << PQF_SD_BASE, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        }
        // the median of three and this element's record in one batch of loads: x > f, and x's
        // virtual record is E[f] when x is the median (__move_median_to_first's swap)
        const uint32_t x = f + 1 + q * PQ_T + tid;
        const bool valid = x < e;
        const uint32_t a = f + 1, b = f + (e - f) / 2, c = e - 1;
        const uint32_t ka = pqf_key(E, a), kb = pqf_key(E, b), kc = pqf_key(E, c);
        const uint64_t rf = ld64((uint64_t*)E + f);
        const uint64_t rx = ld64((uint64_t*)E + (valid ? x : f));   // (clamped: no branch between the loads)
        // the ticket count for the inline-swap decision, in the same batch: it only grows, so a
        // count read now that covers the range still covers it after the split
        const uint64_t handed = (!swap_entry && tid == 0) ? ld64(&Q.hdr[PQF_TK]) : 0ull;
        const uint32_t m = pb_median(a, b, c, ka, kb, kc);
        const uint32_t p = m == a ? ka : (m == b ? kb : kc);
        const uint64_t vx = x == m ? rf : rx;
        uint32_t gi = 0, li = 0;
        if (!swap_entry) {
            // split: >= / <= counts, the range's look-back over its tiles' tickets, the lists
            // (positions and, beside them, the records: a swap then reads its partner's record
            // with the partner's position, one round of loads)
            const uint32_t k = valid ? pcl_key(vx) : 0u;
            const bool ge = valid && k >= p, le = valid && k <= p;
            const uint64_t gm = __ballot(ge), lm = __ballot(le);
            if (l == 0) { cg[w] = (uint32_t)__popcll(gm); cl[w] = (uint32_t)__popcll(lm); }
            __syncthreads();
            uint32_t tg = 0, tl = 0;
            for (uint32_t v = 0; v < WAVES; v++) { tg += cg[v]; tl += cl[v]; }
            if (w == 0) {
                const uint64_t bs = pq_lookback(Q.lb, tb, t, ((uint64_t)tg << 32) | tl, S.meta + LG_PQ_TIMEOUT);
                if (l == 0) tbase = bs;
            }
            __syncthreads();
            gi = (uint32_t)(tbase >> 32) + mbcnt(gm);
            li = (uint32_t)tbase + mbcnt(lm);
            for (uint32_t v = 0; v < w; v++) { gi += cg[v]; li += cl[v]; }
            if (ge) { st_rlx(S.par + f + 1 + gi, x); st64(recL + f + 1 + gi, vx); }
            if (le) { st_rlx(S.cnt + f + 1 + li, x); st64(recR + f + 1 + li, vx); }
            __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0): the lists are stored
            __syncthreads();
            const uint32_t slot = tb + off + q;   // the tile's swap slot
            if (tid == 0) {
                __hip_atomic_fetch_add(&Q.rw[tb], PQ_RW_TILE | ((uint64_t)tg << 23) | tl, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT);
                // the swaps here only when every ticket of the range is held (or done); the swap
                // slot then takes a nop
                es[6] = handed >= (uint64_t)tb + T ? 1u : 0u;
                if (es[6] && slot < Q.cap) pqf_entry(Q, slot, 0u, 1u, PQF_NOP, 0u);
                CG_HOOK_PQF(S, t, 1, __builtin_amdgcn_s_memrealtime());
            }
            __syncthreads();
            if (!es[6]) {   // defer: the state to HBM, a swap entry in the tile's swap slot
                if (valid) st64(vst + x, ((uint64_t)gi << 32) | li);
                __builtin_amdgcn_s_waitcnt(0x0070);
                __syncthreads();
                if (tid == 0) {
                    if (slot < Q.cap) pqf_entry(Q, slot, f, e, (w2 & 0xffffu) | PQF_KIND_SWAP | (q << 16), tb);
                    else S.meta[LG_PQ_TIMEOUT] = 1u;   // (the capacity bounds every queue: never expected)
                }
                __syncthreads();
                continue;
            }
        } else if (valid) {   // a deferred tile: its split state
            const uint64_t rk = ld64(vst + x);
            gi = (uint32_t)(rk >> 32);
            li = (uint32_t)rk;
        }
        // swaps: once the range word counts every tile, it holds the range's totals
        if (tid == 0) {
            const uint64_t t_0 = __builtin_amdgcn_s_memrealtime();
            uint64_t wv = 0;
            // route 10 (tests) takes the expired path itself on range 0: no wait at all
            while (!(tb == 0 && S.force_wait_fail) && ((wv = ld64(&Q.rw[tb])) >> 46) < T) {
                __builtin_amdgcn_s_sleep(PQ_POLL_SLEEP);
                if (__builtin_amdgcn_s_memrealtime() - t_0 > PQF_WAIT_TICKS) break;   // (never expected)
            }
            if ((wv >> 46) < T) S.meta[LG_PQ_TIMEOUT] = 1u;   // (the frame's fetch fails on it)
            tbase = wv;
            tcut = 0u;
            CG_HOOK_PQF(S, t, 2, __builtin_amdgcn_s_memrealtime());
        }
        __syncthreads();
        const uint64_t rw = tbase;
        if ((rw >> 46) < T) {   // (uniform) the wait gave up: the range's totals and lists are
            // partial, so no list entry is read. The tile's records go out unchanged, the range's
            // first tile queues the whole range as one leaf and the range queues no children:
            // every later index stays inside [f, e); the frame's results are void.
            if (valid) st64(Eo + x, rx);
            if (q == 0 && tid == 0) {
                st64(Eo + f, rf);
                pq_push(S, PQ_LEAFLIST, f, e, d - 1u, (depth + 1u) & 1u);
                __hip_atomic_fetch_add(&Q.hdr[PQF_DONE], (uint64_t)(e - f), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            if (tid == 0) {
                tcut = PQF_SD_BAD;
                // (before the tile's count add, same address: the range's last tile sees it)
                __hip_atomic_fetch_or(&Q.sd[tb], 1ull << 63, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
        } else {
            const uint32_t nL = (uint32_t)(rw >> 23) & (uint32_t)PQ_RW_N, nR = (uint32_t)rw & (uint32_t)PQ_RW_N;
            if (q == 0 && tid == 0) st64(Eo + f, ld64((uint64_t*)E + m));
            if (valid) {
                const uint32_t k = pcl_key(vx);
                const bool ge = k >= p, le = k <= p;
                // the partners (position and record) and the next pair in one batch of loads
                // (indices clamped when unused)
                const bool hasL = ge && gi < nR;
                const bool nx = hasL && gi + 1 < min(nL, nR);
                const uint32_t ri = nR - 1 - li;
                const bool hasR = le && ri < nL;
                const uint32_t iR = f + 1 + (hasL ? nR - 1 - gi : 0u), iL = f + 1 + (hasR ? ri : 0u);
                const uint32_t jj = ld_rlx(S.cnt + iR);                                           // R_gi
                const uint64_t rjj = ld64(recR + iR);
                const uint32_t l2 = ld_rlx(S.par + f + 1 + (gi + 1 < nL ? gi + 1 : 0u));          // L_gi+1
                const uint32_t r2 = ld_rlx(S.cnt + f + 1 + (nx ? nR - 2 - gi : 0u));              // R_gi+1
                const uint32_t il = ld_rlx(S.par + iL);                                           // L_ri
                const uint64_t ril = ld64(recL + iL);
                uint64_t rec = vx;
                bool cutter = false;
                uint32_t cut = 0;
                if (hasL) {
                    if (x < jj) {
                        rec = rjj;
                        if (!nx || !(l2 < r2)) {   // swap gi is the last: s = gi + 1
                            cutter = true;
                            cut = min(gi + 1 < nL ? l2 : 0xffffffffu, jj);
                        }
                    } else if (gi == 0) {   // no swap at all: the left scan stops at L_0
                        cutter = true;
                        cut = x;
                    }
                }
                if (hasR && il < x) rec = ril;
                st64(Eo + x, rec);
                if (cutter) tcut = min(max(cut, f), e) + 1u;
            }
        }
        // the tile's swaps are stored; the range's last tile queues the children in the block
        __builtin_amdgcn_s_waitcnt(0x0070);
        __syncthreads();
        if (tid == 0) {
            // one add per tile: its count, and the cut when the cutter is here; the first tile
            // added the children block's base when it started
            const uint64_t add = 1ull | (tcut == PQF_SD_BAD ? 0ull : ((uint64_t)tcut << 16));
            const uint64_t tot = __hip_atomic_fetch_add(&Q.sd[tb], add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + add;
            const uint32_t done = (uint32_t)(tot & 0xffffull) - 1u;
            const uint32_t base = (uint32_t)((tot >> PQF_SD_BASE) & 0xffffffull);
            uint32_t nch = 0;
            if (done == T - 1u) {
                // no children after a wait that gave up (the range went to the leaves whole)
                const uint32_t cw = (tot >> 63) ? 0u : (uint32_t)((tot >> 16) & 0x7fffffull);
                const bool fits = (uint64_t)base + 2ull * (T + 1u) <= Q.cap;
                uint32_t placed = 0;
                if (cw) {
                    const uint32_t cut = cw - 1u;
                    const uint32_t lo[2] = {f, cut}, hi[2] = {cut, e};
                    uint32_t used = 0;
                    for (int cc = 0; cc < 2; cc++) {
                        const uint32_t tcc = pqf_tiles(lo[cc], hi[cc]);
                        const bool rng = hi[cc] - lo[cc] > LG_PCL_CUT && d > 1 && !(depth_cap && depth + 1u >= depth_cap) &&
                                         fits;   // (a block past the capacity: the leaves finish it in HBM)
                        if (rng) {
                            ch[2 + 2 * nch] = lo[cc]; ch[3 + 2 * nch] = hi[cc];
                            ch[6 + nch] = tcc;
                            used += tcc;
                            nch++;
                        } else {
                            pq_push(S, PQ_LEAFLIST, lo[cc], hi[cc], d - 1u, (depth + 1u) & 1u);
                            placed += hi[cc] - lo[cc];
                        }
                    }
                } else {
                    S.meta[LG_PQ_TIMEOUT] = 1u;   // (no cut stored, or a wait gave up: never expected)
                }
                // records now in leaves: the launch ends when every record is (no ordering with
                // the children's entries needed: a child range holds records that are not)
                if (placed)
                    __hip_atomic_fetch_add(&Q.hdr[PQF_DONE], (uint64_t)placed, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            ch[0] = nch; ch[1] = base;
            ch[8] = done == T - 1u ? 1u : 0u;
        }
        __syncthreads();
        if (ch[8]) {   // (uniform) this workgroup finished the range
            const uint32_t nch = ch[0], base = ch[1];
            const uint32_t used = (nch > 0 ? ch[6] : 0u) + (nch > 1 ? ch[7] : 0u);
            // split slots [base, base + T + 1): the children's tiles (their swap slots T + 1 on),
            // then nops; swap slots [base + T + 1, base + 2 T + 2): the children's tiles publish
            // their own, the rest are nops
            const uint32_t w2c = (d - 1u) | ((depth + 1u) << 8) | ((T + 1u) << 16);
            for (uint32_t i = tid; i < 2u * (T + 1u); i += CG_BLOCK) {
                const uint32_t k = base + i;
                if (k >= Q.cap) break;
                if (i < used) {
                    const uint32_t cc = (nch == 2 && i >= ch[6]) ? 1u : 0u;
                    const uint32_t fb = base + (cc ? ch[6] : 0u);   // the child's first ticket
                    pqf_entry(Q, k, ch[2 + 2 * cc], ch[3 + 2 * cc], w2c, fb);
                } else if (i < T + 1u || i >= T + 1u + used) {
                    pqf_entry(Q, k, 0u, 1u, PQF_NOP, 0u);
                }
            }
        }
        if (tid == 0) CG_HOOK_PQF(S, t, 3, __builtin_amdgcn_s_memrealtime() | (ch[8] ? (1ull << 63) : 0ull));
        __syncthreads();   // (es and ch are rewritten for the next ticket)
    }
}

// ------------------------------------------------------------------------------------------
// Euclidean clustering over the V voxels (FLANN L2_Simple predicate, PCL's seed = the lowest
// index of each component):
//   dense neighbour grid: voxel -> cell (atomic slot), exclusive scan of the cell counts,
//   fill: ord holds the voxels cell by cell, cstart[c] the first of cell c;
//   forest: every voxel points at its lowest adjacent voxel (<= itself), no atomics; the
//   trees lie inside components and are rooted at their lowest index;
//   flatten: pointer jumping;
//   cross: only edges between different trees are united (uf_union hooks the larger root
//   under the smaller, so roots stay the components' lowest indices).
// exclusive scan of cstart[0, ncell] in place (single pass, lg_tile_scan)
__global__ __launch_bounds__(CG_BLOCK) void lg_dgrid_scan(LgScratch S) {
    const uint32_t n = S.meta[LG_NCELL] + 1;
    const uint32_t active = (n + LG_TILE - 1) / LG_TILE;
    if (blockIdx.x >= active) return;
    const uint32_t t = lg_tile_ticket(S.sstat);
    const uint64_t b0 = (uint64_t)t * LG_TILE + (uint64_t)threadIdx.x * 8;
    uint32_t x[8], c = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) { x[q] = (b0 + q < n) ? S.cstart[b0 + q] : 0u; c += x[q]; }
    uint32_t pos = lg_tile_scan(S.sstat, t, active, c, nullptr);
#pragma unroll
    for (int q = 0; q < 8; q++)
        if (b0 + q < n) { S.cstart[b0 + q] = pos; pos += x[q]; }
    lg_tile_done(S.sstat, active);
}
// lg_dgrid_scan and lg_dgrid_fill in one launch (the device-sized path): the tiles publish
// their cell starts with sc1 stores, every thread waits for its stores before its tile counts as
// done, and the last tile to finish fills ord reading the starts with sc1 loads (the hand-off
// of MI355X_MICROARCH.md's table, row 1; no release fence).
__global__ __launch_bounds__(CG_BLOCK) void lg_dgrid_scan_fill(LgScratch S) {
    __shared__ uint32_t last;
    const uint32_t n = S.meta[LG_NCELL] + 1;
    const uint32_t active = (n + LG_TILE - 1) / LG_TILE;
    if (blockIdx.x >= active) return;
    const uint32_t t = lg_tile_ticket(S.sstat);
    const uint64_t b0 = (uint64_t)t * LG_TILE + (uint64_t)threadIdx.x * 8;
    uint32_t x[8], c = 0;
#pragma unroll
    for (int q = 0; q < 8; q++) { x[q] = (b0 + q < n) ? S.cstart[b0 + q] : 0u; c += x[q]; }
    uint32_t pos = lg_tile_scan(S.sstat, t, active, c, nullptr);
#pragma unroll
    for (int q = 0; q < 8; q++)
        if (b0 + q < n) { st_rlx(&S.cstart[b0 + q], pos); pos += x[q]; }
    __builtin_amdgcn_s_waitcnt(0x0070);   // vmcnt(0) lgkmcnt(0): this thread's starts are stored
    __syncthreads();
    if (threadIdx.x == 0)
        last = __hip_atomic_fetch_add(&S.sstat[1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == active - 1;
    __syncthreads();
    if (!last) return;
    for (uint32_t i = threadIdx.x; i < active + 2; i += CG_BLOCK) S.sstat[i] = 0;   // (lg_tile_done's reset)
    const uint32_t V = S.meta[LG_V];
    for (uint32_t vb = 0; vb < V; vb += 8 * CG_BLOCK) {   // eight voxels in flight per thread
        uint32_t uk[8], ca[8], st[8];
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t v = vb + (uint32_t)q * CG_BLOCK + threadIdx.x;
            uk[q] = v < V ? S.uk[v] : 0u;
            ca[q] = v < V ? S.ca[v] : 0u;
        }
#pragma unroll
        for (int q = 0; q < 8; q++) st[q] = vb + (uint32_t)q * CG_BLOCK + threadIdx.x < V ? ld_rlx(&S.cstart[uk[q]]) : 0u;
#pragma unroll
        for (int q = 0; q < 8; q++) {
            const uint32_t v = vb + (uint32_t)q * CG_BLOCK + threadIdx.x;
            if (v < V) S.ord[st[q] + ca[q]] = v;
        }
    }
}
__global__ __launch_bounds__(CG_BLOCK) void lg_dgrid_fill(LgScratch S) {
    const uint32_t v = blockIdx.x * CG_BLOCK + threadIdx.x, V = S.meta[LG_V];
    if (v < V) S.ord[S.cstart[S.uk[v]] + S.ca[v]] = v;
}
// The lanes of the wave whose value v (< 2^nb) equals this lane's, among the lanes of `act`:
// one ballot per bit (a constant cost, where a loop over the distinct values of a wave costs a
// round per value).
__device__ __forceinline__ uint64_t lg_match(uint32_t v, uint32_t nb, uint64_t act) {
    uint64_t m = act;
    for (uint32_t b = 0; b < nb; b++) {
        const bool bit = (v >> b) & 1u;
        const uint64_t bb = __ballot(bit);
        m &= bit ? bb : ~bb;
    }
    return m;
}
// lg_match for waves that hold few distinct values (a chunk of voxels in PCL order meets a few
// clusters): one round per distinct value, the leader's value broadcast and compared, for at
// most nb rounds; the lanes still unmatched then take lg_match's nb ballots. (Active lanes
// only: the result of a lane outside `act` is 0.)
__device__ __forceinline__ uint64_t lg_match_few(uint32_t v, uint32_t nb, uint64_t act) {
    const uint32_t l = lane_id();
    uint64_t rem = act, same = 0ull;
    for (uint32_t r = 0; r < nb && rem; r++) {
        const uint32_t v0 = (uint32_t)__builtin_amdgcn_readlane((int)v, (int)__builtin_ctzll(rem));
        const uint64_t m = __ballot(v == v0) & rem;
        if ((m >> l) & 1ull) same = m;
        rem &= ~m;
    }
    if (rem) {
        const uint64_t m = lg_match(v, nb, rem);
        if ((rem >> l) & 1ull) same = m;
    }
    return same;
}
// The voxels of the 27 cells around voxel q, visited by one wave: lanes 0-8 look up the nine
// (z, y) rows, whose cells x-1..x+1 are consecutive in ord; then the 64 lanes stride each row.
template <class F>
__device__ __forceinline__ void lg_neighbours(const LgScratch& S, const LgGrid& g, const float4& q, F visit) {
    const uint32_t l = lane_id();
    uint32_t cx, cy, cz;
    g.cell(q, cx, cy, cz);
    uint32_t b = 0, e = 0;
    if (l < 9) {
        const int zz = (int)cz + (int)(l / 3) - 1, yy = (int)cy + (int)(l % 3) - 1;
        if (zz >= 0 && zz < (int)g.n[2] && yy >= 0 && yy < (int)g.n[1]) {
            const uint32_t xlo = cx > 0 ? cx - 1 : 0u, xhi = cx + 1 < g.n[0] ? cx + 1 : g.n[0] - 1;
            b = S.cstart[g.id(xlo, (uint32_t)yy, (uint32_t)zz)];
            e = S.cstart[g.id(xhi, (uint32_t)yy, (uint32_t)zz) + 1];
        }
    }
    // the nine row ranges as one index space over the lanes: ceil(total / 64) rounds instead of
    // one round (or more) per row
    uint32_t rb[9], rx[9], tot = 0;
#pragma unroll
    for (int r = 0; r < 9; r++) {
        rb[r] = (uint32_t)__builtin_amdgcn_readlane((int)b, r);
        rx[r] = tot;
        tot += (uint32_t)__builtin_amdgcn_readlane((int)e, r) - rb[r];
    }
    // two rounds' neighbour indices loaded together, then visited
    for (uint32_t t0 = l; t0 < tot; t0 += 128) {
        uint32_t o[2];
#pragma unroll
        for (int u = 0; u < 2; u++) {
            const uint32_t t = t0 + 64u * u;
            uint32_t j = 0;
#pragma unroll
            for (int r = 0; r < 9; r++)
                if (t >= rx[r]) j = rb[r] + (t - rx[r]);   // the last row starting at or before t
            o[u] = t < tot ? S.ord[j] : 0xffffffffu;
        }
#pragma unroll
        for (int u = 0; u < 2; u++)
            if (o[u] != 0xffffffffu) visit(o[u]);
    }
}
__device__ __forceinline__ bool lg_adjacent(const float4& q, const float4& p, float r2) {
    const float ddx = q.x - p.x, ddy = q.y - p.y, ddz = q.z - p.z;
    float acc = ddx * ddx;
    acc = acc + ddy * ddy;
    acc = acc + ddz * ddz;
    return acc < r2;
}
// forest: par[v] = lowest adjacent voxel index, or v (one wave per voxel)
__device__ __forceinline__ void lg_forest_one(const LgScratch& S, const CgDevParams& P, uint32_t v) {
    const LgGrid g(S.meta);
    const float4 q = S.vox[v];
    uint32_t lo = v;
    lg_neighbours(S, g, q, [&](uint32_t o) {   // (the load depends on o < v only: the visits' loads go together)
        if (o < v) {
            const float4 p = S.vox[o];
            if (o < lo && lg_adjacent(q, p, P.r2)) lo = o;
        }
    });
    lo = wave_umin(lo);
    if (lane_id() == 0) S.par[v] = lo;
}
__global__ __launch_bounds__(CG_BLOCK) void lg_forest(LgScratch S, CgDevParams P) {
    for (uint32_t v = blockIdx.x * WAVES + wave_id(), V = S.meta[LG_V]; v < V; v += gridDim.x * WAVES)
        lg_forest_one(S, P, v);
}
// flatten: every voxel's parent replaced by its forest root. Each thread chases its voxels' paths
// to the root, four chases interleaved, and writes the root in place: a path read meanwhile
// sees either the old parent or the root, both ancestors on its way to the same root, so the
// chases need no rounds or barriers (the pointer-jumping rounds this replaces took two
// barriers each). In LDS when V <= LG_FLAT_LDS, else on the HBM array (one workgroup).
#define LG_FLAT_LDS 32768
template <class P32>
__device__ __forceinline__ void lg_roots_in_place(P32 par, uint32_t V) {
    const uint32_t tid = threadIdx.x;
    for (uint32_t vb = 0; vb < V; vb += 4 * CG_BLOCK) {
        uint32_t r[4], p[4];
        bool go = true;
#pragma unroll
        for (int q = 0; q < 4; q++) r[q] = min(vb + (uint32_t)q * CG_BLOCK + tid, V - 1);
        while (go) {
#pragma unroll
            for (int q = 0; q < 4; q++) p[q] = par[r[q]];
            go = false;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                go |= p[q] != r[q];
                r[q] = p[q];
            }
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t v = vb + (uint32_t)q * CG_BLOCK + tid;
            if (v < V) par[v] = r[q];
        }
    }
}
__global__ __launch_bounds__(CG_BLOCK) void lg_flatten(LgScratch S) {
    __shared__ uint32_t lpar[LG_FLAT_LDS];
    const uint32_t tid = threadIdx.x, V = S.meta[LG_V];
    if (V == 0) return;
    if (V <= LG_FLAT_LDS) {
        lds_u32* const lp = (lds_u32*)(uint32_t*)lpar;
        for (uint32_t vb = 0; vb < V; vb += 16 * CG_BLOCK) {   // sixteen loads in flight per thread
            uint32_t pv[16];
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint32_t v = vb + (uint32_t)q * CG_BLOCK + tid;
                pv[q] = v < V ? S.par[v] : 0u;
            }
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint32_t v = vb + (uint32_t)q * CG_BLOCK + tid;
                if (v < V) lp[v] = pv[q];
            }
        }
        __syncthreads();
        lg_roots_in_place(lp, V);
        __syncthreads();
        for (uint32_t x = tid; x < V; x += CG_BLOCK) S.par[x] = lp[x];
    } else {
        lg_roots_in_place(S.par, V);
    }
}
// cross-tree edges (v < o): united unless both ends already share a parent
__device__ __forceinline__ void lg_cross_one(const LgScratch& S, const CgDevParams& P, uint32_t v, uint32_t vb) {
    const LgGrid g(S.meta);
    const float4 q = S.vox[v];
    const uint32_t pv = S.par[v];
    const uint64_t lt = (1ull << lane_id()) - 1ull;
    lg_neighbours(S, g, q, [&](uint32_t o) {
        // each edge once, from its lower end: the higher neighbours only are loaded. Plain loads,
        // issued together: a stale pair of equal parents still lies in one tree (trees only
        // merge); different ones go through uf_union, which re-reads
        const bool hi = o > v;
        float4 p = q;
        uint32_t po = pv;
        if (hi) { p = S.vox[o]; po = S.par[o]; }
        // pv / po (the flattened parents) lie on v's / o's paths to their roots (unions only
        // hook roots under roots), so the finds start there. The lanes whose edges join v's tree
        // to the same parent po make one union, by the lowest of them: the others' would only
        // race it for the same root (a failed CAS and a second find each)
        const bool cut = hi && po != pv && lg_adjacent(q, p, P.r2);
        const uint64_t need = __ballot(cut);
        if (need) {
            const uint64_t same = lg_match_few(po, vb, need);
            if (cut && (same & lt) == 0ull) uf_union(S.par, pv, po);
        }
    });
}
__global__ __launch_bounds__(CG_BLOCK) void lg_cross(LgScratch S, CgDevParams P) {
    const uint32_t V = S.meta[LG_V], vb = V ? 32u - (uint32_t)__builtin_clz(V) : 1u;   // (parents < V)
    for (uint32_t v = blockIdx.x * WAVES + wave_id(); v < V; v += gridDim.x * WAVES)
        lg_cross_one(S, P, v, vb);
}
// roots and component sizes: the lanes of a wave that share a root add their count with one
// atomic (a component's voxels are mostly neighbours in idx order; same-address atomics from
// every voxel of a large component serialise)
__global__ __launch_bounds__(CG_BLOCK) void lg_find(LgScratch S) {
    const uint32_t v = blockIdx.x * CG_BLOCK + threadIdx.x, V = S.meta[LG_V];
    const bool in = v < V;
    uint32_t r = 0;
    if (in) {
        r = uf_find(S.par, v);
        S.lab[v] = r;
    }
    uint64_t m = __ballot(in);
    while (m) {
        const uint32_t lead = (uint32_t)__builtin_amdgcn_readlane((int)r, (int)__builtin_ctzll(m));
        const uint64_t same = __ballot(in && r == lead) & m;
        if (lane_id() == (uint32_t)__builtin_ctzll(m)) atomicAdd(&S.cnt[lead], (uint32_t)__builtin_popcountll(same));
        m &= ~same;
    }
}
struct KeepRoot {   // component seeds whose size passes min <= size <= max, in seed order
    const uint32_t* lab; const uint32_t* cnt; uint32_t lo, hi;
    __device__ uint32_t operator()(uint32_t v) const {
        const uint32_t c = cnt[v];
        return (lab[v] == v && c >= lo && c <= hi) ? 1u : 0u;
    }
};
struct KeepEmit {
    const uint32_t* cnt; uint32_t* droot; uint32_t* dsz;
    __device__ void operator()(uint32_t v, uint32_t d) const { droot[d] = v; dsz[d] = cnt[v]; }
};

#define LG_ORDER_LDS 8192
// cluster order: PCL sorts the reversed discovery list ascending by size with std::sort
// (restated, cg_sort.h); <= 16 clusters is an insertion sort: (size desc, seed asc)
__global__ __launch_bounds__(CG_BLOCK) void lg_order(LgScratch S) {
    __shared__ int32_t stk[3 * CG_SORT_STACK];
    __shared__ uint32_t red[8 * WAVES];
    const uint32_t tid = threadIdx.x;
    const uint32_t C = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.meta[LG_C]);
    if (C > CG_SORT_THRESHOLD && C <= 64) {
        // wave 0 runs the introsort restatement on records held one per lane (scalar control,
        // v_readlane / v_writelane element accesses instead of dependent LDS round trips)
        if (wave_id() == 0) {
            const uint32_t l = lane_id();
            const uint32_t big = (uint32_t)__builtin_amdgcn_readfirstlane((int)wave_umax(l < C ? S.dsz[C - 1 - l] : 0u));
            int32_t st[3] = {0, 0, 0};
            const CgWaveStack sk{st};
            uint32_t d = 0;
            if (big < 65536u) {   // (size << 16 | d) records in one VGPR, ballot-scan introsort
                uint32_t r = l < C ? (S.dsz[C - 1 - l] << 16) | (C - 1 - l) : 0u;
                cg_std_sort_wave32(r, (int)C);
                d = r & 0xffffu;
            } else {
                uint32_t lo = 0, hi = 0;
                if (l < C) { lo = C - 1 - l; hi = S.dsz[lo]; }
                const CgWaveRegs64 f{&lo, &hi, 0};
                cg_std_sort(f, (long)C, [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); }, sk);
                d = lo;
            }
            if (l < C) {
                S.fin[C - 1 - l] = d;
                S.rank[d] = C - 1 - l;
            }
        }
    } else if (C > CG_SORT_THRESHOLD) {
        // one lane runs the introsort restatement, on LDS records when they fit
        __shared__ uint64_t lrec[LG_ORDER_LDS];
        uint64_t* rec = C <= LG_ORDER_LDS ? lrec : S.key0;
        for (uint32_t i = tid; i < C; i += CG_BLOCK) {
            const uint32_t d = C - 1 - i;
            rec[i] = ((uint64_t)S.dsz[d] << 32) | d;
        }
        __syncthreads();
        if (tid == 0)
            cg_std_sort(rec, (long)C, [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); }, stk);
        __syncthreads();
        for (uint32_t k = tid; k < C; k += CG_BLOCK) {
            const uint32_t d = (uint32_t)rec[C - 1 - k];
            S.fin[k] = d;
            S.rank[d] = k;
        }
    } else {
        for (uint32_t d = tid; d < C; d += CG_BLOCK) {
            const uint32_t sd = S.dsz[d];
            uint32_t r = 0;
            for (uint32_t e = 0; e < C; e++) {
                const uint32_t se = S.dsz[e];
                r += (se > sd) || (se == sd && e < d);
            }
            S.rank[d] = r;
            S.fin[r] = d;
        }
    }
    __syncthreads();
    const uint32_t tot = block_scan(C, [&](uint32_t k) -> uint32_t { return S.dsz[S.fin[k]]; },
                                    [&](uint32_t k, uint32_t e) { S.off[k] = e; }, red);
    if (tid == 0) S.off[C] = tot;
    for (uint32_t d = tid; d < C; d += CG_BLOCK) S.rk[S.droot[d]] = S.rank[d];
}
// labels (cluster rank or -1) and the (rank, voxel) keys of the CSR sort
__global__ __launch_bounds__(CG_BLOCK) void lg_labels(CgLaunch L, LgScratch S, uint32_t f, uint32_t VB) {
    const uint32_t v = blockIdx.x * CG_BLOCK + threadIdx.x, V = S.meta[LG_V];
    // kept keys: rank < C in bits [VB, VB + bits(C)); dropped keys are all ones there, so one
    // bit more orders them last and the digits above are skipped
    if (v == 0) S.meta[LG_SORT_LIM] = VB + (32u - (uint32_t)__clz(S.meta[LG_C])) + 1u;
    if (v >= V) return;
    const uint32_t rk = S.rk[S.lab[v]];
    (L.lab + (uint64_t)f * L.cap)[v] = rk == 0xffffffffu ? -1 : (int32_t)rk;
    S.key0[v] = rk == 0xffffffffu ? ~0ull : (((uint64_t)rk << VB) | v);
    S.val0[v] = v;
}
// CSR indices (ascending voxel index inside each cluster), per-cluster centroid + radial push
// (src/cone_detection.cpp:261-279), offsets and the frame header
__device__ __forceinline__ void lg_csr_one(const CgLaunch& L, const CgDevParams& P, const LgScratch& S, uint32_t f,
                                           uint32_t VB, int buf, uint32_t Mtot, uint32_t K, uint32_t b) {
    const uint32_t i = b * CG_BLOCK + threadIdx.x;
    const uint32_t* m = S.meta;
    const uint32_t C = m[LG_C], tot = C ? S.off[C] : 0u;
    const uint64_t* key = buf ? S.key1 : S.key0;
    if (i < tot) (L.idx + (uint64_t)f * L.cap)[i] = (int32_t)(key[i] & ((1ull << VB) - 1ull));
    if (i <= C) (L.offs + (uint64_t)f * (L.cap + 1))[i] = C ? (int32_t)S.off[i] : 0;
    if (i == 0) {
        uint32_t* h = L.hdr + (uint64_t)f * 8;
        h[CG_HDR_N] = L.n_points;
        h[CG_HDR_K] = K;
        h[CG_HDR_M] = Mtot;
        h[CG_HDR_V] = m[LG_V];
        h[CG_HDR_C] = C;
        h[CG_HDR_FLAGS] = CG_F_GLOBAL_SCRATCH | (m[LG_PASS] ? CG_F_VOXEL_PASSTHROUGH : 0u) |
                          (P.voxel_order == CG_VOXEL_ORDER_PCL ? 0u : CG_F_VOXEL_POINT_ORDER);
        h[CG_HDR_ERR] = 0u;
    }
}
__device__ __forceinline__ void lg_centroids_one(const CgLaunch& L, const CgDevParams& P, const LgScratch& S,
                                                 uint32_t f, uint32_t k, const uint64_t* key, uint64_t vmask) {
    // one wave per cluster: the lanes fetch 64 members at a time, the sums run through them in
    // ascending member order (lane order), as the reference's loop does
    const uint32_t l = lane_id();
    const uint32_t s = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.off[k]);
    const uint32_t e = (uint32_t)__builtin_amdgcn_readfirstlane((int)S.off[k + 1]);
    float x = 0.0f, y = 0.0f;
    for (uint32_t g0 = s; g0 < e; g0 += 8 * 64) {   // eight chunks of 64 members in flight
        float px[8], py[8];
        uint32_t vi[8];
#pragma unroll
        for (int c = 0; c < 8; c++) {   // all member indices first, then all voxel loads
            const uint32_t i = g0 + 64 * c + l;
            vi[c] = i < e ? (uint32_t)(key[i] & vmask) : 0xffffffffu;   // lg_csr's member index
        }
#pragma unroll
        for (int c = 0; c < 8; c++) {
            px[c] = py[c] = 0.f;
            if (vi[c] != 0xffffffffu) { const float4 p = S.vox[vi[c]]; px[c] = p.x; py[c] = p.y; }
        }
#pragma unroll
        for (int c = 0; c < 8; c++) {
            const uint32_t i0 = g0 + 64 * c;
            const uint32_t n = i0 < e ? min(64u, e - i0) : 0u;
            float z0 = 0.f, z1 = 0.f;   // two sums only (lg_sum_lanes' zero terms stay zero)
            lg_sum_lanes(n, px[c], py[c], 0.f, 0.f, x, y, z0, z1);
        }
    }
    if (l != 0) return;
    const int j = (int)(e - s);
    const float px = x / (float)j, py = y / (float)j;
    const double Sq = ((double)px * (double)px + (double)py * (double)py) + 0.0;
    const float len = (float)__builtin_sqrt(Sq);
    const float qx = (float)((double)px + (double)(px / len) * P.ext);
    const float qy = (float)((double)py + (double)(py / len) * P.ext);
    (L.cen + (uint64_t)f * L.cap)[k] = make_float2(qx, qy);
}
// CSR, header and cluster centroids in one launch: the first cb workgroups write the CSR
// arrays, the others sum the clusters (member indices from the sorted keys, as lg_csr reads them)
// (the backend sized on the device: Mtot = K = CG_K_FROM_META read from the meta words, and buf
// < 0: the sort's buffer from the passes its key width needed, lg_rs_passes over [VB, sort_hi))
__device__ __forceinline__ uint32_t lg_rs_passes(uint32_t lo, uint32_t hi, uint32_t lim) {
    const uint32_t top = min(hi, lim);
    return top > lo ? (top - lo + 7u) / 8u : 0u;
}
__global__ __launch_bounds__(CG_BLOCK) void lg_csr_centroids(CgLaunch L, CgDevParams P, LgScratch S, uint32_t f,
                                                             uint32_t VB, int buf, uint32_t Mtot, uint32_t K,
                                                             uint32_t cb, uint32_t sort_hi) {
    if (Mtot == CG_K_FROM_META) Mtot = S.meta[LG_MALL];
    if (K == CG_K_FROM_META) K = S.meta[LG_KHDR];
    if (buf < 0) buf = (int)(lg_rs_passes(VB, sort_hi, S.meta[LG_SORT_LIM]) & 1u);   // (device-sized)
    if (blockIdx.x < cb) {
        lg_csr_one(L, P, S, f, VB, buf, Mtot, K, blockIdx.x);
        return;
    }
    const uint64_t* key = buf ? S.key1 : S.key0;
    const uint64_t vmask = (1ull << VB) - 1ull;
    for (uint32_t k = (blockIdx.x - cb) * WAVES + wave_id(), C = S.meta[LG_C]; k < C; k += (gridDim.x - cb) * WAVES)
        lg_centroids_one(L, P, S, f, k, key, vmask);
}

// ------------------------------------------------------------------------------------------
// The clustering's tail in one workgroup (the device-sized path): roots, component sizes, the
// size filter, PCL's cluster order, labels, the CSR and the per-cluster centroids -- what
// lg_find, the KeepRoot scan, lg_order, lg_labels, the CSR's rank sort and lg_csr_centroids do
// in seven launches, here in one (the stages are short: a few thousand voxels, tens of clusters;
// each launch boundary cost more than its stage). The voxel arrays live in LDS below
// LG_TAIL_LDS voxels, else in the HBM scratch (same code, slower).
//   A: parents, then the kept roots (droot, ascending = PCL's discovery order), then the
//      cluster offsets; B: each voxel's root, then its cluster rank (or ~0);
//   Cc: component sizes by root, then each root's cluster rank; D: kept sizes (dsz);
//   Ef: the cluster order (fin), then the CSR member list; B and Cc hold the members' x, y in
//   CSR order for the centroid sums at the end (LDS form).
// The CSR lists cluster k's members in ascending voxel index (PCL's extract sorts them): each
// wave places a block of consecutive voxels at per-(wave, cluster) starts (C5: 36 clusters,
// 5,363 voxels).
#define LG_TAIL_LDS 7168
// LDS word add (ds_add_u32) or global atomic add, by pointer kind
__device__ __forceinline__ void lg_add(lds_u32* p, uint32_t v) { __atomic_fetch_add(p, v, __ATOMIC_RELAXED); }
__device__ __forceinline__ void lg_add(uint32_t* p, uint32_t v) { atomicAdd(p, v); }
template <class K>
__device__ __forceinline__ void lg_tail_body(const CgLaunch& L, const CgDevParams& P, const LgScratch& S, uint32_t f,
                                             uint32_t V, typename K::P32 A, typename K::P32 B, typename K::P32 Cc,
                                             typename K::P32 D, typename K::P32 Ef, bool lds, uint32_t* red,
                                             int32_t* stk) {
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    const uint64_t lt = (1ull << l) - 1ull;
    CG_HOOK_LG_STAMP(S, 1);
    // 1. parents (flattened by lg_flatten, then united across trees by lg_cross), sixteen
    //    loads in flight per thread (one round trip for C5's 5,363 voxels); the size counters
    //    zeroed
    if (lds) {
        for (uint32_t vb = 0; vb < V; vb += 16 * CG_BLOCK) {
            uint32_t pv[16];
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint32_t v = vb + (uint32_t)q * CG_BLOCK + tid;
                pv[q] = v < V ? S.par[v] : 0u;
            }
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint32_t v = vb + (uint32_t)q * CG_BLOCK + tid;
                if (v < V) { A[v] = pv[q]; Cc[v] = 0u; }
            }
        }
    } else {
        for (uint32_t v = tid; v < V; v += CG_BLOCK) Cc[v] = 0u;
    }
    __syncthreads();
    CG_HOOK_LG_STAMP(S, 2);
    // 2. roots (the forest's roots are the components' lowest indices = PCL's seeds) and the
    //    component sizes (LDS atomics: the LDS unit takes a wave's same-address adds in turn,
    //    cheaper than matching the lanes' roots first)
    for (uint32_t vb = 0; vb < V; vb += 4 * CG_BLOCK) {   // four chases interleaved
        uint32_t r[4], p[4];
        bool go = true;
#pragma unroll
        for (int q = 0; q < 4; q++) r[q] = min(vb + (uint32_t)q * CG_BLOCK + tid, V - 1);
        while (go) {
#pragma unroll
            for (int q = 0; q < 4; q++) p[q] = A[r[q]];
            go = false;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                go |= p[q] != r[q];
                r[q] = p[q];
            }
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const uint32_t v = vb + (uint32_t)q * CG_BLOCK + tid;
            if (v < V) {
                B[v] = r[q];
                lg_add(&Cc[r[q]], 1u);
            }
        }
    }
    __syncthreads();
    CG_HOOK_LG_STAMP(S, 3);   // (stage 3, the sizes, is part of stage 2)
    CG_HOOK_LG_STAMP(S, 4);
    // 4. the size filter over the seeds in ascending order (PCL's discovery order): droot in A,
    //    sizes in D; each thread scans `per` consecutive voxels (a ballot form over 64-voxel
    //    chunks measured no faster, profiles/r5_c5_tail_csr_ab.txt)
    uint32_t C = 0;
    const uint32_t per = (V + CG_BLOCK - 1) / CG_BLOCK;
    const uint32_t v0 = min(V, tid * per), v1 = min(V, v0 + per);
    uint32_t mine = 0;
    for (uint32_t v = v0; v < v1; v++) {
        const uint32_t c = Cc[v];
        mine += (B[v] == v && c >= P.min_cl && c <= P.max_cl) ? 1u : 0u;
    }
    const uint32_t inc = wave_incl_scan(mine);
    if (l == 63) red[w] = inc;
    __syncthreads();
    uint32_t base = inc - mine;
    for (uint32_t q = 0; q < WAVES; q++) {
        base += q < w ? red[q] : 0u;
        C += red[q];
    }
    for (uint32_t v = v0; v < v1; v++) {
        const uint32_t c = Cc[v];
        if (B[v] == v && c >= P.min_cl && c <= P.max_cl) { A[base] = v; D[base] = c; base++; }
    }
    __syncthreads();
    for (uint32_t v = tid; v < V; v += CG_BLOCK) Cc[v] = 0xffffffffu;   // ranks by root (~0: dropped)
    CG_HOOK_LG_STAMP(S, 5);
    // 5. PCL's cluster order: the reversed discovery list sorted by size with std::sort
    //    (cg_sort.h); fin (Ef): cluster k -> its index d in the discovery list
    if (C > CG_SORT_THRESHOLD && C <= 64) {
        // one wave, one record (size << 32 | d) per lane: pw_range64 is libstdc++'s introsort on
        // at most 64 records in registers (the PCL voxel order's wave form), here with the
        // whole sort's depth budget; the records go out through Ef's upper half (free)
        if (w == 0) {
            typename K::P64 rec = (typename K::P64)(Ef + ((LG_TAIL_LDS / 2) & ~1u));
            if (!lds) rec = (typename K::P64)S.key0;
            if (l < C) rec[l] = ((uint64_t)D[C - 1 - l] << 32) | (C - 1 - l);
            pw_range64(rec, 0u, C, (uint32_t)(2 * cg_lg((long)C)), [&](uint32_t i, uint64_t r) {
                Ef[C - 1 - i] = (uint32_t)r;
            });
        }
    } else if (C > CG_SORT_THRESHOLD) {   // one lane, the records in the HBM scratch (rare)
        uint64_t* rec = S.key0;
        for (uint32_t i = tid; i < C; i += CG_BLOCK) {
            const uint32_t d = C - 1 - i;
            rec[i] = ((uint64_t)D[d] << 32) | d;
        }
        __syncthreads();
        if (tid == 0) cg_std_sort(rec, (long)C, [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); }, stk);
        __syncthreads();
        for (uint32_t k = tid; k < C; k += CG_BLOCK) Ef[k] = (uint32_t)rec[C - 1 - k];
    } else {   // <= 16 clusters: an insertion sort, (size desc, seed asc)
        for (uint32_t d = tid; d < C; d += CG_BLOCK) {
            const uint32_t sd = D[d];
            uint32_t r = 0;
            for (uint32_t e = 0; e < C; e++) {
                const uint32_t se = D[e];
                r += (se > sd) || (se == sd && e < d);
            }
            Ef[r] = d;
        }
    }
    __syncthreads();
    for (uint32_t k = tid; k < C; k += CG_BLOCK) Cc[A[Ef[k]]] = k;   // each kept root's rank
    __syncthreads();
    CG_HOOK_LG_STAMP(S, 6);
    // 6. cluster offsets in A (the discovery list is used up), each thread over consecutive k
    {
        const uint32_t pk = (C + CG_BLOCK - 1) / CG_BLOCK;
        const uint32_t k0 = min(C, tid * pk), k1 = min(C, k0 + pk);
        uint32_t s = 0;
        for (uint32_t k = k0; k < k1; k++) s += D[Ef[k]];
        const uint32_t in2 = wave_incl_scan(s);
        if (l == 63) red[w] = in2;
        __syncthreads();
        uint32_t b2 = in2 - s, tot = 0;
        for (uint32_t q = 0; q < WAVES; q++) {
            b2 += q < w ? red[q] : 0u;
            tot += red[q];
        }
        for (uint32_t k = k0; k < k1; k++) {
            const uint32_t c = D[Ef[k]];
            A[k] = b2;
            b2 += c;
        }
        if (tid == 0) A[C] = tot;
    }
    __syncthreads();
    CG_HOOK_LG_STAMP(S, 7);
    // 7. labels (cluster rank or -1) to the output; B becomes each voxel's rank
    int32_t* const lab_out = L.lab + (uint64_t)f * L.cap;
    for (uint32_t v = tid; v < V; v += CG_BLOCK) {
        const uint32_t rk = Cc[B[v]];
        lab_out[v] = rk == 0xffffffffu ? -1 : (int32_t)rk;
        B[v] = rk;
    }
    __syncthreads();
    CG_HOOK_LG_STAMP(S, 8);
    // 8. the CSR: every cluster's members in ascending voxel index. Each wave takes a block of
    //    consecutive voxels: it counts its members per cluster (D as WAVES x C counters, free
    //    now), the counts become each wave's start per cluster, and the wave writes its members
    //    there in voxel order, each 64-voxel chunk's same-cluster lanes found by lg_match. (More
    //    than (V + 2) / WAVES clusters: one wave per cluster collects them by ballots instead.)
    int32_t* const idx_out = L.idx + (uint64_t)f * L.cap;
    typename K::P32 XY = B;   // LDS form: the members' x, y in CSR order (two words per slot:
                              // B and Cc are adjacent), for stage 10
    bool xy_ready = false;
    if ((uint64_t)WAVES * C <= V + 2) {
        const uint32_t blk = ((V + WAVES * 64 - 1) / (WAVES * 64)) * 64;   // voxels per wave
        const uint32_t wb0 = min(V, w * blk), wb1 = min(V, wb0 + blk);
        typename K::P32 cw = D + w * C;
        for (uint32_t k = l; k < C; k += 64) cw[k] = 0u;
        const uint32_t cbits = cg_bits_of(C);
        auto to_starts = [&]() {   // counts -> each wave's start per cluster
            for (uint32_t k = tid; k < C; k += CG_BLOCK) {
                uint32_t run = A[k];
                for (uint32_t q = 0; q < WAVES; q++) {
                    const uint32_t c = D[q * C + k];
                    D[q * C + k] = run;
                    run += c;
                }
            }
        };
        if constexpr (K::in_lds) {
            // LDS form (at most NCH chunks per wave): the chunks' ranks and same-rank lane masks
            // stay in registers between the count and the placement, and each group's leader
            // adds its group's size (distinct addresses: no same-address atomics to serialise)
            constexpr int NCH = (LG_TAIL_LDS + WAVES * 64 - 1) / (WAVES * 64);
            uint32_t rr[NCH];
            uint64_t same[NCH];
            float cx[NCH], cy[NCH];   // the voxels' x, y, for stage 10 (loads in flight meanwhile)
#pragma unroll
            for (int j = 0; j < NCH; j++) {
                const uint32_t v = wb0 + 64u * j + l;
                rr[j] = v < wb1 ? B[v] : 0xffffffffu;
                const float4 c = v < wb1 ? S.vox[v] : make_float4(0.f, 0.f, 0.f, 0.f);
                cx[j] = c.x;
                cy[j] = c.y;
            }
#pragma unroll
            for (int j = 0; j < NCH; j++) {
                same[j] = 0ull;
                if (wb0 + 64u * j >= wb1) continue;   // (wave-uniform)
                const bool in = rr[j] != 0xffffffffu;
                same[j] = lg_match(rr[j], cbits, __ballot(in));
                if (in && (same[j] & lt) == 0ull) lg_add(&cw[rr[j]], (uint32_t)__popcll(same[j]));
            }
            __syncthreads();
            CG_HOOK_LG_STAMP(S, 64);
            to_starts();
            __syncthreads();
            CG_HOOK_LG_STAMP(S, 65);
#pragma unroll
            for (int j = 0; j < NCH; j++) {
                const uint32_t v = wb0 + 64u * j + l;
                if (rr[j] != 0xffffffffu) {
                    const uint32_t o = cw[rr[j]];   // (every lane of the group reads before its leader writes)
                    const uint32_t pos = o + (uint32_t)__popcll(same[j] & lt);
                    idx_out[pos] = (int32_t)v;
                    XY[2 * pos] = __float_as_uint(cx[j]);   // (B is in registers, Cc used up)
                    XY[2 * pos + 1] = __float_as_uint(cy[j]);
                    if ((same[j] & lt) == 0ull) cw[rr[j]] = o + (uint32_t)__popcll(same[j]);
                }
            }
            xy_ready = true;
        } else {
            for (uint32_t v = wb0 + l; v < wb1; v += 64) {
                const uint32_t rr = B[v];
                if (rr != 0xffffffffu) lg_add(&cw[rr], 1u);
            }
            __syncthreads();
            CG_HOOK_LG_STAMP(S, 64);
            to_starts();
            __syncthreads();
            CG_HOOK_LG_STAMP(S, 65);
            for (uint32_t vb = wb0; vb < wb1; vb += 64) {
                const uint32_t v = vb + l;
                const uint32_t rr = v < wb1 ? B[v] : 0xffffffffu;
                const bool in = rr != 0xffffffffu;
                const uint64_t same = lg_match(rr, cbits, __ballot(in));
                if (in) {
                    const uint32_t o = cw[rr];   // (every lane of the group reads before its first writes)
                    const uint32_t pos = o + (uint32_t)__popcll(same & lt);
                    Ef[pos] = v;
                    idx_out[pos] = (int32_t)v;
                    if ((same & lt) == 0ull) cw[rr] = o + (uint32_t)__popcll(same);
                }
            }
        }
    } else {
        for (uint32_t k = w; k < C; k += WAVES) {
            const uint32_t o = A[k], sz = A[k + 1] - o;
            uint32_t got = 0;
            for (uint32_t b0 = 0; b0 < V && got < sz; b0 += 64) {
                const uint32_t v = b0 + l;
                const bool hit = v < V && B[v] == k;
                const uint64_t m = __ballot(hit);
                if (hit) {
                    const uint32_t pos = o + got + (uint32_t)__popcll(m & lt);
                    Ef[pos] = v;
                    idx_out[pos] = (int32_t)v;
                }
                got += (uint32_t)__popcll(m);
            }
        }
    }
    __syncthreads();
    CG_HOOK_LG_STAMP(S, 9);
    // 9. (LDS form, when the ballot form above has not placed them) the members' x, y in CSR
    //    order, next to each other, so each cluster's sum below reads one contiguous run
    const uint32_t nmem = A[C];
    if (K::in_lds && !xy_ready && nmem) {
        for (uint32_t pb = 0; pb < nmem; pb += 16 * CG_BLOCK) {   // sixteen loads in flight per thread
            float cx[16], cy[16];
#pragma unroll
            for (int q = 0; q < 16; q++) {   // (clamped: no branch between the loads)
                const float4 c = S.vox[Ef[min(pb + (uint32_t)q * CG_BLOCK + tid, nmem - 1)]];
                cx[q] = c.x;
                cy[q] = c.y;
            }
#pragma unroll
            for (int q = 0; q < 16; q++) {
                const uint32_t p = pb + (uint32_t)q * CG_BLOCK + tid;
                if (p < nmem) {
                    XY[2 * p] = __float_as_uint(cx[q]);
                    XY[2 * p + 1] = __float_as_uint(cy[q]);
                }
            }
        }
    }
    __syncthreads();
    CG_HOOK_LG_STAMP(S, 10);
    // 10. per-cluster centroid + radial push (src/cone_detection.cpp:261-279): float sums in
    //     ascending member order (lg_centroids_one's arithmetic), one lane per cluster: each sum
    //     is a sequential chain, kept in the lane's registers while its loads run ahead (LDS
    //     form: 16-byte reads of the contiguous x, y pairs, two members each)
    float2* const cen_out = L.cen + (uint64_t)f * L.cap;
    for (uint32_t k = tid; k < C; k += CG_BLOCK) {
        const uint32_t s0 = A[k], e0 = A[k + 1];
        float x = 0.0f, y = 0.0f;
        uint32_t i = s0;
        if constexpr (K::in_lds) {
            typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
            typedef __attribute__((address_space(3))) u32x4 lds_u32x4;
            if ((i & 1u) && i < e0) {   // to an even slot: 16-byte aligned pairs from there
                x += __uint_as_float(XY[2 * i]);
                y += __uint_as_float(XY[2 * i + 1]);
                i++;
            }
            for (; i + 16 <= e0; i += 16) {
                u32x4 q[8];
#pragma unroll
                for (int u = 0; u < 8; u++) q[u] = ((const lds_u32x4*)(XY + 2 * i))[u];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    x += __uint_as_float(q[u].x);
                    y += __uint_as_float(q[u].y);
                    x += __uint_as_float(q[u].z);
                    y += __uint_as_float(q[u].w);
                }
            }
            for (; i < e0; i++) {
                x += __uint_as_float(XY[2 * i]);
                y += __uint_as_float(XY[2 * i + 1]);
            }
        } else {
            for (; i + 8 <= e0; i += 8) {
                float px[8], py[8];
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const float4 c = S.vox[Ef[i + u]];
                    px[u] = c.x;
                    py[u] = c.y;
                }
#pragma unroll
                for (int u = 0; u < 8; u++) { x += px[u]; y += py[u]; }
            }
            for (; i < e0; i++) {
                const float4 c = S.vox[Ef[i]];
                x += c.x;
                y += c.y;
            }
        }
        {
            const int j = (int)(e0 - s0);
            const float qx0 = x / (float)j, qy0 = y / (float)j;
            const double Sq = ((double)qx0 * (double)qx0 + (double)qy0 * (double)qy0) + 0.0;
            const float len = (float)__builtin_sqrt(Sq);
            const float qx = (float)((double)qx0 + (double)(qx0 / len) * P.ext);
            const float qy = (float)((double)qy0 + (double)(qy0 / len) * P.ext);
            cen_out[k] = make_float2(qx, qy);
        }
    }
    CG_HOOK_LG_STAMP(S, 11);
    // 11. offsets and the frame header
    int32_t* const offs_out = L.offs + (uint64_t)f * (L.cap + 1);
    for (uint32_t i = tid; i <= C; i += CG_BLOCK) offs_out[i] = C ? (int32_t)A[i] : 0;
    if (tid == 0) {
        uint32_t* m = S.meta;
        m[LG_C] = C;
        uint32_t* h = L.hdr + (uint64_t)f * 8;
        h[CG_HDR_N] = L.n_points;
        h[CG_HDR_K] = m[LG_KHDR];
        h[CG_HDR_M] = m[LG_MALL];
        h[CG_HDR_V] = V;
        h[CG_HDR_C] = C;
        h[CG_HDR_FLAGS] = CG_F_GLOBAL_SCRATCH | (m[LG_PASS] ? CG_F_VOXEL_PASSTHROUGH : 0u) |
                          (P.voxel_order == CG_VOXEL_ORDER_PCL ? 0u : CG_F_VOXEL_POINT_ORDER);
        h[CG_HDR_ERR] = m[LG_PQ_TIMEOUT] ? CG_HDR_E_WAIT : 0u;   // (the fetch fails on it)
    }
    CG_HOOK_LG_STAMP(S, 12);
}
__global__ __launch_bounds__(CG_BLOCK) void lg_cluster_tail(CgLaunch L, CgDevParams P, LgScratch S, uint32_t f) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[5 * LG_TAIL_LDS];   // (16-byte reads in stage 10)
    __shared__ uint32_t red[8 * WAVES];
    __shared__ int32_t stk[3 * CG_SORT_STACK];
    const uint32_t V = S.meta[LG_V];
    if (V < LG_TAIL_LDS) {
        lds_u32* const b = (lds_u32*)(uint32_t*)lds;
        lg_tail_body<PbLds>(L, P, S, f, V, b, b + LG_TAIL_LDS, b + 2 * LG_TAIL_LDS, b + 3 * LG_TAIL_LDS,
                            b + 4 * LG_TAIL_LDS, true, red, stk);
    } else {
        lg_tail_body<PbGen>(L, P, S, f, V, S.par, S.lab, S.cnt, S.dsz, S.fin, false, red, stk);
    }
}

// Gathered survivors of a tiled frame (cg_tile_backend): meta reset, survivors copied into
// scratch, the merged counts written where the backend reads them.
__global__ void lg_set_counts(LgScratch S, uint32_t K, uint32_t Ms, uint32_t nfin, uint32_t b0, uint32_t b1,
                              uint32_t b2, uint32_t b3, uint32_t b4, uint32_t b5) {
    if (threadIdx.x != 0) return;
    uint32_t* m = S.meta;
    m[LG_K] = K; m[LG_MS] = Ms; m[LG_NFIN] = nfin;
    m[LG_BMIN] = b0; m[LG_BMIN + 1] = b1; m[LG_BMIN + 2] = b2;
    m[LG_BMAX] = b3; m[LG_BMAX + 1] = b4; m[LG_BMAX + 2] = b5;
}
// The tile's counts as cg_tile_decide reports them (K, survivors, finite survivors, bounds
// keys min x3, max x3), written on the device for a device-side merge.
__global__ void lg_tile_counts(LgScratch S, uint32_t* out) {
    const uint32_t t = threadIdx.x;
    if (t >= CG_TILE_COUNTS) return;
    const uint32_t* m = S.meta;
    out[t] = t == 0 ? m[LG_K] : t == 1 ? m[LG_MS] : t == 2 ? m[LG_NFIN] : t < 6 ? m[LG_BMIN + t - 3] : m[LG_BMAX + t - 6];
}
int cg_large_tile_counts(LgScratch S, uint32_t* d_counts, hipStream_t s) {
    hipLaunchKernelGGL(lg_tile_counts, dim3(1), dim3(64), 0, s, S, d_counts);
    return hipGetLastError();
}
__global__ __launch_bounds__(CG_BLOCK) void lg_check_sorted(LgScratch S, uint32_t n) {
    const uint32_t j = blockIdx.x * CG_BLOCK + threadIdx.x;
    if (j + 1 < n && !(S.surv_i[j] < S.surv_i[j + 1])) S.meta[LG_UNSORTED] = 1;
}
int cg_large_set_survivors(LgScratch S, const CgDevParams& P, const float* d_points, const uint32_t* d_index,
                           uint32_t n, const uint32_t* c, hipStream_t s) {
    hipError_t e;
    hipLaunchKernelGGL(lg_init, dim3(1), dim3(64), 0, s, S, P);
    if (n) {
        if ((e = hipMemcpyAsync(S.surv_p, d_points, (size_t)n * 16, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
        if ((e = hipMemcpyAsync(S.surv_i, d_index, (size_t)n * 4, hipMemcpyDeviceToDevice, s)) != hipSuccess) return e;
    }
    if (n > 1) hipLaunchKernelGGL(lg_check_sorted, dim3((n + CG_BLOCK - 1) / CG_BLOCK), dim3(CG_BLOCK), 0, s, S, n);
    hipLaunchKernelGGL(lg_set_counts, dim3(1), dim3(64), 0, s, S, c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8]);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Host phases (cg_run_large below, and the tiles of cg_tile_*): front, decide, backend.
int cg_large_front(const CgLaunch& L, const CgDevParams& P, int kmode, LgScratch S, hipStream_t s, uint32_t f,
                   bool init, uint32_t szfl) {
    const uint32_t N = L.n_points;
    const uint32_t nch = (uint32_t)(((uint64_t)N + LG_CHUNK - 1) / LG_CHUNK);
    const bool xyzi16 = L.point_step == 16 && L.off_x == 0 && L.off_y == 4 && L.off_z == 8 && L.off_i == 12;
    if (nch == 0) {
        if (init) hipLaunchKernelGGL(lg_init, dim3(1), dim3(64), 0, s, S, P);
        return hipGetLastError();
    }
    const uint32_t fi = init ? 1u : 0u;   // lg_front's workgroup 0 resets the meta words
    // the device-sized path: lg_decide_write folds the chunks' keys (no lg_reduce_chunks launch after
    // the pipeline front); the counts' fold also sizes the detector input (LG_FOLD_SIZE)
    const bool dev = (szfl & LG_SZ_ON) != 0;
    const dim3 g(nch), b(CG_BLOCK);
#define LG_FRONT_MODES(LAY)                                                                       \
    if (kmode == CG_KMODE_PIPELINE) {                                                             \
        hipLaunchKernelGGL((lg_front<LAY, CG_KMODE_PIPELINE>), g, b, 0, s, L, P, S, f, fi);           \
        if (!dev) hipLaunchKernelGGL(lg_reduce_chunks, dim3(1), b, 0, s, S, nch, 1u, 0u, 0u);            \
    } else if (kmode == CG_KMODE_DETECT) {                                                        \
        hipLaunchKernelGGL((lg_front<LAY, CG_KMODE_DETECT>), g, b, 0, s, L, P, S, f, fi);             \
        hipLaunchKernelGGL(lg_surv_write<LAY>, g, b, 0, s, L, S, f, dev ? 4u | LG_FOLD_SIZE : 0u, N, szfl); \
        if (!dev) hipLaunchKernelGGL(lg_reduce_chunks, dim3(1), b, 0, s, S, nch, 4u, N, szfl);     \
    } else {                                                                                      \
        hipLaunchKernelGGL((lg_front<LAY, CG_KMODE_GROUND>), g, b, 0, s, L, P, S, f, fi);             \
        hipLaunchKernelGGL(lg_reduce_chunks, dim3(1), b, 0, s, S, nch, 1u, 0u, 0u);                      \
        hipLaunchKernelGGL((lg_decide<LAY, CG_KMODE_GROUND>), g, b, 0, s, L, P, S, f);            \
        hipLaunchKernelGGL(lg_reduce_chunks, dim3(1), b, 0, s, S, nch, 2u, 0u, 0u);                      \
        hipLaunchKernelGGL(lg_ground_out<LAY>, g, b, 0, s, L, P, S, f);                           \
    }
    if (xyzi16) {
        LG_FRONT_MODES(CG_LAYOUT_XYZI16)
    } else {
        LG_FRONT_MODES(CG_LAYOUT_GENERIC)
    }
#undef LG_FRONT_MODES
    return hipGetLastError();
}

int cg_large_decide(const CgLaunch& L, const CgDevParams& P, LgScratch S, hipStream_t s, uint32_t f, uint32_t szfl) {
    const uint32_t nch = (uint32_t)(((uint64_t)L.n_points + LG_CHUNK - 1) / LG_CHUNK);
    if (nch == 0) return hipSuccess;
    const bool xyzi16 = L.point_step == 16 && L.off_x == 0 && L.off_y == 4 && L.off_z == 8 && L.off_i == 12;
    const dim3 g(nch), b(CG_BLOCK);
    // the device-sized path: decisions and survivors in one launch, the counts and bounds
    // folded by its last workgroup (lg_decide_write; round 4's lg_decide + lg_surv_write pair
    // 9.2 + 11.6 us on C5). Otherwise the decisions, the survivors, then one workgroup folds
    // (folded in every lg_voxel_keys workgroup instead, 2,048 of them on C5 each reading the
    // 256 chunk records: 15.6 against 5.0 + 5.0 us, profiles/r4_c5_fold_ab.txt).
    if (szfl & LG_SZ_ON) {
        if (xyzi16)
            hipLaunchKernelGGL(lg_decide_write<CG_LAYOUT_XYZI16>, g, b, 0, s, L, P, S, f, nch, L.n_points, szfl);
        else
            hipLaunchKernelGGL(lg_decide_write<CG_LAYOUT_GENERIC>, g, b, 0, s, L, P, S, f, nch, L.n_points, szfl);
        return hipGetLastError();
    }
    if (xyzi16) {
        hipLaunchKernelGGL((lg_decide<CG_LAYOUT_XYZI16, CG_KMODE_PIPELINE>), g, b, 0, s, L, P, S, f);
        hipLaunchKernelGGL(lg_surv_write<CG_LAYOUT_XYZI16>, g, b, 0, s, L, S, f, 0u, L.n_points, szfl);
    } else {
        hipLaunchKernelGGL((lg_decide<CG_LAYOUT_GENERIC, CG_KMODE_PIPELINE>), g, b, 0, s, L, P, S, f);
        hipLaunchKernelGGL(lg_surv_write<CG_LAYOUT_GENERIC>, g, b, 0, s, L, S, f, 0u, L.n_points, szfl);
    }
    hipLaunchKernelGGL(lg_reduce_chunks, dim3(1), b, 0, s, S, nch, 2u | 4u, L.n_points, szfl);
    return hipGetLastError();
}

// Detector backend over meta[LG_MS] survivors (surv_p / surv_i, frame indices < n_total) and,
// in pipeline mode with zero_pass, the n_total - K pads; results in frame slot f.
#ifndef LG_PQ_SPARE
#define LG_PQ_SPARE 3   // partition levels beyond an even split's, for uneven median-of-three cuts
#endif
static int large_backend_from(const CgLaunch& L, const CgDevParams& P0, int kmode, LgScratch S, hipStream_t s,
                              uint32_t f, uint32_t N, uint32_t K, const uint32_t* hm);
int cg_large_backend(const CgLaunch& L, const CgDevParams& P0, int kmode, LgScratch S, hipStream_t s, uint32_t f,
                     uint32_t N, uint32_t K) {
    hipError_t e;
    uint32_t hstack[LG_META_WORDS];
    uint32_t* const hm = S.hmeta ? S.hmeta : hstack;   // pinned when the handle has one
    if ((e = hipMemcpyAsync(hm, S.meta, LG_META_WORDS * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = cg_stream_wait(s)) != hipSuccess) return e;
    return large_backend_from(L, P0, kmode, S, s, f, N, K, hm);
}
// The backend's launches, sized from the frame's meta words already on the host (hm).
static int large_backend_from(const CgLaunch& L, const CgDevParams& P0, int kmode, LgScratch S, hipStream_t s,
                              uint32_t f, uint32_t N, uint32_t K, const uint32_t* hm) {
    CgDevParams P = P0;
    const uint32_t Ms = hm[LG_MS];
    if (K == CG_K_FROM_META) K = hm[LG_K];   // pipeline frames: the ground stage's kept count
    const uint32_t npad = (kmode == CG_KMODE_PIPELINE && P.zero_pass) ? N - K : 0u;
    const uint32_t Mtot = Ms + npad;
    // PCL's order keeps at most PQ_MAXR ranges per partition level: a detector input beyond
    // PQ_MAXR * LG_PCL_CUT / 2 records (2M at LG_PCL_CUT = 2,048) is summed in point order instead, and flagged
    // (CG_F_VOXEL_POINT_ORDER): same voxels and clusters, last bits of some coordinates
    if ((uint64_t)Mtot > (uint64_t)PQ_MAXR * LG_PCL_CUT / 2) P.voxel_order = CG_VOXEL_ORDER_POINT;
    CgLaunch Lh = L;
    Lh.n_points = N;   // the header's N is the whole frame's
    if (Mtot <= CG_MMAX && !S.force_global) return cg_launch_lg_back_small(Lh, P, S, f, npad, K, s);
    // survivors arrive in frame-index order (lg_surv_write; tiles checked by lg_check_sorted):
    // then the voxel keys need no frame-index bits (PB = 0)
    const uint32_t PB = hm[LG_UNSORTED] ? bits_of((uint64_t)N + npad) : 0u;
    const uint32_t mb = std::max<uint32_t>(1, blocks_of(Mtot));
    // the voxel keys' idx width from the bounds the host already holds (lg_grid_setup's own
    // computation): one bit above the largest idx keeps non-finite points (idx all ones) last
    uint32_t key_bits = 32 + PB;
    {
        float bmn[3], bmx[3];
        uint32_t nfin = hm[LG_NFIN];
        for (int a = 0; a < 3; a++) {
            bmn[a] = nfin ? cg_fkey_inv(hm[LG_BMIN + a]) : INFINITY;
            bmx[a] = nfin ? cg_fkey_inv(hm[LG_BMAX + a]) : -INFINITY;
            if (npad) { bmn[a] = std::min(bmn[a], 0.f); bmx[a] = std::max(bmx[a], 0.f); }
        }
        nfin += npad;
        uint32_t pass = 0;
        int min_b[3], div_b[3];
        voxel_grid_setup(nfin, bmn, bmx, P, pass, min_b, div_b);
        if (pass) key_bits = PB;   // passthrough: frame-index order (nothing to sort when ordered)
        else key_bits = PB + 1 + bits_of((uint64_t)div_b[0] * (uint64_t)div_b[1] * (uint64_t)div_b[2]);
        key_bits = std::min<uint32_t>(key_bits, 32 + PB);
    }
    hipLaunchKernelGGL(lg_voxel_keys, dim3(mb), dim3(CG_BLOCK), 0, s, S, P, Mtot, N, PB, npad);
    int buf;
    uint32_t run_pb = PB;
    if (key_bits == PB || P.voxel_order != CG_VOXEL_ORDER_PCL) {
        // passthrough (a sort of the frame-index bits), or point order: a stable radix sort
        // of (idx, frame index) keys keeps each voxel's points in frame-index order
        buf = radix_sort(S, Mtot, key_bits, s);
    } else {
        // PCL's order: index_vector (finite points in frame-index order) as (idx, slot)
        // records, then std::sort's permutation of it (lg_pq_split, lg_pq_swap, lg_pcl_leaf)
        buf = PB ? radix_sort(S, Mtot, PB, s) : 0;   // unsorted tiles: frame-index order first
        uint64_t* kb[2] = {S.key0, S.key1};
        uint32_t* vb2[2] = {S.val0, S.val1};
        scan_emit(S, Mtot, -1, PclCompactFlag{kb[buf], PB, nullptr}, PclCompactEmit{kb[buf], vb2[buf], kb[buf ^ 1], PB},
                  LG_PCL_N, s);
        // the levels an even split needs until every range fits a leaf, three more for uneven
        // median-of-three cuts; levels with no range to cut return at once; then the leaves
        uint32_t levels = 0;
        while (((uint64_t)LG_PCL_CUT << levels) < Mtot) levels++;
        if (levels) levels = std::min<uint32_t>(levels + LG_PQ_SPARE, LG_PQ_LEVELS_MAX);
        if (S.pcl_levels_cap) levels = std::min(levels, S.pcl_levels_cap);
        const uint32_t tb = (Mtot + PQ_T - 1) / PQ_T;
        hipLaunchKernelGGL(lg_pq_split, dim3(std::max<uint32_t>(tb, 1)), dim3(CG_BLOCK), 0, s, S, kb[buf ^ 1], 0u);
        for (uint32_t lv = 0; lv < levels; lv++) {
            uint64_t* const Ein = lv % 2 ? kb[buf] : kb[buf ^ 1];
            uint64_t* const Eout = lv % 2 ? kb[buf ^ 1] : kb[buf];
            const uint32_t grid = tb + (1u << lv);
            if (lv) hipLaunchKernelGGL(lg_pq_split, dim3(grid), dim3(CG_BLOCK), 0, s, S, Ein, lv);
            hipLaunchKernelGGL(lg_pq_swap, dim3(grid), dim3(CG_BLOCK), 0, s, S, Ein, Eout, lv, levels - 1, (lv + 1) % 2);
        }
        hipLaunchKernelGGL(lg_pcl_leaf, dim3(std::min<uint32_t>(1024, (2u << levels) + 1)), dim3(CG_BLOCK), 0, s, S,
                           kb[buf ^ 1], kb[buf], kb[buf], vb2[buf], 0u);
        // ranges of 65-512 records: at most Mtot / 65
        hipLaunchKernelGGL(lg_pcl_mid, dim3(std::min<uint32_t>(2048, Mtot / 65 + 1)), dim3(CG_BLOCK), 0, s, S,
                           kb[buf ^ 1], kb[buf], kb[buf], vb2[buf]);
        run_pb = 0;   // sorted keys are the idx alone
    }
    const uint64_t* vkey = buf ? S.key1 : S.key0;
    // runs over the finite points (non-finite keys sort last); passthrough: every point
    scan_emit(S, Mtot, LG_SCAN_N, VoxelHead{vkey, S.meta, run_pb}, VoxelEmit{S.run}, LG_V, s);
    hipLaunchKernelGGL(lg_voxel_centroids, dim3(lg_wave_blocks(Mtot)), dim3(CG_BLOCK), 0, s,
                       Lh, S, f, Mtot, buf);
    // V is known on the device only: the clustering launches are sized for V <= Mtot and read
    // V from the meta words (no host round trip)
    const uint32_t VB = bits_of(Mtot);
    const uint32_t vb = std::max<uint32_t>(1, blocks_of(Mtot)), wb = lg_wave_blocks(Mtot);
    const uint32_t gt = LG_DCELLS_MAX / LG_TILE + 1;   // tiles past ncell return at once
    hipLaunchKernelGGL(lg_dgrid_scan, dim3(gt), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_dgrid_fill, dim3(vb), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_forest, dim3(wb), dim3(CG_BLOCK), 0, s, S, P);
    hipLaunchKernelGGL(lg_flatten, dim3(1), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_cross, dim3(wb), dim3(CG_BLOCK), 0, s, S, P);
    hipLaunchKernelGGL(lg_find, dim3(vb), dim3(CG_BLOCK), 0, s, S);
    scan_emit(S, Mtot, LG_V, KeepRoot{S.lab, S.cnt, P.min_cl, P.max_cl}, KeepEmit{S.cnt, S.droot, S.dsz}, LG_C, s);
    hipLaunchKernelGGL(lg_order, dim3(1), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_labels, dim3(vb), dim3(CG_BLOCK), 0, s, Lh, S, f, VB);
    // (rank, voxel) keys are written in voxel order: only the rank bits need sorting. rank < C
    // <= Mtot / min_cluster_size; one bit more tells ranks from the non-members' ~0 keys
    const uint32_t cmax = P.min_cl > 1 ? Mtot / P.min_cl : Mtot;
    const int kb = radix_sort(S, Mtot, VB + bits_of(std::max<uint32_t>(cmax, 1)) + 1, s, VB, S.meta + LG_V,
                               S.meta + LG_SORT_LIM);
    const uint32_t cb = blocks_of((uint64_t)Mtot + 1);
    hipLaunchKernelGGL(lg_csr_centroids, dim3(cb + wb), dim3(CG_BLOCK), 0, s, Lh, P, S, f, VB, kb, Mtot, K, cb, 0u);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// The backend sized on the device (cg_run_large, PCL's voxel order, survivors in frame-index
// order): every launch is sized from the frame's N (M <= N) and reads the counts it needs from
// the meta words, which the decisions' fold filled (LG_MALL ... LG_SMALL). Nothing returns to
// the host between the front and the results, so a frame is one uninterrupted run of launches
// (and one hipGraph replay). Workgroups past a launch's work return after one or two loads. The
// LDS backend (M <= CG_MMAX) runs last and returns unless the fold chose it; then the global
// launches before it found M = 0 and did nothing.
// The partition levels the device-sized path launches for index_vector length n (upper bound
// or a previous frame's length): an even split's until every range fits a leaf, three more for
// uneven median-of-three cuts (LG_PQ_SPARE). Levels past a frame's need return at once; ranges
// still longer than a leaf after the last are finished in HBM (lg_pcl_leaf).
static uint32_t lg_levels_for(uint32_t n, uint32_t cap) {
    uint32_t levels = 0;
    while (((uint64_t)LG_PCL_CUT << levels) < n) levels++;
    if (levels) levels = std::min<uint32_t>(levels + LG_PQ_SPARE, LG_PQ_LEVELS_MAX);
    if (cap) levels = std::min(levels, cap);
    return levels;
}
static int large_backend_dev(const CgLaunch& L, const CgDevParams& P, LgScratch S, hipStream_t s, uint32_t f,
                             uint32_t N, uint32_t levels, bool small, uint32_t szfl) {
    CgLaunch Lh = L;
    Lh.n_points = N;
    const uint32_t nmax = std::max<uint32_t>(N, 1);
    uint64_t* kb[2] = {S.key0, S.key1};
    uint32_t* vb2[2] = {S.val0, S.val1};
    // index_vector (finite points in frame-index order) as (idx, slot) records, with the voxel
    // keys computed on the way (lg_pcl_index), then std::sort's permutation of it: levels for the
    // frame's N (levels with no range return at once)
    hipLaunchKernelGGL(lg_pcl_index, dim3(std::max<uint32_t>(1, (nmax + LG_IDX_TILE - 1) / LG_IDX_TILE)), dim3(CG_BLOCK), 0,
                       s, S, P, kb[1]);
    const uint32_t tb = (nmax + PQ_T - 1) / PQ_T;
#ifndef LG_PQ_MODE
// 1: lg_pq_flow (round 6); 0: one lg_pq_level launch per partition level (round 5)
#define LG_PQ_MODE 1
#endif
#if LG_PQ_MODE != 0
    // the partition as one dataflow launch (lg_pq_flow): depth-0 records in kb[1], parity 1 in
    // kb[0]; route 5's level cap as a depth cap
    (void)levels;
    hipLaunchKernelGGL(lg_pq_flow, dim3(std::min<uint32_t>(LG_FLOW_GRID, tb + 64)), dim3(CG_BLOCK), 0, s, S, kb[1], kb[0],
                       S.pcl_levels_cap);
#ifndef LG_LEAF_GRID_MAX
#define LG_LEAF_GRID_MAX 1024   // (256 / 128: no faster on C5, profiles/r6_c5_leaf_grid_ab.txt)
#endif
    hipLaunchKernelGGL(lg_pcl_leaf, dim3(std::min<uint32_t>(LG_LEAF_GRID_MAX, nmax / LG_PCL_CUT * 2 + 2)), dim3(CG_BLOCK), 0,
                       s, S, kb[1], kb[0], kb[0], vb2[0], LG_CLEAR_FLOW);
    hipLaunchKernelGGL(lg_pcl_mid, dim3(std::min<uint32_t>(2048, nmax / 65 + 1)), dim3(CG_BLOCK), 0, s, S, kb[1], kb[0],
                       kb[0], vb2[0], 1u);
#else
    // one launch per level (lg_pq_level); a level's tiles
    // number at most tb + its ranges (<= 2^lv), taken by at most 512 workgroups (more when a
    // workgroup would hold more than PQ_OWN tiles) (level 0 always runs: with no level to cut
    // it queues the whole index_vector as a leaf)
    levels = std::max<uint32_t>(levels, 1);
    for (uint32_t lv = 0; lv < levels; lv++) {
        uint64_t* const Ein = lv % 2 ? kb[0] : kb[1];
        uint64_t* const Eout = lv % 2 ? kb[1] : kb[0];
        const uint32_t tiles = tb + (1u << lv);
        const uint32_t grid = std::min(tiles, std::max<uint32_t>(LG_PQ_GRID, (tiles + PQ_OWN - 1) / PQ_OWN));
        hipLaunchKernelGGL(lg_pq_level, dim3(grid), dim3(CG_BLOCK), 0, s, S, Ein, Eout, lv, levels - 1, (lv + 1) % 2);
    }
    hipLaunchKernelGGL(lg_pcl_leaf, dim3(std::min<uint32_t>(1024, (2u << levels) + 1)), dim3(CG_BLOCK), 0, s, S, kb[1],
                       kb[0], kb[0], vb2[0], ((levels - 1) & 1u) + 1u);
    hipLaunchKernelGGL(lg_pcl_mid, dim3(std::min<uint32_t>(2048, nmax / 65 + 1)), dim3(CG_BLOCK), 0, s, S, kb[1], kb[0],
                       kb[0], vb2[0], 0u);
#endif
    // voxel runs over the finite points (LG_SCAN_N; every point if passthrough), centroids
    scan_emit<LG_IDX_PER>(S, nmax, LG_SCAN_N, VoxelHead{S.key0, S.meta, 0u}, VoxelEmit{S.run}, LG_V, s);
    hipLaunchKernelGGL(lg_voxel_centroids, dim3(lg_wave_blocks(nmax)), dim3(CG_BLOCK), 0, s, Lh, S, f, nmax, 0);
    const uint32_t wb = lg_wave_blocks(nmax);
    const uint32_t gt = LG_DCELLS_MAX / LG_TILE + 1;
    hipLaunchKernelGGL(lg_dgrid_scan_fill, dim3(gt), dim3(CG_BLOCK), 0, s, S);
    // (the flattening in lg_forest's last workgroup instead: 19.8 against 7.1 + 5.9 us, the
    // last-arrival counting and sc1 parents costing more than the launch)
    hipLaunchKernelGGL(lg_forest, dim3(wb), dim3(CG_BLOCK), 0, s, S, P);
    hipLaunchKernelGGL(lg_flatten, dim3(1), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_cross, dim3(wb), dim3(CG_BLOCK), 0, s, S, P);
    // roots, sizes, the size filter, PCL's cluster order, labels, CSR, centroids, header: one
    // workgroup (lg_cluster_tail)
    hipLaunchKernelGGL(lg_cluster_tail, dim3(1), dim3(CG_BLOCK), 0, s, Lh, P, S, f);
    // (left out after a large frame: the fold then hands every frame to the launches above)
    return small ? cg_launch_lg_back_small(Lh, P, S, f, CG_K_FROM_META, 0u, s) : hipGetLastError();
}

// One frame through the device-sized path: front, decisions (their fold sizes the backend),
// backend. Pipeline and detect modes.
static int large_frame_dev(const CgLaunch& L, const CgDevParams& P, int kmode, LgScratch S, hipStream_t s,
                           uint32_t f, uint32_t levels, bool small) {
    const uint32_t szfl = LG_SZ_ON | (kmode == CG_KMODE_PIPELINE ? LG_SZ_PIPE : 0u) |
                          (kmode == CG_KMODE_PIPELINE && P.zero_pass ? LG_SZ_ZPAD : 0u) |
                          (S.force_global || !small ? LG_SZ_GLOBAL : 0u);
    int e;
    if ((e = cg_large_front(L, P, kmode, S, s, f, true, szfl)) != hipSuccess) return e;
    if (kmode == CG_KMODE_PIPELINE && (e = cg_large_decide(L, P, S, s, f, szfl)) != hipSuccess) return e;
    if ((e = large_backend_dev(L, P, S, s, f, L.n_points, levels, small, szfl)) != hipSuccess) return e;
    return hipGetLastError();
}

// Captured frames: one hipGraph per (launch arguments, frame), instantiated once and replayed:
// the frame's ~25 launches cost the host one graph launch instead of one call each. Captured on
// a private stream (nothing runs there); at most LG_GRAPHS entries, the least recently used one
// replaced when a new key arrives (a caller rotating input buffers keys a graph per buffer;
// graphs of freed buffers age out instead of pinning the cache).
#define LG_GRAPHS 32
struct LgGraphs {
    hipStream_t cap = nullptr;
    uint64_t clock = 0;
    struct Entry {
        std::vector<unsigned char> key;
        hipGraphExec_t exec;
        uint64_t used;
    };
    std::vector<Entry> e;
};
void cg_large_graphs_free(LgGraphs* g) {
    if (!g) return;
    for (auto& x : g->e) (void)hipGraphExecDestroy(x.exec);
    if (g->cap) (void)hipStreamDestroy(g->cap);
    delete g;
}
static std::vector<unsigned char> lg_graph_key(const CgLaunch& L, const CgDevParams& P, int kmode, const LgScratch& S,
                                               uint32_t f, uint32_t levels, bool small) {
    std::vector<unsigned char> k(sizeof(L) + sizeof(P) + sizeof(S) + 4 * sizeof(uint32_t));
    unsigned char* q = k.data();
    std::memcpy(q, &L, sizeof(L)); q += sizeof(L);
    std::memcpy(q, &P, sizeof(P)); q += sizeof(P);
    std::memcpy(q, &S, sizeof(S)); q += sizeof(S);
    const uint32_t t[4] = {(uint32_t)kmode, f, levels, small ? 1u : 0u};
    std::memcpy(q, t, sizeof(t));
    return k;
}
static int large_frame_graph(LgGraphs* g, const CgLaunch& L, const CgDevParams& P, int kmode, const LgScratch& S,
                             hipStream_t s, uint32_t f, uint32_t levels, bool small) {
    std::vector<unsigned char> key = lg_graph_key(L, P, kmode, S, f, levels, small);
    g->clock++;
    for (auto& x : g->e)
        if (x.key == key) {
            x.used = g->clock;
            return hipGraphLaunch(x.exec, s);
        }
    if (g->e.size() >= LG_GRAPHS) {   // the least recently used entry makes room
        size_t lru = 0;
        for (size_t i = 1; i < g->e.size(); i++)
            if (g->e[i].used < g->e[lru].used) lru = i;
        (void)hipDeviceSynchronize();   // (it may still be queued on some stream; eviction is rare)
        (void)hipGraphExecDestroy(g->e[lru].exec);
        g->e.erase(g->e.begin() + (long)lru);
    }
    hipError_t e;
    if (!g->cap && (e = hipStreamCreateWithFlags(&g->cap, hipStreamNonBlocking)) != hipSuccess) return e;
    if ((e = hipStreamBeginCapture(g->cap, hipStreamCaptureModeThreadLocal)) != hipSuccess) return e;
    const int rc = large_frame_dev(L, P, kmode, S, g->cap, f, levels, small);
    hipGraph_t graph = nullptr;
    e = hipStreamEndCapture(g->cap, &graph);
    if (rc != hipSuccess) {
        if (graph) (void)hipGraphDestroy(graph);
        return rc;
    }
    if (e != hipSuccess) return e;
    hipGraphExec_t exec = nullptr;
    e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
    (void)hipGraphDestroy(graph);
    if (e != hipSuccess) return e;
    g->e.push_back({std::move(key), exec, g->clock});
    return hipGraphLaunch(exec, s);
}

// ------------------------------------------------------------------------------------------
// Host driver: one frame at a time on stream s. Synchronises once per frame: the survivor
// count and bounds size the backend launches.
//
// With a second scratch set (S2, several detector frames) the frames are software-pipelined:
// frame f + 1's front and decide are enqueued before frame f's backend, on the other set, so
// the stream holds work while the host reads frame f's counts and sizes its backend. The
// stream order keeps every set's reads before its next writes (frame f + 2's front follows
// frame f's backend).
int cg_run_large(const CgLaunch& L, const CgDevParams& P, int kmode, LgScratch S, hipStream_t s, const LgScratch* S2,
                 LgGraphs** graphs, const uint32_t* hint) {
    const uint32_t N = L.n_points;
    hipError_t e;
    S.pidx_base = 0;
    if (kmode != CG_KMODE_GROUND && P.voxel_order == CG_VOXEL_ORDER_PCL && N > 0 && N <= LG_DEV_MAX_POINTS) {
        if (graphs && !*graphs) *graphs = new LgGraphs();
        // partition levels from N (levels with no range to cut return at once). Round 4 sized
        // them from the previous frame's index_vector instead (fewer launches): 575-580 against
        // 309-311 us per C5 frame, reverted (profiles/r4_c5_hint_reverted.txt)
        const uint32_t levels = lg_levels_for(N, S.pcl_levels_cap);
        bool small = true;
        if (hint && hint[LG_HINT_SMALL] == 1u) small = false;   // the last frame was a large one
        for (uint32_t f = 0; f < L.n_frames; f++) {
            const int rc = graphs ? large_frame_graph(*graphs, L, P, kmode, S, s, f, levels, small)
                                  : large_frame_dev(L, P, kmode, S, s, f, levels, small);
            if (rc != hipSuccess) return rc;
        }
        return hipSuccess;
    }
    if (S2 && L.n_frames > 1 && kmode != CG_KMODE_GROUND && S.hmeta && S2->hmeta) {
        LgScratch set[2] = {S, *S2};
        set[1].pidx_base = 0;
        hipEvent_t ev[2] = {nullptr, nullptr};
        for (int k = 0; k < 2; k++)
            if ((e = hipEventCreateWithFlags(&ev[k], hipEventDisableTiming)) != hipSuccess) return e;
        auto fetch = [&](uint32_t f) -> hipError_t {
            LgScratch& Q = set[f & 1];
            hipError_t r;
            if ((r = (hipError_t)cg_large_front(L, P, kmode, Q, s, f, true)) != hipSuccess) return r;
            if (kmode == CG_KMODE_PIPELINE && (r = (hipError_t)cg_large_decide(L, P, Q, s, f)) != hipSuccess) return r;
            if ((r = hipMemcpyAsync(Q.hmeta, Q.meta, LG_META_WORDS * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return r;
            return hipEventRecord(ev[f & 1], s);
        };
        e = fetch(0);
        for (uint32_t f = 0; f < L.n_frames && e == hipSuccess; f++) {
            if (f + 1 < L.n_frames && (e = fetch(f + 1)) != hipSuccess) break;
            if ((e = hipEventSynchronize(ev[f & 1])) != hipSuccess) break;
            uint32_t hm[LG_META_WORDS];   // frame f + 2's copy lands in this buffer after the backend below
            std::memcpy(hm, set[f & 1].hmeta, sizeof(hm));
            const uint32_t K = kmode == CG_KMODE_PIPELINE ? CG_K_FROM_META : N;
            e = (hipError_t)large_backend_from(L, P, kmode, set[f & 1], s, f, N, K, hm);
        }
        for (int k = 0; k < 2; k++) (void)hipEventDestroy(ev[k]);
        return e;
    }
    for (uint32_t f = 0; f < L.n_frames; f++) {
        if ((e = (hipError_t)cg_large_front(L, P, kmode, S, s, f, true)) != hipSuccess) return e;
        if (kmode == CG_KMODE_GROUND) continue;
        if (kmode == CG_KMODE_PIPELINE && (e = (hipError_t)cg_large_decide(L, P, S, s, f)) != hipSuccess) return e;
        const uint32_t K = kmode == CG_KMODE_PIPELINE ? CG_K_FROM_META : N;
        if ((e = (hipError_t)cg_large_backend(L, P, kmode, S, s, f, N, K)) != hipSuccess) return e;
    }
    return hipSuccess;
}

// ------------------------------------------------------------------------------------------
// Scratch layout (one frame at a time).
namespace {

uint64_t lg_pq_tmax(uint64_t n) { return (n + PQ_T - 1) / PQ_T + PQ_MAXR; }
// lg_pq_flow's tickets for index_vectors of up to n records: ranges of one depth are disjoint and
// longer than LG_PCL_CUT, so a depth holds at most n / PQ_T + n / LG_PCL_CUT + 1 tiles; the
// budget bounds the depth by 2 lg n; every tile at most twice (split, and a deferred swap)
uint64_t lg_pqf_cap(uint64_t n) {
    uint64_t lg = 0;
    while ((2ull << lg) <= n) lg++;
    return 2 * (2 * lg + 2) * (n / PQ_T + n / LG_PCL_CUT + 2) + 1024;
}
template <class F>
uint64_t lg_walk(uint32_t n, F place) {
    const uint64_t N = std::max<uint32_t>(n, 1), nch = (N + LG_CHUNK - 1) / LG_CHUNK;
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) { const uint64_t o = off; off += (bytes + 255) & ~255ull; return o; };
    place(0, take(LG_META_WORDS * 4));
    place(1, take(nch * LG_CHUNK));
    place(2, take(nch * CG_BLOCK * 2 * 8));
    place(3, take(nch * 4 + 4));
    place(6, take(N * 16)); place(7, take(N * 4));
    place(8, take(N * 8)); place(9, take(N * 8));
    place(10, take(N * 4)); place(11, take(N * 4));
    const uint64_t nrs = (N + LG_RS_TILE - 1) / LG_RS_TILE;
    place(12, take((std::max<uint64_t>(256 * nrs, LG_DCELLS_MAX / LG_TILE + 1) + 2) * 4));
    place(13, take((std::max<uint64_t>(N / CG_BLOCK + 1, LG_DCELLS_MAX / LG_TILE + 1) + 2) * 4));   // (tiles of >= 512)
    place(14, take(N * 16));
    place(15, take((N + 2) * 4));
    for (int a = 0; a < 12; a++) place(16 + a, take((N + 2) * 4));
    place(28, take((uint64_t)(LG_DCELLS_MAX + 2) * 4));
    place(29, take(nch * LG_CS_WORDS * 4));
    place(30, take((LG_PQ_HDR + 4 * PQ_EW * LG_PQ_CAP) * 4));   // PCL sort range lists
    // their look-back words: two sets (tickets, finished, one per tile) and the range counts
    place(31, take((2 * (2 + lg_pq_tmax(N)) + 2 * PQ_MAXR + 16) * 8));   // + lg_arrivals' words
    place(32, take(PQF_HDR * 8 + lg_pqf_cap(N) * 40));   // lg_pq_flow: 16 + 8 + 8 + 8 B per ticket
    place(33, take(N * 16));                               // lg_pq_flow: the lists' records
    return off;
}
}  // namespace
uint64_t cg_large_bytes(uint32_t n) { return lg_walk(n, [](int, uint64_t) {}); }
uint32_t cg_large_pq_words() { return LG_PQ_HDR + 4 * PQ_EW * LG_PQ_CAP; }
void cg_large_layout(uint8_t* base, uint32_t n, LgScratch& S) {
    uint32_t** arr[12] = {&S.par, &S.cnt, &S.lab, &S.uk, &S.ca, &S.ord, &S.droot, &S.dsz, &S.rank, &S.fin, &S.off, &S.rk};
    lg_walk(n, [&](int k, uint64_t o) {
        uint8_t* p = base + o;
        switch (k) {
            case 0: S.meta = (uint32_t*)p; break;
            case 1: S.codes = (uint64_t*)p; break;
            case 2: S.keep = (uint64_t*)p; break;
            case 3: S.chunk_cnt = (uint32_t*)p; break;
            case 6: S.surv_p = (float4*)p; break;
            case 7: S.surv_i = (uint32_t*)p; break;
            case 8: S.key0 = (uint64_t*)p; break;
            case 9: S.key1 = (uint64_t*)p; break;
            case 10: S.val0 = (uint32_t*)p; break;
            case 11: S.val1 = (uint32_t*)p; break;
            case 12: S.hist = (uint32_t*)p; break;
            case 13: S.sstat = (uint32_t*)p; break;
            case 14: S.vox = (float4*)p; break;
            case 15: S.run = (uint32_t*)p; break;
            case 28: S.cstart = (uint32_t*)p; break;
            case 29: S.cstat = (uint32_t*)p; break;
            case 30: S.pq = (uint32_t*)p; S.pq_cap = LG_PQ_CAP; break;
            case 31: S.pqst = (uint64_t*)p; S.pq_tmax = (uint32_t)lg_pq_tmax(std::max<uint32_t>(n, 1)); break;
            case 32: S.pqf = (uint64_t*)p; S.pqf_cap = (uint32_t)lg_pqf_cap(std::max<uint32_t>(n, 1)); break;
            case 33: S.pqr = (uint64_t*)p; break;

            default: *arr[k - 16] = (uint32_t*)p; break;
        }
    });
}

// ------------------------------------------------------------------------------------------
// C5 spatial tiling with a halo exchange (include/cones_gpu.h, cg_halo_*). The frame's PCL
// voxel lattice (global bounds, so idx is the whole frame's) is cut into slabs of voxel columns
// along x. A voxel lies in one slab, so each rank's voxel sums are the whole frame's (its
// survivors arrive in frame-index order); clustering runs per slab, and only the edges across
// a slab boundary need the neighbour's voxels: those within `band` columns of the boundary.
//
// Records (CG_HALO_REC_WORDS words): x, y, z, intensity (voxel centroid), idx, idx of the
// lowest voxel of the voxel's component in its slab, 0, 0.

// slab of each survivor by its voxel column (lg_voxel_keys's arithmetic); -1: non-finite
__global__ __launch_bounds__(CG_BLOCK) void lg_halo_owner(const float4* pts, uint32_t n, float inv0, int32_t min_b0,
                                                          uint32_t slab_w, uint32_t slabs, int32_t* out) {
    const uint32_t j = blockIdx.x * CG_BLOCK + threadIdx.x;
    if (j >= n) return;
    const float4 p = pts[j];
    int32_t s = -1;
    if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
        const int i0 = (int)(floorf(p.x * inv0) - (float)min_b0);
        s = (int32_t)min((uint32_t)i0 / slab_w, slabs - 1);
    }
    out[j] = s;
}
// the local backend's run ends and scan length cover the slab's points only (the lattice
// came from the whole frame's bounds)
__global__ __launch_bounds__(CG_BLOCK) void lg_halo_records(LgScratch S, int buf, uint32_t PB, uint32_t* rec,
                                                            uint32_t cap) {
    const uint32_t v = blockIdx.x * CG_BLOCK + threadIdx.x, V = S.meta[LG_V];
    if (v >= V || v >= cap) return;
    const uint64_t* vkey = buf ? S.key1 : S.key0;
    const float4 c = S.vox[v];
    const uint32_t root = S.lab[v];
    uint4* r = (uint4*)(rec + (uint64_t)v * CG_HALO_REC_WORDS);
    r[0] = make_uint4(__float_as_uint(c.x), __float_as_uint(c.y), __float_as_uint(c.z), __float_as_uint(c.w));
    r[1] = make_uint4((uint32_t)(vkey[S.run[v]] >> PB), (uint32_t)(vkey[S.run[root]] >> PB), 0u, 0u);
}

int cg_halo_local_run(const CgLaunch& L, const CgDevParams& P, LgScratch S, hipStream_t s, const float* d_points,
                      const uint32_t* d_index, uint32_t n, uint32_t npad_local, uint32_t npad_all,
                      const uint32_t* counts, uint32_t N, uint32_t key_bits, uint32_t* d_rec, uint32_t cap,
                      uint32_t* n_vox) {
    hipError_t e;
    uint32_t c[CG_TILE_COUNTS];
    for (int a = 0; a < CG_TILE_COUNTS; a++) c[a] = counts[a];
    c[1] = n;   // the slab's survivors; nfin and bounds stay the whole frame's (the lattice)
    int rc = cg_large_set_survivors(S, P, d_points, d_index, n, c, s);
    if (rc) return rc;
    uint32_t hstack[LG_META_WORDS];
    uint32_t* const hm = S.hmeta ? S.hmeta : hstack;
    if ((e = hipMemcpyAsync(hm, S.meta, LG_META_WORDS * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = cg_stream_wait(s)) != hipSuccess) return e;
    const uint32_t Mtot = n + npad_local;
    *n_vox = 0;
    if (Mtot == 0) return hipSuccess;
    const uint32_t PB = hm[LG_UNSORTED] ? bits_of((uint64_t)N + npad_all) : 0u;
    key_bits = std::min<uint32_t>(key_bits + PB, 32 + PB);
    const uint32_t mb = std::max<uint32_t>(1, blocks_of(Mtot));
    hipLaunchKernelGGL(lg_voxel_keys, dim3(mb), dim3(CG_BLOCK), 0, s, S, P, Mtot, N, PB, npad_all, Mtot);
    const int buf = radix_sort(S, Mtot, key_bits, s);
    const uint64_t* vkey = buf ? S.key1 : S.key0;
    scan_emit(S, Mtot, LG_SCAN_N, VoxelHead{vkey, S.meta, PB}, VoxelEmit{S.run}, LG_V, s);
    hipLaunchKernelGGL(lg_voxel_centroids, dim3(lg_wave_blocks(Mtot)), dim3(CG_BLOCK), 0, s,
                       L, S, 0u, Mtot, buf);
    const uint32_t vb = std::max<uint32_t>(1, blocks_of(Mtot)), wb = lg_wave_blocks(Mtot);
    const uint32_t gt = LG_DCELLS_MAX / LG_TILE + 1;
    hipLaunchKernelGGL(lg_dgrid_scan, dim3(gt), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_dgrid_fill, dim3(vb), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_forest, dim3(wb), dim3(CG_BLOCK), 0, s, S, P);
    hipLaunchKernelGGL(lg_flatten, dim3(1), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_cross, dim3(wb), dim3(CG_BLOCK), 0, s, S, P);
    hipLaunchKernelGGL(lg_find, dim3(vb), dim3(CG_BLOCK), 0, s, S);
    hipLaunchKernelGGL(lg_halo_records, dim3(vb), dim3(CG_BLOCK), 0, s, S, buf, PB, d_rec, cap);
    if ((e = hipMemcpyAsync(hm, S.meta, LG_META_WORDS * 4, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    if ((e = cg_stream_wait(s)) != hipSuccess) return e;
    *n_vox = hm[LG_V];
    return hipGetLastError();
}

// Cross-slab edges: one wave per halo record, the lanes test 64 own records at a time with the
// clustering predicate; every distinct own component a halo voxel touches gives one pair
// (own component key, halo component key). The count is exact; pairs past cap are dropped.
#define LG_HALO_SEEN 8
__global__ __launch_bounds__(CG_BLOCK) void lg_halo_edges(const uint32_t* own, uint32_t n_own, const uint32_t* halo,
                                                          uint32_t n_halo, float r2, uint32_t* pairs, uint32_t cap,
                                                          uint32_t* count) {
    const uint32_t t = blockIdx.x * WAVES + wave_id(), l = lane_id();
    if (t >= n_halo) return;
    const uint4* hr = (const uint4*)(halo + (uint64_t)t * CG_HALO_REC_WORDS);
    const uint4 h0 = hr[0], h1 = hr[1];
    const float4 q = make_float4(__uint_as_float(h0.x), __uint_as_float(h0.y), __uint_as_float(h0.z), 0.f);
    uint32_t seen[LG_HALO_SEEN];
    uint32_t nseen = 0;
    for (uint32_t g0 = 0; g0 < n_own; g0 += 64) {
        const uint32_t j = g0 + l;
        bool adj = false;
        uint32_t root = 0;
        if (j < n_own) {
            const uint4* orr = (const uint4*)(own + (uint64_t)j * CG_HALO_REC_WORDS);
            const uint4 o0 = orr[0];
            const float4 p = make_float4(__uint_as_float(o0.x), __uint_as_float(o0.y), __uint_as_float(o0.z), 0.f);
            adj = lg_adjacent(p, q, r2);
            if (adj) root = orr[1].y;
        }
        for (uint32_t k = 0; k < nseen; k++) adj = adj && root != seen[k];
        uint64_t m = __ballot(adj);
        while (m) {
            const uint32_t key = __builtin_amdgcn_readlane(root, (int)__builtin_ctzll(m));
            if (l == 0) {
                const uint32_t at = atomicAdd(count, 1u);
                if (at < cap) { pairs[2 * at] = key; pairs[2 * at + 1] = h1.y; }
            }
            if (nseen < LG_HALO_SEEN) seen[nseen++] = key;
            adj = adj && root != key;
            m = __ballot(adj);
        }
    }
}
int cg_halo_edges_run(const uint32_t* own, uint32_t n_own, const uint32_t* halo, uint32_t n_halo, float r2,
                      uint32_t* pairs, uint32_t cap, uint32_t* d_count, hipStream_t s) {
    if (hipMemsetAsync(d_count, 0, 4, s) != hipSuccess) return hipGetLastError();
    if (n_halo && n_own)
        hipLaunchKernelGGL(lg_halo_edges, dim3((n_halo + WAVES - 1) / WAVES), dim3(CG_BLOCK), 0, s, own, n_own, halo,
                           n_halo, r2, pairs, cap, d_count);
    return hipGetLastError();
}

// Merge on one rank: the records of every slab sorted by idx (the global voxel order), the
// slab components as a forest (every voxel under its component's lowest voxel), the pairs
// united; then the backend's tail (size filter, PCL's cluster order, CSR, centroids).
__global__ void lg_halo_meta(LgScratch S, uint32_t V) {
    if (threadIdx.x != 0) return;
    S.meta[LG_V] = V;
    S.meta[LG_PASS] = 0;
}
__global__ __launch_bounds__(CG_BLOCK) void lg_halo_keys(LgScratch S, const uint32_t* rec, uint32_t V) {
    const uint32_t j = blockIdx.x * CG_BLOCK + threadIdx.x;
    if (j >= V) return;
    S.key0[j] = rec[(uint64_t)j * CG_HALO_REC_WORDS + 4];
    S.val0[j] = j;
}
__global__ __launch_bounds__(CG_BLOCK) void lg_halo_place(CgLaunch L, LgScratch S, const uint32_t* rec, uint32_t V,
                                                          int buf) {
    const uint32_t v = blockIdx.x * CG_BLOCK + threadIdx.x;
    if (v >= V) return;
    const uint32_t j = (buf ? S.val1 : S.val0)[v];
    const uint4 r0 = ((const uint4*)(rec + (uint64_t)j * CG_HALO_REC_WORDS))[0];
    const float4 c = make_float4(__uint_as_float(r0.x), __uint_as_float(r0.y), __uint_as_float(r0.z),
                                 __uint_as_float(r0.w));
    S.vox[v] = c;
    L.vox[v] = c;
    S.uk[v] = (uint32_t)(buf ? S.key1 : S.key0)[v];
    S.cnt[v] = 0;
    S.rk[v] = 0xffffffffu;
}
__device__ __forceinline__ uint32_t lg_halo_find_key(const uint32_t* uk, uint32_t V, uint32_t key) {
    uint32_t lo = 0, hi = V;   // first position with uk >= key (keys are unique and present)
    while (lo < hi) {
        const uint32_t mid = (lo + hi) >> 1;
        if (uk[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo < V ? lo : V - 1;
}
__global__ __launch_bounds__(CG_BLOCK) void lg_halo_forest(LgScratch S, const uint32_t* rec, uint32_t V, int buf) {
    const uint32_t v = blockIdx.x * CG_BLOCK + threadIdx.x;
    if (v >= V) return;
    const uint32_t j = (buf ? S.val1 : S.val0)[v];
    S.par[v] = lg_halo_find_key(S.uk, V, rec[(uint64_t)j * CG_HALO_REC_WORDS + 5]);
}
__global__ __launch_bounds__(CG_BLOCK) void lg_halo_unite(LgScratch S, const uint32_t* pairs, uint32_t np, uint32_t V) {
    const uint32_t i = blockIdx.x * CG_BLOCK + threadIdx.x;
    if (i >= np) return;
    uf_union(S.par, lg_halo_find_key(S.uk, V, pairs[2 * i]), lg_halo_find_key(S.uk, V, pairs[2 * i + 1]));
}

int cg_halo_merge_run(const CgLaunch& L, const CgDevParams& P, LgScratch S, hipStream_t s, const uint32_t* d_rec,
                      uint32_t V, const uint32_t* d_pairs, uint32_t np, uint32_t key_bits, uint32_t Mtot,
                      uint32_t K) {
    hipLaunchKernelGGL(lg_init, dim3(1), dim3(64), 0, s, S, P);
    hipLaunchKernelGGL(lg_halo_meta, dim3(1), dim3(64), 0, s, S, V);
    const uint32_t n = std::max<uint32_t>(V, 1);
    const uint32_t vb = blocks_of(n), wb = lg_wave_blocks(n);
    int buf = 0;
    if (V) {
        hipLaunchKernelGGL(lg_halo_keys, dim3(vb), dim3(CG_BLOCK), 0, s, S, d_rec, V);
        buf = radix_sort(S, V, key_bits, s);
        hipLaunchKernelGGL(lg_halo_place, dim3(vb), dim3(CG_BLOCK), 0, s, L, S, d_rec, V, buf);
        hipLaunchKernelGGL(lg_halo_forest, dim3(vb), dim3(CG_BLOCK), 0, s, S, d_rec, V, buf);
        if (np) hipLaunchKernelGGL(lg_halo_unite, dim3(blocks_of(np)), dim3(CG_BLOCK), 0, s, S, d_pairs, np, V);
        hipLaunchKernelGGL(lg_find, dim3(vb), dim3(CG_BLOCK), 0, s, S);
    }
    scan_emit(S, n, LG_V, KeepRoot{S.lab, S.cnt, P.min_cl, P.max_cl}, KeepEmit{S.cnt, S.droot, S.dsz}, LG_C, s);
    hipLaunchKernelGGL(lg_order, dim3(1), dim3(CG_BLOCK), 0, s, S);
    const uint32_t VB = bits_of(n);
    hipLaunchKernelGGL(lg_labels, dim3(vb), dim3(CG_BLOCK), 0, s, L, S, 0u, VB);
    const uint32_t cmax = P.min_cl > 1 ? n / P.min_cl : n;
    const int kb = radix_sort(S, n, VB + bits_of(std::max<uint32_t>(cmax, 1)) + 1, s, VB, S.meta + LG_V,
                               S.meta + LG_SORT_LIM);
    const uint32_t cb = blocks_of((uint64_t)n + 1);
    CgDevParams Pm = P;
    Pm.voxel_order = CG_VOXEL_ORDER_POINT;   // each slab summed its voxels in frame-index order
    hipLaunchKernelGGL(lg_csr_centroids, dim3(cb + wb), dim3(CG_BLOCK), 0, s, L, Pm, S, 0u, VB, kb, Mtot, K, cb, 0u);
    return hipGetLastError();
}
int cg_launch_halo_owner(const float* pts, uint32_t n, float inv0, int32_t min_b0, uint32_t slab_w, uint32_t slabs,
                         int32_t* out, hipStream_t s) {
    if (n) hipLaunchKernelGGL(lg_halo_owner, dim3(blocks_of(n)), dim3(CG_BLOCK), 0, s, (const float4*)pts, n, inv0,
                              min_b0, slab_w, slabs, out);
    return hipGetLastError();
}
