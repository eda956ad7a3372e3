// cg_pcl.h — PCL VoxelGrid's voxel order on the device (frame kernel, large-frame path).
#pragma once
#include <hip/hip_runtime.h>
#include "cg_internal.h"
#include "cg_sort.h"
#include "cg_device.h"

// The backend's working arrays (LDS for M <= CG_MMAX, else HBM scratch), one slot per point.
struct Work {
    float4* P; uint64_t* KEY; float4* VOX; uint32_t* A; uint32_t* PAR; uint32_t* CNT;
    uint32_t* UK; int32_t* LAB; uint32_t* ORD; uint32_t* IDX; uint32_t* OFF;
};

// ------------------------------------------------------------------------------------------
// PCL's voxel order. VoxelGrid::applyFilter (PCL 1.10, src/cone_detection.cpp:240-249) builds
// index_vector = (idx, cloud_point_index) over the finite points of the filtered cloud in
// cloud order and sorts it with std::sort(less on idx): an unstable introsort, so the order
// of equal idx -- the order each voxel's float sums run in -- is libstdc++'s permutation.
// It is reproduced exactly:
//  1. index_vector order: the rank of a kept survivor among the finite kept survivors by point
//     index (a bitmap of point indices, popcount prefix), then the zero pads;
//  2. __introsort_loop level-synchronously: per range, the
//     median of three moved to first, then the unguarded Hoare partition in parallel. Its
//     k-th swap exchanges the k-th element >= pivot from the left (L_k) with the k-th element
//     <= pivot from the right (R_k) while L_k < R_k; both lists are read off prefix counts of
//     the original range, because the scans pass only unswapped positions until they cross.
//     With s swaps the cut (where the left scan stops next) is L_0 if s = 0, else
//     min(L_s, R_{s-1}). Depth budget and heapsort fallback per range as in the sequential
//     code (cg_sort.h);
//  3. up to PMAX * CG_BLOCK elements (pcl_block_sort) each thread keeps its elements' ranges in
//     registers; the workgroup levels stop at ranges of at most 64, which one wave each
//     finishes in registers (pw_range64); longer arrays (HBM scratch) run block levels until
//     every range fits, then pcl_block_sort on each range. The large path (cg_large.hip) runs
//     the first levels across workgroups and hands the leaves to pcl_block_sort in LDS;
//  4. the final insertion passes: a stable sort inside each range of at most 16 (the ranges
//     are weakly ordered, so this is the stable sort of the whole array).
// The permutation is checked against std::sort on the host (tests/test_math_host.py and the
// thread-level model tests/pb_model.py), on the device directly against libstdc++
// (tools/pcl_probe.hip, tools/pcl_leaf_probe.hip: tests/test_gpu_pcl_probe.py) and against the
// oracle's ORDER_PCL (tests/test_gpu_pcl_order.py).
#ifdef CG_PCL_PROBE
__device__ unsigned long long g_pcl_probe[64];
__device__ unsigned int g_pcl_probe_n;
// workgroup 0 only (other workgroups of a probe launch share the counter), bounded slot
#define PCL_STAMP()                                                                      \
    do {                                                                                 \
        if (threadIdx.x == 0 && blockIdx.x == 0) {                                      \
            const unsigned int s_ = atomicAdd(&g_pcl_probe_n, 1u);                       \
            if (s_ < 64) g_pcl_probe[s_] = __builtin_amdgcn_s_memrealtime();             \
        }                                                                                \
    } while (0)
#ifdef CG_PCL_PROBE_NOSTEP   // (the whole sort's time only)
#define PCL_STEP() ((void)0)
#else
#define PCL_STEP() PCL_STAMP()
#endif
#else
#define PCL_STAMP() ((void)0)
#define PCL_STEP() ((void)0)
#endif
#define PCL_INACT 0xffffffffu
#define PCL_HEAD 1u
#define PCL_HEAP 2u
__device__ __forceinline__ uint32_t pcl_key(uint64_t r) { return (uint32_t)(r >> 32); }

// Records (idx << 32 | slot) of the Mf finite points of W.P in index_vector order -> E.
// Kept survivors are slots [0, Ms) with W.IDX[slot] < 32 * nbw (point indices of a 64k frame:
// nbw = 2048; ranks in point order: fewer); zero pads are slots [Ms, M). Uses W.VOX (bitmap,
// word prefix: 2 * nbw words; then E) and W.ORD. Ends with a barrier.
template <class KF>
__device__ __forceinline__ void pcl_index_vector(const Work& W, uint32_t M, uint32_t Ms, uint64_t* E,
                                                 uint32_t* red, uint32_t nbw, KF voxel_idx) {
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    uint32_t* BM = (uint32_t*)W.VOX;       // nbw words: one bit per point index (or rank)
    uint32_t* WP = BM + nbw;               // exclusive popcount prefix per word
    for (uint32_t i = tid; i < nbw; i += CG_BLOCK) BM[i] = 0u;
    __syncthreads();
    for (uint32_t j = tid; j < Ms; j += CG_BLOCK) {
        const float4 p = W.P[j];
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            const uint32_t q = W.IDX[j];
            atomicOr(&BM[q >> 5], 1u << (q & 31u));
        }
    }
    __syncthreads();
    const uint32_t per = (nbw + CG_BLOCK - 1) / CG_BLOCK;   // consecutive words per lane
    uint32_t sum = 0;
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t i = tid * per + k;
        sum += i < nbw ? (uint32_t)__popc(BM[i]) : 0u;
    }
    const uint32_t inc = wave_incl_scan(sum);
    if (l == 63) red[w] = inc;
    __syncthreads();
    uint32_t base = inc - sum;
    for (uint32_t v = 0; v < w; v++) base += red[v];
    for (uint32_t k = 0; k < per; k++) {
        const uint32_t i = tid * per + k;
        if (i < nbw) { WP[i] = base; base += (uint32_t)__popc(BM[i]); }
    }
    __syncthreads();
    uint32_t total = 0;
    for (uint32_t v = 0; v < WAVES; v++) total += red[v];   // finite kept survivors
    for (uint32_t j = tid; j < M; j += CG_BLOCK) {
        uint32_t r = PCL_INACT;
        if (j < Ms) {
            const float4 p = W.P[j];
            if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
                const uint32_t q = W.IDX[j];
                r = WP[q >> 5] + __popc(BM[q >> 5] & ((1u << (q & 31u)) - 1u));
            }
        } else {
            r = total + (j - Ms);   // pads follow the kept points (and are finite)
        }
        W.ORD[j] = r;
    }
    __syncthreads();
    for (uint32_t j = tid; j < M; j += CG_BLOCK) {
        const uint32_t r = W.ORD[j];
        if (r != PCL_INACT) E[r] = ((uint64_t)voxel_idx(j) << 32) | j;
    }
    __syncthreads();
}

// ------------------------------------------------------------------------------------------
// The whole workgroup sorts n <= CG_BLOCK * PER elements, every partition of a level of
// __introsort_loop at once. Element x = tid + CG_BLOCK * k (k < PER); each thread keeps the
// range [f, e) of its elements and the range's depth budget in registers and follows the cut
// after every level. Per level (a barrier after each step):
//   S1. every element of a range to partition (longer than WMAX, budget left) reads the range's
//       median of three itself (__move_median_to_first's swap stays virtual: position m holds
//       E[f]'s record, position f the median's) and compares with the pivot; per (chunk, wave)
//       counts; the barrier's OR ends the levels when no range is left to partition;
//   S2. the counts scanned: every position's inclusive >= / <= counts over the whole array
//       (RLO); the >= elements listed at their exclusive count in PL, the <= ones in PR, so
//       a range's L list is the stretch of PL from RLO[f] and its R list the stretch of PR
//       below RLO[e - 1], read from the right;
//   S4. the swaps (L_k, R_k) while L_k < R_k: every partner is read, then every element
//       written (or the records go out of place to E2) with V of its partner; the range's
//       cutter stores the cut: the element holding the last swap's L (min(L_s, R_{s-1})), or
//       L_0 when there is no swap;
//   S0. every element follows the cut into its child range, budget - 1.
// Then a range longer than 16 with its budget spent is heapsorted by its first element's
// thread (__partial_sort); the ranges of 17-WMAX records go one wave each (pw_range64, or a
// deferring functor); the rest get the final insertion passes: a stable rank inside each range
// of at most 16. A (wave, k) slot whose elements are all in final ranges skips every step of
// the later levels. Scratch: RLO, PL, PR, CUT, n + 1 words each; cnt: 8 * PER words. E is
// permuted in place. (Round 4's form set each range up in a fourth step by its first element's
// thread; the three-step form takes 8.4-8.8 against 9.4-9.6 us for C3's 243 records,
// profiles/r5_pb3_ab.txt.)
#define PW_MAX 64
typedef __attribute__((address_space(3))) uint32_t lds_u32;
typedef __attribute__((address_space(3))) uint64_t lds_u64;
// Pointer kinds: LDS (ds_* instructions) when the arrays live in LDS, generic otherwise.
struct PbLds { typedef lds_u32* P32; typedef lds_u64* P64; static constexpr bool in_lds = true; };
struct PbGen { typedef uint32_t* P32; typedef uint64_t* P64; static constexpr bool in_lds = false; };
template <class K> struct PbScratch { typename K::P32 RLO, PL, PR, CUT; };
struct PwLess {   // a functor, not a function: a function pointer could become an indirect call
    __device__ __forceinline__ bool operator()(uint64_t a, uint64_t b) const { return pcl_key(a) < pcl_key(b); }
};

// __move_median_to_first(first, first + 1, mid, last - 1) of a range longer than 16: the
// index of the median, decided exactly as libstdc++ does on keys ka, kb, kc at a, b, c.
__device__ __forceinline__ uint32_t pb_median(uint32_t a, uint32_t b, uint32_t c, uint32_t ka, uint32_t kb, uint32_t kc) {
    if (ka < kb) return kb < kc ? b : (ka < kc ? c : a);
    if (ka < kc) return a;
    return kb < kc ? c : b;
}

// Always inlined: an out-of-line call takes its arguments through scratch memory (and
// tests/test_isa.py asserts that no kernel makes a call).
// The sorted records go through out(position, record): an array store, or straight to the
// caller's global outputs (lg_pcl_leaf).
template <class P> struct PbStore {
    P a;
    __device__ __forceinline__ void operator()(uint32_t i, uint64_t r) const { a[i] = r; }
};
// ------------------------------------------------------------------------------------------
// One wave finishes a range of m <= 64 records (__introsort_loop with the budget left on its
// path, then __final_insertion_sort) in registers: lane i holds record f + i, and every lane
// knows its sub-range [hd, en) and that sub-range's budget. All sub-ranges longer than 16
// partition in the same round (segmented): median of three by ds_bpermute (the swap with the
// first virtual), >= / <= ballots, the swap count s = one ballot of the <= lanes with more
// >= lanes than their reverse rank before them (L_r < R_r), L_k = the k-th set bit of the
// sub-range's >= mask and R_k the (nR-1-k)-th of its <= mask (read from lane-index tables
// that one ds_permute per mask builds), the records moved once by ds_bpermute, the cut from s. A spent budget heapsorts its sub-range in the caller's buffer (rare). The final
// insertion passes are a stable rank inside each sub-range of at most 16 records (sub-ranges
// are weakly ordered, so insertion never crosses one).
__device__ __forceinline__ uint32_t pw_b32(uint32_t src, uint32_t x) {   // x of lane src
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)x);
}
__device__ __forceinline__ uint64_t pw_low(uint32_t b) {   // bits below b (b <= 64)
    return b >= 64u ? ~0ull : (1ull << b) - 1ull;
}
template <class P64, class OUT>
__device__ __forceinline__ void pw_range64(P64 E, uint32_t f, uint32_t m, uint32_t depth, OUT out) {
    const uint32_t l = lane_id();
    const bool live = l < m;
    uint64_t v = live ? (uint64_t)E[f + (live ? l : 0u)] : ~0ull;
    uint32_t hd = live ? 0u : l, en = live ? m : l + 1u, dep = depth;
    for (;;) {
        const bool act = live && en - hd > CG_SORT_THRESHOLD && dep > 0;
        if (!__ballot(act)) break;
        // __move_median_to_first(hd, hd + 1, mid, en - 1)
        const uint32_t a = hd + 1, b = hd + (en - hd) / 2, c = en - 1;
        const uint32_t key = (uint32_t)(v >> 32);
        const uint32_t ka = pw_b32(a, key), kb = pw_b32(b, key), kc = pw_b32(c, key), kh = pw_b32(hd, key);
        const uint32_t mi = pb_median(a, b, c, ka, kb, kc);
        const uint32_t p = mi == a ? ka : (mi == b ? kb : kc);
        // __move_median_to_first, virtually: position mi holds the first's record (key kh),
        // position hd the median's; the records move once, with the partition's swaps
        const uint32_t k = act && l == mi ? kh : key;
        // __unguarded_partition(hd + 1, en, hd), in parallel over the sub-ranges
        const bool in = act && l > hd;
        const uint64_t GE = __ballot(in && k >= p), LE = __ballot(in && k <= p);
        const uint64_t lo = pw_low(hd + 1), hi = pw_low(en);
        const uint32_t bG = (uint32_t)__popcll(GE & lo), bL = (uint32_t)__popcll(LE & lo);
        const uint32_t nL = (uint32_t)__popcll(GE & hi) - bG, nR = (uint32_t)__popcll(LE & hi) - bL;
        const bool isG = (GE >> l) & 1ull, isL = (LE >> l) & 1ull;
        const uint32_t gk = mbcnt(GE) - bG, rk = nR - 1u - (mbcnt(LE) - bL);
        // lane tables: PG[j] = the j-th set bit of GE (j < popc(GE)), PL likewise
        const uint32_t tG = (uint32_t)__popcll(GE), tL = (uint32_t)__popcll(LE);
        const uint32_t PG = (uint32_t)__builtin_amdgcn_ds_permute(
            (int)((isG ? mbcnt(GE) : tG + mbcnt(~GE)) << 2), (int)l);
        const uint32_t PL = (uint32_t)__builtin_amdgcn_ds_permute(
            (int)((isL ? mbcnt(LE) : tL + mbcnt(~LE)) << 2), (int)l);
        // R_r (a <= lane, reverse rank r) is swapped iff L_r < R_r, i.e. iff more than r >=
        // lanes precede it in the sub-range: the swap count s is one ballot, no lane lookup
        const uint64_t SW = __ballot(isL && mbcnt(GE) - bG > rk);
        const uint32_t s = (uint32_t)__popcll(SW & hi) - (uint32_t)__popcll(SW & lo);
        const uint32_t Rk = pw_b32(isG && gk < s ? bL + nR - 1u - gk : 0u, PL);
        const uint32_t Lk = pw_b32(isL && rk < s ? bG + rk : 0u, PG);
        uint32_t partner = l;
        if (isG && gk < s) partner = Rk;
        if (isL && rk < s) partner = Lk;
        // the virtual records: position mi holds v[hd], position hd holds v[mi]
        uint32_t src = partner;
        if (act) src = partner == mi ? hd : (partner == hd ? mi : partner);
        v = ((uint64_t)pw_b32(src, (uint32_t)(v >> 32)) << 32) | pw_b32(src, (uint32_t)v);
        const uint32_t gc = pw_b32(bG + (s < nL ? s : 0u), PG);
        const uint32_t lc = pw_b32(bL + nR - (s ? s : nR), PL);
        const uint32_t cut = s == 0 ? gc : min(s < nL ? gc : 64u, lc);
        if (act) {
            if (l >= cut) hd = cut; else en = cut;
            dep -= 1u;
        }
    }
    // spent budgets: __partial_sort(first, last, last) of the sub-range, in the caller's buffer
    const bool heap = live && en - hd > CG_SORT_THRESHOLD;
    if (__ballot(heap)) {
        if (live) E[f + l] = v;
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");   // E may be in HBM (rare path)
        if (heap && l == hd) cg_heap_sort_range((uint64_t*)(E + f + hd), (long)(en - hd), PwLess{});
        __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "agent");
        if (live) v = E[f + l];
    }
    // the final insertion passes: a stable rank inside each sub-range of at most 16
    const uint32_t kx = (uint32_t)(v >> 32);
    uint32_t rank = 0;
#pragma unroll
    for (uint32_t j = 0; j < CG_SORT_THRESHOLD; j++) {
        const uint32_t kj = pw_b32(hd + j, kx);
        rank += hd + j < en && ((kj < kx) || (kj == kx && hd + j < l));
    }
    if (heap) rank = l - hd;   // already sorted
    if (live) out(f + hd + rank, v);
}

// The ranges of 17-WMAX records: by the workgroup's own waves (PwInline, WMAX = 64), or
// handed to another launch (a functor of the same shape: the large path, PqDefer).
struct PwInline {
    template <class P64, class OUT>
    __device__ __forceinline__ void operator()(P64 E, uint32_t f, uint32_t m, uint32_t d, OUT out) const {
        pw_range64(E, f, m, d, out);
    }
};

// OOP: a second record buffer E2 (n records) takes the swapped records, so a level's swap
// step reads and writes in one barrier interval (E and E2 trade places every level); without
// it the records are swapped in place (reads, barrier, writes). cnt: PER * WAVES words (the
// per-slot counts). S.RLO holds n + 1 words.
// WMAX: ranges of at most WMAX records (with budget left) leave the levels as tasks for wt;
// PwInline takes at most PW_MAX.
// Three barrier-separated steps per level. Each thread keeps, for each of its elements, the
// element's range [f, e) and the range's depth budget in registers, so a range's set-up needs
// no heads step: in S1 every element of a range longer than WMAX (budget left) reads the
// range's median of three itself (__move_median_to_first's swap stays virtual: position m
// holds E[f]'s record, position f the median's), in S4 the swaps write V(partner) and the
// range's cutter -- the element holding the last swap's L (cut = min(L_s, R_{s-1})), or L_0
// when there is no swap (cut = L_0) -- stores the cut, and S0 follows it. (tests/pb_model.py
// block_sort models it thread by thread against std::sort.)
template <int PER, class K, class OUT = PbStore<typename K::P64>, bool OOP = false, class WT = PwInline,
          uint32_t WMAX = PW_MAX>
__device__ __forceinline__ void pcl_block_sort(typename K::P64 E, OUT out, uint32_t n, uint32_t depth0,
                                               const PbScratch<K> S, typename K::P32 cnt,
                                               typename K::P64 E2 = nullptr, WT wt = WT{}) {
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    constexpr uint32_t GE = 1u << 24, LE = 1u << 25, IN = 1u << 26, PART = 1u << 27;
    constexpr uint32_t NS = PER * WAVES;   // (chunk, wave) slots: position x is in slot x / 64
    uint32_t fe[PER], dp[PER];
#pragma unroll
    for (int k = 0; k < PER; k++) { fe[k] = n << 16; dp[k] = depth0; }
    // (wave, k) slots with an element in a partitioned range; a slot without one has nothing
    // to do in any later level (ranges only shrink, and a final range stays final)
    uint32_t live = (1u << PER) - 1u;
    const uint32_t top = n ? n - 1 : 0u;
    for (;;) {
        uint32_t st[PER], mm[PER];
        bool mine = false;
        // S1: the range's median of three and pivot, >= / <= against it; per-slot counts
#pragma unroll
        for (int k = 0; k < PER; k++) {
            mm[k] = 0u;
            if (!((live >> k) & 1u)) {
                if (l == 0) cnt[k * WAVES + w] = 0u;
                st[k] = 0u;
                continue;
            }
            const uint32_t x = tid + CG_BLOCK * k, f = fe[k] & 0xffffu, e = fe[k] >> 16;
            const bool part = x < n && e - f > CG_SORT_THRESHOLD && e - f > WMAX && dp[k] > 0;
            // the five keys in one batch (indices clamped: no branch between the loads)
            const uint32_t a = f + 1, b = f + (e - f) / 2, c = e - 1;
            const uint32_t ka = pcl_key(E[part ? a : 0u]), kb = pcl_key(E[part ? b : 0u]), kc = pcl_key(E[part ? c : 0u]);
            const uint32_t kf = pcl_key(E[part ? f : 0u]), kx0 = pcl_key(E[min(x, top)]);
            const uint32_t m = pb_median(a, b, c, ka, kb, kc);
            const uint32_t p = m == a ? ka : (m == b ? kb : kc);
            const uint32_t kx = x == m ? kf : kx0;
            const bool in = part && x > f;
            const bool ge = in && kx >= p, le = in && kx <= p;
            const uint64_t gm = __ballot(ge), lm = __ballot(le);
            if (l == 0) cnt[k * WAVES + w] = (uint32_t)__popcll(gm) | ((uint32_t)__popcll(lm) << 16);
            st[k] = mbcnt(gm) | (mbcnt(lm) << 12) | (ge ? GE : 0u) | (le ? LE : 0u) | (in ? IN : 0u) | (part ? PART : 0u);
            mm[k] = m;
            mine |= part;
            if (!__ballot(part)) live &= ~(1u << k);
        }
        if (!__syncthreads_or(mine)) break;   // (uniform) no range left to partition
        PCL_STEP();
        // S2: lane j of every wave scans the slot counts; every position's >= / <= counts over
        // the whole array, inclusive, go to RLO, and the >= elements are listed in position
        // order at their exclusive >= count in PL, the <= elements at theirs in PR: a range's
        // L list is then a contiguous stretch of PL from RLO[f] (the first position counts for
        // nothing), its R list the stretch of PR below RLO[e - 1], read from the right.
        {
            // both counts in one scan of the packed word (totals <= n <= 4,096: no carry
            // between the halves)
            const uint32_t cj = l < NS ? cnt[l] : 0u;
            const uint32_t ex = wave_incl_scan(cj) - cj;
            const uint32_t gex = ex & 0xffffu, hex = ex >> 16;
#pragma unroll
            for (int k = 0; k < PER; k++) {
                if (!((live >> k) & 1u)) continue;
                const uint32_t x = tid + CG_BLOCK * k;
                const uint32_t src = (uint32_t)k * WAVES + w;
                const uint32_t gx = (uint32_t)__builtin_amdgcn_readlane((int)gex, (int)src) + (st[k] & 0xfffu);
                const uint32_t lx = (uint32_t)__builtin_amdgcn_readlane((int)hex, (int)src) + ((st[k] >> 12) & 0xfffu);
                if (x < n) S.RLO[x] = (gx + ((st[k] & GE) ? 1u : 0u)) | ((lx + ((st[k] & LE) ? 1u : 0u)) << 16);
                if (st[k] & GE) S.PL[gx] = x;
                if (st[k] & LE) S.PR[lx] = x;
                st[k] = (gx & 0xfffu) | ((lx & 0xfffu) << 12) | (st[k] & (GE | LE | IN | PART));
            }
        }
        __syncthreads();
        PCL_STEP();
        // S4: the range's list bounds, the partners and the next pair in one batch, then V of
        // the partner; the cutter stores the cut
        uint64_t val[PER];
        uint32_t sw = 0;
        uint32_t bf[PER], be[PER];
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const uint32_t f = fe[k] & 0xffffu, e = fe[k] >> 16;
            const bool part = (st[k] & PART) != 0;
            bf[k] = part ? S.RLO[f] : 0u;
            be[k] = part ? S.RLO[e - 1] : 0u;
        }
#pragma unroll
        for (int k = 0; k < PER; k++) {
            if (!OOP && !((live >> k) & 1u)) continue;   // out of place, every record moves
            const uint32_t x = tid + CG_BLOCK * k, f = fe[k] & 0xffffu;
            const bool in = (st[k] & IN) != 0, part = (st[k] & PART) != 0;
            const uint32_t gf = bf[k] & 0xffffu, lend = be[k] >> 16;
            const uint32_t nL = (be[k] & 0xffffu) - gf, nR = lend - (bf[k] >> 16);
            const uint32_t li = in ? (st[k] & 0xfffu) - gf : 0u, ri = in ? lend - 1u - ((st[k] >> 12) & 0xfffu) : 0u;
            const bool hasL = in && (st[k] & GE) && li < nR, hasR = in && (st[k] & LE) && ri < nL;
            const bool nxt = hasL && li + 1 < min(nL, nR);
            const uint32_t j = S.PR[hasL ? lend - 1u - li : 0u];                     // R_li
            const uint32_t i = S.PL[hasR ? gf + ri : 0u];                             // L_ri
            const uint32_t pl2 = S.PL[min(hasL && li + 1 < nL ? gf + li + 1u : 0u, top)];   // L_li+1
            const uint32_t pr2 = S.PR[nxt ? lend - 2u - li : 0u];                    // R_li+1
            uint32_t partner = x;
            if (hasL) {
                if (x < j) {
                    partner = j;
                    if (!nxt || !(pl2 < pr2)) S.CUT[f] = min(li + 1 < nL ? pl2 : 0xffffffffu, j);   // the last swap
                } else if (li == 0) {
                    S.CUT[f] = x;   // no swap: the left scan stops at L_0
                }
            }
            if (hasR && i < x) partner = i;
            if (x < n) {
                // V(partner): position m holds E[f]'s record, position f the median's
                uint32_t src = partner;
                if (part) src = x == f ? mm[k] : (partner == mm[k] ? f : partner);
                if (OOP) {
                    val[k] = E[src];
                } else if (src != x) {
                    val[k] = E[src];
                    sw |= 1u << k;
                }
            }
        }
        if constexpr (OOP) {
#pragma unroll
            for (int k = 0; k < PER; k++)
                if (tid + CG_BLOCK * k < n) E2[tid + CG_BLOCK * k] = val[k];
            const typename K::P64 t = E;
            E = E2;
            E2 = t;
        } else {
            __syncthreads();
#pragma unroll
            for (int k = 0; k < PER; k++)
                if (sw & (1u << k)) E[tid + CG_BLOCK * k] = val[k];
        }
        __syncthreads();
        PCL_STEP();
        // S0: every element follows the cut into its child range
#pragma unroll
        for (int k = 0; k < PER; k++) {
            const uint32_t x = tid + CG_BLOCK * k, f = fe[k] & 0xffffu, e = fe[k] >> 16;
            if (st[k] & PART) {
                const uint32_t c = S.CUT[f];
                fe[k] = x < c ? (f | (c << 16)) : (c | (e << 16));
                dp[k] -= 1u;
            }
        }
    }
    // the ranges left longer than 16: a spent budget is heapsorted (__partial_sort) and stored
    // by its first element's thread; the others (at most WMAX records) go to one wave each (wt),
    // listed in PL (first | last << 16) and PR (budget), the count in cnt[0]
    if (tid == 0) cnt[0] = 0u;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const uint32_t x = tid + CG_BLOCK * k, f = fe[k] & 0xffffu, e = fe[k] >> 16;
        if (x < n && x == f && e - f > CG_SORT_THRESHOLD) {
            if (dp[k] == 0) {
                cg_heap_sort_range((uint64_t*)(E + f), (long)(e - f), PwLess{});
                for (uint32_t y = f; y < e; y++) out(y, E[y]);
            } else {
                const uint32_t q = atomicAdd((uint32_t*)(cnt + 0), 1u);
                S.PL[q] = fe[k];
                S.PR[q] = dp[k];
            }
        }
    }
    __syncthreads();
    {
        const uint32_t nw = cnt[0];
        for (uint32_t q = w; q < nw; q += WAVES) {
            const uint32_t r = S.PL[q];
            wt(E, r & 0xffffu, (r >> 16) - (r & 0xffffu), S.PR[q], out);
        }
    }
    PCL_STEP();
    // the final insertion passes of the ranges of at most 16
#pragma unroll
    for (int k = 0; k < PER; k++) {
        const uint32_t x = tid + CG_BLOCK * k, f = fe[k] & 0xffffu, e = fe[k] >> 16;
        if (x < n && e - f <= CG_SORT_THRESHOLD) {
            const uint64_t r = E[x];
            uint32_t kj[CG_SORT_THRESHOLD];
#pragma unroll
            for (uint32_t j = 0; j < CG_SORT_THRESHOLD; j++) kj[j] = f + j < e ? pcl_key(E[f + j]) : 0u;
            const uint32_t kx = pcl_key(r);
            uint32_t rank = 0;
#pragma unroll
            for (uint32_t j = 0; j < CG_SORT_THRESHOLD; j++)
                rank += f + j < e && ((kj[j] < kx) || (kj[j] == kx && f + j < x));
            out(f + rank, r);
        }
    }
    __syncthreads();
}

// std::sort(E, E + n) by key (E in W.VOX) into KEY, libstdc++'s permutation. Up to
// PCL_BLOCK_MAX elements: pcl_block_sort (scratch W.A, W.PAR, W.CNT, W.ORD; red
// for the counts). Longer arrays (the HBM-scratch backend, large-frame leaves in HBM): block
// levels over W.A (prefix, n + 1), W.PAR / W.CNT (L and R lists), W.UK (range of each
// position), W.ORD (flags), W.LAB (size | depth << 26 at each range's first), W.OFF (pivot,
// later last), KEY as words (s, later cut), until every range is at most PCL_BLOCK_MAX; those
// are then sorted one after another by pcl_block_sort. Every thread calls it; ends with a
// barrier.
// PMAX: the largest pcl_block_sort instantiation (elements per thread) the caller affords;
// LDS: the arrays of W live in LDS (n <= PMAX * CG_BLOCK then).
// E2: a second buffer of n records in LDS for the out-of-place swaps (LDS form only), or null.
template <int PMAX, bool LDS>
__device__ __forceinline__ void pcl_sort(const Work& W, uint64_t* E, uint32_t n, uint32_t* red, int depth0 = -1,
                                         uint64_t* E2 = nullptr) {
    constexpr uint32_t PCL_BLOCK_MAX = PMAX * CG_BLOCK;
    const uint32_t tid = threadIdx.x;
    uint32_t* PRE = W.A;
    uint32_t* PL = W.PAR;
    uint32_t* PR = W.CNT;
    uint32_t* RID = W.UK;
    uint32_t* FLG = W.ORD;
    uint32_t* INFO = (uint32_t*)W.LAB;
    uint32_t* PIV = W.OFF;
    uint32_t* SC = (uint32_t*)W.KEY;
    const uint32_t d0 = (uint32_t)(depth0 >= 0 ? depth0 : 2 * cg_lg((long)n));
    PCL_STAMP();
    if constexpr (LDS) {
        const PbScratch<PbLds> PS{(lds_u32*)W.A, (lds_u32*)W.PAR, (lds_u32*)W.CNT, (lds_u32*)W.ORD};
        lds_u64* const El = (lds_u64*)E;
        lds_u64* const Ko = (lds_u64*)W.KEY;
        lds_u32* const Rl = (lds_u32*)red;
        const PbStore<lds_u64*> out{Ko};
        if (E2) {
            lds_u64* const E2l = (lds_u64*)E2;
            if (n <= CG_BLOCK) pcl_block_sort<1, PbLds, PbStore<lds_u64*>, true>(El, out, n, d0, PS, Rl, E2l);
            else if (PMAX == 2 || n <= 2 * CG_BLOCK)
                pcl_block_sort<2, PbLds, PbStore<lds_u64*>, true>(El, out, n, d0, PS, Rl, E2l);
            else pcl_block_sort<PMAX, PbLds, PbStore<lds_u64*>, true>(El, out, n, d0, PS, Rl, E2l);
        } else {
            if (n <= CG_BLOCK) pcl_block_sort<1, PbLds>(El, out, n, d0, PS, Rl);
            else if (PMAX == 2 || n <= 2 * CG_BLOCK) pcl_block_sort<2, PbLds>(El, out, n, d0, PS, Rl);
            else pcl_block_sort<PMAX, PbLds>(El, out, n, d0, PS, Rl);
        }
        PCL_STAMP();
        return;
    }
    const PbScratch<PbGen> PS{W.A, W.PAR, W.CNT, W.ORD};
    if (n <= PMAX * CG_BLOCK) {
        pcl_block_sort<PMAX, PbGen>(E, PbStore<uint64_t*>{W.KEY}, n, d0, PS, red);
        PCL_STAMP();
        return;
    }
    // INFO at a range's first: size (26 bits) | depth budget << 26 (2 lg n <= 62)
    constexpr uint32_t ISZ = (1u << 26) - 1u;
    // per position, the exclusive counts of >= pivot and of <= pivot elements before it: two
    // 16-bit halves of one scan word while n < 65,536 (no carry between the halves); longer
    // arrays (a large frame's leaf in HBM) scan them separately, the <= counts in KEY's words
    // [n, 2n), which are free until the sorted records land in KEY after the levels
    const bool wide = n > 0xffffu;
    uint32_t* const PRL = SC + n;
    for (uint32_t i = tid; i < n; i += CG_BLOCK) {
        RID[i] = 0u;
        FLG[i] = i == 0 ? PCL_HEAD : 0u;
    }
    if (tid == 0 && n) INFO[0] = n | (d0 << 26);
    __syncthreads();
    bool any = n > 0;
    while (any) {
        // (1) per range: depth budget, heapsort fallback or median of three to first
        for (uint32_t i = tid; i < n; i += CG_BLOCK) {
            if (RID[i] != i) continue;
            const uint32_t size = INFO[i] & ISZ, depth = INFO[i] >> 26, last = i + size;
            if (depth == 0) {
                cg_heap_sort_range(E + i, (long)size, [](uint64_t a, uint64_t b) { return pcl_key(a) < pcl_key(b); });
                for (uint32_t j = i; j < last; j++) { FLG[j] |= PCL_HEAP; RID[j] = PCL_INACT; }
                continue;
            }
            const uint32_t mid = i + size / 2;
            cg_move_median_to_first(E, (long)i, (long)i + 1, (long)mid, (long)last - 1,
                                    [](uint64_t a, uint64_t b) { return pcl_key(a) < pcl_key(b); });
            PIV[i] = pcl_key(E[i]);
            INFO[i] = size | ((depth - 1u) << 26);
            SC[i] = 0u;
        }
        __syncthreads();
        // (2) counts of >= pivot and <= pivot before each position; the totals (the counts
        // before position n) stay on chip: the word after the array is the next range's first
        // word when leaves of one frame run side by side in HBM
        auto is_ge = [&](uint32_t i) -> bool {
            const uint32_t r = RID[i];
            return r != PCL_INACT && r != i && pcl_key(E[i]) >= PIV[r];
        };
        auto is_le = [&](uint32_t i) -> bool {
            const uint32_t r = RID[i];
            return r != PCL_INACT && r != i && pcl_key(E[i]) <= PIV[r];
        };
        uint32_t totg, totl;
        if (!wide) {
            const uint32_t ptot = block_scan(
                n, [&](uint32_t i) -> uint32_t { return (is_ge(i) ? 1u : 0u) | (is_le(i) ? 0x10000u : 0u); },
                [&](uint32_t i, uint32_t e) { PRE[i] = e; }, red);
            totg = ptot & 0xffffu;
            totl = ptot >> 16;
        } else {
            totg = block_scan(n, [&](uint32_t i) -> uint32_t { return is_ge(i) ? 1u : 0u; },
                              [&](uint32_t i, uint32_t e) { PRE[i] = e; }, red);
            totl = block_scan(n, [&](uint32_t i) -> uint32_t { return is_le(i) ? 1u : 0u; },
                              [&](uint32_t i, uint32_t e) { PRL[i] = e; }, red);
        }
        __syncthreads();
        auto preg = [&](uint32_t i) -> uint32_t { return i < n ? (wide ? PRE[i] : PRE[i] & 0xffffu) : totg; };
        auto prel = [&](uint32_t i) -> uint32_t { return i < n ? (wide ? PRL[i] : PRE[i] >> 16) : totl; };
        // (3) L and R lists of every range, stored from first + 1
        for (uint32_t i = tid; i < n; i += CG_BLOCK) {
            const uint32_t r = RID[i];
            if (r == PCL_INACT || r == i) continue;
            const uint32_t last = r + (INFO[r] & ISZ);
            const uint32_t k = pcl_key(E[i]), p = PIV[r];
            if (k >= p) PL[r + 1 + preg(i) - preg(r + 1)] = i;
            if (k <= p) PR[r + 1 + prel(last) - prel(i + 1)] = i;
        }
        __syncthreads();
        // (4) swap pairs (L_k, R_k) while L_k < R_k, by the thread at L_k; the last one
        // records the swap count s
        for (uint32_t i = tid; i < n; i += CG_BLOCK) {
            const uint32_t r = RID[i];
            if (r == PCL_INACT || r == i) continue;
            // >= pivot from the counts, not from E: other threads are swapping elements
            if (preg(i + 1) == preg(i)) continue;
            const uint32_t last = r + (INFO[r] & ISZ);
            const uint32_t nL = preg(last) - preg(r + 1), nR = prel(last) - prel(r + 1);
            const uint32_t k = preg(i) - preg(r + 1);
            const bool c0 = k < nR && i < PR[r + 1 + k];
            const bool c1 = k + 1 < nL && k + 1 < nR && PL[r + 2 + k] < PR[r + 2 + k];
            if (c0) {
                const uint32_t j = PR[r + 1 + k];
                const uint64_t t = E[i];
                E[i] = E[j];
                E[j] = t;
                if (!c1) SC[r] = k + 1;
            }
        }
        __syncthreads();
        // (5) per range: the cut, the two children (active while longer than 64)
        for (uint32_t i = tid; i < n; i += CG_BLOCK) {
            if (RID[i] != i) continue;
            const uint32_t size = INFO[i] & ISZ, dep = INFO[i] >> 26, last = i + size;
            const uint32_t nL = preg(last) - preg(i + 1);
            const uint32_t sw = SC[i];
            uint32_t cut;
            if (sw == 0) cut = PL[i + 1];
            else cut = min(sw < nL ? PL[i + 1 + sw] : 0xffffffffu, PR[i + sw]);
            FLG[cut] |= PCL_HEAD;
            INFO[i] = (cut - i) | (dep << 26);
            INFO[cut] = (last - cut) | (dep << 26);
            PIV[i] = last;
            SC[i] = cut;
        }
        __syncthreads();
        // (6) every position follows its child range
        bool mine = false;
        for (uint32_t i = tid; i < n; i += CG_BLOCK) {
            const uint32_t r = RID[i];
            if (r == PCL_INACT) continue;
            const uint32_t cut = SC[r], last = PIV[r];
            const uint32_t nr = i < cut ? (cut - r > PCL_BLOCK_MAX ? r : PCL_INACT)
                                        : (last - cut > PCL_BLOCK_MAX ? cut : PCL_INACT);
            RID[i] = nr;
            mine |= nr != PCL_INACT;
        }
        any = __syncthreads_or(mine);
        PCL_STAMP();
    }
    // the remaining ranges (at most PCL_BLOCK_MAX): those longer than 16 (not heapsorted) are
    // listed as tasks; the others get their final insertion pass here, a stable rank
    // inside the range (heapsorted ranges are sorted already)
    uint32_t* CUR = RID;                    // range firsts (RID is free after the block levels)
    uint64_t* KEY = W.KEY;
    const uint32_t ncur = block_scan(
        n,
        [&](uint32_t i) -> uint32_t {
            return (FLG[i] & (PCL_HEAD | PCL_HEAP)) == PCL_HEAD && (INFO[i] & ISZ) > CG_SORT_THRESHOLD ? 1u : 0u;
        },
        [&](uint32_t i, uint32_t e) {
            if ((FLG[i] & (PCL_HEAD | PCL_HEAP)) == PCL_HEAD && (INFO[i] & ISZ) > CG_SORT_THRESHOLD) CUR[e] = i;
        },
        red);
    for (uint32_t i = tid; i < n; i += CG_BLOCK) {
        const uint64_t ri = E[i];
        if (FLG[i] & PCL_HEAP) { KEY[i] = ri; continue; }
        uint32_t s0 = i;   // the range's first, if within 16 positions
        while (!(FLG[s0] & PCL_HEAD) && s0 + CG_SORT_THRESHOLD > i) s0--;
        if (!(FLG[s0] & PCL_HEAD)) continue;
        const uint32_t size = INFO[s0] & ISZ;
        if (size > CG_SORT_THRESHOLD) continue;   // a task
        const uint32_t ki = pcl_key(ri);
        uint32_t rank = 0;
        for (uint32_t j = s0; j < s0 + size; j++) {
            const uint32_t kj = pcl_key(E[j]);
            rank += (kj < ki) || (kj == ki && j < i);
        }
        KEY[s0 + rank] = ri;
    }
    __syncthreads();
    PCL_STAMP();
    // tasks, one after another: each range by the whole workgroup, scratch at its own positions
    for (uint32_t q = 0; q < ncur; q++) {
        const uint32_t first = CUR[q];
        const uint32_t size = INFO[first] & ISZ, depth = INFO[first] >> 26;
        __syncthreads();   // every thread has the range before pcl_block_sort rewrites INFO[first]
        pcl_block_sort<PMAX, PbGen>(E + first, PbStore<uint64_t*>{KEY + first}, size, depth,
                                    PbScratch<PbGen>{W.A + first, W.PAR + first, W.CNT + first, W.ORD + first},
                                    red);
    }
    __syncthreads();
    PCL_STAMP();
}

