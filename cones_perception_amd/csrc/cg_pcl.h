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
//  2. __introsort_loop level-synchronously while any range is longer than PCL_WAVE_MAX: per range, the
//     median of three moved to first, then the unguarded Hoare partition in parallel. Its
//     k-th swap exchanges the k-th element >= pivot from the left (L_k) with the k-th element
//     <= pivot from the right (R_k) while L_k < R_k; both lists are read off prefix counts of
//     the original range, because the scans pass only unswapped positions until they cross.
//     With s swaps the cut (where the left scan stops next) is L_0 if s = 0, else
//     min(L_s, R_{s-1}). Depth budget and heapsort fallback per range as in the sequential
//     code (cg_sort.h);
//  3. ranges of at most PCL_WAVE_MAX on single waves, in rounds: each round every wave
//     partitions ranges of the round's list with the same parallel formulas (ballots, LDS
//     lists) and lists the parts longer than 16 for the next round (no wave waits on another
//     except at the round's barrier);
//  4. the final insertion passes: a stable sort inside each range of at most 16 (the ranges
//     are weakly ordered, so this is the stable sort of the whole array).
// The permutation is checked against std::sort on the host (tests/test_math_host.py, the
// level model) and on the device against the oracle's ORDER_PCL (tests/test_gpu_pcl_order.py).
#ifdef CG_PCL_PROBE
__device__ unsigned long long g_pcl_probe[64];
__device__ unsigned int g_pcl_probe_n;
#define PCL_STAMP()                                                                      \
    do {                                                                                 \
        if (threadIdx.x == 0 && g_pcl_probe_n < 64) g_pcl_probe[g_pcl_probe_n++] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PCL_STAMP() ((void)0)
#endif
#define PCL_INACT 0xffffffffu
#define PCL_HEAD 1u
#define PCL_HEAP 2u
#define PCL_WAVE_MAX 512   // ranges up to this length are partitioned by single waves
__device__ __forceinline__ uint32_t pcl_key(uint64_t r) { return (uint32_t)(r >> 32); }

// Records (idx << 32 | slot) of the Mf finite points of W.P in index_vector order -> E.
// Kept survivors are slots [0, Ms) with point index W.IDX[slot] < 65536; zero pads are slots
// [Ms, M). Uses W.VOX (bitmap, word prefix; then E) and W.ORD. Ends with a barrier.
template <class KF>
__device__ __forceinline__ void pcl_index_vector(const Work& W, uint32_t M, uint32_t Ms, uint64_t* E,
                                                 uint32_t* red, KF voxel_idx) {
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    uint32_t* BM = (uint32_t*)W.VOX;       // 2048 words: one bit per point index
    uint32_t* WP = BM + 2048;              // exclusive popcount prefix per word
    for (uint32_t i = tid; i < 2048; i += CG_BLOCK) BM[i] = 0u;
    __syncthreads();
    for (uint32_t j = tid; j < Ms; j += CG_BLOCK) {
        const float4 p = W.P[j];
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            const uint32_t q = W.IDX[j];
            atomicOr(&BM[q >> 5], 1u << (q & 31u));
        }
    }
    __syncthreads();
    constexpr uint32_t PER = 2048 / CG_BLOCK;   // words per lane
    uint32_t c[PER], sum = 0;
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) { c[k] = __popc(BM[tid * PER + k]); sum += c[k]; }
    const uint32_t inc = wave_incl_scan(sum);
    if (l == 63) red[w] = inc;
    __syncthreads();
    uint32_t base = inc - sum;
    for (uint32_t v = 0; v < w; v++) base += red[v];
#pragma unroll
    for (uint32_t k = 0; k < PER; k++) { WP[tid * PER + k] = base; base += c[k]; }
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

// One wave: __move_median_to_first + __unguarded_partition(first + 1, last, first) of E by
// key, the parallel form (see above), for a range of at most PCL_WAVE_MAX: the keys held in
// registers (one 64-element chunk per register), the L and R lists in PL / PR from first + 1,
// then the swaps of the pairs (L_k, R_k) with L_k < R_k. Returns the cut (wave-uniform).
#define PCL_WAVE_CHUNKS (PCL_WAVE_MAX / 64)
__device__ inline uint32_t pcl_wave_partition(uint64_t* E, uint32_t* PL, uint32_t* PR, uint32_t first, uint32_t last) {
    const uint32_t l = lane_id();
    const uint32_t a = first + 1, mid = first + (last - first) / 2;
    // __move_median_to_first(first, first + 1, mid, last - 1): the three keys in one round trip
    const uint32_t ka = pcl_key(E[a]), kb = pcl_key(E[mid]), kc = pcl_key(E[last - 1]);
    uint32_t m, p;
    if (ka < kb) { if (kb < kc) { m = mid; p = kb; } else if (ka < kc) { m = last - 1; p = kc; } else { m = a; p = ka; } }
    else if (ka < kc) { m = a; p = ka; }
    else if (kb < kc) { m = last - 1; p = kc; }
    else { m = mid; p = kb; }
    if (l == 0) {
        const uint64_t t = E[first];
        E[first] = E[m];
        E[m] = t;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    // keys of [first + 1, last) in registers (after the median swap)
    uint32_t kr[PCL_WAVE_CHUNKS];
#pragma unroll
    for (int c = 0; c < PCL_WAVE_CHUNKS; c++) {
        const uint32_t x = a + 64u * c + l;
        kr[c] = x < last ? pcl_key(E[x]) : 0u;
    }
    uint64_t gem[PCL_WAVE_CHUNKS], lem[PCL_WAVE_CHUNKS];
    uint32_t nL = 0, nR = 0;
#pragma unroll
    for (int c = 0; c < PCL_WAVE_CHUNKS; c++) {
        const uint32_t x = a + 64u * c + l;
        gem[c] = __ballot(x < last && kr[c] >= p);
        lem[c] = __ballot(x < last && kr[c] <= p);
        nL += (uint32_t)__popcll(gem[c]);
        nR += (uint32_t)__popcll(lem[c]);
    }
    uint32_t bge = 0, ble = 0;
#pragma unroll
    for (int c = 0; c < PCL_WAVE_CHUNKS; c++) {
        const uint32_t x = a + 64u * c + l;
        if ((gem[c] >> l) & 1u) PL[a + bge + mbcnt(gem[c])] = x;
        if ((lem[c] >> l) & 1u) PR[a + nR - 1u - (ble + mbcnt(lem[c]))] = x;
        bge += (uint32_t)__popcll(gem[c]);
        ble += (uint32_t)__popcll(lem[c]);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    const uint32_t m2 = min(nL, nR);
    uint32_t sw = 0;
    for (uint32_t k0c = 0; k0c < m2; k0c += 64) {
        const uint32_t k = k0c + l;
        bool c = false;
        if (k < m2) {
            const uint32_t i = PL[a + k], j = PR[a + k];
            c = i < j;
            if (c) {
                const uint64_t t = E[i];
                E[i] = E[j];
                E[j] = t;
            }
        }
        const uint64_t cm = __ballot(c);
        sw += (uint32_t)__popcll(cm);
        if (~cm & __ballot(k < m2)) break;   // the pairs past the first failure all fail
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    return sw == 0 ? PL[a] : min(sw < nL ? PL[a + sw] : 0xffffffffu, PR[a + sw - 1u]);
}

// std::sort(E, E + n) by key (E in W.VOX) into KEY, libstdc++'s permutation. Scratch: W.A
// (prefix, n + 1), W.PAR / W.CNT (L and R lists), W.UK (range of each position), W.ORD
// (flags), W.LAB (size | depth << 20 at each range's first), W.OFF (pivot, later last),
// KEY as words (s, later cut). Every thread calls it; ends with a barrier.
__device__ inline void pcl_sort(const Work& W, uint64_t* E, uint32_t n, uint32_t* red, int depth0 = -1) {
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    uint32_t* PRE = W.A;
    uint32_t* PL = W.PAR;
    uint32_t* PR = W.CNT;
    uint32_t* RID = W.UK;
    uint32_t* FLG = W.ORD;
    uint32_t* INFO = (uint32_t*)W.LAB;
    uint32_t* PIV = W.OFF;
    uint32_t* SC = (uint32_t*)W.KEY;
    const bool big = n > PCL_WAVE_MAX;
    for (uint32_t i = tid; i < n; i += CG_BLOCK) {
        RID[i] = big ? 0u : PCL_INACT;
        FLG[i] = i == 0 ? PCL_HEAD : 0u;
    }
    if (tid == 0 && n) INFO[0] = n | ((uint32_t)(depth0 >= 0 ? depth0 : 2 * cg_lg((long)n)) << 20);
    __syncthreads();
    bool any = big;
    PCL_STAMP();
    while (any) {
        // (1) per range: depth budget, heapsort fallback or median of three to first
        for (uint32_t i = tid; i < n; i += CG_BLOCK) {
            if (RID[i] != i) continue;
            const uint32_t size = INFO[i] & 0xfffffu, depth = INFO[i] >> 20, last = i + size;
            if (depth == 0) {
                cg_heap_sort_range(E + i, (long)size, [](uint64_t a, uint64_t b) { return pcl_key(a) < pcl_key(b); });
                for (uint32_t j = i; j < last; j++) { FLG[j] |= PCL_HEAP; RID[j] = PCL_INACT; }
                continue;
            }
            const uint32_t mid = i + size / 2;
            cg_move_median_to_first(E, (long)i, (long)i + 1, (long)mid, (long)last - 1,
                                    [](uint64_t a, uint64_t b) { return pcl_key(a) < pcl_key(b); });
            PIV[i] = pcl_key(E[i]);
            INFO[i] = size | ((depth - 1u) << 20);
            SC[i] = 0u;
        }
        __syncthreads();
        // (2) counts of >= pivot (low half) and <= pivot (high half) before each position
        block_scan(
            n + 1,
            [&](uint32_t i) -> uint32_t {
                if (i >= n) return 0u;
                const uint32_t r = RID[i];
                if (r == PCL_INACT || r == i) return 0u;
                const uint32_t k = pcl_key(E[i]), p = PIV[r];
                return (k >= p ? 1u : 0u) | (k <= p ? 0x10000u : 0u);
            },
            [&](uint32_t i, uint32_t e) { PRE[i] = e; }, red);
        // (3) L and R lists of every range, stored from first + 1
        for (uint32_t i = tid; i < n; i += CG_BLOCK) {
            const uint32_t r = RID[i];
            if (r == PCL_INACT || r == i) continue;
            const uint32_t last = r + (INFO[r] & 0xfffffu), lo = PRE[r + 1];
            const uint32_t k = pcl_key(E[i]), p = PIV[r];
            if (k >= p) PL[r + 1 + (PRE[i] & 0xffffu) - (lo & 0xffffu)] = i;
            if (k <= p) PR[r + 1 + (PRE[last] >> 16) - (PRE[i + 1] >> 16)] = i;
        }
        __syncthreads();
        // (4) swap pairs (L_k, R_k) while L_k < R_k, by the thread at L_k; the last one
        // records the swap count s
        for (uint32_t i = tid; i < n; i += CG_BLOCK) {
            const uint32_t r = RID[i];
            if (r == PCL_INACT || r == i) continue;
            // >= pivot from the counts, not from E: other threads are swapping elements
            if (((PRE[i + 1] - PRE[i]) & 0xffffu) == 0u) continue;
            const uint32_t last = r + (INFO[r] & 0xfffffu), lo = PRE[r + 1], hiw = PRE[last];
            const uint32_t nL = (hiw & 0xffffu) - (lo & 0xffffu), nR = (hiw >> 16) - (lo >> 16);
            const uint32_t k = (PRE[i] & 0xffffu) - (lo & 0xffffu);
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
            const uint32_t size = INFO[i] & 0xfffffu, dep = INFO[i] >> 20, last = i + size;
            const uint32_t lo = PRE[i + 1], hiw = PRE[last];
            const uint32_t nL = (hiw & 0xffffu) - (lo & 0xffffu);
            const uint32_t sw = SC[i];
            uint32_t cut;
            if (sw == 0) cut = PL[i + 1];
            else cut = min(sw < nL ? PL[i + 1 + sw] : 0xffffffffu, PR[i + sw]);
            FLG[cut] |= PCL_HEAD;
            INFO[i] = (cut - i) | (dep << 20);
            INFO[cut] = (last - cut) | (dep << 20);
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
            const uint32_t nr = i < cut ? (cut - r > PCL_WAVE_MAX ? r : PCL_INACT)
                                        : (last - cut > PCL_WAVE_MAX ? cut : PCL_INACT);
            RID[i] = nr;
            mine |= nr != PCL_INACT;
        }
        any = __syncthreads_or(mine);
        PCL_STAMP();
    }
    // the remaining ranges (at most PCL_WAVE_MAX, longer than 16) in rounds: in each round
    // every wave takes ranges of the round's list (round robin), partitions each once by
    // itself and lists the parts still longer than 16 for the next round
    uint32_t* CUR = RID;                    // range firsts (RID is free after the block levels)
    uint32_t* NXT = PIV;                    // (PIV too)
    uint32_t* qc = red + 3 * WAVES;         // [0]: next round's count
    uint32_t ncur = block_scan(
        n,
        [&](uint32_t i) -> uint32_t {
            return (FLG[i] & (PCL_HEAD | PCL_HEAP)) == PCL_HEAD && (INFO[i] & 0xfffffu) > CG_SORT_THRESHOLD ? 1u : 0u;
        },
        [&](uint32_t i, uint32_t e) {
            if ((FLG[i] & (PCL_HEAD | PCL_HEAP)) == PCL_HEAD && (INFO[i] & 0xfffffu) > CG_SORT_THRESHOLD) CUR[e] = i;
        },
        red);
    if (tid == 0) qc[0] = 0u;
    __syncthreads();
    PCL_STAMP();
    while (ncur) {
        for (uint32_t q = w; q < ncur; q += WAVES) {
            const uint32_t first = CUR[q];
            const uint32_t last = first + (INFO[first] & 0xfffffu), depth = INFO[first] >> 20;
            if (depth == 0) {   // __partial_sort (heapsort) of the range: final
                if (l == 0)
                    cg_heap_sort_range(E + first, (long)(last - first),
                                       [](uint64_t a, uint64_t b) { return pcl_key(a) < pcl_key(b); });
                for (uint32_t x = first + l; x < last; x += 64) FLG[x] |= PCL_HEAP;
                continue;
            }
            const uint32_t cut = pcl_wave_partition(E, PL, PR, first, last);
            if (l == 0) {
                FLG[cut] |= PCL_HEAD;
                const uint32_t d = (depth - 1u) << 20;
                INFO[first] = (cut - first) | d;
                INFO[cut] = (last - cut) | d;
                if (cut - first > CG_SORT_THRESHOLD) NXT[atomicAdd(&qc[0], 1u)] = first;
                if (last - cut > CG_SORT_THRESHOLD) NXT[atomicAdd(&qc[0], 1u)] = cut;
            }
        }
        __syncthreads();
        ncur = qc[0];
        uint32_t* t = CUR; CUR = NXT; NXT = t;
        __syncthreads();
        if (tid == 0) qc[0] = 0u;
        __syncthreads();
    }
    __syncthreads();
    PCL_STAMP();
    // the final insertion passes: a stable sort inside each range of at most 16 (the ranges
    // are weakly ordered); heapsorted ranges are final. Each range's first lists its positions.
    uint32_t* SEG = PRE;
    for (uint32_t i = tid; i < n; i += CG_BLOCK)
        if ((FLG[i] & (PCL_HEAD | PCL_HEAP)) == PCL_HEAD) {
            const uint32_t e = i + (INFO[i] & 0xfffffu);
            for (uint32_t j = i; j < e; j++) SEG[j] = i;
        }
    __syncthreads();
    uint64_t* KEY = W.KEY;
    for (uint32_t i = tid; i < n; i += CG_BLOCK) {
        const uint64_t ri = E[i];
        if (FLG[i] & PCL_HEAP) { KEY[i] = ri; continue; }
        const uint32_t s0 = SEG[i], e0 = s0 + (INFO[s0] & 0xfffffu);
        const uint32_t ki = pcl_key(ri);
        uint32_t rank = 0;
        for (uint32_t j = s0; j < e0; j++) {
            const uint32_t kj = pcl_key(E[j]);
            rank += (kj < ki) || (kj == ki && j < i);
        }
        KEY[s0 + rank] = ri;
    }
    __syncthreads();
    PCL_STAMP();
}

