// cg_sort.h — restatement of libstdc++'s std::sort (introsort) for device code.
//
// PCL's EuclideanClusterExtraction::extract orders clusters with
//   std::sort(clusters.rbegin(), clusters.rend(), comparePointClusters)
// (size-ascending over the reversed vector), and VoxelGrid orders points with
//   std::sort(index_vector.begin(), index_vector.end(), std::less<cloud_point_index_idx>())
// Both comparators look at one key only, so the relative order of equal keys is whatever the
// introsort permutation produces. Reproducing PCL's output order therefore means reproducing
// libstdc++'s algorithm step for step: median-of-three pivot moved to first, unguarded Hoare
// partition, depth limit 2*floor(log2 n) with heapsort fallback, threshold 16, final insertion
// sort (guarded on the first 16, unguarded after). The GCC 9-13 implementation is unchanged
// across those releases. The GPU parity tests check it against the oracle's host std::sort on
// tie-heavy cluster lists (frames with more than 16 clusters of repeated sizes).
//
// Sequential by design. The array is any A with f[i] (read, assign) and f + d (a view at
// offset d): a pointer (one lane over LDS or memory), or CgWaveRegs64 below (every lane of
// one wave runs the same uniform program over records held one per lane, so that indices
// and compares stay scalar and element accesses are v_readlane / v_writelane).
#pragma once
#include <stdint.h>
#include "cg_math.h"

#define CG_SORT_THRESHOLD 16

template <class A> struct cg_elem { using type = typename A::value_type; };
template <class T> struct cg_elem<T*> { using type = T; };

template <class A>
CG_HD void cg_iter_swap(A a, long i, long j) {
    typename cg_elem<A>::type t = a[i];
    a[i] = a[j];
    a[j] = t;
}

template <class A, class T, class L>
CG_HD void cg_adjust_heap(A f, long hole, long len, T value, L less) {
    const long top = hole;
    long second = hole;
    while (second < (len - 1) / 2) {
        second = 2 * (second + 1);
        if (less(f[second], f[second - 1])) second--;
        f[hole] = f[second];
        hole = second;
    }
    if ((len & 1) == 0 && second == (len - 2) / 2) {
        second = 2 * (second + 1);
        f[hole] = f[second - 1];
        hole = second - 1;
    }
    long parent = (hole - 1) / 2;
    while (hole > top && less(f[parent], value)) {
        f[hole] = f[parent];
        hole = parent;
        parent = (hole - 1) / 2;
    }
    f[hole] = value;
}

template <class A, class L>
CG_HD void cg_make_heap(A f, long len, L less) {
    if (len < 2) return;
    long parent = (len - 2) / 2;
    while (true) {
        typename cg_elem<A>::type v = f[parent];
        cg_adjust_heap(f, parent, len, v, less);
        if (parent == 0) return;
        parent--;
    }
}

template <class A, class L>
CG_HD void cg_heap_sort_range(A f, long len, L less) {   // __partial_sort(first, last, last)
    cg_make_heap(f, len, less);
    while (len > 1) {
        --len;
        typename cg_elem<A>::type v = f[len];
        f[len] = f[0];
        cg_adjust_heap(f, 0L, len, v, less);
    }
}

template <class A, class L>
CG_HD void cg_move_median_to_first(A f, long result, long a, long b, long c, L less) {
    if (less(f[a], f[b])) {
        if (less(f[b], f[c])) cg_iter_swap(f, result, b);
        else if (less(f[a], f[c])) cg_iter_swap(f, result, c);
        else cg_iter_swap(f, result, a);
    } else if (less(f[a], f[c])) cg_iter_swap(f, result, a);
    else if (less(f[b], f[c])) cg_iter_swap(f, result, c);
    else cg_iter_swap(f, result, b);
}

template <class A, class L>
CG_HD long cg_unguarded_partition(A f, long first, long last, long pivot, L less) {
    while (true) {
        while (less(f[first], f[pivot])) ++first;
        --last;
        while (less(f[pivot], f[last])) --last;
        if (!(first < last)) return first;
        cg_iter_swap(f, first, last);
        ++first;
    }
}

template <class A, class L>
CG_HD void cg_insertion_sort(A f, long first, long last, L less) {
    if (first == last) return;
    for (long i = first + 1; i != last; ++i) {
        typename cg_elem<A>::type val = f[i];
        if (less(val, f[first])) {
            for (long k = i; k > first; --k) f[k] = f[k - 1];
            f[first] = val;
        } else {
            long hole = i, next = i - 1;
            while (less(val, f[next])) { f[hole] = f[next]; hole = next; --next; }
            f[hole] = val;
        }
    }
}

template <class A, class L>
CG_HD void cg_unguarded_insertion_sort(A f, long first, long last, L less) {
    for (long i = first; i != last; ++i) {
        typename cg_elem<A>::type val = f[i];
        long hole = i, next = i - 1;
        while (less(val, f[next])) { f[hole] = f[next]; hole = next; --next; }
        f[hole] = val;
    }
}

CG_HD int cg_lg(long n) { int r = 0; while (n > 1) { n >>= 1; r++; } return r; }

// std::sort(f, f + n, less). The recursion of __introsort_loop on the right part is replaced
// by an explicit stack: sub-ranges are disjoint, so processing order does not change the
// result, only each range's depth budget matters (kept per stack entry). `stk` holds
// 3 * CG_SORT_STACK ints (LDS on the device); pending entries never exceed 2*floor(log2 n).
#define CG_SORT_STACK 64
template <class A, class L, class STK>
CG_HD void cg_std_sort(A f, long n, L less, STK stk) {
    if (n <= 1) return;
    int sp = 0;
    stk[0] = 0; stk[1] = (int)n; stk[2] = cg_lg(n) * 2; sp = 1;
    while (sp > 0) {
        --sp;
        long first = stk[3 * sp], last = stk[3 * sp + 1];
        int depth = stk[3 * sp + 2];
        while (last - first > CG_SORT_THRESHOLD) {
            if (depth == 0) { cg_heap_sort_range(f + first, last - first, less); break; }
            --depth;
            long mid = first + (last - first) / 2;
            cg_move_median_to_first(f, first, first + 1, mid, last - 1, less);
            long cut = cg_unguarded_partition(f, first + 1, last, first, less);
            stk[3 * sp] = (int)cut; stk[3 * sp + 1] = (int)last; stk[3 * sp + 2] = depth; sp++;
            last = cut;
        }
    }
    if (n > CG_SORT_THRESHOLD) {
        cg_insertion_sort(f, 0L, (long)CG_SORT_THRESHOLD, less);
        cg_unguarded_insertion_sort(f, (long)CG_SORT_THRESHOLD, n, less);
    } else {
        cg_insertion_sort(f, 0L, n, less);
    }
}

#ifdef __HIPCC__
// v_writelane: lane k of v takes x (k uniform)
__device__ __forceinline__ int cg_writelane(int x, int k, int v) {
    return (int)(__builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u))) == k ? x : v;
}
// Records of one wave, element i in lane i (64-bit: two VGPRs). Every lane of the wave must
// run the same program with uniform indices (the sort above, called by the whole wave).
struct CgWaveRegs64 {
    using value_type = uint64_t;
    uint32_t* lo;
    uint32_t* hi;
    long base;
    struct Ref {
        const CgWaveRegs64* a;
        long i;
        __device__ __forceinline__ operator uint64_t() const { return a->get(i); }
        __device__ __forceinline__ Ref& operator=(uint64_t v) { a->set(i, v); return *this; }
        __device__ __forceinline__ Ref& operator=(const Ref& o) { a->set(i, (uint64_t)o); return *this; }
    };
    __device__ __forceinline__ uint64_t get(long i) const {
        const int k = (int)(base + i);
        return ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)*hi, k) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)*lo, k);
    }
    __device__ __forceinline__ void set(long i, uint64_t v) const {
        const int k = (int)(base + i);
        *lo = (uint32_t)cg_writelane((int)(uint32_t)v, k, (int)*lo);
        *hi = (uint32_t)cg_writelane((int)(uint32_t)(v >> 32), k, (int)*hi);
    }
    __device__ __forceinline__ Ref operator[](long i) const { return Ref{this, i}; }
    __device__ __forceinline__ CgWaveRegs64 operator+(long d) const { return CgWaveRegs64{lo, hi, base + d}; }
};
// 32-bit records of one wave, element i in lane i (one VGPR)
struct CgWaveRegs32 {
    using value_type = uint32_t;
    uint32_t* v;
    long base;
    struct Ref {
        const CgWaveRegs32* a;
        long i;
        __device__ __forceinline__ operator uint32_t() const { return a->get(i); }
        __device__ __forceinline__ Ref& operator=(uint32_t x) { a->set(i, x); return *this; }
        __device__ __forceinline__ Ref& operator=(const Ref& o) { a->set(i, (uint32_t)o); return *this; }
    };
    __device__ __forceinline__ uint32_t get(long i) const {
        return (uint32_t)__builtin_amdgcn_readlane((int)*v, (int)(base + i));
    }
    __device__ __forceinline__ void set(long i, uint32_t x) const {
        *v = (uint32_t)cg_writelane((int)x, (int)(base + i), (int)*v);
    }
    __device__ __forceinline__ Ref operator[](long i) const { return Ref{this, i}; }
    __device__ __forceinline__ CgWaveRegs32 operator+(long d) const { return CgWaveRegs32{v, base + d}; }
};
// cg_std_sort's stack of (first, last, depth) triples, entry s in lane s of three VGPRs
struct CgWaveStack {
    int32_t* r;   // r[0..2]
    struct Ref {
        const CgWaveStack* a;
        int i;
        __device__ __forceinline__ operator int() const {
            const int q = i / 3, k = i - 3 * q;
            return __builtin_amdgcn_readlane(k == 0 ? a->r[0] : k == 1 ? a->r[1] : a->r[2], q);
        }
        __device__ __forceinline__ Ref& operator=(int v) {
            const int q = i / 3, k = i - 3 * q;
            if (k == 0) a->r[0] = cg_writelane(v, q, a->r[0]);
            else if (k == 1) a->r[1] = cg_writelane(v, q, a->r[1]);
            else a->r[2] = cg_writelane(v, q, a->r[2]);
            return *this;
        }
    };
    __device__ __forceinline__ Ref operator[](int i) const { return Ref{this, i}; }
};
#endif

#ifdef __HIPCC__
// std::sort of n <= 64 records (size << 16 | payload, ordered by size only) held one per lane
// of one wave (lane i: element i), with libstdc++'s control flow (the stack of ranges, depth
// budget, median-of-three, Hoare partition, guarded then unguarded insertion sort, heapsort
// fallback) but every linear scan replaced by one ballot: a scan that stops at the first (or
// last) element satisfying a compare is the lowest (or highest) set bit of the compare's
// ballot over the scanned range, and the final insertion passes are one stable rank sort.
// Called by every lane of the wave with the same n. Same permutation as cg_std_sort.
__device__ __forceinline__ uint32_t cg_wave_lane() {
    return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
}
__device__ __forceinline__ uint32_t cg_wave_get(uint32_t v, int i) {
    return (uint32_t)__builtin_amdgcn_readlane((int)v, i);
}
__device__ __forceinline__ void cg_wave_swap(uint32_t& v, int i, int j) {
    const uint32_t a = cg_wave_get(v, i), b = cg_wave_get(v, j);
    const int l = (int)cg_wave_lane();
    v = l == i ? b : (l == j ? a : v);
}
__device__ __forceinline__ uint64_t cg_lanes_below(int k) {   // lanes [0, k)
    return k >= 64 ? ~0ull : (k <= 0 ? 0ull : (1ull << k) - 1ull);
}
// Stable sort of lanes [0, n) by size: each element's rank counts the smaller sizes and the
// equal sizes before it; one forward permute moves it there. libstdc++'s final pass (a guarded
// insertion sort of the first 16, then unguarded insertion of the rest into the sorted prefix)
// is an insertion sort of the whole range, i.e. exactly this stable sort.
__device__ __forceinline__ void cg_wave_stable_sort(uint32_t& v, int n) {
    const int l = (int)cg_wave_lane();
    const uint32_t k = v >> 16;
    uint32_t rank = 0;
    for (int j = 0; j < n; j++) {
        const uint32_t kj = cg_wave_get(v, j) >> 16;
        rank += (kj < k) || (kj == k && j < l);
    }
    if (l >= n) rank = (uint32_t)l;
    v = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank * 4), (int)v);
}
__device__ inline void cg_std_sort_wave32(uint32_t& v, int n) {
    if (n <= 1) return;
    const int l = (int)cg_wave_lane();
    auto less = [](uint32_t a, uint32_t b) { return (a >> 16) < (b >> 16); };
    int32_t st[3] = {0, 0, 0};
    const CgWaveStack stk{st};
    int sp = 0;
    stk[0] = 0; stk[1] = n; stk[2] = cg_lg(n) * 2; sp = 1;
    while (sp > 0) {
        --sp;
        int first = stk[3 * sp], last = stk[3 * sp + 1];
        int depth = stk[3 * sp + 2];
        while (last - first > CG_SORT_THRESHOLD) {
            if (depth == 0) {
                const CgWaveRegs32 f{&v, 0};
                cg_heap_sort_range(f + first, (long)(last - first), less);
                break;
            }
            --depth;
            const int mid = first + (last - first) / 2;
            {   // __move_median_to_first(first, first + 1, mid, last - 1)
                const int a = first + 1, b = mid, c = last - 1;
                const uint32_t fa = cg_wave_get(v, a), fb = cg_wave_get(v, b), fc = cg_wave_get(v, c);
                int m;
                if (less(fa, fb)) m = less(fb, fc) ? b : (less(fa, fc) ? c : a);
                else m = less(fa, fc) ? a : (less(fb, fc) ? c : b);
                cg_wave_swap(v, first, m);
            }
            // __unguarded_partition(first + 1, last, pivot = first): the pivot stays put
            const uint32_t p = cg_wave_get(v, first) >> 16;
            int lo = first + 1, hi = last;
            while (true) {
                lo = __builtin_ctzll(__ballot((v >> 16) >= p) & ~cg_lanes_below(lo));   // first f[i] >= p
                --hi;
                hi = 63 - __builtin_clzll(__ballot((v >> 16) <= p) & cg_lanes_below(hi + 1));   // last f[j] <= p
                if (!(lo < hi)) break;
                cg_wave_swap(v, lo, hi);
                ++lo;
            }
            stk[3 * sp] = lo; stk[3 * sp + 1] = last; stk[3 * sp + 2] = depth; sp++;
            last = lo;
        }
    }
    (void)l;
    cg_wave_stable_sort(v, n);   // the final insertion passes
}
#endif

