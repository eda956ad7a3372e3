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
// across those releases. tests/test_sort_host.py checks this restatement against the host
// std::sort permutation for many tie-heavy inputs.
//
// Single-threaded by design (runs in one lane over short arrays such as the cluster list).
#pragma once
#include <stdint.h>
#include "cg_math.h"

#define CG_SORT_THRESHOLD 16

template <class T>
CG_HD void cg_iter_swap(T* a, long i, long j) { T t = a[i]; a[i] = a[j]; a[j] = t; }

template <class T, class L>
CG_HD void cg_adjust_heap(T* f, long hole, long len, T value, L less) {
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

template <class T, class L>
CG_HD void cg_make_heap(T* f, long len, L less) {
    if (len < 2) return;
    long parent = (len - 2) / 2;
    while (true) {
        T v = f[parent];
        cg_adjust_heap(f, parent, len, v, less);
        if (parent == 0) return;
        parent--;
    }
}

template <class T, class L>
CG_HD void cg_heap_sort_range(T* f, long len, L less) {   // __partial_sort(first, last, last)
    cg_make_heap(f, len, less);
    while (len > 1) {
        --len;
        T v = f[len];
        f[len] = f[0];
        cg_adjust_heap(f, 0L, len, v, less);
    }
}

template <class T, class L>
CG_HD void cg_move_median_to_first(T* f, long result, long a, long b, long c, L less) {
    if (less(f[a], f[b])) {
        if (less(f[b], f[c])) cg_iter_swap(f, result, b);
        else if (less(f[a], f[c])) cg_iter_swap(f, result, c);
        else cg_iter_swap(f, result, a);
    } else if (less(f[a], f[c])) cg_iter_swap(f, result, a);
    else if (less(f[b], f[c])) cg_iter_swap(f, result, c);
    else cg_iter_swap(f, result, b);
}

template <class T, class L>
CG_HD long cg_unguarded_partition(T* f, long first, long last, long pivot, L less) {
    while (true) {
        while (less(f[first], f[pivot])) ++first;
        --last;
        while (less(f[pivot], f[last])) --last;
        if (!(first < last)) return first;
        cg_iter_swap(f, first, last);
        ++first;
    }
}

template <class T, class L>
CG_HD void cg_insertion_sort(T* f, long first, long last, L less) {
    if (first == last) return;
    for (long i = first + 1; i != last; ++i) {
        T val = f[i];
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

template <class T, class L>
CG_HD void cg_unguarded_insertion_sort(T* f, long first, long last, L less) {
    for (long i = first; i != last; ++i) {
        T val = f[i];
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
template <class T, class L>
CG_HD void cg_std_sort(T* f, long n, L less, int* stk) {
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
