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
//            thresholds, exact re-read of x, y, z for band codes only
//                                                       (src/ground_removal.cpp:70-77, and
//                                                        src/cone_detection.cpp:189-204)
//    gather  per-wave atomic append of the survivors (x, y, z, intensity, point index) into LDS
//            (M <= CG_MMAX) or the frame's HBM scratch
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

#define CG_BRUTE_V 256        // voxel count up to which clustering tests all pairs

// ------------------------------------------------------------------------------------------
// LDS map. The frontend's 16-bit z-key prefixes (zq) overlay the backend arrays, which are
// dead until pass 3 begins; pass 2 leaves its decisions in registers.
struct FrontShared {
    float4 rays[CG_NUM_BINS];      // sector edge rays of the pass-1 fast path
    uint32_t sec_key[CG_NUM_BINS + 1];
    float thr[CG_NUM_BINS + 1];
    uint32_t tkey[CG_NUM_BINS + 1];
    uint32_t cnt[CG_MAX_POINTS / 64];  // ground-only mode: kept per (k, wave), then offsets
    uint32_t red[8 * WAVES];       // wave partials
    uint32_t scal[64];             // broadcast scalars
    int32_t stk[3 * CG_SORT_STACK];// introsort stack (cluster order)
};
#define FRONT_BYTES ((sizeof(FrontShared) + 255) & ~(size_t)255)

struct BackLds {
    float4 P[CG_MMAX];
    uint64_t KEY[CG_MMAX];
    float4 VOX[CG_MMAX];
    uint32_t A[CG_MMAX + 4];
    uint32_t PAR[CG_MMAX];
    uint32_t CNT[CG_MMAX];
    uint32_t UK[CG_MMAX];
    int32_t LAB[CG_MMAX];
    uint32_t ORD[CG_MMAX];
    uint32_t IDX[CG_MMAX];
    uint32_t OFF[CG_MMAX + 4];
};
#define SMEM_BYTES (FRONT_BYTES + sizeof(BackLds))
static_assert(SMEM_BYTES <= 163840, "LDS budget");
// pcl_index_vector keeps a 2,048-word point bitmap and its 2,048-word prefix in VOX
static_assert(sizeof(((BackLds*)nullptr)->VOX) >= 4096 * sizeof(uint32_t), "VOX holds the index_vector bitmap");
// the LDS PCL sort (pcl_sort<2, true>) covers at most two records per thread
static_assert(CG_MMAX <= 2 * CG_BLOCK, "LDS backend capacity within pcl_block_sort<2>");
#ifndef CG_CODES_HBM
static_assert(sizeof(BackLds) >= CG_MAX_POINTS * sizeof(uint8_t), "z-code overlay must fit");
#endif
// (experiment, -DCG_CODES_HBM: the z codes in the frame's HBM scratch instead of LDS, so that a
// smaller CG_MMAX lets more workgroups share a CU)

#ifndef CG_PREFETCH
#define CG_PREFETCH 2   // filter survivors per lane loaded right after pass 1
#endif

// Scalar slots in FrontShared::scal
enum {
    S_K = 0, S_MS, S_M, S_MF, S_V, S_C, S_U, S_FLAGS, S_PASS,
    S_MINB0, S_MINB1, S_MINB2, S_MUL1, S_MUL2,
    S_ORGX, S_ORGY, S_ORGZ, S_TKMIN, S_TKMAX, S_TOUCHED,
    S_BMIN0, S_BMIN1, S_BMIN2, S_BMAX0, S_BMAX1, S_BMAX2, S_TMP, S_LAST
};



uint64_t cg_scratch_bytes(uint32_t n) {
    uint64_t n2 = 1; while (n2 < n) n2 <<= 1;
    uint64_t c = (uint64_t)n + 4;
    const uint64_t b = 16 * c + 8 * n2 + 16 * c + 4 * c * 8 + 256;
#ifdef CG_CODES_HBM
    return b > CG_MAX_POINTS ? b : (uint64_t)CG_MAX_POINTS;   // the codes overlay it until compaction
#else
    return b;
#endif
}

__device__ __forceinline__ Work global_work(uint8_t* base, uint32_t n) {
    uint64_t n2 = 1; while (n2 < n) n2 <<= 1;
    const uint64_t c = (uint64_t)n + 4;
    Work w;
    uint8_t* p = base;
    w.P = (float4*)p; p += 16 * c;
    w.VOX = (float4*)p; p += 16 * c;
    w.KEY = (uint64_t*)p; p += 8 * n2;
    w.A = (uint32_t*)p; p += 4 * c;
    w.PAR = (uint32_t*)p; p += 4 * c;
    w.CNT = (uint32_t*)p; p += 4 * c;
    w.UK = (uint32_t*)p; p += 4 * c;
    w.LAB = (int32_t*)p; p += 4 * c;
    w.ORD = (uint32_t*)p; p += 4 * c;
    w.IDX = (uint32_t*)p; p += 4 * c;
    w.OFF = (uint32_t*)p; p += 4 * c;
    return w;
}

// ------------------------------------------------------------------------------------------
// Backend: voxel grid + Euclidean clustering + centroids for one frame of M survivors in W.P.
__device__ __forceinline__ void backend(const Work& W, uint32_t M, FrontShared* fs, const CgLaunch& L,
                                        const CgDevParams& P, uint32_t f, uint32_t flags) {
    const uint32_t tid = threadIdx.x, l = lane_id(), w = wave_id();
    uint32_t* red = fs->red;
    // ---- voxel grid: getMinMax3D (finite points; bounds gathered by the frontend) ----
    if (w == 0) {
        const uint32_t nfin = fs->scal[S_MF];
        float bmn[3], bmx[3];
#pragma unroll
        for (int a = 0; a < 3; a++) {
            bmn[a] = cg_fkey_inv(fs->scal[S_BMIN0 + a]);
            bmx[a] = cg_fkey_inv(fs->scal[S_BMAX0 + a]);
        }
        uint32_t pass = 0;
        int min_b[3], div_b[3];
        voxel_grid_setup(nfin, bmn, bmx, P, pass, min_b, div_b);
        if (l == 0) {
            fs->scal[S_PASS] = pass;
            fs->scal[S_MINB0] = (uint32_t)min_b[0];
            fs->scal[S_MINB1] = (uint32_t)min_b[1];
            fs->scal[S_MINB2] = (uint32_t)min_b[2];
            fs->scal[S_MUL1] = (uint32_t)div_b[0];
            fs->scal[S_MUL2] = (uint32_t)div_b[0] * (uint32_t)div_b[1];
        }
    }
    __syncthreads();
    STAMP(6);
    const uint32_t pass = fs->scal[S_PASS];
    uint32_t V;
    float4* const vox_out = L.vox + (uint64_t)f * L.cap;
    if (pass) {
        // overflow guard: output = *input_ (all M points in point order)
        uint64_t* tmp = (uint64_t*)W.VOX;
        for (uint32_t j = tid; j < M; j += CG_BLOCK) tmp[j] = ((uint64_t)W.IDX[j] << 16) | j;
        __syncthreads();
        if (M <= CG_RANK_SORT_MAX) {
            rank_sort(tmp, W.KEY, M);
        } else {
            uint32_t n2 = 1;
            while (n2 < M) n2 <<= 1;
            for (uint32_t j = tid; j < n2; j += CG_BLOCK) W.KEY[j] = j < M ? tmp[j] : ~0ull;
            __syncthreads();
            bitonic_sort(W.KEY, n2);
        }
        for (uint32_t r = tid; r < M; r += CG_BLOCK) {
            const float4 pp = W.P[(uint32_t)(W.KEY[r] & 0xffffu)];
            W.VOX[r] = pp;
            vox_out[r] = pp;
        }
        V = M;
        flags |= 0x1u;
        __syncthreads();
    } else {
        const float mnb0 = (float)(int)fs->scal[S_MINB0], mnb1 = (float)(int)fs->scal[S_MINB1],
                    mnb2 = (float)(int)fs->scal[S_MINB2];
        const uint32_t mul1 = fs->scal[S_MUL1], mul2 = fs->scal[S_MUL2];
        const uint32_t Mf = fs->scal[S_MF];
        auto voxel_idx = [&](const float4& p) -> uint32_t {
            const int i0 = (int)(floorf(p.x * P.inv_leaf[0]) - mnb0);
            const int i1 = (int)(floorf(p.y * P.inv_leaf[1]) - mnb1);
            const int i2 = (int)(floorf(p.z * P.inv_leaf[2]) - mnb2);
            return (uint32_t)i0 + (uint32_t)i1 * mul1 + (uint32_t)i2 * mul2;
        };
        if (P.voxel_order == CG_VOXEL_ORDER_PCL) {
            // index_vector in cloud order (VOX is free until the centroids), then std::sort's
            // permutation of it into KEY (cg_pcl.h)
            uint64_t* E = (uint64_t*)W.VOX;
            pcl_index_vector(W, M, fs->scal[S_MS], E, red, [&](uint32_t j) -> uint32_t { return voxel_idx(W.P[j]); });
            STAMP(7);
            if (flags & CG_F_GLOBAL_SCRATCH) pcl_sort<2, false>(W, E, Mf, red);
            else pcl_sort<2, true>(W, E, Mf, red, -1, E + CG_MMAX);   // VOX's upper half: swaps out of place
        } else {
            // keys (idx << 32 | point index << 16 | slot): unique, so any sort yields PCL's idx
            // order with ties in point order. Non-finite points get idx 0xffffffff (beyond every
            // real idx, which the overflow guard keeps below 2^31) and sort last.
            flags |= CG_F_VOXEL_POINT_ORDER;
            auto voxel_key = [&](uint32_t j) -> uint64_t {
                const float4 p = W.P[j];
                const uint64_t lowbits = ((uint64_t)(W.IDX[j] & 0xffffu) << 16) | j;
                if (!(isfinite(p.x) && isfinite(p.y) && isfinite(p.z))) return (0xffffffffull << 32) | lowbits;
                return ((uint64_t)voxel_idx(p) << 32) | lowbits;
            };
            if (M <= CG_RANK_SORT_MAX) {
                uint64_t* tmp = (uint64_t*)W.VOX;      // VOX is free until the centroids
                for (uint32_t j = tid; j < M; j += CG_BLOCK) tmp[j] = voxel_key(j);
                __syncthreads();
                STAMP(7);
                rank_sort(tmp, W.KEY, M);
            } else {
                uint32_t n2 = 1;
                while (n2 < M) n2 <<= 1;
                for (uint32_t j = tid; j < n2; j += CG_BLOCK) W.KEY[j] = j < M ? voxel_key(j) : ~0ull;
                __syncthreads();
                STAMP(7);
                bitonic_sort(W.KEY, n2);
            }
        }
        STAMP(8);
        V = block_scan(
            Mf,
            [&](uint32_t j) -> uint32_t { return (j == 0 || (W.KEY[j] >> 32) != (W.KEY[j - 1] >> 32)) ? 1u : 0u; },
            [&](uint32_t j, uint32_t e) {
                if (j == 0 || (W.KEY[j] >> 32) != (W.KEY[j - 1] >> 32)) W.A[e] = j;
            },
            red);
        if (tid == 0) W.A[V] = Mf;
        __syncthreads();
        STAMP(9);
        // CentroidPoint<PointXYZI>: float sums in ascending point position, / float(n)
        for (uint32_t v = tid; v < V; v += CG_BLOCK) {
            const uint32_t s = W.A[v], e = W.A[v + 1];
            float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
            for (uint32_t j = s; j < e; j++) {
                const float4 p = W.P[(uint32_t)(W.KEY[j] & 0xffffu)];
                sx += p.x; sy += p.y; sz += p.z; si += p.w;
            }
            const float n = (float)(e - s);
            const float4 c = make_float4(sx / n, sy / n, sz / n, si / n);
            W.VOX[v] = c;
            vox_out[v] = c;
        }
        __syncthreads();
    }
    STAMP(10);
    // ---- Euclidean clustering over the V voxel points ----
    uint32_t C = 0;
    if (V > 0) {
        if (V <= CG_BRUTE_V) {
            // (1) adjacency bitmasks: row v, 16-column chunk c is one task; lanes of a wave share
            // c, so the column voxels are LDS broadcasts. A voxel is its own neighbour (distance
            // 0 < r2) unless it is not finite (passthrough clouds), then it is isolated.
            // (2) every voxel points at its lowest neighbour (<= itself): a forest whose trees
            // lie inside components; (3) pointer jumping flattens it; (4) only edges leaving a
            // tree (row & ~members(tree)) are united. Roots stay each component's lowest index.
            uint16_t* const adj = (uint16_t*)W.KEY;                // [V][16] chunks, 32 B rows
            unsigned long long* const tm = (unsigned long long*)W.P;   // [V][4] tree members
            const uint32_t nc = (V + 15) >> 4, nw = (V + 63) >> 6;
            for (uint32_t t = tid; t < V * nc; t += CG_BLOCK) {
                const uint32_t c = t / V, v = t - c * V;
                const float4 q = W.VOX[v];
                uint32_t bits = 0;
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    float4 pc[8];
#pragma unroll
                    for (int b = 0; b < 8; b++) pc[b] = W.VOX[min(16 * c + 8 * h + b, V - 1)];
#pragma unroll
                    for (int b = 0; b < 8; b++) {
                        const float ddx = q.x - pc[b].x, ddy = q.y - pc[b].y, ddz = q.z - pc[b].z;
                        float acc = ddx * ddx;
                        acc = acc + ddy * ddy;
                        acc = acc + ddz * ddz;
                        bits |= (uint32_t)(acc < P.r2 && 16 * c + 8 * h + b < V) << (8 * h + b);
                    }
                }
                adj[v * 16 + c] = (uint16_t)bits;
            }
            for (uint32_t t = tid; t < V * 4; t += CG_BLOCK) tm[t] = 0ull;
            if (tid == 0) { fs->scal[S_TMP] = 0; fs->scal[S_TMP + 1] = 0; fs->scal[S_TMP + 2] = 0; }
            __syncthreads();
            STAMP(11);
            auto row = [&](uint32_t v, uint32_t i) -> unsigned long long {
                const unsigned long long x = ((const unsigned long long*)(adj + v * 16))[i];
                const uint32_t hi = V - 64 * i;   // columns >= V were never written
                return hi >= 64 ? x : x & ((1ull << hi) - 1ull);
            };
            for (uint32_t v = tid; v < V; v += CG_BLOCK) {
                uint32_t p = v;
                for (uint32_t i = 0; i < nw; i++) {
                    const unsigned long long x = row(v, i);
                    if (x) { p = min(v, 64 * i + (uint32_t)__builtin_ctzll(x)); break; }
                }
                W.PAR[v] = p;
                W.CNT[v] = 0;
            }
            __syncthreads();
            STAMP(23);
            // flatten: one barrier per round; round r sets flag r%3 and clears flag (r+1)%3,
            // which every thread last read before the barrier ending round r-1
            for (uint32_t r = 0;; r++) {
                bool changed = false;
                for (uint32_t x = tid; x < V; x += CG_BLOCK) {
                    const uint32_t p = W.PAR[x], pp = W.PAR[p];
                    if (pp != p) { W.PAR[x] = pp; changed = true; }
                }
                if (__ballot(changed) && l == 0) atomicOr(&fs->scal[S_TMP + r % 3], 1u);
                if (tid == 0) fs->scal[S_TMP + (r + 1) % 3] = 0;
                __syncthreads();
                if (!fs->scal[S_TMP + r % 3]) break;
            }
            for (uint32_t v = tid; v < V; v += CG_BLOCK)
                atomicOr(&tm[W.PAR[v] * 4 + (v >> 6)], 1ull << (v & 63));
            __syncthreads();
            STAMP(24);
            for (uint32_t v = tid; v < V; v += CG_BLOCK) {
                const uint32_t rv = W.PAR[v];
                for (uint32_t i = v >> 6; i < nw; i++) {
                    unsigned long long x = row(v, i) & ~tm[rv * 4 + i];
                    if (i == (v >> 6)) x &= ~((2ull << (v & 63)) - 1ull);   // u > v only
                    while (x) {
                        const uint32_t u = 64 * i + (uint32_t)__builtin_ctzll(x);
                        x &= x - 1;
                        uf_union(W.PAR, v, u);
                    }
                }
            }
            __syncthreads();
        } else {
            {   // neighbour-grid origin
                float mn[3] = {INFINITY, INFINITY, INFINITY};
                for (uint32_t v = tid; v < V; v += CG_BLOCK) {
                    const float4 p = W.VOX[v];
                    mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
                }
#pragma unroll
                for (int a = 0; a < 3; a++) mn[a] = wave_min(mn[a]);
                if (l == 0) {
#pragma unroll
                    for (int a = 0; a < 3; a++) red[8 * w + a] = __float_as_uint(mn[a]);
                }
                __syncthreads();
                if (tid == 0) {
                    float o[3] = {INFINITY, INFINITY, INFINITY};
                    for (int q = 0; q < WAVES; q++)
#pragma unroll
                        for (int a = 0; a < 3; a++) o[a] = fminf(o[a], __uint_as_float(red[8 * q + a]));
#pragma unroll
                    for (int a = 0; a < 3; a++) if (!isfinite(o[a])) o[a] = 0.f;
                    fs->scal[S_ORGX] = __float_as_uint(o[0]);
                    fs->scal[S_ORGY] = __float_as_uint(o[1]);
                    fs->scal[S_ORGZ] = __float_as_uint(o[2]);
                }
                __syncthreads();
            }
            const float ox = __uint_as_float(fs->scal[S_ORGX]), oy = __uint_as_float(fs->scal[S_ORGY]),
                        oz = __uint_as_float(fs->scal[S_ORGZ]);
            auto cell = [&](float c, float o) -> uint32_t {
                const float q = floorf((c - o) * P.cell_inv);
                if (!(q >= 0.f)) return 0u;           // NaN or below origin
                return q >= 1023.f ? 1023u : (uint32_t)q;
            };
            auto cell_key = [&](const float4& p) -> uint32_t {
                return (cell(p.z, oz) << 20) | (cell(p.y, oy) << 10) | cell(p.x, ox);
            };
            uint32_t n2 = 1;
            while (n2 < V) n2 <<= 1;
            for (uint32_t j = tid; j < n2; j += CG_BLOCK)
                W.KEY[j] = j < V ? (((uint64_t)cell_key(W.VOX[j]) << 16) | j) : ~0ull;
            __syncthreads();
            bitonic_sort(W.KEY, n2);
            const uint32_t U = block_scan(
                V,
                [&](uint32_t j) -> uint32_t { return (j == 0 || (W.KEY[j] >> 16) != (W.KEY[j - 1] >> 16)) ? 1u : 0u; },
                [&](uint32_t j, uint32_t e) {
                    const uint64_t k = W.KEY[j];
                    W.ORD[j] = (uint32_t)(k & 0xffffu);
                    if (j == 0 || (k >> 16) != (W.KEY[j - 1] >> 16)) { W.UK[e] = (uint32_t)(k >> 16); W.A[e] = j; }
                },
                red);
            if (tid == 0) W.A[U] = V;
            for (uint32_t v = tid; v < V; v += CG_BLOCK) { W.PAR[v] = v; W.CNT[v] = 0; }
            __syncthreads();
            // union over all pairs (v < u) with fl(((dx^2) + dy^2) + dz^2) < r2 (FLANN L2_Simple)
            for (uint32_t v = tid; v < V; v += CG_BLOCK) {
                const float4 q = W.VOX[v];
                const uint32_t cx = cell(q.x, ox), cy = cell(q.y, oy), cz = cell(q.z, oz);
                const uint32_t xlo = cx > 0 ? cx - 1 : 0, xhi = cx < 1023 ? cx + 1 : 1023;
                for (int dz = -1; dz <= 1; dz++) {
                    const int zz = (int)cz + dz;
                    if (zz < 0 || zz > 1023) continue;
                    for (int dy = -1; dy <= 1; dy++) {
                        const int yy = (int)cy + dy;
                        if (yy < 0 || yy > 1023) continue;
                        const uint32_t lo = ((uint32_t)zz << 20) | ((uint32_t)yy << 10) | xlo;
                        const uint32_t hi = ((uint32_t)zz << 20) | ((uint32_t)yy << 10) | xhi;
                        uint32_t a = 0, b = U;
                        while (a < b) {
                            const uint32_t m = (a + b) >> 1;
                            if (W.UK[m] < lo) a = m + 1; else b = m;
                        }
                        for (uint32_t u = a; u < U && W.UK[u] <= hi; u++) {
                            const uint32_t e = W.A[u + 1];
                            for (uint32_t j = W.A[u]; j < e; j++) {
                                const uint32_t o = W.ORD[j];
                                if (o <= v) continue;
                                const float4 p = W.VOX[o];
                                const float ddx = q.x - p.x, ddy = q.y - p.y, ddz = q.z - p.z;
                                float acc = ddx * ddx;
                                acc = acc + ddy * ddy;
                                acc = acc + ddz * ddz;
                                if (acc < P.r2) uf_union(W.PAR, v, o);
                            }
                        }
                    }
                }
            }
            __syncthreads();
        }
        STAMP(12);
        for (uint32_t v = tid; v < V; v += CG_BLOCK) {
            W.LAB[v] = (int32_t)uf_find(W.PAR, v);
            W.ORD[v] = 0xffffffffu;   // becomes root -> output rank
        }
        __syncthreads();
        STAMP(13);
        for (uint32_t v = tid; v < V; v += CG_BLOCK) atomicAdd(&W.CNT[W.LAB[v]], 1u);
        __syncthreads();
        STAMP(14);
        // kept components in discovery (seed) order; DROOT/DSZ/RANK/FIN overlay W.P (dead)
        uint32_t* const DROOT = (uint32_t*)W.P;
        uint32_t* const DSZ = DROOT + V;
        uint32_t* const RANK = DSZ + V;
        uint32_t* const FIN = RANK + V;
        C = block_scan(
            V,
            [&](uint32_t v) -> uint32_t {
                const uint32_t c = W.CNT[v];
                return ((uint32_t)W.LAB[v] == v && c >= P.min_cl && c <= P.max_cl) ? 1u : 0u;
            },
            [&](uint32_t v, uint32_t d) {
                const uint32_t c = W.CNT[v];
                if ((uint32_t)W.LAB[v] == v && c >= P.min_cl && c <= P.max_cl) { DROOT[d] = v; DSZ[d] = c; }
            },
            red);
        STAMP(15);
        // cluster order: PCL sorts the reversed discovery list ascending by size with std::sort
        if (C > CG_SORT_THRESHOLD && C <= 64) {
            // wave 0, records one per lane (cg_sort.h CgWaveRegs64): scalar control flow
            if (tid < 64) {   // sizes <= V < 65536: (size << 16 | d) records in one VGPR
                const uint32_t Cu = (uint32_t)__builtin_amdgcn_readfirstlane((int)C);
                uint32_t r = tid < Cu ? (DSZ[Cu - 1 - tid] << 16) | (Cu - 1 - tid) : 0u;
                cg_std_sort_wave32(r, (int)Cu);
                if (tid < Cu) {
                    FIN[Cu - 1 - tid] = r & 0xffffu;
                    RANK[r & 0xffffu] = Cu - 1 - tid;
                }
            }
        } else if (C > CG_SORT_THRESHOLD) {
            if (tid == 0) {
                uint64_t* rec = W.KEY;
                for (uint32_t i = 0; i < C; i++) {
                    const uint32_t d = C - 1 - i;
                    rec[i] = ((uint64_t)DSZ[d] << 32) | d;
                }
                cg_std_sort(rec, (long)C, [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); }, fs->stk);
                for (uint32_t k = 0; k < C; k++) {
                    const uint32_t d = (uint32_t)rec[C - 1 - k];
                    FIN[k] = d;
                    RANK[d] = k;
                }
            }
        } else {
            // <= 16 clusters: insertion sort is stable, so order = (size desc, seed asc)
            for (uint32_t d = tid; d < C; d += CG_BLOCK) {
                const uint32_t sd = DSZ[d];
                uint32_t r = 0;
                for (uint32_t e = 0; e < C; e++) {
                    const uint32_t se = DSZ[e];
                    r += (se > sd) || (se == sd && e < d);
                }
                RANK[d] = r;
                FIN[r] = d;
            }
        }
        __syncthreads();
        STAMP(16);
        const uint32_t tot = block_scan(
            C, [&](uint32_t k) -> uint32_t { return DSZ[FIN[k]]; },
            [&](uint32_t k, uint32_t e) { W.OFF[k] = e; }, red);
        if (tid == 0) W.OFF[C] = tot;
        for (uint32_t d = tid; d < C; d += CG_BLOCK) W.ORD[DROOT[d]] = RANK[d];
        for (uint32_t k = tid; k < C; k += CG_BLOCK) W.CNT[k] = 0;   // CSR cursors
        __syncthreads();
        STAMP(17);
        int32_t* const lab_out = L.lab + (uint64_t)f * L.cap;
        for (uint32_t v = tid; v < V; v += CG_BLOCK) {
            const int32_t lb = (int32_t)W.ORD[(uint32_t)W.LAB[v]];
            W.LAB[v] = lb;
            lab_out[v] = lb;
        }
        __syncthreads();
        STAMP(18);
        // CSR indices, ascending voxel index inside each cluster
        int32_t* const idx_out = L.idx + (uint64_t)f * L.cap;
        if (V <= CG_BRUTE_V) {
            // rank inside the cluster = popcount of the cluster's membership bits below v;
            // the bitmasks overlay A | PAR | CNT (dead here), 6 words per cluster
            constexpr uint32_t MW = (CG_BRUTE_V + 63) / 64;
            unsigned long long* mask = (unsigned long long*)W.A;
            for (uint32_t x = tid; x < C * MW; x += CG_BLOCK) mask[x] = 0ull;
            __syncthreads();
            for (uint32_t v = tid; v < V; v += CG_BLOCK) {
                const int32_t k = W.LAB[v];
                if (k >= 0) atomicOr(&mask[(uint32_t)k * MW + (v >> 6)], 1ull << (v & 63));
            }
            __syncthreads();
            for (uint32_t v = tid; v < V; v += CG_BLOCK) {
                const int32_t k = W.LAB[v];
                if (k < 0) continue;
                const unsigned long long* mk = mask + (uint32_t)k * MW;
                uint32_t r = (uint32_t)__popcll(mk[v >> 6] & ((1ull << (v & 63)) - 1ull));
                for (uint32_t q = 0; q < (v >> 6); q++) r += (uint32_t)__popcll(mk[q]);
                const uint32_t pos = W.OFF[k] + r;
                W.IDX[pos] = v;
                idx_out[pos] = (int32_t)v;
            }
        } else if (w == 0) {
            // stable counting sort by cluster rank (one wave, ascending v)
            for (uint32_t base = 0; base < V; base += 64) {
                const uint32_t v = base + l;
                const int32_t k = v < V ? W.LAB[v] : -1;
                uint64_t pending = __ballot(k >= 0);
                while (pending) {
                    const uint32_t leader = (uint32_t)__builtin_ctzll(pending);
                    const int32_t kk = __shfl(k, (int)leader, 64);
                    const uint64_t same = __ballot(k == kk) & pending;
                    uint32_t cur = 0;
                    if (l == leader) cur = atomicAdd(&W.CNT[kk], (uint32_t)__popcll(same));
                    cur = __shfl(cur, (int)leader, 64);
                    if (k == kk) {
                        const uint32_t pos = W.OFF[kk] + cur + (uint32_t)__popcll(same & ((1ull << l) - 1ull));
                        W.IDX[pos] = v;
                        idx_out[pos] = (int32_t)v;
                    }
                    pending &= ~same;
                }
            }
        }
        __syncthreads();
        // src/cone_detection.cpp:261-279: xy mean (float, ascending index, starts at 0), then
        // p += p / len * ext with len = float(sqrt((double)x^2 + (double)y^2 + 0))
        float2* const cen_out = L.cen + (uint64_t)f * L.cap;
        int32_t* const off_out = L.offs + (uint64_t)f * (L.cap + 1);
        for (uint32_t k = tid; k < C; k += CG_BLOCK) {
            const uint32_t s = W.OFF[k], e = W.OFF[k + 1];
            float x = 0.0f, y = 0.0f;
            uint32_t i = s;
            for (; i + 8 <= e; i += 8) {   // members fetched eight at a time, summed in order
                uint32_t id[8];
                float2 pv[8];
#pragma unroll
                for (int b = 0; b < 8; b++) id[b] = W.IDX[i + b];
#pragma unroll
                for (int b = 0; b < 8; b++) { const float4 p = W.VOX[id[b]]; pv[b] = make_float2(p.x, p.y); }
#pragma unroll
                for (int b = 0; b < 8; b++) { x += pv[b].x; y += pv[b].y; }
            }
            for (; i < e; i++) {
                const float4 p = W.VOX[W.IDX[i]];
                x += p.x;
                y += p.y;
            }
            const int j = (int)(e - s);
            const float px = x / (float)j, py = y / (float)j;
            const double S = ((double)px * (double)px + (double)py * (double)py) + 0.0;
            const float len = (float)__builtin_sqrt(S);
            const float qx = (float)((double)px + (double)(px / len) * P.ext);
            const float qy = (float)((double)py + (double)(py / len) * P.ext);
            cen_out[k] = make_float2(qx, qy);
        }
        for (uint32_t k = tid; k <= C; k += CG_BLOCK) off_out[k] = (int32_t)W.OFF[k];
    } else if (tid == 0) {
        L.offs[(uint64_t)f * (L.cap + 1)] = 0;
    }
    if (tid == 0) {
        uint32_t* h = L.hdr + (uint64_t)f * 8;
        h[CG_HDR_M] = M;
        h[CG_HDR_V] = V;
        h[CG_HDR_C] = C;
        h[CG_HDR_FLAGS] = flags;
    }
    STAMP(20);
}

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
__global__ __launch_bounds__(CG_BLOCK, 4) void cg_frame_kernel(CgLaunch L, CgDevParams P) {
    constexpr int G = 8;                          // points per load group (double-buffered)
    constexpr int NW = (PPT + 63) / 64;
    static_assert(PPT % (2 * G) == 0, "PPT must be a multiple of two load groups");
    constexpr bool GROUND = KMODE != CG_KMODE_DETECT;
    constexpr bool FILTER = KMODE != CG_KMODE_GROUND;
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
    FrontShared* fs = (FrontShared*)smem;
    BackLds* bl = (BackLds*)(smem + FRONT_BYTES);
    uint8_t* zq = (uint8_t*)bl;                   // z codes, [k/8][lane][k%8]

    const uint32_t f = SPLIT ? 0u : blockIdx.x, tid = threadIdx.x, l = lane_id(), w = wave_id();
    const uint8_t* fb = L.in + (uint64_t)f * L.frame_stride;
    const uint32_t N = L.n_points;
    STAMP(0);
    if (L.span && tid == 0) atomicMin(&L.span[0], (unsigned long long)__builtin_amdgcn_s_memrealtime());

    if (tid <= CG_NUM_BINS) fs->sec_key[tid] = cg_fkey(P.default_low);
    init_rays<FILTER>(P, fs->rays, tid);
    if (tid < 64) fs->scal[tid] = (tid >= S_BMIN0 && tid <= S_BMIN2) ? 0xffffffffu : 0u;
    __syncthreads();

    // ---- pass 1: stream the frame ----
    LaneBits<NW> posm;
    uint32_t touched = 0;
    uint2* const sp_codes = SPLIT ? (uint2*)(L.split + CG_SPLIT_CODES) : nullptr;
    if constexpr (SPLIT) {
        static_assert(PPT * CG_BLOCK == CG_MAX_POINTS, "split frames use the 64k tail");
        static_assert(CG_SPLIT_CHUNK == 8 * CG_BLOCK, "a chunk's codes are one uint2 and its bits one byte per lane");
        const uint32_t c = blockIdx.x, c0 = c * CG_SPLIT_CHUNK;
        const uint32_t Nc = N > c0 ? min((uint32_t)CG_SPLIT_CHUNK, N - c0) : 0u;
        if (L.in_host) {   // the chunk over PCIe from pinned host memory into the device copy
            const uint64_t b0 = (uint64_t)c0 * L.point_step, nb = (uint64_t)Nc * L.point_step;
            uint8_t* dst = (uint8_t*)L.in + b0;
            const uint8_t* src = L.in_host + b0;
            const uint64_t n16 = nb / 16;
            // four 16-byte reads in flight per lane; named registers (an array with
            // conditional elements was kept in scratch)
            const uint4* s4 = (const uint4*)src;
            uint4* d4 = (uint4*)dst;
            for (uint64_t i = tid; i < n16; i += CG_BLOCK * 4) {
                const uint64_t i1 = i + CG_BLOCK, i2 = i + 2 * CG_BLOCK, i3 = i + 3 * CG_BLOCK;
                const uint4 v0 = s4[i];
                const uint4 v1 = s4[i1 < n16 ? i1 : i];
                const uint4 v2 = s4[i2 < n16 ? i2 : i];
                const uint4 v3 = s4[i3 < n16 ? i3 : i];
                d4[i] = v0;
                if (i1 < n16) d4[i1] = v1;
                if (i2 < n16) d4[i2] = v2;
                if (i3 < n16) d4[i3] = v3;
            }
            for (uint64_t i = n16 * 16 + 4 * (uint64_t)tid; i < nb; i += 4 * CG_BLOCK)
                *(uint32_t*)(dst + i) = *(const uint32_t*)(src + i);
            __threadfence();
            __syncthreads();
        }
        LaneBits<1> pm;
        uint2 code = make_uint2(0u, 0u);
        stream_pass1<CG_SPLIT_CHUNK / CG_BLOCK, LAYOUT, GROUND, FILTER>(
            fb + (uint64_t)c0 * L.point_step, Nc, L, P, fs->sec_key, fs->rays, pm, touched,
            [&](int, uint2 cw) { code = cw; });
        sp_codes[c * CG_BLOCK + tid] = code;
        ((uint8_t*)(L.split + CG_SPLIT_POSM))[c * CG_BLOCK + tid] = (uint8_t)pm.w[0];
        if (GROUND) {
            touched = wave_or(touched);
            if (l == 0 && touched) atomicOr(L.split + 1, touched);
        }
        __syncthreads();   // the chunk's sector minima are final in LDS
        if (GROUND && tid <= CG_NUM_BINS) atomicMin(L.split + 2 + tid, fs->sec_key[tid]);
        __threadfence();
        __syncthreads();
        if (tid == 0)
            fs->scal[S_LAST] = __hip_atomic_fetch_add(L.split, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
                               gridDim.x - 1;
        __syncthreads();
        if (!fs->scal[S_LAST]) return;
        __threadfence();
        // the last workgroup: the frame's sector keys and used bins (state reset for the next
        // frame), every lane's filter bits over the chunks
        if (GROUND && tid <= CG_NUM_BINS) fs->sec_key[tid] = atomicExch(L.split + 2 + tid, 0xffffffffu);
        if (tid == 0) {
            fs->scal[S_TOUCHED] = GROUND ? atomicExch(L.split + 1, 0u) : 0u;
            atomicExch(L.split, 0u);
        }
        posm.clear();
        const uint8_t* pb = (const uint8_t*)(L.split + CG_SPLIT_POSM);
        const uint32_t nch = (N + CG_SPLIT_CHUNK - 1) / CG_SPLIT_CHUNK;
#pragma unroll
        for (int cc = 0; cc < PPT / 8; cc++)
            if ((uint32_t)cc < nch) posm.set_byte(cc, pb[cc * CG_BLOCK + tid]);
        __syncthreads();
    } else {
#ifdef CG_CODES_HBM
        uint2* const zc = (uint2*)(L.scratch + (uint64_t)f * L.scratch_stride);
        auto store = [&](int g, uint2 c) { zc[g * CG_BLOCK + tid] = c; };
#else
        auto store = [&](int g, uint2 c) { ((uint2*)zq)[g * CG_BLOCK + tid] = c; };
#endif
        if (LAYOUT == CG_LAYOUT_XYZI16 && N == (uint32_t)(PPT * CG_BLOCK))   // whole groups only
            stream_pass1<PPT, LAYOUT, GROUND, FILTER, decltype(store), true>(fb, N, L, P, fs->sec_key, fs->rays,
                                                                          posm, touched, store);
        else
            stream_pass1<PPT, LAYOUT, GROUND, FILTER>(fb, N, L, P, fs->sec_key, fs->rays, posm, touched, store);
    }
    const uint32_t nlast = N ? N - 1 : 0u;
    if (GROUND && !SPLIT) {
        touched = wave_or(touched);
        if (l == 0) atomicOr(&fs->scal[S_TOUCHED], touched);
    }
    // the lane's first CG_PREFETCH filter survivors are the likely first gather loads: issue them now,
    // they land while the thresholds and pass 2 run (a survivor that turns out to be ground
    // costs one wasted load)
    int pk[CG_PREFETCH];
    float4 pv[CG_PREFETCH];
#pragma unroll
    for (int q = 0; q < CG_PREFETCH; q++) pk[q] = -1;
    if (FILTER) {
#pragma unroll
        for (int wi = 0; wi < NW; wi++) {
            uint64_t m = posm.w[wi];
#pragma unroll
            for (int q = 0; q < CG_PREFETCH; q++)
                if (pk[q] < 0 && m) { pk[q] = 64 * wi + __builtin_ctzll(m); m &= m - 1; }
        }
#pragma unroll
        for (int q = 0; q < CG_PREFETCH; q++)
            pv[q] = load_xyzi<LAYOUT>(fb, min((uint32_t)(pk[q] < 0 ? 0 : pk[q]) * CG_BLOCK + tid, nlast), L);
    }
    __syncthreads();
    STAMP(1);

#if defined(CG_EXP_STOP) && CG_EXP_STOP == 1
    if (tid == 0) { uint32_t* h = L.hdr + (uint64_t)f * 8; h[0] = N; h[1] = h[2] = h[3] = h[4] = h[5] = 0; }
    if (L.span && tid == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    return;
#endif
    if (GROUND && tid < 64) {
        sector_thresholds(fs->sec_key, fs->scal[S_TOUCHED], P, fs->thr, fs->tkey, &fs->scal[S_TKMIN], &fs->scal[S_TKMAX]);
        if (L.seckeys && tid <= CG_NUM_BINS) L.seckeys[(uint64_t)f * (CG_NUM_BINS + 1) + tid] = fs->sec_key[tid];
    }
    __syncthreads();
    STAMP(2);

    // ---- pass 2: ground decisions from the LDS codes ----
    LaneBits<NW> keepgm;
    keepgm.clear();
    if (GROUND) {
        pass2_keep<PPT, LAYOUT>(fb, N, L, P, fs->scal[S_TKMIN], fs->scal[S_TKMAX], fs->tkey,
                                [&](int g) {
#ifdef CG_CODES_HBM
                                    return SPLIT ? sp_codes[g * CG_BLOCK + tid]
                                                 : ((const uint2*)(L.scratch + (uint64_t)f * L.scratch_stride))[g * CG_BLOCK + tid];
#else
                                    return SPLIT ? sp_codes[g * CG_BLOCK + tid] : ((const uint2*)zq)[g * CG_BLOCK + tid];
#endif
                                }, keepgm);
        const uint32_t kc = wave_sum(keepgm.count());
        if (l == 0) atomicAdd(&fs->scal[S_K], kc);
    } else {
#pragma unroll
        for (int k = 0; k < PPT; k++)
            if ((uint32_t)k * CG_BLOCK + tid < N) keepgm.w[k >> 6] |= 1ull << (k & 63);
    }
    STAMP(22);

    if (KMODE == CG_KMODE_GROUND) {
        // groundless cloud: K kept points in point order, then N-K PointXYZI()
        // (ground_removal.cpp:70-79); stable order comes from per-(k, wave) ballot counts
#pragma unroll 8
        for (int k = 0; k < PPT; k++) {
            const uint64_t bb = __ballot(keepgm.get(k));
            if (l == 0) fs->cnt[k * WAVES + w] = (uint32_t)__popcll(bb);
        }
        __syncthreads();
        STAMP(3);
        const uint32_t Kc = block_scan(
            PPT * WAVES, [&](uint32_t i) -> uint32_t { return fs->cnt[i]; },
            [&](uint32_t i, uint32_t e) { fs->cnt[i] = e; }, fs->red);
        STAMP(4);
        float4* out = (float4*)(L.ground + (uint64_t)f * N * 32);
#pragma unroll 4
        for (int k = 0; k < PPT; k++) {
            const bool kp = keepgm.get(k);
            const uint64_t bb = __ballot(kp);
            if (kp) {
                const uint32_t i = (uint32_t)k * CG_BLOCK + tid;
                const uint32_t dst = fs->cnt[k * WAVES + w] + (uint32_t)__popcll(bb & ((1ull << l) - 1ull));
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

    // ---- compaction: per-wave atomic append; each survivor carries its point index, and
    // the voxel sort orders by (voxel idx, point index), so append order does not matter ----
    LaneBits<NW> keepm;
#pragma unroll
    for (int i = 0; i < NW; i++) keepm.w[i] = FILTER ? (keepgm.w[i] & posm.w[i]) : keepgm.w[i];
    const uint32_t nsv = keepm.count();
    const uint32_t incl = wave_incl_scan(nsv);
    uint32_t wbase = 0;
    if (l == 63) wbase = atomicAdd(&fs->scal[S_MS], incl);
    wbase = (uint32_t)__builtin_amdgcn_readlane((int)wbase, 63);
    uint32_t pos = wbase + incl - nsv;
    __syncthreads();   // counts complete; z-code overlay in LDS is dead from here on
    STAMP(3);

#if defined(CG_EXP_STOP) && CG_EXP_STOP == 2
    if (tid == 0) { uint32_t* h = L.hdr + (uint64_t)f * 8; h[0] = N; h[1] = h[2] = h[3] = h[4] = h[5] = 0; }
    if (L.span && tid == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    return;
#endif
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
    STAMP(4);
    Work W;
    if (use_lds) {
        W.P = bl->P; W.KEY = bl->KEY; W.VOX = bl->VOX; W.A = bl->A; W.PAR = bl->PAR; W.CNT = bl->CNT;
        W.UK = bl->UK; W.LAB = bl->LAB; W.ORD = bl->ORD; W.IDX = bl->IDX; W.OFF = bl->OFF;
    } else {
        W = global_work(L.scratch + (uint64_t)f * L.scratch_stride, N);
    }
    // ---- gather survivors (4 loads in flight per lane) and the VoxelGrid bounds ----
    float mn[3] = {INFINITY, INFINITY, INFINITY}, mx[3] = {-INFINITY, -INFINITY, -INFINITY};
    uint32_t nfin = 0;
    auto bound = [&](const float4& p) {
        if (isfinite(p.x) && isfinite(p.y) && isfinite(p.z)) {
            mn[0] = fminf(mn[0], p.x); mn[1] = fminf(mn[1], p.y); mn[2] = fminf(mn[2], p.z);
            mx[0] = fmaxf(mx[0], p.x); mx[1] = fmaxf(mx[1], p.y); mx[2] = fmaxf(mx[2], p.z);
            nfin++;
        }
    };
#pragma unroll
    for (int q = 0; q < CG_PREFETCH; q++) {
        if (pk[q] >= 0 && keepm.get(pk[q])) {
            keepm.clear_bit(pk[q]);
            W.P[pos] = pv[q];
            W.IDX[pos] = (uint32_t)pk[q] * CG_BLOCK + tid;
            bound(pv[q]);
            pos++;
        }
    }
#pragma unroll
    for (int wi = 0; wi < NW; wi++) {
        uint64_t m = keepm.w[wi];
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
                if (ks[q] >= 0) pt[q] = load_xyzi<LAYOUT>(fb, (uint32_t)(64 * wi + ks[q]) * CG_BLOCK + tid, L);
#pragma unroll
            for (int q = 0; q < 4; q++) {
                if (ks[q] < 0) continue;
                W.P[pos] = pt[q];
                W.IDX[pos] = (uint32_t)(64 * wi + ks[q]) * CG_BLOCK + tid;   // point index
                bound(pt[q]);
                pos++;
            }
        }
    }
    STAMP(25);
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

#if defined(CG_EXP_STOP) && CG_EXP_STOP == 3
    if (tid == 0) { uint32_t* h = L.hdr + (uint64_t)f * 8; h[0] = N; h[1] = h[2] = h[3] = h[4] = h[5] = 0; }
    if (L.span && tid == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
    return;
#endif
    if (use_lds) {
        Work WL;
        WL.P = bl->P; WL.KEY = bl->KEY; WL.VOX = bl->VOX; WL.A = bl->A; WL.PAR = bl->PAR; WL.CNT = bl->CNT;
        WL.UK = bl->UK; WL.LAB = bl->LAB; WL.ORD = bl->ORD; WL.IDX = bl->IDX; WL.OFF = bl->OFF;
        backend(WL, M, fs, L, P, f, flags);
    } else {
        backend(W, M, fs, L, P, f, flags);
    }
    if constexpr (SPLIT) {   // the results packed for the host's one copy (fetch_frame)
        if (L.pack) {
            __threadfence();
            __syncthreads();
            pack_frame(L, f, L.pack);
        }
    }
    if (L.span && tid == 0) atomicMax(&L.span[1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
}

// ------------------------------------------------------------------------------------------
// Large frames whose detector input fits the LDS path (M <= CG_MMAX): the survivors come from
// HBM in append order; sorted by frame index they get ranks as point indices, so the voxel
// keys order ties exactly as the frame kernel does. npad PointXYZI() pads follow.
__global__ __launch_bounds__(CG_BLOCK, 2) void cg_lg_back_small(CgLaunch L, CgDevParams P, LgScratch S,
                                                                uint32_t f, uint32_t npad, uint32_t K) {
    __shared__ __attribute__((aligned(16))) unsigned char smem[SMEM_BYTES];
    FrontShared* fs = (FrontShared*)smem;
    BackLds* bl = (BackLds*)(smem + FRONT_BYTES);
    const uint32_t tid = threadIdx.x;
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
    backend(W, M, fs, L, P, f, 0u);
}
int cg_launch_lg_back_small(const CgLaunch& L, const CgDevParams& P, const LgScratch& S, uint32_t f,
                            uint32_t npad, uint32_t K, hipStream_t s) {
    hipLaunchKernelGGL(cg_lg_back_small, dim3(1), dim3(CG_BLOCK), 0, s, L, P, S, f, npad, K);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Launchers.
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
        if (xyzi16) hipLaunchKernelGGL((cg_frame_kernel<PPT, CG_LAYOUT_XYZI16, CG_KMODE_PIPELINE, true>), grid, block, 0, s, L, P);
        else hipLaunchKernelGGL((cg_frame_kernel<PPT, CG_LAYOUT_GENERIC, CG_KMODE_PIPELINE, true>), grid, block, 0, s, L, P);
    } else {
        if (xyzi16) hipLaunchKernelGGL((cg_frame_kernel<PPT, CG_LAYOUT_XYZI16, CG_KMODE_DETECT, true>), grid, block, 0, s, L, P);
        else hipLaunchKernelGGL((cg_frame_kernel<PPT, CG_LAYOUT_GENERIC, CG_KMODE_DETECT, true>), grid, block, 0, s, L, P);
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
    const uint32_t nt = blockDim.x;
    const uint32_t* hdr = L.hdr + (uint64_t)f * CG_HDR_WORDS;
    const uint32_t V = min(hdr[CG_HDR_V], (uint32_t)CG_PACK_MAX), C = min(hdr[CG_HDR_C], (uint32_t)CG_PACK_MAX);
    const int32_t* offs = L.offs + (uint64_t)f * (L.cap + 1);
    const uint32_t nidx = min(C ? (uint32_t)offs[C] : 0u, (uint32_t)CG_PACK_MAX);
    const float4* vox = L.vox + (uint64_t)f * L.cap;
    const int32_t* lab = L.lab + (uint64_t)f * L.cap;
    const int32_t* idx = L.idx + (uint64_t)f * L.cap;
    const float2* cen = L.cen + (uint64_t)f * L.cap;
    for (uint32_t i = threadIdx.x; i < CG_HDR_WORDS; i += nt) out[i] = hdr[i];
    for (uint32_t i = threadIdx.x; i < V; i += nt) {
        const float4 p = vox[i];
        uint32_t* q = out + CG_PACK_VOX + 4 * i;
        q[0] = __float_as_uint(p.x); q[1] = __float_as_uint(p.y); q[2] = __float_as_uint(p.z); q[3] = __float_as_uint(p.w);
        out[CG_PACK_LAB + i] = (uint32_t)lab[i];
    }
    for (uint32_t i = threadIdx.x; i <= C; i += nt) out[CG_PACK_OFFS + i] = (uint32_t)offs[i];
    for (uint32_t i = threadIdx.x; i < nidx; i += nt) out[CG_PACK_IDX + i] = (uint32_t)idx[i];
    for (uint32_t i = threadIdx.x; i < C; i += nt) {
        out[CG_PACK_CEN + 2 * i] = __float_as_uint(cen[i].x);
        out[CG_PACK_CEN + 2 * i + 1] = __float_as_uint(cen[i].y);
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
