// cg_backend.h — the frame backend (VoxelGrid, Euclidean clustering, cluster order, CSR,
// centroids) for one frame's detector points, in one 512-lane workgroup: the fused frame kernel
// and the large path's LDS backend (cg_kernels.hip).
#pragma once
#include <hip/hip_runtime.h>
#include "cg_internal.h"
#include "../../include/cones_gpu.h"
#include "cg_math.h"
#include "cg_sort.h"
#include "cg_device.h"
#include "cg_pcl.h"

#ifndef CG_BRUTE_V
#define CG_BRUTE_V 256        // voxel count up to which clustering tests all pairs
#endif

// ------------------------------------------------------------------------------------------
// LDS map. The frontend's 16-bit z-key prefixes (zq) overlay the backend arrays, which are
// dead until pass 3 begins; pass 2 leaves its decisions in registers.
struct FrontShared {
    float4 rays[CG_NUM_BINS];      // sector edge rays of the pass-1 fast path
    uint32_t sec_key[CG_NUM_BINS + 1];
    float thr[CG_NUM_BINS + 1];
    uint32_t tkey[CG_NUM_BINS + 1];
    uint32_t red[8 * WAVES];       // wave partials
    uint32_t scal[64];             // broadcast scalars
};
#define FRONT_BYTES ((sizeof(FrontShared) + 255) & ~(size_t)255)

// The backend's arrays in LDS for up to CAP detector points (the frame kernel: CG_MMAX).
constexpr uint32_t cg_pow2_ceil(uint32_t n) { uint32_t p = 1; while (p < n) p <<= 1; return p; }
template <uint32_t CAP>
struct BackLdsT {
    float4 P[CAP];
    uint64_t KEY[cg_pow2_ceil(CAP)];   // bitonic sorts of up to CAP keys run over the next power of two
    float4 VOX[CAP];
    uint32_t A[CAP + 4];
    uint32_t PAR[CAP];
    uint32_t CNT[CAP];
    uint32_t UK[CAP];
    int32_t LAB[CAP];
    uint32_t ORD[CAP];
    uint32_t IDX[CAP];
    uint32_t OFF[CAP + 4];
};
// What the backend overlays on its LDS arrays, for a capacity of CAP points (V <= M <= CAP):
// the brute-force adjacency rows (V x 32 B) on KEY and the tree masks (V x 32 B) on P; the CSR
// membership masks (C x ceil(CG_BRUTE_V / 64) words, C <= V) on A | PAR | CNT; the cluster
// order's introsort stack on UK; pcl_index_vector's bitmap (2 x nbw words) and the
// out-of-place sort buffer (E + CAP) in VOX. Every instantiation is checked with this.
template <uint32_t CAP, uint32_t NBW>
constexpr bool backend_lds_fits() {
    constexpr uint32_t bv = CG_BRUTE_V < CAP ? CG_BRUTE_V : CAP;
    return bv * 32 <= sizeof(BackLdsT<CAP>::KEY) && bv * 32 <= sizeof(BackLdsT<CAP>::P) &&
           bv * ((CG_BRUTE_V + 63) / 64) * 8 <= sizeof(BackLdsT<CAP>::A) + sizeof(BackLdsT<CAP>::PAR) + sizeof(BackLdsT<CAP>::CNT) &&
           3 * CG_SORT_STACK <= CAP && 2 * NBW <= 4 * CAP && 2 * CAP * 8 <= sizeof(BackLdsT<CAP>::VOX) &&
           cg_pow2_ceil(CAP) <= sizeof(BackLdsT<CAP>::KEY) / 8;
}
template <uint32_t CAP>
__device__ __forceinline__ Work lds_work(BackLdsT<CAP>* bl) {
    Work W;
    W.P = bl->P; W.KEY = bl->KEY; W.VOX = bl->VOX; W.A = bl->A; W.PAR = bl->PAR; W.CNT = bl->CNT;
    W.UK = bl->UK; W.LAB = bl->LAB; W.ORD = bl->ORD; W.IDX = bl->IDX; W.OFF = bl->OFF;
    return W;
}


// Scalar slots in FrontShared::scal
enum {
    S_K = 0, S_MS, S_M, S_MF, S_V, S_C, S_U, S_FLAGS, S_PASS,
    S_MINB0, S_MINB1, S_MINB2, S_MUL1, S_MUL2,
    S_ORGX, S_ORGY, S_ORGZ, S_TKMIN, S_TKMAX, S_TOUCHED,
    S_BMIN0, S_BMIN1, S_BMIN2, S_BMAX0, S_BMAX1, S_BMAX2, S_TMP, S_LAST,
    S_ERR = 40   // (the backend's flatten rounds use S_TMP .. S_TMP + 2)
};



// The backend's arrays in a frame's HBM scratch slot (M > the LDS capacity), sized for n
// points; cg_work_bytes(n) bytes.
__host__ __device__ inline uint64_t cg_work_bytes(uint32_t n) {
    uint64_t n2 = 1; while (n2 < n) n2 <<= 1;
    const uint64_t c = (uint64_t)n + 4;
    return 16 * c + 16 * c + 8 * n2 + 4 * c * 8;
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
// nbw: words of pcl_index_vector's bitmap, which covers every kept survivor's W.IDX (2,048
// for point indices of a 64k frame; fewer when W.IDX holds ranks).
// lds_cap: the LDS capacity when W is in LDS (the out-of-place sort buffer starts at VOX's
// second half, E + lds_cap).
__device__ __forceinline__ void backend(const Work& W, uint32_t M, FrontShared* fs, const CgLaunch& L,
                                        const CgDevParams& P, uint32_t f, uint32_t flags, uint32_t nbw,
                                        uint32_t lds_cap) {
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
            pcl_index_vector(W, M, fs->scal[S_MS], E, red, nbw, [&](uint32_t j) -> uint32_t { return voxel_idx(W.P[j]); });
            STAMP(7);
            if (flags & CG_F_GLOBAL_SCRATCH) pcl_sort<2, false>(W, E, Mf, red);
            else pcl_sort<2, true>(W, E, Mf, red, -1, E + lds_cap);   // VOX's upper half: swaps out of place
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
                // the introsort stack in W.UK (dead since the clustering; >= 3 * CG_SORT_STACK words
                // whenever C > 64: UK holds at least M >= V >= C entries, M being <= its capacity)
                cg_std_sort(rec, (long)C, [](uint64_t a, uint64_t b) { return (a >> 32) < (b >> 32); }, (int32_t*)W.UK);
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
        h[CG_HDR_ERR] = 0u;   // (a split launch overwrites it after the backend)
    }
    STAMP(20);
}


