// cg_device.h — device building blocks shared by the frame kernel (cg_kernels.hip) and the
// large-frame path (cg_large.hip): wave primitives, block scan and sorts, union-find, point
// loads, the certified classification of pass 1, the z codes and the pass-1 stream itself.
#pragma once
#include <hip/hip_runtime.h>
#include "cg_internal.h"
#include "cg_math.h"

#define WAVES (CG_BLOCK / 64)

// Diagnostic phase stamps (s_memrealtime by lane 0 of each workgroup), only when L.stamps != 0.
#define STAMP(ph)                                                                          \
    do {                                                                                   \
        if (L.stamps && threadIdx.x == 0)                                                  \
            L.stamps[(uint64_t)blockIdx.x * 32 + (ph)] = __builtin_amdgcn_s_memrealtime();     \
    } while (0)

// ------------------------------------------------------------------------------------------
// Wave / block primitives (wave = 64 lanes).
__device__ __forceinline__ uint32_t lane_id() { return threadIdx.x & 63; }
__device__ __forceinline__ uint32_t wave_id() { return threadIdx.x >> 6; }
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}
// Cross-lane steps use DPP (row_shr within 16-lane rows, row_bcast15/31 across rows), which
// stay in the VALU; __shfl would go through ds_bpermute and pay an LDS round trip per step.
// v = 2v + bit: per-point decisions packed into per-lane bit strings, first point in the
// highest bit (bit-reversed once per group by the callers). Plain C on purpose: a hand-written
// v_addc_co_u32 taking the compare mask as carry-in was faster, but gfx950 needs wait states
// between a VALU write of a lane mask and a VALU read of it (the compiler pads its own code
// with s_nop), and inline assembly is invisible to the hazard recognizer, so it read stale
// masks under some schedules.
__device__ __forceinline__ uint32_t shl1_add_if(uint32_t v, bool b) { return v + v + (uint32_t)b; }

template <int CTRL, int ROWS, int BANKS>
__device__ __forceinline__ uint32_t dpp(uint32_t identity, uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)identity, (int)v, CTRL, ROWS, BANKS, false);
}
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    uint32_t v = x;
    v += dpp<0x111, 0xf, 0xf>(0u, x);    // row_shr:1
    v += dpp<0x112, 0xf, 0xf>(0u, x);    // row_shr:2
    v += dpp<0x113, 0xf, 0xf>(0u, x);    // row_shr:3   -> sums of 4
    v += dpp<0x114, 0xf, 0xe>(0u, v);    // row_shr:4, banks 1-3 -> 8
    v += dpp<0x118, 0xf, 0xc>(0u, v);    // row_shr:8, banks 2-3 -> 16
    v += dpp<0x142, 0xa, 0xf>(0u, v);    // row_bcast:15 into rows 1, 3
    v += dpp<0x143, 0xc, 0xf>(0u, v);    // row_bcast:31 into rows 2, 3
    return v;
}
// Reductions to lane 63 (Kogge-Stone in each row, then the two row broadcasts), read back
// through an SGPR so every lane gets the result.
template <class OP>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t v, uint32_t id, OP op) {
    v = op(v, dpp<0x111, 0xf, 0xf>(id, v));
    v = op(v, dpp<0x112, 0xf, 0xf>(id, v));
    v = op(v, dpp<0x114, 0xf, 0xf>(id, v));
    v = op(v, dpp<0x118, 0xf, 0xf>(id, v));
    v = op(v, dpp<0x142, 0xa, 0xf>(id, v));
    v = op(v, dpp<0x143, 0xc, 0xf>(id, v));
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ __forceinline__ float wave_min(float v) {
    return __uint_as_float(wave_reduce(__float_as_uint(v), __float_as_uint(INFINITY), [](uint32_t a, uint32_t b) {
        return __float_as_uint(fminf(__uint_as_float(a), __uint_as_float(b)));
    }));
}
__device__ __forceinline__ float wave_max(float v) {
    return __uint_as_float(wave_reduce(__float_as_uint(v), __float_as_uint(-INFINITY), [](uint32_t a, uint32_t b) {
        return __float_as_uint(fmaxf(__uint_as_float(a), __uint_as_float(b)));
    }));
}
__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
    return wave_reduce(v, 0u, [](uint32_t a, uint32_t b) { return a + b; });
}
__device__ __forceinline__ uint32_t wave_or(uint32_t v) {
    return wave_reduce(v, 0u, [](uint32_t a, uint32_t b) { return a | b; });
}
__device__ __forceinline__ uint32_t wave_umin(uint32_t v) {
    return wave_reduce(v, 0xffffffffu, [](uint32_t a, uint32_t b) { return a < b ? a : b; });
}
__device__ __forceinline__ uint32_t wave_umax(uint32_t v) {
    return wave_reduce(v, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
}

// Exclusive scan over i in [0, n) in chunks of 1024: val(i) -> emit(i, excl). Returns total.
// Every thread of the block must call it.
template <class FV, class FE>
__device__ __forceinline__ uint32_t block_scan(uint32_t n, FV val, FE emit, uint32_t* red) {
    uint32_t carry = 0;
    const uint32_t l = lane_id(), w = wave_id();
    for (uint32_t base = 0; base < n; base += CG_BLOCK) {
        const uint32_t i = base + threadIdx.x;
        const uint32_t v = i < n ? val(i) : 0u;
        const uint32_t inc = wave_incl_scan(v);
        if (l == 63) red[w] = inc;
        __syncthreads();
        if (w == 0) {
            uint32_t t = l < WAVES ? red[l] : 0u;
            uint32_t ti = wave_incl_scan(t);
            if (l < WAVES) red[WAVES + l] = ti - t;
            if (l == WAVES - 1) red[2 * WAVES] = ti;
        }
        __syncthreads();
        if (i < n) emit(i, carry + red[WAVES + w] + inc - v);
        const uint32_t tot = red[2 * WAVES];
        __syncthreads();
        carry += tot;
    }
    return carry;
}

// Ascending bitonic sort of S[0, n2), n2 a power of two.
__device__ __forceinline__ void bitonic_sort(uint64_t* S, uint32_t n2) {
    for (uint32_t k = 2; k <= n2; k <<= 1)
        for (uint32_t j = k >> 1; j > 0; j >>= 1) {
            for (uint32_t t = threadIdx.x; t < (n2 >> 1); t += CG_BLOCK) {
                const uint32_t l = 2 * t - (t & (j - 1)), r = l + j;
                const bool up = (l & k) == 0;
                const uint64_t a = S[l], b = S[r];
                if ((a > b) == up) { S[l] = b; S[r] = a; }
            }
            __syncthreads();
        }
}

// Sort n <= CG_RANK_SORT_MAX distinct keys: out[rank(in[j])] = in[j], rank by a broadcast
// sweep (every lane reads the same in[i]). Ends with a barrier.
#define CG_RANK_SORT_MAX 512
__device__ __forceinline__ void rank_sort(const uint64_t* in, uint64_t* out, uint32_t n) {
    // g lanes (a power of two, consecutive in a wave) share one key's count, each over a
    // contiguous slice read as 16-byte pairs, eight keys in flight
    uint32_t g = 1;
    while (g < 64 && (uint64_t)n * g * 2 <= CG_BLOCK) g <<= 1;
    const uint32_t sub = threadIdx.x & (g - 1);
    const uint32_t per = ((n + g - 1) / g + 1) & ~1u;   // even: slices start 16-byte aligned
    const ulonglong2* in2 = (const ulonglong2*)in;
    for (uint32_t base = 0; base < n * g; base += CG_BLOCK) {
        const uint32_t t = base + threadIdx.x, j = t / g;
        const uint64_t kj = j < n ? in[j] : 0ull;
        uint32_t r = 0;
        if (j < n) {
            const uint32_t lo = min(n, sub * per), hi = min(n, lo + per);
            uint32_t i = lo;
            for (; i + 8 <= hi; i += 8) {
                const ulonglong2 a = in2[i / 2], b = in2[i / 2 + 1], c = in2[i / 2 + 2], d = in2[i / 2 + 3];
                r += (a.x < kj) + (a.y < kj) + (b.x < kj) + (b.y < kj) + (c.x < kj) + (c.y < kj) +
                     (d.x < kj) + (d.y < kj);
            }
            for (; i < hi; i++) r += in[i] < kj;
        }
        for (uint32_t o = 1; o < g; o <<= 1) r += (uint32_t)__shfl_xor((int)r, (int)o, 64);
        if (j < n && sub == 0) out[r] = kj;
    }
    __syncthreads();
}

__device__ __forceinline__ uint32_t ld_rlx(uint32_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(uint32_t* p, uint32_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st64(uint64_t* p, uint64_t v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld64(uint64_t* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// float4 records through device-coherent 64-bit halves (visible to workgroups on other XCDs
// without an L2 writeback)
__device__ __forceinline__ void st_f4(float4* p, float4 v) {
    st64((uint64_t*)p, ((uint64_t)__float_as_uint(v.y) << 32) | __float_as_uint(v.x));
    st64((uint64_t*)p + 1, ((uint64_t)__float_as_uint(v.w) << 32) | __float_as_uint(v.z));
}
__device__ __forceinline__ float4 ld_f4(const float4* p) {
    const uint64_t a = ld64((uint64_t*)p), b = ld64((uint64_t*)p + 1);
    return make_float4(__uint_as_float((uint32_t)a), __uint_as_float((uint32_t)(a >> 32)),
                       __uint_as_float((uint32_t)b), __uint_as_float((uint32_t)(b >> 32)));
}
// Union-find with path halving; roots only ever point to smaller indices.
__device__ __forceinline__ uint32_t uf_find(uint32_t* par, uint32_t x) {
    while (true) {
        uint32_t p = ld_rlx(par + x);
        if (p == x) return x;
        uint32_t gp = ld_rlx(par + p);
        if (gp == p) return p;
        st_rlx(par + x, gp);
        x = gp;
    }
}
__device__ __forceinline__ void uf_union(uint32_t* par, uint32_t a, uint32_t b) {
    while (true) {
        a = uf_find(par, a);
        b = uf_find(par, b);
        if (a == b) return;
        if (a > b) { uint32_t t = a; a = b; b = t; }
        if (atomicCAS(par + b, b, a) == b) return;
    }
}

// ------------------------------------------------------------------------------------------
// Point access.
template <int LAYOUT>
__device__ __forceinline__ void load_xyz(const uint8_t* fb, uint32_t i, const CgLaunch& L,
                                         float& x, float& y, float& z) {
    if (LAYOUT == CG_LAYOUT_XYZI16) {
        const float4 v = *(const float4*)(fb + (uint64_t)i * 16);
        x = v.x; y = v.y; z = v.z;
    } else if (LAYOUT == CG_LAYOUT_PCL32) {
        const float4 v = *(const float4*)(fb + (uint64_t)i * 32);
        x = v.x; y = v.y; z = v.z;
    } else {
        const uint8_t* p = fb + (uint64_t)i * L.point_step;
        x = L.off_x >= 0 ? *(const float*)(p + L.off_x) : 0.f;
        y = L.off_y >= 0 ? *(const float*)(p + L.off_y) : 0.f;
        z = L.off_z >= 0 ? *(const float*)(p + L.off_z) : 0.f;
    }
}
template <int LAYOUT>
__device__ __forceinline__ float3 load_xyz3(const uint8_t* fb, uint32_t i, const CgLaunch& L) {
    if (LAYOUT == CG_LAYOUT_XYZI16) return *(const float3*)(fb + (uint64_t)i * 16);
    if (LAYOUT == CG_LAYOUT_PCL32) return *(const float3*)(fb + (uint64_t)i * 32);
    float x, y, z;
    load_xyz<CG_LAYOUT_GENERIC>(fb, i, L, x, y, z);
    return make_float3(x, y, z);
}
// Order-preserving key with -0 folded onto +0 and every NaN onto one key above +inf, so
// that for non-NaN T:  z < T  <=>  cg_zkey(z) < cg_zkey(T)  (NaN z: never below, as in C).
__device__ __forceinline__ uint32_t cg_zkey(float z) {
    if (z != z) return 0xffffffffu;
    if (z == 0.0f) z = 0.0f;
    return cg_fkey(z);
}
template <int LAYOUT>
__device__ __forceinline__ float4 load_xyzi(const uint8_t* fb, uint32_t i, const CgLaunch& L) {
    if (LAYOUT == CG_LAYOUT_XYZI16) return *(const float4*)(fb + (uint64_t)i * 16);
    if (LAYOUT == CG_LAYOUT_PCL32) {
        const float4 v = *(const float4*)(fb + (uint64_t)i * 32);
        const float in = *(const float*)(fb + (uint64_t)i * 32 + 16);
        return make_float4(v.x, v.y, v.z, in);
    }
    float x, y, z;
    load_xyz<CG_LAYOUT_GENERIC>(fb, i, L, x, y, z);
    const uint8_t* p = fb + (uint64_t)i * L.point_step;
    const float in = L.off_i >= 0 ? *(const float*)(p + L.off_i) : 0.f;
    return make_float4(x, y, z, in);
}

// filter_points_position (src/cone_detection.cpp:195-201), distance and level part:
// true = removed. The float sum of squares decides unless it lies within 1e-6 (relative) of
// a threshold; then the exact double S decides.
// Fast form: decides from the float sum alone; returns false (uncertain) when only the
// exact double S can decide.
__device__ __forceinline__ bool dist_level_fast(const CgDevParams& P, float x, float y, float z, bool& rm) {
    const float sf = fmaf(x, x, fmaf(y, y, z * z));   // a certificate only: 3 roundings
    const bool far_c = sf > P.sfar_hi, nfar_c = sf < P.sfar_lo;
    const bool near_c = sf < P.snear_lo, nnear_c = sf > P.snear_hi;
    rm = (z < P.level_f) | far_c | near_c;
    return (far_c | nfar_c) & (near_c | nnear_c);
}
__device__ __forceinline__ bool dist_level_remove(const CgDevParams& P, float x, float y, float z) {
    bool rm;
    if (!dist_level_fast(P, x, y, z, rm)) {
        const double S = cg_sumsq_d(x, y, z);
        rm = (z < P.level_f) || (S >= P.s_far) || (S < P.s_near);
    }
    return rm;
}

// Certified angle classification: sector (src/ground_removal.cpp:61-64) and the angle part of
// filter_points_position (src/cone_detection.cpp:200-201) from a cheap atan2 approximation
// (|error| < 2.3e-6 rad incl. glibc's own error; checked on device by cg_selftest_atan2f)
// whenever the approximation lies more than CG_ANG_MARGIN from every sector boundary and both
// angle thresholds. Otherwise the exact glibc restatement decides. Both decisions are
// monotone step functions of the float angle, so equal classes at a - E and a + E certify.
// The exact restatement, for the rare points the fast classification cannot certify. Inlined
// into those (cold) branches: an out-of-line call from inside divergent loops corrupted the
// caller's per-lane state under some schedules (lanes that took the call lost their keep bits
// in lg_decide; no scratch or register overlap explained it), and the call-free form is
// deterministic.
__device__ __forceinline__ float cg_atan2f_cold(float y, float x) { return cg_atan2f(y, x); }
// Fast form: returns false (uncertain) where only the exact restatement can decide.
template <bool NEED_SECTOR, bool NEED_ANGLE>
__device__ __forceinline__ bool classify_angle_fast(const CgDevParams& P, float x, float y, int& sector,
                                                    bool& ang_rm) {
    // |x|, |y| ordered as unsigned bit patterns (monotone for non-NaN; a NaN fails `ok`):
    // no IEEE canonicalisation as fmaxf / fminf would need
    const uint32_t bx = __float_as_uint(x) & 0x7fffffffu, by = __float_as_uint(y) & 0x7fffffffu;
    const float mx = __uint_as_float(max(bx, by)), mn = __uint_as_float(min(bx, by));
    const float r = mn * __builtin_amdgcn_rcpf(mx);
    const float q = r * r;
    // (explicit FMAs: this is our approximation, not a reference expression)
    // (6-term fit of atan(r)/r in r^2 on [0, 1]: 1.7e-6 rad; tools/ has no generator, the
    // bound is checked on device by cg_selftest_atan2f across every decision boundary)
    float p = -0.011719568632543087f;
    p = fmaf(p, q, 0.05264842137694359f);
    p = fmaf(p, q, -0.11642742902040482f);
    p = fmaf(p, q, 0.19354073703289032f);
    p = fmaf(p, q, -0.3326228857040405f);
    p = fmaf(p, q, 0.9999772310256958f);
    float aa = r * p;                        // |a|
    if (by > bx) aa = 1.5707964f - aa;
    if (x < 0.f) aa = 3.1415927f - aa;
    const bool yneg = y < 0.f;               // a = yneg ? -aa : aa
    // off-axis, not NaN, and inside the range where v_rcp_f32(mx) is a normal number
    // (mx < 2^126) and r does not underflow badly. A NaN x or y has the largest magnitude bit
    // pattern, so mx is NaN and fails mx < 8e37.
    bool ok = (mn > 1.0e-30f) & (mx < 8.0e37f);
    if (NEED_SECTOR) {
        // t ~ wrap(a) / sector: the reference floors fl(fl(wrap(ae)) / SEC) (cg_sector). With
        // |a - ae| <= 2.3e-6 rad, |t - wrap(ae)/SEC| <= 1.0e-5 (6.0e-6 from the angle, the rest
        // from the roundings of both wraps, 1/SEC, 2pi/SEC, this fma and the reference's
        // division), so a fractional part farther than CG_SEC_MARGIN_T from an integer certifies
        // the bin. Near a = 0 the two wraps may disagree: |a| > CG_ANG_MARGIN certifies the sign.
        // fma(-aa, 1/SEC, c) == fma(aa, -1/SEC, c) exactly; t >= 0, so trunc is floor and
        // v_fract_f32 is t - floor(t) exactly.
        const float t = fmaf(aa, yneg ? -1.0f / CG_SECTOR_ANGLE_RAD : 1.0f / CG_SECTOR_ANGLE_RAD,
                             yneg ? 6.2831855f / CG_SECTOR_ANGLE_RAD : 0.f);
        ok = ok & (fabsf(__builtin_amdgcn_fractf(t) - 0.5f) < 0.5f - CG_SEC_MARGIN_T) & (aa > CG_ANG_MARGIN);
        sector = (int)t;   // <= 16: t <= 2pi / SEC + rounding = 16.37
    }
    if (NEED_ANGLE) {
        // ang_lo == -ang_hi exactly (cg_api.cpp prepare), so a <= ang_lo || a >= ang_hi is
        // |a| >= ang_hi (NaN thresholds: false either way)
        ang_rm = aa >= P.ang_cert_hi;
        ok = ok & (ang_rm | (aa < P.ang_cert_lo));
    }
    return ok;
}
template <bool NEED_SECTOR, bool NEED_ANGLE>
__device__ __forceinline__ void classify_angle(const CgDevParams& P, float x, float y, int& sector, bool& ang_rm) {
    if (!classify_angle_fast<NEED_SECTOR, NEED_ANGLE>(P, x, y, sector, ang_rm)) {
        const float ae = cg_atan2f_cold(y, x);
        if (NEED_SECTOR) sector = cg_sector(ae);
        if (NEED_ANGLE) ang_rm = (ae <= P.ang_lo) || (ae >= P.ang_hi);
    }
}

// ------------------------------------------------------------------------------------------
// Per-lane bit sets over the PPT points of a lane (NW 64-bit words; word index may be a
// run-time value, resolved with selects so the words stay in VGPRs).
template <int NW>
struct LaneBits {
    uint64_t w[NW];
    __device__ __forceinline__ void clear() {
#pragma unroll
        for (int i = 0; i < NW; i++) w[i] = 0;
    }
    template <int WIDTH>
    __device__ __forceinline__ void set_bits(int grp, uint32_t v) {   // WIDTH bits at WIDTH*grp
        const int wi = grp / (64 / WIDTH), sh = (grp % (64 / WIDTH)) * WIDTH;
#pragma unroll
        for (int i = 0; i < NW; i++)
            if (i == wi) w[i] |= (uint64_t)v << sh;
    }
    __device__ __forceinline__ void set_byte(int byte_idx, uint32_t v8) { set_bits<8>(byte_idx, v8); }
    __device__ __forceinline__ void clear_bit(int k) {
#pragma unroll
        for (int i = 0; i < NW; i++)
            if ((k >> 6) == i) w[i] &= ~(1ull << (k & 63));
    }
    __device__ __forceinline__ bool get(int k) const {
        uint64_t x = w[0];
#pragma unroll
        for (int i = 1; i < NW; i++)
            if ((k >> 6) == i) x = w[i];
        return (x >> (k & 63)) & 1ull;
    }
    __device__ __forceinline__ uint32_t count() const {
        uint32_t c = 0;
#pragma unroll
        for (int i = 0; i < NW; i++) c += (uint32_t)__popcll(w[i]);
        return c;
    }
};

// 8-bit z code, monotone NON-INCREASING in z: d(z) = sat_u8(rne(fl(zq_bias - 64 z))), one
// v_cvt_pk_u8_f32 (round to nearest even, saturating to [0, 255], NaN -> 0; measured by
// tools/isa_probe.hip) that also packs the byte into its code word. For any threshold T:
// d(z) > d(T) implies z < T, and d(z) < d(T) implies !(z < T); equal codes are ambiguous.
// A NaN z codes 0, the "above every threshold" end, where z < T is false too. Thresholds are
// coded by this same function, so the rounding and the window (zq_bias) only decide how many
// points are ambiguous, never a result.
#define CG_ZQ_SCALE (-64.0f)
// cache policy (aux) bits of pass 1's streaming buffer loads: 2 = nt (every byte of a frame is
// streamed once; the survivor gather re-reads a few lines). Measured at 200 steps, interleaved:
// +2.7% / +3.8% C3 frames/s against the default policy; sc0 (1) no change
// (profiles/r4_nt_ab.txt)
#ifndef CG_PASS1_AUX
#define CG_PASS1_AUX 2
#endif
__device__ __forceinline__ uint32_t zcode_into(float z, float zq_bias, uint32_t byte, uint32_t word) {
    return __builtin_amdgcn_cvt_pk_u8_f32(fmaf(z, CG_ZQ_SCALE, zq_bias), byte, word);
}
__device__ __forceinline__ uint32_t zcode(float z, const CgDevParams& P) { return zcode_into(z, P.zq_bias, 0u, 0u); }
// Pass-2 classes of a point's code c against the band [qlo, qhi] = [min, max] of the used
// sectors' threshold codes: kept in every sector if c < qlo, ground in every sector if c > qhi,
// otherwise ambiguous (exact re-read).
__device__ __forceinline__ bool zc_kept(uint32_t c, uint32_t qlo) { return c < qlo; }
__device__ __forceinline__ bool zc_not_ground(uint32_t c, uint32_t qhi) { return c <= qhi; }


// ------------------------------------------------------------------------------------------
// Sector-coherent fast path. A lane's consecutive points are CG_BLOCK apart; on a spinning
// sensor stored column by column that is a few degrees of azimuth, and the 64 lanes of a wave
// are one column. So the lane's current sector is re-certified per point by two cross products
// against the sector's edge rays (7 VALU), and the approximate atan2 of
// classify_angle_fast runs only where that fails: at sector changes (wave-uniform on such
// data), in sectors the angle filter cuts through, and near edges. Any point order is
// correct; only the speed depends on it.
static_assert(sizeof(((CgDevParams*)0)->ray) / sizeof(float4) == CG_NUM_BINS, "one ray pair per bin");
// The lane-table of rays (LDS, CG_NUM_BINS entries) for this mode: with the angle filter on,
// a sector the filter cuts through gets zero rays, which certify nothing.
template <bool FILTER>
__device__ __forceinline__ void init_rays(const CgDevParams& P, float4* rays, uint32_t t) {
    if (t < CG_NUM_BINS)
        rays[t] = (!FILTER || ((P.ray_filter_ok >> t) & 1u)) ? P.ray[t] : make_float4(0.f, 0.f, 0.f, 0.f);
}
// (x, y) strictly inside the wedge of rays r (lower edge r.xy, upper edge r.zw) by the margin
// CG_RAY_EPS (cg_internal.h): y cos(b) - x sin(b) = |p| sin(angle - b), computed with <= 3
// roundings of |x| + |y|. Tiny, huge and NaN points fail (the 1e-30 floor, inf/NaN compares).
__device__ __forceinline__ bool ray_inside(float x, float y, const float4& r) {
    const float m = fmaf(fabsf(x) + fabsf(y), CG_RAY_EPS, 1.0e-30f);
    const float dlo = fmaf(y, r.x, -(x * r.y));
    const float dhi = fmaf(y, r.z, -(x * r.w));
    return (dlo > m) & (dhi < -m);
}

// ------------------------------------------------------------------------------------------
// Pass 1 over N points at fb (lane t owns points k*512 + t, k < PPT): the certified
// classification of every point, the lane's sector-minimum runs flushed into the 17 bins of
// sec_key (LDS, order-preserving keys), the position-filter bits of the lane's points (posm)
// and the 8-bit z codes, handed to store_codes(group, {codes of points 0-3, 4-7}) once per
// group of 8 points. Points the fast classification cannot certify are redone exactly after
// the loop. touched returns the lane's used sector bins (bit 17: NaN angle).
template <int PPT, int LAYOUT, bool GROUND, bool FILTER, class STORE, bool FULL = false>
__device__ __forceinline__ void stream_pass1(const uint8_t* fb, uint32_t N, const CgLaunch& L,
                                             const CgDevParams& P, uint32_t* sec_key, const float4* rays,
                                             LaneBits<(PPT + 63) / 64>& posm, uint32_t& touched,
                                             STORE store_codes) {
    constexpr int G = 8;                          // points per load group (double-buffered)
    constexpr int NG = PPT / G;
    constexpr int NW = (PPT + 63) / 64;
    static_assert(PPT == G || PPT % (2 * G) == 0, "PPT must be one load group or a multiple of two");
    const uint32_t tid = threadIdx.x;
    // ---- pass 1: stream the frame ----
    // Two explicit load buffers (A, B), the loop unrolled by two: group g+1 is in flight while
    // group g is classified, with no register copies between iterations (a copy of a buffer
    // whose loads are outstanding would force a full vmcnt drain). Loads are branch-free: an
    // index past the frame reads point N-1 again, which can only repeat that point's own
    // sector-min contribution; its filter and uncertainty bits are masked. Points the
    // certified fast classification cannot decide are redone exactly after the loop.
    LaneBits<NW> uncm;
    posm.clear();
    uncm.clear();
    int cur_s = -1;              // the lane's current sector (-1: none yet)
    float4 cur_r = make_float4(0.f, 0.f, 0.f, 0.f);   // its rays (zero: certify nothing)
    bool cur_arm = false;        // the angle filter removes all of it
    float cur_m = INFINITY;      // minimum z of the lane's current run of sector cur_s
    touched = 0;                 // sector bins this lane saw (bit 17: NaN angle)
    const uint32_t nlast = N ? N - 1 : 0u;
    // the z-code bias as a loop-invariant VGPR (v_fmamk takes it from a VGPR only; left to
    // itself the compiler re-materialises it from its SGPR once per point)
    float zbias = P.zq_bias;
    asm volatile("" : "+v"(zbias));
    auto load_group = [&](float3* buf, int g) {
        if (FULL && LAYOUT == CG_LAYOUT_XYZI16) {
            // every group is whole (N = PPT * CG_BLOCK): the group past the end (the loop's last
            // prefetch) is clamped as a whole, a scalar min on the uniform group base, so the
            // per-point address is the loop-invariant lane offset (no per-point VALU)
            // buffer loads: the row offset in an SGPR (soffset), the lane's offset a
            // loop-invariant VGPR (voffset); gfx9 raw-buffer descriptor word 3 = 0x00020000
            const uint32_t gc = (uint32_t)g < (uint32_t)NG ? (uint32_t)g : (uint32_t)NG - 1u;
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void*)fb, (short)0, (int)(N * 16u), 0x00020000);
            typedef uint32_t v3u __attribute__((ext_vector_type(3)));
#pragma unroll
            for (int j = 0; j < G; j++) {
                const v3u v = __builtin_amdgcn_raw_buffer_load_b96(rs, tid * 16u, (gc * G + (uint32_t)j) * (CG_BLOCK * 16u),
                                                                   CG_PASS1_AUX);
                buf[j] = make_float3(__uint_as_float(v.x), __uint_as_float(v.y), __uint_as_float(v.z));
            }
        } else {
#pragma unroll
            for (int j = 0; j < G; j++)
                buf[j] = load_xyz3<LAYOUT>(fb, min((uint32_t)(g * G + j) * CG_BLOCK + tid, nlast), L);
        }
    };
    auto run_group = [&](const float3* buf, int g) {
        // per-point bits are accumulated as v = 2v + bit (one add-with-carry from the compare
        // mask), i.e. point j lands in bit G-1-j; a bit reverse per group restores the order
        uint32_t rpos = 0, runc = 0, clo = 0, chi = 0;
#pragma unroll
        for (int j = 0; j < G; j++) {
            const float x = buf[j].x, y = buf[j].y, z = buf[j].z;
            int s = cur_s;
            bool ang_rm = cur_arm, drm = false;
            bool ok = true;
            if (!ray_inside(x, y, cur_r)) ok = classify_angle_fast<true, FILTER>(P, x, y, s, ang_rm);
            if (FILTER) {
                ok = dist_level_fast(P, x, y, z, drm) & ok;
                rpos = shl1_add_if(rpos, ok & !ang_rm & !drm);
            }
            runc = shl1_add_if(runc, !ok);
            if (GROUND) {
                if (j < 4) clo = zcode_into(z, zbias, j, clo);
                else chi = zcode_into(z, zbias, j - 4, chi);
                // materialise this point's bits now: left alone, the compiler sinks the packing
                // below the run-flush branches and keeps every point's compare masks alive in
                // SGPRs across them (spilled to VGPR lanes: +6 VALU per point, -6% throughput).
                // An empty asm emits no instruction, so it hides nothing from the hazard
                // recognizer.
                asm volatile("" : "+v"(rpos), "+v"(runc), "+v"(clo), "+v"(chi));
                // run-length sector minimum: an uncertain point continues the run without
                // contributing, a NaN z never lowers it; a sector change flushes the run (rare: a lane's consecutive points
                // are 512 apart, a few degrees of azimuth on a spinning sensor)
                const int ss = ok ? s : cur_s;
                if (ss != cur_s) {
                    if (cur_m != INFINITY) {
                        atomicMin(&sec_key[cur_s], cg_fkey(cur_m));
                        touched |= 1u << cur_s;
                    }
                    cur_m = INFINITY;
                    cur_r = rays[ss];
                    if (FILTER) cur_arm = (P.ray_arm >> ss) & 1u;
                }
                if (ok & (z < cur_m)) cur_m = z;   // a NaN z never lowers it
                cur_s = ss;
            } else {
                const int ss = ok ? s : cur_s;
                if (ss != cur_s) {
                    cur_r = rays[ss];
                    cur_arm = (P.ray_arm >> ss) & 1u;
                }
                cur_s = ss;
            }
        }
        if (FILTER) posm.template set_bits<G>(g, __builtin_bitreverse32(rpos) >> (32 - G));
        uncm.template set_bits<G>(g, __builtin_bitreverse32(runc) >> (32 - G));
        if (GROUND) store_codes(g, make_uint2(clo, chi));
    };
    if (N && NG == 1) {
        float3 A[G];
        load_group(A, 0);
        run_group(A, 0);
    } else if (N) {
        float3 A[G], B[G];
        load_group(A, 0);
#pragma unroll 1
        for (int g = 0; g < NG; g += 2) {
            load_group(B, g + 1);
            run_group(A, g);
            load_group(A, g + 2);   // past the frame on the last trip: every lane reads point N-1
            run_group(B, g + 1);
        }
    }
    {   // points k*512 + tid >= N do not exist: drop their bits
        const uint32_t nv = tid < N ? (N - tid + CG_BLOCK - 1) / CG_BLOCK : 0u;
#pragma unroll
        for (int wi = 0; wi < NW; wi++) {
            const int c = (int)nv - 64 * wi;
            const uint64_t vm = c >= 64 ? ~0ull : (c <= 0 ? 0ull : (1ull << c) - 1ull);
            posm.w[wi] &= vm;
            uncm.w[wi] &= vm;
        }
    }
    if (GROUND && cur_m != INFINITY) {
        atomicMin(&sec_key[cur_s], cg_fkey(cur_m));
        touched |= 1u << cur_s;
    }
    // uncertain points: exact angle (glibc restatement) and exact double distance
#pragma unroll
    for (int wi = 0; wi < NW; wi++) {
        uint64_t m = uncm.w[wi];
        while (m) {
            const int k = __builtin_ctzll(m);
            m &= m - 1;
            const float3 p = load_xyz3<LAYOUT>(fb, (uint32_t)(64 * wi + k) * CG_BLOCK + tid, L);
            const float ae = cg_atan2f_cold(p.y, p.x);
            if (GROUND) {
                const int s = cg_sector(ae);
                if (s < CG_NUM_BINS && p.z == p.z) {
                    atomicMin(&sec_key[s], cg_fkey(p.z));
                    touched |= 1u << s;
                } else if (s == CG_NAN_BIN) {
                    touched |= 1u << CG_NAN_BIN;
                }
            }
            if (FILTER && !((ae <= P.ang_lo) || (ae >= P.ang_hi)) && !dist_level_remove(P, p.x, p.y, p.z))
                posm.w[wi] |= 1ull << k;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Ground thresholds, run by wave 0 (tid < 64) once the 17 sector minima are final:
// (double)z < (double)low + 0.1  <=>  z < ceil_to_float(low + 0.1)  (src/ground_removal.cpp:75).
// thr/tkey per bin (18 entries, bin 17 = NaN angles) and the band [qlo, qhi] of threshold
// codes over the bins that hold points (an empty bin's threshold constrains nothing).
__device__ __forceinline__ void sector_thresholds(const uint32_t* sec_key, uint32_t touched_mask,
                                                  const CgDevParams& P, float* thr, uint32_t* tkey,
                                                  uint32_t* qlo_out, uint32_t* qhi_out) {
    const uint32_t tid = threadIdx.x;
    uint32_t tq = 0xffffffffu, tqmax = 0u;
    const bool used = tid <= CG_NUM_BINS && ((touched_mask >> tid) & 1u);
    if (tid <= CG_NUM_BINS) {
        const float low = cg_fkey_inv(sec_key[tid]);
        const float T = cg_ceil_to_float((double)low + 0.1);
        thr[tid] = T;
        tkey[tid] = T != T ? 0u : cg_zkey(T);          // NaN threshold: nothing is below it
        // a NaN threshold keeps every point (z < NaN is false): it must not make the band
        // declare any point ground (qhi = 255) and constrains nothing on the kept side
        if (used) { tq = T != T ? 0xffffffffu : zcode(T, P); tqmax = T != T ? 255u : tq; }
    }
    const uint32_t qlo = wave_umin(tq), qhi = wave_umax(tqmax);
    if (tid == 0) { *qlo_out = qlo; *qhi_out = qhi; }
}

// Pass 2 over the lane's PPT points: codes(g) returns the lane's code word of group g (8
// points). Two compares per code (zc_kept, zc_not_ground): c < qlo keeps, qlo <= c <= qhi is
// ambiguous, c > qhi is ground. Ambiguous points re-read x, y, z and compare exactly against
// their own sector's threshold key. keep returns the lane's kept points (points past N
// excluded).
// pass2_codes is the part the codes settle: keep, and the ambiguous points in amb, with no
// memory traffic past the codes. The caller resolves amb: pass2_keep below, or the frame
// kernel's survivor loads, which load most of those points anyway.
template <int PPT, class CODES>
__device__ __forceinline__ void pass2_codes(uint32_t N, uint32_t qlo, uint32_t qhi, CODES codes,
                                            LaneBits<(PPT + 63) / 64>& keep, LaneBits<(PPT + 63) / 64>& amb) {
    constexpr int NG = PPT / 8;
    constexpr int NW = (PPT + 63) / 64;
    const uint32_t tid = threadIdx.x;
    keep.clear();
    amb.clear();
    // all of the lane's code words first, then the compares; bits accumulate as v = 2v + bit
    // and are bit-reversed per group, as in pass 1
    uint2 cw[NG];
#pragma unroll
    for (int g = 0; g < NG; g++) cw[g] = codes(g);
#pragma unroll
    for (int g = 0; g < NG; g++) {
        uint32_t kr = 0, ar = 0;
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t c = ((j < 4 ? cw[g].x : cw[g].y) >> (8 * (j & 3))) & 0xffu;
            const bool kp = zc_kept(c, qlo), nb = zc_not_ground(c, qhi);
            kr = shl1_add_if(kr, kp);
            ar = shl1_add_if(ar, nb & !kp);
        }
        keep.set_byte(g, __builtin_bitreverse32(kr) >> 24);
        amb.set_byte(g, __builtin_bitreverse32(ar) >> 24);
    }
    {   // points k*512 + tid >= N do not exist
        const uint32_t nv = tid < N ? (N - tid + CG_BLOCK - 1) / CG_BLOCK : 0u;
#pragma unroll
        for (int wi = 0; wi < NW; wi++) {
            const int c = (int)nv - 64 * wi;
            const uint64_t vm = c >= 64 ? ~0ull : (c <= 0 ? 0ull : (1ull << c) - 1ull);
            keep.w[wi] &= vm;
            amb.w[wi] &= vm;
        }
    }
}
// An ambiguous point's exact decision (src/ground_removal.cpp:75): its own sector's threshold key.
__device__ __forceinline__ bool pass2_exact(const CgDevParams& P, const uint32_t* tkey, float x, float y, float z) {
    int sx = 0;
    bool unused = false;
    classify_angle<true, false>(P, x, y, sx, unused);
    return !(cg_zkey(z) < tkey[sx]);
}
template <int PPT, int LAYOUT, class CODES>
__device__ __forceinline__ void pass2_keep(const uint8_t* fb, uint32_t N, const CgLaunch& L,
                                           const CgDevParams& P, uint32_t qlo, uint32_t qhi,
                                           const uint32_t* tkey, CODES codes,
                                           LaneBits<(PPT + 63) / 64>& keep) {
    constexpr int NW = (PPT + 63) / 64;
    const uint32_t tid = threadIdx.x;
    LaneBits<NW> amb;
    pass2_codes<PPT>(N, qlo, qhi, codes, keep, amb);
    STAMP(21);
    // ambiguous: exact z and sector from HBM (rare: tens per frame), four loads in flight
#pragma unroll
    for (int wi = 0; wi < NW; wi++) {
        uint64_t m = amb.w[wi];
        while (m) {
            int ks[4];
            float3 pt[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                ks[q] = m ? __builtin_ctzll(m) : -1;
                if (m) m &= m - 1;
            }
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (ks[q] >= 0) pt[q] = load_xyz3<LAYOUT>(fb, (uint32_t)(64 * wi + ks[q]) * CG_BLOCK + tid, L);
#pragma unroll
            for (int q = 0; q < 4; q++)
                if (ks[q] >= 0 && pass2_exact(P, tkey, pt[q].x, pt[q].y, pt[q].z)) keep.w[wi] |= 1ull << ks[q];
        }
    }
}

#include "cg_grid.h"   // voxel_grid_setup (shared with the host plan, cg_host.cpp)
