// cg_math.h — exact scalar restatements shared by the HIP kernels and their host checks.
//
// Every function here reproduces, bit for bit, a scalar operation of the reference hot path
// (dmn-sjk/cones_perception) as it executes on an x86-64 host with glibc libm and no FMA:
//
//   * cg_atan2f      — glibc's fdlibm-derived atan2f/atanf (sysdeps/ieee754/flt-32), which the
//                      reference reaches through `atan2(float,float)` at
//                      src/ground_removal.cpp:61,72 and src/cone_detection.cpp:200-201.
//                      Validated against the host libm: 0 mismatches over all 2^32 atanf inputs
//                      and 2e8 random atan2f pairs (tests/test_math_host.py re-checks a sample).
//   * cg_sector      — wrap + floor division of src/ground_removal.cpp:61-64 (rule G2/G3).
//   * cg_ceil_to_float / cg_floor_to_float / cg_next_up — turn the reference's
//                      float-vs-double comparisons into exact float comparisons.
//
// All device code that includes this header is compiled with -ffp-contract=off: the reference
// is a stock x86-64 build with no FMA, so contraction would change results.
#pragma once
#include <stdint.h>
#include <math.h>
#include <string.h>

#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define CG_HD __host__ __device__ __forceinline__
#else
#define CG_HD static inline
#endif

CG_HD uint32_t cg_fbits(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
CG_HD float cg_bitsf(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }
CG_HD uint64_t cg_dbits(double d) { uint64_t u; memcpy(&u, &d, 8); return u; }
CG_HD double cg_bitsd(uint64_t u) { double d; memcpy(&d, &u, 8); return d; }

// glibc sysdeps/ieee754/flt-32/s_atanf.c restated (fdlibm): argument reduction into four
// intervals, 11-term odd/even polynomial split, hi/lo table correction.
CG_HD float cg_atanf(float x) {
    const float atanhi0 = 4.6364760399e-01f, atanhi1 = 7.8539812565e-01f,
                atanhi2 = 9.8279368877e-01f, atanhi3 = 1.5707962513e+00f;
    const float atanlo0 = 5.0121582440e-09f, atanlo1 = 3.7748947079e-08f,
                atanlo2 = 3.4473217170e-08f, atanlo3 = 7.5497894159e-08f;
    const float aT0 = 3.3333334327e-01f, aT1 = -2.0000000298e-01f, aT2 = 1.4285714924e-01f,
                aT3 = -1.1111110449e-01f, aT4 = 9.0908870101e-02f, aT5 = -7.6918758452e-02f,
                aT6 = 6.6610731184e-02f, aT7 = -5.8335702866e-02f, aT8 = 4.9768779427e-02f,
                aT9 = -3.6531571299e-02f, aT10 = 1.6285819933e-02f;
    int32_t hx = (int32_t)cg_fbits(x);
    int32_t ix = hx & 0x7fffffff;
    int id;
    if (ix >= 0x4c000000) {                        // |x| >= 2^25
        if (ix > 0x7f800000) return x + x;         // NaN
        return hx > 0 ? atanhi3 + atanlo3 : -atanhi3 - atanlo3;
    }
    if (ix < 0x3ee00000) {                         // |x| < 0.4375
        if (ix < 0x31000000) return x;             // |x| < 2^-29
        id = -1;
    } else {
        x = fabsf(x);
        if (ix < 0x3f980000) {                     // |x| < 1.1875
            if (ix < 0x3f300000) { id = 0; x = (2.0f * x - 1.0f) / (2.0f + x); }
            else                 { id = 1; x = (x - 1.0f) / (x + 1.0f); }
        } else {
            if (ix < 0x401c0000) { id = 2; x = (x - 1.5f) / (1.0f + 1.5f * x); }
            else                 { id = 3; x = -1.0f / x; }
        }
    }
    float z = x * x;
    float w = z * z;
    float s1 = z * (aT0 + w * (aT2 + w * (aT4 + w * (aT6 + w * (aT8 + w * aT10)))));
    float s2 = w * (aT1 + w * (aT3 + w * (aT5 + w * (aT7 + w * aT9))));
    if (id < 0) return x - x * (s1 + s2);
    float hi = id == 0 ? atanhi0 : id == 1 ? atanhi1 : id == 2 ? atanhi2 : atanhi3;
    float lo = id == 0 ? atanlo0 : id == 1 ? atanlo1 : id == 2 ? atanlo2 : atanlo3;
    z = hi - ((x * (s1 + s2) - lo) - x);
    return hx < 0 ? -z : z;
}

// glibc sysdeps/ieee754/flt-32/e_atan2f.c restated: special cases, quadrant code m, ratio
// cut-offs at 2^60, then atanf(|y/x|) with the pi_lo correction.
CG_HD float cg_atan2f(float y, float x) {
    const float tiny = 1.0e-30f, pi_o_4 = 7.8539818525e-01f, pi_o_2 = 1.5707963705e+00f,
                pi = 3.1415927410e+00f, pi_lo = -8.7422776573e-08f;
    int32_t hx = (int32_t)cg_fbits(x), hy = (int32_t)cg_fbits(y);
    int32_t ix = hx & 0x7fffffff, iy = hy & 0x7fffffff;
    if (ix > 0x7f800000 || iy > 0x7f800000) return x + y;    // NaN
    if (hx == 0x3f800000) return cg_atanf(y);                   // x == 1.0
    int m = ((hy >> 31) & 1) | ((hx >> 30) & 2);
    if (iy == 0) {
        if (m <= 1) return y;
        return m == 2 ? pi + tiny : -pi - tiny;
    }
    if (ix == 0) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    if (ix == 0x7f800000) {
        if (iy == 0x7f800000) {
            switch (m) {
                case 0: return pi_o_4 + tiny;
                case 1: return -pi_o_4 - tiny;
                case 2: return 3.0f * pi_o_4 + tiny;
                default: return -3.0f * pi_o_4 - tiny;
            }
        }
        switch (m) {
            case 0: return 0.0f;
            case 1: return -0.0f;
            case 2: return pi + tiny;
            default: return -pi - tiny;
        }
    }
    if (iy == 0x7f800000) return hy < 0 ? -pi_o_2 - tiny : pi_o_2 + tiny;
    int32_t k = (iy - ix) >> 23;
    float z;
    if (k > 60) z = pi_o_2 + 0.5f * pi_lo;
    else if (hx < 0 && k < -60) z = 0.0f;
    else z = cg_atanf(fabsf(y / x));
    switch (m) {
        case 0: return z;
        case 1: return cg_bitsf(cg_fbits(z) ^ 0x80000000u);
        case 2: return pi - (z - pi_lo);
        default: return (z - pi_lo) - pi;
    }
}

// Number of polar sectors actually addressed by the reference. sector_angle_rad is fixed at
// float(22*pi/180) by a default member initializer (src/ground_removal.cpp:18-20, rule G1), so
// wrapped angles in [0, 2pi] map to bins 0..16; bin 16 is past the end of a 16-entry vector in
// the reference (UB, rule G3) and is defined here as its own bin initialised to
// default_lowest_point. Bin 17 collects points whose angle is NaN (reference: int(NaN) index,
// UB); it is never updated and always compares against default_lowest_point.
#define CG_NUM_BINS 17
#define CG_NAN_BIN 17
#define CG_SECTOR_ANGLE_RAD 0.38397244f   /* float(22 * M_PI / 180) = 0x3ec49809 */

// src/ground_removal.cpp:61-64: angle wrap in double then floor of a float quotient.
CG_HD int cg_sector(float a) {
    if (a != a) return CG_NAN_BIN;
    float angle = a;
    if (a < 0.0f) angle = (float)((double)a + 2.0 * 3.14159265358979323846);
    float q = floorf(angle / CG_SECTOR_ANGLE_RAD);
    int s = (int)q;
    return s > 16 ? 16 : s;   // cannot exceed 16 for finite a; kept as a guard
}

// Order-preserving map float -> uint32 (for LDS atomicMin on floats); NaN never enters.
CG_HD uint32_t cg_fkey(float f) {
    uint32_t u = cg_fbits(f);
    return (u & 0x80000000u) ? ~u : (u | 0x80000000u);
}
CG_HD float cg_fkey_inv(uint32_t k) {
    return cg_bitsf((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k);
}

// Smallest float strictly greater than f (f finite or -inf).
CG_HD float cg_next_up(float f) {
    uint32_t u = cg_fbits(f);
    if (f != f || u == 0x7f800000u) return f;
    if (f == 0.0f) return cg_bitsf(1u);
    return cg_bitsf((u & 0x80000000u) ? u - 1 : u + 1);
}
CG_HD float cg_next_down(float f) { return -cg_next_up(-f); }

// Smallest float F with (double)F >= t, so that for every float z:
//   (double)z < t   <=>   z < F.
CG_HD float cg_ceil_to_float(double t) {
    if (t != t) return cg_bitsf(0x7fc00000u);
    float f = (float)t;                       // round-to-nearest-even
    if ((double)f < t) f = cg_next_up(f);
    return f;
}
// Largest float F with (double)F <= t, so that for every float z:
//   (double)z <= t   <=>   z <= F.
CG_HD float cg_floor_to_float(double t) {
    if (t != t) return cg_bitsf(0x7fc00000u);
    float f = (float)t;
    if ((double)f > t) f = cg_next_down(f);
    return f;
}

// src/perception_handling/utils.cpp:32-34 euclidan_dist(p, origin) before the sqrt:
// pow(float,2) promotes to double and is exact, summed left to right in double.
CG_HD double cg_sumsq_d(float x, float y, float z) {
    double dx = (double)x, dy = (double)y, dz = (double)z;
    return (dx * dx + dy * dy) + dz * dz;
}
