// cg_host.cpp — the host-only logic of the C-ABI, free of HIP runtime calls, so that it is
// built and driven under AddressSanitizer + UndefinedBehaviorSanitizer on the CPU as well
// (oracle/Makefile `asan`, tests/sanitize/asan_driver.cpp): the error channel, the exact
// parameter preparation (the reference's float-vs-double compares resolved into device
// thresholds), the argument and cloud-view checks, and the halo tiling plan of a C5 frame.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <string>
#include "../../include/cones_gpu.h"
#include "cg_internal.h"
#include "cg_math.h"
#include "cg_grid.h"
#include "cg_host.h"

namespace {
thread_local std::string g_err;
}  // namespace

int cg_vfail(int code, const char* fmt, va_list ap) {
    char buf[512];
    vsnprintf(buf, sizeof(buf), fmt, ap);
    g_err = buf;
    return code;
}

int cg_fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    const int rc = cg_vfail(code, fmt, ap);
    va_end(ap);
    return rc;
}

// shared with the other host translation units (cg_api.cpp, cg_track.cpp)
int cg_set_error(int code, const char* msg) { return cg_fail(code, "%s", msg); }

extern "C" const char* cg_last_error(void) { return g_err.c_str(); }

namespace {
// Smallest S >= 0 (a double) with pred(S) true; pred must be monotone in S. Returns
// `none` if pred(+inf) is false.
template <class F>
double min_double_where(F pred, double none) {
    const uint64_t inf_bits = cg_dbits(INFINITY);
    if (!pred(INFINITY)) return none;
    if (pred(0.0)) return 0.0;
    uint64_t lo = 0, hi = inf_bits;   // pred(lo) false, pred(hi) true
    while (hi - lo > 1) {
        const uint64_t mid = lo + (hi - lo) / 2;
        if (pred(cg_bitsd(mid))) hi = mid; else lo = mid;
    }
    return cg_bitsd(hi);
}

// euclidan_dist(p, 0) as a function of S = (x^2 + y^2) + z^2 (src/perception_handling/utils.cpp:33)
float dist_of_sumsq(double S) { return (float)std::sqrt(S); }

}  // namespace

int cg_prepare_params(const cg_params& p, CgDevParams& d) {
    if (!(p.voxel_filter_leaf_size_x > 0) || !(p.voxel_filter_leaf_size_y > 0) ||
        !(p.voxel_filter_leaf_size_z > 0))
        return cg_fail(CG_E_INVALID, "voxel_filter_leaf_size_* must be > 0");
    std::memset(&d, 0, sizeof(d));
    d.default_low = p.default_lowest_point;
    // (double)z < level_threshold
    d.level_f = cg_ceil_to_float(p.level_threshold);
    // euclidan_dist(...) > distance_treshold_max  <=>  S >= s_far
    const double dmax = p.distance_treshold_max, dmin = p.distance_treshold_min;
    d.s_far = (dmax != dmax) ? NAN
                             : min_double_where([&](double S) { return (double)dist_of_sumsq(S) > dmax; }, NAN);
    // euclidan_dist(...) < distance_treshold_min  <=>  S < s_near
    d.s_near = (dmin != dmin) ? 0.0
                              : min_double_where([&](double S) { return (double)dist_of_sumsq(S) >= dmin; },
                                                 INFINITY);
    // -angle*pi/180 >= atan2f  <=>  a <= ang_lo ;  atan2f >= angle*pi/180  <=>  a >= ang_hi
    const double theta = p.angle_threshold * M_PI / 180;
    const double ntheta = -p.angle_threshold * M_PI / 180;
    d.ang_lo = cg_floor_to_float(ntheta);
    d.ang_hi = cg_ceil_to_float(theta);
    d.ang_cert_hi = cg_ceil_to_float((double)d.ang_hi + (double)CG_ANG_MARGIN);
    d.ang_cert_lo = cg_floor_to_float((double)d.ang_hi - (double)CG_ANG_MARGIN);
    // sector rays and the angle-filter class of each sector's wedge (cg_device.h ray_inside)
    for (int sct = 0; sct < CG_NUM_BINS; sct++) {
        const double lo = sct * (double)CG_SECTOR_ANGLE_RAD;             // exact product
        const double hi = sct + 1 < CG_NUM_BINS ? (sct + 1) * (double)CG_SECTOR_ANGLE_RAD : 2.0 * M_PI;
        d.ray[sct] = make_float4((float)std::cos(lo), (float)std::sin(lo), (float)std::cos(hi), (float)std::sin(hi));
        // unwrapped angles a in (-pi, pi] of the padded wedge: one or two intervals
        const double wl = lo - CG_RAY_WEDGE_PAD, wh = hi + CG_RAY_WEDGE_PAD;
        double iv[2][2];
        int niv = 0;
        if (wh <= M_PI) { iv[0][0] = wl; iv[0][1] = wh; niv = 1; }
        else if (wl >= M_PI) { iv[0][0] = wl - 2 * M_PI; iv[0][1] = wh - 2 * M_PI; niv = 1; }
        else { iv[0][0] = wl; iv[0][1] = M_PI; iv[1][0] = -M_PI; iv[1][1] = wh - 2 * M_PI; niv = 2; }
        bool keep = true, rm = true;
        for (int k = 0; k < niv; k++) {
            // keep: ang_lo < a < ang_hi on the whole interval; remove: a <= ang_lo or a >= ang_hi
            keep = keep && iv[k][0] > (double)d.ang_lo && iv[k][1] < (double)d.ang_hi;
            rm = rm && (iv[k][1] <= (double)d.ang_lo || iv[k][0] >= (double)d.ang_hi);
        }
        if (keep || rm) d.ray_filter_ok |= 1u << sct;
        if (rm) d.ray_arm |= 1u << sct;
    }
    // pcl::VoxelGrid::setLeafSize(float, float, float): inverse = 1.0f / leaf
    d.inv_leaf[0] = 1.0f / (float)p.voxel_filter_leaf_size_x;
    d.inv_leaf[1] = 1.0f / (float)p.voxel_filter_leaf_size_y;
    d.inv_leaf[2] = 1.0f / (float)p.voxel_filter_leaf_size_z;
    // tolerance (src/cone_detection.cpp:22-23,212): const float members promoted by pow
    const float cone_width = 0.228, cone_height = 0.325;
    const double tol = std::sqrt(std::pow(cone_height, 2) + std::pow(cone_width, 2));
    const float tol_f = (float)tol;                               // extract(): float tolerance
    d.r2 = (float)((double)tol_f * (double)tol_f);                 // KdTreeFLANN::radiusSearch
    d.cell_inv = 1.0f / (tol_f * 1.0625f);
    d.min_cl = (uint32_t)p.min_cluster_size;
    d.max_cl = (uint32_t)p.max_cluster_size;
    d.ext = p.cone_position_extension_length;
    // float certificates for the distance compares: the device's fma(x,x,fma(y,y,z*z)) is
    // within 3 roundings (2e-7 relative) of S, far inside the 1e-6 slack
    d.sfar_lo = cg_floor_to_float(d.s_far * (1.0 - 1e-6));
    d.sfar_hi = cg_ceil_to_float(d.s_far * (1.0 + 1e-6));
    d.snear_lo = cg_floor_to_float(d.s_near * (1.0 - 1e-6));
    d.snear_hi = cg_ceil_to_float(d.s_near * (1.0 + 1e-6));
    // z-code window: every sector threshold is ceil(low + 0.1) with low <= default_lowest_point,
    // so thresholds lie at or below T_max; codes resolve 1/64 m over ~4 m below it
    const float tmax = cg_ceil_to_float((double)p.default_lowest_point + 0.1);
    // (descending code: T_max codes 1, so a NaN z, coded 0, is below qlo whenever it can be)
    d.zq_z0 = (tmax == tmax && std::isfinite(tmax)) ? tmax : 0.0f;
    d.zq_bias = 64.0f * d.zq_z0 + 1.0f;
    // does PointXYZI() (0,0,0) survive filter_points_position?
    const float a0 = cg_atan2f(0.0f, 0.0f);
    const double S0 = 0.0;
    const bool rm = (0.0f < d.level_f) || (S0 >= d.s_far) || (S0 < d.s_near) || (a0 <= d.ang_lo) ||
                    (a0 >= d.ang_hi);
    d.zero_pass = rm ? 0 : 1;
    return CG_OK;
}

int cg_check_view(const cg_cloud_view* v) {
    if (!v) return cg_fail(CG_E_INVALID, "null cloud view");
    const uint64_t n = (uint64_t)v->width * v->height;
    if (n > CG_MAX_FRAME_POINTS)
        return cg_fail(CG_E_CAPACITY, "cloud has %llu points; the engine supports <= %u",
                    (unsigned long long)n, (unsigned)CG_MAX_FRAME_POINTS);
    if (n == 0) return CG_OK;
    if (!v->data) return cg_fail(CG_E_INVALID, "null cloud data");
    if (v->point_step == 0) return cg_fail(CG_E_INVALID, "point_step is 0");
    if ((uint64_t)v->row_step < (uint64_t)v->width * v->point_step)
        return cg_fail(CG_E_INVALID, "row_step < width * point_step");
    const int32_t offs[4] = {v->off_x, v->off_y, v->off_z, v->off_intensity};
    for (int32_t o : offs)
        if (o >= 0 && (uint64_t)o + 4 > v->point_step)
            return cg_fail(CG_E_INVALID, "field offset %d outside point_step %u", o, v->point_step);
    return CG_OK;
}

int cg_check_tile(const cg_tile* t) {
    if (t->n && !t->d_data) return cg_fail(CG_E_INVALID, "null tile data");
    if (t->n_total > CG_MAX_FRAME_POINTS || (uint64_t)t->first + t->n > t->n_total)
        return cg_fail(CG_E_INVALID, "tile [%u, %u + %u) outside a frame of %u points", t->first, t->first, t->n, t->n_total);
    if (t->point_step == 0 || t->point_step % 4) return cg_fail(CG_E_INVALID, "bad point_step");
    const int32_t offs[4] = {t->off_x, t->off_y, t->off_z, t->off_intensity};
    for (int32_t o : offs)
        if (o >= 0 && (o % 4 || (uint32_t)o + 4 > t->point_step)) return cg_fail(CG_E_INVALID, "bad field offset %d", o);
    return CG_OK;
}

int cg_halo_counts_check(const uint32_t* c, uint32_t n_total) {
    if (!c) return cg_fail(CG_E_INVALID, "null merged counts");
    if (n_total == 0 || n_total > CG_MAX_FRAME_POINTS || c[0] > n_total || c[1] > n_total || c[2] > c[1])
        return cg_fail(CG_E_INVALID, "inconsistent tile counts (K %u, survivors %u, finite %u, N %u)", c[0], c[1], c[2],
                    n_total);
    return CG_OK;
}
int cg_halo_plan_check(const cg_halo_plan* p) {
    if (!p) return cg_fail(CG_E_INVALID, "null plan");
    if (p->passthrough) return cg_fail(CG_E_INVALID, "passthrough frame: no voxel lattice to tile");
    if (p->slabs == 0 || p->slab_w == 0) return cg_fail(CG_E_INVALID, "empty slab plan");
    return CG_OK;
}

// The plan (cg_halo_plan_frame): the whole frame's lattice from the merged counts, as
// cg_large_backend computes it, cut into slabs at least `band` columns wide.
void cg_halo_plan_compute(const CgDevParams& P, const uint32_t* c, uint32_t N, uint32_t n_ranks, struct cg_halo_plan* out) {
    const uint32_t K = c[0];
    const uint32_t npad = P.zero_pass ? N - K : 0u;
    float bmn[3], bmx[3];
    uint32_t nfin = c[2];
    for (int a = 0; a < 3; a++) {
        bmn[a] = nfin ? cg_fkey_inv(c[3 + a]) : INFINITY;
        bmx[a] = nfin ? cg_fkey_inv(c[6 + a]) : -INFINITY;
        if (npad) { bmn[a] = std::min(bmn[a], 0.f); bmx[a] = std::max(bmx[a], 0.f); }
    }
    nfin += npad;
    uint32_t pass = 0;
    int min_b[3], div_b[3];
    voxel_grid_setup(nfin, bmn, bmx, P, pass, min_b, div_b);
    *out = cg_halo_plan{};
    out->passthrough = pass;
    for (int a = 0; a < 3; a++) { out->min_b[a] = min_b[a]; out->div_b[a] = (uint32_t)div_b[a]; }
    // |x1 - x2| < tol between centroids of columns i1 < i2 needs i2 - i1 <= tol / leaf + 1;
    // one column more covers a centroid rounded across its cell edge
    out->band = (uint32_t)std::ceil((double)std::sqrt(P.r2) * (double)P.inv_leaf[0]) + 2u;
    const uint32_t dx = (uint32_t)div_b[0];
    out->slabs = std::max<uint32_t>(1, std::min<uint32_t>(std::max<uint32_t>(n_ranks, 1), dx / out->band));
    out->slab_w = (dx + out->slabs - 1) / out->slabs;
    out->n_pads = npad;
    out->pad_slab = -1;
    if (npad && !pass) {
        const int i0 = (int)(floorf(0.f * P.inv_leaf[0]) - (float)min_b[0]);
        out->pad_slab = (int32_t)std::min<uint32_t>((uint32_t)i0 / out->slab_w, out->slabs - 1);
    }
    out->key_bits = pass ? 0u
                         : 1u + cg_bits_of((uint64_t)(uint32_t)div_b[0] * (uint64_t)(uint32_t)div_b[1] *
                                        (uint64_t)(uint32_t)div_b[2]);
    out->key_bits = std::min<uint32_t>(out->key_bits, 32u);
}
