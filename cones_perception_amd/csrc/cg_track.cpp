// cg_track.cpp — host side of the detector node after the hot path: frame-to-frame cone
// matching and the four colour clouds (ConeDetector::get_centroid_clouds,
// src/cone_detection.cpp:251-339). Scalar work over tens of centroids per frame; it stays on
// the host, as in the reference, next to the colour-classifier call it gates.
//
// One frame is two calls, split where the reference calls the colour service
// (src/cone_detection.cpp:320-327):
//   cg_tracker_match   decides per centroid: dropped, published in a known colour's cloud, or
//                      to be classified (then the caller re-crops the cone, cg_recrop, and
//                      asks its classifier);
//   cg_tracker_commit  takes the classifier's colours and builds the frame's clouds in the
//                      reference's push order, then rolls prev_* state.
#include <cmath>
#include <cstdint>
#include <cstring>
#include <new>
#include <vector>

#include "../../include/cones_gpu.h"
#include "cg_internal.h"

struct cg_tracker {
    cg_track_params p;
    bool have_prev = false;                 // prev_detected_cones != NULL
    std::vector<float> prev_detected;       // (x, y) pairs, z = 0
    std::vector<float> prev_clouds[CG_NUM_COLORS];
    // the frame between match and commit
    bool matched = false;
    std::vector<float> cur;                 // currently_detected_cones
    std::vector<int32_t> status;
    std::vector<float> clouds[CG_NUM_COLORS];
};

namespace {

int fail(int code, const char* msg) { return cg_set_error(code, msg); }

// perception_handling::euclidan_dist (src/perception_handling/utils.cpp:32-34): float
// differences, pow(.,2) of their double promotions (exact), double sum and sqrt, float result.
float euclidan_dist(float x1, float y1, float z1, float x2, float y2, float z2) {
    const double dx = (double)(x1 - x2), dy = (double)(y1 - y2), dz = (double)(z1 - z2);
    return (float)std::sqrt(dx * dx + dy * dy + dz * dz);
}

bool near(const cg_track_params& p, float x, float y, float qx, float qy) {
    return (double)euclidan_dist(x, y, 0.0f, qx, qy, 0.0f) < p.cones_matching_dist_theshold;
}

}  // namespace

extern "C" void cg_track_params_init(cg_track_params* p) {
    if (!p) return;
    std::memset(p, 0, sizeof *p);
    p->classify_colors = 1;                   // src/cone_detection.cpp:34-35
    p->use_points_buffer = 0;
    p->cones_matching_dist_theshold = 0.5;    // src/cone_detection.cpp:38
}

extern "C" int cg_tracker_create(const cg_track_params* p, cg_tracker** out) {
    if (!out) return fail(CG_E_INVALID, "null argument");
    *out = nullptr;
    cg_tracker* t = new (std::nothrow) cg_tracker;
    if (!t) return fail(CG_E_OOM, "tracker allocation failed");
    if (p) t->p = *p;
    else cg_track_params_init(&t->p);
    *out = t;
    return CG_OK;
}

extern "C" int cg_tracker_destroy(cg_tracker* t) {
    delete t;
    return CG_OK;
}

extern "C" int cg_tracker_set_params(cg_tracker* t, const cg_track_params* p) {
    if (!t || !p) return fail(CG_E_INVALID, "null argument");
    t->p = *p;
    return CG_OK;
}

// src/cone_detection.cpp:259-315: for each centroid in cluster order, the first previous cone
// that matches (any previous cone when use_points_buffer is off) publishes it: in the colour
// cloud of the first previous coloured cone within the threshold (colours 1..3 in order), or
// for classification; in the unknown cloud when classify_colors is off.
extern "C" int cg_tracker_match(cg_tracker* t, const float* centroids_xy, uint32_t n, int32_t* status,
                                uint32_t* n_need) {
    if (!t || (n && !centroids_xy)) return fail(CG_E_INVALID, "null argument");
    t->cur.assign(centroids_xy, centroids_xy + 2 * (size_t)n);
    t->status.assign(n, CG_TRACK_DROPPED);
    for (auto& c : t->clouds) c.clear();
    uint32_t need = 0;
    for (uint32_t c = 0; c < n; c++) {
        const float x = centroids_xy[2 * c], y = centroids_xy[2 * c + 1];
        if (!t->have_prev) continue;
        const std::vector<float>& prev = t->prev_detected;
        for (size_t q = 0; q < prev.size() / 2; q++) {
            if (t->p.use_points_buffer && !near(t->p, x, y, prev[2 * q], prev[2 * q + 1])) continue;
            if (t->p.classify_colors) {
                int32_t colour = CG_TRACK_NEED_COLOR;
                for (int i = 1; i < CG_NUM_COLORS && colour == CG_TRACK_NEED_COLOR; i++) {
                    const std::vector<float>& pc = t->prev_clouds[i];
                    for (size_t k = 0; k < pc.size() / 2; k++)
                        if (near(t->p, x, y, pc[2 * k], pc[2 * k + 1])) { colour = i; break; }
                }
                t->status[c] = colour;
                if (colour == CG_TRACK_NEED_COLOR) need++;
                else t->clouds[colour].insert(t->clouds[colour].end(), {x, y});
            } else {
                t->status[c] = 0;   // kUnknownColor
                t->clouds[0].insert(t->clouds[0].end(), {x, y});
            }
            break;
        }
    }
    if (status && n) std::memcpy(status, t->status.data(), n * sizeof(int32_t));
    if (n_need) *n_need = need;
    t->matched = true;
    return CG_OK;
}

// src/cone_detection.cpp:320-339: the classified centroids follow the known-colour ones in
// their clouds, in classification order; then prev_centroid_clouds = this frame's clouds and
// prev_detected_cones = every centroid of this frame.
//
// The colours are the service's response, applied as the reference applies it: colors(n_need,
// kUnknownColor) (line 328), then std::transform of the response over its first entries
// (357-358). The reference's server answers only non-empty crops
// (scripts/color_classifier_server.py:83-84), so n_colors < n_need colours the first n_colors
// cones in request order and leaves the rest unknown. colors == NULL is a failed call (every
// colour unknown, 359-361). n_colors > n_need would write past the reference's vector: refused.
extern "C" int cg_tracker_commit(cg_tracker* t, const int32_t* colors, uint32_t n_colors) {
    if (!t) return fail(CG_E_INVALID, "null argument");
    if (!t->matched) return fail(CG_E_INVALID, "cg_tracker_commit without cg_tracker_match");
    uint32_t need = 0;
    for (int32_t s : t->status) need += s == CG_TRACK_NEED_COLOR;
    if (!colors) n_colors = 0;
    if (n_colors > need) return fail(CG_E_INVALID, "more colours than centroids that need one");
    for (uint32_t k = 0; k < n_colors; k++)
        if (colors[k] < 0 || colors[k] >= CG_NUM_COLORS) return fail(CG_E_INVALID, "colour out of range");
    uint32_t k = 0;
    for (size_t c = 0; c < t->status.size(); c++) {
        if (t->status[c] != CG_TRACK_NEED_COLOR) continue;
        const int colour = k < n_colors ? colors[k] : 0;   // kUnknownColor past the response
        k++;
        t->clouds[colour].insert(t->clouds[colour].end(), {t->cur[2 * c], t->cur[2 * c + 1]});
    }
    for (int i = 0; i < CG_NUM_COLORS; i++) t->prev_clouds[i] = t->clouds[i];
    t->prev_detected = t->cur;
    t->have_prev = true;
    t->matched = false;
    return CG_OK;
}

extern "C" int cg_tracker_cloud(const cg_tracker* t, int color, const float** xy, uint32_t* n) {
    if (!t || !xy || !n || color < 0 || color >= CG_NUM_COLORS) return fail(CG_E_INVALID, "bad argument");
    *xy = t->clouds[color].empty() ? nullptr : t->clouds[color].data();
    *n = (uint32_t)(t->clouds[color].size() / 2);
    return CG_OK;
}
