/* cg_synth.c — deterministic synthetic cone-field LiDAR frames (test/bench input generator).
 *
 * The reference ships no recorded clouds on the hot path, so every config is fed
 * synthetic frames shaped like the reference's use case (images/mp_pcl2.png: a ring LiDAR over a
 * cone track). SURVEY.md §8(d) fixes the geometry:
 *   ring LiDAR at the origin, mount height 0.5 m (ground plane z = -0.5), elevations
 *   linspace(-25 deg, +15 deg, R), azimuth 360 deg * c / C; rays end on the ground, a cone
 *   (0.228 m base x 0.325 m tall, src/cone_detection.cpp:22-23), an optional post, or a far
 *   cylindrical wall at 25 m so every ray returns and N = R*C exactly; two cone rows 3 m apart
 *   with ~4 m spacing along a gently curved centreline, 5 cm placement jitter; range noise
 *   N(0, 1 cm); intensity U[0, 100].
 * Output is a PointCloud2 data block: xyzi float32 at offsets 0,4,8,12 (point_step 16) or the
 * PCL PointXYZI layout (point_step 32: x,y,z,1.0f,intensity,0,0,0).
 * Every random draw is a counter-based hash of (seed, frame, object/ray), so a frame's bytes do
 * not depend on threading or on which other frames are generated.
 */
#include <math.h>
#include <stdint.h>
#include <string.h>
#include <pthread.h>
#include "../../include/cones_gpu.h"

static uint64_t mix64(uint64_t z) {
    z += 0x9e3779b97f4a7c15ull;
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
    return z ^ (z >> 31);
}
static double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
static double rnd(uint64_t seed, uint64_t a, uint64_t b) {
    return u01(mix64(mix64(mix64(seed) ^ a) ^ (b * 0xd1b54a32d192ed03ull)));
}
static double gauss(uint64_t seed, uint64_t a, uint64_t b) {
    double u1 = rnd(seed, a, 2 * b + 0), u2 = rnd(seed, a, 2 * b + 1);
    if (u1 < 1e-300) u1 = 1e-300;
    return sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
}

#define MAX_OBJ 4096
typedef struct { double x, y, r, h; int kind; } obj_t; /* kind 0 cone (r=base radius), 1 post */

static int build_scene(const cg_synth_cfg* cfg, uint64_t frame, obj_t* o) {
    const uint64_t s = cfg->seed ^ mix64(frame + 1);
    const double ground = -cfg->mount_height;
    int n = 0;
    /* cone track: centreline y_c(x) = A sin(x / L + phi), rows at +-1.5 m, spacing ~4 m */
    double A = 2.0 * rnd(s, 1, 0), L = 6.0 + 6.0 * rnd(s, 1, 1), phi = 6.283185307 * rnd(s, 1, 2);
    double yaw = (rnd(s, 1, 3) - 0.5) * 0.6;   /* +-17 deg heading of the track */
    double x0 = -3.0 + 4.0 * rnd(s, 1, 4);
    for (int i = 0; i < 2 * cfg->cones_per_row && n < MAX_OBJ; i++) {
        int row = i & 1, k = i >> 1;
        double along = x0 + 4.0 * k + 0.3 * (rnd(s, 2, (uint64_t)i) - 0.5);
        double yc = A * sin(along / L + phi) + (row ? 1.5 : -1.5);
        double jx = 0.05 * gauss(s, 3, (uint64_t)i), jy = 0.05 * gauss(s, 4, (uint64_t)i);
        double px = along + jx, py = yc + jy;
        o[n].x = px * cos(yaw) - py * sin(yaw);
        o[n].y = px * sin(yaw) + py * cos(yaw);
        o[n].r = 0.114; o[n].h = 0.325; o[n].kind = 0;
        if (o[n].x * o[n].x + o[n].y * o[n].y > 0.8 * 0.8) n++;   /* nothing on the sensor */
    }
    /* clutter posts (dense scenes): radius 4-10 cm, height 0.4-1.5 m, range 2-14 m */
    for (uint32_t i = 0; i < cfg->clutter && n < MAX_OBJ; i++) {
        double rr = 2.0 + 12.0 * rnd(s, 5, i), th = 6.283185307 * rnd(s, 6, i);
        o[n].x = rr * cos(th); o[n].y = rr * sin(th);
        o[n].r = 0.04 + 0.06 * rnd(s, 7, i); o[n].h = 0.4 + 1.1 * rnd(s, 8, i); o[n].kind = 1;
        n++;
    }
    (void)ground;
    return n;
}

/* Nearest positive hit of the ray t*d (|d| = 1) with an object; returns +inf if none. */
static double hit_obj(const obj_t* ob, double dx, double dy, double dz, double ground) {
    double ox = -ob->x, oy = -ob->y;
    double hd2 = dx * dx + dy * dy;
    double tc = -(ox * dx + oy * dy) / (hd2 > 1e-300 ? hd2 : 1e-300);   /* closest approach */
    double cx = ox + tc * dx, cy = oy + tc * dy;
    if (cx * cx + cy * cy > ob->r * ob->r || tc <= 0.0) return INFINITY;
    double best = INFINITY;
    if (ob->kind == 1) {
        double a = hd2, b = 2.0 * (ox * dx + oy * dy), c = ox * ox + oy * oy - ob->r * ob->r;
        double disc = b * b - 4 * a * c;
        if (disc < 0) return INFINITY;
        double t = (-b - sqrt(disc)) / (2 * a);
        double z = t * dz;
        if (t > 0 && z >= ground && z <= ground + ob->h) best = t;
        return best;
    }
    double za = ground + ob->h, k = ob->r / ob->h, k2 = k * k;
    double a = hd2 - k2 * dz * dz;
    double b = 2.0 * (ox * dx + oy * dy + k2 * za * dz);
    double c = ox * ox + oy * oy - k2 * za * za;
    if (fabs(a) < 1e-12) {
        if (fabs(b) < 1e-300) return INFINITY;
        double t = -c / b, z = t * dz;
        if (t > 0 && z >= ground && z <= za) best = t;
        return best;
    }
    double disc = b * b - 4 * a * c;
    if (disc < 0) return INFINITY;
    double sq = sqrt(disc);
    double t1 = (-b - sq) / (2 * a), t2 = (-b + sq) / (2 * a);
    if (t1 > t2) { double tmp = t1; t1 = t2; t2 = tmp; }
    double z1 = t1 * dz, z2 = t2 * dz;
    if (t1 > 0 && z1 >= ground && z1 <= za) best = t1;
    else if (t2 > 0 && z2 >= ground && z2 <= za) best = t2;
    return best;
}

static void gen_frame(const cg_synth_cfg* cfg, uint64_t frame, uint8_t* out) {
    obj_t objs[MAX_OBJ];
    const int nobj = build_scene(cfg, frame, objs);
    const double ground = -cfg->mount_height;
    const uint64_t s = cfg->seed ^ mix64(frame + 1) ^ 0x5bd1e995ull;
    const uint32_t R = cfg->rings, C = cfg->cols;
    for (uint32_t c = 0; c < C; c++) {
        double az = 6.283185307179586 * (double)c / (double)C;
        double ca = cos(az), sa = sin(az);
        for (uint32_t r = 0; r < R; r++) {
            double el_deg = R > 1 ? cfg->elev_min_deg + (cfg->elev_max_deg - cfg->elev_min_deg) *
                                        (double)r / (double)(R - 1)
                                  : cfg->elev_min_deg;
            double el = el_deg * 3.14159265358979323846 / 180.0;
            double ce = cos(el), dz = sin(el), dx = ce * ca, dy = ce * sa;
            double t = cfg->wall_radius / (ce > 1e-9 ? ce : 1e-9);
            if (dz < 0) { double tg = ground / dz; if (tg < t) t = tg; }
            for (int i = 0; i < nobj; i++) {
                double th = hit_obj(&objs[i], dx, dy, dz, ground);
                if (th < t) t = th;
            }
            uint64_t ray = (uint64_t)c * R + r;
            t += cfg->range_noise * gauss(s, 9, ray);
            float p[8] = {(float)(t * dx), (float)(t * dy), (float)(t * dz), 1.0f,
                          (float)(100.0 * rnd(s, 10, ray)), 0.f, 0.f, 0.f};
            uint64_t idx = cfg->column_major ? (uint64_t)c * R + r : (uint64_t)r * C + c;
            uint8_t* dst = out + idx * cfg->point_step;
            if (cfg->point_step == 32) memcpy(dst, p, 32);
            else { float q[4] = {p[0], p[1], p[2], p[4]}; memcpy(dst, q, 16); }
        }
    }
}

typedef struct { const cg_synth_cfg* cfg; uint64_t first; uint32_t n, t, nt; uint8_t* out; uint64_t stride; } job_t;
static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    for (uint32_t f = j->t; f < j->n; f += j->nt) gen_frame(j->cfg, j->first + f, j->out + f * j->stride);
    return 0;
}

void cg_synth_default(cg_synth_cfg* c) {
    memset(c, 0, sizeof(*c));
    c->rings = 64; c->cols = 1024;
    c->elev_min_deg = -25.0f; c->elev_max_deg = 15.0f;
    c->mount_height = 0.5f; c->wall_radius = 25.0f; c->range_noise = 0.01f;
    c->point_step = 16; c->column_major = 1; c->cones_per_row = 5; c->clutter = 0;
    c->seed = 0x00c0ffee;
}

int cg_synth_frames(const cg_synth_cfg* cfg, uint64_t first_frame, uint32_t n_frames, void* out,
                    uint64_t frame_stride, uint32_t n_threads) {
    if (!cfg || !out || (cfg->point_step != 16 && cfg->point_step != 32) || cfg->rings == 0 ||
        cfg->cols == 0)
        return CG_E_INVALID;
    if (frame_stride < (uint64_t)cfg->rings * cfg->cols * cfg->point_step) return CG_E_INVALID;
    if (n_threads < 1) n_threads = 1;
    if (n_threads > 64) n_threads = 64;
    if (n_threads > n_frames) n_threads = n_frames ? n_frames : 1;
    pthread_t th[64];
    job_t jobs[64];
    for (uint32_t t = 0; t < n_threads; t++) {
        jobs[t] = (job_t){cfg, first_frame, n_frames, t, n_threads, (uint8_t*)out, frame_stride};
        if (n_threads == 1) worker(&jobs[t]);
        else pthread_create(&th[t], 0, worker, &jobs[t]);
    }
    if (n_threads > 1)
        for (uint32_t t = 0; t < n_threads; t++) pthread_join(th[t], 0);
    return CG_OK;
}
