// Host sanitizer driver (AddressSanitizer + UndefinedBehaviorSanitizer, -fno-sanitize-recover):
// the CPU restatement (oracle/cg_oracle.cpp) and the host-only parts of the C-ABI library
// (csrc/cg_track.cpp, csrc/cg_synth.c, csrc/cg_host.cpp) built with the sanitizers and driven over synthetic
// frames of every size class, edge clouds (empty, non-finite, all pads, the voxel overflow
// guard), the three parameter profiles, both voxel orders, the re-crop, the node's tracking
// with full / short / failed colour responses, and the tracker's own C-ABI. Test
// infrastructure (tests/test_sanitizers.py builds and runs it); no GPU.
//   asan_driver <params blob> [<params blob> ...]   (bytes of cg_params, one per profile)
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "cones_gpu.h"

typedef int (*ServiceFn)(void* ctx, const float* pts, const uint32_t* offs, uint32_t n, int32_t* out, uint32_t cap);
extern "C" {
int oracle_run(const void* params, const void* view, int mode, int order, uint32_t* hdr, float* ground,
               float* voxels, int32_t* labels, int32_t* offsets, int32_t* indices, float* centroids);
uint32_t oracle_recrop(const void* params, const void* view, int mode, const float* centres, uint32_t n,
                       uint32_t* offsets, float* points, uint32_t cap);
void* oracle_node_create(int classify_colors, int use_points_buffer, double matching);
void oracle_node_destroy(void* node);
int oracle_node_step(void* node, const void* params, const void* view, int mode, const float* centroids,
                     uint32_t n, ServiceFn service, void* ctx, uint32_t* counts, float* xy, uint32_t cap);
}
#include "cg_math.h"
#include "cg_host.h"   // the C-ABI's host-only logic (csrc/cg_host.cpp): checks, parameters, halo plan

// The C-ABI's host-only logic under the sanitizers: parameter preparation over the profiles and
// random / degenerate values, the cloud-view and tile argument checks, and the halo tiling plan
// of a tiled frame over random merged counts and bounds, with the plan's invariants checked.
static int host_api(const std::vector<cg_params>& profiles) {
    std::mt19937 rng(17);
    auto unif = [&](double lo, double hi) { return lo + (hi - lo) * (double)(rng() % 1000001) / 1e6; };
    const double specials[] = {NAN, INFINITY, -INFINITY, 0.0, -0.0, 1e-300, 1e300, -1.0, 0.04, 25.0};
    for (const cg_params& p0 : profiles) {
        CgDevParams d;
        if (cg_prepare_params(p0, d) != CG_OK) return 20;
        for (int k = 0; k < 3000; k++) {
            cg_params p = p0;
            double* dbl[] = {&p.distance_treshold_max, &p.distance_treshold_min, &p.angle_threshold,
                             &p.level_threshold, &p.cone_position_extension_length};
            for (double* x : dbl) if (rng() % 3 == 0) *x = rng() % 2 ? specials[rng() % 10] : unif(-400.0, 400.0);
            if (rng() % 3 == 0) p.default_lowest_point = rng() % 2 ? (float)specials[rng() % 10] : (float)unif(-10, 10);
            double* leaf[] = {&p.voxel_filter_leaf_size_x, &p.voxel_filter_leaf_size_y, &p.voxel_filter_leaf_size_z};
            for (double* x : leaf) if (rng() % 4 == 0) *x = rng() % 2 ? specials[rng() % 10] : unif(1e-4, 2.0);
            if (rng() % 4 == 0) p.min_cluster_size = (int)(rng() % 200) - 20;
            if (rng() % 4 == 0) p.max_cluster_size = (int)(rng() % 100000) - 20;
            const bool leaf_ok = p.voxel_filter_leaf_size_x > 0 && p.voxel_filter_leaf_size_y > 0 && p.voxel_filter_leaf_size_z > 0;
            const int rc = cg_prepare_params(p, d);
            if ((rc == CG_OK) != leaf_ok) return 21;
            if (rc != CG_OK && !*cg_last_error()) return 22;
            if (rc == CG_OK && d.s_far == d.s_far && !(d.sfar_lo <= d.sfar_hi)) return 23;
        }
    }
    // cloud views
    std::vector<uint8_t> buf(64 * 32);
    if (cg_check_view(nullptr) == CG_OK) return 30;
    for (int k = 0; k < 20000; k++) {
        cg_cloud_view v;
        std::memset(&v, 0, sizeof(v));
        v.data = rng() % 8 ? buf.data() : nullptr;
        v.width = rng() % 4 ? rng() % 70 : rng();
        v.height = rng() % 4 ? 1 + rng() % 3 : rng();
        v.point_step = rng() % 6 ? 4 * (rng() % 9) : rng() % 40;
        v.row_step = rng() % 3 ? v.width * v.point_step : rng();
        int32_t* offs[] = {&v.off_x, &v.off_y, &v.off_z, &v.off_intensity};
        for (int32_t* o : offs) *o = rng() % 5 ? 4 * (int32_t)(rng() % 8) : (int32_t)(rng() % 64) - 8;
        const int rc = cg_check_view(&v);
        const uint64_t n = (uint64_t)v.width * v.height;
        if (rc == CG_OK && n && (!v.data || !v.point_step || (uint64_t)v.row_step < (uint64_t)v.width * v.point_step))
            return 31;
        if (rc == CG_OK) {
            for (int32_t* o : offs) if (*o >= 0 && (uint64_t)*o + 4 > v.point_step && n) return 32;
        }
    }
    // tiles
    for (int k = 0; k < 20000; k++) {
        cg_tile t;
        std::memset(&t, 0, sizeof(t));
        t.d_data = rng() % 8 ? buf.data() : nullptr;
        t.n_total = rng() % 4 ? rng() % 5000 : rng();
        t.first = rng() % 3000;
        t.n = rng() % 3000;
        t.point_step = rng() % 6 ? 4 * (rng() % 9) : rng() % 40;
        int32_t* offs[] = {&t.off_x, &t.off_y, &t.off_z, &t.off_intensity};
        for (int32_t* o : offs) *o = rng() % 5 ? 4 * (int32_t)(rng() % 8) : (int32_t)(rng() % 64) - 8;
        const int rc = cg_check_tile(&t);
        if (rc == CG_OK && ((uint64_t)t.first + t.n > t.n_total || !t.point_step || t.point_step % 4)) return 33;
    }
    // halo plans of tiled frames: merged counts (K, survivors, finite survivors, bounds keys)
    if (cg_halo_counts_check(nullptr, 10) == CG_OK || cg_halo_plan_check(nullptr) == CG_OK) return 40;
    long plans = 0;
    for (const cg_params& p0 : profiles) {
        for (int zp = 0; zp < 2; zp++) {
            cg_params p = p0;
            if (zp) p.distance_treshold_min = 0.0;   // zero pads survive: they join the lattice
            CgDevParams d;
            if (cg_prepare_params(p, d) != CG_OK) return 41;
            for (int k = 0; k < 5000; k++) {
                const uint32_t N = rng() % 5 ? 1 + rng() % (1u << 20) : 1 + rng() % (1u << 28);
                uint32_t c[9];
                c[0] = rng() % 4 ? rng() % (N + 1) : rng();
                c[1] = rng() % 4 ? rng() % (N + 1) : rng();
                c[2] = rng() % 4 ? (c[1] ? rng() % (c[1] + 1) : 0u) : rng();
                const double span = rng() % 8 ? unif(0.0, 60.0) : unif(0.0, 2e5);   // wide spans trip PCL's guard
                for (int a = 0; a < 3; a++) {
                    const float lo = (float)unif(-1e5, 1e5);
                    c[3 + a] = cg_fkey(lo);
                    c[6 + a] = cg_fkey((float)((double)lo + (a == 2 ? span / 20 : span)));
                }
                const uint32_t ranks = rng() % 10;
                const int ok = cg_halo_counts_check(c, N);
                if (ok == CG_OK && (c[0] > N || c[1] > N || c[2] > c[1])) return 42;
                if (ok != CG_OK) continue;
                cg_halo_plan plan;
                cg_halo_plan_compute(d, c, N, ranks, &plan);
                plans++;
                if (plan.slabs < 1 || plan.slabs > (ranks > 1 ? ranks : 1u) || plan.key_bits > 32) return 43;
                if (!plan.passthrough) {
                    if ((uint64_t)plan.slab_w * plan.slabs < plan.div_b[0]) return 44;
                    if (plan.slabs > 1 && plan.slab_w < plan.band) return 45;
                    if (plan.n_pads && (plan.pad_slab < 0 || (uint32_t)plan.pad_slab >= plan.slabs)) return 46;
                    if (cg_halo_plan_check(&plan) != CG_OK) return 47;
                } else if (cg_halo_plan_check(&plan) == CG_OK) {
                    return 48;
                }
            }
        }
    }
    std::printf("host C-ABI checks: %ld halo plans\n", plans);
    return 0;
}

static cg_cloud_view view_of(const std::vector<uint8_t>& d, uint32_t n, uint32_t step) {
    cg_cloud_view v;
    std::memset(&v, 0, sizeof(v));
    v.data = d.empty() ? nullptr : d.data();
    v.width = n; v.height = 1; v.point_step = step; v.row_step = n * step;
    v.off_x = 0; v.off_y = 4; v.off_z = 8; v.off_intensity = step == 32 ? 16 : 12;
    v.is_dense = 0;
    return v;
}

struct Result { std::vector<float> centroids; uint32_t hdr[8]; };

static Result run_all(const cg_params& p, const std::vector<uint8_t>& data, uint32_t n, uint32_t step) {
    const cg_cloud_view v = view_of(data, n, step);
    const size_t cap = n ? n : 1;
    std::vector<float> ground(cap * 8), vox(cap * 4), cen(cap * 2);
    std::vector<int32_t> lab(cap), offs(cap + 1), idx(cap);
    Result r{};
    for (int mode = 0; mode < 3; mode++)
        for (int order = 0; order < 2; order++) {
            uint32_t hdr[8];
            if (oracle_run(&p, &v, mode, order, hdr, ground.data(), vox.data(), lab.data(), offs.data(), idx.data(),
                           cen.data()) != 0) { std::printf("oracle_run failed\n"); std::exit(3); }
            if (mode == 0 && order == 1) {
                std::memcpy(r.hdr, hdr, sizeof(hdr));
                r.centroids.assign(cen.begin(), cen.begin() + 2 * hdr[4]);
            }
        }
    // re-crop around every centroid and two far points, both cloud modes
    std::vector<float> centres = r.centroids;
    centres.insert(centres.end(), {1e6f, -1e6f, 0.f, 0.f});
    const uint32_t nc = (uint32_t)centres.size() / 2;
    std::vector<uint32_t> co(nc + 1);
    std::vector<float> pts(4 * 4096);
    for (int mode = 0; mode < 2; mode++) oracle_recrop(&p, &v, mode, centres.data(), nc, co.data(), pts.data(), 4096);
    return r;
}

// colour service stand-in: colour by crop size; short responses (empty crops skipped, as the
// reference's server does) and failed calls on some frames
struct Svc { int frame; };
static int service(void* ctx, const float* pts, const uint32_t* offs, uint32_t n, int32_t* out, uint32_t cap) {
    const Svc* s = (const Svc*)ctx;
    if (s->frame % 7 == 3) return -1;
    uint32_t k = 0;
    for (uint32_t c = 0; c < n && k < cap; c++) {
        const uint32_t m = offs[c + 1] - offs[c];
        if (!m) continue;
        float acc = 0.f;
        for (uint32_t q = offs[c]; q < offs[c + 1]; q++) acc += pts[4 * q + 3];
        out[k++] = (int32_t)((m + (uint32_t)std::fabs(acc)) % 4u);
    }
    if (s->frame % 5 == 1 && k) k--;   // a shorter response still
    return (int)k;
}

int main(int argc, char** argv) {
    std::vector<cg_params> profiles;
    for (int a = 1; a < argc; a++) {
        FILE* f = std::fopen(argv[a], "rb");
        cg_params p;
        if (!f || std::fread(&p, sizeof(p), 1, f) != 1) { std::printf("bad params file %s\n", argv[a]); return 2; }
        std::fclose(f);
        profiles.push_back(p);
    }
    if (profiles.empty()) return 2;
    cg_synth_cfg cfg;
    long frames = 0;
    for (size_t pi = 0; pi < profiles.size(); pi++) {
        const cg_params& p = profiles[pi];
        struct Shape { uint32_t rings, cols, step, clutter, cpr, colmajor; } shapes[] = {
            {16, 1024, 16, 0, 5, 1}, {16, 1024, 32, 0, 5, 0}, {64, 1024, 16, 0, 5, 1}, {64, 1024, 16, 60, 10, 1}};
        void* node = oracle_node_create(1, (int)(pi & 1), p.cones_matching_dist_theshold);
        int fr = 0;
        for (const Shape& s : shapes) {
            cg_synth_default(&cfg);
            cfg.rings = s.rings; cfg.cols = s.cols; cfg.point_step = s.step; cfg.clutter = s.clutter;
            cfg.cones_per_row = s.cpr; cfg.column_major = s.colmajor;
            const uint32_t n = s.rings * s.cols, nf = 2;
            std::vector<uint8_t> buf((size_t)n * s.step * nf);
            if (cg_synth_frames(&cfg, 3 + pi, nf, buf.data(), (uint64_t)n * s.step, 2) != 0) return 4;
            for (uint32_t f = 0; f < nf; f++) {
                std::vector<uint8_t> one(buf.begin() + (size_t)f * n * s.step, buf.begin() + (size_t)(f + 1) * n * s.step);
                Result r = run_all(p, one, n, s.step);
                const cg_cloud_view v = view_of(one, n, s.step);
                Svc sv{fr++};
                std::vector<uint32_t> counts(4);
                const uint32_t cap = r.hdr[4] ? r.hdr[4] : 1;
                std::vector<float> xy((size_t)4 * cap * 2);
                oracle_node_step(node, &p, &v, 0, r.centroids.data(), r.hdr[4], service, &sv, counts.data(), xy.data(),
                                 cap);
                frames++;
            }
        }
        oracle_node_destroy(node);
        // edge clouds
        std::mt19937 rng(11 + (unsigned)pi);
        std::vector<std::vector<float>> edge;
        edge.push_back({});                                              // empty
        edge.push_back({NAN, 1.f, 0.f, 0.f, INFINITY, 2.f, -0.5f, 1.f});  // non-finite only
        edge.push_back(std::vector<float>(4 * 300, 0.f));                // all zero points
        edge.push_back({1e30f, 1e30f, 0.f, 0.f, -1e30f, -1e30f, 0.f, 0.f, 3.f, 0.2f, -0.3f, 5.f});   // overflow guard
        {
            std::vector<float> e;
            for (int i = 0; i < 4000; i++) {   // one dense blob: many points per voxel, ties everywhere
                e.push_back(4.f + 0.01f * (float)(rng() % 50)); e.push_back(0.01f * (float)(rng() % 50));
                e.push_back(-0.2f + 0.01f * (float)(rng() % 20)); e.push_back((float)(rng() % 256));
            }
            edge.push_back(e);
        }
        for (const auto& e : edge) {
            const uint32_t n = (uint32_t)e.size() / 4;
            std::vector<uint8_t> d(e.size() * 4);
            if (!e.empty()) std::memcpy(d.data(), e.data(), d.size());
            run_all(p, d, n, 16);
            frames++;
        }
    }
    // the tracker's C-ABI (cg_track.cpp) over random sequences and every response kind
    std::mt19937 rng(5);
    for (int variant = 0; variant < 4; variant++) {
        cg_track_params tp;
        tp.classify_colors = (uint8_t)(variant & 1);
        tp.use_points_buffer = (uint8_t)((variant >> 1) & 1);
        tp.cones_matching_dist_theshold = 0.5;
        cg_tracker* t = nullptr;
        if (cg_tracker_create(&tp, &t) != CG_OK) return 5;
        for (int f = 0; f < 60; f++) {
            const uint32_t n = rng() % 30;
            std::vector<float> c(2 * n);
            for (float& x : c) x = (float)(rng() % 2000) * 0.01f - 10.f;
            std::vector<int32_t> status(n + 1);
            uint32_t need = 0;
            if (cg_tracker_match(t, n ? c.data() : nullptr, n, status.data(), &need) != CG_OK) return 6;
            std::vector<int32_t> colors(need + 2);
            for (auto& x : colors) x = (int32_t)(rng() % 4);
            int rc;
            switch (f % 4) {
                case 0: rc = cg_tracker_commit(t, colors.data(), need); break;
                case 1: rc = cg_tracker_commit(t, nullptr, 0); break;
                case 2: rc = cg_tracker_commit(t, colors.data(), need / 2); break;
                default:
                    if (cg_tracker_commit(t, colors.data(), need + 1) == CG_OK) return 7;   // too long: refused
                    rc = cg_tracker_commit(t, colors.data(), need);
            }
            if (rc != CG_OK) return 8;
            for (int col = 0; col < CG_NUM_COLORS; col++) {
                const float* xy = nullptr;
                uint32_t m = 0;
                if (cg_tracker_cloud(t, col, &xy, &m) != CG_OK) return 9;
                volatile float s = 0.f;
                for (uint32_t k = 0; k < 2 * m; k++) s += xy[k];
            }
        }
        cg_tracker_destroy(t);
    }
    if (int rc = host_api(profiles)) { std::printf("host C-ABI check %d failed\n", rc); return rc; }
    std::printf("sanitizers clean: %ld clouds, 4 tracker variants, the C-ABI's host logic\n", frames);
    return 0;
}
