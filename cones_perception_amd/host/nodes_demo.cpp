// nodes_demo.cpp — runs the two-node composition of launch/cones_perception.launch
// (GroundRemover -> groundless_cloud -> ConeDetector) through the C++ mirror and checks that
// it equals the fused cg_pipeline on the same frames, bit for bit. Exit 0 on success.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>

#include "cones_nodes.hpp"

using namespace cones_gpu;

static PointCloud2 synth_cloud(uint64_t frame) {
    cg_synth_cfg cfg;
    cg_synth_default(&cfg);
    PointCloud2 msg;
    msg.width = cfg.rings * cfg.cols;
    msg.fields = {{"x", 0}, {"y", 4}, {"z", 8}, {"intensity", 12}};
    msg.point_step = 16;
    msg.row_step = 16 * msg.width;
    msg.data.resize((size_t)msg.row_step);
    check(cg_synth_frames(&cfg, frame, 1, msg.data.data(), msg.row_step, 1));
    return msg;
}

static bool same(const std::vector<float>& a, const std::vector<float>& b) {
    if (a.size() != b.size()) return false;
    for (size_t i = 0; i < a.size(); i++) {
        if (std::isnan(a[i]) && std::isnan(b[i])) continue;
        uint32_t x, y;
        std::memcpy(&x, &a[i], 4);
        std::memcpy(&y, &b[i], 4);
        if (x != y) return false;
    }
    return true;
}

// `nodes_demo --latency R`: the C2 regime of the reference (one 64k-point frame per ROS
// callback, in C++): R synchronous ConePipeline::cloud_handler calls on the first synthetic
// frame with the simulation profile; prints one JSON line with the mean latency.
static int latency(int reps) {
    cg_params p;
    cg_params_init(&p);
    p.num_of_sectors = 16; p.default_lowest_point = -0.1;   // config/ground_removal_params.yaml
    p.distance_treshold_max = 10.0; p.distance_treshold_min = 1.0; p.level_threshold = -5.0;
    p.angle_threshold = 160.0; p.min_cluster_size = 2; p.max_cluster_size = 500;
    p.cone_position_extension_length = 0.05;
    ConePipeline fused(p);
    const PointCloud2 msg = synth_cloud(0);
    uint32_t c = 0;
    for (int i = 0; i < 20; i++) c += (uint32_t)fused.cloud_handler(msg).clusters.size();
    // each call timed too (the clock reads cost ~20 ns a call): the mean, and the median and
    // 90th percentile of the calls
    std::vector<double> each((size_t)std::max(reps, 1));
    const auto t0 = std::chrono::steady_clock::now();
    auto ti = t0;
    for (int i = 0; i < reps; i++) {
        c += (uint32_t)fused.cloud_handler(msg).clusters.size();
        const auto tj = std::chrono::steady_clock::now();
        each[(size_t)i] = std::chrono::duration<double>(tj - ti).count();
        ti = tj;
    }
    const double s = std::chrono::duration<double>(ti - t0).count();
    std::sort(each.begin(), each.begin() + reps);
    const double p50 = reps ? each[(size_t)reps / 2] : 0.0, p90 = reps ? each[(size_t)(reps * 9) / 10] : 0.0;
    std::printf("{\"latency_ms\": %.6f, \"latency_p50_ms\": %.6f, \"latency_p90_ms\": %.6f, \"frames_per_s\": %.3f, "
                "\"calls\": %d, \"clusters\": %u}\n",
                s / reps * 1e3, p50 * 1e3, p90 * 1e3, reps / s, reps, c / (uint32_t)(reps + 20));
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 2 && std::strcmp(argv[1], "--latency") == 0) {
        try {
            return latency(std::atoi(argv[2]));
        } catch (const std::exception& e) {
            std::fprintf(stderr, "%s\n", e.what());
            return 2;
        }
    }
    const int frames = argc > 1 ? std::atoi(argv[1]) : 4;
    cg_params p;
    cg_params_init(&p);   // reference defaults, then the simulation profile
    p.distance_treshold_max = 10.0; p.distance_treshold_min = 1.0; p.level_threshold = -5.0;
    p.angle_threshold = 160.0; p.min_cluster_size = 2; p.max_cluster_size = 500;
    try {
        GroundRemover ground(p);
        ConeDetector detector(p);
        ConePipeline fused(p);
        for (int f = 0; f < frames; f++) {
            const PointCloud2 msg = synth_cloud((uint64_t)f);
            const PointCloud2 groundless = ground.cloud_handler(msg);
            const Detection a = detector.cloud_handler(groundless);
            const Detection b = fused.cloud_handler(msg);
            const bool ok = a.n_filtered == b.n_filtered && ground.n_kept == b.n_kept &&
                            same(a.voxels, b.voxels) && a.clusters == b.clusters &&
                            same(a.centroids, b.centroids);
            std::printf("frame %d: N=%u K=%u M=%u V=%zu C=%zu %s\n", f, msg.width, b.n_kept, b.n_filtered,
                        b.voxels.size() / 4, b.clusters.size(), ok ? "two-node == fused" : "MISMATCH");
            for (size_t c = 0; c < b.clusters.size(); c++)
                std::printf("  cone %zu: %zu voxels at (%.3f, %.3f)\n", c, b.clusters[c].size(),
                            b.centroids[2 * c], b.centroids[2 * c + 1]);
            if (!ok) return 1;
        }
        // the whole detector node over one scene seen from a creeping vehicle: fused pipeline vs
        // the two-node chain (ground node -> detector node); published clouds must agree
        cg_track_params tp;
        cg_track_params_init(&tp);
        tp.classify_colors = 1;
        tp.use_points_buffer = 1;
        ColourService service = [](const std::vector<PointCloud2>& cones, std::vector<int32_t>& colours) {
            colours.clear();
            for (const PointCloud2& c : cones) {   // a stand-in classifier: point count + intensity sum
                double s = 0.0;
                for (uint32_t i = 0; i < c.width; i++) {
                    float v;
                    std::memcpy(&v, c.data.data() + 32 * (size_t)i + 16, 4);
                    s += v;
                }
                colours.push_back((int32_t)((c.width + (uint64_t)std::floor(s)) % CG_NUM_COLORS));
            }
            return true;
        };
        ConeDetectorNode<ConePipeline> fused_node(p, tp, service);
        ConeDetectorNode<ConeDetector> chain_node(p, tp, service);
        const PointCloud2 scene = synth_cloud(10);
        for (int f = 0; f < frames; f++) {
            PointCloud2 msg = scene;
            msg.header.seq = (uint32_t)f;
            msg.header.stamp_sec = 1000 + (uint32_t)f;
            msg.header.stamp_nsec = 123456789;
            for (uint32_t i = 0; i < msg.width; i++) {   // x -= 0.07 m per frame
                float x;
                std::memcpy(&x, msg.data.data() + 16 * (size_t)i, 4);
                x -= 0.07f * (float)f;
                std::memcpy(msg.data.data() + 16 * (size_t)i, &x, 4);
            }
            const auto a = fused_node.cloud_handler(msg);
            const auto b = chain_node.cloud_handler(ground.cloud_handler(msg));
            bool ok = true;
            std::printf("node frame %d:", f);
            for (int i = 0; i < CG_NUM_COLORS; i++) {
                ok = ok && a[i].data == b[i].data && a[i].header == msg.header;
                std::printf(" %s=%u", i == 0 ? "unknown" : i == 1 ? "yellow" : i == 2 ? "blue" : "orange", a[i].width);
            }
            std::printf(" %s\n", ok ? "fused == two-node" : "MISMATCH");
            if (!ok) return 1;
        }
        // with a weights file (argv[2], CG_COLORNET_WEIGHTS raw float32): the colour service
        // served on the GPU by the dam_net classifier
        if (argc > 2) {
            std::vector<float> w(CG_COLORNET_WEIGHTS);
            FILE* fw = std::fopen(argv[2], "rb");
            if (!fw || std::fread(w.data(), 4, w.size(), fw) != w.size()) throw std::runtime_error("bad weights file");
            std::fclose(fw);
            ColorClassifier clf(w);
            ConeDetectorNode<ConePipeline> gpu_node(p, tp, [&clf](const std::vector<PointCloud2>& c, std::vector<int32_t>& k) {
                return clf(c, k);
            });
            uint32_t published = 0;
            for (int f = 0; f < frames; f++) {
                const auto a = gpu_node.cloud_handler(synth_cloud(10));
                std::printf("gpu colour service frame %d:", f);
                for (int i = 0; i < CG_NUM_COLORS; i++) {
                    std::printf(" %u", a[i].width);
                    published += a[i].width;
                }
                std::printf("\n");
            }
            if (frames > 1 && published == 0) return 1;
        }
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 2;
    }
    return 0;
}
