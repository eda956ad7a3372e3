// cones_nodes.hpp — ROS-free C++ mirror of the reference's two node classes over the C-ABI.
//
// The reference's hot path lives in two ROS callbacks:
//   GroundRemover::cloud_handler  (src/ground_removal.cpp:50-89)
//   ConeDetector::cloud_handler   (src/cone_detection.cpp:130-187)
// This header keeps their names, argument meaning and behaviour (parameter defaults, the
// one-time intensity probe of src/cone_detection.cpp:131-151, the groundless cloud's PCL
// PointXYZI layout) but takes a plain PointCloud2 struct instead of a ROS message, and
// calls include/cones_gpu.h for every per-point operation. INTEGRATION.md shows the same
// calls inside the real nodes.
#pragma once
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "cones_gpu.h"

namespace cones_gpu {

struct PointField {           // sensor_msgs/PointField
    std::string name;
    uint32_t offset = 0;
    uint8_t datatype = 7;     // FLOAT32
    uint32_t count = 1;
};

struct PointCloud2 {          // sensor_msgs/PointCloud2 (header reduced to stamp + frame)
    double stamp = 0.0;
    std::string frame_id;
    uint32_t height = 1, width = 0;
    std::vector<PointField> fields;
    bool is_bigendian = false;
    uint32_t point_step = 0, row_step = 0;
    std::vector<uint8_t> data;
    bool is_dense = true;

    int32_t offset_of(const std::string& n) const {   // pcl::fromROSMsg field match
        for (const auto& f : fields)
            if (f.name == n && f.datatype == 7 && f.count == 1) return (int32_t)f.offset;
        return -1;
    }
    bool has_field(const std::string& n) const {      // perception_handling::intensity_in_cloud
        for (const auto& f : fields)
            if (f.name == n) return true;
        return false;
    }
    cg_cloud_view view(int32_t off_intensity) const {
        cg_cloud_view v{};
        v.data = data.empty() ? nullptr : data.data();
        v.width = width; v.height = height; v.point_step = point_step; v.row_step = row_step;
        v.off_x = offset_of("x"); v.off_y = offset_of("y"); v.off_z = offset_of("z");
        v.off_intensity = off_intensity;
        v.is_dense = is_dense ? 1 : 0;
        return v;
    }
};

// Pre-tracking output of ConeDetector::cloud_handler: what get_centroid_clouds receives
// (voxel cloud + cluster indices) and the centroids it computes (src/cone_detection.cpp:261-279).
struct Detection {
    uint32_t n_points = 0, n_kept = 0, n_filtered = 0, flags = 0;
    std::vector<float> voxels;                    // V x 4
    std::vector<std::vector<int32_t>> clusters;   // pcl::PointIndices, PCL order
    std::vector<float> centroids;                 // C x 2 (z = 0)
};

inline void check(int rc) {
    if (rc != CG_OK) throw std::runtime_error(std::string("cones_gpu: ") + cg_last_error());
}

class Handle {
public:
    Handle(const cg_params& p, int device) { check(cg_create(&p, device, &h_)); }
    ~Handle() { cg_destroy(h_); }
    Handle(const Handle&) = delete;
    Handle& operator=(const Handle&) = delete;
protected:
    cg_handle* h_ = nullptr;
};

inline Detection to_detection(const cg_detect_result& r) {
    Detection d;
    d.n_points = r.n_points; d.n_kept = r.n_kept; d.n_filtered = r.n_filtered; d.flags = r.flags;
    d.voxels.assign(r.voxels, r.voxels + 4 * (size_t)r.n_voxels);
    for (uint32_t c = 0; c < r.n_clusters; c++)
        d.clusters.emplace_back(r.cluster_indices + r.cluster_offsets[c], r.cluster_indices + r.cluster_offsets[c + 1]);
    d.centroids.assign(r.centroids, r.centroids + 2 * (size_t)r.n_clusters);
    return d;
}

// GroundRemover (src/ground_removal.cpp:16-90). Parameters: num_of_sectors,
// default_lowest_point (config/ground_removal_params.yaml).
class GroundRemover : public Handle {
public:
    explicit GroundRemover(const cg_params& p, int device = 0) : Handle(p, device) {}
    // Returns the groundless cloud the node publishes: header copied, fields = PointXYZI's
    // (x, y, z, intensity at 0, 4, 8, 16), point_step 32, N points (K kept + zero pads).
    PointCloud2 cloud_handler(const PointCloud2& msg) {
        const cg_cloud_view v = msg.view(msg.offset_of("intensity"));
        cg_ground_result r{};
        check(cg_ground_remove(h_, &v, &r));
        PointCloud2 out;
        out.stamp = msg.stamp; out.frame_id = msg.frame_id;
        out.width = r.width; out.height = r.height;
        out.fields = {{"x", 0}, {"y", 4}, {"z", 8}, {"intensity", 16}};
        out.point_step = 32; out.row_step = 32 * r.width;
        out.data.assign(r.data, r.data + 32 * (size_t)r.n_points);
        out.is_dense = msg.is_dense;
        n_kept = r.n_kept;
        return out;
    }
    uint32_t n_kept = 0;
};

// ConeDetector (src/cone_detection.cpp:19-364), hot part. Parameters: the keys of
// config/cones_detection_params_*.yaml.
class ConeDetector : public Handle {
public:
    explicit ConeDetector(const cg_params& p, int device = 0) : Handle(p, device) {}
    Detection cloud_handler(const PointCloud2& msg) {
        if (!intensity_in_cloud_checked) {                         // lines 131-136
            if (!msg.has_field("intensity")) intensity_in_cloud = false;
            intensity_in_cloud_checked = true;
        }
        // lines 142-151: no intensity -> fake FLOAT32 field at offset 0 (intensity = x bytes)
        const cg_cloud_view v = msg.view(intensity_in_cloud ? msg.offset_of("intensity") : 0);
        cg_detect_result r{};
        check(cg_detect(h_, &v, &r));
        return to_detection(r);
    }
    bool intensity_in_cloud_checked = false;
    bool intensity_in_cloud = true;
};

// launch/cones_perception.launch:17-37 (ground_removal:=true) fused into one device pass.
class ConePipeline : public Handle {
public:
    explicit ConePipeline(const cg_params& p, int device = 0) : Handle(p, device) {}
    Detection cloud_handler(const PointCloud2& msg) {
        const cg_cloud_view v = msg.view(msg.offset_of("intensity"));
        cg_detect_result r{};
        check(cg_pipeline(h_, &v, &r));
        return to_detection(r);
    }
};

}  // namespace cones_gpu
