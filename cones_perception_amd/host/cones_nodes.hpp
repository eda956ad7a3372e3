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
#include <array>
#include <cstdint>
#include <cstring>
#include <functional>
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

struct Header {               // std_msgs/Header
    uint32_t seq = 0;
    uint32_t stamp_sec = 0, stamp_nsec = 0;
    std::string frame_id;
    bool operator==(const Header& o) const {
        return seq == o.seq && stamp_sec == o.stamp_sec && stamp_nsec == o.stamp_nsec && frame_id == o.frame_id;
    }
};

// The header after pcl::fromROSMsg then pcl::toROSMsg (pcl_conversions, PCL 1.10): the stamp
// travels as microseconds (toNSec() / 1000, then * 1000), so nanoseconds truncate.
inline Header pcl_header(Header h) {
    h.stamp_nsec = h.stamp_nsec / 1000u * 1000u;
    return h;
}

struct PointCloud2 {          // sensor_msgs/PointCloud2
    Header header;
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
    std::vector<std::vector<float>> crops(const std::vector<float>& centres_xy) {
        cg_crop_result r{};
        check(cg_recrop(h_, centres_xy.empty() ? nullptr : centres_xy.data(), (uint32_t)(centres_xy.size() / 2), &r));
        std::vector<std::vector<float>> out(r.n_centers);
        for (uint32_t c = 0; c < r.n_centers; c++)
            out[c].assign(r.points + 4 * (size_t)r.offsets[c], r.points + 4 * (size_t)r.offsets[c + 1]);
        return out;
    }
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
        // lines 83-86: header and fields set before toROSMsg, which replaces both
        out.header = pcl_header(msg.header);
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
    // get_reconstructed_cone (lines 222-238) around each centre over the last call's whole
    // cloud: one x,y,z,intensity array per centre.
    std::vector<std::vector<float>> recrop(const std::vector<float>& centres_xy) { return crops(centres_xy); }
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
    std::vector<std::vector<float>> recrop(const std::vector<float>& centres_xy) {   // over the groundless cloud
        return crops(centres_xy);
    }
};

// pcl::toROSMsg of a PointCloud<PointXYZI> filled by push_back (PCL 1.10): height 1, width n,
// PointXYZI's fields, point_step 32, is_dense; x, y, z, 1.0f, intensity, 12 zero padding bytes.
inline PointCloud2 to_ros_msg(const std::vector<float>& xyzi) {
    PointCloud2 m;
    const size_t n = xyzi.size() / 4;
    m.width = (uint32_t)n; m.height = 1;
    m.fields = {{"x", 0}, {"y", 4}, {"z", 8}, {"intensity", 16}};
    m.point_step = 32; m.row_step = 32 * m.width;
    m.data.assign(32 * n, 0);
    for (size_t i = 0; i < n; i++) {
        const float rec[5] = {xyzi[4 * i], xyzi[4 * i + 1], xyzi[4 * i + 2], 1.0f, xyzi[4 * i + 3]};
        std::memcpy(m.data.data() + 32 * i, rec, sizeof rec);
    }
    return m;
}

// Tracking and the colour clouds, get_centroid_clouds (src/cone_detection.cpp:251-339).
class ConeTracker {
public:
    explicit ConeTracker(const cg_track_params& p) { check(cg_tracker_create(&p, &t_)); }
    ~ConeTracker() { cg_tracker_destroy(t_); }
    ConeTracker(const ConeTracker&) = delete;
    ConeTracker& operator=(const ConeTracker&) = delete;
    std::vector<int32_t> match(const std::vector<float>& centroids_xy, uint32_t& n_need) {
        std::vector<int32_t> st(centroids_xy.size() / 2);
        check(cg_tracker_match(t_, centroids_xy.empty() ? nullptr : centroids_xy.data(), (uint32_t)st.size(),
                               st.empty() ? nullptr : st.data(), &n_need));
        return st;
    }
    void commit(const std::vector<int32_t>* colours) {   // nullptr: the service call failed
        check(cg_tracker_commit(t_, colours ? colours->data() : nullptr, colours ? (uint32_t)colours->size() : 0u));
    }
    std::vector<float> cloud(int colour) const {          // (x, y) pairs
        const float* xy = nullptr;
        uint32_t n = 0;
        check(cg_tracker_cloud(t_, colour, &xy, &n));
        return std::vector<float>(xy, xy + 2 * (size_t)n);
    }
private:
    cg_tracker* t_ = nullptr;
};

// The colour classifier service (scripts/color_classifier_server.py:81-124) on the GPU: usable
// as the ColourService below. weights: CG_COLORNET_WEIGHTS floats (python -m
// cones_perception_amd.colornet dam_net.tflite dam_net.f32 writes them). Like the reference's
// handler it answers one colour per non-empty cloud, and fails the call (false) where the
// reference raises (a point outside the 15 image rows, an intensity outside [0, 255]).
class ColorClassifier : public Handle {
public:
    ColorClassifier(const std::vector<float>& weights, int device = 0) : Handle(default_params(), device) {
        check(cg_colornet_set(h_, weights.data(), (uint32_t)weights.size()));
    }
    bool operator()(const std::vector<PointCloud2>& cones, std::vector<int32_t>& colours) {
        std::vector<float> pts;
        std::vector<uint32_t> offs{0};
        for (const auto& m : cones) {   // pc2.read_points: x, y, z, intensity by field name
            const int32_t o[4] = {m.offset_of("x"), m.offset_of("y"), m.offset_of("z"), m.offset_of("intensity")};
            for (uint32_t r = 0; r < m.height; r++)
                for (uint32_t c = 0; c < m.width; c++) {
                    const uint8_t* p = m.data.data() + (size_t)r * m.row_step + (size_t)c * m.point_step;
                    for (int a = 0; a < 4; a++) {
                        float v = 0.f;
                        if (o[a] >= 0) std::memcpy(&v, p + o[a], 4);
                        pts.push_back(v);
                    }
                }
            offs.push_back((uint32_t)(pts.size() / 4));
        }
        std::vector<int32_t> st(cones.size());
        check(cg_classify_colors(h_, pts.empty() ? nullptr : pts.data(), offs.data(), (uint32_t)cones.size(),
                                 st.data(), nullptr, nullptr));
        colours.clear();
        for (int32_t c : st) {
            if (c == CG_COLOR_SKIPPED) continue;
            if (c < 0) return false;
            colours.push_back(c);
        }
        return true;
    }
private:
    static cg_params default_params() { cg_params p; cg_params_init(&p); return p; }
};

// The whole ConeDetector::cloud_handler (src/cone_detection.cpp:130-187): the hot path, tracking,
// the re-crop of cones that need a colour, the colour service (a callback standing in for
// ClassifyColorSrv: it gets one PointXYZI message per cone, frame_id = cones_frame_id, and returns
// false for a failed call) and the four messages published on cones_topics (index = colour),
// each with the input's header and field list (lines 182-183). DETECTOR is ConeDetector, or
// ConePipeline for the fused ground_removal:=true composition.
using ColourService = std::function<bool(const std::vector<PointCloud2>& cones, std::vector<int32_t>& colours)>;

template <class DETECTOR>
class ConeDetectorNode {
public:
    ConeDetectorNode(const cg_params& p, const cg_track_params& tp, ColourService service = nullptr,
                     std::string cones_frame_id = "cloud", int device = 0)
        : detector(p, device), tracker(tp), service_(std::move(service)), frame_id_(std::move(cones_frame_id)) {}

    std::array<PointCloud2, CG_NUM_COLORS> cloud_handler(const PointCloud2& msg) {
        last = detector.cloud_handler(msg);
        uint32_t n_need = 0;
        const std::vector<int32_t> st = tracker.match(last.centroids, n_need);
        std::vector<int32_t> colours;
        bool ok = false;
        if (n_need) {
            std::vector<float> need;
            for (size_t c = 0; c < st.size(); c++)
                if (st[c] == CG_TRACK_NEED_COLOR) need.insert(need.end(), {last.centroids[2 * c], last.centroids[2 * c + 1]});
            std::vector<PointCloud2> cones;
            for (const auto& crop : detector.recrop(need)) {
                cones.push_back(to_ros_msg(crop));
                cones.back().header.frame_id = frame_id_;
            }
            // the response may be shorter than the request (the reference's server skips empty
            // crops); the tracker applies it positionally (src/cone_detection.cpp:328,357-358)
            ok = service_ && service_(cones, colours);
        }
        tracker.commit(ok ? &colours : nullptr);
        std::array<PointCloud2, CG_NUM_COLORS> out;
        for (int i = 0; i < CG_NUM_COLORS; i++) {
            const std::vector<float> xy = tracker.cloud(i);
            std::vector<float> xyzi;
            for (size_t k = 0; k < xy.size() / 2; k++) xyzi.insert(xyzi.end(), {xy[2 * k], xy[2 * k + 1], 0.f, 0.f});
            out[i] = to_ros_msg(xyzi);
            out[i].header = msg.header;   // line 182
            out[i].fields = msg.fields;   // line 183
        }
        return out;
    }

    DETECTOR detector;
    ConeTracker tracker;
    Detection last;
private:
    ColourService service_;
    std::string frame_id_;
};

}  // namespace cones_gpu
