// cg_oracle.cpp — CPU restatement of the dmn-sjk/cones_perception LiDAR hot path.
//
// TEST INFRASTRUCTURE ONLY. Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
// leg may load this library, and only as the checker / the timed CPU baseline. The product
// (cones_perception_amd, libcones_gpu.so) never links or calls it.
//
// PARITY UNPINNED: the reference ships no tests, golden vectors or fixtures (SURVEY.md §4,
// §8c), and it cannot be built here (ROS, PCL 1.10, FLANN 1.9.1, Eigen and Boost are absent).
// This file restates, from the reference sources and from PCL 1.10 / FLANN 1.9.1 as shipped
// with ROS Noetic (not present here, restated from their published algorithms):
//   decode            pcl::fromROSMsg field mapping by name           src/ground_removal.cpp:54
//   ground removal    GroundRemover::cloud_handler                    src/ground_removal.cpp:56-79
//   position filter   ConeDetector::filter_points_position            src/cone_detection.cpp:189-204
//   distance          perception_handling::euclidan_dist              src/perception_handling/utils.cpp:32-34
//   voxel grid        pcl::VoxelGrid<PointXYZI>::applyFilter (1.10)   called src/cone_detection.cpp:240-249
//   clustering        pcl::extractEuclideanClusters + KdTreeFLANN     called src/cone_detection.cpp:206-220
//                     (default: the exact L2_Simple radius predicate; checker mode SEARCH_FLANN:
//                     FLANN 1.9.1's own KDTreeSingleIndex and float-pruned search, FlannIndex)
//   cluster order     std::sort(clusters.rbegin(), rend(), size<)     (EuclideanClusterExtraction::extract)
//   centroid          ConeDetector::get_centroid_clouds (centroid)    src/cone_detection.cpp:261-279
//   re-crop           ConeDetector::get_reconstructed_cone            src/cone_detection.cpp:222-238
//   tracking          ConeDetector::get_centroid_clouds (matching)    src/cone_detection.cpp:251-339
//                     with the colour service as a callback           src/cone_detection.cpp:342-363
// libm calls (atan2f, sqrt, pow, floorf) go to the host glibc, as in the reference build.
// Compiled with -O2 -ffp-contract=off and no -march flags (a stock x86-64 Noetic build has no
// FMA). Defined divergences from the reference's undefined behaviour:
//   G3  sector 16 (angles in [352,360) deg) is its own bin initialised to default_lowest_point;
//       a NaN angle uses a never-updated bin (the reference indexes with int(NaN)).
//   C1  the first cluster's x sum starts at 0 (uninitialised in src/cone_detection.cpp:264).
// Voxel summation order: VOXEL_ORDER_PCL sorts with std::sort exactly as PCL (unstable
// introsort order); VOXEL_ORDER_STABLE sums each voxel in ascending point index (the device
// path's order). Both are exposed so tests can count where they differ.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <vector>

namespace {

struct Params {
    int32_t num_of_sectors;
    float default_lowest_point;
    double distance_treshold_max, distance_treshold_min, level_threshold, angle_threshold;
    int32_t min_cluster_size, max_cluster_size;
    double cone_position_extension_length;
    double voxel_filter_leaf_size_x, voxel_filter_leaf_size_y, voxel_filter_leaf_size_z;
    double cones_matching_dist_theshold;
};  // layout-identical to cg_params (include/cones_gpu.h)

struct View {
    const void* data;
    uint32_t width, height, point_step, row_step;
    int32_t off_x, off_y, off_z, off_intensity;
    uint8_t is_dense;
};  // layout-identical to cg_cloud_view

// pcl::PointXYZI: x,y,z, data[3] = 1, intensity, padding (32 bytes).
struct Pt {
    float x = 0.f, y = 0.f, z = 0.f, w = 1.f;
    float intensity = 0.f, pad[3] = {0.f, 0.f, 0.f};
};

float read_f32(const uint8_t* p, int32_t off) {
    if (off < 0) return 0.f;
    float v;
    std::memcpy(&v, p + off, 4);
    return v;
}

// pcl::fromROSMsg: row-major over height x width, fields copied by offset.
std::vector<Pt> decode(const View& v) {
    std::vector<Pt> out((size_t)v.width * v.height);
    const uint8_t* base = (const uint8_t*)v.data;
    for (uint32_t r = 0; r < v.height; r++)
        for (uint32_t c = 0; c < v.width; c++) {
            const uint8_t* p = base + (size_t)r * v.row_step + (size_t)c * v.point_step;
            Pt& q = out[(size_t)r * v.width + c];
            q.x = read_f32(p, v.off_x);
            q.y = read_f32(p, v.off_y);
            q.z = read_f32(p, v.off_z);
            q.intensity = read_f32(p, v.off_intensity);
        }
    return out;
}

// ---------------- ground removal: src/ground_removal.cpp:56-79 ----------------
const float kSectorAngleRad = (float)((360 / 16) * M_PI / 180);  // member init, ground_removal.cpp:20

int sector_of(float y, float x) {
    float atan_angle = atan2f(y, x);
    float angle = (atan_angle < 0) ? atan_angle += 2 * M_PI : atan_angle;
    if (std::isnan(angle)) return 17;                     // defined: NaN bin, never updated
    return (int)std::floor(angle / kSectorAngleRad);      // 0..16
}

size_t ground_remove(std::vector<Pt>& cloud, const Params& prm) {
    const size_t n = cloud.size();
    std::vector<float> lowest(18, prm.default_lowest_point);   // 17 addressed bins + NaN bin
    for (const Pt& p : cloud) {
        int s = sector_of(p.y, p.x);
        if (s < 17 && lowest[s] > p.z) lowest[s] = p.z;
    }
    auto it = std::remove_if(cloud.begin(), cloud.end(), [&](const Pt& p) {
        return p.z < lowest[sector_of(p.y, p.x)] + 0.1;   // float + double -> double compare
    });
    cloud.erase(it, cloud.end());
    size_t kept = cloud.size();
    cloud.resize(n);    // PointCloud::resize(n): appends PointXYZI()
    return kept;
}

// ---------------- detector: src/cone_detection.cpp:189-204 ----------------
float euclidan_dist(float x1, float y1, float z1, float x2, float y2, float z2) {
    return std::sqrt(std::pow(x1 - x2, 2) + std::pow(y1 - y2, 2) + std::pow(z1 - z2, 2));
}

void filter_points_position(std::vector<Pt>& cloud, const Params& prm) {
    auto it = std::remove_if(cloud.begin(), cloud.end(), [&](const Pt& p) {
        return p.z < prm.level_threshold ||
               euclidan_dist(p.x, p.y, p.z, 0, 0, 0) > prm.distance_treshold_max ||
               euclidan_dist(p.x, p.y, p.z, 0, 0, 0) < prm.distance_treshold_min ||
               -prm.angle_threshold * M_PI / 180 >= atan2f(p.y, p.x) ||
               atan2f(p.y, p.x) >= prm.angle_threshold * M_PI / 180;
    });
    cloud.erase(it, cloud.end());
}

// ---------------- pcl::VoxelGrid<PointXYZI>::applyFilter (PCL 1.10) ----------------
struct IdxPair {
    unsigned int idx, cloud_point_index;
    bool operator<(const IdxPair& o) const { return idx < o.idx; }
};

bool voxel_grid(const std::vector<Pt>& in, bool is_dense, const Params& prm, int order,
                std::vector<Pt>& out) {
    // setLeafSize(float,float,float): inverse = Ones / leaf (float division)
    const float leaf[3] = {(float)prm.voxel_filter_leaf_size_x, (float)prm.voxel_filter_leaf_size_y,
                           (float)prm.voxel_filter_leaf_size_z};
    const float inv[3] = {1.0f / leaf[0], 1.0f / leaf[1], 1.0f / leaf[2]};
    auto finite = [](const Pt& p) {
        return std::isfinite(p.x) && std::isfinite(p.y) && std::isfinite(p.z);
    };
    // getMinMax3D (skips non-finite when !is_dense; our inputs treat NaN that way always)
    float mn[3] = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(),
                   std::numeric_limits<float>::max()};
    float mx[3] = {-std::numeric_limits<float>::max(), -std::numeric_limits<float>::max(),
                   -std::numeric_limits<float>::max()};
    size_t nfin = 0;
    for (const Pt& p : in) {
        if (!finite(p)) continue;
        nfin++;
        const float c[3] = {p.x, p.y, p.z};
        for (int a = 0; a < 3; a++) { mn[a] = std::min(mn[a], c[a]); mx[a] = std::max(mx[a], c[a]); }
    }
    (void)is_dense;
    out.clear();
    if (nfin == 0) return false;
    // overflow guard: output = *input_
    int64_t d[3];
    for (int a = 0; a < 3; a++) {
        float span = (mx[a] - mn[a]) * inv[a];
        d[a] = span >= 9.0e18f ? (int64_t)9e18 : (int64_t)span + 1;
    }
    const double prod = (double)d[0] * (double)d[1] * (double)d[2];
    if (prod > (double)std::numeric_limits<int32_t>::max()) {
        out = in;
        return true;
    }
    int min_b[3], max_b[3], div_b[3];
    for (int a = 0; a < 3; a++) {
        min_b[a] = (int)std::floor(mn[a] * inv[a]);
        max_b[a] = (int)std::floor(mx[a] * inv[a]);
        div_b[a] = max_b[a] - min_b[a] + 1;
    }
    const int mul[3] = {1, div_b[0], div_b[0] * div_b[1]};
    std::vector<IdxPair> index_vector;
    index_vector.reserve(in.size());
    for (size_t i = 0; i < in.size(); i++) {
        const Pt& p = in[i];
        if (!finite(p)) continue;
        int ijk0 = (int)(std::floor(p.x * inv[0]) - (float)min_b[0]);
        int ijk1 = (int)(std::floor(p.y * inv[1]) - (float)min_b[1]);
        int ijk2 = (int)(std::floor(p.z * inv[2]) - (float)min_b[2]);
        unsigned int idx = (unsigned int)ijk0 * (unsigned)mul[0] + (unsigned int)ijk1 * (unsigned)mul[1] +
                           (unsigned int)ijk2 * (unsigned)mul[2];
        index_vector.push_back({idx, (unsigned int)i});
    }
    if (order == 1) std::sort(index_vector.begin(), index_vector.end(), std::less<IdxPair>());
    else std::stable_sort(index_vector.begin(), index_vector.end(), std::less<IdxPair>());
    size_t index = 0;
    while (index < index_vector.size()) {
        size_t i = index + 1;
        while (i < index_vector.size() && index_vector[i].idx == index_vector[index].idx) ++i;
        // CentroidPoint<PointXYZI>: float sums of x,y,z and intensity, then / float(n)
        float sx = 0.f, sy = 0.f, sz = 0.f, si = 0.f;
        for (size_t li = index; li < i; li++) {
            const Pt& p = in[index_vector[li].cloud_point_index];
            sx += p.x; sy += p.y; sz += p.z; si += p.intensity;
        }
        const float n = (float)(i - index);
        Pt c;
        c.x = sx / n; c.y = sy / n; c.z = sz / n; c.intensity = si / n;
        out.push_back(c);
        index = i;
    }
    return false;
}

// ---------------- radius search: KdTreeFLANN / FLANN KDTreeSingleIndex ----------------
// Leaf size 15 as PCL configures FLANN. Distances are FLANN L2_Simple<float>:
// acc = 0; acc += (q-p)^2 over x, y, z in float; neighbour iff acc < r2 (strict).
// Results sorted by (distance, index) (KdTree(sorted = true)). Pruning is conservative so the
// result is the exact float predicate over all points.
struct KdTree {
    struct Node { int lo, hi, left, right, dim; float split; };
    const std::vector<Pt>* pts = nullptr;
    std::vector<int> idx;
    std::vector<Node> nodes;

    int build(int lo, int hi) {
        Node nd{lo, hi, -1, -1, 0, 0.f};
        if (hi - lo > 15) {
            float bmin[3] = {INFINITY, INFINITY, INFINITY}, bmax[3] = {-INFINITY, -INFINITY, -INFINITY};
            for (int i = lo; i < hi; i++) {
                const Pt& p = (*pts)[idx[i]];
                const float c[3] = {p.x, p.y, p.z};
                for (int a = 0; a < 3; a++) { bmin[a] = std::min(bmin[a], c[a]); bmax[a] = std::max(bmax[a], c[a]); }
            }
            int dim = 0;
            for (int a = 1; a < 3; a++) if (bmax[a] - bmin[a] > bmax[dim] - bmin[dim]) dim = a;
            int mid = (lo + hi) / 2;
            auto key = [&](int i) { const Pt& p = (*pts)[i]; return dim == 0 ? p.x : dim == 1 ? p.y : p.z; };
            std::nth_element(idx.begin() + lo, idx.begin() + mid, idx.begin() + hi,
                             [&](int a, int b) { return key(a) < key(b); });
            nd.dim = dim;
            nd.split = key(idx[mid]);
            int me = (int)nodes.size();
            nodes.push_back(nd);
            int l = build(lo, mid), r = build(mid, hi);
            nodes[me].left = l; nodes[me].right = r;
            return me;
        }
        nodes.push_back(nd);
        return (int)nodes.size() - 1;
    }
    void init(const std::vector<Pt>& p) {
        pts = &p;
        idx.resize(p.size());
        for (size_t i = 0; i < p.size(); i++) idx[i] = (int)i;
        nodes.clear();
        if (!p.empty()) build(0, (int)p.size());
    }
    void search(int node, const Pt& q, float r2, double rr, std::vector<std::pair<float, int>>& res) const {
        const Node& nd = nodes[node];
        if (nd.left < 0) {
            for (int i = nd.lo; i < nd.hi; i++) {
                const Pt& p = (*pts)[idx[i]];
                float acc = 0.f, diff;
                diff = q.x - p.x; acc += diff * diff;
                diff = q.y - p.y; acc += diff * diff;
                diff = q.z - p.z; acc += diff * diff;
                if (acc < r2) res.push_back({acc, idx[i]});
            }
            return;
        }
        const float qv = nd.dim == 0 ? q.x : nd.dim == 1 ? q.y : q.z;
        const double gap = (double)qv - (double)nd.split;     // exact in double
        const int first = gap < 0 ? nd.left : nd.right, second = gap < 0 ? nd.right : nd.left;
        search(first, q, r2, rr, res);
        if (gap * gap <= rr) search(second, q, r2, rr, res);
    }
    void radius(const Pt& q, float r2, std::vector<std::pair<float, int>>& res) const {
        res.clear();
        if (nodes.empty()) return;
        search(0, q, r2, (double)r2 * 1.0001 + 1e-12, res);
        std::sort(res.begin(), res.end());   // (dist, index)
    }
};

// ---------------- checker mode: FLANN 1.9.1's own tree and search ----------------
// The exact predicate above assumes FLANN returns every point with acc < r2. FLANN prunes with
// a float lower bound that it updates incrementally, which could in principle overshoot by an
// ulp and drop a neighbour within a few ulps of r2. This restates the search PCL 1.10 actually
// runs, so the assumption can be checked frame by frame (tests/test_flann.py, bench parity):
//   pcl::search::KdTree<PointXYZI>(sorted = true) -> pcl::KdTreeFLANN<PointXYZI,
//   flann::L2_Simple<float>>::setInputCloud: x, y, z of every valid point, in cloud order,
//   flann::KDTreeSingleIndex with KDTreeSingleIndexParams(15) (leaf_max_size 15, reorder true);
//   radiusSearch: r2 = float(radius * radius) (radius a double), SearchParams(checks -1,
//   eps 0, sorted true), max_neighbors -1: RadiusResultSet, KDTreeSingleIndex::findNeighbors.
// FLANN 1.9.1 (flann/algorithms/kdtree_single_index.h, flann/util/result_set.h) is not in this
// image or in the reference; restated from its published source:
//   buildIndex: vind = 0..N-1, root bbox = per-dim min / max over all points, divideTree;
//   divideTree(left, right, bbox&): a leaf when right - left <= leaf_max_size (bbox := its
//     points' bounds); else middleSplit_ on the CELL bbox it was given, child1 over
//     [left, left + idx) with bbox[cutfeat].high = cutval, child2 over the rest with
//     bbox[cutfeat].low = cutval; divlow / divhigh = the children's actual bounds in cutfeat;
//     bbox := the union of the children's actual bounds;
//   middleSplit_: max_span over the cell's dims; among dims with span > (1 - 1e-5f) * max_span
//     the one of largest actual spread of the points (first on ties); split_val = the cell's
//     middle, clamped to the points' [min, max]; planeSplit gives lim1 (< cutval first), lim2
//     (<= cutval); index = lim1 if lim1 > count / 2, else lim2 if lim2 < count / 2, else count / 2;
//   findNeighbors: epsError = 1 + eps = 1; dists[] = 0 and distsq = 0 for a query inside the
//     root bbox (computeInitialDistances); searchLevel: leaf -> every point with
//     L2_Simple acc < worstDist() (= r2) is added; inner node -> diff1 = val - divlow,
//     diff2 = val - divhigh, the nearer child first (diff1 + diff2 < 0: child1), then
//     mindistsq = mindistsq + cut_dist - dists[idx] (float), the other child only if
//     mindistsq * epsError <= r2;
//   copy(sorted): std::sort of (dist, index) pairs, DistIndex::operator< (dist, then index).
// All of it in float (DistanceType = ElementType = float), no contraction (-ffp-contract=off).
struct FlannIndex {
    struct Node { int left = 0, right = 0, divfeat = 0; float divlow = 0.f, divhigh = 0.f; int child1 = -1, child2 = -1; };
    struct Iv { float low, high; };
    static constexpr int kLeafMax = 15;
    std::vector<float> pts;    // points_: N x 3 (the KdTreeFLANN array)
    std::vector<int> vind;
    std::vector<Node> nodes;
    std::vector<Iv> root_bbox;
    int root = -1;

    float at(int i, int d) const { return pts[3 * (size_t)i + d]; }
    void compute_min_max(const int* ind, int count, int dim, float& mn, float& mx) const {
        mn = at(ind[0], dim);
        mx = at(ind[0], dim);
        for (int i = 1; i < count; ++i) {
            const float v = at(ind[i], dim);
            if (v < mn) mn = v;
            if (v > mx) mx = v;
        }
    }
    void plane_split(int* ind, int count, int cutfeat, float cutval, int& lim1, int& lim2) const {
        int left = 0, right = count - 1;
        for (;;) {
            while (left <= right && at(ind[left], cutfeat) < cutval) ++left;
            while (left <= right && at(ind[right], cutfeat) >= cutval) --right;
            if (left > right) break;
            std::swap(ind[left], ind[right]); ++left; --right;
        }
        lim1 = left;
        right = count - 1;
        for (;;) {
            while (left <= right && at(ind[left], cutfeat) <= cutval) ++left;
            while (left <= right && at(ind[right], cutfeat) > cutval) --right;
            if (left > right) break;
            std::swap(ind[left], ind[right]); ++left; --right;
        }
        lim2 = left;
    }
    void middle_split(int* ind, int count, int& index, int& cutfeat, float& cutval, const std::vector<Iv>& bbox) const {
        const float EPS = 0.00001f;
        float max_span = bbox[0].high - bbox[0].low;
        for (int i = 1; i < 3; ++i) {
            const float span = bbox[i].high - bbox[i].low;
            if (span > max_span) max_span = span;
        }
        float max_spread = -1;
        cutfeat = 0;
        for (int i = 0; i < 3; ++i) {
            const float span = bbox[i].high - bbox[i].low;
            if (span > (1 - EPS) * max_span) {
                float mn, mx;
                compute_min_max(ind, count, i, mn, mx);
                const float spread = mx - mn;
                if (spread > max_spread) { cutfeat = i; max_spread = spread; }
            }
        }
        const float split_val = (bbox[cutfeat].low + bbox[cutfeat].high) / 2;
        float mn, mx;
        compute_min_max(ind, count, cutfeat, mn, mx);
        if (split_val < mn) cutval = mn;
        else if (split_val > mx) cutval = mx;
        else cutval = split_val;
        int lim1, lim2;
        plane_split(ind, count, cutfeat, cutval, lim1, lim2);
        if (lim1 > count / 2) index = lim1;
        else if (lim2 < count / 2) index = lim2;
        else index = count / 2;
    }
    int divide(int left, int right, std::vector<Iv>& bbox) {
        const int me = (int)nodes.size();
        nodes.emplace_back();
        if (right - left <= kLeafMax) {
            nodes[me].left = left; nodes[me].right = right;
            for (int i = 0; i < 3; ++i) bbox[i].low = bbox[i].high = at(vind[left], i);
            for (int k = left + 1; k < right; ++k)
                for (int i = 0; i < 3; ++i) {
                    if (bbox[i].low > at(vind[k], i)) bbox[i].low = at(vind[k], i);
                    if (bbox[i].high < at(vind[k], i)) bbox[i].high = at(vind[k], i);
                }
            return me;
        }
        int idx, cutfeat;
        float cutval;
        middle_split(&vind[0] + left, right - left, idx, cutfeat, cutval, bbox);
        nodes[me].divfeat = cutfeat;
        std::vector<Iv> left_bbox(bbox);
        left_bbox[cutfeat].high = cutval;
        const int c1 = divide(left, left + idx, left_bbox);
        std::vector<Iv> right_bbox(bbox);
        right_bbox[cutfeat].low = cutval;
        const int c2 = divide(left + idx, right, right_bbox);
        nodes[me].child1 = c1; nodes[me].child2 = c2;
        nodes[me].divlow = left_bbox[cutfeat].high;
        nodes[me].divhigh = right_bbox[cutfeat].low;
        for (int i = 0; i < 3; ++i) {
            bbox[i].low = std::min(left_bbox[i].low, right_bbox[i].low);
            bbox[i].high = std::max(left_bbox[i].high, right_bbox[i].high);
        }
        return me;
    }
    void build(const std::vector<Pt>& cloud) {
        pts.clear();
        for (const Pt& p : cloud) pts.insert(pts.end(), {p.x, p.y, p.z});
        const int n = (int)cloud.size();
        vind.resize(n);
        for (int i = 0; i < n; i++) vind[i] = i;
        nodes.clear();
        root = -1;
        if (n == 0) return;
        root_bbox.assign(3, Iv{0.f, 0.f});
        for (int i = 0; i < 3; ++i) root_bbox[i].low = root_bbox[i].high = at(0, i);
        for (int k = 1; k < n; ++k)
            for (int i = 0; i < 3; ++i) {
                if (at(k, i) < root_bbox[i].low) root_bbox[i].low = at(k, i);
                if (at(k, i) > root_bbox[i].high) root_bbox[i].high = at(k, i);
            }
        root = divide(0, n, root_bbox);
    }
    void search_level(std::vector<std::pair<float, int>>& res, const float* vec, int node, float mindistsq,
                      float* dists, float r2) const {
        const Node& nd = nodes[node];
        if (nd.child1 < 0 && nd.child2 < 0) {
            const float worst_dist = r2;
            for (int i = nd.left; i < nd.right; ++i) {
                const int j = vind[i];   // data_[i] (reordered) holds points_[vind_[i]]
                float result = 0.f, diff;
                for (int d = 0; d < 3; ++d) {
                    diff = vec[d] - at(j, d);
                    result += diff * diff;
                }
                if (result < worst_dist) res.push_back({result, j});   // (RadiusResultSet: dist < radius)
            }
            return;
        }
        const int idx = nd.divfeat;
        const float val = vec[idx];
        const float diff1 = val - nd.divlow, diff2 = val - nd.divhigh;
        int best, other;
        float cut_dist;
        if ((diff1 + diff2) < 0) {
            best = nd.child1; other = nd.child2;
            cut_dist = (val - nd.divhigh) * (val - nd.divhigh);
        } else {
            best = nd.child2; other = nd.child1;
            cut_dist = (val - nd.divlow) * (val - nd.divlow);
        }
        search_level(res, vec, best, mindistsq, dists, r2);
        const float dst = dists[idx];
        mindistsq = mindistsq + cut_dist - dst;
        dists[idx] = cut_dist;
        if (mindistsq * 1.0f <= r2) search_level(res, vec, other, mindistsq, dists, r2);
        dists[idx] = dst;
    }
    void radius(const Pt& q, float r2, std::vector<std::pair<float, int>>& res) const {
        res.clear();
        if (root < 0) return;
        const float vec[3] = {q.x, q.y, q.z};
        float dists[3] = {0.f, 0.f, 0.f};
        float distsq = 0.f;
        for (int i = 0; i < 3; ++i) {   // computeInitialDistances
            if (vec[i] < root_bbox[i].low) { dists[i] = (vec[i] - root_bbox[i].low) * (vec[i] - root_bbox[i].low); distsq += dists[i]; }
            if (vec[i] > root_bbox[i].high) { dists[i] = (vec[i] - root_bbox[i].high) * (vec[i] - root_bbox[i].high); distsq += dists[i]; }
        }
        search_level(res, vec, root, distsq, dists, r2);
        std::sort(res.begin(), res.end());   // DistIndex: (dist, index)
    }
};

enum { SEARCH_EXACT = 0, SEARCH_FLANN = 1 };

// pcl::extractEuclideanClusters (PCL 1.10) + EuclideanClusterExtraction::extract ordering.
std::vector<std::vector<int>> euclidean_clusters(const std::vector<Pt>& cloud, float tolerance,
                                                 unsigned min_pts, unsigned max_pts, int search = SEARCH_EXACT) {
    std::vector<std::vector<int>> clusters;
    if (cloud.empty()) return clusters;
    KdTree tree;
    FlannIndex flann;
    if (search == SEARCH_FLANN) flann.build(cloud);
    else tree.init(cloud);
    const float r2 = (float)((double)tolerance * (double)tolerance);   // KdTreeFLANN::radiusSearch
    const size_t nn_start_idx = 1;                                     // sorted results
    std::vector<bool> processed(cloud.size(), false);
    std::vector<std::pair<float, int>> nn;
    for (size_t i = 0; i < cloud.size(); i++) {
        if (processed[i]) continue;
        std::vector<int> seed_queue{(int)i};
        processed[i] = true;
        for (size_t sq = 0; sq < seed_queue.size(); sq++) {
            if (search == SEARCH_FLANN) flann.radius(cloud[seed_queue[sq]], r2, nn);
            else tree.radius(cloud[seed_queue[sq]], r2, nn);
            for (size_t j = nn_start_idx; j < nn.size(); j++) {
                int k = nn[j].second;
                if (processed[k]) continue;
                seed_queue.push_back(k);
                processed[k] = true;
            }
        }
        if (seed_queue.size() >= min_pts && seed_queue.size() <= max_pts) {
            std::sort(seed_queue.begin(), seed_queue.end());
            seed_queue.erase(std::unique(seed_queue.begin(), seed_queue.end()), seed_queue.end());
            clusters.push_back(seed_queue);
        }
    }
    std::sort(clusters.rbegin(), clusters.rend(),
              [](const std::vector<int>& a, const std::vector<int>& b) { return a.size() < b.size(); });
    return clusters;
}

struct Out {
    uint32_t* hdr;      // [8]: N, K, M, V, C, flags, duplicate voxel points, 0
    float* ground;      // N x 8 floats (mode 2) or null
    float* voxels;      // V x 4
    int32_t* labels;    // V
    int32_t* offsets;   // C + 1
    int32_t* indices;   // offsets[C]
    float* centroids;   // C x 2
};

// ConeDetector constants (src/cone_detection.cpp:22-23) and the tolerance (line 212): the double
// sqrt, passed to setClusterTolerance (double) and on to extractEuclideanClusters as a float.
float cluster_tolerance() {
    const float CONE_WIDTH = 0.228, CONE_HEIGHT = 0.325;
    return (float)std::sqrt(std::pow(CONE_HEIGHT, 2) + std::pow(CONE_WIDTH, 2));
}

void detect(std::vector<Pt>& cloud, bool is_dense, const Params& prm, int order, Out& o, int search = SEARCH_EXACT) {
    filter_points_position(cloud, prm);
    o.hdr[2] = (uint32_t)cloud.size();
    std::vector<Pt> vox;
    bool passthrough = voxel_grid(cloud, is_dense, prm, order, vox);
    o.hdr[3] = (uint32_t)vox.size();
    o.hdr[5] = passthrough ? 1u : 0u;
    auto clusters = euclidean_clusters(vox, cluster_tolerance(), (unsigned)prm.min_cluster_size,
                                       (unsigned)prm.max_cluster_size, search);
    o.hdr[4] = (uint32_t)clusters.size();
    // duplicate (bit-identical) voxel points break the nn_start_idx = 1 assumption (rule E2)
    {
        std::vector<std::tuple<uint32_t, uint32_t, uint32_t>> keys;
        keys.reserve(vox.size());
        for (const Pt& p : vox) {
            uint32_t a, b, c;
            std::memcpy(&a, &p.x, 4); std::memcpy(&b, &p.y, 4); std::memcpy(&c, &p.z, 4);
            keys.emplace_back(a, b, c);
        }
        std::sort(keys.begin(), keys.end());
        uint32_t dups = 0;
        for (size_t i = 1; i < keys.size(); i++) dups += keys[i] == keys[i - 1];
        o.hdr[6] = dups;
    }
    for (size_t v = 0; v < vox.size(); v++) {
        o.voxels[4 * v + 0] = vox[v].x; o.voxels[4 * v + 1] = vox[v].y;
        o.voxels[4 * v + 2] = vox[v].z; o.voxels[4 * v + 3] = vox[v].intensity;
        o.labels[v] = -1;
    }
    int32_t off = 0;
    for (size_t c = 0; c < clusters.size(); c++) {
        o.offsets[c] = off;
        // src/cone_detection.cpp:261-279 (x starts at 0: rule C1)
        float x = 0.0f, y = 0.0f;
        int j = 0;
        for (int idx : clusters[c]) {
            x += vox[idx].x;
            y += vox[idx].y;
            j++;
            o.indices[off++] = idx;
            o.labels[idx] = (int32_t)c;
        }
        float px = x / j, py = y / j, pz = 0.0f;
        float vector_len = euclidan_dist(px, py, pz, 0, 0, 0);
        px = px + px / vector_len * prm.cone_position_extension_length;
        py = py + py / vector_len * prm.cone_position_extension_length;
        o.centroids[2 * c + 0] = px;
        o.centroids[2 * c + 1] = py;
    }
    o.offsets[clusters.size()] = off;
}

// ---------------- detector node after the hot path ----------------
// ConeDetector::get_reconstructed_cone (src/cone_detection.cpp:222-238): the whole cloud's
// points within CONE_WIDTH / 1.5 of the centre in x and in y, double compares, in cloud order.
const float kConeWidth = 0.228;   // src/cone_detection.cpp:22

std::vector<Pt> reconstructed_cone(const Pt& centre, const std::vector<Pt>& whole) {
    const double half = kConeWidth / 1.5;
    std::vector<Pt> crop;
    for (const Pt& q : whole) {
        const bool in_x = centre.x + half >= q.x && centre.x - half <= q.x;
        const bool in_y = centre.y + half >= q.y && centre.y - half <= q.y;
        if (!(in_x && in_y)) continue;
        Pt r;   // a fresh PointXYZI with the four fields copied
        r.x = q.x; r.y = q.y; r.z = q.z; r.intensity = q.intensity;
        crop.push_back(r);
    }
    return crop;
}

// The whole cloud get_centroid_clouds receives (input_cloud_copy, src/cone_detection.cpp:158):
// the decoded detector input; for the fused pipeline, the ground node's output.
std::vector<Pt> whole_cloud(const View& v, int mode, const Params& prm) {
    std::vector<Pt> cloud = decode(v);
    if (mode == 0) ground_remove(cloud, prm);
    return cloud;
}

// The colour service call (src/cone_detection.cpp:342-363): the request is every crop
// (xyzi floats, crop k at offsets[k]..offsets[k+1]); the callback writes the response colours
// (at most cap) and returns their count, or -1 for a failed call. The reference's server
// answers only non-empty crops (scripts/color_classifier_server.py:83-84), so a response may
// be shorter than the request; the test's restatement of the server decides that.
typedef int (*ServiceFn)(void* ctx, const float* xyzi, const uint32_t* offsets, uint32_t n_crops, int32_t* colours,
                         uint32_t cap);

// ConeDetector's tracking state (src/cone_detection.cpp:60-63): null until the first frame.
struct Node {
    bool classify_colors = true, use_points_buffer = false;
    double matching = 0.5;
    std::unique_ptr<std::vector<Pt>> prev_detected;
    std::unique_ptr<std::vector<Pt>> prev_clouds[4];
};

bool matches(const Node& nd, const Pt& a, const Pt& b) {
    return euclidan_dist(a.x, a.y, a.z, b.x, b.y, b.z) < nd.matching;
}

// get_centroid_clouds (src/cone_detection.cpp:251-339) after the centroid arithmetic: the
// centroids arrive in cluster order; clouds[i] receives what cones_pubs[i] publishes.
int centroid_clouds(Node& nd, const std::vector<Pt>& whole, const float* cen, uint32_t n, ServiceFn service,
                    void* ctx, std::vector<Pt> clouds[4]) {
    auto current = std::make_unique<std::vector<Pt>>();
    std::vector<std::vector<Pt>> to_classify;
    std::vector<Pt> to_classify_centroids;
    for (uint32_t c = 0; c < n; c++) {
        Pt p;
        p.x = cen[2 * c]; p.y = cen[2 * c + 1]; p.z = 0.0f;
        current->push_back(p);
        if (!nd.prev_detected) continue;
        for (const Pt& prev : *nd.prev_detected) {
            if (nd.use_points_buffer && !matches(nd, p, prev)) continue;
            if (!nd.classify_colors) {
                clouds[0].push_back(p);
                break;
            }
            int known = -1;
            for (int i = 1; i < 4 && known < 0; i++) {
                if (!nd.prev_clouds[i]) continue;
                for (const Pt& q : *nd.prev_clouds[i])
                    if (matches(nd, p, q)) { known = i; break; }
            }
            if (known >= 0) {
                clouds[known].push_back(p);
            } else {
                to_classify.push_back(reconstructed_cone(p, whole));
                to_classify_centroids.push_back(p);
            }
            break;
        }
    }
    if (nd.classify_colors) {
        // colors(n, kUnknownColor) (line 328); a successful call overwrites the first
        // len(response) entries in order, std::transform(resp.begin(), resp.end(), colors.begin())
        // (357-358); a failed call leaves them all unknown (359-361)
        const size_t n_req = to_classify.size();
        std::vector<int> colours(n_req, 0);
        std::vector<float> xyzi;
        std::vector<uint32_t> offs(1, 0);
        for (const std::vector<Pt>& crop : to_classify) {
            for (const Pt& q : crop) xyzi.insert(xyzi.end(), {q.x, q.y, q.z, q.intensity});
            offs.push_back((uint32_t)(xyzi.size() / 4));
        }
        std::vector<int32_t> resp(n_req + 1, 0);
        const int r = service ? service(ctx, xyzi.data(), offs.data(), (uint32_t)n_req, resp.data(),
                                        (uint32_t)resp.size())
                              : -1;
        if (r > (int)n_req) return -1;   // writes past colors' end in the reference (UB)
        for (int k = 0; k < r; k++) {
            if (resp[k] < 0 || resp[k] >= 4) return -1;
            colours[k] = resp[k];
        }
        for (size_t k = 0; k < n_req; k++) clouds[colours[k]].push_back(to_classify_centroids[k]);
    }
    for (int i = 0; i < 4; i++) nd.prev_clouds[i] = std::make_unique<std::vector<Pt>>(clouds[i]);
    nd.prev_detected = std::move(current);
    return 0;
}

}  // namespace

extern "C" {

// get_reconstructed_cone for n centres over the whole cloud of `view` (mode 0: the groundless
// cloud of the pipeline, 1: the detector input). offsets: n + 1; points: cap x 4 floats.
// Returns the total point count (which may exceed cap; then points holds the first cap).
uint32_t oracle_recrop(const void* params, const void* view, int mode, const float* centres, uint32_t n,
                       uint32_t* offsets, float* points, uint32_t cap) {
    const Params& prm = *(const Params*)params;
    const std::vector<Pt> whole = whole_cloud(*(const View*)view, mode, prm);
    uint32_t total = 0;
    offsets[0] = 0;
    for (uint32_t c = 0; c < n; c++) {
        Pt ctr;
        ctr.x = centres[2 * c]; ctr.y = centres[2 * c + 1]; ctr.z = 0.0f;
        for (const Pt& q : reconstructed_cone(ctr, whole)) {
            if (total < cap) {
                float* o = points + 4 * (size_t)total;
                o[0] = q.x; o[1] = q.y; o[2] = q.z; o[3] = q.intensity;
            }
            total++;
        }
        offsets[c + 1] = total;
    }
    return total;
}

void* oracle_node_create(int classify_colors, int use_points_buffer, double matching) {
    Node* nd = new Node;
    nd->classify_colors = classify_colors != 0;
    nd->use_points_buffer = use_points_buffer != 0;
    nd->matching = matching;
    return nd;
}
void oracle_node_destroy(void* node) { delete (Node*)node; }

// One frame of the node after the hot path: centroids (n x 2, cluster order) and the frame's
// whole cloud (view, mode as oracle_recrop). counts[4] = points per colour cloud; xy holds
// colour i's points at xy + i * cap * 2.
int oracle_node_step(void* node, const void* params, const void* view, int mode, const float* centroids,
                     uint32_t n, ServiceFn service, void* ctx, uint32_t* counts, float* xy, uint32_t cap) {
    const Params& prm = *(const Params*)params;
    const std::vector<Pt> whole = whole_cloud(*(const View*)view, mode, prm);
    std::vector<Pt> clouds[4];
    if (centroid_clouds(*(Node*)node, whole, centroids, n, service, ctx, clouds) != 0) return -1;
    for (int i = 0; i < 4; i++) {
        counts[i] = (uint32_t)clouds[i].size();
        for (size_t k = 0; k < clouds[i].size() && k < cap; k++) {
            xy[((size_t)i * cap + k) * 2] = clouds[i][k].x;
            xy[((size_t)i * cap + k) * 2 + 1] = clouds[i][k].y;
        }
    }
    return 0;
}

// mode: 0 = pipeline (ground removal then detector), 1 = detector only, 2 = ground only.
// order: 0 = stable voxel sums (device order), 1 = PCL std::sort order.
// search: 0 = the exact radius predicate (the default), 1 = FLANN 1.9.1's own tree and search.
// All output arrays must hold N entries (N+1 for offsets; 8N floats for ground).
int oracle_run_search(const void* params, const void* view, int mode, int order, int search, uint32_t* hdr,
                      float* ground, float* voxels, int32_t* labels, int32_t* offsets, int32_t* indices,
                      float* centroids) {
    const Params& prm = *(const Params*)params;
    const View& v = *(const View*)view;
    std::vector<Pt> cloud = decode(v);
    std::memset(hdr, 0, 8 * sizeof(uint32_t));
    hdr[0] = (uint32_t)cloud.size();
    hdr[1] = (uint32_t)cloud.size();
    if (mode == 0 || mode == 2) hdr[1] = (uint32_t)ground_remove(cloud, prm);
    if (mode == 2) {
        for (size_t i = 0; i < cloud.size(); i++) std::memcpy(ground + 8 * i, &cloud[i], 32);
        return 0;
    }
    Out o{hdr, ground, voxels, labels, offsets, indices, centroids};
    detect(cloud, v.is_dense != 0, prm, order, o, search);
    return 0;
}
int oracle_run(const void* params, const void* view, int mode, int order, uint32_t* hdr,
               float* ground, float* voxels, int32_t* labels, int32_t* offsets, int32_t* indices,
               float* centroids) {
    return oracle_run_search(params, view, mode, order, SEARCH_EXACT, hdr, ground, voxels, labels, offsets, indices,
                             centroids);
}

// The FLANN check of one frame (mode 0 / 1, voxel order as oracle_run): the voxel cloud the
// clustering sees, every voxel as a query through both searches, and both clusterings.
// stats (ORACLE_FLANN_WORDS words):
//   [0] V voxels                       [1] queries whose neighbour sets differ
//   [2] pairs the exact predicate has and FLANN's search misses (ordered: query, neighbour)
//   [3] pairs FLANN returns that the exact predicate lacks (ordered)
//   [4] near-tolerance pairs: unordered pairs whose float L2_Simple acc lies within 4 ulp of r2
//       (either side), the only pairs a float pruning error could drop
//   [5] of them, the pairs inside (acc < r2)
//   [6] 1 when both clusterings are identical (index sets and order)
//   [7] C exact                        [8] C FLANN
//   [9] ulps from r2 of the closest in-tolerance pair (acc < r2), 0xffffffff when none
int oracle_flann_check(const void* params, const void* view, int mode, int order, uint32_t* stats) {
    const Params& prm = *(const Params*)params;
    const View& v = *(const View*)view;
    std::memset(stats, 0, 10 * sizeof(uint32_t));
    stats[9] = 0xffffffffu;
    std::vector<Pt> cloud = decode(v);
    if (mode == 0) ground_remove(cloud, prm);
    filter_points_position(cloud, prm);
    std::vector<Pt> vox;
    voxel_grid(cloud, v.is_dense != 0, prm, order, vox);
    stats[0] = (uint32_t)vox.size();
    if (vox.empty()) { stats[6] = 1; return 0; }
    const float tol = cluster_tolerance();
    const float r2 = (float)((double)tol * (double)tol);
    KdTree tree;
    tree.init(vox);
    FlannIndex flann;
    flann.build(vox);
    uint32_t r2b;
    std::memcpy(&r2b, &r2, 4);
    std::vector<std::pair<float, int>> a, b, wide;
    const float wide_r2 = std::nextafter(r2, INFINITY) * 1.0001f;
    for (size_t i = 0; i < vox.size(); i++) {
        tree.radius(vox[i], r2, a);
        flann.radius(vox[i], r2, b);
        if (a != b) stats[1]++;
        size_t x = 0, y = 0;   // both sorted by (dist, index)
        while (x < a.size() || y < b.size()) {
            if (y == b.size() || (x < a.size() && a[x] < b[y])) { stats[2]++; x++; }
            else if (x == a.size() || b[y] < a[x]) { stats[3]++; y++; }
            else { x++; y++; }
        }
        tree.radius(vox[i], wide_r2, wide);   // candidates just past r2 too
        for (const auto& pr : wide) {
            if ((size_t)pr.second <= i) continue;   // unordered pairs, no self pair
            uint32_t ab;
            std::memcpy(&ab, &pr.first, 4);
            const uint32_t ulps = ab > r2b ? ab - r2b : r2b - ab;   // (both positive floats)
            if (ulps <= 4) {
                stats[4]++;
                if (pr.first < r2) stats[5]++;
            }
            if (pr.first < r2 && ulps < stats[9]) stats[9] = ulps;
        }
    }
    const auto ce = euclidean_clusters(vox, tol, (unsigned)prm.min_cluster_size, (unsigned)prm.max_cluster_size,
                                       SEARCH_EXACT);
    const auto cf = euclidean_clusters(vox, tol, (unsigned)prm.min_cluster_size, (unsigned)prm.max_cluster_size,
                                       SEARCH_FLANN);
    stats[6] = ce == cf ? 1u : 0u;
    stats[7] = (uint32_t)ce.size();
    stats[8] = (uint32_t)cf.size();
    return 0;
}

// FLANN's radius search alone on n points (xyz float triples) for every point as the query:
// out_counts[i] = its neighbour count, out_idx the neighbours (sorted by (dist, index)) up to
// cap in all. Returns the total. (tests: the restatement against brute force.)
uint32_t oracle_flann_radius_all(const float* xyz, uint32_t n, float r2, uint32_t* out_counts, int32_t* out_idx,
                                 uint32_t cap) {
    std::vector<Pt> c(n);
    for (uint32_t i = 0; i < n; i++) { c[i].x = xyz[3 * i]; c[i].y = xyz[3 * i + 1]; c[i].z = xyz[3 * i + 2]; }
    FlannIndex flann;
    flann.build(c);
    std::vector<std::pair<float, int>> res;
    uint32_t tot = 0;
    for (uint32_t i = 0; i < n; i++) {
        flann.radius(c[i], r2, res);
        out_counts[i] = (uint32_t)res.size();
        for (const auto& pr : res) {
            if (tot < cap) out_idx[tot] = pr.second;
            tot++;
        }
    }
    return tot;
}

// Host libm probes for the device-restatement checks.
float oracle_atan2f(float y, float x) { return atan2f(y, x); }
int oracle_sector(float y, float x) { return sector_of(y, x); }
double oracle_sqrt(double s) { return std::sqrt(s); }
float oracle_euclid(float x, float y, float z) { return euclidan_dist(x, y, z, 0, 0, 0); }

}  // extern "C"
