"""cones_perception_amd — MI355X (gfx950) LiDAR cone-detection hot path.

Python mirror of the reference's two ROS node interfaces over the C-ABI
(include/cones_gpu.h). The names follow the reference:

  GroundRemover.cloud_handler   src/ground_removal.cpp:50-89
  ConeDetector.cloud_handler    src/cone_detection.cpp:130-187 (up to the pre-tracking centroids)
  ConePipeline.cloud_handler    launch/cones_perception.launch:17-37 (ground_removal:=true)

Parameters use the YAML keys of config/*.yaml verbatim. All compute runs in the HIP library;
this module only marshals PointCloud2 bytes. Importing it without the built library raises.
"""
from dataclasses import dataclass, field
import ctypes as C
from typing import List, Optional

import numpy as np

from . import _abi
from ._abi import (CG_VOXEL_ORDER_PCL, CG_VOXEL_ORDER_POINT, CG_F_VOXEL_POINT_ORDER,  # noqa: F401
                   CG_MODE_DETECT, CG_MODE_PIPELINE, CG_F_GLOBAL_SCRATCH, CG_F_ORDER_CANONICAL,
                   CG_F_VOXEL_PASSTHROUGH, CgError, check, lib)

lib()   # fail loudly at import if the gfx950 library is missing

__all__ = ["PROFILES", "load_params", "PointField", "PointCloud2", "Detection", "GroundRemover",
           "ConeDetector", "ConePipeline", "BatchEngine", "synth_frames", "CgError", "ColorClassifier",
           "read_tflite"]

# ---------------------------------------------------------------------------------------
# Parameter profiles: the reference's config/*.yaml (keys verbatim, misspellings kept).
GROUND_PARAMS = {"num_of_sectors": 16, "default_lowest_point": -0.1}   # ground_removal_params.yaml
PROFILES = {
    # config/cones_detection_params_simulation.yaml:1-11 (the metric's profile)
    "simulation": {"cones_matching_dist_theshold": 0.5, "cone_position_extension_length": 0.05,
                   "distance_treshold_max": 10.0, "distance_treshold_min": 1.0,
                   "level_threshold": -5.0, "angle_threshold": 160.0,
                   "min_cluster_size": 2, "max_cluster_size": 500,
                   "voxel_filter_leaf_size_x": 0.04, "voxel_filter_leaf_size_y": 0.04,
                   "voxel_filter_leaf_size_z": 0.04},
    # config/cones_detection_params_our.yaml:1-11
    "our": {"cones_matching_dist_theshold": 0.5, "cone_position_extension_length": 0.05,
            "distance_treshold_max": 7.0, "distance_treshold_min": 0.7, "level_threshold": -0.5,
            "angle_threshold": 90.0, "min_cluster_size": 3, "max_cluster_size": 50,
            "voxel_filter_leaf_size_x": 0.04, "voxel_filter_leaf_size_y": 0.04,
            "voxel_filter_leaf_size_z": 0.04},
    # config/cones_detection_params_fsai.yaml:1-11
    "fsai": {"cones_matching_dist_theshold": 0.5, "cone_position_extension_length": 0.05,
             "distance_treshold_max": 6.0, "distance_treshold_min": 1.0, "level_threshold": -0.09,
             "angle_threshold": 160.0, "min_cluster_size": 3, "max_cluster_size": 500,
             "voxel_filter_leaf_size_x": 0.04, "voxel_filter_leaf_size_y": 0.04,
             "voxel_filter_leaf_size_z": 0.04},
}


def load_params(profile: Optional[str] = "simulation", *overrides) -> _abi.cg_params:
    """cg_params from the reference defaults, a named profile, then YAML files / dicts.

    Missing keys keep the reference's class-member defaults (cg_params_init), as a missing
    ROS param does in the nodes. Unknown keys are ignored like unused ROS params.
    """
    p = _abi.cg_params()
    lib().cg_params_init(C.byref(p))
    layers = [GROUND_PARAMS]
    if profile:
        layers.append(PROFILES[profile])
    for o in overrides:
        if isinstance(o, str):
            import yaml
            with open(o) as fh:
                o = yaml.safe_load(fh) or {}
        layers.append(o)
    names = {n for n, _ in _abi.cg_params._fields_}
    for layer in layers:
        for k, v in layer.items():
            if k in names:
                setattr(p, k, v)
    return p


# ---------------------------------------------------------------------------------------
# sensor_msgs/PointCloud2 (ROS-free)
FLOAT32 = 7


@dataclass
class PointField:
    name: str
    offset: int
    datatype: int = FLOAT32
    count: int = 1


@dataclass
class PointCloud2:
    width: int
    height: int
    fields: List[PointField]
    point_step: int
    row_step: int
    data: np.ndarray            # uint8 buffer
    is_dense: bool = True
    header: dict = field(default_factory=dict)

    @staticmethod
    def from_xyzi(points: np.ndarray, layout: int = 16, height: int = 1, intensity: bool = True):
        """Pack an (N, 4) float32 array as xyzi (point_step 16) or PCL PointXYZI (32)."""
        pts = np.ascontiguousarray(points, dtype=np.float32).reshape(-1, 4)
        n = pts.shape[0]
        if layout == 16:
            buf = pts.copy()
            fields = [PointField("x", 0), PointField("y", 4), PointField("z", 8)]
            if intensity:
                fields.append(PointField("intensity", 12))
        elif layout == 32:
            buf = np.zeros((n, 8), np.float32)
            buf[:, 0:3] = pts[:, 0:3]
            buf[:, 3] = 1.0
            buf[:, 4] = pts[:, 3]
            fields = [PointField("x", 0), PointField("y", 4), PointField("z", 8)]
            if intensity:
                fields.append(PointField("intensity", 16))
        else:
            raise ValueError("layout must be 16 or 32")
        width = n // height if height else n
        return PointCloud2(width, height, fields, layout, layout * width,
                           buf.view(np.uint8).reshape(-1), True)

    def offset_of(self, name: str) -> int:
        for f in self.fields:
            if f.name == name and f.datatype == FLOAT32 and f.count == 1:
                return f.offset
        return -1

    def has_field(self, name: str) -> bool:
        return any(f.name == name for f in self.fields)

    def view(self, intensity_offset: Optional[int] = None) -> _abi.cg_cloud_view:
        data = np.ascontiguousarray(self.data, dtype=np.uint8)
        self.data = data
        v = _abi.cg_cloud_view()
        v.data = data.ctypes.data if data.size else None
        v.width, v.height = self.width, self.height
        v.point_step, v.row_step = self.point_step, self.row_step
        v.off_x, v.off_y, v.off_z = self.offset_of("x"), self.offset_of("y"), self.offset_of("z")
        v.off_intensity = self.offset_of("intensity") if intensity_offset is None else intensity_offset
        v.is_dense = 1 if self.is_dense else 0
        return v

    def xyzi(self) -> np.ndarray:
        """Decode to (N, 4) float32 like pcl::fromROSMsg (missing fields read as 0)."""
        n = self.width * self.height
        out = np.zeros((n, 4), np.float32)
        raw = np.ascontiguousarray(self.data, dtype=np.uint8)
        rows = raw[: self.height * self.row_step].reshape(self.height, self.row_step)
        for a, name in enumerate(("x", "y", "z", "intensity")):
            off = self.offset_of(name)
            if off < 0:
                continue
            cols = rows[:, : self.width * self.point_step].reshape(self.height, self.width, self.point_step)
            out[:, a] = cols[:, :, off:off + 4].copy().view(np.float32).reshape(-1)
        return out


@dataclass
class Detection:
    """Hot-path output of one frame (what get_centroid_clouds receives, plus centroids)."""
    n_points: int
    n_kept: int
    n_filtered: int
    voxels: np.ndarray              # (V, 4) x, y, z, intensity
    labels: np.ndarray              # (V,) cluster rank or -1
    cluster_offsets: np.ndarray     # (C + 1,)
    cluster_indices: np.ndarray     # (offsets[C],)
    centroids: np.ndarray           # (C, 2) after the radial push
    flags: int = 0

    @property
    def clusters(self) -> List[np.ndarray]:
        o = self.cluster_offsets
        return [self.cluster_indices[o[i]:o[i + 1]] for i in range(len(o) - 1)]


def _copied(ptr, n: int, dtype) -> np.ndarray:
    """n elements at a result pointer, copied into a new writable array (ctypes.string_at and
    np.frombuffer: ~1.3 us less per array than np.ctypeslib.as_array on the synchronous call)."""
    dt = np.dtype(dtype)
    return np.frombuffer(C.string_at(ptr, n * dt.itemsize), dt).copy() if n else np.zeros(0, dt)


def _detection(r: _abi.cg_detect_result) -> Detection:
    V, Cn = r.n_voxels, r.n_clusters
    vox = _copied(r.voxels, V * 4, np.float32).reshape(V, 4)
    lab = _copied(r.labels, V, np.int32)
    offs = _copied(r.cluster_offsets, Cn + 1, np.int32)
    nidx = int(offs[-1]) if Cn else 0
    idx = _copied(r.cluster_indices, nidx, np.int32)
    cen = _copied(r.centroids, Cn * 2, np.float32).reshape(Cn, 2)
    return Detection(r.n_points, r.n_kept, r.n_filtered, vox, lab, offs, idx, cen, r.flags)


class _Handle:
    def __init__(self, params=None, device: int = 0):
        self.params = params if params is not None else load_params()
        h = C.c_void_p()
        check(lib().cg_create(C.byref(self.params), device, C.byref(h)))
        self._h = h
        self.voxel_order = _abi.CG_VOXEL_ORDER_PCL   # (cg_create's default)

    def close(self):
        if getattr(self, "_h", None):
            lib().cg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_voxel_order(self, order: int):
        """CG_VOXEL_ORDER_PCL (default): each voxel's float sums in PCL's std::sort order, every
        voxel bit as the reference; CG_VOXEL_ORDER_POINT: in ascending point order."""
        check(lib().cg_set_voxel_order(self._h, order))
        self.voxel_order = order
        return self

    def debug_route(self, route: int):
        """Diagnostics: 1 = every frame through the large-frame path, 2 = also its global
        backend, 0 = automatic (frames of > 65,536 points take the large path)."""
        check(lib().cg_debug_route(self._h, route))
        return self


def pcl_header(header: dict) -> dict:
    """The header after pcl::fromROSMsg then pcl::toROSMsg (pcl_conversions, PCL 1.10): the
    stamp is carried as microseconds (toNSec() / 1000, then * 1000), so nanoseconds truncate.
    Header dicts use the keys seq, stamp_sec, stamp_nsec, frame_id."""
    out = dict(header)
    if "stamp_nsec" in out:
        out["stamp_nsec"] = int(out["stamp_nsec"]) // 1000 * 1000
    return out


class GroundRemover(_Handle):
    """GroundRemover::cloud_handler (src/ground_removal.cpp:50-89) on the GPU. The published
    message takes toROSMsg's fields and header (set before toROSMsg, lines 83-86, and then
    overwritten by it): PointXYZI's fields, the PCL round trip of the input header."""

    def cloud_handler(self, msg: PointCloud2) -> PointCloud2:
        v = msg.view(intensity_offset=msg.offset_of("intensity"))
        r = _abi.cg_ground_result()
        check(lib().cg_ground_remove(self._h, C.byref(v), C.byref(r)))
        n = r.n_points
        data = np.ctypeslib.as_array(r.data, (n * 32,)).copy() if n else np.zeros(0, np.uint8)
        out = PointCloud2(r.width, r.height,
                          [PointField("x", 0), PointField("y", 4), PointField("z", 8),
                           PointField("intensity", 16)], 32, 32 * r.width, data, msg.is_dense,
                          pcl_header(msg.header))
        out.n_kept = r.n_kept
        return out


class ConeDetector(_Handle):
    """ConeDetector::cloud_handler (src/cone_detection.cpp:130-175) up to the centroids.

    Reproduces the intensity probe (lines 131-151): the first cloud decides, once, whether
    clouds carry an intensity field; if not, a fake FLOAT32 field at offset 0 is appended,
    so intensity reads the bytes of x.
    """
    _mode = "detect"

    def __init__(self, params=None, device: int = 0):
        super().__init__(params, device)
        self.intensity_in_cloud_checked = False
        self.intensity_in_cloud = True

    def recrop(self, centers) -> List[np.ndarray]:
        """get_reconstructed_cone (src/cone_detection.cpp:222-238) around each (x, y) centre,
        over the last cloud_handler call's whole cloud: one (n, 4) x,y,z,intensity array each."""
        return _recrop(self._h, centers)

    def cloud_handler(self, msg: PointCloud2) -> Detection:
        if not self.intensity_in_cloud_checked:
            if not msg.has_field("intensity"):
                self.intensity_in_cloud = False
            self.intensity_in_cloud_checked = True
        off_i = msg.offset_of("intensity") if self.intensity_in_cloud else 0
        v = msg.view(intensity_offset=off_i)
        r = _abi.cg_detect_result()
        fn = lib().cg_detect if self._mode == "detect" else lib().cg_pipeline
        check(fn(self._h, C.byref(v), C.byref(r)))
        return _detection(r)


def _recrop(h, centers, frame: Optional[int] = None) -> List[np.ndarray]:
    cen = np.ascontiguousarray(np.asarray(centers, np.float32).reshape(-1, 2))
    r = _abi.cg_crop_result()
    if frame is None:
        check(lib().cg_recrop(h, cen.ctypes.data if cen.size else None, cen.shape[0], C.byref(r)))
    else:
        check(lib().cg_batch_recrop(h, frame, cen.ctypes.data if cen.size else None, cen.shape[0], C.byref(r)))
    n = r.n_centers
    offs = np.ctypeslib.as_array(r.offsets, (n + 1,)).copy()
    tot = int(offs[-1])
    pts = np.ctypeslib.as_array(r.points, (tot * 4,)).reshape(tot, 4).copy() if tot else np.zeros((0, 4), np.float32)
    return [pts[offs[i]:offs[i + 1]] for i in range(n)]


class ConePipeline(ConeDetector):
    """ground_removal -> cone_detection (launch/cones_perception.launch:17-37), fused."""
    _mode = "pipeline"

    def cloud_handler(self, msg: PointCloud2) -> Detection:
        off_i = msg.offset_of("intensity")   # ground node: missing intensity reads 0
        v = msg.view(intensity_offset=off_i)
        r = _abi.cg_detect_result()
        check(lib().cg_pipeline(self._h, C.byref(v), C.byref(r)))
        return _detection(r)


# ---------------------------------------------------------------------------------------
# The detector node after the hot path: tracking, re-crop, colour service, publication
# (src/cone_detection.cpp:171-186, 222-363).
UNKNOWN, YELLOW, BLUE, ORANGE = range(4)         # perception_handling::Color (color.hpp)
CONES_TOPICS = ("cones_cloud_unknowns", "cones_cloud_yellows", "cones_cloud_blues", "cones_cloud_oranges")
POINTXYZI_FIELDS = (("x", 0), ("y", 4), ("z", 8), ("intensity", 16))


def to_ros_msg(xyzi: np.ndarray, header: Optional[dict] = None) -> PointCloud2:
    """pcl::toROSMsg of a pcl::PointCloud<PointXYZI> filled by push_back (PCL 1.10): height 1,
    width n (an empty cloud: width 0, height 1), PointXYZI's fields, point_step 32, is_dense.
    Point bytes: x, y, z, data[3] = 1.0f, intensity, then 12 padding bytes (written as zeros;
    the reference's are uninitialised, so only declared fields are comparable)."""
    pts = np.asarray(xyzi, np.float32).reshape(-1, 4)
    n = pts.shape[0]
    buf = np.zeros((n, 8), np.float32)
    buf[:, 0:3] = pts[:, 0:3]
    buf[:, 3] = 1.0
    buf[:, 4] = pts[:, 3]
    return PointCloud2(n, 1, [PointField(a, o) for a, o in POINTXYZI_FIELDS], 32, 32 * n,
                       buf.view(np.uint8).reshape(-1), True, dict(header or {}))


class ConeTracker:
    """get_centroid_clouds' frame-to-frame matching (src/cone_detection.cpp:251-339) through the
    C-ABI tracker: match() -> statuses (colour 0..3, CG_TRACK_DROPPED, CG_TRACK_NEED_COLOR),
    commit(colours of the NEED_COLOR centroids, or None when the service call failed),
    clouds() -> the four colour clouds as (k, 2) x, y arrays."""

    def __init__(self, classify_colors: bool = True, use_points_buffer: bool = False,
                 cones_matching_dist_theshold: float = 0.5):
        p = _abi.cg_track_params()
        lib().cg_track_params_init(C.byref(p))
        p.classify_colors = 1 if classify_colors else 0
        p.use_points_buffer = 1 if use_points_buffer else 0
        p.cones_matching_dist_theshold = cones_matching_dist_theshold
        self.params = p
        t = C.c_void_p()
        check(lib().cg_tracker_create(C.byref(p), C.byref(t)))
        self._t = t

    def close(self):
        if getattr(self, "_t", None):
            lib().cg_tracker_destroy(self._t)
            self._t = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def match(self, centroids):
        cen = np.ascontiguousarray(np.asarray(centroids, np.float32).reshape(-1, 2))
        st = np.zeros(max(cen.shape[0], 1), np.int32)
        need = C.c_uint32()
        check(lib().cg_tracker_match(self._t, cen.ctypes.data if cen.size else None, cen.shape[0],
                                     st.ctypes.data, C.byref(need)))
        return st[: cen.shape[0]], need.value

    def commit(self, colors=None):
        """colors: the colour service's response for the NEED_COLOR centroids in request order
        (it may be shorter: the rest stay unknown), or None for a failed call."""
        if colors is None:
            check(lib().cg_tracker_commit(self._t, None, 0))
        else:
            c = np.ascontiguousarray(np.asarray(colors, np.int32).reshape(-1))
            check(lib().cg_tracker_commit(self._t, c.ctypes.data if c.size else None, c.size))

    def clouds(self) -> List[np.ndarray]:
        out = []
        for i in range(_abi.CG_NUM_COLORS):
            xy = C.POINTER(C.c_float)()
            n = C.c_uint32()
            check(lib().cg_tracker_cloud(self._t, i, C.byref(xy), C.byref(n)))
            out.append(np.ctypeslib.as_array(xy, (n.value * 2,)).reshape(-1, 2).copy() if n.value
                       else np.zeros((0, 2), np.float32))
        return out


class ConeDetectorNode:
    """The whole ConeDetector::cloud_handler (src/cone_detection.cpp:130-187): the hot path on the
    GPU (cg_detect, or cg_pipeline when it stands in for the ground_removal:=true composition),
    tracking, the re-crop of cones that need a colour, the colour service and the four published
    clouds. `classifier(crop_msgs) -> colours or None` stands in for the ClassifyColorSrv call
    (src/cone_detection.cpp:342-363): it receives one PointXYZI message per cone with
    header.frame_id = cones_frame_id; None (or no classifier) is a failed call. cloud_handler
    returns the four messages published on CONES_TOPICS, index = colour."""

    def __init__(self, params=None, device: int = 0, classify_colors: bool = True, use_points_buffer: bool = False,
                 classifier=None, cones_frame_id: str = "cloud", fused_ground_removal: bool = False):
        self.params = params if params is not None else load_params()
        self.detector = (ConePipeline if fused_ground_removal else ConeDetector)(self.params, device)
        self.tracker = ConeTracker(classify_colors, use_points_buffer, self.params.cones_matching_dist_theshold)
        self.classifier = classifier
        self.cones_frame_id = cones_frame_id
        self.last_detection: Optional[Detection] = None

    def cloud_handler(self, msg: PointCloud2) -> List[PointCloud2]:
        det = self.detector.cloud_handler(msg)
        self.last_detection = det
        status, n_need = self.tracker.match(det.centroids)
        colors = None
        if n_need:
            need = det.centroids[status == _abi.CG_TRACK_NEED_COLOR]
            crops = [to_ros_msg(c, {"frame_id": self.cones_frame_id}) for c in self.detector.recrop(need)]
            # the service's response: possibly shorter than the request (the reference's server
            # skips empty crops); the tracker applies it positionally (src/cone_detection.cpp:357-358)
            colors = self.classifier(crops) if self.classifier is not None else None
        self.tracker.commit(colors)
        out = []
        for xy in self.tracker.clouds():
            pts = np.zeros((xy.shape[0], 4), np.float32)
            pts[:, 0:2] = xy
            m = to_ros_msg(pts)
            m.header = dict(msg.header)                            # line 182
            m.fields = [PointField(f.name, f.offset, f.datatype, f.count) for f in msg.fields]   # 183
            out.append(m)
        return out


class BatchEngine(_Handle):
    """Device-resident batch engine (cg_run_batch): frames already in HBM."""

    def run(self, d_ptr: int, n_frames: int, n_points: int, point_step: int = 16,
            frame_stride: Optional[int] = None, mode: int = CG_MODE_PIPELINE, stream: int = 0,
            offsets=(0, 4, 8, 12), is_dense: bool = True):
        """cg_run_batch on `stream` (0: the handle's own)."""
        b = batch_desc(d_ptr, n_frames, n_points, point_step, frame_stride, offsets, is_dense)
        check(lib().cg_run_batch(self._h, C.byref(b), mode, C.c_void_p(stream) if stream else None))

    def spans(self, d_spans: int, n_launches: int):
        """cg_debug_launch_spans: the next n_launches launches record their execution spans."""
        check(lib().cg_debug_launch_spans(self._h, C.c_void_p(d_spans), n_launches))
        return self

    def results(self) -> _abi.cg_batch_results:
        r = _abi.cg_batch_results()
        check(lib().cg_batch_results_get(self._h, C.byref(r)))
        return r

    def fetch(self, frame: int) -> Detection:
        r = _abi.cg_detect_result()
        check(lib().cg_batch_fetch(self._h, frame, C.byref(r)))
        return _detection(r)

    def recrop(self, frame: int, centers) -> List[np.ndarray]:
        """get_reconstructed_cone for frame `frame` of the last batch (cg_batch_recrop): the
        batch's input must still be resident."""
        return _recrop(self._h, centers, frame)


def batch_desc(d_ptr: int, n_frames: int, n_points: int, point_step: int = 16,
               frame_stride: Optional[int] = None, offsets=(0, 4, 8, 12), is_dense: bool = True) -> _abi.cg_batch:
    """A cg_batch for frames in device memory."""
    b = _abi.cg_batch()
    b.d_data = d_ptr
    b.frame_stride = frame_stride if frame_stride is not None else n_points * point_step
    b.n_frames, b.n_points, b.point_step = n_frames, n_points, point_step
    b.off_x, b.off_y, b.off_z, b.off_intensity = offsets
    b.is_dense = 1 if is_dense else 0
    return b


class BatchQueue:
    """A sequence of batch calls enqueued in one cg_run_batches crossing: call i runs batches[i]
    on engines[i] on streams[i] (stream handles; 0 = the engine's own). Built once, run many
    times (the descriptors stay in ctypes arrays)."""

    def __init__(self, engines, batches, streams, mode: int = CG_MODE_PIPELINE):
        n = len(engines)
        if not (len(batches) == len(streams) == n):
            raise ValueError("engines, batches and streams differ in length")
        self.n, self.mode = n, mode
        self._keep = list(engines)
        self._h = (C.c_void_p * n)(*[e.handle.value for e in engines])
        self._b = (_abi.cg_batch * n)(*batches)
        self._s = (C.c_void_p * n)(*[s or None for s in streams])
        self._done = C.c_uint32(0)

    def run(self) -> int:
        check(lib().cg_run_batches(self._h, self._b, self.n, self.mode, self._s, C.byref(self._done)))
        return self._done.value


# ---------------------------------------------------------------------------------------
def synth_config(rings=64, cols=1024, point_step=16, seed=0x00C0FFEE, cones_per_row=5, clutter=0,
                 column_major=True) -> _abi.cg_synth_cfg:
    c = _abi.cg_synth_cfg()
    lib().cg_synth_default(C.byref(c))
    c.rings, c.cols, c.point_step, c.seed = rings, cols, point_step, seed
    c.cones_per_row, c.clutter, c.column_major = cones_per_row, clutter, 1 if column_major else 0
    return c


def synth_frames(n_frames=1, first_frame=0, threads=8, out: Optional[np.ndarray] = None, **kw) -> np.ndarray:
    """Deterministic synthetic cone-field frames as a (n_frames, N*point_step) uint8 array."""
    cfg = synth_config(**kw)
    stride = cfg.rings * cfg.cols * cfg.point_step
    if out is None:
        out = np.empty((n_frames, stride), np.uint8)
    check(lib().cg_synth_frames(C.byref(cfg), first_frame, n_frames, out.ctypes.data, stride, threads))
    return out


def frame_cloud(raw: np.ndarray, point_step=16) -> PointCloud2:
    """Wrap one synthetic frame's bytes as a PointCloud2."""
    n = raw.size // point_step
    if point_step == 16:
        fields = [PointField("x", 0), PointField("y", 4), PointField("z", 8), PointField("intensity", 12)]
    else:
        fields = [PointField("x", 0), PointField("y", 4), PointField("z", 8), PointField("intensity", 16)]
    return PointCloud2(n, 1, fields, point_step, n * point_step, raw.reshape(-1), True)


from .colornet import ColorClassifier, read_tflite  # noqa: E402  (the colour service, §8f row 4)
