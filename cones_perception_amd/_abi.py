"""ctypes mirror of include/cones_gpu.h.

Loads the in-tree gfx950 library (cones_perception_amd/lib/libcones_gpu.so). There is no CPU
fallback: if the library is missing the import fails loudly; if no gfx950 device is present,
cg_create returns CG_E_DEVICE.
"""
import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
# CONES_GPU_LIB: an alternative build of the same library (tools/build_variant.sh experiments)
LIB_PATH = os.environ.get("CONES_GPU_LIB") or os.path.join(_HERE, "lib", "libcones_gpu.so")

CG_OK, CG_E_INVALID, CG_E_DEVICE, CG_E_OOM, CG_E_CAPACITY = 0, 1, 2, 3, 4
CG_F_VOXEL_PASSTHROUGH, CG_F_GLOBAL_SCRATCH, CG_F_ORDER_CANONICAL, CG_F_VOXEL_POINT_ORDER = 0x1, 0x2, 0x4, 0x8
CG_VOXEL_ORDER_POINT, CG_VOXEL_ORDER_PCL = 0, 1
CG_MODE_PIPELINE, CG_MODE_DETECT = 0, 1
CG_HDR_N, CG_HDR_K, CG_HDR_M, CG_HDR_V, CG_HDR_C, CG_HDR_FLAGS, CG_HDR_ERR, CG_HDR_WORDS = 0, 1, 2, 3, 4, 5, 7, 8
CG_HDR_E_WAIT = 0x57414954


class cg_params(C.Structure):
    _fields_ = [
        ("num_of_sectors", C.c_int32),
        ("default_lowest_point", C.c_float),
        ("distance_treshold_max", C.c_double),
        ("distance_treshold_min", C.c_double),
        ("level_threshold", C.c_double),
        ("angle_threshold", C.c_double),
        ("min_cluster_size", C.c_int32),
        ("max_cluster_size", C.c_int32),
        ("cone_position_extension_length", C.c_double),
        ("voxel_filter_leaf_size_x", C.c_double),
        ("voxel_filter_leaf_size_y", C.c_double),
        ("voxel_filter_leaf_size_z", C.c_double),
        ("cones_matching_dist_theshold", C.c_double),
    ]


class cg_cloud_view(C.Structure):
    _fields_ = [
        ("data", C.c_void_p),
        ("width", C.c_uint32), ("height", C.c_uint32),
        ("point_step", C.c_uint32), ("row_step", C.c_uint32),
        ("off_x", C.c_int32), ("off_y", C.c_int32), ("off_z", C.c_int32), ("off_intensity", C.c_int32),
        ("is_dense", C.c_uint8),
    ]


class cg_ground_result(C.Structure):
    _fields_ = [
        ("n_points", C.c_uint32), ("n_kept", C.c_uint32),
        ("width", C.c_uint32), ("height", C.c_uint32),
        ("data", C.POINTER(C.c_uint8)),
    ]


class cg_detect_result(C.Structure):
    _fields_ = [
        ("n_points", C.c_uint32), ("n_kept", C.c_uint32), ("n_filtered", C.c_uint32),
        ("n_voxels", C.c_uint32), ("n_clusters", C.c_uint32), ("flags", C.c_uint32),
        ("voxels", C.POINTER(C.c_float)),
        ("labels", C.POINTER(C.c_int32)),
        ("cluster_offsets", C.POINTER(C.c_int32)),
        ("cluster_indices", C.POINTER(C.c_int32)),
        ("centroids", C.POINTER(C.c_float)),
    ]


class cg_batch(C.Structure):
    _fields_ = [
        ("d_data", C.c_void_p),
        ("frame_stride", C.c_uint64),
        ("n_frames", C.c_uint32), ("n_points", C.c_uint32), ("point_step", C.c_uint32),
        ("off_x", C.c_int32), ("off_y", C.c_int32), ("off_z", C.c_int32), ("off_intensity", C.c_int32),
        ("is_dense", C.c_uint8),
    ]


class cg_batch_results(C.Structure):
    _fields_ = [
        ("n_frames", C.c_uint32), ("capacity", C.c_uint32),
        ("d_header", C.c_void_p), ("d_voxels", C.c_void_p), ("d_labels", C.c_void_p),
        ("d_cluster_offsets", C.c_void_p), ("d_cluster_indices", C.c_void_p), ("d_centroids", C.c_void_p),
    ]


class cg_tile(C.Structure):
    _fields_ = [("d_data", C.c_void_p), ("first", C.c_uint32), ("n", C.c_uint32), ("n_total", C.c_uint32),
                ("point_step", C.c_uint32), ("off_x", C.c_int32), ("off_y", C.c_int32), ("off_z", C.c_int32),
                ("off_intensity", C.c_int32)]


CG_TILE_KEYS, CG_TILE_COUNTS = 19, 9
CG_HALO_REC_WORDS = 8


class cg_halo_plan(C.Structure):
    _fields_ = [("passthrough", C.c_uint32), ("min_b", C.c_int32 * 3), ("div_b", C.c_uint32 * 3),
                ("slabs", C.c_uint32), ("slab_w", C.c_uint32), ("band", C.c_uint32), ("pad_slab", C.c_int32),
                ("n_pads", C.c_uint32), ("key_bits", C.c_uint32)]


class cg_crop_result(C.Structure):
    _fields_ = [("n_centers", C.c_uint32), ("offsets", C.POINTER(C.c_uint32)), ("points", C.POINTER(C.c_float))]


class cg_track_params(C.Structure):
    _fields_ = [("classify_colors", C.c_uint8), ("use_points_buffer", C.c_uint8),
                ("cones_matching_dist_theshold", C.c_double)]


CG_NUM_COLORS, CG_TRACK_DROPPED, CG_TRACK_NEED_COLOR = 4, -1, -2


class cg_synth_cfg(C.Structure):
    _fields_ = [
        ("rings", C.c_uint32), ("cols", C.c_uint32),
        ("elev_min_deg", C.c_float), ("elev_max_deg", C.c_float), ("mount_height", C.c_float),
        ("wall_radius", C.c_float), ("range_noise", C.c_float),
        ("point_step", C.c_uint32), ("column_major", C.c_uint32),
        ("cones_per_row", C.c_uint32), ("clutter", C.c_uint32),
        ("seed", C.c_uint64),
    ]


_SIGS = {
    "cg_params_init": (None, [C.POINTER(cg_params)]),
    "cg_create": (C.c_int, [C.POINTER(cg_params), C.c_int, C.POINTER(C.c_void_p)]),
    "cg_destroy": (C.c_int, [C.c_void_p]),
    "cg_set_params": (C.c_int, [C.c_void_p, C.POINTER(cg_params)]),
    "cg_set_voxel_order": (C.c_int, [C.c_void_p, C.c_int]),
    "cg_last_error": (C.c_char_p, []),
    "cg_version": (C.c_char_p, []),
    "cg_ground_remove": (C.c_int, [C.c_void_p, C.POINTER(cg_cloud_view), C.POINTER(cg_ground_result)]),
    "cg_detect": (C.c_int, [C.c_void_p, C.POINTER(cg_cloud_view), C.POINTER(cg_detect_result)]),
    "cg_pipeline": (C.c_int, [C.c_void_p, C.POINTER(cg_cloud_view), C.POINTER(cg_detect_result)]),
    "cg_run_batch": (C.c_int, [C.c_void_p, C.POINTER(cg_batch), C.c_int, C.c_void_p]),
    "cg_run_batches": (C.c_int, [C.POINTER(C.c_void_p), C.POINTER(cg_batch), C.c_uint32, C.c_int,
                                 C.POINTER(C.c_void_p), C.POINTER(C.c_uint32)]),
    "cg_tile_front": (C.c_int, [C.c_void_p, C.POINTER(cg_tile), C.c_void_p]),
    "cg_tile_decide": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p]),
    "cg_tile_survivors": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    "cg_tile_backend": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32]),
    "cg_tile_front_async": (C.c_int, [C.c_void_p, C.POINTER(cg_tile), C.c_void_p, C.c_void_p]),
    "cg_tile_decide_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "cg_tile_survivors_async": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p]),
    "cg_tile_backend_own": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p]),
    "cg_halo_plan_frame": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32, C.POINTER(cg_halo_plan)]),
    "cg_halo_owner": (C.c_int, [C.c_void_p, C.POINTER(cg_halo_plan), C.c_void_p, C.c_uint32, C.c_void_p]),
    "cg_halo_local": (C.c_int, [C.c_void_p, C.POINTER(cg_halo_plan), C.c_void_p, C.c_void_p, C.c_uint32, C.c_uint32,
                                C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.POINTER(C.c_uint32)]),
    "cg_halo_edges": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                C.POINTER(C.c_uint32)]),
    "cg_halo_merge": (C.c_int, [C.c_void_p, C.POINTER(cg_halo_plan), C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32,
                                C.c_void_p, C.c_uint32]),
    "cg_colornet_set": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "cg_classify_colors": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                     C.c_void_p]),
    "cg_batch_results_get": (C.c_int, [C.c_void_p, C.POINTER(cg_batch_results)]),
    "cg_batch_fetch": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(cg_detect_result)]),
    "cg_selftest_atan2f": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    "cg_selftest_sqrt": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint32]),
    "cg_debug_stamps": (C.c_int, [C.c_void_p, C.c_int]),
    "cg_debug_route": (C.c_int, [C.c_void_p, C.c_int]),
    "cg_debug_launch_span": (C.c_int, [C.c_void_p, C.c_void_p]),
    "cg_debug_launch_spans": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "cg_debug_large_meta": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "cg_debug_large_buffer": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p, C.c_uint64]),
    "cg_debug_stamps_fetch": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "cg_recrop": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.POINTER(cg_crop_result)]),
    "cg_batch_recrop": (C.c_int, [C.c_void_p, C.c_uint32, C.c_void_p, C.c_uint32, C.POINTER(cg_crop_result)]),
    "cg_track_params_init": (None, [C.POINTER(cg_track_params)]),
    "cg_tracker_create": (C.c_int, [C.POINTER(cg_track_params), C.POINTER(C.c_void_p)]),
    "cg_tracker_destroy": (C.c_int, [C.c_void_p]),
    "cg_tracker_set_params": (C.c_int, [C.c_void_p, C.POINTER(cg_track_params)]),
    "cg_tracker_match": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32, C.c_void_p, C.POINTER(C.c_uint32)]),
    "cg_tracker_commit": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint32]),
    "cg_tracker_cloud": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.POINTER(C.c_float)),
                                   C.POINTER(C.c_uint32)]),
    "cg_synth_default": (None, [C.POINTER(cg_synth_cfg)]),
    "cg_synth_frames": (C.c_int, [C.POINTER(cg_synth_cfg), C.c_uint64, C.c_uint32, C.c_void_p,
                                  C.c_uint64, C.c_uint32]),
}

_lib = None


def lib():
    """The loaded libcones_gpu.so (raises if it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} not found: the gfx950 HIP library is required (no CPU fallback). "
                "Build it with `python -m cones_perception_amd.build` or __graft_entry__.build().")
        # One HIP runtime per process: torch ships its own libamdhip64.so.7 (same soname).
        # If torch is importable it must be loaded first so our DT_NEEDED binds to its copy;
        # loading /opt/rocm's runtime first makes torch bring a second one and HIP device
        # enumeration fails in whichever initialises second.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        _lib = C.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            fn = getattr(_lib, name)
            fn.restype = res
            fn.argtypes = args
    return _lib


class CgError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"cones_gpu error {code}: {msg}")
        self.code = code


def check(rc):
    if rc != CG_OK:
        raise CgError(rc, lib().cg_last_error().decode(errors="replace"))
    return rc
