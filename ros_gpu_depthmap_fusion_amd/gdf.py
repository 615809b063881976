"""ctypes binding of the C-ABI in include/gdf.h, with a Python mirror of the reference engine.

`GPUDepthmapFusion` exposes the method names of the reference class
(include/gpu_depthmap_fusion/gpu_depthmap_fusion.h:219-309, src/gpu_depthmap_fusion.cpp) so the
parity tests read like the reference's call sequence (GPUDepthmapFusionComponent::processDepthmaps,
src/gpu_depthmap_fusion_component.cpp:92-300).  Errors raise `GDFError` carrying the C status and
gdf_last_error().  There is no CPU fallback: if libgdf.so is missing or no GPU is present, the
constructor raises.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "lib", "libgdf.so")

GDF_OK = 0
STATUS_NAMES = {
    -1: "GDF_ERR_ARG", -2: "GDF_ERR_STATE", -3: "GDF_ERR_HIP", -4: "GDF_ERR_NOMEM",
    -5: "GDF_ERR_CAPACITY", -6: "GDF_ERR_TIME", -7: "GDF_ERR_DEVICE",
}

_f16 = C.c_float * 16
_f3 = C.c_float * 3


class RollbufferState(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "num_points", "num_seqs", "selection_point_start", "selection_point_count",
        "selection_sequence_start", "selection_sequence_count", "earliest_time_sec",
        "earliest_time_nsec", "last_time_sec", "last_time_nsec")]

    def as_tuple(self):
        return tuple(getattr(self, n) for n, _ in self._fields_)


class FrameParams(C.Structure):
    _fields_ = [
        ("ps_filter_threshold", C.c_float), ("ps_filter_size", C.c_uint32),
        ("ps_timespan", C.c_float), ("move_transform_available", C.c_int32),
        ("T_world_move", _f16), ("T_crop_move", _f16),
        ("flying_filter_size", C.c_uint32), ("flying_threshold", C.c_float),
        ("flying_rot45", C.c_int32), ("crop_min", _f3), ("crop_max", _f3),
        ("enable_voxel_filter", C.c_int32), ("voxel_min", _f3), ("voxel_max", _f3),
        ("voxel_size", _f3), ("voxel_average", C.c_int32), ("occupancy_lifetime", C.c_uint32),
        ("defer_occupancy_grid", C.c_int32), ("synchronous", C.c_int32),
        ("defer_voxelize", C.c_int32),
    ]


# gdf_kernel_slot order (include/gdf.h): launch groups, then single kernels
KERNEL_SLOTS = ("frame", "grid", "voxelize", "ps_insert", "mask", "scan", "emit", "sort",
                "group", "sel", "event_floor")


class StreamCamera(C.Structure):
    """gdf_stream_camera (include/gdf_driver.h)."""
    _fields_ = [
        ("frames", C.POINTER(C.c_void_p)), ("ring", C.c_uint32), ("width", C.c_uint32),
        ("height", C.c_uint32), ("depth_scale", C.c_float), ("fx", C.c_float), ("fy", C.c_float),
        ("cx", C.c_float), ("cy", C.c_float), ("T_world", _f16), ("T_crop", _f16),
    ]


class FrameResult(C.Structure):
    _fields_ = [("processed", C.c_int32), ("num_depth_points", C.c_uint32),
                ("num_points_total", C.c_uint32), ("num_points", C.c_uint32),
                ("num_voxelized", C.c_uint32), ("latest_time_sec", C.c_uint32),
                ("latest_time_nsec", C.c_uint32)]


class HostFrame(C.Structure):
    _fields_ = [("points", C.c_void_p), ("voxel_coords", C.c_void_p), ("num_points", C.c_uint32),
                ("voxelized", C.c_void_p), ("num_voxelized", C.c_uint32),
                ("occupancy", C.c_void_p), ("num_cells", C.c_uint64)]


DL_POINTS, DL_COORDS, DL_VOXELIZED, DL_GRID = 1, 2, 4, 8


class SegCounts(C.Structure):
    """gdf_seg_counts (include/gdf_segment.h)."""
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("layers", C.c_uint32),
                ("total_labels", C.c_uint32), ("total_contours", C.c_uint32),
                ("total_contour_points", C.c_uint64), ("connection_bytes", C.c_uint64)]


class CCObject(C.Structure):
    """gdf_cc_object (include/gdf_segment.h): createCCObjects' aggregate fields."""
    _fields_ = [("label", C.c_uint32), ("num_components", C.c_uint32),
                ("num_layers", C.c_uint32), ("first_component", C.c_uint32),
                ("centroid", C.c_float * 2), ("min_voxel", C.c_int32 * 3),
                ("max_voxel", C.c_int32 * 3), ("aabb_voxel", C.c_int32 * 3),
                ("center_voxel", C.c_float * 3), ("center_world", C.c_float * 3),
                ("min_world", C.c_float * 3), ("max_world", C.c_float * 3),
                ("aabb_world", C.c_float * 3), ("num_contour_points", C.c_uint32)]


def cc_objects_as_dict(objs) -> dict:
    """Columns of a CCObject array (the layout oracle.create_cc_objects returns)."""
    names = [n for n, _ in CCObject._fields_]
    return {n: np.array([np.ctypeslib.as_array(getattr(o, n)) if hasattr(getattr(o, n), "_length_")
                         else getattr(o, n) for o in objs]) for n in names}


class LocalOp(C.Structure):
    """gdf_local_op (include/gdf_fused.h): one operation of a local-transport round (kind 0
    all-gather, 1 send, 2 receive)."""
    _fields_ = [("kind", C.c_int), ("src", C.c_void_p), ("dst", C.c_void_p),
                ("bytes", C.c_uint64), ("peer", C.c_int)]


class GDFError(RuntimeError):
    def __init__(self, status: int, msg: str):
        super().__init__(f"{STATUS_NAMES.get(status, status)}: {msg}")
        self.status = status


_lib = None

# every symbol declared in include/gdf.h (checked by tests/test_abi.py)
EXPORTED = [
    "gdf_create", "gdf_destroy", "gdf_last_error", "gdf_version", "gdf_set_stream",
    "gdf_synchronize", "gdf_set_pipeline_depth", "gdf_set_graphs", "gdf_set_voxel_group_size", "gdf_clear", "gdf_add_depthmap",
    "gdf_add_depthmap_device", "gdf_add_point_sequence", "gdf_add_point_sequence_device",
    "gdf_num_collected_point_sequence_points",
    "gdf_upload_point_sequences", "gdf_filter_new_point_sequences", "gdf_insert_new_point_sequences",
    "gdf_roll_rollbuffer", "gdf_select_timespan", "gdf_prepare_point_and_mask_buffers",
    "gdf_insert_selected_point_sequence", "gdf_transform_point_sequence", "gdf_get_rollbuffer_state",
    "gdf_set_rollbuffer_shard", "gdf_get_rollbuffer_pieces",
    "gdf_upload_depthmaps", "gdf_convert_depthmaps", "gdf_filter_flying_pixels", "gdf_crop_points",
    "gdf_apply_point_mask", "gdf_compute_voxel_coords", "gdf_voxelize", "gdf_voxel_occupancy_grid",
    "gdf_get_point_count", "gdf_download_points", "gdf_download_voxel_coords",
    "gdf_download_voxelized_points", "gdf_download_occupancy_grid", "gdf_get_grid_size",
    "gdf_get_device_results", "gdf_process_frame", "gdf_export_occupancy_marks",
    "gdf_import_occupancy_marks", "gdf_take_occupancy_marks", "gdf_import_occupancy_marks_strided",
    "gdf_voxel_occupancy_grid_batch", "gdf_take_occupancy_marks_sparse", "gdf_union_occupancy_pairs",
    "gdf_set_profiling", "gdf_get_kernel_times", "gdf_set_debug", "gdf_debug_stage_masks", "gdf_debug_rollbuffer",
    "gdf_debug_historic_grid",
    # include/gdf_driver.h: the component's depth loop in C++ over the C-ABI
    "gdf_run_depth_stream", "gdf_run_host_stream", "gdf_run_depth_stream_batched",
    "gdf_run_depth_stream_alternating",
    "gdf_next_frame_in_batch", "gdf_get_batch_ranges", "gdf_download_batch_occupancy_grid",
    "gdf_mask_dilate", "gdf_transform_points", "gdf_add_halo_depthmap_device",
    "gdf_partition_points", "gdf_voxelize_points", "gdf_partition_runs", "gdf_voxelize_runs", "gdf_voxelize_runs_marked", "gdf_voxelize_runs_recv", "gdf_set_partition_marks", "gdf_set_emit_partition", "gdf_set_partition_segments", "gdf_last_sort_items", "gdf_get_stream",
    "gdf_get_graph_stats", "gdf_get_slot", "gdf_select_slot", "gdf_build_info", "gdf_get_tuning",
    "gdf_download_frame", "gdf_set_slot_streams",
    # include/gdf_fused.h: a rank of the multi-GPU fused cloud in C++ over RCCL
    "gdf_fused_unique_id", "gdf_fused_create", "gdf_fused_destroy", "gdf_fused_halo_pixels",
    "gdf_fused_start", "gdf_fused_finish", "gdf_fused_run", "gdf_fused_local_create",
    "gdf_fused_local_destroy", "gdf_fused_create_local", "gdf_fused_info",
    "gdf_fused_set_rollbuffer_shard", "gdf_fused_local_check_round", "gdf_fused_local_check_arrival",
    # include/gdf_segment.h: the GPU object-segmentation front end
    "gdf_seg_create", "gdf_seg_destroy", "gdf_seg_set_stream", "gdf_seg_label_layers",
    "gdf_seg_label_engine_grid", "gdf_seg_get_counts", "gdf_seg_download_labels",
    "gdf_seg_download_num_labels", "gdf_seg_download_stats", "gdf_seg_download_connections",
    "gdf_seg_download_contours", "gdf_seg_merge_labels", "gdf_seg_get_device_results",
    "gdf_seg_create_objects",
]


ABI_VERSION = (0, 4)  # include/gdf.h GDF_VERSION_MAJOR / _MINOR


def load_library(path: str = LIB_PATH):
    """Load libgdf.so (raises if it was not built: there is no fallback path)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise GDFError(-2, f"{path} not built (run __graft_entry__.build())")
    lib = C.CDLL(path)
    vp, u32, i32, f, u64 = C.c_void_p, C.c_uint32, C.c_int, C.c_float, C.c_uint64
    P = C.POINTER
    sig = {
        "gdf_create": (i32, [i32, P(vp)]),
        "gdf_destroy": (i32, [vp]),
        "gdf_last_error": (C.c_char_p, []),
        "gdf_version": (i32, [P(i32), P(i32)]),
        "gdf_set_stream": (i32, [vp, vp]),
        "gdf_synchronize": (i32, [vp]),
        "gdf_set_pipeline_depth": (i32, [vp, i32]),
        "gdf_set_graphs": (i32, [vp, i32]),
        "gdf_set_voxel_group_size": (i32, [vp, i32]),
        "gdf_clear": (i32, [vp]),
        "gdf_add_depthmap": (i32, [vp, vp, u32, u32, f, f, f, f, f, vp, vp]),
        "gdf_add_depthmap_device": (i32, [vp, vp, u32, u32, f, f, f, f, f, vp, vp]),
        "gdf_add_point_sequence": (i32, [vp, vp, u32, u32, u32, u32, vp]),
        "gdf_add_point_sequence_device": (i32, [vp, vp, u32, u32, u32, u32, vp]),
        "gdf_num_collected_point_sequence_points": (i32, [vp, P(u32)]),
        "gdf_upload_point_sequences": (i32, [vp]),
        "gdf_filter_new_point_sequences": (i32, [vp, f, u32]),
        "gdf_insert_new_point_sequences": (i32, [vp]),
        "gdf_roll_rollbuffer": (i32, [vp, u32, u32]),
        "gdf_select_timespan": (i32, [vp, u32, u32, u32, u32]),
        "gdf_prepare_point_and_mask_buffers": (i32, [vp]),
        "gdf_insert_selected_point_sequence": (i32, [vp, vp, vp]),
        "gdf_transform_point_sequence": (i32, [vp]),
        "gdf_get_rollbuffer_state": (i32, [vp, P(RollbufferState)]),
        "gdf_upload_depthmaps": (i32, [vp]),
        "gdf_convert_depthmaps": (i32, [vp]),
        "gdf_filter_flying_pixels": (i32, [vp, u32, f, i32]),
        "gdf_crop_points": (i32, [vp, vp, vp]),
        "gdf_apply_point_mask": (i32, [vp, P(u32)]),
        "gdf_compute_voxel_coords": (i32, [vp, vp, vp, vp]),
        "gdf_voxelize": (i32, [vp, i32]),
        "gdf_voxel_occupancy_grid": (i32, [vp, u32]),
        "gdf_get_point_count": (i32, [vp, P(u32)]),
        "gdf_download_points": (i32, [vp, vp, u32, P(u32)]),
        "gdf_download_voxel_coords": (i32, [vp, vp, u32, P(u32)]),
        "gdf_download_voxelized_points": (i32, [vp, vp, u32, P(u32)]),
        "gdf_download_occupancy_grid": (i32, [vp, vp, u64]),
        "gdf_get_grid_size": (i32, [vp, vp, P(u64)]),
        "gdf_get_device_results": (i32, [vp, P(vp), P(vp), P(vp), P(vp)]),
        "gdf_process_frame": (i32, [vp, P(FrameParams), P(FrameResult)]),
        "gdf_export_occupancy_marks": (i32, [vp, vp, u64]),
        "gdf_import_occupancy_marks": (i32, [vp, vp, u64, u32]),
        "gdf_take_occupancy_marks": (i32, [vp, vp, u64]),
        "gdf_import_occupancy_marks_strided": (i32, [vp, vp, u64, u32, u64]),
        "gdf_voxel_occupancy_grid_batch": (i32, [vp, vp, u64, u32, u32, u64, u64, u32]),
        "gdf_take_occupancy_marks_sparse": (i32, [vp, vp, u64, vp, u32]),
        "gdf_union_occupancy_pairs": (i32, [vp, vp, u64, vp, u32, u32, u32, u64]),
        "gdf_set_profiling": (i32, [vp, i32]),
        "gdf_get_kernel_times": (i32, [vp, vp, vp, i32]),
        "gdf_set_debug": (i32, [vp, i32]),
        "gdf_debug_stage_masks": (i32, [vp, vp, u32, P(u32)]),
        "gdf_debug_rollbuffer": (i32, [vp, vp, vp, vp, u32, vp, u32]),
        "gdf_debug_historic_grid": (i32, [vp, vp, u64]),
        "gdf_run_depth_stream": (i32, [vp, P(StreamCamera), u32, P(FrameParams), u64, u64]),
        "gdf_run_host_stream": (i32, [vp, P(StreamCamera), u32, P(FrameParams), u64, u64]),
        "gdf_run_depth_stream_batched": (i32, [vp, P(StreamCamera), u32, P(FrameParams), u64,
                                               u64, u32, i32]),
        "gdf_run_depth_stream_alternating": (i32, [vp, P(StreamCamera), u32, vp, u32, u64, u64,
                                                   u32]),
        "gdf_next_frame_in_batch": (i32, [vp]),
        "gdf_mask_dilate": (i32, [vp, vp, vp, u32, u32, u32, i32]),
        "gdf_add_halo_depthmap_device": (i32, [vp, vp, u32, u32, u32, f, f, f, f, f, vp, vp]),
        "gdf_partition_points": (i32, [vp, u32, vp, vp, u32, vp]),
        "gdf_voxelize_points": (i32, [vp, vp, vp, u32, i32]),
        "gdf_partition_runs": (i32, [vp, u32, vp, vp, vp, u32, vp]),
        "gdf_set_emit_partition": (i32, [vp, u32, vp, vp, vp, u32, vp]),
        "gdf_voxelize_runs": (i32, [vp, vp, vp, vp, u32, vp, vp, i32]),
        "gdf_voxelize_runs_marked": (i32, [vp, vp, vp, vp, u32, vp, vp, i32, vp, u64]),
        "gdf_voxelize_runs_recv": (i32, [vp, vp, vp, vp, u32, vp, vp, i32, vp, u64, vp]),
        "gdf_set_partition_marks": (i32, [vp, i32]),
        "gdf_transform_points": (i32, [vp, vp, vp, vp, u32, vp]),
        "gdf_get_batch_ranges": (i32, [vp, vp, vp, u32, P(u32)]),
        "gdf_download_batch_occupancy_grid": (i32, [vp, u32, vp, u64]),
        "gdf_last_sort_items": (i32, [vp, P(u32), P(i32)]),
        "gdf_get_stream": (i32, [vp, P(vp)]),
        "gdf_get_graph_stats": (i32, [vp, P(u64), P(u64)]),
        "gdf_get_slot": (i32, [vp, P(i32)]),
        "gdf_select_slot": (i32, [vp, i32]),
        "gdf_build_info": (C.c_char_p, []),
        "gdf_get_tuning": (i32, [vp, C.c_char_p, u32]),
        "gdf_download_frame": (i32, [vp, u32, P(HostFrame)]),
        "gdf_set_slot_streams": (i32, [vp, vp, i32]),
        "gdf_fused_unique_id": (i32, [C.c_char_p, vp]),
        "gdf_fused_create": (i32, [vp, C.c_char_p, vp, i32, i32, P(StreamCamera), u32, P(vp)]),
        "gdf_fused_destroy": (i32, [vp]),
        "gdf_fused_halo_pixels": (i32, [vp, P(u32)]),
        "gdf_fused_start": (i32, [vp, vp, u32, P(FrameParams), P(i32)]),
        "gdf_fused_finish": (i32, [vp, i32, vp, P(u32)]),
        "gdf_fused_run": (i32, [vp, P(StreamCamera), P(FrameParams), u64, u64, u32, i32]),
        "gdf_set_rollbuffer_shard": (i32, [vp, u32, u32, u32]),
        "gdf_get_rollbuffer_pieces": (i32, [vp, vp, u32, P(u32)]),
        "gdf_set_partition_segments": (i32, [vp, u32]),
        "gdf_fused_local_create": (i32, [i32, P(vp)]),
        "gdf_fused_local_destroy": (i32, [vp]),
        "gdf_fused_create_local": (i32, [vp, vp, i32, i32, P(StreamCamera), u32, P(vp)]),
        "gdf_fused_info": (i32, [vp, P(i32), P(i32), P(i32), P(C.c_char_p)]),
        "gdf_fused_set_rollbuffer_shard": (i32, [vp, u32]),
        "gdf_fused_local_check_round": (i32, [i32, P(LocalOp), P(u32), P(u64)]),
        "gdf_fused_local_check_arrival": (i32, [i32, i32, i32, u64, u64, P(C.c_int64)]),
        "gdf_seg_create": (i32, [i32, P(vp)]),
        "gdf_seg_destroy": (i32, [vp]),
        "gdf_seg_set_stream": (i32, [vp, vp]),
        "gdf_seg_label_layers": (i32, [vp, vp, u32, u32, u32, u32]),
        "gdf_seg_label_engine_grid": (i32, [vp, vp, u32]),
        "gdf_seg_get_counts": (i32, [vp, P(SegCounts)]),
        "gdf_seg_download_labels": (i32, [vp, vp, u64]),
        "gdf_seg_download_num_labels": (i32, [vp, vp, u32]),
        "gdf_seg_download_stats": (i32, [vp, vp, vp, u32]),
        "gdf_seg_download_connections": (i32, [vp, vp, u64, vp, u32]),
        "gdf_seg_download_contours": (i32, [vp, vp, vp, vp, vp, u64]),
        "gdf_seg_merge_labels": (i32, [vp, vp, u32, P(u32)]),
        "gdf_seg_get_device_results": (i32, [vp, P(vp), P(vp), P(vp), P(vp)]),
        "gdf_seg_create_objects": (i32, [vp, vp, vp, vp, u32, vp, u32, P(u32)]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    major, minor = C.c_int(), C.c_int()
    lib.gdf_version(C.byref(major), C.byref(minor))
    if (major.value, minor.value) != ABI_VERSION:  # the structs below are those of ABI_VERSION
        raise GDFError(-2, f"{path}: ABI {major.value}.{minor.value}, binding expects "
                           f"{ABI_VERSION[0]}.{ABI_VERSION[1]} (rebuild the library)")
    info = build_info(lib)
    from .build import source_digest
    want = source_digest()
    if want is not None and info.get("source_sha") != want:  # sources present: must match
        raise GDFError(-2, f"{path} was built from other sources (library {info.get('source_sha')}, "
                           f"tree {want}): rebuild it (build_library())")
    _lib = lib
    return lib


def build_info(lib=None) -> dict:
    """Provenance stamped into libgdf.so at compile time (gdf_build_info): the digest of the
    sources it was built from, the host that compiled it and when."""
    lib = lib or load_library()
    out = {}
    for kv in lib.gdf_build_info().decode().split(";"):
        if "=" in kv:
            k, v = kv.split("=", 1)
            out[k] = v
    return out


def _ptr(a: Optional[np.ndarray]):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


def _mat(m) -> np.ndarray:
    a = np.ascontiguousarray(np.asarray(m, dtype=np.float32).reshape(16))
    return a


def _vec3(v) -> np.ndarray:
    return np.ascontiguousarray(np.asarray(v, dtype=np.float32).reshape(3))


@dataclass
class ComponentParams:
    """GPUDepthmapFusionComponent parameters (component.cpp:1115-1187) with the launch-file
    defaults (launch/gpu_depthmap_fusion.launch:20-195)."""
    ps_filter_threshold: float = 0.05
    ps_filter_size: int = 1
    ps_timespan: float = 1.0
    flying_filter_size: int = 4
    flying_threshold: float = 0.3
    flying_rot45: bool = False
    crop_min: Sequence[float] = (-10.0, -20.0, -1.0)
    crop_max: Sequence[float] = (30.0, 20.0, 1.5)
    enable_voxel_filter: bool = True
    voxel_min: Sequence[float] = (-10.0, -20.0, -1.0)
    voxel_max: Sequence[float] = (30.0, 20.0, 1.5)
    voxel_size: Sequence[float] = (0.1, 0.1, 0.12)
    voxel_average: bool = True
    occupancy_lifetime: int = 10

    @staticmethod
    def code_defaults() -> "ComponentParams":
        """Defaults compiled into onInit when the launch file sets nothing."""
        return ComponentParams(ps_filter_threshold=0.5, ps_filter_size=1, ps_timespan=0.1,
                               flying_filter_size=1, flying_threshold=0.5, flying_rot45=True,
                               crop_min=(-1, -1, -1), crop_max=(1, 1, 1), voxel_min=(-1, -1, -1),
                               voxel_max=(1, 1, 1), voxel_size=(0.1, 0.1, 0.1),
                               occupancy_lifetime=1)

    def to_c(self, T_world_move=None, T_crop_move=None, synchronous=True,
             defer_occupancy_grid=False, defer_voxelize=False) -> FrameParams:
        p = FrameParams()
        p.ps_filter_threshold = self.ps_filter_threshold
        p.ps_filter_size = self.ps_filter_size
        p.ps_timespan = self.ps_timespan
        p.move_transform_available = 1 if T_world_move is not None else 0
        eye = np.eye(4, dtype=np.float32).reshape(16)
        p.T_world_move = _f16(*(eye if T_world_move is None else _mat(T_world_move)))
        p.T_crop_move = _f16(*(eye if T_crop_move is None else _mat(T_crop_move)))
        p.flying_filter_size = self.flying_filter_size
        p.flying_threshold = self.flying_threshold
        p.flying_rot45 = 1 if self.flying_rot45 else 0
        p.crop_min = _f3(*self.crop_min)
        p.crop_max = _f3(*self.crop_max)
        p.enable_voxel_filter = 1 if self.enable_voxel_filter else 0
        p.voxel_min = _f3(*self.voxel_min)
        p.voxel_max = _f3(*self.voxel_max)
        p.voxel_size = _f3(*self.voxel_size)
        p.voxel_average = 1 if self.voxel_average else 0
        p.occupancy_lifetime = self.occupancy_lifetime
        p.defer_occupancy_grid = 1 if defer_occupancy_grid else 0
        p.synchronous = 1 if synchronous else 0
        p.defer_voxelize = 1 if defer_voxelize else 0
        return p


class GPUDepthmapFusion:
    """Python mirror of GPUDepthmapFusion (gpu_depthmap_fusion.h:159-526) over libgdf.so."""

    def __init__(self, device: int = 0, lib_path: str = LIB_PATH):
        self._lib = load_library(lib_path)
        h = C.c_void_p()
        self._check(self._lib.gdf_create(device, C.byref(h)))
        self._h = h
        self._keep = []  # host depth maps borrowed until uploadDepthmaps

    # ---- plumbing ----
    def _check(self, rc: int):
        if rc != GDF_OK:
            raise GDFError(rc, self._lib.gdf_last_error().decode())

    def close(self):
        if getattr(self, "_h", None):
            self._lib.gdf_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def set_stream(self, stream_ptr: int):
        self._check(self._lib.gdf_set_stream(self._h, C.c_void_p(stream_ptr)))

    def set_pipeline_depth(self, depth: int):
        """Frames in flight (1..4): clear() starts the next frame on the next slot."""
        self._check(self._lib.gdf_set_pipeline_depth(self._h, depth))

    def set_graphs(self, on: bool = True):
        """Replay steady-state frames from HIP graphs (default on)."""
        self._check(self._lib.gdf_set_graphs(self._h, 1 if on else 0))

    def synchronize(self):
        self._check(self._lib.gdf_synchronize(self._h))

    def slot(self) -> int:
        """The pipeline slot the engine's calls address (gdf_get_slot)."""
        k = C.c_int(0)
        self._check(self._lib.gdf_get_slot(self._h, C.byref(k)))
        return k.value

    def set_slot_streams(self, streams: Sequence[int]):
        """Run the pipeline slots on caller-owned streams (gdf_set_slot_streams)."""
        arr = (C.c_void_p * max(len(streams), 1))(*[C.c_void_p(x) for x in streams])
        self._check(self._lib.gdf_set_slot_streams(self._h, arr, len(streams)))

    def select_slot(self, slot: int):
        """Address the frame still resident in `slot` (gdf_select_slot)."""
        self._check(self._lib.gdf_select_slot(self._h, slot))

    def stream(self) -> int:
        """The HIP stream of the addressed slot (gdf_get_stream), as an integer handle."""
        s = C.c_void_p()
        self._check(self._lib.gdf_get_stream(self._h, C.byref(s)))
        return s.value or 0

    def set_debug(self, on: bool = True):
        self._check(self._lib.gdf_set_debug(self._h, 1 if on else 0))

    # ---- inputs ----
    def clear(self):
        self._keep = []
        self._check(self._lib.gdf_clear(self._h))

    def addDepthmap(self, depth: np.ndarray, depthScale: float, fx: float, fy: float, cx: float,
                    cy: float, transform_world, transform_crop):
        d = np.ascontiguousarray(depth, dtype=np.uint16)
        H, W = d.shape
        tw, tc = _mat(transform_world), _mat(transform_crop)
        self._keep.append((d, tw, tc))
        self._check(self._lib.gdf_add_depthmap(self._h, _ptr(d), W, H, depthScale, fx, fy, cx, cy,
                                               _ptr(tw), _ptr(tc)))

    def addDepthmapDevice(self, dev_ptr: int, width: int, height: int, depthScale: float,
                          fx: float, fy: float, cx: float, cy: float, transform_world,
                          transform_crop):
        tw, tc = _mat(transform_world), _mat(transform_crop)
        self._check(self._lib.gdf_add_depthmap_device(self._h, C.c_void_p(dev_ptr), width, height,
                                                      depthScale, fx, fy, cx, cy, _ptr(tw),
                                                      _ptr(tc)))

    def addPointSequence(self, xyz: np.ndarray, timestampSec: int, timestampNSec: int,
                         transform_move):
        """xyz: (n, k>=3) float32 records (PointCloud2 with x,y,z at offsets 0/4/8)."""
        rec = np.ascontiguousarray(xyz, dtype=np.float32)
        if rec.ndim != 2 or rec.shape[1] < 3:
            raise ValueError("point records must be (n, >=3) float32")
        tm = _mat(transform_move)
        self._check(self._lib.gdf_add_point_sequence(self._h, _ptr(rec), rec.shape[0],
                                                     rec.shape[1] * 4, timestampSec,
                                                     timestampNSec, _ptr(tm)))

    def addPointSequenceDevice(self, dev_ptr: int, num_points: int, point_step: int,
                               timestampSec: int, timestampNSec: int, transform_move):
        """Records already in device memory (x,y,z f32 at byte offsets 0/4/8 of each
        point_step record); borrowed until the next uploadPointSequences / processFrame."""
        tm = _mat(transform_move)
        self._check(self._lib.gdf_add_point_sequence_device(
            self._h, C.c_void_p(dev_ptr), num_points, point_step, timestampSec, timestampNSec,
            _ptr(tm)))

    def addHaloDepthmapDevice(self, tail_ptr: int, tail_pixels: int, width: int, height: int,
                              depthScale: float, fx: float, fy: float, cx: float, cy: float,
                              transform_world, transform_crop):
        """Multi-GPU: the last `tail_pixels` depth values of the camera before this engine's
        first one (rank k-1), read by the flying-pixel filter's top-row wraps."""
        tw, tc = _mat(transform_world), _mat(transform_crop)
        self._check(self._lib.gdf_add_halo_depthmap_device(
            self._h, C.c_void_p(tail_ptr), tail_pixels, width, height, depthScale, fx, fy, cx, cy,
            _ptr(tw), _ptr(tc)))

    def numCollectedPointSequencePoints(self) -> int:
        n = C.c_uint32()
        self._check(self._lib.gdf_num_collected_point_sequence_points(self._h, C.byref(n)))
        return n.value

    # ---- point-sequence chain ----
    def uploadPointSequences(self):
        self._check(self._lib.gdf_upload_point_sequences(self._h))

    def filterNewPointSequences(self, threshold: float, filter_size: int):
        self._check(self._lib.gdf_filter_new_point_sequences(self._h, threshold, filter_size))

    def insertNewPointSequencesInRollbuffer(self):
        self._check(self._lib.gdf_insert_new_point_sequences(self._h))

    def rollPointSequenceRollbufferCPU(self, minSec: int, minNSec: int):
        self._check(self._lib.gdf_roll_rollbuffer(self._h, minSec, minNSec))

    def selectPointSequenceTimespanCPU(self, minSec, minNSec, maxSec, maxNSec):
        self._check(self._lib.gdf_select_timespan(self._h, minSec, minNSec, maxSec, maxNSec))

    def preparePointAndMaskBuffers(self):
        self._check(self._lib.gdf_prepare_point_and_mask_buffers(self._h))

    def insertSelectedPointSequence(self, tf_world_move, tf_crop_move):
        a, b = _mat(tf_world_move), _mat(tf_crop_move)
        self._check(self._lib.gdf_insert_selected_point_sequence(self._h, _ptr(a), _ptr(b)))

    def transformPointSequence(self):
        self._check(self._lib.gdf_transform_point_sequence(self._h))

    def set_rollbuffer_shard(self, shard: int, nshards: int, block: int):
        """gdf_set_rollbuffer_shard: keep the points of sequences (k // block) % nshards == shard."""
        self._check(self._lib.gdf_set_rollbuffer_shard(self._h, shard, nshards, block))

    def rollbuffer_pieces(self):
        """gdf_get_rollbuffer_pieces: the shard holding each piece of the selected window, in the
        selection's order."""
        out = (C.c_uint32 * 64)()
        n = C.c_uint32()
        self._check(self._lib.gdf_get_rollbuffer_pieces(self._h, out, 64, C.byref(n)))
        return list(out[:n.value])

    def rollbuffer_state(self) -> RollbufferState:
        st = RollbufferState()
        self._check(self._lib.gdf_get_rollbuffer_state(self._h, C.byref(st)))
        return st

    # ---- depth chain ----
    def uploadDepthmaps(self):
        self._check(self._lib.gdf_upload_depthmaps(self._h))
        self._keep = []

    def convertDepthmaps(self):
        self._check(self._lib.gdf_convert_depthmaps(self._h))

    def filterFlyingPixels(self, filter_size: int, threshold: float, enable_rot45: bool):
        self._check(self._lib.gdf_filter_flying_pixels(self._h, filter_size, threshold,
                                                       1 if enable_rot45 else 0))

    def cropPoints(self, lower_bound, upper_bound):
        lo, hi = _vec3(lower_bound), _vec3(upper_bound)
        self._check(self._lib.gdf_crop_points(self._h, _ptr(lo), _ptr(hi)))

    def applyPointMask(self) -> int:
        n = C.c_uint32()
        self._check(self._lib.gdf_apply_point_mask(self._h, C.byref(n)))
        return n.value

    def computeVoxelCoords(self, lower_bound, upper_bound, cell_size):
        lo, hi, cs = _vec3(lower_bound), _vec3(upper_bound), _vec3(cell_size)
        self._check(self._lib.gdf_compute_voxel_coords(self._h, _ptr(lo), _ptr(hi), _ptr(cs)))

    def voxelize(self, average_voxels: bool):
        self._check(self._lib.gdf_voxelize(self._h, 1 if average_voxels else 0))

    def voxelOccupancyGrid(self, lifetime: int):
        self._check(self._lib.gdf_voxel_occupancy_grid(self._h, lifetime))

    # ---- results ----
    def point_count(self) -> int:
        n = C.c_uint32()
        self._check(self._lib.gdf_get_point_count(self._h, C.byref(n)))
        return n.value

    def download_frame(self, what: int = 15) -> dict:
        """gdf_download_frame: the frame's points / voxel coords / voxelized cloud / u8 grid in
        one pass into the engine's pinned host mirrors - numpy views of them (no copy), valid
        until the slot's next download_frame."""
        hf = HostFrame()
        self._check(self._lib.gdf_download_frame(self._h, what, C.byref(hf)))

        def view(ptr, ctype, count, shape):
            if not ptr or count == 0:
                return np.zeros(shape if count == 0 else (0,), dtype=np.dtype(ctype))
            buf = (ctype * count).from_address(ptr)
            return np.ctypeslib.as_array(buf).reshape(shape)
        out = {}
        if what & DL_POINTS:
            out["points"] = view(hf.points, C.c_float, 4 * hf.num_points, (hf.num_points, 4))
        if what & DL_COORDS:
            out["voxel_coords"] = view(hf.voxel_coords, C.c_uint32, hf.num_points, (hf.num_points,))
        if what & DL_VOXELIZED:
            out["voxelized"] = view(hf.voxelized, C.c_float, 4 * hf.num_voxelized,
                                    (hf.num_voxelized, 4))
        if what & DL_GRID:
            out["occupancy"] = view(hf.occupancy, C.c_uint8, hf.num_cells, (hf.num_cells,))
        return out

    def downloadPoints(self) -> np.ndarray:
        n = self.point_count()
        out = np.empty((max(n, 1), 4), np.float32)
        cnt = C.c_uint32()
        self._check(self._lib.gdf_download_points(self._h, _ptr(out), out.shape[0], C.byref(cnt)))
        return out[:cnt.value]

    def downloadVoxelCoords(self) -> np.ndarray:
        n = self.point_count()
        out = np.empty(max(n, 1), np.uint32)
        cnt = C.c_uint32()
        self._check(self._lib.gdf_download_voxel_coords(self._h, _ptr(out), out.shape[0],
                                                        C.byref(cnt)))
        return out[:cnt.value]

    def voxelized_count(self) -> int:
        """Voxels of the last voxelize (waits for the engine's stream)."""
        cnt = C.c_uint32()
        self._check(self._lib.gdf_download_voxelized_points(self._h, None, 0, C.byref(cnt)))
        return cnt.value

    def downloadVoxelizedPoints(self) -> np.ndarray:
        cnt = C.c_uint32()
        self._check(self._lib.gdf_download_voxelized_points(self._h, None, 0, C.byref(cnt)))
        out = np.empty((max(cnt.value, 1), 4), np.float32)
        self._check(self._lib.gdf_download_voxelized_points(self._h, _ptr(out), out.shape[0],
                                                            C.byref(cnt)))
        return out[:cnt.value]

    def grid_size(self):
        g = np.zeros(3, np.uint32)
        nc = C.c_uint64()
        self._check(self._lib.gdf_get_grid_size(self._h, _ptr(g), C.byref(nc)))
        return tuple(int(x) for x in g), nc.value

    def downloadVoxelOccupancyGrid(self) -> np.ndarray:
        _, nc = self.grid_size()
        out = np.empty(max(nc, 1), np.uint8)
        self._check(self._lib.gdf_download_occupancy_grid(self._h, _ptr(out), out.shape[0]))
        return out[:nc]

    def historic_grid(self) -> np.ndarray:
        _, nc = self.grid_size()
        out = np.empty(max(nc, 1), np.uint32)
        self._check(self._lib.gdf_debug_historic_grid(self._h, _ptr(out), out.shape[0]))
        return out[:nc]

    def stage_masks(self) -> np.ndarray:
        cnt = C.c_uint32()
        self._check(self._lib.gdf_debug_stage_masks(self._h, None, 0, C.byref(cnt)))
        out = np.empty(max(cnt.value, 1), np.uint8)
        self._check(self._lib.gdf_debug_stage_masks(self._h, _ptr(out), out.shape[0],
                                                    C.byref(cnt)))
        return out[:cnt.value]

    def rollbuffer_arrays(self):
        st = self.rollbuffer_state()
        R, S = st.num_points, st.num_seqs
        pts = np.empty((max(R, 1), 4), np.float32)
        mask = np.empty(max(R, 1), np.uint32)
        seq = np.empty(max(R, 1), np.uint32)
        hdr = np.empty((max(S, 1), 4), np.uint32)
        self._check(self._lib.gdf_debug_rollbuffer(self._h, _ptr(pts), _ptr(mask), _ptr(seq),
                                                   pts.shape[0], _ptr(hdr), hdr.shape[0]))
        return pts[:R], mask[:R], seq[:R], hdr[:S]

    def device_results(self):
        p, c, v, o = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        self._check(self._lib.gdf_get_device_results(self._h, C.byref(p), C.byref(c),
                                                     C.byref(v), C.byref(o)))
        return p.value, c.value, v.value, o.value

    def export_marks(self, dev_ptr: int, words: int):
        self._check(self._lib.gdf_export_occupancy_marks(self._h, C.c_void_p(dev_ptr), words))

    def import_marks(self, dev_ptr: int, words: int, nranks: int, rank_stride: int = 0):
        if rank_stride:
            self._check(self._lib.gdf_import_occupancy_marks_strided(
                self._h, C.c_void_p(dev_ptr), words, nranks, rank_stride))
        else:
            self._check(self._lib.gdf_import_occupancy_marks(self._h, C.c_void_p(dev_ptr), words,
                                                             nranks))

    def voxelOccupancyGridBatch(self, dev_ptr: int, words: int, nranks: int, nframes: int,
                                frame_stride: int, rank_stride: int, lifetime: int):
        """nframes grid updates in one pass from all-gathered mark masks (batched exchange)."""
        self._check(self._lib.gdf_voxel_occupancy_grid_batch(
            self._h, C.c_void_p(dev_ptr), words, nranks, nframes, frame_stride, rank_stride,
            lifetime))

    def take_marks_sparse(self, dev_ptr: int, words: int, pairs_ptr: int, cap: int):
        """take_marks plus the non-zero words as (index, word) pairs (pairs[0] = count)."""
        self._check(self._lib.gdf_take_occupancy_marks_sparse(
            self._h, C.c_void_p(dev_ptr), words, C.c_void_p(pairs_ptr), cap))

    def union_pairs(self, union_ptr: int, words: int, pairs_ptr: int, nranks: int, nframes: int,
                    record_words: int, frames_per_rank: int = 0):
        """OR the first `nframes` sparse records of every rank (records laid out
        [rank, frames_per_rank, record_words]) into per-frame bitmasks."""
        self._check(self._lib.gdf_union_occupancy_pairs(
            self._h, C.c_void_p(union_ptr), words, C.c_void_p(pairs_ptr), nranks, nframes,
            frames_per_rank or nframes, record_words))

    def take_marks(self, dev_ptr: int, words: int):
        """Export the marks of the frame just processed and clear them (batched exchange)."""
        self._check(self._lib.gdf_take_occupancy_marks(self._h, C.c_void_p(dev_ptr), words))

    # ---- whole frame ----
    def set_profiling(self, on: bool = True):
        self._check(self._lib.gdf_set_profiling(self._h, 1 if on else 0))

    def kernel_times(self):
        """{slot: (ms_sum, launches)} of the event-timed launches since set_profiling."""
        k = len(KERNEL_SLOTS)
        ms = np.zeros(k, np.float64)
        n = np.zeros(k, np.uint64)
        self._check(self._lib.gdf_get_kernel_times(self._h, _ptr(ms), _ptr(n), k))
        return {k: (float(ms[i]), int(n[i])) for i, k in enumerate(KERNEL_SLOTS)}

    def processFrame(self, params: ComponentParams, T_world_move=None, T_crop_move=None,
                     synchronous: bool = True, defer_occupancy_grid: bool = False,
                     defer_voxelize: bool = False) -> FrameResult:
        p = params.to_c(T_world_move, T_crop_move, synchronous, defer_occupancy_grid,
                        defer_voxelize)
        return self.processFramePrepared(p)

    def make_stream_camera(self, dev_ptrs: Sequence[int], width: int, height: int,
                           depthScale: float, fx: float, fy: float, cx: float, cy: float,
                           T_world, T_crop) -> StreamCamera:
        """A camera of gdf_run_depth_stream: a ring of device depth maps + its geometry."""
        c = StreamCamera()
        arr = (C.c_void_p * len(dev_ptrs))(*dev_ptrs)
        c.frames = C.cast(arr, C.POINTER(C.c_void_p))
        c._frames_keepalive = arr
        c.ring, c.width, c.height = len(dev_ptrs), width, height
        c.depth_scale, c.fx, c.fy, c.cx, c.cy = depthScale, fx, fy, cx, cy
        c.T_world[:] = _mat(T_world).ravel().tolist()
        c.T_crop[:] = _mat(T_crop).ravel().tolist()
        return c

    def run_depth_stream(self, cameras: Sequence[StreamCamera], p: FrameParams, first: int,
                         count: int):
        """Frames first..first+count-1 through the C++ component loop (gdf_run_depth_stream):
        clear + addDepthmapDevice per camera + processFrame, without Python per frame."""
        arr = (StreamCamera * len(cameras))(*cameras)
        self._check(self._lib.gdf_run_depth_stream(self._h, arr, len(cameras), C.byref(p),
                                                   first, count))

    def run_host_stream(self, cameras: Sequence[StreamCamera], p: FrameParams, first: int,
                        count: int):
        """gdf_run_host_stream: the same loop with HOST depth maps (copied through the slot's
        pinned staging, H2D on the slot's stream, overlapped with the frames in flight)."""
        arr = (StreamCamera * len(cameras))(*cameras)
        self._check(self._lib.gdf_run_host_stream(self._h, arr, len(cameras), C.byref(p),
                                                  first, count))

    def run_depth_stream_batched(self, cameras: Sequence[StreamCamera], p: FrameParams,
                                 first: int, batches: int, batch: int, host: bool = False):
        """gdf_run_depth_stream_batched: `batches` multi-frame batches of `batch` frames."""
        arr = (StreamCamera * len(cameras))(*cameras)
        self._check(self._lib.gdf_run_depth_stream_batched(self._h, arr, len(cameras), C.byref(p),
                                                           first, batches, batch,
                                                           1 if host else 0))

    def run_depth_stream_alternating(self, cameras: Sequence[StreamCamera],
                                     params: Sequence[FrameParams], first: int, batches: int,
                                     batch: int):
        """gdf_run_depth_stream_alternating: step b uses params[(first + b) % len(params)]."""
        arr = (StreamCamera * len(cameras))(*cameras)
        ps = (FrameParams * len(params))(*params)
        self._check(self._lib.gdf_run_depth_stream_alternating(self._h, arr, len(cameras), ps,
                                                               len(params), first, batches, batch))

    # ---- multi-GPU fused cloud ----
    def partition_points(self, nparts: int, send_pts_ptr: int, send_keys_ptr: int,
                         capacity: int, part_counts_ptr: int):
        """Split the frame's (point, key) list by voxel-key range into part-major buffers."""
        self._check(self._lib.gdf_partition_points(self._h, nparts, C.c_void_p(send_pts_ptr),
                                                   C.c_void_p(send_keys_ptr), capacity,
                                                   C.c_void_p(part_counts_ptr)))

    def voxelize_points(self, pts_ptr: int, keys_ptr: int, count: int, average: bool = True):
        """Voxelize an external (point, key) list (what this rank received)."""
        self._check(self._lib.gdf_voxelize_points(self._h, C.c_void_p(pts_ptr),
                                                  C.c_void_p(keys_ptr), count,
                                                  1 if average else 0))

    def partition_runs(self, nparts: int, send_pts_ptr: int, send_run_keys_ptr: int,
                       send_run_starts_ptr: int, capacity: int, part_counts_ptr: int):
        """partition_points with runs of equal keys instead of per-point keys (gdf_partition_runs):
        part_counts = points per part, then runs per part."""
        self._check(self._lib.gdf_partition_runs(
            self._h, nparts, C.c_void_p(send_pts_ptr), C.c_void_p(send_run_keys_ptr),
            C.c_void_p(send_run_starts_ptr), capacity, C.c_void_p(part_counts_ptr)))

    def set_emit_partition(self, nparts: int, send_pts_ptr: int = 0, send_run_keys_ptr: int = 0,
                           send_run_starts_ptr: int = 0, capacity: int = 0, part_counts_ptr: int = 0):
        """The next deferred frame's compaction writes partition_runs' send lists itself
        (gdf_set_emit_partition; nparts = 0 disarms)."""
        self._check(self._lib.gdf_set_emit_partition(
            self._h, nparts, C.c_void_p(send_pts_ptr), C.c_void_p(send_run_keys_ptr),
            C.c_void_p(send_run_starts_ptr), capacity, C.c_void_p(part_counts_ptr)))

    def voxelize_runs(self, pts_ptr: int, run_keys_ptr: int, run_starts_ptr: int,
                      point_base, run_base, average: bool = True):
        """Voxelize received run segments (gdf_voxelize_runs): point_base / run_base = the
        sources' offsets, nsources + 1 entries each."""
        pb = np.ascontiguousarray(point_base, np.uint32)
        rb = np.ascontiguousarray(run_base, np.uint32)
        self._check(self._lib.gdf_voxelize_runs(self._h, C.c_void_p(pts_ptr),
                                                C.c_void_p(run_keys_ptr), C.c_void_p(run_starts_ptr),
                                                len(pb) - 1, _ptr(pb), _ptr(rb),
                                                1 if average else 0))

    def set_partition_marks(self, enabled: bool):
        """Whether frames armed with set_emit_partition set their occupancy marks
        (gdf_set_partition_marks; off when the union comes from voxelize_runs_marked)."""
        self._check(self._lib.gdf_set_partition_marks(self._h, 1 if enabled else 0))

    def voxelize_runs_marked(self, pts_ptr: int, run_keys_ptr: int, run_starts_ptr: int,
                             point_base, run_base, marks_ptr: int, frame_stride_words: int,
                             average: bool = True):
        """voxelize_runs that also ORs every voxel's occupancy mark into marks_ptr (device, frame
        f at f * frame_stride_words, zeroed by the caller; gdf_voxelize_runs_marked)."""
        pb = np.ascontiguousarray(point_base, np.uint32)
        rb = np.ascontiguousarray(run_base, np.uint32)
        self._check(self._lib.gdf_voxelize_runs_marked(
            self._h, C.c_void_p(pts_ptr), C.c_void_p(run_keys_ptr), C.c_void_p(run_starts_ptr),
            len(pb) - 1, _ptr(pb), _ptr(rb), 1 if average else 0, C.c_void_p(marks_ptr),
            frame_stride_words))

    # ---- orphan shaders (device buffers) ----
    def maskDilate(self, in_ptr: int, out_ptr: int, width: int, height: int, filter_size: int,
                   as_written: bool = False):
        """sh/mask_dilate.glsl on device u32 masks (intended erosion, or as written)."""
        self._check(self._lib.gdf_mask_dilate(self._h, C.c_void_p(in_ptr), C.c_void_p(out_ptr),
                                              width, height, filter_size, 1 if as_written else 0))

    def transformPoints(self, in_ptr: int, mask_ptr: int, out_ptr: int, num_items: int,
                        transform):
        """sh/transform_points.glsl on device float4 points + u32 mask."""
        t = _mat(transform)
        self._check(self._lib.gdf_transform_points(self._h, C.c_void_p(in_ptr),
                                                   C.c_void_p(mask_ptr), C.c_void_p(out_ptr),
                                                   num_items, _ptr(t)))

    # ---- multi-frame batches ----
    def nextFrameInBatch(self):
        """The depth maps added from now on belong to the next frame of this batch."""
        self._check(self._lib.gdf_next_frame_in_batch(self._h))

    def batch_ranges(self):
        """(point_start, voxel_start) arrays of nframes + 1 entries of the last batch."""
        nf = C.c_uint32()
        self._check(self._lib.gdf_get_batch_ranges(self._h, None, None, 0, C.byref(nf)))
        ps = np.zeros(nf.value + 1, np.uint32)
        vs = np.zeros(nf.value + 1, np.uint32)
        self._check(self._lib.gdf_get_batch_ranges(self._h, _ptr(ps), _ptr(vs), nf.value + 1,
                                                   C.byref(nf)))
        return ps, vs

    def downloadBatchVoxelOccupancyGrid(self, frame: int) -> np.ndarray:
        _, nc = self.grid_size()
        out = np.empty(max(nc, 1), np.uint8)
        self._check(self._lib.gdf_download_batch_occupancy_grid(self._h, frame, _ptr(out),
                                                                out.shape[0]))
        return out[:nc]

    def graph_stats(self):
        """(captures, replays) of the slots' frame graphs (instrumentation; include/gdf.h)."""
        c, r = C.c_uint64(0), C.c_uint64(0)
        self._check(self._lib.gdf_get_graph_stats(self._h, C.byref(c), C.byref(r)))
        return c.value, r.value

    def tuning(self) -> str:
        """gdf_get_tuning: the GDF_* tuning variables this engine was created under ("" = the
        built-in defaults)."""
        buf = C.create_string_buffer(4096)
        self._check(self._lib.gdf_get_tuning(self._h, buf, len(buf)))
        return buf.value.decode()

    def last_sort_items(self):
        """(items, runs): what the last synchronous processFrame's voxelize sorted - runs of
        equal voxel keys (runs True) or points (instrumentation; include/gdf.h)."""
        n, r = C.c_uint32(0), C.c_int(0)
        self._check(self._lib.gdf_last_sort_items(self._h, C.byref(n), C.byref(r)))
        return n.value, bool(r.value)

    def processFramePrepared(self, p: FrameParams) -> FrameResult:
        """processFrame with parameters already converted by ComponentParams.to_c (a stream of
        frames with fixed parameters converts them once)."""
        r = FrameResult()
        self._check(self._lib.gdf_process_frame(self._h, C.byref(p), C.byref(r)))
        self._keep = []
        return r


# segmentation flags (include/gdf_segment.h)
SEG_CONTOURS, SEG_CONNECTIONS, SEG_ALL = 1, 2, 3


class Segmenter:
    """GPU object-segmentation front end (include/gdf_segment.h): labelVoxels +
    layers connections + mergeLabelsAcrossLayers of the reference's objectSegmentation
    (src/gpu_depthmap_fusion.cpp:1872-2361) on a device u8 grid [layers, height, width]."""

    def __init__(self, device: int = 0, lib_path: str = LIB_PATH):
        self._lib = load_library(lib_path)
        h = C.c_void_p()
        self._check(self._lib.gdf_seg_create(device, C.byref(h)))
        self._h = h

    def _check(self, rc: int):
        if rc != GDF_OK:
            raise GDFError(rc, (self._lib.gdf_last_error() or b"").decode())

    def close(self):
        if getattr(self, "_h", None):
            self._lib.gdf_seg_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_ptr: int):
        self._check(self._lib.gdf_seg_set_stream(self._h, C.c_void_p(stream_ptr)))

    def label_layers(self, grid_ptr: int, width: int, height: int, layers: int,
                     flags: int = SEG_ALL):
        """objectSegmentation front end on a device grid (a torch uint8 tensor's data_ptr())."""
        self._check(self._lib.gdf_seg_label_layers(self._h, C.c_void_p(grid_ptr), width, height,
                                                   layers, flags))

    def label_engine_grid(self, engine: "GPUDepthmapFusion", flags: int = SEG_ALL):
        """The same on the engine's current occupancy grid (after voxelOccupancyGrid)."""
        self._check(self._lib.gdf_seg_label_engine_grid(self._h, engine._h, flags))

    def counts(self) -> SegCounts:
        c = SegCounts()
        self._check(self._lib.gdf_seg_get_counts(self._h, C.byref(c)))
        return c

    def results(self, contours: bool = True, connections: bool = True) -> dict:
        """Every output as flat arrays with the keys of oracle.object_segmentation_front."""
        c = self.counts()
        L, H, W, T = c.layers, c.height, c.width, c.total_labels
        r = {}
        r["labels"] = np.zeros((L, H, W), np.uint16)
        self._check(self._lib.gdf_seg_download_labels(self._h, _ptr(r["labels"]), L * H * W))
        r["num_labels"] = np.zeros(L, np.uint32)
        self._check(self._lib.gdf_seg_download_num_labels(self._h, _ptr(r["num_labels"]), L))
        r["stats"] = np.zeros((T, 5), np.int32)
        r["centroids"] = np.zeros((T, 2), np.float64)
        self._check(self._lib.gdf_seg_download_stats(self._h, _ptr(r["stats"]),
                                                     _ptr(r["centroids"]), T))
        if contours:
            r["labels_to_contours"] = np.zeros(T, np.int32)
            r["contours_per_layer"] = np.zeros(L, np.uint32)
            r["contour_sizes"] = np.zeros(c.total_contours, np.uint32)
            r["contour_points"] = np.zeros((c.total_contour_points, 2), np.int32)
            self._check(self._lib.gdf_seg_download_contours(
                self._h, _ptr(r["labels_to_contours"]), _ptr(r["contours_per_layer"]),
                _ptr(r["contour_sizes"]), _ptr(r["contour_points"]), c.total_contour_points))
        if connections:
            r["connections"] = np.zeros(c.connection_bytes, np.uint8)
            r["connection_starts"] = np.zeros(max(L - 1, 0), np.uint64)
            self._check(self._lib.gdf_seg_download_connections(
                self._h, _ptr(r["connections"]), c.connection_bytes,
                _ptr(r["connection_starts"]), max(L - 1, 0)))
            r["merged"] = np.zeros(T, np.uint32)
            nobj = C.c_uint32(0)
            self._check(self._lib.gdf_seg_merge_labels(self._h, _ptr(r["merged"]), T,
                                                       C.byref(nobj)))
            r["num_objects"] = nobj.value
        return r

    def merge_labels(self):
        """mergeLabelsAcrossLayers (fusion.cpp:2243-2361, on the device): (merged ids [T], n)."""
        T = self.counts().total_labels
        merged = np.zeros(T, np.uint32)
        nobj = C.c_uint32(0)
        self._check(self._lib.gdf_seg_merge_labels(self._h, _ptr(merged), T, C.byref(nobj)))
        return merged, nobj.value

    def create_objects(self, lower, cell_size):
        """createCCObjects' aggregate fields (no OpenCV shapes): (columns dict, components)."""
        lo, cs = _vec3(lower), _vec3(cell_size)
        n = C.c_uint32(0)
        self._check(self._lib.gdf_seg_create_objects(self._h, _ptr(lo), _ptr(cs), None, 0, None,
                                                     0, C.byref(n)))
        objs = (CCObject * max(n.value, 1))()
        T = self.counts().total_labels
        comps = np.zeros(T, np.uint32)
        self._check(self._lib.gdf_seg_create_objects(self._h, _ptr(lo), _ptr(cs), objs, n.value,
                                                     _ptr(comps), T, C.byref(n)))
        return cc_objects_as_dict(objs[:n.value]), comps
