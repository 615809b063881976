"""ctypes binding of the CPU oracle (oracle/gdf_oracle.c) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
`OracleFusion` has the same method names as ros_gpu_depthmap_fusion_amd.gdf.GPUDepthmapFusion
(which mirror the reference's GPUDepthmapFusion), so a parity test drives both through one call
sequence.  `RefRadix` wraps oracle/_ref/libref_radix.so: the reference's own radix_grouper.h /
radix_sort.h compiled from /root/reference (present only in the build container).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")
REF_LIB = os.path.join(HERE, "_ref", "libref_radix.so")

_f3 = C.c_float * 3
_f16 = C.c_float * 16


def build(quiet: bool = True) -> None:
    """Compile the oracle (and oracle/_ref when the reference sources are present)."""
    out = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)


class OrcFrameParams(C.Structure):
    _fields_ = [
        ("ps_filter_threshold", C.c_float), ("ps_filter_size", C.c_uint32),
        ("ps_timespan", C.c_float), ("move_transform_available", C.c_int32),
        ("T_world_move", _f16), ("T_crop_move", _f16),
        ("flying_filter_size", C.c_uint32), ("flying_threshold", C.c_float),
        ("flying_rot45", C.c_int32), ("crop_min", _f3), ("crop_max", _f3),
        ("enable_voxel_filter", C.c_int32), ("voxel_min", _f3), ("voxel_max", _f3),
        ("voxel_size", _f3), ("voxel_average", C.c_int32), ("occupancy_lifetime", C.c_uint32),
        ("synchronous", C.c_int32),
    ]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    vp, u32, i32, f, u64 = C.c_void_p, C.c_uint32, C.c_int, C.c_float, C.c_uint64
    P = C.POINTER
    sig = {
        "orc_create": (vp, []), "orc_destroy": (None, [vp]), "orc_set_threads": (None, [vp, i32]),
        "orc_clear": (None, [vp]),
        "orc_add_depthmap": (i32, [vp, vp, u32, u32, f, f, f, f, f, vp, vp]),
        "orc_add_point_sequence": (i32, [vp, vp, u32, u32, u32, u32, vp]),
        "orc_num_collected_point_sequence_points": (u32, [vp]),
        "orc_upload_point_sequences": (i32, [vp]),
        "orc_filter_new_point_sequences": (i32, [vp, f, u32]),
        "orc_insert_new_point_sequences": (i32, [vp]),
        "orc_roll_rollbuffer": (i32, [vp, u32, u32]),
        "orc_select_timespan": (i32, [vp, u32, u32, u32, u32]),
        "orc_prepare_point_and_mask_buffers": (i32, [vp]),
        "orc_insert_selected_point_sequence": (i32, [vp, vp, vp]),
        "orc_transform_point_sequence": (i32, [vp]),
        "orc_upload_depthmaps": (i32, [vp]), "orc_convert_depthmaps": (i32, [vp]),
        "orc_filter_flying_pixels": (i32, [vp, u32, f, i32]),
        "orc_crop_points": (i32, [vp, vp, vp]),
        "orc_apply_point_mask": (i32, [vp, P(u32)]),
        "orc_compute_voxel_coords": (i32, [vp, vp, vp, vp]),
        "orc_voxelize": (i32, [vp, i32]), "orc_voxel_occupancy_grid": (i32, [vp, u32]),
        "orc_process_frame": (i32, [vp, P(OrcFrameParams), P(C.c_int32), P(u32), P(u32)]),
        "orc_ros_time_minus": (i32, [u32, u32, C.c_double, P(u32), P(u32)]),
        "orc_num_points_total": (u32, [vp]), "orc_num_depth_points": (u32, [vp]),
        "orc_num_points": (u32, [vp]),
        "orc_mask_a": (vp, [vp]), "orc_mask_b": (vp, [vp]),
        "orc_points_a": (vp, [vp]), "orc_points_b": (vp, [vp]), "orc_points_c": (vp, [vp]),
        "orc_voxel_coords": (vp, [vp]), "orc_voxelized": (vp, [vp, P(u32)]),
        "orc_occupancy": (vp, [vp, P(u64)]), "orc_historic": (vp, [vp, P(u64)]),
        "orc_grid_size": (None, [vp, vp]), "orc_new_ps_mask": (vp, [vp, P(u32)]),
        "orc_rollbuffer_state": (None, [vp, vp]),
        "orc_rollbuffer_b": (u32, [vp, P(vp), P(vp), P(vp), P(vp), P(u32)]),
        "orc_stable_sort_keys": (None, [vp, u32, vp, vp]),
        "orc_mask_dilate": (None, [vp, vp, u32, u32, u32, i32]),
        "orc_transform_points": (None, [vp, vp, vp, u32, vp]),
        "orc_seg_run": (vp, [vp, u32, u32, u32]), "orc_seg_counts": (None, [vp, vp]),
        "orc_seg_get": (None, [vp] + [vp] * 11), "orc_seg_free": (None, [vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def _arr(ptr, dtype, shape):
    n = int(np.prod(shape))
    if n == 0 or not ptr:
        return np.zeros(shape, dtype)
    buf = (C.c_char * (n * np.dtype(dtype).itemsize)).from_address(ptr)
    return np.frombuffer(buf, dtype=dtype).reshape(shape).copy()


def _p(a):
    return a.ctypes.data_as(C.c_void_p)


def _m(m):
    return np.ascontiguousarray(np.asarray(m, np.float32).reshape(16))


def _v(v):
    return np.ascontiguousarray(np.asarray(v, np.float32).reshape(3))


class OracleError(RuntimeError):
    pass


class OracleFusion:
    """CPU restatement with the reference's method names (see gdf_oracle.h)."""

    def __init__(self, threads: int = 1):
        self._lib = load()
        self._h = self._lib.orc_create()
        self._lib.orc_set_threads(self._h, threads)
        self._keep = []

    def close(self):
        if self._h:
            self._lib.orc_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _ck(self, rc):
        if rc != 0:
            raise OracleError(f"oracle call failed with {rc}")

    def set_threads(self, n):
        self._lib.orc_set_threads(self._h, n)

    # inputs
    def clear(self):
        self._lib.orc_clear(self._h)

    def addDepthmap(self, depth, depthScale, fx, fy, cx, cy, transform_world, transform_crop):
        d = np.ascontiguousarray(depth, np.uint16)
        tw, tc = _m(transform_world), _m(transform_crop)
        self._keep.append((d, tw, tc))
        H, W = d.shape
        self._ck(self._lib.orc_add_depthmap(self._h, _p(d), W, H, depthScale, fx, fy, cx, cy,
                                            _p(tw), _p(tc)))

    def addPointSequence(self, xyz, timestampSec, timestampNSec, transform_move):
        rec = np.ascontiguousarray(xyz, np.float32)
        tm = _m(transform_move)
        self._ck(self._lib.orc_add_point_sequence(self._h, _p(rec), rec.shape[0],
                                                  rec.shape[1] * 4, timestampSec, timestampNSec,
                                                  _p(tm)))

    def numCollectedPointSequencePoints(self):
        return self._lib.orc_num_collected_point_sequence_points(self._h)

    # point-sequence chain
    def uploadPointSequences(self):
        self._ck(self._lib.orc_upload_point_sequences(self._h))

    def filterNewPointSequences(self, threshold, filter_size):
        self._ck(self._lib.orc_filter_new_point_sequences(self._h, threshold, filter_size))

    def insertNewPointSequencesInRollbuffer(self):
        self._ck(self._lib.orc_insert_new_point_sequences(self._h))

    def rollPointSequenceRollbufferCPU(self, s, ns):
        self._ck(self._lib.orc_roll_rollbuffer(self._h, s, ns))

    def selectPointSequenceTimespanCPU(self, a, b, c, d):
        self._ck(self._lib.orc_select_timespan(self._h, a, b, c, d))

    def preparePointAndMaskBuffers(self):
        self._ck(self._lib.orc_prepare_point_and_mask_buffers(self._h))

    def insertSelectedPointSequence(self, twm, tcm):
        a, b = _m(twm), _m(tcm)
        self._ck(self._lib.orc_insert_selected_point_sequence(self._h, _p(a), _p(b)))

    def transformPointSequence(self):
        self._ck(self._lib.orc_transform_point_sequence(self._h))

    def rollbuffer_state(self):
        o = np.zeros(10, np.uint32)
        self._lib.orc_rollbuffer_state(self._h, _p(o))
        return tuple(int(x) for x in o)

    # depth chain
    def uploadDepthmaps(self):
        self._ck(self._lib.orc_upload_depthmaps(self._h))

    def convertDepthmaps(self):
        self._ck(self._lib.orc_convert_depthmaps(self._h))

    def filterFlyingPixels(self, filter_size, threshold, enable_rot45):
        self._ck(self._lib.orc_filter_flying_pixels(self._h, filter_size, threshold,
                                                    1 if enable_rot45 else 0))

    def cropPoints(self, lo, hi):
        a, b = _v(lo), _v(hi)
        self._ck(self._lib.orc_crop_points(self._h, _p(a), _p(b)))

    def applyPointMask(self):
        n = C.c_uint32()
        self._ck(self._lib.orc_apply_point_mask(self._h, C.byref(n)))
        return n.value

    def computeVoxelCoords(self, lo, hi, cs):
        a, b, c = _v(lo), _v(hi), _v(cs)
        self._ck(self._lib.orc_compute_voxel_coords(self._h, _p(a), _p(b), _p(c)))

    def voxelize(self, average):
        self._ck(self._lib.orc_voxelize(self._h, 1 if average else 0))

    def voxelOccupancyGrid(self, lifetime):
        self._ck(self._lib.orc_voxel_occupancy_grid(self._h, lifetime))

    def processFrame(self, params, T_world_move=None, T_crop_move=None, synchronous=True):
        p = OrcFrameParams()
        p.ps_filter_threshold = params.ps_filter_threshold
        p.ps_filter_size = params.ps_filter_size
        p.ps_timespan = params.ps_timespan
        p.move_transform_available = 1 if T_world_move is not None else 0
        eye = np.eye(4, dtype=np.float32).reshape(16)
        p.T_world_move = _f16(*(eye if T_world_move is None else _m(T_world_move)))
        p.T_crop_move = _f16(*(eye if T_crop_move is None else _m(T_crop_move)))
        p.flying_filter_size = params.flying_filter_size
        p.flying_threshold = params.flying_threshold
        p.flying_rot45 = 1 if params.flying_rot45 else 0
        p.crop_min = _f3(*params.crop_min)
        p.crop_max = _f3(*params.crop_max)
        p.enable_voxel_filter = 1 if params.enable_voxel_filter else 0
        p.voxel_min = _f3(*params.voxel_min)
        p.voxel_max = _f3(*params.voxel_max)
        p.voxel_size = _f3(*params.voxel_size)
        p.voxel_average = 1 if params.voxel_average else 0
        p.occupancy_lifetime = params.occupancy_lifetime
        processed, ls, lns = C.c_int32(), C.c_uint32(), C.c_uint32()
        self._ck(self._lib.orc_process_frame(self._h, C.byref(p), C.byref(processed),
                                             C.byref(ls), C.byref(lns)))
        self._keep = []
        return processed.value, ls.value, lns.value

    # results
    def point_count(self):
        return self._lib.orc_num_points(self._h)

    def num_points_total(self):
        return self._lib.orc_num_points_total(self._h)

    def downloadPoints(self):
        n = self.point_count()
        return _arr(self._lib.orc_points_a(self._h), np.float32, (n, 4))

    def downloadVoxelCoords(self):
        return _arr(self._lib.orc_voxel_coords(self._h), np.uint32, (self.point_count(),))

    def downloadVoxelizedPoints(self):
        n = C.c_uint32()
        p = self._lib.orc_voxelized(self._h, C.byref(n))
        return _arr(p, np.float32, (n.value, 4))

    def downloadVoxelOccupancyGrid(self):
        nc = C.c_uint64()
        p = self._lib.orc_occupancy(self._h, C.byref(nc))
        return _arr(p, np.uint8, (nc.value,))

    def historic_grid(self):
        nc = C.c_uint64()
        p = self._lib.orc_historic(self._h, C.byref(nc))
        return _arr(p, np.uint32, (nc.value,))

    def grid_size(self):
        g = np.zeros(3, np.uint32)
        self._lib.orc_grid_size(self._h, _p(g))
        return tuple(int(x) for x in g)

    def stage_arrays(self):
        n = self.num_points_total()
        return dict(
            maskA=_arr(self._lib.orc_mask_a(self._h), np.uint32, (n,)),
            maskB=_arr(self._lib.orc_mask_b(self._h), np.uint32, (n,)),
            A=_arr(self._lib.orc_points_a(self._h), np.float32, (n, 4)),
            B=_arr(self._lib.orc_points_b(self._h), np.float32, (n, 4)),
            C=_arr(self._lib.orc_points_c(self._h), np.float32, (n, 4)),
        )

    def rollbuffer_arrays(self):
        pts, mask, seq, hdr = C.c_void_p(), C.c_void_p(), C.c_void_p(), C.c_void_p()
        ns = C.c_uint32()
        R = self._lib.orc_rollbuffer_b(self._h, C.byref(pts), C.byref(mask), C.byref(seq),
                                       C.byref(hdr), C.byref(ns))
        return (_arr(pts.value, np.float32, (R, 4)), _arr(mask.value, np.uint32, (R,)),
                _arr(seq.value, np.uint32, (R,)), _arr(hdr.value, np.uint32, (ns.value, 4)))

    def new_ps_mask(self):
        n = C.c_uint32()
        p = self._lib.orc_new_ps_mask(self._h, C.byref(n))
        return _arr(p, np.uint32, (n.value,))


def stable_sort_keys(keys: np.ndarray):
    lib = load()
    k = np.ascontiguousarray(keys, np.uint32)
    idx = np.empty(len(k), np.uint32)
    sk = np.empty(len(k), np.uint32)
    lib.orc_stable_sort_keys(_p(k), len(k), _p(idx), _p(sk))
    return idx, sk


def mask_dilate(mask: np.ndarray, filter_size: int, as_written: bool = False) -> np.ndarray:
    """sh/mask_dilate.glsl:40-67 on an (H, W) u32 mask (see gdf_oracle.h)."""
    lib = load()
    m = np.ascontiguousarray(mask, np.uint32)
    H, W = m.shape
    out = np.empty_like(m)
    lib.orc_mask_dilate(_p(m), _p(out), W, H, filter_size, 1 if as_written else 0)
    return out


def transform_points(points: np.ndarray, mask: np.ndarray, T, out: np.ndarray) -> np.ndarray:
    """sh/transform_points.glsl:37-54: out[i] = T * points[i] where mask[i] != 0 (others kept)."""
    lib = load()
    pts = np.ascontiguousarray(points, np.float32)
    m = np.ascontiguousarray(mask, np.uint32)
    o = np.ascontiguousarray(out, np.float32).copy()
    lib.orc_transform_points(_p(pts), _p(m), _p(o), len(pts), _p(_m(T)))
    return o


def ros_time_minus(sec, nsec, seconds):
    lib = load()
    a, b = C.c_uint32(), C.c_uint32()
    rc = lib.orc_ros_time_minus(sec, nsec, float(seconds), C.byref(a), C.byref(b))
    return None if rc else (a.value, b.value)


class RefRadix:
    """The reference's own RadixGrouper (oracle/_ref), when built in this container."""

    def __init__(self):
        if not os.path.exists(REF_LIB):
            raise FileNotFoundError(REF_LIB)
        self._lib = C.CDLL(REF_LIB)
        self._lib.ref_radix_group.restype = C.c_int
        self._lib.ref_radix_group.argtypes = [C.c_void_p, C.c_uint32, C.c_int] + [C.c_void_p] * 5 + [
            C.POINTER(C.c_uint32)]

    @staticmethod
    def available() -> bool:
        return os.path.exists(REF_LIB)

    def group(self, keys: np.ndarray, group_size: int = 8):
        k = np.ascontiguousarray(keys, np.uint32)
        n = len(k)
        si = np.empty(max(n, 1), np.uint32)
        sk = np.empty(max(n, 1), np.uint32)
        gs = np.empty(max(n, 1), np.uint32)
        gz = np.empty(max(n, 1), np.uint32)
        gv = np.empty(max(n, 1), np.uint32)
        ng = C.c_uint32()
        self._lib.ref_radix_group(_p(k), n, group_size, _p(si), _p(sk), _p(gs), _p(gz), _p(gv),
                                  C.byref(ng))
        g = ng.value
        return si[:n], sk[:n], gs[:g], gz[:g], gv[:g]


def object_segmentation_front(grid: np.ndarray) -> dict:
    """labelVoxels + layers connections + mergeLabelsAcrossLayers (oracle/seg_oracle.c) on a u8
    grid [layers, height, width]; flat arrays with the keys of gdf.Segmenter.results()."""
    lib = load()
    g = np.ascontiguousarray(grid, np.uint8)
    L, H, W = g.shape
    h = lib.orc_seg_run(_p(g), W, H, L)
    try:
        c = np.zeros(5, np.uint64)
        lib.orc_seg_counts(h, _p(c))
        T, NC, NP, CB, nobj = (int(v) for v in c)
        r = dict(labels=np.zeros((L, H, W), np.uint16), num_labels=np.zeros(L, np.uint32),
                 stats=np.zeros((T, 5), np.int32), centroids=np.zeros((T, 2), np.float64),
                 labels_to_contours=np.zeros(T, np.int32),
                 contours_per_layer=np.zeros(L, np.uint32), contour_sizes=np.zeros(NC, np.uint32),
                 contour_points=np.zeros((NP, 2), np.int32), connections=np.zeros(CB, np.uint8),
                 connection_starts=np.zeros(max(L - 1, 0), np.uint64),
                 merged=np.zeros(T, np.uint32), num_objects=nobj)
        lib.orc_seg_get(h, *[_p(r[k]) for k in (
            "labels", "num_labels", "stats", "centroids", "labels_to_contours",
            "contours_per_layer", "contour_sizes", "contour_points", "connections",
            "connection_starts", "merged")])
        return r
    finally:
        lib.orc_seg_free(h)


def create_cc_objects(front: dict, lower, cell_size):
    """createCCObjects (src/gpu_depthmap_fusion.cpp:2364-2550) without the OpenCV shapes, from the
    result of object_segmentation_front: per merged object (UIntGrouper order) the reference's
    float / int arithmetic - centroid += (double) x / num_components into a cv::Point2f (:2409),
    min / max voxel coords from the stats (:2397-2418), center = vec3(max + min) * 0.5f (:2421),
    voxelCoordToWorldCoord x * cs + lb in f32 (:1720-1730), aabb and num_layers (:2427-2430),
    and the contour points of the components (:2439-2460).  Returns (columns, components)."""
    f32 = np.float32
    merged = front["merged"].astype(np.int64)
    nl = front["num_labels"].astype(np.int64)
    layer = np.repeat(np.arange(len(nl)), nl)
    order = np.argsort(merged, kind="stable")
    n = int(front["num_objects"])
    sizes_by_layer, q = [], 0
    for z, c in enumerate(front["contours_per_layer"].astype(int)):
        sizes_by_layer.append(front["contour_sizes"][q:q + c])
        q += c
    lo = [f32(v) for v in lower]
    cs = [f32(v) for v in cell_size]

    def world(v):
        return [f32(f32(v[d]) * cs[d]) + lo[d] for d in range(3)]

    cols = {k: [] for k in ("label", "num_components", "num_layers", "first_component",
                            "centroid", "min_voxel", "max_voxel", "aabb_voxel", "center_voxel",
                            "center_world", "min_world", "max_world", "aabb_world",
                            "num_contour_points")}
    first = 0
    for i in range(n):
        idxs = order[first:first + int(np.count_nonzero(merged == i))]
        nc = len(idxs)
        cx = cy = f32(0.0)
        mn, mx, pts = [0, 0, 0], [0, 0, 0], 0
        for k, idx in enumerate(idxs):
            left, top, w, h, _ = (int(v) for v in front["stats"][idx])
            x, y = (float(v) for v in front["centroids"][idx])
            z = int(layer[idx])
            cx = f32(float(cx) + x / nc)
            cy = f32(float(cy) + y / nc)
            for d, lo_v, hi_v in ((0, left, left + w), (1, top, top + h), (2, z, z)):
                if k == 0 or lo_v < mn[d]:
                    mn[d] = lo_v
                if k == 0 or hi_v > mx[d]:
                    mx[d] = hi_v
            c = int(front["labels_to_contours"][idx])
            if c >= 0:
                pts += int(sizes_by_layer[z][c])
        center = [f32(f32(mx[d] + mn[d]) * f32(0.5)) for d in range(3)]
        mnw, mxw = world(mn), world(mx)
        cols["label"].append(i)
        cols["num_components"].append(nc)
        cols["num_layers"].append(1 + mx[2] - mn[2])
        cols["first_component"].append(first)
        cols["centroid"].append([cx, cy])
        cols["min_voxel"].append(mn)
        cols["max_voxel"].append(mx)
        cols["aabb_voxel"].append([mx[d] - mn[d] for d in range(3)])
        cols["center_voxel"].append(center)
        cols["center_world"].append(world(center))
        cols["min_world"].append(mnw)
        cols["max_world"].append(mxw)
        cols["aabb_world"].append([f32(mxw[d] - mnw[d]) for d in range(3)])
        cols["num_contour_points"].append(pts)
        first += nc
    dt = {"centroid": np.float32, "center_voxel": np.float32, "center_world": np.float32,
          "min_world": np.float32, "max_world": np.float32, "aabb_world": np.float32,
          "min_voxel": np.int32, "max_voxel": np.int32, "aabb_voxel": np.int32}
    out = {k: np.array(v, dtype=dt.get(k, np.uint32)) for k, v in cols.items()}
    return out, order.astype(np.uint32)
