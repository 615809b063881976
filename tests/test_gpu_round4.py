"""GPU tests added in round 4 (bar: bit-exact against the oracle, as test_gpu_parity.py).

* gdf_download_frame (the component's four per-frame downloads in one pass into pinned host
  mirrors) returns exactly what the per-call downloads return, and the oracle's outputs - the
  grid through its host mirror, updated from the changed 32-cell groups of each single-frame
  update once the mirror holds the previous grid (full copies after batches, skipped downloads,
  lifetime changes);
* the packed-f32 two-pixel flying filter (k_mask_px<2>, default) and the in-kernel group scans
  (segment counts in k_mask, group starts in k_group_count, default) against their switched-off
  forms and the oracle, on 8-frame VGA batches (9600 segments: the group-scan range) and a 4K
  frame (32 400 segments, the group phase over runs of a single frame).
"""
import os

import numpy as np
import pytest

from drive import compare_results
from oracle import OracleFusion
from ros_gpu_depthmap_fusion_amd import synth
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine(gpu_engine_factory):
    return gpu_engine_factory


def cam_args(cam, depth):
    return (depth, *cam.intrinsics(), cam.T_world, cam.T_crop)


def engine_with(Engine, **env):
    """An engine created with the given GDF_* environment knobs (read at creation)."""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update({k: v for k, v in env.items() if v is not None})
    for k, v in env.items():
        if v is None:
            os.environ.pop(k, None)
    try:
        return Engine()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def test_download_frame_equals_per_call_downloads(Engine):
    p = ComponentParams()
    cam = synth.make_camera(0, 640, 480)
    gpu, orc = Engine(), OracleFusion(threads=8)
    for f in range(3):
        for e in (gpu, orc):
            e.clear()
            e.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, f)))
            e.processFrame(p)
        d = gpu.download_frame()
        assert np.array_equal(d["points"].view(np.uint32), gpu.downloadPoints().view(np.uint32))
        assert np.array_equal(d["voxel_coords"], gpu.downloadVoxelCoords())
        assert np.array_equal(d["voxelized"].view(np.uint32),
                              gpu.downloadVoxelizedPoints().view(np.uint32))
        assert np.array_equal(d["occupancy"], gpu.downloadVoxelOccupancyGrid())
        assert np.array_equal(d["points"].view(np.uint32), orc.downloadPoints().view(np.uint32))
        assert np.array_equal(d["occupancy"], orc.downloadVoxelOccupancyGrid())
        w = orc.downloadVoxelizedPoints()[:, :3]
        assert np.array_equal(d["voxelized"][:, :3].view(np.uint32), w.view(np.uint32))
    only = gpu.download_frame(8)  # the grid alone
    assert set(only) == {"occupancy"}


def test_download_frame_grid_mirror_deltas(Engine):
    """The grid mirror across single frames (delta path), a skipped download, a 3-frame batch
    (full copy), a rollbuffer frame (k_grid_u8: delta), the stage-by-stage grid call and a
    lifetime above 255 (u32 history: full copies): every downloaded grid equals the oracle's."""
    p = ComponentParams()
    cam = synth.make_camera(0, 320, 240)
    lidar = synth.make_camera(1, 64, 48)
    pts = synth.back_project(lidar, synth.dense_frame(lidar, 1, 0))
    eye = np.eye(4, dtype=np.float32)
    gpu, orc = Engine(), OracleFusion(threads=8)
    f = 0

    def frame(download=True, seq=False):
        nonlocal f
        for e in (gpu, orc):
            if seq:
                e.addPointSequence(pts, *synth.sequence_time(f), synth.move_transform(f))
            e.clear()
            e.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, f)))
            if seq:
                e.processFrame(p, T_world_move=eye, T_crop_move=eye)
            else:
                e.processFrame(p)
        f += 1
        if download:
            g = gpu.download_frame(8)["occupancy"]
            assert np.array_equal(g, orc.downloadVoxelOccupancyGrid()), f"frame {f - 1}"

    for _ in range(5):
        frame()
    frame(download=False)
    frame()
    frame()
    # a batch of 3 frames (the batched update keeps no delta: the next download is a full copy)
    gpu.clear()
    for j in range(3):
        if j:
            gpu.nextFrameInBatch()
        gpu.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, f + j)))
    gpu.processFrame(p)
    for j in range(3):
        orc.clear()
        orc.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, f + j)))
        orc.processFrame(p)
    f += 3
    assert np.array_equal(gpu.download_frame(8)["occupancy"], orc.downloadVoxelOccupancyGrid())
    frame()
    frame(seq=True)  # rollbuffer frame: marks from the voxel groups, k_grid_u8 update
    frame(seq=True)
    frame()
    p.occupancy_lifetime = 300  # u32 history from here on
    frame()
    frame()


@pytest.mark.parametrize("knobs", [{}, {"GDF_NO_MASK_PACKED": "1"}, {"GDF_NO_GROUP_SCAN": "1"},
                                   {"GDF_NO_PACK_RUNS": "1"}, {"GDF_GROUP_FIRST": "0"},
                                   # sizes and alternative forms of the sort and group phases
                                   {"GDF_RUN_HIST_SORT": "1"}, {"GDF_RUN_HIST_ALL": "1"},
                                   {"GDF_SORT_BLOCKS": "1024"}, {"GDF_GROUP_BLOCKS": "1024"},
                                   {"GDF_GRID_WPT": "4"}, {"GDF_RUN_STAGE": "512"},
                                   {"GDF_SMALL_GROUP": "64"}, {"GDF_RUN_WAVE": "1"},
                                   {"GDF_RUN_WAVE": "0"}, {"GDF_RUN_Q16": "1"},
                                   {"GDF_RUN_BIG_BLOCKS": "512"},
                                   # the segment's camera by the lane ballot, not by division
                                   {"GDF_NO_SEG_UNIFORM": "1"},
                                   # (an engine created after all of them: the built-in values)
                                   {}])
def test_batch8_vga_knobs_match_oracle(Engine, knobs):
    """8-frame VGA batches (the C2 bench step) with the round-4 paths on and off: every frame's
    points, keys, voxel means and grid equal the oracle's frame-by-frame results."""
    p = ComponentParams()
    cam = synth.make_camera(0, 640, 480)
    gpu = engine_with(Engine, **knobs)
    orc = OracleFusion(threads=16)
    B = 8
    for b in range(2):
        frames = [synth.dense_frame(cam, 0, b * B + j) for j in range(B)]
        gpu.clear()
        for j in range(B):
            if j:
                gpu.nextFrameInBatch()
            gpu.addDepthmap(*cam_args(cam, frames[j]))
        gpu.processFrame(p)
        pts, keys, vox = gpu.downloadPoints(), gpu.downloadVoxelCoords(), gpu.downloadVoxelizedPoints()
        ps, vs = gpu.batch_ranges()
        for j in range(B):
            orc.clear()
            orc.addDepthmap(*cam_args(cam, frames[j]))
            orc.processFrame(p)
            assert np.array_equal(pts[ps[j]:ps[j + 1]].view(np.uint32),
                                  orc.downloadPoints().view(np.uint32)), (knobs, b, j)
            assert np.array_equal(keys[ps[j]:ps[j + 1]], orc.downloadVoxelCoords()), (knobs, b, j)
            w = orc.downloadVoxelizedPoints()[:, :3]
            assert np.array_equal(vox[vs[j]:vs[j + 1], :3].view(np.uint32), w.view(np.uint32)), (knobs, b, j)
            assert np.array_equal(gpu.downloadBatchVoxelOccupancyGrid(j),
                                  orc.downloadVoxelOccupancyGrid()), (knobs, b, j)


@pytest.mark.parametrize("knobs", [{}, {"GDF_NO_GROUP_SCAN": "1"}, {"GDF_NO_PACK_RUNS": "1"},
                                   {"GDF_RUN_WAVE_MODE": "2"}, {"GDF_GROUP_FIRST": "0"},
                                   # ~650 queued long groups on the small-frame batches' grid
                                   {"GDF_RUN_BIG_BLOCKS": "32"}])
def test_4k_frame_knobs_match_oracle(Engine, knobs):
    """A dense 4K frame (32 400 compaction segments, runs of equal keys): the group scans on and
    off, every output equal to the oracle's."""
    p = ComponentParams()
    cam = synth.make_camera(0, 3840, 2160)
    gpu = engine_with(Engine, **knobs)
    orc = OracleFusion(threads=16)
    for e in (gpu, orc):
        e.clear()
        e.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, 0)))
        e.processFrame(p)
    compare_results(gpu, orc, tag=f"4K {knobs}")


@pytest.mark.parametrize("nparts,B,emit", [(1, 1, False), (3, 1, False), (5, 3, False),
                                            (16, 8, False), (1, 8, True), (3, 8, True),
                                            (8, 8, True), (16, 4, True), (3, 1, True)])
def test_partition_runs_voxelize_runs_match_oracle(Engine, nparts, B, emit):
    """gdf_partition_runs (points + runs of equal frame|voxel keys, part-major) and
    gdf_voxelize_runs per part, in one process: every part voxelized on its own, the parts'
    voxels concatenated in part order, equal the oracle's voxel means of each frame bit for bit
    (the fused cloud's key ranges without the transport).  Also: sources split at arbitrary
    points of a part (several "ranks" sending one key range) rebase to the same result.  emit:
    the same send lists from gdf_set_emit_partition (the compaction writes them: k_mask_px +
    k_emit_px2 on the 256-pixel segments of frames over 1 Mi pixels; a single VGA frame takes the
    compaction + partition pass)."""
    from ros_gpu_depthmap_fusion_amd import hiprt, multi
    p = ComponentParams()
    cam = synth.make_camera(0, 640, 480)
    gpu, orc = Engine(), OracleFusion(threads=16)
    frames = [synth.dense_frame(cam, 0, 11 + j) for j in range(B)]
    gpu.clear()
    for j in range(B):
        if j:
            gpu.nextFrameInBatch()
        gpu.addDepthmap(*cam_args(cam, frames[j]))
    cap = 640 * 480 * B  # (the send buffers hold the frame's pixels before compaction)
    sp, srk, srs = hiprt.DeviceArray(16 * cap), hiprt.DeviceArray(4 * cap), hiprt.DeviceArray(4 * cap)
    cnt = hiprt.DeviceArray(8 * nparts)
    if emit:
        gpu.set_emit_partition(nparts, sp.ptr, srk.ptr, srs.ptr, cap, cnt.ptr)
    gpu.processFrame(p, synchronous=True, defer_occupancy_grid=True, defer_voxelize=True)
    if not emit:
        gpu.partition_runs(nparts, sp.ptr, srk.ptr, srs.ptr, cap, cnt.ptr)
    gpu.synchronize()
    c = cnt.to_numpy(np.uint32, 2 * nparts)
    pts, runs = c[:nparts].astype(np.int64), c[nparts:].astype(np.int64)
    n = int(pts.sum())
    assert (runs <= pts).all() and ((runs > 0) == (pts > 0)).all()
    P0, R0 = np.concatenate([[0], np.cumsum(pts)]), np.concatenate([[0], np.cumsum(runs)])
    h_rs = srs.to_numpy(np.uint32, max(n, 1))
    # every part's voxel marks (gdf_voxelize_runs_marked): frame j at j * stride words; part q's
    # keys are whole mark words [q S, (q + 1) S) (the fused step all-gathers those slices)
    ncells = int(gpu.grid_size()[1])
    words = (ncells + 31) // 32
    S = multi.part_slice_words(nparts, ncells)
    stride = S * nparts
    union = np.zeros((B, stride), np.uint32)
    want, want_marks = [], np.zeros((B, words), np.uint32)
    for j in range(B):
        orc.clear()
        orc.addDepthmap(*cam_args(cam, frames[j]))
        orc.processFrame(p)
        want.append(orc.downloadVoxelizedPoints()[:, :3])
        k = np.unique(orc.downloadVoxelCoords().astype(np.int64))
        np.bitwise_or.at(want_marks[j], k >> 5, (np.uint32(1) << (k & 31).astype(np.uint32)))
    got = [[] for _ in range(B)]
    for q in range(nparts):
        if pts[q] == 0:
            continue
        rs = h_rs[R0[q]:R0[q + 1]]
        assert rs[0] == 0 and (np.diff(rs.astype(np.int64)) > 0).all() and rs[-1] < pts[q]
        # the part as two sources split at a run boundary (a key range from two ranks)
        cut = len(rs) // 2
        pb = np.array([0, rs[cut], pts[q]] if cut else [0, pts[q]], np.uint32)
        rb = np.array([0, cut, len(rs)] if cut else [0, len(rs)], np.uint32)
        local = rs.astype(np.uint32).copy()
        if cut:
            local[cut:] -= rs[cut]
        drs = hiprt.DeviceArray.from_numpy(np.concatenate([local, np.zeros(1, np.uint32)]))
        dmk = hiprt.DeviceArray.from_numpy(np.zeros(B * stride, np.uint32))
        gpu.voxelize_runs_marked(sp.ptr + 16 * int(P0[q]), srk.ptr + 4 * int(R0[q]), drs.ptr, pb, rb,
                                 dmk.ptr, stride)
        gpu.synchronize()
        mk = dmk.to_numpy(np.uint32, B * stride).reshape(B, stride)
        outside = np.ones(stride, bool)
        outside[q * S:(q + 1) * S] = False
        assert not mk[:, outside].any(), (nparts, B, q)
        union |= mk
        vox = gpu.downloadVoxelizedPoints()[:, :3]
        if B > 1:
            _, vs = gpu.batch_ranges()
            for j in range(B):
                got[j].append(vox[vs[j]:vs[j + 1]])
        else:
            got[0].append(vox)
    for j in range(B):
        g = np.concatenate(got[j]) if got[j] else np.zeros((0, 3), np.float32)
        assert len(g) == len(want[j]) > 0, (nparts, B, j)
        assert np.array_equal(g.view(np.uint32), want[j].view(np.uint32)), (nparts, B, j)
        assert np.array_equal(union[j, :words], want_marks[j]), (nparts, B, j)
        assert not union[j, words:].any()


def test_tuning_is_a_snapshot_per_engine(Engine):
    """Each engine keeps the tuning taken at its creation (gdf_get_tuning): an engine created
    under GDF_RUN_STAGE=512 / GDF_RUN_WAVE=1 reports them, one created afterwards without them
    reports the built-in defaults, and the first one - still running its own shapes after the
    second was created - stays bit-exact against the oracle on an 8-frame VGA batch."""
    a = engine_with(Engine, GDF_RUN_STAGE="512", GDF_RUN_WAVE="1")
    b = engine_with(Engine, GDF_RUN_STAGE=None, GDF_RUN_WAVE=None)
    assert {"GDF_RUN_STAGE=512", "GDF_RUN_WAVE=1"} <= set(a.tuning().split()), a.tuning()
    assert all(not t.startswith(("GDF_RUN_STAGE", "GDF_RUN_WAVE=")) for t in b.tuning().split())
    p = ComponentParams()
    cam = synth.make_camera(0, 640, 480)
    frames = [synth.dense_frame(cam, 0, j) for j in range(8)]
    orc = OracleFusion(threads=16)
    for gpu in (a, b):
        gpu.clear()
        for j, f in enumerate(frames):
            if j:
                gpu.nextFrameInBatch()
            gpu.addDepthmap(*cam_args(cam, f))
        gpu.processFrame(p)
    vox_a, vox_b = a.downloadVoxelizedPoints(), b.downloadVoxelizedPoints()
    assert np.array_equal(vox_a[:, :3].view(np.uint32), vox_b[:, :3].view(np.uint32))
    _, vs = a.batch_ranges()
    orc.clear()
    orc.addDepthmap(*cam_args(cam, frames[7]))
    orc.processFrame(p)
    w = orc.downloadVoxelizedPoints()[:, :3]
    assert np.array_equal(vox_a[vs[7]:vs[8], :3].view(np.uint32), w.view(np.uint32))
