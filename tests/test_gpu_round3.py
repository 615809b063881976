"""GPU parity tests added in round 3.

* C3 against the oracle at scale: rollbuffer windows of 64 and 256 (= C3) x 720p sequences
  (59 M and 236 M selected points per frame, voxels of > 50 K points streamed by
  k_group_runs_big) - points, keys, voxel means, grid, history and rollbuffer state bit for bit (VERDICT r2 "next" 1; the reference methods are
  fusion.cpp:1509-1581 for the selection / transform and voxelize.h:9-48 for the means).

Bar as in test_gpu_parity.py: bit-exact.
"""
import os

import numpy as np
import pytest

from drive import compare_results
from oracle import OracleFusion
from ros_gpu_depthmap_fusion_amd import hiprt, synth
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine(gpu_engine_factory):
    return gpu_engine_factory


def cam_args(cam, depth):
    return (depth, *cam.intrinsics(), cam.T_world, cam.T_crop)


@pytest.mark.parametrize("nwin", [64, 256])
def test_c3_window_oracle_parity_720p(Engine, nwin):
    """C3 shape (nwin = 256 is C3 itself): 720p depth + nwin point sequences of 921 600 points
    (a 720p lidar frame back-projected; T_move(k) = 0.01 k m along x, so one surface patch lands
    in the same voxel in every sequence and voxels reach ~10^5 points at 64 sequences, ~4 x 10^5 at
    256).  Frame 1 ingests nwin - 2 sequences at once (one filter pass over all new points, as
    the reference's uploadPointSequences does), frames 2 and 3 one each (the window is full),
    frame 4 one more, so its roll discards the oldest.  Every output of the last two frames is
    compared with the oracle bit for bit."""
    p = ComponentParams()
    W, H = 1280, 720
    n = W * H
    p.ps_timespan = (nwin - 0.5) / 30.0
    lidar = synth.make_camera(1, W, H)
    cam = synth.make_camera(0, W, H)
    host = [np.concatenate([synth.back_project(lidar, synth.dense_frame(lidar, 1, f)),
                            np.ones((n, 1), np.float32)], 1) for f in range(2)]
    dev = [hiprt.DeviceArray.from_numpy(h) for h in host]
    depth = [synth.dense_frame(cam, 0, f) for f in range(2)]
    gpu, orc = Engine(), OracleFusion(threads=16)
    batches = [nwin - 2, 1, 1, 1]  # sequences ingested per frame (the last frame rolls one out)
    k = 0
    for fi, nb in enumerate(batches):
        for _ in range(nb):
            s, ns = synth.sequence_time(k)
            T = synth.move_transform(k)
            gpu.addPointSequenceDevice(dev[k % 2].ptr, n, 16, s, ns, T)
            orc.addPointSequence(host[k % 2], s, ns, T)
            k += 1
        for e in (gpu, orc):
            e.clear()
            e.addDepthmap(*cam_args(cam, depth[fi % 2]))
            e.processFrame(p, T_world_move=lidar.T_world, T_crop_move=lidar.T_crop)
        if fi < len(batches) - 2:
            continue
        st = gpu.rollbuffer_state()
        assert st.as_tuple() == orc.rollbuffer_state(), f"frame {fi} rollbuffer state"
        assert st.selection_sequence_count == nwin
        assert st.selection_point_count == nwin * n
        keys = gpu.downloadVoxelCoords()
        longest = int(np.bincount(keys).max())
        assert len(keys) > 25_000_000 and longest > 50_000, (len(keys), longest)
        compare_results(gpu, orc, tag=f"C3 window {nwin} frame {fi}")


def _nan_equal_bits(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    both_nan = np.isnan(a) & np.isnan(b)
    return (a.view(np.uint32) == b.view(np.uint32)) | both_nan


@pytest.mark.parametrize("xruns", [False, True])
def test_voxel_sums_adversarial_points_mode(Engine, xruns):
    """gdf_voxelize_points (points mode - GDF_NO_XRUNS: k_group in-thread / staged / gathered wave
    sums and, with > 1 K tiles, k_group_big; or, by default, the received list's runs of equal
    keys through k_group_runs / k_group_runs_big) on voxels built from the adversarial term lists
    of tests/test_spec_sum_model.py - ties at every binade, sums through zero, exact cancellation,
    subnormals, overflow to inf, inf and NaN terms, 70 K ones - interleaved with 400 K ordinary
    points: every voxel mean equals the reference's sequential f32 chain (inc/voxelize.h:29-35),
    bit for bit (NaN: any NaN)."""
    import os
    from test_spec_sum_model import cases
    from spec_sum_model import sequential_sum
    if not xruns:
        os.environ["GDF_NO_XRUNS"] = "1"
    try:
        gpu = Engine()
    finally:
        os.environ.pop("GDF_NO_XRUNS", None)
    p = ComponentParams()
    cam = synth.make_camera(0, 64, 48)
    gpu.clear()
    gpu.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, 0)))
    gpu.processFrame(p)
    _, ncells = gpu.grid_size()
    rng = np.random.default_rng(99)
    cs = cases()
    names = sorted(cs)
    groups = []  # (key, (n, 4) float32 terms in order)
    for i, nm in enumerate(names):
        n = len(cs[nm])
        comps = [cs[names[(i + j) % len(names)]] for j in range(4)]
        t = np.stack([np.resize(c, n) for c in comps], 1).astype(np.float32)
        groups.append((1000 + 7919 * i, t))
    for j in range(3000):  # ordinary voxels, 1..400 points
        n = int(rng.integers(1, 400))
        groups.append((200_000 + 613 * j, rng.normal(0, 1, (n, 4)).astype(np.float32)))
    # interleave the groups' points (each group keeps its own order: the stable sort restores it);
    # runs mode: blocks of consecutive points of one group (runs of 1..64 points)
    owner = np.concatenate([np.full(len(t), g) for g, (_, t) in enumerate(groups)])
    rng.shuffle(owner)
    if xruns:
        owner = np.sort(owner)
        cut = np.cumsum(rng.integers(1, 65, len(owner)))
        cut = cut[cut < len(owner)]
        blocks = np.split(owner, cut)
        rng.shuffle(blocks)
        owner = np.concatenate(blocks)
    pos = np.zeros(len(groups), np.int64)
    pts = np.empty((len(owner), 4), np.float32)
    keys = np.empty(len(owner), np.uint32)
    for idx, g in enumerate(owner):
        pts[idx] = groups[g][1][pos[g]]
        keys[idx] = groups[g][0]
        pos[g] += 1
    assert keys.max() < ncells
    dp, dk = hiprt.DeviceArray.from_numpy(pts), hiprt.DeviceArray.from_numpy(keys)
    gpu.voxelize_points(dp.ptr, dk.ptr, len(keys))
    got = gpu.downloadVoxelizedPoints()
    order = sorted(range(len(groups)), key=lambda g: groups[g][0])
    assert len(got) == len(groups)
    for out_i, g in enumerate(order):
        t = groups[g][1]
        want = [sequential_sum(t[:, c]) for c in range(4)]
        want = np.array([want[0] / np.float32(len(t)), want[1] / np.float32(len(t)),
                         want[2] / np.float32(len(t)), want[3]], np.float32)
        ok = _nan_equal_bits(got[out_i], want)
        assert ok.all(), (g, len(t), got[out_i], want)


@pytest.mark.parametrize("wave_mode", [None, "2"])
def test_voxel_sums_adversarial_run_mode(Engine, wave_mode):
    """The rollbuffer path (run mode: k_sel runs -> run sort -> k_group_runs staged sums and
    k_group_runs_big streams) on point sequences whose voxels hold adversarial values: z on a
    2^-12 grid around 0 (random walks through zero, exact cancellation), subnormal x, ties from
    one-binade-below terms, long runs of one voxel (> 100 K points) - identity move transforms,
    bit-exact vs the oracle (points, keys, means, grid).  GDF_RUN_WAVE_MODE=2: every queued
    group below the huge region summed by one wave (wave_stream_sum) however short the queue."""
    if wave_mode is not None:
        os.environ["GDF_RUN_WAVE_MODE"] = wave_mode
    try:
        _adversarial_run_mode(Engine)
    finally:
        os.environ.pop("GDF_RUN_WAVE_MODE", None)
        Engine().close()  # (the knob is process-wide: an engine created without it resets it)


def _adversarial_run_mode(Engine):
    p = ComponentParams()
    p.ps_timespan = 2.5 / 30.0
    p.ps_filter_size = 0  # keep every point (the filter's own parity is tested elsewhere)
    rng = np.random.default_rng(5)
    n = 600_000
    vox = rng.integers(0, 40, n // 2000).repeat(2000)  # long runs of one of 40 voxels
    vx = (vox % 8).astype(np.float32)
    vy = (vox // 8).astype(np.float32)
    x = (0.1 * vx + rng.uniform(0.005, 0.095, n)).astype(np.float32)
    x[vox % 5 == 0] = rng.uniform(0, 1e-39, np.count_nonzero(vox % 5 == 0)).astype(np.float32)
    y = (0.1 * vy + 0.0625 + (rng.uniform(0, 0.0375, n))).astype(np.float32)
    y = np.where(vox % 3 == 0, (y.view(np.uint32) | 1).view(np.float32), y)
    z = (rng.integers(-160, 320, n) * 2.0 ** -12).astype(np.float32)
    recs = [np.stack([x, y, z, np.ones(n, np.float32)], 1)]
    recs.append(recs[0][::-1].copy())
    gpu, orc = Engine(), OracleFusion(threads=16)
    eye = np.eye(4, dtype=np.float32)
    dev = [hiprt.DeviceArray.from_numpy(r) for r in recs]
    for k in range(3):
        s, ns = synth.sequence_time(k)
        gpu.addPointSequenceDevice(dev[k % 2].ptr, n, 16, s, ns, eye)
        orc.addPointSequence(recs[k % 2], s, ns, eye)
        for e in (gpu, orc):
            e.clear()
            e.processFrame(p, T_world_move=eye, T_crop_move=eye)
    keys = gpu.downloadVoxelCoords()
    assert len(keys) > 1_000_000 and int(np.bincount(keys).max()) > 100_000
    compare_results(gpu, orc, tag="adversarial run mode")


@pytest.mark.parametrize("lifetime", [10, 300])
def test_deferred_batch_grid_downloads(Engine, lifetime):
    """A batch whose grid update is deferred (the multi-GPU batch path: defer_occupancy_grid +
    defer_voxelize, marks taken, gdf_voxel_occupancy_grid_batch) keeps every frame's grid as the
    fused path does (sparse snapshots written by the batched update): the download of frame f
    equals the oracle's grid after processing the frames one by one (fusion.cpp:1757-1839).
    lifetime 300 (u32 history, frame by frame) keeps no per-frame grids: the download of an
    intermediate frame fails loudly, the last frame's is the grid itself."""
    from ros_gpu_depthmap_fusion_amd import multi
    from ros_gpu_depthmap_fusion_amd.gdf import GDFError
    p = ComponentParams()
    p.occupancy_lifetime = lifetime
    cam = synth.make_camera(0, 320, 240)
    B = 4
    depth = [synth.dense_frame(cam, 0, f) for f in range(2 * B)]
    gpu, orc = Engine(), OracleFusion(threads=8)
    for b in range(2):  # two batches: the second starts from the first's grid
        gpu.clear()
        for j in range(B):
            if j:
                gpu.nextFrameInBatch()
            gpu.addDepthmap(*cam_args(cam, depth[b * B + j]))
        gpu.processFrame(p, synchronous=False, defer_occupancy_grid=True, defer_voxelize=True)
        _, ncells = gpu.grid_size()
        words = multi.words_for(ncells)
        local = hiprt.DeviceArray(B * words * 4)
        gpu.take_marks(local.ptr, B * words)
        gpu.voxelOccupancyGridBatch(local.ptr, words, 1, B, words, B * words, lifetime)
        want = []
        for j in range(B):
            orc.clear()
            orc.addDepthmap(*cam_args(cam, depth[b * B + j]))
            orc.processFrame(p)
            want.append(orc.downloadVoxelOccupancyGrid().reshape(-1).copy())
        for j in range(B):
            if lifetime > 255 and j + 1 < B:
                with pytest.raises(GDFError):
                    gpu.downloadBatchVoxelOccupancyGrid(j)
                continue
            got = gpu.downloadBatchVoxelOccupancyGrid(j)
            assert np.array_equal(got, want[j]), f"batch {b} frame {j}"
