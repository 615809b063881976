"""GPU parity tests added in round 2: the realistic-density workload at VGA / 720p / 4K, host
depth maps through the pinned / overlapped H2D path, the batched grid update and the sparse
union of a partial batch, the full C3 window (256 x 720p sequences) and a window large enough to
reach the multi-segment k_sel tiles and k_group_big against the oracle.

Bar as in test_gpu_parity.py: bit-exact points, keys, voxel means, grids, history.
"""
import numpy as np
import pytest

from drive import bits, compare_results
from oracle import OracleFusion
from ros_gpu_depthmap_fusion_amd import hiprt, multi, synth
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams

pytestmark = pytest.mark.gpu

EYE = np.eye(4, dtype=np.float32)


@pytest.fixture(scope="module")
def Engine(gpu_engine_factory):
    return gpu_engine_factory


def cam_args(cam, depth):
    return (depth, *cam.intrinsics(), cam.T_world, cam.T_crop)


def run_fused(eng, cams_frames, params, **kw):
    eng.clear()
    for c in cams_frames:
        eng.addDepthmap(*c)
    return eng.processFrame(params, **kw)


@pytest.mark.parametrize("W,H,frames", [(640, 480, 3), (1280, 720, 2)])
def test_dense_workload_parity(Engine, W, H, frames):
    """C2 (and 720p) at the realistic density of the benchmark (synth.dense_frame, ~65 % of the
    pixels survive the flying-pixel filter): everything bit-exact, frame after frame."""
    p = ComponentParams()
    gpu, orc = Engine(), OracleFusion(threads=8)
    cam = synth.make_camera(0, W, H)
    for f in range(frames):
        args = [cam_args(cam, synth.dense_frame(cam, 0, f))]
        r = run_fused(gpu, args, p)
        run_fused(orc, args, p)
        assert r.num_points == orc.point_count() > 0.3 * W * H
        compare_results(gpu, orc, tag=f"{W}x{H} frame {f}")


def test_dense_4k_frame_parity(Engine):
    """A full 3840x2160 dense frame (3 M points after crop; 256-px compaction segments, 8-key
    radix tiles, k_group over ~12 K tiles): bit-exact vs the oracle."""
    p = ComponentParams()
    gpu, orc = Engine(), OracleFusion(threads=16)
    cam = synth.make_camera(0, 3840, 2160)
    args = [cam_args(cam, synth.dense_frame(cam, 0, 0))]
    r = run_fused(gpu, args, p)
    run_fused(orc, args, p)
    assert r.num_points == orc.point_count() > 2_000_000
    compare_results(gpu, orc, tag="4k dense")


@pytest.mark.parametrize("pinned,W,H", [(True, 320, 240), (False, 320, 240), (False, 1280, 720)])
def test_host_stream_overlapped_h2d(Engine, pinned, W, H):
    """Host depth maps through gdf_run_host_stream with 3 frames in flight: every host map (pinned
    or pageable) is copied into the slot's pinned staging - 720p maps (1.8 MB) in 256 KB chunks by
    the staging threads - and sent on the slot's stream; the grid after all frames and the last
    frame's outputs equal the oracle's.  The pageable source is overwritten after the call
    returns (the staging copy was taken: borrowed-until-upload)."""
    p = ComponentParams()
    cam = synth.make_camera(0, W, H)
    ring = [synth.dense_frame(cam, 0, f) for f in range(4)]
    if pinned:
        host = [hiprt.PinnedArray.from_numpy(f) for f in ring]
        ptrs = [h.ptr for h in host]
    else:
        host = [f.copy() for f in ring]
        ptrs = [h.ctypes.data for h in host]
    gpu, orc = Engine(), OracleFusion(threads=8)
    gpu.set_pipeline_depth(3)
    sc = gpu.make_stream_camera(ptrs, W, H, *cam.intrinsics(), cam.T_world, cam.T_crop)
    n = 11
    gpu.run_host_stream([sc], p.to_c(None, None, False, False), 0, n)
    if not pinned:
        for h in host:
            h[...] = 0  # the engine holds its own copies by now
    gpu.synchronize()
    for i in range(n):
        run_fused(orc, [cam_args(cam, ring[i % 4])], p)
    compare_results(gpu, orc, tag="host stream")


@pytest.mark.parametrize("lifetime", [10, 300])
def test_grid_batch_update_partial_batch(Engine, lifetime):
    """gdf_voxel_occupancy_grid_batch on an all-gathered [rank, batch, words] buffer of a PARTIAL
    batch (3 live frames of 4, the 4th holding stale garbage): lifetime 10 = the one-pass u8
    kernel, 300 = the u32 frame-by-frame branch; the grid equals the host history of the
    per-frame unions."""
    p = ComponentParams()
    p.occupancy_lifetime = lifetime
    gpu = Engine()
    cam = synth.make_camera(0, 160, 120)
    run_fused(gpu, [cam_args(cam, synth.dense_frame(cam, 0, 0))], p, defer_occupancy_grid=True)
    _, ncells = gpu.grid_size()
    nw = multi.words_for(ncells)
    # the frame's own marks are taken first (pending marks are refused)
    sink = hiprt.DeviceArray(nw * 4)
    gpu.take_marks(sink.ptr, nw)
    gpu.synchronize()
    rng = np.random.default_rng(lifetime)
    world, batch, live = 2, 4, 3
    masks = np.zeros((world, batch, nw), np.uint32)
    for r in range(world):
        for f in range(batch):
            m = rng.random(ncells) < (0.003 if f < live else 0.5)  # frame 3: stale, dense
            masks[r, f] = multi.pack_marks(m)
    dev = hiprt.DeviceArray.from_numpy(masks.reshape(-1))
    gpu.voxelOccupancyGridBatch(dev.ptr, nw, world, live, nw, batch * nw, lifetime)
    hist = np.zeros(ncells, np.uint32)
    for f in range(live):
        u = multi.unpack_marks(masks[0, f] | masks[1, f], ncells)
        hist = multi.historic_update(hist, u, lifetime)
    np.testing.assert_array_equal(gpu.downloadVoxelOccupancyGrid(), (hist & 0xFF).astype(np.uint8))
    np.testing.assert_array_equal(gpu.historic_grid(), hist)


def test_union_pairs_partial_batch_skips_stale_records(Engine):
    """A partial sparse batch (n = 2 live frames of batch 4): the stale records 2..3 carry counts
    far above the cap (a previous, dense batch); union_pairs with frames_per_rank = 4 visits only
    the live records and reads each record up to its own cap."""
    gpu = Engine()
    p = ComponentParams()
    cam = synth.make_camera(0, 64, 48)
    run_fused(gpu, [cam_args(cam, synth.dense_frame(cam, 0, 0))], p)
    _, ncells = gpu.grid_size()
    nw = multi.words_for(ncells)
    cap, batch, live, world = 64, 4, 2, 2
    rec = 1 + 2 * cap
    buf = np.zeros((world, batch, rec), np.uint32)
    want = np.zeros((live, nw), np.uint32)
    rng = np.random.default_rng(7)
    for r in range(world):
        for f in range(batch):
            if f < live:
                k = int(rng.integers(1, cap))
                idx = rng.choice(nw, k, replace=False).astype(np.uint32)
                val = rng.integers(1, 2**32, k, dtype=np.uint64).astype(np.uint32)
                buf[r, f, 0] = k
                buf[r, f, 1:1 + 2 * k:2] = idx
                buf[r, f, 2:2 + 2 * k:2] = val
                np.bitwise_or.at(want[f], idx, val)
            else:
                buf[r, f, 0] = 10_000_000  # stale over-cap count
                buf[r, f, 1:] = 0xFFFFFFFF
    dev = hiprt.DeviceArray.from_numpy(buf.reshape(-1))
    uni = hiprt.DeviceArray(batch * nw * 4)
    gpu.union_pairs(uni.ptr, nw, dev.ptr, world, live, rec, frames_per_rank=batch)
    gpu.synchronize()
    np.testing.assert_array_equal(uni.to_numpy(np.uint32, live * nw).reshape(live, nw), want)


def _window_frames(gpu, orc, lidar, cam, p, nseq, npf, seqs_host, seqs_dev, depth, sync_last):
    for k in range(nseq):
        s, ns = synth.sequence_time(k)
        T = synth.move_transform(k)
        if gpu is not None:
            gpu.addPointSequenceDevice(seqs_dev[k % len(seqs_dev)].ptr, npf, 16, s, ns, T)
        if orc is not None:
            orc.addPointSequence(seqs_host[k % len(seqs_host)], s, ns, T)
        for e in (gpu, orc):
            if e is None:
                continue
            e.clear()
            e.addDepthmap(*cam_args(cam, depth[k % len(depth)]))
            if e is gpu:
                r = e.processFrame(p, T_world_move=lidar.T_world, T_crop_move=lidar.T_crop,
                                   synchronous=sync_last and k == nseq - 1)
            else:
                e.processFrame(p, T_world_move=lidar.T_world, T_crop_move=lidar.T_crop)
    return r


def test_rollbuffer_window_oracle_parity_large(Engine):
    """Rollbuffer window of 28 sequences x 320x240 (dense) + a 320x240 depth map: 2.2 M selected
    points per frame - k_sel's multi-segment tiles (8 x 512 points), tiles straddling two
    sequences, > 8192 group tiles of capacity (group-id offsets by count + scan) and voxels
    longer than the 512 staged points (k_group_big) - bit-exact vs the oracle on the last
    frames."""
    p = ComponentParams()
    p.ps_timespan = 27.5 / 30.0
    lidar = synth.make_camera(1, 320, 240)
    cam = synth.make_camera(0, 320, 240)
    npf = 320 * 240
    host = [np.concatenate([synth.back_project(lidar, synth.dense_frame(lidar, 1, f)),
                            np.ones((npf, 1), np.float32)], 1) for f in range(3)]
    dev = [hiprt.DeviceArray.from_numpy(h) for h in host]
    depth = [synth.dense_frame(cam, 0, f) for f in range(3)]
    gpu, orc = Engine(), OracleFusion(threads=16)
    r = _window_frames(gpu, orc, lidar, cam, p, 31, npf, host, dev, depth, True)
    st = gpu.rollbuffer_state()
    assert st.selection_sequence_count == 28 and st.as_tuple() == orc.rollbuffer_state()
    assert r.num_points_total == 29 * npf and r.num_points > 600_000
    compare_results(gpu, orc, tag="window")


def test_c3_full_window_properties(Engine):
    """C3 at full size: 720p depth + a window of 256 sequences of 921 600 points (236 M selected
    points per frame, 3.8 GB ring): the selection, one voxel mean per distinct key, the grid holds
    exactly the frame's voxels at full lifetime, and the points are the oracle's for the depth
    part (the first N_depth points; rollbuffer survivors follow in selection order)."""
    p = ComponentParams()
    W, H = 1280, 720
    n = W * H
    p.ps_timespan = 255.5 / 30.0
    lidar = synth.make_camera(1, W, H)
    cam = synth.make_camera(0, W, H)
    seqs = [hiprt.DeviceArray.from_numpy(np.concatenate(
        [synth.back_project(lidar, synth.dense_frame(lidar, 1, f)),
         np.ones((n, 1), np.float32)], 1)) for f in range(2)]
    depth = [synth.dense_frame(cam, 0, f) for f in range(2)]
    gpu = Engine()
    r = _window_frames(gpu, None, lidar, cam, p, 260, n, None, seqs, depth, True)
    st = gpu.rollbuffer_state()
    assert st.selection_sequence_count == 256 and st.selection_point_count == 256 * n
    assert r.num_points_total == 257 * n
    c = gpu.downloadVoxelCoords()
    assert len(c) == r.num_points > 10_000_000
    u = np.unique(c)
    assert len(gpu.downloadVoxelizedPoints()) == len(u)
    grid = gpu.downloadVoxelOccupancyGrid().reshape(-1)
    assert np.array_equal(np.flatnonzero(grid == p.occupancy_lifetime), u)
    orc = OracleFusion(threads=8)
    orc.clear()
    orc.addDepthmap(*cam_args(cam, depth[259 % 2]))
    orc.processFrame(p)
    nd = orc.point_count()
    pts = gpu.downloadPoints()
    assert np.array_equal(bits(pts[:nd]), bits(orc.downloadPoints()))


def _batch(gpu, frames_args, p, **kw):
    gpu.clear()
    for j, args in enumerate(frames_args):
        if j:
            gpu.nextFrameInBatch()
        for a in args:
            gpu.addDepthmap(*a)
    return gpu.processFrame(p, **kw)


@pytest.mark.parametrize("case", ["vga_b4", "two_cams_b3_codedefaults", "corners_b2_depth3",
                                  "vga_b8_runs", "small_b8_points"])
def test_batched_frames_equal_frame_by_frame(Engine, case):
    """Multi-frame batches (gdf_next_frame_in_batch): every frame's points, keys, voxel means and
    the grid after every frame equal the oracle processing the frames one by one - incl. two
    cameras per frame (cross-camera reads stay inside the frame), code defaults (F=1, rot45,
    lifetime 1), voxel corners, and batches pipelined over 3 slots.  Batches of 8 frames at the
    launch-default grid sort 25-bit keys (22 voxel bits + 3 frame bits) in 3 radix passes with a
    9-bit last digit: over runs of equal keys (VGA, 2.4 Mi pixels per batch) and over points."""
    if case == "vga_b4":
        p, W, H, ncam, B, nb, depth = ComponentParams(), 640, 480, 1, 4, 3, 1
    elif case == "vga_b8_runs":
        p, W, H, ncam, B, nb, depth = ComponentParams(), 640, 480, 1, 8, 2, 2
    elif case == "small_b8_points":
        p, W, H, ncam, B, nb, depth = ComponentParams(), 160, 120, 1, 8, 2, 1
    elif case == "two_cams_b3_codedefaults":
        p = ComponentParams.code_defaults()
        p.crop_min, p.crop_max = (-3, -3, -1), (6, 3, 2.5)
        p.voxel_min, p.voxel_max = (-3, -3, -1), (6, 3, 2.5)
        W, H, ncam, B, nb, depth = 200, 150, 2, 3, 3, 1
    else:
        p = ComponentParams()
        p.voxel_average = False
        W, H, ncam, B, nb, depth = 160, 120, 1, 2, 5, 3
    cams = [synth.make_camera(k, W, H) for k in range(ncam)]
    gpu, orc = Engine(), OracleFusion(threads=8)
    gpu.set_pipeline_depth(depth)
    f = 0
    for b in range(nb):
        frames = [[cam_args(c, synth.dense_frame(c, k, f + j)) for k, c in enumerate(cams)]
                  for j in range(B)]
        r = _batch(gpu, frames, p)
        pts, keys, vox = gpu.downloadPoints(), gpu.downloadVoxelCoords(), gpu.downloadVoxelizedPoints()
        ps, vs = gpu.batch_ranges()
        assert len(ps) == B + 1 and ps[-1] == len(pts) == r.num_points and vs[-1] == len(vox)
        for j in range(B):
            run_fused(orc, frames[j], p)
            tag = f"batch {b} frame {j}"
            po = orc.downloadPoints()
            assert ps[j + 1] - ps[j] == len(po), tag
            assert np.array_equal(bits(pts[ps[j]:ps[j + 1]]), bits(po)), tag
            np.testing.assert_array_equal(keys[ps[j]:ps[j + 1]], orc.downloadVoxelCoords(), tag)
            vo = orc.downloadVoxelizedPoints()
            assert vs[j + 1] - vs[j] == len(vo), tag
            assert np.array_equal(bits(vox[vs[j]:vs[j + 1], :3]), bits(vo[:, :3])), tag
            np.testing.assert_array_equal(gpu.downloadBatchVoxelOccupancyGrid(j),
                                          orc.downloadVoxelOccupancyGrid(), tag)
        np.testing.assert_array_equal(gpu.historic_grid(), orc.historic_grid())
        f += B


def test_batch_errors_fail_loudly(Engine):
    """A batch frame without a depth map, point sequences in a batch, lifetime > 255."""
    from ros_gpu_depthmap_fusion_amd.gdf import GDFError
    p = ComponentParams()
    cam = synth.make_camera(0, 64, 48)
    gpu = Engine()
    gpu.clear()
    with pytest.raises(GDFError):
        gpu.nextFrameInBatch()  # frame 0 has no depth map yet
    gpu.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, 0)))
    gpu.nextFrameInBatch()
    with pytest.raises(GDFError):
        gpu.processFrame(p)  # frame 1 has no depth map
    gpu.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, 1)))
    q = ComponentParams()
    q.occupancy_lifetime = 300
    with pytest.raises(GDFError):
        gpu.processFrame(q)
    gpu.addPointSequence(synth.back_project(cam, synth.dense_frame(cam, 0, 2)), 1000, 0, EYE)
    with pytest.raises(GDFError):
        gpu.processFrame(p)


@pytest.mark.parametrize("W,H", [(1, 1), (37, 23), (640, 480), (1280, 720)])
def test_mask_dilate_matches_oracle(Engine, W, H):
    """gdf_mask_dilate (LDS-staged separable window AND) vs the oracle's literal restatement of
    mask_dilate.glsl:40-67, intended erosion and as written, F = 0..16."""
    from oracle import mask_dilate
    rng = np.random.default_rng(W * H)
    m = ((rng.random((H, W)) < 0.995) * rng.integers(1, 2**32, (H, W), dtype=np.uint64))
    m = m.astype(np.uint32)
    gpu = Engine()
    din = hiprt.DeviceArray.from_numpy(m)
    dout = hiprt.DeviceArray(m.nbytes)
    for F in (0, 1, 4, 16):
        for aw in (False, True):
            hiprt.check(hiprt.hip().hipMemset(dout.ptr, 0xAB, m.nbytes))
            hiprt.synchronize()  # (the engine's stream does not wait for the null stream)
            gpu.maskDilate(din.ptr, dout.ptr, W, H, F, aw)
            gpu.synchronize()
            got = dout.to_numpy(np.uint32, W * H).reshape(H, W)
            np.testing.assert_array_equal(got, mask_dilate(m, F, aw), f"F={F} as_written={aw}")


def test_transform_points_matches_oracle(Engine):
    """gdf_transform_points vs transform_points.glsl restated: bit-exact where mask != 0,
    untouched elsewhere."""
    from oracle import transform_points
    rng = np.random.default_rng(5)
    n = 300_001
    pts = (rng.standard_normal((n, 4)) * 7).astype(np.float32)
    mask = (rng.random(n) < 0.6).astype(np.uint32) * rng.integers(1, 9, n).astype(np.uint32)
    T = synth.make_camera(3, 64, 48).T_world
    init = np.full((n, 4), np.float32(-1.25))
    gpu = Engine()
    dp, dm, do = (hiprt.DeviceArray.from_numpy(a) for a in (pts, mask, init))
    gpu.transformPoints(dp.ptr, dm.ptr, do.ptr, n, T)
    gpu.synchronize()
    got = do.to_numpy(np.float32, 4 * n).reshape(n, 4)
    want = transform_points(pts, mask, T, init)
    assert np.array_equal(bits(got), bits(want))


def test_run_mode_small_frames_forced(Engine, monkeypatch):
    """The runs-of-equal-keys voxelize (on by default from 2 Mi pixels, 4K is covered above) at
    small sizes through GDF_FORCE_RUNS: single frames with two cameras (the runs stop at camera
    borders), a 3-frame batch (frame bits in the run keys), voxel corners - bit-exact."""
    monkeypatch.setenv("GDF_FORCE_RUNS", "1")
    gpu, orc = Engine(), OracleFusion(threads=8)
    cams = [synth.make_camera(k, 320, 240) for k in range(2)]
    for avg in (True, False):
        p = ComponentParams()
        p.voxel_average = avg
        for f in range(2):
            args = [cam_args(c, synth.dense_frame(c, k, f)) for k, c in enumerate(cams)]
            run_fused(gpu, args, p)
            run_fused(orc, args, p)
            compare_results(gpu, orc, tag=f"avg={avg} frame {f}")
    p = ComponentParams()
    frames = [[cam_args(cams[0], synth.dense_frame(cams[0], 0, 10 + j))] for j in range(3)]
    _batch(gpu, frames, p)
    pts, vox = gpu.downloadPoints(), gpu.downloadVoxelizedPoints()
    ps, vs = gpu.batch_ranges()
    for j in range(3):
        run_fused(orc, frames[j], p)
        assert np.array_equal(bits(pts[ps[j]:ps[j + 1]]), bits(orc.downloadPoints()))
        assert np.array_equal(bits(vox[vs[j]:vs[j + 1], :3]),
                              bits(orc.downloadVoxelizedPoints()[:, :3]))
        np.testing.assert_array_equal(gpu.downloadBatchVoxelOccupancyGrid(j),
                                      orc.downloadVoxelOccupancyGrid())


@pytest.mark.parametrize("cells,runs", [((0.4, 0.4, 0.25), False), ((0.4, 0.4, 0.25), True),
                                         ((4.0, 4.0, 0.5), False), ((4.0, 4.0, 0.5), True)])
def test_wide_last_radix_digit_single_frames(Engine, monkeypatch, cells, runs):
    """Grids of 17-bit keys (100x100x10 cells: passes of 8 + 9 bits) and 9-bit keys (10x10x5:
    one 9-bit pass) - points and runs of equal keys, voxel means and grid bit-exact."""
    if runs:
        monkeypatch.setenv("GDF_FORCE_RUNS", "1")
    p = ComponentParams()
    p.voxel_size = cells
    gpu, orc = Engine(), OracleFusion(threads=8)
    cam = synth.make_camera(0, 320, 240)
    for f in range(2):
        args = [cam_args(cam, synth.dense_frame(cam, 0, f))]
        run_fused(gpu, args, p)
        run_fused(orc, args, p)
        compare_results(gpu, orc, tag=f"cells {cells} runs={runs} frame {f}")


@pytest.mark.gpu
def test_last_sort_items_reports_runs(Engine, monkeypatch):
    """gdf_last_sort_items (the bench's byte model): points when the voxelize sorts points, the
    runs of equal keys (fewer, >= the voxels) when it sorts runs; counts of a synchronous frame."""
    cam = synth.make_camera(0, 320, 240)
    args = [cam_args(cam, synth.dense_frame(cam, 0, 3))]
    p = ComponentParams()
    gpu = Engine()
    r = run_fused(gpu, args, p)
    items, runs = gpu.last_sort_items()
    assert not runs and items == r.num_points
    monkeypatch.setenv("GDF_FORCE_RUNS", "1")
    gpu2 = Engine()
    r2 = run_fused(gpu2, args, p)
    items2, runs2 = gpu2.last_sort_items()
    assert runs2 and r2.num_voxelized <= items2 < r2.num_points
