"""GPU parity tests: libgdf.so (HIP, gfx950) through the C-ABI vs the CPU oracle.

Bar (SURVEY.md §8c / north_star): masks, voxel keys, occupancy grids, historic grid and
rollbuffer indices bit-exact; world points and voxel means compared bit for bit as well (the
kernels follow the oracle's op order; the stated tolerance 1e-5 is the fallback, not needed).
"""
import numpy as np
import pytest

from drive import bits, compare_results, stagewise_frame
from oracle import OracleFusion, RefRadix  # noqa: F401
from ros_gpu_depthmap_fusion_amd import synth
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GDFError

pytestmark = pytest.mark.gpu

EYE = np.eye(4, dtype=np.float32)


def cam_args(cam, depth):
    return (depth, *cam.intrinsics(), cam.T_world, cam.T_crop)


@pytest.fixture(scope="module")
def Engine(gpu_engine_factory):
    return gpu_engine_factory


def run_fused(eng, cams_frames, params, **kw):
    eng.clear()
    for c in cams_frames:
        eng.addDepthmap(*c)
    return eng.processFrame(params, **kw)


def test_fused_vga_launch_defaults_multi_frame(Engine):
    """C2 workload (1 x VGA, launch defaults) over 4 frames: the historic grid evolves."""
    p = ComponentParams()
    gpu, orc = Engine(), OracleFusion(threads=8)
    cam = synth.make_camera(0, 640, 480)
    for f in range(4):
        args = [cam_args(cam, synth.depth_frame(cam, 0, f))]
        r = run_fused(gpu, args, p)
        run_fused(orc, args, p)
        assert r.processed == 1 and r.num_points == orc.point_count()
        compare_results(gpu, orc, tag=f"frame {f}")


def test_stagewise_code_defaults_and_stage_masks(Engine):
    """Stage-by-stage API (the component's exact call order) with the code defaults
    (F=1, thr 0.5, rot45 on, lifetime 1) on two cameras; per-pixel stage masks compared."""
    p = ComponentParams.code_defaults()
    p.crop_min, p.crop_max = (-3, -3, -1), (6, 3, 2.5)
    p.voxel_min, p.voxel_max = (-3, -3, -1), (6, 3, 2.5)
    gpu, orc = Engine(), OracleFusion(threads=4)
    gpu.set_debug(True)
    cams = synth.cameras(2, 200, 150)
    for f in range(3):
        args = [cam_args(c, synth.depth_frame(c, k, f)) for k, c in enumerate(cams)]
        stagewise_frame(gpu, args, p)
        stagewise_frame(orc, args, p)
        sm = gpu.stage_masks()
        st = orc.stage_arrays()
        n = orc.num_points_total()
        assert len(sm) == n
        depth_valid = np.concatenate([a[0].reshape(-1) != 0 for a in args])
        np.testing.assert_array_equal((sm & 1) != 0, depth_valid)
        np.testing.assert_array_equal((sm & 2) != 0, st["maskB"] != 0)
        np.testing.assert_array_equal((sm & 4) != 0, st["maskA"] != 0)
        compare_results(gpu, orc, tag=f"frame {f}")


def test_multicamera_cross_camera_border_semantics(Engine):
    """Cameras concatenated in one point space: camera k>0's top rows read camera k-1's bottom
    rows, left border wraps to the previous row (A.6)."""
    p = ComponentParams()
    p.flying_filter_size = 3
    gpu, orc = Engine(), OracleFusion(threads=4)
    gpu.set_debug(True)
    cams = synth.cameras(3, 128, 96)
    args = [cam_args(c, synth.depth_frame(c, k, 7)) for k, c in enumerate(cams)]
    run_fused(gpu, args, p)
    run_fused(orc, args, p)
    np.testing.assert_array_equal((gpu.stage_masks() & 4) != 0, orc.stage_arrays()["maskA"] != 0)
    compare_results(gpu, orc)


def test_six_cameras_mixed_sizes_rings_beyond_lds_halo(Engine):
    """More cameras than travel in the kernel arguments (descriptors read from the device),
    ragged sizes (tiles cut at right/bottom borders) and F=9: rings 1..8 read the LDS depth tile,
    ring 9 the linear-index global path; rot45 doubles every ring."""
    p = ComponentParams()
    p.flying_filter_size = 9
    p.flying_rot45 = True
    p.flying_threshold = 0.1
    gpu, orc = Engine(), OracleFusion(threads=8)
    gpu.set_debug(True)
    sizes = [(64, 48), (100, 75), (33, 20), (128, 96), (50, 50), (80, 61)]
    cams = [synth.make_camera(k, w, h) for k, (w, h) in enumerate(sizes)]
    for f in range(2):
        args = [cam_args(c, synth.depth_frame(c, k, f)) for k, c in enumerate(cams)]
        run_fused(gpu, args, p)
        run_fused(orc, args, p)
        np.testing.assert_array_equal((gpu.stage_masks() & 4) != 0,
                                      orc.stage_arrays()["maskA"] != 0)
        compare_results(gpu, orc, tag=f"frame {f}")


def test_alternating_frame_sizes_count_buffers(Engine):
    """Frames alternating between > 1 Mi items (separate tile-count scan) and small frames
    (k_emit sums the tile counts; the two count buffers are cleared frame to frame) in one
    engine."""
    p = ComponentParams()
    gpu, orc = Engine(), OracleFusion(threads=8)
    big = synth.make_camera(0, 1280, 960)
    small = synth.make_camera(1, 160, 120)
    mid = synth.make_camera(2, 640, 480)
    seq = [big, small, small, big, mid, big, mid, mid, small]
    for f, cam in enumerate(seq):
        args = [cam_args(cam, synth.depth_frame(cam, f % 3, f))]
        r = run_fused(gpu, args, p)
        run_fused(orc, args, p)
        assert r.num_points == orc.point_count(), f"frame {f}"
        compare_results(gpu, orc, tag=f"frame {f}")


def test_uniform_random_depth_stress(Engine):
    p = ComponentParams()
    p.flying_rot45 = True
    gpu, orc = Engine(), OracleFusion(threads=8)
    cam = synth.make_camera(1, 320, 240)
    for f in range(2):
        args = [cam_args(cam, synth.uniform_frame(cam, 1, f))]
        run_fused(gpu, args, p)
        run_fused(orc, args, p)
        compare_results(gpu, orc, tag=f"frame {f}")


@pytest.mark.parametrize("W,H", [(1, 1), (2, 3), (5, 1), (1, 7), (33, 31)])
def test_tiny_and_ragged_images(Engine, W, H):
    p = ComponentParams.code_defaults()
    p.crop_min = p.voxel_min = (-5, -5, -5)
    p.crop_max = p.voxel_max = (5, 5, 5)
    gpu, orc = Engine(), OracleFusion()
    rng = np.random.default_rng(W * 100 + H)
    cam = synth.make_camera(0, W, H)
    for f in range(2):
        d = rng.integers(0, 4000, (H, W)).astype(np.uint16)
        d[rng.random((H, W)) < 0.2] = 0
        run_fused(gpu, [cam_args(cam, d)], p)
        run_fused(orc, [cam_args(cam, d)], p)
        compare_results(gpu, orc)


def test_empty_and_all_zero_frames(Engine):
    p = ComponentParams()
    gpu, orc = Engine(), OracleFusion()
    gpu.clear()
    r = gpu.processFrame(p)
    assert r.processed == 0
    cam = synth.make_camera(0, 64, 48)
    # a populated frame, then an all-zero frame: no points, the grid only decays
    for d in (synth.depth_frame(cam, 0, 0), np.zeros((48, 64), np.uint16)):
        run_fused(gpu, [cam_args(cam, d)], p)
        run_fused(orc, [cam_args(cam, d)], p)
        compare_results(gpu, orc)
    assert gpu.point_count() == 0 and len(gpu.downloadVoxelizedPoints()) == 0
    assert gpu.downloadVoxelOccupancyGrid().max() == p.occupancy_lifetime - 1


def test_lifetime_u8_range_then_u32_history(Engine):
    """Lifetimes up to 255 keep the u8 grid as the history; 256+ switches to the u32 history
    (output byte = hist & 0xFF, uints_to_chars.glsl) and stays there."""
    p = ComponentParams()
    cam = synth.make_camera(0, 160, 120)
    gpu, orc = Engine(), OracleFusion()
    for f, life in enumerate([10, 200, 255, 255, 256, 300, 5, 1000]):
        p.occupancy_lifetime = life
        args = [cam_args(cam, synth.depth_frame(cam, 0, f))]
        run_fused(gpu, args, p)
        run_fused(orc, args, p)
        compare_results(gpu, orc, tag=f"frame {f} lifetime {life}")


def test_voxelize_corners_mode(Engine):
    p = ComponentParams()
    p.voxel_average = False
    cam = synth.make_camera(2, 160, 120)
    gpu, orc = Engine(), OracleFusion()
    args = [cam_args(cam, synth.depth_frame(cam, 2, 3))]
    run_fused(gpu, args, p)
    run_fused(orc, args, p)
    compare_results(gpu, orc)


def _add_sequences(engines, k0, nseq, cam, depth_fn, rng, empty_every=0, nan_frac=0.0):
    for k in range(k0, k0 + nseq):
        if empty_every and k % empty_every == 0:
            pts = np.zeros((0, 3), np.float32)
        else:
            pts = synth.back_project(cam, depth_fn(k))
            if nan_frac:
                pts[rng.random(len(pts)) < nan_frac] = np.nan
        s, ns = synth.sequence_time(k)
        for e in engines:
            e.addPointSequence(pts, s, ns, synth.move_transform(k))


@pytest.mark.parametrize("fused,depth", [(True, 1), (False, 1), (True, 3), (False, 2)])
def test_rollbuffer_chain(Engine, fused, depth):
    """Point sequences (with empty sequences and NaN points) through filter / insert / roll /
    select / transform over 8 frames, window of ~5 sequences (rollbuffer indices bit-exact);
    depth > 1: frame pipelining, where the rollbuffer frames wait for their predecessor."""
    p = ComponentParams()
    p.ps_timespan = 4.0 / 30.0
    p.ps_filter_size = 2
    lidar = synth.make_camera(0, 96, 64)
    cam = synth.make_camera(1, 120, 90)
    gpu, orc = Engine(), OracleFusion(threads=4)
    gpu.set_pipeline_depth(depth)
    rng = np.random.default_rng(9)
    Twm = synth.move_transform(3)
    Tcm = EYE
    k = 0
    for f in range(8):
        nseq = 1 + (f % 3)
        _add_sequences([gpu, orc], k, nseq, lidar, lambda kk: synth.depth_frame(lidar, 5, kk), rng,
                       empty_every=4, nan_frac=0.01)
        k += nseq
        args = [cam_args(cam, synth.depth_frame(cam, 1, f))] if f % 4 != 3 else []
        if fused:
            for e in (gpu, orc):
                e.clear()
                for a in args:
                    e.addDepthmap(*a)
                e.processFrame(p, T_world_move=Twm, T_crop_move=Tcm)
        else:
            stagewise_frame(gpu, args, p, Twm, Tcm)
            stagewise_frame(orc, args, p, Twm, Tcm)
        assert gpu.rollbuffer_state().as_tuple() == orc.rollbuffer_state(), f"frame {f}"
        gp, gm, gs, gh = gpu.rollbuffer_arrays()
        op, om, os_, oh = orc.rollbuffer_arrays()
        np.testing.assert_array_equal(gm, om)
        np.testing.assert_array_equal(gs, os_)
        np.testing.assert_array_equal(gh, oh)
        np.testing.assert_array_equal(bits(gp), bits(op))
        compare_results(gpu, orc, tag=f"frame {f}")


def test_voxelize_pinned_to_reference_radix_golden(Engine):
    """Points placed at voxel centres (through the rollbuffer with identity transforms) so the
    voxel keys ARE the golden keys of tests/golden/radix_ref.npz; the GPU voxel groups must come
    out in the reference RadixGrouper's order with the reference's group sizes."""
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "radix_ref.npz"))
    p = ComponentParams()
    p.ps_filter_size = 0
    p.ps_timespan = 1000.0
    p.voxel_min = p.crop_min = (0.0, 0.0, 0.0)
    p.voxel_max = p.crop_max = (2048.0, 2048.0, 1.0)
    p.voxel_size = (1.0, 1.0, 1.0)
    for name in ("voxelish", "dups", "ragged_tiles"):
        keys = g[name + "_keys"] % np.uint32(2048 * 2048)
        if name == "voxelish":
            keys = g[name + "_keys"]
            keys = keys[keys < 2048 * 2048]
        x = (keys % 2048).astype(np.float32) + np.float32(0.5)
        y = (keys // 2048).astype(np.float32) + np.float32(0.5)
        pts = np.stack([x, y, np.full_like(x, 0.5)], -1)
        gpu = Engine()
        gpu.clear()
        gpu.addPointSequence(pts, 5000, 0, EYE)
        gpu.processFrame(p, T_world_move=EYE, T_crop_move=EYE)
        assert gpu.point_count() == len(keys)
        np.testing.assert_array_equal(gpu.downloadVoxelCoords(), keys)
        vox = gpu.downloadVoxelizedPoints()
        # expected groups from the reference radix sort of exactly these keys
        ref_idx = np.argsort(keys, kind="stable")
        sk = keys[ref_idx]
        starts = np.flatnonzero(np.r_[True, sk[1:] != sk[:-1]])
        sizes = np.diff(np.r_[starts, len(sk)])
        assert len(vox) == len(starts)
        np.testing.assert_array_equal(vox[:, 0], x[ref_idx[starts]])  # all points of a voxel equal
        np.testing.assert_array_equal(vox[:, 3], sizes.astype(np.float32))  # w = sum of w = count
        if name != "voxelish":
            full = g[name + "_keys"]
            if np.array_equal(full, keys):
                np.testing.assert_array_equal(ref_idx, g[name + "_sorted_idx"])


def test_large_4k_frame_properties(Engine):
    """Full-size 4K frame: oracle parity (8 threads) plus size-independent properties."""
    p = ComponentParams()
    gpu, orc = Engine(), OracleFusion(threads=8)
    gpu.set_debug(True)
    cam = synth.make_camera(3, 3840, 2160)
    args = [cam_args(cam, synth.depth_frame(cam, 3, 0))]
    run_fused(gpu, args, p)
    run_fused(orc, args, p)
    compare_results(gpu, orc)
    sm = gpu.stage_masks()
    assert gpu.point_count() == int(np.count_nonzero(sm & 4))
    c = gpu.downloadVoxelCoords()
    vox = gpu.downloadVoxelizedPoints()
    assert len(vox) == len(np.unique(c))
    grid = gpu.downloadVoxelOccupancyGrid()
    assert np.count_nonzero(grid == p.occupancy_lifetime) == len(np.unique(c))


def test_errors_fail_loudly(Engine):
    gpu = Engine()
    with pytest.raises(GDFError):
        gpu.computeVoxelCoords((0, 0, 0), (1, 1, 1), (0.1, 0.1, 0.1))  # before applyPointMask
    gpu.clear()
    cam = synth.make_camera(0, 8, 8)
    gpu.addDepthmap(synth.depth_frame(cam, 0, 0), *cam.intrinsics(), cam.T_world, cam.T_crop)
    p = ComponentParams()
    p.voxel_min, p.voxel_max = (1, 1, 1), (0, 0, 0)
    with pytest.raises(GDFError):
        gpu.processFrame(p)


def test_multi_gpu_mark_export_import(Engine):
    """The multi-GPU exchange kernels on one device: two engines (one camera each) defer their
    grid, export marks (k_export_marks bit layout = multi.pack_marks), import the concatenated
    masks of both (k_import_marks ORs them) and update; both grids must equal the oracle
    history of the union of the two cameras' marks, frame after frame."""
    from ros_gpu_depthmap_fusion_amd import hiprt, multi
    p = ComponentParams()
    p.occupancy_lifetime = 4
    cams = [synth.make_camera(k, 160, 120) for k in range(2)]
    gpus = [Engine() for _ in cams]
    orcs = [OracleFusion(threads=4) for _ in cams]
    hist = None
    for f in range(3):
        words = []
        union = None
        for k, (c, g, o) in enumerate(zip(cams, gpus, orcs)):
            args = [cam_args(c, synth.depth_frame(c, k, f))]
            run_fused(g, args, p, defer_occupancy_grid=True)
            run_fused(o, args, p)
            (_, _, _), ncells = g.grid_size()
            nw = multi.words_for(ncells)
            buf = hiprt.DeviceArray(nw * 4)
            g.export_marks(buf.ptr, nw)
            g.synchronize()
            w = buf.to_numpy(np.uint32, nw)
            m = np.zeros(ncells, bool)
            m[o.downloadVoxelCoords()] = True
            np.testing.assert_array_equal(w, multi.pack_marks(m), err_msg=f"export cam {k}")
            words.append(w)
            union = m if union is None else union | m
        both = hiprt.DeviceArray.from_numpy(np.concatenate(words))
        hist = np.zeros(union.size, np.uint32) if hist is None else hist
        hist = multi.historic_update(hist, union, p.occupancy_lifetime)
        for k, g in enumerate(gpus):
            g.import_marks(both.ptr, len(words[0]), 2)
            g.voxelOccupancyGrid(p.occupancy_lifetime)
            np.testing.assert_array_equal(g.downloadVoxelOccupancyGrid().reshape(-1),
                                          (hist & 0xFF).astype(np.uint8),
                                          err_msg=f"frame {f} rank {k}")


def _gpu_outputs(e):
    return (e.downloadPoints(), e.downloadVoxelizedPoints(), e.downloadVoxelOccupancyGrid())


def test_pipelined_frames_match_sequential(Engine):
    """Frame pipelining (3 slots): synchronous frames give the sequential engine's outputs frame
    by frame; then 40 asynchronous frames of two cameras, including a change of the flying
    filter and of the lifetime (u8 -> u32 history), end in the same grid and last-frame outputs."""
    p = ComponentParams()
    cams = synth.cameras(2, 160, 120)
    seq, pipe = Engine(), Engine()
    pipe.set_pipeline_depth(3)
    for f in range(6):
        args = [cam_args(c, synth.depth_frame(c, k, f)) for k, c in enumerate(cams)]
        for e in (seq, pipe):
            run_fused(e, args, p)
        for a, b in zip(_gpu_outputs(seq), _gpu_outputs(pipe)):
            np.testing.assert_array_equal(bits(a) if a.dtype == np.float32 else a,
                                          bits(b) if b.dtype == np.float32 else b,
                                          err_msg=f"frame {f}")
    for f in range(6, 46):
        if f == 20:
            p.flying_filter_size = 2
        if f == 30:
            p.occupancy_lifetime = 300
        args = [cam_args(c, synth.depth_frame(c, k, f % 9)) for k, c in enumerate(cams)]
        for e in (seq, pipe):
            run_fused(e, args, p, synchronous=False)
    seq.synchronize()
    pipe.synchronize()
    for a, b in zip(_gpu_outputs(seq), _gpu_outputs(pipe)):
        np.testing.assert_array_equal(bits(a) if a.dtype == np.float32 else a,
                                      bits(b) if b.dtype == np.float32 else b)
    np.testing.assert_array_equal(seq.historic_grid(), pipe.historic_grid())


def test_cpp_stream_loop_matches_oracle(Engine):
    """gdf_run_depth_stream (the component loop in C++, include/gdf_driver.h) over a ring of
    device depth maps of two cameras, pipelined 3 deep, ends in the oracle's grid and last-frame
    outputs; the ring index wraps."""
    from ros_gpu_depthmap_fusion_amd import hiprt
    p = ComponentParams()
    cams = synth.cameras(2, 160, 120)
    ring = 5
    host = [[synth.depth_frame(c, k, f) for f in range(ring)] for k, c in enumerate(cams)]
    dev = [[hiprt.DeviceArray.from_numpy(d) for d in h] for h in host]
    gpu, orc = Engine(), OracleFusion(threads=4)
    gpu.set_pipeline_depth(3)
    scams = [gpu.make_stream_camera([d.ptr for d in dev[k]], c.width, c.height, *c.intrinsics(),
                                    c.T_world, c.T_crop) for k, c in enumerate(cams)]
    nframes = 13
    gpu.run_depth_stream(scams, p.to_c(None, None, False, False), 0, nframes)
    gpu.synchronize()
    for f in range(nframes):
        run_fused(orc, [cam_args(c, host[k][f % ring]) for k, c in enumerate(cams)], p)
    compare_results(gpu, orc, tag="stream")
    np.testing.assert_array_equal(gpu.historic_grid(), orc.historic_grid())


def test_graph_replay_matches_direct_launches(Engine):
    """Steady-state frames replayed from HIP graphs (kernel-node updates of the depth pointers
    and the grid ticket) give the direct launches' outputs frame by frame: device depth maps of
    two cameras from a ring (a new pointer every frame), 3 slots; then an asynchronous stretch
    with a parameter change (recapture) ends in the same grid, checked against the oracle too."""
    from ros_gpu_depthmap_fusion_amd import hiprt
    p = ComponentParams()
    cams = synth.cameras(2, 160, 120)
    ring = 7
    host = [[synth.depth_frame(c, k, f) for f in range(ring)] for k, c in enumerate(cams)]
    dev = [[hiprt.DeviceArray.from_numpy(d) for d in h] for h in host]
    direct, graph = Engine(), Engine()
    direct.set_graphs(False)
    graph.set_graphs(True)
    for e in (direct, graph):
        e.set_pipeline_depth(3)

    def frame(e, f, **kw):
        e.clear()
        for k, c in enumerate(cams):
            e.addDepthmapDevice(dev[k][f % ring].ptr, c.width, c.height, *c.intrinsics(),
                                c.T_world, c.T_crop)
        return e.processFrame(p, **kw)

    for f in range(12):
        for e in (direct, graph):
            frame(e, f, synchronous=True)
        for a, b in zip(_gpu_outputs(direct), _gpu_outputs(graph)):
            np.testing.assert_array_equal(bits(a) if a.dtype == np.float32 else a,
                                          bits(b) if b.dtype == np.float32 else b,
                                          err_msg=f"frame {f}")
    orc = OracleFusion(threads=4)
    for f in range(12):
        run_fused(orc, [cam_args(c, host[k][f % ring]) for k, c in enumerate(cams)], p)
    for f in range(12, 40):
        if f == 25:
            p.flying_threshold = 0.4
            p.voxel_average = False
        for e in (direct, graph):
            frame(e, f, synchronous=False)
        run_fused(orc, [cam_args(c, host[k][f % ring]) for k, c in enumerate(cams)], p)
    direct.synchronize()
    graph.synchronize()
    for a, b in zip(_gpu_outputs(direct), _gpu_outputs(graph)):
        np.testing.assert_array_equal(bits(a) if a.dtype == np.float32 else a,
                                      bits(b) if b.dtype == np.float32 else b)
    np.testing.assert_array_equal(graph.historic_grid(), orc.historic_grid())
    compare_results(graph, orc, tag="graph")


@pytest.mark.parametrize("step", [16, 20, 12])
def test_device_point_sequences_match_host(Engine, step):
    """addPointSequenceDevice (PointCloud2 records in device memory, gathered on the GPU) gives
    the host path's rollbuffer and frame outputs, mixed with host sequences in one frame and
    with records of other point_step (extra fields after x,y,z); oracle checked too."""
    from ros_gpu_depthmap_fusion_amd import hiprt
    p = ComponentParams()
    p.ps_timespan = 3.0 / 30.0
    lidar = synth.make_camera(0, 64, 48)
    cam = synth.make_camera(1, 96, 72)
    host, dev, orc = Engine(), Engine(), OracleFusion(threads=4)
    keep = []
    rng = np.random.default_rng(step)
    k = 0
    for f in range(5):
        for j in range(2):
            pts = synth.back_project(lidar, synth.depth_frame(lidar, 5, k))
            if f == 2 and j == 0:
                pts = pts[:0]  # an empty sequence
            s, ns = synth.sequence_time(k)
            T = synth.move_transform(k)
            host.addPointSequence(pts, s, ns, T)
            orc.addPointSequence(pts, s, ns, T)
            if j == 1 and f % 2:  # a host sequence inside a device-fed frame
                dev.addPointSequence(pts, s, ns, T)
            else:
                rec = np.zeros((len(pts), step // 4), np.float32)
                rec[:, :3] = pts
                if step > 12:
                    rec[:, 3:] = rng.random((len(pts), step // 4 - 3))
                d = hiprt.DeviceArray.from_numpy(rec) if len(pts) else None
                keep.append(d)
                dev.addPointSequenceDevice(d.ptr if d else 0, len(pts), step, s, ns, T)
            k += 1
        args = [cam_args(cam, synth.depth_frame(cam, 1, f))]
        for e in (host, dev, orc):
            e.clear()
            for a in args:
                e.addDepthmap(*a)
            e.processFrame(p, T_world_move=cam.T_world, T_crop_move=cam.T_crop)
        assert dev.rollbuffer_state().as_tuple() == orc.rollbuffer_state(), f"frame {f}"
        for a, b in zip(_gpu_outputs(host), _gpu_outputs(dev)):
            np.testing.assert_array_equal(bits(a) if a.dtype == np.float32 else a,
                                          bits(b) if b.dtype == np.float32 else b,
                                          err_msg=f"frame {f}")
        gp, gm, gs, gh = dev.rollbuffer_arrays()
        op, om, os_, oh = orc.rollbuffer_arrays()
        np.testing.assert_array_equal(gm, om)
        np.testing.assert_array_equal(bits(gp), bits(op))
        compare_results(dev, orc, tag=f"frame {f}")
    with pytest.raises(GDFError):  # misaligned records
        dev.addPointSequenceDevice(keep[1].ptr + 2, 4, 16, 0, 0, EYE)


def test_large_rollbuffer_window_properties(Engine):
    """A C3-like window at reduced size (48 sequences of 320x240 device records = 3.7 M selected
    points per frame; radix tiles at 16 keys per thread): the compaction count equals the
    stage-mask count, one voxel mean per distinct key, and the grid holds exactly the frame's
    voxels at full lifetime."""
    from ros_gpu_depthmap_fusion_amd import hiprt
    p = ComponentParams()
    p.ps_timespan = 47.5 / 30.0
    lidar = synth.make_camera(0, 320, 240)
    n = 320 * 240
    seqs = [hiprt.DeviceArray.from_numpy(np.concatenate(
        [synth.back_project(lidar, synth.depth_frame(lidar, 0, f)),
         np.ones((n, 1), np.float32)], 1)) for f in range(4)]
    gpu = Engine()
    gpu.set_debug(True)
    for k in range(56):
        s, ns = synth.sequence_time(k)
        gpu.addPointSequenceDevice(seqs[k % 4].ptr, n, 16, s, ns, synth.move_transform(k))
        gpu.clear()
        r = gpu.processFrame(p, T_world_move=lidar.T_world, T_crop_move=lidar.T_crop,
                             synchronous=k == 55)
    st = gpu.rollbuffer_state()
    assert st.selection_sequence_count == 48 and r.num_points_total == 48 * n
    sm = gpu.stage_masks()
    assert gpu.point_count() == int(np.count_nonzero(sm & 4)) > 1_000_000
    c = gpu.downloadVoxelCoords()
    assert len(gpu.downloadVoxelizedPoints()) == len(np.unique(c))
    grid = gpu.downloadVoxelOccupancyGrid().reshape(-1)
    assert np.array_equal(np.flatnonzero(grid == p.occupancy_lifetime), np.unique(c))


@pytest.mark.parametrize("lifetime", [5, 300])
def test_batched_mark_exchange_pipelined(Engine, lifetime):
    """Batched multi-GPU exchange on one device: two engines (one camera each, 3 frames in
    flight) process 7 frames with deferred grids, take (export + clear) their marks into
    [batch, words] buffers, then import each frame's union from the concatenated
    [rank, batch, words] masks (stride batch * words) and update in frame order; every rank's
    grid equals the host history of the union, and the u32 history of a per-frame engine."""
    from ros_gpu_depthmap_fusion_amd import hiprt, multi
    p = ComponentParams()
    p.occupancy_lifetime = lifetime  # 300: the u32 history (frame-by-frame inside the batch call)
    cams = [synth.make_camera(k, 160, 120) for k in range(2)]
    gpus = [Engine() for _ in cams]
    for g in gpus:
        g.set_pipeline_depth(3)
    orcs = [OracleFusion(threads=4) for _ in cams]
    batch, nframes = 4, 7
    hist = None
    done = 0
    while done < nframes:
        nb = min(batch, nframes - done)
        bufs, unions = [], []
        for k, (c, g, o) in enumerate(zip(cams, gpus, orcs)):
            (_, _, _), ncells = (None, None, None), None
            local = None
            for i in range(nb):
                f = done + i
                args = [cam_args(c, synth.depth_frame(c, k, f))]
                run_fused(g, args, p, defer_occupancy_grid=True, synchronous=False)
                run_fused(o, args, p)
                _, ncells = g.grid_size()
                nw = multi.words_for(ncells)
                if local is None:
                    local = hiprt.DeviceArray(batch * nw * 4)
                g.take_marks(local.ptr + 4 * i * nw, nw)
                m = np.zeros(ncells, bool)
                m[o.downloadVoxelCoords()] = True
                if k == 0:
                    unions.append(m)
                else:
                    unions[i] |= m
            g.synchronize()
            bufs.append(local.to_numpy(np.uint32, batch * nw))
        both = hiprt.DeviceArray.from_numpy(np.concatenate(bufs))
        for i in range(nb):
            hist = np.zeros(ncells, np.uint32) if hist is None else hist
            hist = multi.historic_update(hist, unions[i], p.occupancy_lifetime)
            for g in gpus:
                g.import_marks(both.ptr + 4 * i * nw, nw, 2, rank_stride=batch * nw)
                g.voxelOccupancyGrid(p.occupancy_lifetime)
        for k, g in enumerate(gpus):
            np.testing.assert_array_equal(g.downloadVoxelOccupancyGrid().reshape(-1),
                                          (hist & 0xFF).astype(np.uint8),
                                          err_msg=f"frames {done}..{done + nb} rank {k}")
        done += nb


def test_sparse_mark_pairs_and_union(Engine):
    """take_marks_sparse: the pairs are exactly the non-zero words of the taken bitmask (any
    order), the engine's marks are cleared; union_pairs of two records ORs them; an over-cap
    record reports its full count (the caller then falls back to the bitmasks)."""
    from ros_gpu_depthmap_fusion_amd import hiprt, multi
    p = ComponentParams()
    gpu = Engine()
    recs, masks = [], []
    cap = 4096
    for k in range(2):
        cam = synth.make_camera(k, 200, 150)
        run_fused(gpu, [cam_args(cam, synth.depth_frame(cam, k, 3))], p, defer_occupancy_grid=True)
        _, ncells = gpu.grid_size()
        nw = multi.words_for(ncells)
        bits = hiprt.DeviceArray(nw * 4)
        pairs = hiprt.DeviceArray((1 + 2 * cap) * 4)
        gpu.take_marks_sparse(bits.ptr, nw, pairs.ptr, cap)
        gpu.synchronize()
        b = bits.to_numpy(np.uint32, nw)
        pr = pairs.to_numpy(np.uint32, 1 + 2 * cap)
        nz = np.flatnonzero(b)
        assert pr[0] == len(nz) <= cap
        idx, val = pr[1:1 + 2 * pr[0]:2], pr[2:2 + 2 * pr[0]:2]
        order = np.argsort(idx)
        np.testing.assert_array_equal(idx[order], nz)
        np.testing.assert_array_equal(val[order], b[nz])
        recs.append(pr)
        masks.append(b)
        # marks were cleared: a second take finds none
        gpu.take_marks_sparse(bits.ptr, nw, pairs.ptr, cap)
        gpu.synchronize()
        assert pairs.to_numpy(np.uint32, 1)[0] == 0 and not bits.to_numpy(np.uint32, nw).any()
    both = hiprt.DeviceArray.from_numpy(np.concatenate(recs))
    uni = hiprt.DeviceArray(nw * 4)
    gpu.union_pairs(uni.ptr, nw, both.ptr, 2, 1, 1 + 2 * cap)
    gpu.synchronize()
    np.testing.assert_array_equal(uni.to_numpy(np.uint32, nw), masks[0] | masks[1])
    # over cap: count is complete, the pairs stop at cap
    cam = synth.make_camera(0, 200, 150)
    run_fused(gpu, [cam_args(cam, synth.depth_frame(cam, 0, 4))], p, defer_occupancy_grid=True)
    small = hiprt.DeviceArray((1 + 2 * 8) * 4)
    gpu.take_marks_sparse(bits.ptr, nw, small.ptr, 8)
    gpu.synchronize()
    assert small.to_numpy(np.uint32, 1)[0] == np.count_nonzero(bits.to_numpy(np.uint32, nw)) > 8


def test_graph_cache_alternating_parameters(Engine):
    """A caller alternating between parameter sets every frame (the component's runtime config
    topics, component.cpp:970-990) replays one cached graph per set and slot instead of
    re-capturing: frame by frame equal to direct launches, the grid equal to the oracle's, and
    each (slot, set) captured once."""
    from ros_gpu_depthmap_fusion_amd import hiprt
    cams = synth.cameras(2, 160, 120)
    ring = 5
    host = [[synth.dense_frame(c, f, k) for f in range(ring)] for k, c in enumerate(cams)]
    dev = [[hiprt.DeviceArray.from_numpy(d) for d in h] for h in host]
    sets = [ComponentParams(), ComponentParams(flying_threshold=0.35),
            ComponentParams(voxel_average=False)]
    direct, graph = Engine(), Engine()
    direct.set_graphs(False)
    graph.set_graphs(True)
    for e in (direct, graph):
        e.set_pipeline_depth(3)
    orc = OracleFusion(threads=4)
    nframes = 36
    for f in range(nframes):
        p = sets[f % 2] if f < 24 else sets[f % 3]
        for e in (direct, graph):
            e.clear()
            for k, c in enumerate(cams):
                e.addDepthmapDevice(dev[k][f % ring].ptr, c.width, c.height, *c.intrinsics(),
                                    c.T_world, c.T_crop)
            e.processFrame(p, synchronous=False)
        run_fused(orc, [cam_args(c, host[k][f % ring]) for k, c in enumerate(cams)], p)
        if f % 6 == 5:
            direct.synchronize()
            graph.synchronize()
            for a, b in zip(_gpu_outputs(direct), _gpu_outputs(graph)):
                np.testing.assert_array_equal(bits(a) if a.dtype == np.float32 else a,
                                              bits(b) if b.dtype == np.float32 else b,
                                              err_msg=f"frame {f}")
    graph.synchronize()
    np.testing.assert_array_equal(graph.historic_grid(), orc.historic_grid())
    captures, replays = graph.graph_stats()
    assert captures <= 3 * 3, captures   # <= one per (slot, parameter set)
    assert replays >= nframes - 2 * 3 * 3 - 3 * 3, replays
