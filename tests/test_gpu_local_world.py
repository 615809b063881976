"""The product multi-GPU step - the C++ gdf_fused_* step that `bench.py --gpus N` runs - at
world 2, 3, 4 and 8 on the box's one GPU, through the in-process transport (gdf_fused_local: one
engine and one host thread per rank, the step's collectives as device copies on the ranks' streams,
include/gdf_fused.h).  The step's code is the RCCL ranks' code: halo tails all-gathered and
indexed per rank, the split sizes' all-gather, the grouped send / recv of points and runs at their
offsets, the key-range voxelize, the in-place mark-slice all-gather, the batched grid update.

Every check is against ONE oracle engine over all cameras (the reference fuses every camera in
one process: src/gpu_depthmap_fusion.cpp:1583-1756, buffer order :1509-1581, one voxelize
:1743-1756): per frame the ranks' voxel ranges concatenated in rank order, every rank's grid, and
the rollbuffer state, bit for bit."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

from ros_gpu_depthmap_fusion_amd import synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams  # noqa: E402

pytestmark = pytest.mark.gpu


def small_params(F=4):
    p = ComponentParams()
    p.flying_filter_size = F
    p.voxel_min, p.voxel_max = (-8.0, -8.0, -1.0), (8.0, 8.0, 2.0)
    p.crop_min, p.crop_max = p.voxel_min, p.voxel_max
    return p


def run_local_world(world, W_, H_, steps, B, params, depth, rb=None, fused_run=False, shard=0):
    """`steps` steps of B frames of `world` cameras through `world` C++ ranks of one local world,
    pipelined `depth` deep.  rb = (LW, LH, first): the last rank ingests fused_ref.schedule's
    point sequences (one step per frame, B = 1); shard > 0: EVERY rank ingests them and keeps its
    blocks of `shard` sequences (the sharded window).  Returns (depth frames, per-rank results)."""
    import fused_ref
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    from ros_gpu_depthmap_fusion_amd.multi import LocalFusedWorld, NativeFusedRank
    build_library()
    nf = steps * B
    cams = [synth.make_camera(k, W_, H_) for k in range(world)]
    depths = [[synth.dense_frame(cams[k], k, f) for f in range(nf)] for k in range(world)]
    dev = [[hiprt.DeviceArray.from_numpy(depths[k][f]) for f in range(nf)] for k in range(world)]
    recs, sched, lidar = None, None, None
    if rb is not None:
        LW, LH, first = rb
        lidar = fused_ref.lidar_camera(LW, LH)
        recs = [hiprt.DeviceArray.from_numpy(fused_ref.sequence_records(lidar, k)) for k in range(2)]
        sched = fused_ref.schedule(first, nf)
    lw = LocalFusedWorld(world)
    engines = [GPUDepthmapFusion(0) for _ in range(world)]
    ranks = [NativeFusedRank(engines[r], cams, r, world, params, depth=depth, local=lw)
             for r in range(world)]
    assert all(fr.info() == (r, world, world, "local") for r, fr in enumerate(ranks))
    if shard:
        for fr in ranks:
            fr.shard_rollbuffer(shard)

    def body(r):
        fr, eng = ranks[r], engines[r]
        vox, grids, states = {}, {}, {}

        def move(i):
            if i:  # the rollbuffer state after step i - 1 (engine state, read before step i starts)
                states[i - 1] = tuple(eng.rollbuffer_state().as_tuple())
            for k in sched[i]:
                eng.addPointSequenceDevice(recs[k % 2].ptr, LW * LH, 16, *synth.sequence_time(k),
                                           synth.move_transform(k))
            return (lidar.T_world, lidar.T_crop)

        def done(i):
            eng.synchronize()
            v = eng.downloadVoxelizedPoints()[:, :3]
            if B == 1:
                vox[i] = v
            else:
                _, vs = eng.batch_ranges()
                for j in range(B):
                    vox[B * i + j] = v[vs[j]:vs[j + 1]]
            grids[i] = eng.downloadVoxelOccupancyGrid()

        fr.run(steps, lambda i: [dev[r][B * i + j].ptr for j in range(B)], lambda i: None,
               move_of=move if (rb is not None and fr.has_rollbuffer) else None, on_finish=done)
        eng.synchronize()
        if rb is not None and fr.has_rollbuffer:
            states[steps - 1] = tuple(eng.rollbuffer_state().as_tuple())
        last = None
        if fused_run:  # gdf_fused_run: the C++ loop over the same frames (depth in flight)
            fr.run_stream([d.ptr for d in dev[r]], 0, steps, B)
            eng.synchronize()
            last = eng.downloadVoxelizedPoints()[:, :3]
        return vox, grids, states, last

    try:
        res = lw.run(body)
    finally:
        for fr in ranks:
            fr.close()
        lw.close()
    return cams, depths, res


def oracle_frames(cams, depths, params, threads=16, rb=None, nf=None):
    """ONE oracle engine over all cameras (+ the point sequences): per frame (voxel means, grid,
    rollbuffer state)."""
    import fused_ref
    from oracle import OracleFusion
    orc = OracleFusion(threads=threads)
    nf = len(depths[0]) if nf is None else nf
    lidar = recs = sched = None
    if rb is not None:
        LW, LH, first = rb
        lidar = fused_ref.lidar_camera(LW, LH)
        recs = [fused_ref.sequence_records(lidar, k) for k in range(2)]
        sched = fused_ref.schedule(first, nf)
    for f in range(nf):
        if rb is not None:
            for k in sched[f]:
                orc.addPointSequence(recs[k % 2], *synth.sequence_time(k), synth.move_transform(k))
        orc.clear()
        for k, c in enumerate(cams):
            orc.addDepthmap(depths[k][f], *c.intrinsics(), c.T_world, c.T_crop)
        if rb is not None:
            orc.processFrame(params, T_world_move=lidar.T_world, T_crop_move=lidar.T_crop)
        else:
            orc.processFrame(params)
        yield (orc.downloadVoxelizedPoints()[:, :3], orc.downloadVoxelOccupancyGrid(),
               tuple(orc.rollbuffer_state()) if rb is not None else None)


def check(tag, world, B, res, oracle_iter, rb=False, sharded=False):
    n_checked = 0
    for f, (want, grid, st) in enumerate(oracle_iter):
        got = np.concatenate([res[r][0][f] for r in range(world)])
        assert len(got) == len(want) > 0, f"{tag} frame {f}: {len(got)} vs {len(want)} voxels"
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"{tag} frame {f}"
        if f % B == B - 1:  # the grid after the step (the batch's last frame)
            for r in range(world):
                np.testing.assert_array_equal(res[r][1][f // B], grid, f"{tag} frame {f} rank {r}")
        if rb and not sharded:
            assert st[3] > 0, f"{tag} frame {f}: rollbuffer points selected"
            assert res[world - 1][2][f] == st, f"{tag} frame {f} rollbuffer state"
        elif rb:  # the shards' states: point counts add up, the sequence bookkeeping is the same
            sts = [res[r][2][f] for r in range(world)]
            assert st[3] > 0 and sum(1 for x in sts if x[3] > 0) >= 2, f"{tag} frame {f}: shares"
            assert sum(x[0] for x in sts) == st[0], f"{tag} frame {f}: rollbuffer points"
            assert sum(x[3] for x in sts) == st[3], f"{tag} frame {f}: selected points"
            for x in sts:  # num_seqs, selected sequences, earliest / last times
                assert (x[1],) + tuple(x[4:]) == (st[1],) + tuple(st[4:]), f"{tag} frame {f}"
        n_checked += 1
    return n_checked


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_local_world_batches_pipelined(world):
    """world ranks x 160x120 cameras, F = 4, 4 steps of 3 frames, 3 steps in flight (and
    gdf_fused_run's C++ loop over the same frames): every frame's fused cloud and every rank's
    grid after every step equal one oracle engine over all cameras."""
    p = small_params(4)
    steps, B = 4, 3
    cams, depths, res = run_local_world(world, 160, 120, steps, B, p, depth=3, fused_run=True)
    assert check(f"w{world}", world, B, res, oracle_frames(cams, depths, p, threads=8)) == steps * B
    # gdf_fused_run's last step: its voxels = the last step's frames' voxels
    for r in range(world):
        want = np.concatenate([res[r][0][f] for f in range(steps * B - B, steps * B)])
        assert np.array_equal(res[r][3].view(np.uint32), want.view(np.uint32)), f"fused_run rank {r}"


@pytest.mark.parametrize("world,F", [(2, 0), (3, 9)])
def test_local_world_single_frames(world, F):
    """Single-frame steps (no batch), F = 0 (no halo) and F = 9 (a 9-row halo), one step in
    flight."""
    p = small_params(F)
    cams, depths, res = run_local_world(world, 160, 120, 3, 1, p, depth=1)
    assert check(f"w{world}F{F}", world, 1, res, oracle_frames(cams, depths, p, threads=8)) == 3


def test_local_world_c4_shape():
    """4 ranks x 1280x720 at launch defaults, steps of B = 8 frames (2 steps, 2
    in flight) - 16 frames of 4 cameras fused per rank's key range."""
    p = ComponentParams()
    cams, depths, res = run_local_world(4, 1280, 720, 2, 8, p, depth=2)
    assert check("C4", 4, 8, res, oracle_frames(cams, depths, p)) == 16


def test_local_world_c5_shape():
    """8 ranks x 3840x2160 at launch defaults, single-frame steps (2 frames, 2
    in flight): 66 M depth pixels per frame fused into one cloud."""
    p = ComponentParams()
    cams, depths, res = run_local_world(8, 3840, 2160, 2, 1, p, depth=2)
    assert check("C5", 8, 1, res, oracle_frames(cams, depths, p)) == 2


@pytest.mark.parametrize("world", [2, 4])
def test_local_world_rollbuffer_leg(world):
    """The rollbuffer leg through the C++ step: the last rank ingests a window of 8 x 720p point
    sequences (6.4 M points; one more per frame, the oldest rolled out from frame 1), its selected
    points follow its camera's in its send lists; VGA cameras at launch defaults, 3 single-frame
    steps, 2 in flight: fused clouds, grids and the rollbuffer state equal one oracle engine."""
    p = ComponentParams()
    win = 8
    p.ps_timespan = (win - 0.5) / 30.0
    rb = (1280, 720, win)
    cams, depths, res = run_local_world(world, 640, 480, 3, 1, p, depth=2, rb=rb)
    assert check(f"rb{world}", world, 1, res, oracle_frames(cams, depths, p, rb=rb), rb=True) == 3


@pytest.mark.parametrize("world", [2, 3, 4])
def test_local_world_sharded_rollbuffer(world):
    """The rollbuffer window SHARDED over the ranks (gdf_fused_set_rollbuffer_shard): every rank
    ingests every 720p point sequence of an 8-sequence window and keeps its blocks of
    ceil(7 / (world - 1)) sequences; the exchange carries [depth | rollbuffer] buckets, placed as
    [every rank's depth points, the rollbuffer segments in the selection's order].  VGA cameras at
    launch defaults, 4 single-frame steps (the window rolls from frame 1, the blocks rotate over
    the ranks), 2 in flight: every fused cloud and grid equals ONE unsharded oracle engine's, the
    shards' rollbuffer points add up to its own."""
    p = ComponentParams()
    win = 8
    p.ps_timespan = (win - 0.5) / 30.0
    rb = (1280, 720, win)
    block = -(-(win - 1) // (world - 1))
    cams, depths, res = run_local_world(world, 640, 480, 4, 1, p, depth=2, rb=rb, shard=block)
    assert check(f"shard{world}", world, 1, res, oracle_frames(cams, depths, p, rb=rb), rb=True,
                 sharded=True) == 4


@pytest.mark.parametrize("world,block", [(3, 2), (4, 1), (8, 1)])
def test_local_world_sharded_window_over_the_limit(world, block):
    """A window spanning MORE than `world` blocks (a burst of sequences against a block size made
    for a shorter window): a rank holds several separate pieces of the selection (world 3 /
    block 2: up to 2; world 4 / block 1: 2 each; world 8 / block 1: the 8-sequence window on 8
    ranks, 1 each, the 9th sequence wrapping onto rank 0 from frame 1).  The partition cuts the
    rank's rollbuffer points where each piece starts (k_sel records the survivors before the cut)
    and every owner places the pieces in the selection's order: every fused cloud and grid equal
    ONE unsharded oracle engine's."""
    p = ComponentParams()
    win = 8
    p.ps_timespan = (win - 0.5) / 30.0
    rb = (1280, 720, win)
    cams, depths, res = run_local_world(world, 640, 480, 4, 1, p, depth=2, rb=rb, shard=block)
    assert check(f"burst{world}", world, 1, res, oracle_frames(cams, depths, p, rb=rb), rb=True,
                 sharded=True) == 4


def test_local_world_sharded_window_too_many_pieces_fails_alike():
    """World 2, block 1, an 8-sequence window: each rank would hold 4 pieces, more than the 3 the
    exchange carries - the step fails on EVERY rank with GDF_ERR_STATE at once (the headers are
    replicated, so the ranks decide alike), naming the pieces; no rank waits for another."""
    import time
    from ros_gpu_depthmap_fusion_amd.gdf import GDFError
    p = ComponentParams()
    win = 8
    p.ps_timespan = (win - 0.5) / 30.0
    t0 = time.time()
    with pytest.raises(GDFError) as ei:
        run_local_world(2, 640, 480, 1, 1, p, depth=1, rb=(1280, 720, win), shard=1)
    assert "separate pieces" in str(ei.value) or "aborted" in str(ei.value), str(ei.value)
    assert time.time() - t0 < 120


def test_local_world_c5_sharded_full_window():
    """SURVEY §8(d) C5 as BASELINE states it - 8 cameras x 3840x2160 at launch defaults WITH the
    rollbuffer - through the product step at world 8: a window of 32 x 720p point sequences (29.5 M
    points) sharded over the 8 ranks in blocks of ceil(31 / 7) = 5 (up to 2N = 16 sources per
    voxelize), 3 single-frame steps (the window rolls from frame 1, the blocks rotate), 2 in
    flight.  The reference's order: depth, then rollbuffer points at offset sum(P)
    (src/gpu_depthmap_fusion.cpp:1509-1581), one voxelize (:1743-1756) - every fused cloud and
    every rank's grid equal ONE unsharded oracle engine's, the shards' rollbuffer points add up."""
    p = ComponentParams()
    win, world = 32, 8
    p.ps_timespan = (win - 0.5) / 30.0
    rb = (1280, 720, win)
    block = -(-(win - 1) // (world - 1))
    cams, depths, res = run_local_world(world, 3840, 2160, 3, 1, p, depth=2, rb=rb, shard=block)
    assert check("C5rb", world, 1, res, oracle_frames(cams, depths, p, rb=rb), rb=True,
                 sharded=True) == 3


def test_one_rank_bad_argument_aborts_the_world_at_once():
    """One rank of a world-2 step is given a null depth map (GDF_ERR_ARG on that rank alone): its
    peer, already waiting in the step's first collective, fails with GDF_ERR_STATE at once - not
    after the transport's 300 s timeout (a failed step aborts the world whatever the error)."""
    import ctypes as C
    import time
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    from ros_gpu_depthmap_fusion_amd.multi import LocalFusedWorld, NativeFusedRank
    build_library()
    p = small_params(4)
    cams = [synth.make_camera(k, 160, 120) for k in range(2)]
    d = [hiprt.DeviceArray.from_numpy(synth.dense_frame(cams[k], k, 0)) for k in range(2)]
    lw = LocalFusedWorld(2)
    engines = [GPUDepthmapFusion(0) for _ in range(2)]
    ranks = [NativeFusedRank(engines[r], cams, r, 2, p, local=lw) for r in range(2)]

    def body(r):
        fr = ranks[r]
        arr = (C.c_void_p * 1)(d[r].ptr if r == 0 else None)
        k = C.c_int()
        if r == 1:
            time.sleep(0.5)  # (rank 0 is waiting in the halo all-gather by now)
        t0 = time.time()
        rc = fr._lib.gdf_fused_start(fr._h, arr, 1, C.byref(fr.pc), C.byref(k))
        return rc, fr._lib.gdf_last_error().decode(), time.time() - t0

    try:
        res = lw.run(body, timeout=120)
    finally:
        for e in engines:
            e.synchronize()
        for fr in ranks:
            fr.close()
        lw.close()
    (rc0, msg0, t0), (rc1, msg1, _) = res
    assert rc1 == -1 and "null depth map" in msg1, (rc1, msg1)
    assert rc0 == -2 and "aborted" in msg0 and "rank 1 failed" in msg0, (rc0, msg0)
    assert t0 < 30, f"rank 0 waited {t0:.1f} s"


def test_fused_start_rejects_batched_rollbuffer_frame():
    """gdf_fused_start with nframes > 1 and a move transform fails with GDF_ERR_ARG (a batch has no
    rollbuffer frame; the window's points must not be dropped silently)."""
    import ctypes as C
    import fused_ref
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt
    from ros_gpu_depthmap_fusion_amd.gdf import GDFError, GPUDepthmapFusion
    from ros_gpu_depthmap_fusion_amd.multi import LocalFusedWorld, NativeFusedRank
    build_library()
    p = small_params(0)
    cams = [synth.make_camera(0, 160, 120)]
    lw = LocalFusedWorld(1)
    eng = GPUDepthmapFusion(0)
    fr = NativeFusedRank(eng, cams, 0, 1, p, local=lw)
    try:
        d = [hiprt.DeviceArray.from_numpy(synth.dense_frame(cams[0], 0, f)) for f in range(2)]
        lidar = fused_ref.lidar_camera(80, 60)
        pc = p.to_c(lidar.T_world, lidar.T_crop, False, True, True)
        arr = (C.c_void_p * 2)(d[0].ptr, d[1].ptr)
        k = C.c_int()
        rc = fr._lib.gdf_fused_start(fr._h, arr, 2, C.byref(pc), C.byref(k))
        assert rc == -1 and b"nframes == 1" in fr._lib.gdf_last_error()
        with pytest.raises(GDFError):  # and the step's state is untouched: a valid step runs
            eng._check(rc)
        fr.finish(fr.start([d[0].ptr]))
    finally:
        fr.close()
        lw.close()
