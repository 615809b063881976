"""Multi-rank fused voxel cloud on CPU (torch.distributed gloo, world 2 and 3): every rank plays
one camera (the oracle as its engine, camera k-1's tail as halo), the compacted (point, key)
lists are all-to-all'ed by voxel-key range (multi.exchange_points), each rank voxelizes its range;
the concatenated ranges equal ONE engine over all cameras (src/gpu_depthmap_fusion.cpp:1743-1756)
bit for bit - at F = 0 and at F = 4, where camera k's top rows read camera k-1 -
and the occupancy union gives every rank the single engine's grid.  With the rollbuffer leg the
last rank also ingests point sequences (filter, insert, roll, select, transform, crop) and sends
its selected points after its camera's: the fused cloud is the single engine's over all cameras
AND the rollbuffer (fusion.cpp:1509-1581: the selection sits at offset sum(P), after every
camera)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

from ros_gpu_depthmap_fusion_amd import multi, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams  # noqa: E402

W, H, FRAMES, LIFETIME = 96, 72, 2, 3


def params(F):
    p = ComponentParams()
    p.flying_filter_size = F
    p.occupancy_lifetime = LIFETIME
    p.voxel_min, p.voxel_max = (-8.0, -8.0, -1.0), (8.0, 8.0, 2.0)
    p.crop_min, p.crop_max = p.voxel_min, p.voxel_max
    return p


RB_FRAMES, RB_FIRST, RB_WIN = 4, 2, 3  # rollbuffer leg: frames, sequences at frame 0, window


def rb_params(F):
    p = params(F)
    p.ps_timespan = (RB_WIN - 0.5) / 30.0  # the window keeps RB_WIN sequences
    return p


def _rank(rank, world, port, F, out_dir, rollbuffer=False):
    import torch
    import torch.distributed as dist
    import fused_ref
    from oracle import OracleFusion
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = rb_params(F) if rollbuffer else params(F)
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    orc = OracleFusion()
    hist = None
    lidar = fused_ref.lidar_camera(W // 2, H // 2)
    frames = RB_FRAMES if rollbuffer else FRAMES
    sched = fused_ref.schedule(RB_FIRST, frames)
    for f in range(frames):
        move = None
        if rollbuffer and rank == world - 1:  # the rollbuffer rank (multi.FusedCloudRank)
            for k in sched[f]:
                orc.addPointSequence(fused_ref.sequence_records(lidar, k), *synth.sequence_time(k),
                                     synth.move_transform(k))
            move = (lidar.T_world, lidar.T_crop)
        pts, keys = fused_ref.rank_points(orc, cams, rank, f, p, halo=F > 0, move=move)
        if move is not None:
            np.save(os.path.join(out_dir, f"rb_f{f}.npy"), np.array(orc.rollbuffer_state()))
            np.save(os.path.join(out_dir, f"rbsel_f{f}.npy"),
                    np.array([orc.rollbuffer_state()[3], len(keys)]))
        ncells = int(np.prod(orc.grid_size()))
        sp, sk, counts = fused_ref.partition(pts, keys, world, ncells)
        rp, rk, rc = multi.exchange_points(torch.from_numpy(np.ascontiguousarray(sp)),
                                           torch.from_numpy(sk.view(np.int32).copy()), counts)
        keys_r = rk.numpy().view(np.uint32)
        lo = -(-rank * ncells // world)
        hi = -(-(rank + 1) * ncells // world)
        assert ((keys_r >= lo) & (keys_r < hi)).all()  # this rank's key range only
        vox = fused_ref.voxelize(rp.numpy(), keys_r)
        marks = np.zeros(ncells, bool)
        marks[keys] = True
        merged = multi.all_gather_or(torch.from_numpy(multi.pack_marks(marks).view(np.int32).copy()))
        union = multi.unpack_marks(merged.numpy().view(np.uint32), ncells)
        hist = np.zeros(ncells, np.uint32) if hist is None else hist
        hist = multi.historic_update(hist, union, LIFETIME)
        np.save(os.path.join(out_dir, f"vox_r{rank}_f{f}.npy"), vox)
        np.save(os.path.join(out_dir, f"grid_r{rank}_f{f}.npy"), hist)
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,F", [(2, 4), (3, 4)])
def test_fused_cloud_with_rollbuffer_equals_single_engine(tmp_path, world, F):
    """The rollbuffer leg: the last rank ingests the point sequences and
    appends its selected points behind its camera's; per frame the ranks' voxel ranges
    concatenated equal ONE engine over all cameras + the rollbuffer bit for bit, every rank's grid
    equals its grid, and the rollbuffer rank's state equals its state (frames 2 and 3 roll)."""
    import fused_ref
    from oracle import OracleFusion
    mp.start_processes(_rank, args=(world, _free_port(), F, str(tmp_path), True), nprocs=world,
                       join=True, start_method="spawn")
    p = rb_params(F)
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    lidar = fused_ref.lidar_camera(W // 2, H // 2)
    sched = fused_ref.schedule(RB_FIRST, RB_FRAMES)
    orc = OracleFusion()
    for f in range(RB_FRAMES):
        for k in sched[f]:
            orc.addPointSequence(fused_ref.sequence_records(lidar, k), *synth.sequence_time(k),
                                 synth.move_transform(k))
        orc.clear()
        for k, c in enumerate(cams):
            orc.addDepthmap(synth.dense_frame(c, k, f), *c.intrinsics(), c.T_world, c.T_crop)
        orc.processFrame(p, T_world_move=lidar.T_world, T_crop_move=lidar.T_crop)
        st = orc.rollbuffer_state()
        assert st[3] > 0, "the frame selected rollbuffer points"
        assert tuple(np.load(tmp_path / f"rb_f{f}.npy").tolist()) == tuple(st), f"frame {f} state"
        sel, kept = np.load(tmp_path / f"rbsel_f{f}.npy").tolist()
        assert kept > 0
        want = orc.downloadVoxelizedPoints()[:, :3]
        got = np.concatenate([np.load(tmp_path / f"vox_r{r}_f{f}.npy") for r in range(world)])
        assert len(got) == len(want) > 0, f"frame {f}"
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"frame {f}"
        g = orc.historic_grid().reshape(-1)
        for r in range(world):
            np.testing.assert_array_equal(np.load(tmp_path / f"grid_r{r}_f{f}.npy"), g)
    # the rollbuffer actually moved the result: without it the fused cloud differs
    orc2 = OracleFusion()
    orc2.clear()
    for k, c in enumerate(cams):
        orc2.addDepthmap(synth.dense_frame(c, k, RB_FRAMES - 1), *c.intrinsics(), c.T_world, c.T_crop)
    orc2.processFrame(p)
    assert len(orc2.downloadVoxelizedPoints()) != len(want) or not np.array_equal(
        orc2.downloadVoxelizedPoints()[:, :3].view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("world,F", [(2, 0), (2, 4), (3, 4)])
def test_fused_cloud_equals_single_engine(tmp_path, world, F):
    from oracle import OracleFusion
    mp.start_processes(_rank, args=(world, _free_port(), F, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    p = params(F)
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    orc = OracleFusion()
    for f in range(FRAMES):
        orc.clear()
        for k, c in enumerate(cams):
            orc.addDepthmap(synth.dense_frame(c, k, f), *c.intrinsics(), c.T_world, c.T_crop)
        orc.processFrame(p)
        want = orc.downloadVoxelizedPoints()[:, :3]
        got = np.concatenate([np.load(tmp_path / f"vox_r{r}_f{f}.npy") for r in range(world)])
        assert len(got) == len(want) > 0, f"frame {f}"
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"frame {f}"
        g = orc.historic_grid().reshape(-1)
        for r in range(world):
            np.testing.assert_array_equal(np.load(tmp_path / f"grid_r{r}_f{f}.npy"), g)


def test_key_range_partition_rule():
    """part_of_keys: contiguous ascending ranges of whole 32-key mark words covering every key."""
    ncells = 3_360_000
    keys = np.arange(0, ncells, 997, dtype=np.uint32)
    for n in (1, 2, 3, 7, 8, 16):
        part = multi.part_of_keys(keys, n, ncells)
        assert part.min() == 0 and part.max() == n - 1 and (np.diff(part) >= 0).all()
        S = multi.part_slice_words(n, ncells)
        assert S * n * 32 >= ncells
        word = np.arange((ncells + 31) // 32, dtype=np.uint32)
        # every key of a word has the word's part, and part j = words [j S, (j + 1) S)
        for off in (0, 17, 31):
            k = np.minimum(word * 32 + off, ncells - 1).astype(np.uint32)
            pk = multi.part_of_keys(k, n, ncells)
            np.testing.assert_array_equal(pk[k // 32 == word], np.minimum(word // S, n - 1)[k // 32 == word])
