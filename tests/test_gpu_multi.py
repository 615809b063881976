"""Multi-rank fused cloud through the HIP kernels: two processes on the one GPU of the box, gloo
collectives (host-staged), each rank a GPUDepthmapFusion with its camera (camera k-1's depth
tail as halo, gdf_add_halo_depthmap_device), the key-range partition (gdf_partition_points), the
all-to-all, gdf_voxelize_points, the occupancy-mark union: the ranks' voxel ranges concatenated
equal ONE oracle engine over both cameras bit for bit, and every rank holds its grid."""
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

from ros_gpu_depthmap_fusion_amd import synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams  # noqa: E402

pytestmark = pytest.mark.gpu
W, H, FRAMES = 160, 120, 3


def params(F):
    p = ComponentParams()
    p.flying_filter_size = F
    p.voxel_min, p.voxel_max = (-8.0, -8.0, -1.0), (8.0, 8.0, 2.0)
    p.crop_min, p.crop_max = p.voxel_min, p.voxel_max
    return p


def _rank(rank, world, port, F, out_dir):
    import torch.distributed as dist
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt, multi
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    build_library()
    p = params(F)
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    eng = GPUDepthmapFusion(0)
    fr = multi.FusedCloudRank(eng, cams, rank, world, p, dev="cpu")
    n = W * H
    for f in range(FRAMES):
        d = hiprt.DeviceArray.from_numpy(synth.dense_frame(cams[rank], rank, f))
        fr.frame(d.ptr, d.ptr + 2 * (n - fr.Lmax))
        np.save(os.path.join(out_dir, f"vox_r{rank}_f{f}.npy"), eng.downloadVoxelizedPoints()[:, :3])
        np.save(os.path.join(out_dir, f"grid_r{rank}_f{f}.npy"), eng.downloadVoxelOccupancyGrid())
        pub = multi.gather_fused_cloud(fr, root=0)  # the publishing rank's fused cloud
        if rank == 0:
            np.save(os.path.join(out_dir, f"pub_f{f}.npy"), pub.numpy()[:, :3])
        else:
            assert pub is None
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("F", [0, 4])
def test_two_rank_fused_cloud_hip(tmp_path, F):
    from oracle import OracleFusion
    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), F, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    p = params(F)
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    orc = OracleFusion(threads=4)
    for f in range(FRAMES):
        orc.clear()
        for k, c in enumerate(cams):
            orc.addDepthmap(synth.dense_frame(c, k, f), *c.intrinsics(), c.T_world, c.T_crop)
        orc.processFrame(p)
        want = orc.downloadVoxelizedPoints()[:, :3]
        got = np.concatenate([np.load(tmp_path / f"vox_r{r}_f{f}.npy") for r in range(world)])
        assert len(got) == len(want) > 0, f"frame {f}"
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"frame {f}"
        pub = np.load(tmp_path / f"pub_f{f}.npy")  # gathered on rank 0 = the single engine's
        assert np.array_equal(pub.view(np.uint32), want.view(np.uint32)), f"published frame {f}"
        for r in range(world):
            np.testing.assert_array_equal(np.load(tmp_path / f"grid_r{r}_f{f}.npy"),
                                          orc.downloadVoxelOccupancyGrid(), f"frame {f} rank {r}")


def _rank_batch(rank, world, port, F, out_dir, nf=FRAMES, mark_slices=False):
    import torch.distributed as dist
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt, multi
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    build_library()
    p = params(F)
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    eng = GPUDepthmapFusion(0)
    fr = multi.FusedCloudRank(eng, cams, rank, world, p, dev="cpu", mark_slices=mark_slices)
    n = W * H
    ds = [hiprt.DeviceArray.from_numpy(synth.dense_frame(cams[rank], rank, f)) for f in range(nf)]
    fr.batch([d.ptr for d in ds], [d.ptr + 2 * (n - fr.Lmax) for d in ds])
    vox = eng.downloadVoxelizedPoints()[:, :3]
    _, vs = eng.batch_ranges()
    for f in range(nf):
        np.save(os.path.join(out_dir, f"bvox_r{rank}_f{f}.npy"), vox[vs[f]:vs[f + 1]])
    np.save(os.path.join(out_dir, f"bgrid_r{rank}.npy"), eng.downloadVoxelOccupancyGrid())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("F,nf,slices", [(0, FRAMES, False), (4, FRAMES, False), (4, 8, False),
                                          (4, FRAMES, True), (0, 8, True)])
def test_two_rank_fused_cloud_hip_batch(tmp_path, F, nf, slices):
    """FusedCloudRank.batch: the three frames of each rank in one launch chain and one exchange
    (a halo per frame, the frames' marks in one all-gather + one batched grid update, the
    (point, frame | key) lists partitioned by key range): per frame, the ranks' voxel ranges
    concatenated equal one oracle engine over both cameras, and the grid after the batch equals
    the oracle's after the three frames - bit for bit.  8 frames: (frame | key) keys of 25 bits,
    sorted by gdf_voxelize_points in 3 passes with a 9-bit last digit.  slices: the occupancy
    union as the C++ step builds it - no compaction marks, every rank's key-range voxelize marks
    its voxels (gdf_voxelize_runs_marked) and the ranks all-gather their slices of the bitmasks -
    at world 2 through the HIP kernels (RCCL cannot put two ranks on one GPU)."""
    from oracle import OracleFusion
    world = 2
    mp.start_processes(_rank_batch, args=(world, _free_port(), F, str(tmp_path), nf, slices),
                       nprocs=world, join=True, start_method="spawn")
    p = params(F)
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    orc = OracleFusion(threads=4)
    for f in range(nf):
        orc.clear()
        for k, c in enumerate(cams):
            orc.addDepthmap(synth.dense_frame(c, k, f), *c.intrinsics(), c.T_world, c.T_crop)
        orc.processFrame(p)
        want = orc.downloadVoxelizedPoints()[:, :3]
        got = np.concatenate([np.load(tmp_path / f"bvox_r{r}_f{f}.npy") for r in range(world)])
        assert len(got) == len(want) > 0, f"frame {f}"
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"frame {f}"
    for r in range(world):
        np.testing.assert_array_equal(np.load(tmp_path / f"bgrid_r{r}.npy"),
                                      orc.downloadVoxelOccupancyGrid(), f"rank {r}")


def _rank_cfg(rank, world, port, W_, H_, frames, out_dir):
    """One rank of a C4 / C5-shaped run: launch-default parameters (F = 4, the 400x400x21 grid),
    camera `rank` at W_ x H_; saves its depth frames for the oracle and its outputs."""
    import torch.distributed as dist
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt, multi
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    build_library()
    p = ComponentParams()
    cams = [synth.make_camera(k, W_, H_) for k in range(world)]
    eng = GPUDepthmapFusion(0)
    fr = multi.FusedCloudRank(eng, cams, rank, world, p, dev="cpu")
    n = W_ * H_
    for f in range(frames):
        depth = synth.dense_frame(cams[rank], rank, f)
        np.save(os.path.join(out_dir, f"depth_r{rank}_f{f}.npy"), depth)
        d = hiprt.DeviceArray.from_numpy(depth)
        fr.frame(d.ptr, d.ptr + 2 * (n - fr.Lmax))
        np.save(os.path.join(out_dir, f"vox_r{rank}_f{f}.npy"), eng.downloadVoxelizedPoints()[:, :3])
        np.save(os.path.join(out_dir, f"grid_r{rank}_f{f}.npy"), eng.downloadVoxelOccupancyGrid())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg", ["C4", "C5"])
def test_fused_cloud_survey_configs(tmp_path, cfg):
    """SURVEY §8(d) C4 (4 x 720p, 4 ranks) and C5 (8 x 4K, 8 ranks) shapes as processes on the
    one GPU of the box (gloo, host-staged): launch-default parameters, the halo, the key-range
    all-to-all and the mark union - the ranks' voxel ranges concatenated equal ONE oracle engine
    over all cameras bit for bit, and every rank's grid equals the oracle's."""
    from oracle import OracleFusion
    world, W_, H_, frames = (4, 1280, 720, 2) if cfg == "C4" else (8, 3840, 2160, 1)
    mp.start_processes(_rank_cfg, args=(world, _free_port(), W_, H_, frames, str(tmp_path)),
                       nprocs=world, join=True, start_method="spawn")
    p = ComponentParams()
    cams = [synth.make_camera(k, W_, H_) for k in range(world)]
    orc = OracleFusion(threads=8)
    for f in range(frames):
        orc.clear()
        for k, c in enumerate(cams):
            orc.addDepthmap(np.load(tmp_path / f"depth_r{k}_f{f}.npy"), *c.intrinsics(), c.T_world,
                            c.T_crop)
        orc.processFrame(p)
        want = orc.downloadVoxelizedPoints()[:, :3]
        got = np.concatenate([np.load(tmp_path / f"vox_r{r}_f{f}.npy") for r in range(world)])
        assert len(got) == len(want) > 0, f"{cfg} frame {f}"
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"{cfg} frame {f}"
        g = orc.downloadVoxelOccupancyGrid()
        for r in range(world):
            np.testing.assert_array_equal(np.load(tmp_path / f"grid_r{r}_f{f}.npy"), g,
                                          f"{cfg} frame {f} rank {r}")


def _rank_nccl(rank, world, port, out_dir, native=False, engine_streams=False):
    """One process, RCCL (backend "nccl") at world 1: FusedCloudRank(dev="cuda") with the engine
    on torch's stream - the device collectives (all-gather of marks, all-to-all of counts and of
    the (point, key) lists, the gather of the fused cloud) over RCCL, frame by frame and per
    batch."""
    import torch
    import torch.distributed as dist
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt, multi
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    build_library()
    p = ComponentParams()
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    eng = GPUDepthmapFusion(0)
    fr = (multi.NativeFusedRank(eng, cams, rank, world, p) if native else
          multi.FusedCloudRank(eng, cams, rank, world, p, dev="cuda", engine_streams=engine_streams))
    n = W * H
    ds = [hiprt.DeviceArray.from_numpy(synth.dense_frame(cams[rank], rank, f)) for f in range(4)]
    for f in range(2):
        fr.frame(ds[f].ptr, ds[f].ptr + 2 * (n - fr.Lmax))
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, f"nvox_f{f}.npy"), eng.downloadVoxelizedPoints()[:, :3])
        np.save(os.path.join(out_dir, f"ngrid_f{f}.npy"), eng.downloadVoxelOccupancyGrid())
        np.save(os.path.join(out_dir, f"npub_f{f}.npy"),
                multi.gather_fused_cloud(fr, root=0).cpu().numpy()[:, :3])
    fr.batch([d.ptr for d in ds[2:]], [d.ptr + 2 * (n - fr.Lmax) for d in ds[2:]])
    torch.cuda.synchronize()
    vox = eng.downloadVoxelizedPoints()[:, :3]
    _, vs = eng.batch_ranges()
    for j in range(2):
        np.save(os.path.join(out_dir, f"nvox_f{2 + j}.npy"), vox[vs[j]:vs[j + 1]])
    np.save(os.path.join(out_dir, "ngrid_f3.npy"), eng.downloadVoxelOccupancyGrid())
    # teardown in dependency order: the rank (its communicators / slot tensors), then the engine
    # (its streams), then the process group - never the engine before what lives on its streams
    fr.close()
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("native,engine_streams", [(False, False), (True, False), (False, True)])
def test_rccl_fused_cloud_world1(tmp_path, native, engine_streams):
    """The RCCL branch of FusedCloudRank (dev="cuda", backend nccl) - and its C++ form
    NativeFusedRank (gdf_fused_*, RCCL from libgdf) - on the box's GPU at world 1: two frames one
    by one, then a 2-frame batch - voxel means, grids and the gathered publishing cloud equal the
    oracle bit for bit.  engine_streams: the Python rank on the ENGINE's slot streams (round 4's
    teardown SIGSEGV configuration), closed in dependency order."""
    from oracle import OracleFusion
    mp.start_processes(_rank_nccl, args=(1, _free_port(), str(tmp_path), native, engine_streams),
                       nprocs=1, join=True, start_method="spawn")
    p = ComponentParams()
    cam = synth.make_camera(0, W, H)
    orc = OracleFusion(threads=4)
    for f in range(4):
        orc.clear()
        orc.addDepthmap(synth.dense_frame(cam, 0, f), *cam.intrinsics(), cam.T_world, cam.T_crop)
        orc.processFrame(p)
        want = orc.downloadVoxelizedPoints()[:, :3]
        got = np.load(tmp_path / f"nvox_f{f}.npy")
        assert len(got) == len(want) > 0 and np.array_equal(got.view(np.uint32), want.view(np.uint32)), f
        if f < 2:
            pub = np.load(tmp_path / f"npub_f{f}.npy")
            assert np.array_equal(pub.view(np.uint32), want.view(np.uint32)), f"published {f}"
        if f != 2:
            np.testing.assert_array_equal(np.load(tmp_path / f"ngrid_f{f}.npy"),
                                          orc.downloadVoxelOccupancyGrid(), f"frame {f}")


# ---- the rollbuffer leg: point sequences on the last rank -----------------
def _rank_rb(rank, world, port, W_, H_, LW, LH, first, win, frames, out_dir, launch_defaults,
             mark_slices=False):
    """One rank of a fused run WITH the rollbuffer: the last rank ingests the point sequences of
    fused_ref.schedule (device PointCloud2 records, gdf_add_point_sequence_device) and sends its
    selected points behind its camera's (multi.FusedCloudRank.frame(move=...))."""
    import torch.distributed as dist
    import fused_ref
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt, multi
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    build_library()
    p = ComponentParams() if launch_defaults else params(4)
    p.ps_timespan = (win - 0.5) / 30.0
    cams = [synth.make_camera(k, W_, H_) for k in range(world)]
    eng = GPUDepthmapFusion(0)
    fr = multi.FusedCloudRank(eng, cams, rank, world, p, dev="cpu", mark_slices=mark_slices)
    n = W_ * H_
    lidar = fused_ref.lidar_camera(LW, LH)
    recs = None
    if fr.has_rollbuffer:
        recs = [hiprt.DeviceArray.from_numpy(fused_ref.sequence_records(lidar, k)) for k in range(2)]
    sched = fused_ref.schedule(first, frames)
    for f in range(frames):
        depth = synth.dense_frame(cams[rank], rank, f)
        move = None
        if fr.has_rollbuffer:
            for k in sched[f]:
                eng.addPointSequenceDevice(recs[k % 2].ptr, LW * LH, 16, *synth.sequence_time(k),
                                           synth.move_transform(k))
            move = (lidar.T_world, lidar.T_crop)
        d = hiprt.DeviceArray.from_numpy(depth)
        fr.frame(d.ptr, d.ptr + 2 * (n - fr.Lmax), move=move)
        np.save(os.path.join(out_dir, f"vox_r{rank}_f{f}.npy"), eng.downloadVoxelizedPoints()[:, :3])
        np.save(os.path.join(out_dir, f"grid_r{rank}_f{f}.npy"), eng.downloadVoxelOccupancyGrid())
        if fr.has_rollbuffer:
            np.save(os.path.join(out_dir, f"rb_f{f}.npy"), np.array(eng.rollbuffer_state().as_tuple()))
    dist.barrier()
    dist.destroy_process_group()


def _oracle_rb(world, W_, H_, LW, LH, first, win, frames, launch_defaults, threads):
    """The single oracle engine over all cameras + the same point sequences, per frame:
    (voxel means, u8 grid, rollbuffer state)."""
    import fused_ref
    from oracle import OracleFusion
    p = ComponentParams() if launch_defaults else params(4)
    p.ps_timespan = (win - 0.5) / 30.0
    cams = [synth.make_camera(k, W_, H_) for k in range(world)]
    lidar = fused_ref.lidar_camera(LW, LH)
    recs = [fused_ref.sequence_records(lidar, k) for k in range(2)]
    orc = OracleFusion(threads=threads)
    for f, seqs in enumerate(fused_ref.schedule(first, frames)):
        for k in seqs:
            orc.addPointSequence(recs[k % 2], *synth.sequence_time(k), synth.move_transform(k))
        orc.clear()
        for k, c in enumerate(cams):
            orc.addDepthmap(synth.dense_frame(c, k, f), *c.intrinsics(), c.T_world, c.T_crop)
        orc.processFrame(p, T_world_move=lidar.T_world, T_crop_move=lidar.T_crop)
        yield orc.downloadVoxelizedPoints()[:, :3], orc.downloadVoxelOccupancyGrid(), orc.rollbuffer_state()


@pytest.mark.parametrize("cfg", ["small", "small_slices", "C5"])
def test_fused_cloud_rollbuffer_leg(tmp_path, cfg):
    """The multi-GPU fused cloud WITH the rollbuffer on the last rank, through the HIP kernels
    (processes on the one GPU, gloo): per frame the ranks' voxel ranges concatenated equal ONE
    oracle engine over all cameras + the rollbuffer (its selected points at offset sum(P),
    fusion.cpp:1509-1581, sorted with the depth points, :1743-1756) bit for bit; every rank's grid
    and the rollbuffer rank's state equal the oracle's.  "small": 3 ranks x 160x120, F = 4,
    sequences of 80x60 points, window 3, 5 frames (rolls from frame 2).  "C5": 8 ranks x 4K at
    launch defaults + a window of 8 x 720p sequences (7.4 M selected points; frame 1 rolls the
    oldest out)."""
    if cfg in ("small", "small_slices"):
        world, W_, H_, LW, LH, first, win, frames, ld, th = 3, 160, 120, 80, 60, 2, 3, 5, False, 4
    else:
        world, W_, H_, LW, LH, first, win, frames, ld, th = 8, 3840, 2160, 1280, 720, 8, 8, 2, True, 16
    mp.start_processes(_rank_rb, args=(world, _free_port(), W_, H_, LW, LH, first, win, frames,
                                       str(tmp_path), ld, cfg == "small_slices"), nprocs=world,
                       join=True, start_method="spawn")
    for f, (want, grid, st) in enumerate(_oracle_rb(world, W_, H_, LW, LH, first, win, frames, ld, th)):
        assert st[3] > 0, f"frame {f}: rollbuffer points selected"
        assert tuple(np.load(tmp_path / f"rb_f{f}.npy").tolist()) == tuple(st), f"{cfg} frame {f} state"
        got = np.concatenate([np.load(tmp_path / f"vox_r{r}_f{f}.npy") for r in range(world)])
        assert len(got) == len(want) > 0, f"{cfg} frame {f}"
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), f"{cfg} frame {f}"
        for r in range(world):
            np.testing.assert_array_equal(np.load(tmp_path / f"grid_r{r}_f{f}.npy"), grid,
                                          f"{cfg} frame {f} rank {r}")


# ---- the pipelined RCCL path: steps in the engine's slots ----------------
def _rank_nccl_pipe(rank, world, port, out_dir, depth, rollbuffer, native=False,
                    engine_streams=False):
    """RCCL at world 1, FusedCloudRank(depth=3).run(): step i+1 starts (compaction, marks, grid
    update, partition, split sizes) before step i's points all-to-all and voxelize - on the
    slots' own streams, the points on their own communicator.  Batches of 2 frames, or (with the
    rollbuffer) single frames each carrying one new point sequence."""
    import torch
    import torch.distributed as dist
    import fused_ref
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt, multi
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    build_library()
    p = ComponentParams()
    p.ps_timespan = 2.5 / 30.0
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    eng = GPUDepthmapFusion(0)
    fr = (multi.NativeFusedRank(eng, cams, rank, world, p, depth=depth) if native else
          multi.FusedCloudRank(eng, cams, rank, world, p, dev="cuda", depth=depth,
                               engine_streams=engine_streams))
    n = W * H
    B = 1 if rollbuffer else 2
    steps = 6
    ds = [hiprt.DeviceArray.from_numpy(synth.dense_frame(cams[rank], rank, f)) for f in range(B * steps)]
    lidar = fused_ref.lidar_camera(80, 60)
    recs = [hiprt.DeviceArray.from_numpy(fused_ref.sequence_records(lidar, k)) for k in range(2)]

    def move(i):
        # (the rollbuffer is engine state, not slot state: frame i-1's state is the one in place
        # right before step i starts - the steps after it may already have run when i-1 finishes)
        if i:
            np.save(os.path.join(out_dir, f"prb_f{i - 1}.npy"),
                    np.array(eng.rollbuffer_state().as_tuple()))
        eng.addPointSequenceDevice(recs[i % 2].ptr, 80 * 60, 16, *synth.sequence_time(i),
                                   synth.move_transform(i))
        return (lidar.T_world, lidar.T_crop)

    def done(i):
        torch.cuda.synchronize()
        vox = eng.downloadVoxelizedPoints()[:, :3]
        _, vs = eng.batch_ranges()
        for j in range(B):
            np.save(os.path.join(out_dir, f"pvox_f{B * i + j}.npy"), vox[vs[j]:vs[j + 1]])

    fr.run(steps, lambda i: [ds[B * i + j].ptr for j in range(B)],
           lambda i: [ds[B * i + j].ptr + 2 * (n - fr.Lmax) for j in range(B)],
           move_of=move if rollbuffer else None, on_finish=done)
    torch.cuda.synchronize()
    if rollbuffer:
        np.save(os.path.join(out_dir, f"prb_f{steps - 1}.npy"), np.array(eng.rollbuffer_state().as_tuple()))
    np.save(os.path.join(out_dir, "pgrid.npy"), eng.downloadVoxelOccupancyGrid())
    if native and not rollbuffer:  # and the C++ loop (gdf_fused_run) over the same frames
        fr.run_stream([d.ptr for d in ds], 0, steps, B)
        torch.cuda.synchronize()
        np.save(os.path.join(out_dir, "pvox_run_last.npy"), eng.downloadVoxelizedPoints()[:, :3])
    fr.close()
    eng.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("rollbuffer,native,engine_streams",
                         [(False, False, False), (True, False, False), (False, True, False),
                          (True, True, False), (False, False, True), (True, False, True)])
def test_rccl_pipelined_fused_cloud_world1(tmp_path, rollbuffer, native, engine_streams):
    """The pipelined fused path (three steps in flight on the engine's slots, the points
    all-to-all on a second communicator) under RCCL at world 1: every frame's voxel means, the
    final grid and (rollbuffer) the rollbuffer state after every frame equal the oracle's bit for
    bit."""
    import fused_ref
    from oracle import OracleFusion
    mp.start_processes(_rank_nccl_pipe, args=(1, _free_port(), str(tmp_path), 3, rollbuffer, native,
                                              engine_streams),
                       nprocs=1, join=True, start_method="spawn")
    p = ComponentParams()
    p.ps_timespan = 2.5 / 30.0
    cam = synth.make_camera(0, W, H)
    lidar = fused_ref.lidar_camera(80, 60)
    recs = [fused_ref.sequence_records(lidar, k) for k in range(2)]
    orc = OracleFusion(threads=4)
    nf = 6 if rollbuffer else 12
    for f in range(nf):
        orc.clear()
        orc.addDepthmap(synth.dense_frame(cam, 0, f), *cam.intrinsics(), cam.T_world, cam.T_crop)
        if rollbuffer:
            orc.addPointSequence(recs[f % 2], *synth.sequence_time(f), synth.move_transform(f))
            orc.processFrame(p, T_world_move=lidar.T_world, T_crop_move=lidar.T_crop)
            assert tuple(np.load(tmp_path / f"prb_f{f}.npy").tolist()) == tuple(orc.rollbuffer_state())
        else:
            orc.processFrame(p)
        want = orc.downloadVoxelizedPoints()[:, :3]
        got = np.load(tmp_path / f"pvox_f{f}.npy")
        assert len(got) == len(want) > 0 and np.array_equal(got.view(np.uint32), want.view(np.uint32)), f
    np.testing.assert_array_equal(np.load(tmp_path / "pgrid.npy"), orc.downloadVoxelOccupancyGrid())
    if native and not rollbuffer:  # gdf_fused_run over the same frames: its last step's
        B = 2  # voxels = the last step's (voxel means depend on the step's frames only)
        last = np.load(tmp_path / "pvox_run_last.npy")
        want = np.concatenate([np.load(tmp_path / f"pvox_f{f}.npy") for f in range(nf - B, nf)])
        assert np.array_equal(last.view(np.uint32), want.view(np.uint32))
