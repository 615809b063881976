"""Multi-rank exchange of the shared occupancy grid on CPU (torch.distributed gloo, world size 2).

Each rank plays one camera of the one-camera-per-GPU layout: it computes its
frame's occupancy marks (here with the CPU oracle), packs them in the k_export_marks bit layout,
the ranks all-gather and OR them (ros_gpu_depthmap_fusion_amd.multi), and each rank runs the
historic-grid update.  Checked: both ranks hold identical grids every frame, equal to a single
engine that processed both cameras (flying filter off, so no cross-camera border reads), and to
the union of per-camera results with the launch-default filter ("independent cameras" mode)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

from ros_gpu_depthmap_fusion_amd import multi, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams  # noqa: E402

W, H, FRAMES, LIFETIME = 96, 72, 3, 3


def params(flying: int) -> ComponentParams:
    p = ComponentParams()
    p.flying_filter_size = flying
    p.occupancy_lifetime = LIFETIME
    p.voxel_min, p.voxel_max = (-8.0, -8.0, -1.0), (8.0, 8.0, 2.0)
    p.crop_min, p.crop_max = p.voxel_min, p.voxel_max
    return p


def frame_marks(orc, cam, k, f, p):
    from oracle import OracleFusion  # noqa: F401
    orc.clear()
    orc.addDepthmap(synth.depth_frame(cam, k, f), *cam.intrinsics(), cam.T_world, cam.T_crop)
    orc.processFrame(p)
    gs = orc.grid_size()
    marks = np.zeros(int(np.prod(gs)), bool)
    marks[orc.downloadVoxelCoords()] = True
    return marks


def _rank(rank, world, port, flying, out_dir):
    import torch
    import torch.distributed as dist
    from oracle import OracleFusion
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    p = params(flying)
    cam = synth.make_camera(rank, W, H)
    orc = OracleFusion()
    hist = None
    grids = []
    for f in range(FRAMES):
        marks = frame_marks(orc, cam, rank, f, p)
        words = torch.from_numpy(multi.pack_marks(marks).view(np.int32).copy())
        merged = multi.all_gather_or(words)
        union = multi.unpack_marks(merged.numpy().view(np.uint32), marks.size)
        hist = np.zeros(marks.size, np.uint32) if hist is None else hist
        hist = multi.historic_update(hist, union, LIFETIME)
        grids.append(hist.copy())
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), np.stack(grids))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_pack_unpack_roundtrip():
    rng = np.random.default_rng(3)
    for n in (1, 31, 32, 33, 1000, 3_360_000):
        m = rng.random(n) < 0.3
        w = multi.pack_marks(m)
        assert w.size == multi.words_for(n)
        np.testing.assert_array_equal(multi.unpack_marks(w, n), m)
        idx = np.flatnonzero(m)[:50]
        assert all((w[i // 32] >> (i % 32)) & 1 for i in idx)  # k_export_marks bit layout


@pytest.mark.parametrize("flying", [0, 4])
def test_two_rank_occupancy_union(tmp_path, flying):
    from oracle import OracleFusion
    world = 2
    mp.start_processes(_rank, args=(world, _free_port(), flying, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    g0 = np.load(tmp_path / "rank0.npy")
    g1 = np.load(tmp_path / "rank1.npy")
    np.testing.assert_array_equal(g0, g1)  # every rank holds the same shared grid
    p = params(flying)
    cams = [synth.make_camera(k, W, H) for k in range(world)]
    if flying == 0:
        # one engine with both cameras concatenated (no cross-camera border reads at F = 0)
        orc = OracleFusion()
        for f in range(FRAMES):
            orc.clear()
            for k, c in enumerate(cams):
                orc.addDepthmap(synth.depth_frame(c, k, f), *c.intrinsics(), c.T_world, c.T_crop)
            orc.processFrame(p)
            np.testing.assert_array_equal(g0[f], orc.historic_grid().reshape(-1),
                                          err_msg=f"frame {f}")
    else:
        # independent cameras: union of the per-camera marks
        engines = [OracleFusion() for _ in cams]
        hist = np.zeros(g0.shape[1], np.uint32)
        for f in range(FRAMES):
            u = np.zeros(g0.shape[1], bool)
            for k, (c, o) in enumerate(zip(cams, engines)):
                u |= frame_marks(o, c, k, f, p)
            hist = multi.historic_update(hist, u, LIFETIME)
            np.testing.assert_array_equal(g0[f], hist, err_msg=f"frame {f}")
