"""GPU tests added in round 5 (bar: bit-exact against the oracle, as test_gpu_parity.py).

* gdf_download_frame's views stay intact across later frames until the next gdf_download_frame:
  the k_download prefetch of the following frames writes the OTHER set of pinned mirrors, also
  when a larger frame makes that set grow (include/gdf.h contract).
* k_frame_sort, the per-frame LDS sort of a batch's runs: resident and chunked forms, empty,
  sparse and fine-voxel frames, against the oracle frame by frame.
"""
import os

import numpy as np
import pytest

from oracle import OracleFusion
from ros_gpu_depthmap_fusion_amd import synth
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def Engine(gpu_engine_factory):
    return gpu_engine_factory


def cam_args(cam, depth):
    return (depth, *cam.intrinsics(), cam.T_world, cam.T_crop)


def test_download_frame_views_survive_later_frames(Engine):
    """Frame sizes small -> small -> LARGE -> large: the views of frame 1 (held like a publisher
    holds a message) are unchanged after frames 2 and 3 were processed (their prefetch wrote the
    other mirror set, which grew for the larger frames); frame 3's download equals the oracle's,
    and frame 1's views are only replaced by that download."""
    p = ComponentParams()
    small, large = synth.make_camera(0, 160, 120), synth.make_camera(0, 640, 480)
    gpu, orc = Engine(), OracleFusion(threads=8)

    def frame(cam, f):
        for e in (gpu, orc):
            e.clear()
            e.addDepthmap(*cam_args(cam, synth.dense_frame(cam, 0, f)))
            e.processFrame(p)

    frame(small, 0)
    gpu.download_frame()  # (turns the k_download prefetch on)
    frame(small, 1)
    held = gpu.download_frame()
    kept = {k: v.copy() for k, v in held.items()}
    want1 = orc.downloadVoxelizedPoints()[:, :3]
    assert np.array_equal(held["voxelized"][:, :3].view(np.uint32), want1.view(np.uint32))
    frame(large, 2)
    frame(large, 3)
    gpu.synchronize()
    for k in ("points", "voxel_coords", "voxelized"):
        assert np.array_equal(held[k].view(np.uint8), kept[k].view(np.uint8)), k
    d = gpu.download_frame()
    assert np.array_equal(d["points"].view(np.uint32), orc.downloadPoints().view(np.uint32))
    assert np.array_equal(d["voxel_coords"], orc.downloadVoxelCoords())
    assert np.array_equal(d["voxelized"][:, :3].view(np.uint32),
                          orc.downloadVoxelizedPoints()[:, :3].view(np.uint32))
    assert np.array_equal(d["occupancy"], orc.downloadVoxelOccupancyGrid())
    assert len(d["points"]) > len(kept["points"])


def engine_with(Engine, **env):
    """An engine created with the given GDF_* environment knobs (read at creation)."""
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        return Engine()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def batch_matches_oracle(gpu, orc, cam, frames, tag, p=None):
    """One batch of `frames` on the engine, frame by frame on the oracle (which holds the same
    grid history as the engine)."""
    p = p or ComponentParams()
    gpu.clear()
    for j, d in enumerate(frames):
        if j:
            gpu.nextFrameInBatch()
        gpu.addDepthmap(*cam_args(cam, d))
    gpu.processFrame(p)
    pts, keys, vox = gpu.downloadPoints(), gpu.downloadVoxelCoords(), gpu.downloadVoxelizedPoints()
    ps, vs = gpu.batch_ranges()
    for j, d in enumerate(frames):
        orc.clear()
        orc.addDepthmap(*cam_args(cam, d))
        orc.processFrame(p)
        assert np.array_equal(pts[ps[j]:ps[j + 1]].view(np.uint32),
                              orc.downloadPoints().view(np.uint32)), (tag, j)
        assert np.array_equal(keys[ps[j]:ps[j + 1]], orc.downloadVoxelCoords()), (tag, j)
        w = orc.downloadVoxelizedPoints()
        assert np.array_equal(vox[vs[j]:vs[j + 1], :3].view(np.uint32), w[:, :3].view(np.uint32)), (tag, j)
        assert np.array_equal(vox[vs[j]:vs[j + 1], 3].view(np.uint32), w[:, 3].view(np.uint32)), (tag, j)
        assert np.array_equal(gpu.downloadBatchVoxelOccupancyGrid(j), orc.downloadVoxelOccupancyGrid()), (tag, j)


@pytest.mark.parametrize("knobs", [{}, {"GDF_NO_PACK_RUNS": "1"}])
def test_mixed_batch_matches_oracle(Engine, knobs):
    """A VGA batch of a dense frame, an empty one, a noise frame (the flying filter leaves few
    points), two dense frames and a half-empty one, then 3 cm voxels in a smaller box (24-bit voxel
    keys: more runs per frame), with the runs' lengths packed into the sort keys and without -
    every frame's points, keys, voxel sums and grid equal the oracle's frame-by-frame results."""
    cam = synth.make_camera(0, 640, 480)
    dense = [synth.dense_frame(cam, 0, f) for f in range(4)]
    half = dense[3].copy()
    half[:, : cam.width // 2] = 0
    frames = [dense[0], np.zeros_like(dense[0]), synth.uniform_frame(cam, 0, 1), dense[1], dense[2], half]
    gpu, orc = engine_with(Engine, **knobs), OracleFusion(threads=16)
    batch_matches_oracle(gpu, orc, cam, frames, (knobs, "mixed"))
    batch_matches_oracle(gpu, orc, cam, dense[1:] + dense[:1], (knobs, "again"))
    fine = ComponentParams(voxel_min=(0.0, -5.0, -1.0), voxel_max=(10.0, 5.0, 1.5),
                           voxel_size=(0.03, 0.03, 0.03))
    batch_matches_oracle(engine_with(Engine, **knobs), OracleFusion(threads=16), cam, dense,
                         (knobs, "fine"), fine)
