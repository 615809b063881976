"""GPU tests added in round 5 (bar: bit-exact against the oracle, as test_gpu_parity.py).

* gdf_download_frame's views stay intact across later frames until the next gdf_download_frame:
  the k_download prefetch of the following frames writes the OTHER set of pinned mirrors, also
  when a larger frame makes that set grow (include/gdf.h contract).
"""
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
