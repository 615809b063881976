"""GPU object-segmentation front end (include/gdf_segment.h) bit for bit against the oracle
(oracle/seg_oracle.c): labels, num_labels, stats, centroids, labelsToContours, contours, layer
connections, merged labels — on random blob grids (odd sizes, tile-crossing components), the
launch-default 400 x 400 x 21 grid, a layer too large for LDS (global-scratch contour path),
empty / full layers, and the engine's own occupancy grid after dense frames."""
import numpy as np
import pytest

import oracle as oracle_mod
from conftest import gpu_available
from test_segment_kat import assert_same, blobs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def seg():
    if not gpu_available():
        pytest.fail("-m gpu test run without a visible GPU")
    from ros_gpu_depthmap_fusion_amd import build_library
    from ros_gpu_depthmap_fusion_amd.gdf import Segmenter
    build_library()
    s = Segmenter(0)
    yield s
    s.close()


def gpu_front(seg, g):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(g, np.uint8)).cuda()
    torch.cuda.synchronize()
    L, H, W = g.shape
    seg.label_layers(t.data_ptr(), W, H, L)
    r = seg.results()
    del t
    return r


@pytest.mark.parametrize("shape,density,seed", [
    ((1, 9, 11), 0.45, 1), ((2, 33, 35), 0.5, 2), ((3, 70, 64), 0.4, 3), ((2, 129, 97), 0.55, 4),
    ((1, 1, 1), 0.5, 5), ((2, 1, 77), 0.5, 6), ((2, 64, 1), 0.5, 7), ((3, 200, 150), 0.6, 8)])
def test_random_blobs_bit_exact(seg, shape, density, seed):
    rng = np.random.default_rng(seed)
    for smooth in (False, True):
        g = blobs(rng, *shape, density, smooth)
        assert_same(gpu_front(seg, g), oracle_mod.object_segmentation_front(g))


@pytest.mark.parametrize("density", [0.02, 0.35])
def test_launch_default_grid(seg, density):
    rng = np.random.default_rng(int(density * 100))
    g = blobs(rng, 21, 400, 400, density, smooth=density > 0.1)
    r = gpu_front(seg, g)
    o = oracle_mod.object_segmentation_front(g)
    assert_same(r, o)
    assert int(r["contours_per_layer"].sum()) > 21


def test_layer_over_lds_uses_global_scratch(seg):
    rng = np.random.default_rng(9)
    g = blobs(rng, 2, 420, 500, 0.4)  # (500 + 2) x (420 + 2) bytes > 160 KiB of LDS
    assert_same(gpu_front(seg, g), oracle_mod.object_segmentation_front(g))


def test_empty_and_full_layers(seg):
    g = np.zeros((3, 40, 30), np.uint8)
    g[1] = 7
    g[2, 5:9, 5:9] = 1
    assert_same(gpu_front(seg, g), oracle_mod.object_segmentation_front(g))


def test_engine_occupancy_grid(seg, gpu_engine_factory):
    from ros_gpu_depthmap_fusion_amd import synth
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams
    eng = gpu_engine_factory(0)
    p = ComponentParams()
    for f in range(3):
        eng.clear()
        for k in range(2):
            cam = synth.make_camera(k, 320, 240)
            eng.addDepthmap(synth.dense_frame(cam, f, k), *cam.intrinsics(), cam.T_world,
                            cam.T_crop)
        eng.processFrame(p)
    grid = eng.downloadVoxelOccupancyGrid()
    gs, _ = eng.grid_size()
    seg.label_engine_grid(eng)
    r = seg.results()
    o = oracle_mod.object_segmentation_front(grid.reshape(gs[2], gs[1], gs[0]))
    assert_same(r, o)
    assert r["num_objects"] > 2
    assert_objects(seg, o, p.voxel_min, p.voxel_size)


def assert_objects(seg, r, lower=(-10, -20, -1), cs=(0.1, 0.1, 0.12)):
    go, gc = seg.create_objects(lower, cs)
    oo, oc = oracle_mod.create_cc_objects(r, lower, cs)
    assert np.array_equal(gc, oc)
    for k in oo:
        assert np.array_equal(np.asarray(go[k]).reshape(oo[k].shape), oo[k]), k


@pytest.mark.parametrize("shape,density,seed", [((3, 70, 64), 0.4, 3), ((21, 120, 100), 0.35, 12)])
def test_cc_objects_match_oracle(seg, shape, density, seed):
    rng = np.random.default_rng(seed)
    g = blobs(rng, *shape, density)
    r = gpu_front(seg, g)
    assert_objects(seg, oracle_mod.object_segmentation_front(g))
    assert r["num_objects"] > 3


def test_errors_fail_loudly(seg):
    import torch
    from ros_gpu_depthmap_fusion_amd.gdf import GDFError
    # more than 65535 components in a layer overflow the reference's CV_16U labels
    g = np.zeros((1, 600, 600), np.uint8)
    g[0, ::2, ::2] = 1  # 90 000 isolated cells
    t = torch.from_numpy(g).cuda()
    torch.cuda.synchronize()
    with pytest.raises(GDFError, match="65535"):
        seg.label_layers(t.data_ptr(), 600, 600, 1)
    with pytest.raises(GDFError):
        seg.counts()  # no result after a failed call
    with pytest.raises(GDFError):
        seg.label_layers(t.data_ptr(), 0, 600, 1)
    # the segmenter stays usable
    g2 = np.zeros((2, 30, 20), np.uint8)
    g2[:, 3:9, 4:7] = 5
    assert_same(gpu_front(seg, g2), oracle_mod.object_segmentation_front(g2))
