"""Segmentation front end: the C oracle (oracle/seg_oracle.c) against
hand-computed known answers, an independent Python restatement (tests/seg_ref.py) and scipy's
labelling.  OpenCV is absent, so these pin the restated semantics, not OpenCV itself
(parity unpinned)."""
import numpy as np
import pytest
from scipy import ndimage

import seg_ref
import oracle as oracle_mod

INT_MAX, INT_MIN = 2**31 - 1, -(2**31)


def front(grid):
    return oracle_mod.object_segmentation_front(np.asarray(grid, np.uint8))


def assert_same(a: dict, b: dict, keys=None):
    for k in keys or a.keys():
        x, y = np.asarray(a[k]), np.asarray(b[k])
        if k == "centroids":
            assert x.shape == y.shape, k
            assert np.array_equal(np.isnan(x), np.isnan(y)), k
            assert np.array_equal(np.nan_to_num(x), np.nan_to_num(y)), k
        else:
            assert x.shape == y.shape and np.array_equal(x, y), (k, x, y)


def blobs(rng, L, H, W, density, smooth=True):
    g = rng.random((L, H, W))
    if smooth:
        g = ndimage.uniform_filter(g, size=(1, 3, 3))
    return ((g < density) * rng.integers(1, 11, (L, H, W))).astype(np.uint8)


def test_square_contour_starts_top_left_and_runs_down_the_left_side():
    g = np.zeros((1, 6, 6), np.uint8)
    g[0, 1:4, 1:4] = 3
    r = front(g)
    assert r["contour_points"].tolist() == [[1, 1], [1, 2], [1, 3], [2, 3], [3, 3], [3, 2],
                                            [3, 1], [2, 1]]
    assert r["stats"].tolist() == [[0, 0, 6, 6, 27], [1, 1, 3, 3, 9]]
    assert r["centroids"][1].tolist() == [2.0, 2.0]
    assert r["labels_to_contours"].tolist() == [-1, 0]


def test_labels_follow_first_2x2_block_not_first_pixel():
    # component A starts at (x=0, y=1), B at (x=10, y=0): both in block row 0, A's block first
    g = np.zeros((1, 4, 12), np.uint8)
    g[0, 1, 0] = 1
    g[0, 0, 10] = 1
    r = front(g)
    assert r["labels"][0, 1, 0] == 1 and r["labels"][0, 0, 10] == 2
    # findContours: B discovered first (row 0), returned last
    assert r["contour_points"].tolist() == [[0, 1], [10, 0]]
    assert r["labels_to_contours"].tolist() == [-1, 0, 1]


def test_external_contours_skip_components_inside_holes():
    g = np.zeros((1, 9, 9), np.uint8)
    g[0, 1:8, 1:8] = 1
    g[0, 2:7, 2:7] = 0
    g[0, 4, 4] = 1  # inside the ring's hole
    r = front(g)
    assert r["num_labels"].tolist() == [3]
    assert r["contours_per_layer"].tolist() == [1] and r["contour_sizes"].tolist() == [24]
    assert r["labels_to_contours"].tolist() == [-1, 0, -1]


def test_single_pixel_and_image_border_components():
    g = np.zeros((1, 5, 7), np.uint8)
    g[0, 0, 0] = 1      # corner pixel
    g[0, 4, 3:7] = 2    # bottom row run to the right border
    g[0, 2, 3] = 9      # isolated pixel
    r = front(g)
    assert r["contour_sizes"].tolist()[::-1][0] == 1  # discovered first: the corner
    pts = r["contour_points"].tolist()
    assert [0, 0] in pts and [3, 2] in pts and [6, 4] in pts
    assert_same(r, seg_ref.front_end(g))


def test_full_layer_leaves_an_empty_background_label():
    g = np.ones((2, 4, 5), np.uint8)
    r = front(g)
    assert r["num_labels"].tolist() == [2, 2]
    bg = r["stats"][0].tolist()
    assert bg[0] == INT_MAX and bg[1] == INT_MAX and bg[4] == 0
    assert bg[2] == np.int32(np.uint32((INT_MIN - INT_MAX + 1) % 2**32).astype(np.int32))
    assert np.isnan(r["centroids"][0]).all()
    # the two empty background labels are never connected: they stay separate objects
    assert r["merged"].tolist() == [0, 1, 2, 1] and r["num_objects"] == 3
    assert_same(r, seg_ref.front_end(g))


@pytest.mark.parametrize("shape,density,seed", [
    ((1, 9, 11), 0.45, 1), ((2, 16, 16), 0.5, 2), ((3, 17, 23), 0.4, 3), ((2, 31, 8), 0.55, 4),
    ((4, 12, 12), 0.6, 5), ((2, 20, 19), 0.3, 6)])
def test_oracle_equals_python_restatement(shape, density, seed):
    rng = np.random.default_rng(seed)
    for smooth in (False, True):
        g = blobs(rng, *shape, density, smooth)
        assert_same(front(g), seg_ref.front_end(g))


def test_partition_bboxes_and_centroids_against_scipy():
    rng = np.random.default_rng(7)
    g = blobs(rng, 3, 64, 57, 0.45)
    r = front(g)
    st0 = 0
    for z in range(3):
        lab, n = ndimage.label(g[z] > 0, structure=np.ones((3, 3)))
        L = r["labels"][z].astype(np.int64)
        assert r["num_labels"][z] == n + 1
        # same partition: a bijection between scipy's labels and ours
        pairs = set(zip(lab.ravel().tolist(), L.ravel().tolist()))
        assert len(pairs) == n + 1
        nl = int(r["num_labels"][z])
        st = r["stats"][st0:st0 + nl]
        ce = r["centroids"][st0:st0 + nl]
        for l in range(nl):
            ys, xs = np.nonzero(L == l)
            assert st[l].tolist() == [xs.min(), ys.min(), xs.max() - xs.min() + 1,
                                      ys.max() - ys.min() + 1, len(xs)]
            assert ce[l].tolist() == [xs.sum() / len(xs), ys.sum() / len(xs)]
        st0 += nl


def test_contours_are_borders_of_external_components():
    rng = np.random.default_rng(11)
    g = blobs(rng, 2, 48, 40, 0.45)
    r = front(g)
    q = c = 0
    for z in range(2):
        lab = r["labels"][z]
        n = int(r["contours_per_layer"][z])
        starts = []
        for j in range(n):
            k = int(r["contour_sizes"][c + j])
            pts = r["contour_points"][q:q + k]
            q += k
            l0 = lab[pts[0, 1], pts[0, 0]]
            assert l0 > 0 and (lab[pts[:, 1], pts[:, 0]] == l0).all()
            ys, xs = np.nonzero(lab == l0)
            first = np.lexsort((xs, ys))[0]
            assert (pts[0] == [xs[first], ys[first]]).all()  # the component's first raster pixel
            starts.append((int(pts[0, 1]), int(pts[0, 0])))
        assert starts == sorted(starts, reverse=True)      # reverse discovery (raster) order
        c += n


def test_connections_and_merge_across_layers():
    g = np.zeros((3, 6, 6), np.uint8)
    g[0, 0:2, 0:2] = 1   # object A in layer 0 ...
    g[1, 1:3, 1:3] = 1   # ... overlaps layer 1's blob
    g[2, 5, 5] = 1       # unconnected blob in layer 2
    g[0, 4:6, 4:6] = 1   # object B only in layer 0
    r = front(g)
    assert r["num_labels"].tolist() == [3, 2, 2]
    m0 = r["connections"][:6].reshape(3, 2)
    assert m0.tolist() == [[1, 1], [1, 1], [1, 0]]  # bg-bg, bg-blob, A-bg, A-blob, B-bg
    # bg (0,1,2) merge, A + layer-1 blob merge, B alone, layer-2 blob alone
    assert r["merged"].tolist() == [0, 1, 2, 0, 1, 0, 3]
    assert r["num_objects"] == 4
    assert_same(r, seg_ref.front_end(g))


def test_cc_objects_aggregate_fields():
    g = np.zeros((3, 6, 6), np.uint8)
    g[0, 0:2, 0:2] = 1
    g[1, 1:3, 1:3] = 1
    g[2, 5, 5] = 1
    g[0, 4:6, 4:6] = 1
    r = front(g)
    o, comps = oracle_mod.create_cc_objects(r, (-10, -20, -1), (0.1, 0.1, 0.12))
    assert o["num_components"].tolist() == [3, 2, 1, 1]
    assert comps.tolist() == [0, 3, 5, 1, 4, 2, 6]  # grouped global labels, ascending per object
    # object 1 = A (layer 0, x,y 0..1) + the layer-1 blob (1..2): right/bottom = left + width
    assert o["min_voxel"][1].tolist() == [0, 0, 0] and o["max_voxel"][1].tolist() == [3, 3, 1]
    assert o["num_layers"].tolist() == [3, 2, 1, 1]
    assert o["centroid"][1].tolist() == [1.0, 1.0]       # (0.5 + 1.5) / 2
    assert o["center_voxel"][1].tolist() == [1.5, 1.5, 0.5]
    assert o["num_contour_points"].tolist() == [0, 8, 4, 1]
    f = np.float32
    assert o["min_world"][2][0] == f(f(4) * f(0.1)) + f(-10)
