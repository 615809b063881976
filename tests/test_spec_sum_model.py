"""CPU check of the voxel-sum algorithms the GPU kernels use (tests/spec_sum_model.py restates
gdf_voxsum.hpp comp_stretch_sum and rows_chunk_sum): the stretch evaluation equals the
reference's sequential f32 chain (inc/voxelize.h:29-35) bit for bit on adversarial inputs -
ties at every binade, sums crossing zero, exact cancellation, subnormals, huge terms, inf/NaN,
long monotone sums - and on the points of a real dense frame's voxels."""
import numpy as np
import pytest

from spec_sum_model import cursor_sum, group_sum, rows_sum, sequential_sum

f32 = np.float32


def same(a, b):
    a, b = f32(a), f32(b)
    if np.isnan(a) and np.isnan(b):
        return True
    return np.array([a], f32).view(np.uint32)[0] == np.array([b], f32).view(np.uint32)[0]


def cases():
    rng = np.random.default_rng(1234)
    out = {}
    out["monotone"] = rng.uniform(5.0, 5.1, 5000).astype(f32)
    out["negative"] = rng.uniform(-12.1, -12.0, 3000).astype(f32)
    out["walk_zero"] = rng.normal(0.0, 0.003, 8000).astype(f32)
    out["coarse_walk"] = (rng.integers(-7, 8, 6000) * 2.0 ** -12).astype(f32)
    out["exact_cancel"] = np.tile(np.array([0.75, -0.75, 0.5, -0.5], f32), 500)
    # ties everywhere: terms one binade below the sum, odd last mantissa bit
    base = rng.uniform(0.0625, 0.125, 4000).astype(f32)
    out["ties"] = (base.view(np.uint32) | 1).view(f32)
    out["ties_mixed_sign"] = (out["ties"] * np.where(rng.random(4000) < 0.5, -1, 1)).astype(f32)
    out["subnormal"] = np.concatenate([rng.uniform(0, 1e-39, 300), rng.uniform(0, 1e-3, 300)]).astype(f32)
    out["tiny_then_big"] = np.concatenate([np.full(100, 1e-30, f32), np.full(200, 3.0e5, f32),
                                           np.full(100, 1e-30, f32)])
    out["huge"] = rng.uniform(1e37, 3e37, 300).astype(f32)  # overflows to inf part way
    out["with_inf"] = np.concatenate([np.ones(70, f32), [np.inf], np.ones(10, f32)]).astype(f32)
    out["with_nan"] = np.concatenate([np.ones(30, f32), [np.nan], np.ones(100, f32)]).astype(f32)
    out["pos_neg_inf"] = np.array([1, np.inf, 2, -np.inf, 3], f32)
    out["ones"] = np.ones(70000, f32)  # w: exact integers across many binades
    out["big_magnitude"] = rng.uniform(29.9, 30.0, 20000).astype(f32)
    out["alternating_scale"] = (rng.uniform(0.5, 1, 4000) * np.where(np.arange(4000) % 2, 1e-6, 1)).astype(f32)
    out["single"] = np.array([0.3], f32)
    out["neg_zero"] = np.array([-0.0, -0.0, 1.0, -1.0, -0.0], f32)
    return out


@pytest.mark.parametrize("name", sorted(cases().keys()))
def test_stretch_sum_equals_sequential_chain(name):
    x = cases()[name]
    assert same(group_sum(x), sequential_sum(x)), name
    for R in (1, 2, 4):  # the GPU's cursor form
        assert same(cursor_sum(x, R), sequential_sum(x)), (name, R)
    for NR in (16, 8, 4, 1):  # the row form (k_group_runs_big: 16 / 8 rows, wave_group_sum: 4)
        assert same(rows_sum(x, NR), sequential_sum(x)), (name, NR)


def test_random_prefixes_and_row_offsets():
    """Every prefix length 0..200 of several distributions (rows end at every lane)."""
    rng = np.random.default_rng(7)
    for dist in range(4):
        x = [rng.uniform(0.01, 0.09, 200), rng.normal(0, 0.02, 200),
             rng.uniform(-0.1, 0.1, 200) * 2.0 ** rng.integers(-20, 2, 200),
             np.round(rng.normal(0, 5, 200)) * 2.0 ** -3][dist].astype(f32)
        for n in range(0, 201, 7):
            assert same(group_sum(x[:n]), sequential_sum(x[:n])), (dist, n)
            assert same(cursor_sum(x[:n], 2), sequential_sum(x[:n])), (dist, n)
            assert same(rows_sum(x[:n], 1), sequential_sum(x[:n])), (dist, n)


def test_dense_frame_voxels_match_and_stretches_are_few():
    """The points of a dense 640x480 frame, grouped by voxel as the reference's stable sort does:
    every component sum equals the chain.  A sum needs about one extra stretch per doubling
    (log2 n per voxel, most of them in the first row): voxels of >= 256 points (~500 on average
    here) take < 3 stretches per 64-term row, and a 20 K-term sum ~1.05."""
    from oracle import OracleFusion
    from ros_gpu_depthmap_fusion_amd import synth
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams
    cam = synth.make_camera(0, 640, 480)
    o = OracleFusion(threads=4)
    o.clear()
    o.addDepthmap(synth.dense_frame(cam, 0, 0), *cam.intrinsics(), cam.T_world, cam.T_crop)
    o.processFrame(ComponentParams())
    P, K, V = o.downloadPoints(), o.downloadVoxelCoords(), o.downloadVoxelizedPoints()
    order = np.argsort(K, kind="stable")
    ks, ps = K[order], P[order]
    starts = np.flatnonzero(np.r_[True, ks[1:] != ks[:-1]])
    ends = np.r_[starts[1:], len(ks)]
    long_stats = {"single": 0, "stretches": 0}
    rows = 0
    for g, (a, e) in enumerate(zip(starts, ends)):
        for c in range(4):
            stats = long_stats if e - a >= 256 else None
            s = group_sum(ps[a:e, c], stats)
            if e - a >= 64:
                assert same(rows_sum(ps[a:e, c]), s)
            want = V[g, c] * f32(e - a) if c < 3 else V[g, c]
            if c == 3:
                assert same(s, want)
            else:
                assert same(f32(s / f32(e - a)), V[g, c])
            rows += (e - a + 63) // 64 if stats is not None else 0
    assert rows > 100 and long_stats["stretches"] < 3.0 * rows, (long_stats, rows)
    st = {"single": 0, "stretches": 0}
    x = np.random.default_rng(3).uniform(5.0, 5.1, 20000).astype(f32)
    assert same(group_sum(x, st), sequential_sum(x))
    assert st["stretches"] < 1.1 * (20000 // 64 + 1), st
