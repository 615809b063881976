"""Known-answer tests pinning the CPU oracle (oracle/gdf_oracle.c).

The reference ships no tests or golden vectors and its GLSL cannot run here, so
the oracle is pinned three ways: (1) hand-computed values from the shader formulas, (2) agreement
with a second, independent pure-Python float32 restatement (tests/shader_ref.py), (3) the
reference's own radix sort compiled in oracle/_ref (test_ref_radix.py).
"""
import numpy as np
import pytest

import shader_ref as sr
from oracle import OracleFusion, ros_time_minus, stable_sort_keys

EYE = np.eye(4, dtype=np.float32)


def T(tx=0.0, ty=0.0, tz=0.0, R=None):
    m = np.eye(4, dtype=np.float32)
    if R is not None:
        m[:3, :3] = R
    m[:3, 3] = (tx, ty, tz)
    return m


def run_stages(o, cams, F, thr, rot45, lo, hi):
    """convert -> flying -> crop -> apply with per-stage snapshots (fusion.cpp:1583-1678)."""
    o.clear()
    for c in cams:
        o.addDepthmap(*c)
    o.preparePointAndMaskBuffers()
    o.uploadDepthmaps()
    o.convertDepthmaps()
    s1 = o.stage_arrays()
    o.filterFlyingPixels(F, thr, rot45)
    s2 = o.stage_arrays()
    o.cropPoints(lo, hi)
    s3 = o.stage_arrays()
    n = o.applyPointMask()
    return s1, s2, s3, n, o.downloadPoints()


def test_convert_known_answer():
    d = np.array([[0, 1000], [2000, 0]], np.uint16)
    o = OracleFusion()
    s1, *_ = run_stages(o, [(d, 0.001, 2.0, 2.0, 0.5, 0.5, T(1, 2, 3), EYE)], 0, 0.0, False,
                        (-9, -9, -9), (9, 9, 9))
    assert list(s1["maskA"]) == [0, 1, 1, 0]
    # pixel 1: u=1, v=0, z=1.0: x=(1-0.5)/2*1, y=(0-0.5)/2*1
    np.testing.assert_array_equal(s1["A"][1], np.float32([0.25, -0.25, 1.0, 1.0]))
    np.testing.assert_array_equal(s1["B"][1], np.float32([1.25, 1.75, 4.0, 1.0]))
    # pixel 2: u=0, v=1, z=2.0
    np.testing.assert_array_equal(s1["A"][2], np.float32([-0.5, 0.5, 2.0, 1.0]))
    np.testing.assert_array_equal(s1["A"][0], np.zeros(4, np.float32))
    np.testing.assert_array_equal(s1["B"][3], np.zeros(4, np.float32))


def _scene(H, W, seed, zero_frac=0.1):
    rng = np.random.default_rng(seed)
    v, u = np.mgrid[0:H, 0:W]
    base = 1500 + 40 * u + 25 * v
    steps = (rng.random((H, W)) < 0.15) * rng.integers(-600, 600, (H, W))
    d = base + steps + rng.integers(-5, 5, (H, W))
    d[rng.random((H, W)) < zero_frac] = 0
    return np.clip(d, 0, 65535).astype(np.uint16)


def _cams(n, H, W, seed):
    cams = []
    for k in range(n):
        R = sr_rot(k)
        cams.append((_scene(H, W, seed + k), 0.001, 0.6 * W, 0.6 * W, W / 2, H / 2,
                     T(0.1 * k, -0.2, 1.0, R), T(0.5, 0.0, 0.0, R)))
    return cams


def sr_rot(k):
    a = np.deg2rad(45.0 * k)
    c, s = np.cos(a), np.sin(a)
    yaw = np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])
    return (yaw @ np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]])).astype(np.float32)


@pytest.mark.parametrize("ncam,H,W,F,thr,rot45", [
    (1, 6, 7, 1, 0.3, False), (1, 9, 8, 2, 0.1, True), (2, 7, 7, 2, 0.3, False),
    (3, 5, 9, 1, 0.5, True), (2, 8, 6, 4, -0.2, True), (1, 1, 1, 1, 0.3, False),
    (2, 3, 2, 1, 0.0, True),
])
def test_oracle_matches_python_restatement(ncam, H, W, F, thr, rot45):
    cams = _cams(ncam, H, W, 1000 + 17 * H + W)
    lo, hi = (-2.0, -2.0, 0.5), (3.0, 2.0, 3.0)
    o = OracleFusion()
    s1, s2, s3, n, pts = run_stages(o, cams, F, thr, rot45, lo, hi)
    mA, A, B, Cc = sr.convert(cams)
    assert list(s1["maskA"]) == mA
    np.testing.assert_array_equal(s1["A"].view(np.uint32), np.array(A, np.float32).view(np.uint32))
    mB = sr.flying(cams, mA, A, F, thr, rot45)
    assert list(s2["maskB"]) == mB
    mC = sr.crop(mB, Cc, lo, hi)
    assert list(s3["maskA"]) == mC
    exp = np.array(sr.apply_mask(mC, B), np.float32).reshape(-1, 4)
    assert n == len(exp)
    np.testing.assert_array_equal(pts.view(np.uint32), exp.view(np.uint32))


def test_flying_borders_and_cross_camera_reads():
    """Right/bottom F-border always invalid; camera 0 top rows read out of bounds (invalid);
    camera 1 top rows read camera 0's last rows."""
    H, W = 6, 6
    d = np.full((H, W), 2000, np.uint16)  # fronto-parallel plane: every interior test passes
    cam = (d, 0.001, 3.0, 3.0, 3.0, 3.0, EYE, EYE)
    o = OracleFusion()
    _, s2, *_ = run_stages(o, [cam, cam], 1, 0.3, False, (-9, -9, -9), (9, 9, 9))
    m0 = s2["maskB"][:36].reshape(H, W)
    m1 = s2["maskB"][36:].reshape(H, W)
    assert m0[:, W - 1].sum() == 0 and m0[H - 1, :].sum() == 0
    assert m0[0, :].sum() == 0                       # wrapped uint index -> OOB -> 0
    # camera 1's top row reads camera 0's bottom row: "up" lies below the pixel, the normal flips
    # (invalid) except at x=0, where "left" also wraps into camera 0 and flips it back
    assert list(m1[0]) == [1, 0, 0, 0, 0, 0]
    assert m0[1:H - 1, 1:W - 1].all() and m1[1:H - 1, 1:W - 1].all()
    # x=0: "left" wraps to the previous row's last pixel, dx points backwards, the normal flips
    assert m0[1:H - 1, 0].sum() == 0


def test_flying_max_distance_and_nan():
    d = np.full((4, 4), 10001, np.uint16)            # 10.001 m > max_distance 10
    o = OracleFusion()
    _, s2, *_ = run_stages(o, [(d, 0.001, 2.0, 2.0, 0.0, 0.0, EYE, EYE)], 1, 0.3, False,
                           (-99, -99, -99), (99, 99, 99))
    assert s2["maskB"].sum() == 0
    # degenerate neighbourhood (identical points -> zero cross product -> NaN normal) passes
    d = np.full((4, 4), 1000, np.uint16)
    o2 = OracleFusion()
    _, s2, *_ = run_stages(o2, [(d, 0.001, np.inf, np.inf, 0.0, 0.0, EYE, EYE)], 1, 0.9, False,
                           (-99, -99, -99), (99, 99, 99))
    assert s2["maskB"].reshape(4, 4)[1:3, 1:3].all()


def test_crop_inclusive_and_nan_pass():
    maskB = [1, 1, 1, 1, 0]
    Cc = [[1.0, 0, 0, 1], [1.0000001, 0, 0, 1], [np.nan, 0, 0, 1], [-1.0, 0, 0, 1], [0, 0, 0, 1]]
    Cc = [[np.float32(x) for x in p] for p in Cc]
    assert sr.crop(maskB, Cc, (-1, -1, -1), (1, 1, 1)) == [1, 0, 1, 1, 0]


def test_voxel_coords_clamp_and_border():
    pts = [[-20.0, 0.0, 0.0], [0.05, 0.05, 0.05], [100.0, 100.0, 100.0], [np.nan, 0.0, 0.0],
           [0.1, 0.0, 0.0]]
    pts = [[np.float32(v) for v in p] for p in pts]
    coords, gs = sr.voxel_coords(pts, (0, 0, 0), (1, 1, 1), (0.1, 0.1, 0.1))
    assert gs == [10, 10, 10]
    assert coords[0] == 0 and coords[1] == 0
    assert coords[2] == 9 + 9 * 10 + 9 * 100
    assert coords[3] == 0
    # oracle agrees
    o = OracleFusion()
    d = np.zeros((1, 1), np.uint16)
    o.clear()
    o.addDepthmap(d, 0.001, 1, 1, 0, 0, EYE, EYE)
    o.preparePointAndMaskBuffers()
    o.uploadDepthmaps()
    o.convertDepthmaps()
    o.filterFlyingPixels(1, 0.3, False)
    o.cropPoints((-1, -1, -1), (1, 1, 1))
    assert o.applyPointMask() == 0
    o.computeVoxelCoords((0, 0, 0), (1, 1, 1), (0.1, 0.1, 0.1))
    assert o.grid_size() == (10, 10, 10)


def test_occupancy_decay_known_answer():
    hist = [0] * 4
    seq = []
    for frame, coords in enumerate([[1, 2], [2], [], [], [3], []]):
        hist, out = sr.occupancy_step(hist, coords, 3)
        seq.append(out)
    assert seq == [[0, 3, 3, 0], [0, 2, 3, 0], [0, 1, 2, 0], [0, 0, 1, 0], [0, 0, 0, 3],
                   [0, 0, 0, 2]]
    hist, out = sr.occupancy_step([0, 0], [0], 300)
    assert hist == [300, 0] and out == [44, 0]  # lifetime > 255 truncates in the u8 output


def test_ps_filter_known_answers():
    # points on one view ray: direction parallel to the ray -> |cos| = 1 -> invalid
    ray = [[0.0, 0.0, 1.0 + 0.1 * i] for i in range(4)]
    assert sr.ps_filter(ray, 0.05, 1) == [0, 0, 0, 0]
    # a line perpendicular to the view direction -> cos = 0 -> valid; near-origin point invalid
    line = [[0.1 * i - 0.2, 0.0, 2.0] for i in range(4)] + [[0.0, 0.0, 0.0005]]
    m = sr.ps_filter(line, 0.05, 1)
    assert m[:3] == [1, 1, 1] and m[4] == 0
    # oracle matches the Python restatement on random sequences, F = 1..3
    rng = np.random.default_rng(5)
    for F in (1, 2, 3):
        pts = rng.normal(size=(60, 3)).astype(np.float32) * 3
        pts[7] = 0
        o = OracleFusion()
        o.addPointSequence(pts, 10, 0, EYE)
        o.uploadPointSequences()
        o.filterNewPointSequences(0.2, F)
        assert list(o.new_ps_mask()) == sr.ps_filter(pts.tolist(), 0.2, F)


def _seq_engine(o, specs):
    """specs: list of (npts, sec, nsec); returns the points added."""
    rng = np.random.default_rng(11)
    out = []
    for k, (n, s, ns) in enumerate(specs):
        p = rng.normal(size=(n, 3)).astype(np.float32) + np.float32([0, 0, 3])
        o.addPointSequence(p, s, ns, T(0.01 * k))
        out.append(p)
    return out


def test_rollbuffer_roll_and_select():
    o = OracleFusion()
    _seq_engine(o, [(5, 10, 0), (0, 11, 0), (4, 12, 5), (3, 13, 0)])
    o.uploadPointSequences()
    o.filterNewPointSequences(0.05, 1)
    o.insertNewPointSequencesInRollbuffer()
    st = o.rollbuffer_state()
    assert st[0] == 12 and st[1] == 4 and st[8:] == (13, 0)
    o.rollPointSequenceRollbufferCPU(11, 0)          # discards seq 0 (5 points)
    st = o.rollbuffer_state()
    assert st[0] == 7 and st[1] == 3 and (st[6], st[7]) == (11, 0)
    _, _, seq, hdr = o.rollbuffer_arrays()
    assert list(seq) == [1] * 4 + [2] * 3             # seq_idx renumbered by -d_seqs
    o.selectPointSequenceTimespanCPU(11, 0, 12, 5)   # seqs 0 (empty) and 1
    st = o.rollbuffer_state()
    assert st[2:6] == (0, 4, 0, 2)
    # nothing in range: start = num_seqs, count 0, point start = all points
    o.selectPointSequenceTimespanCPU(50, 0, 60, 0)
    assert o.rollbuffer_state()[2:6] == (7, 0, 3, 0)


def test_rollbuffer_roll_quirk_none_newer():
    """If no sequence is >= min, all points are discarded but 0 sequences (fusion.cpp:1108-1122);
    the headers stay, so a later roll would discard more points than exist (the reference's uint
    underflow), which the oracle reports as an error."""
    from oracle import OracleError
    o = OracleFusion()
    _seq_engine(o, [(3, 1, 0), (2, 2, 0)])
    o.uploadPointSequences()
    o.insertNewPointSequencesInRollbuffer()
    o.rollPointSequenceRollbufferCPU(5, 0)
    st = o.rollbuffer_state()
    assert st[0] == 0 and st[1] == 2 and st[6:8] == (1, 0) and st[8:] == (2, 0)
    _seq_engine(o, [(1, 6, 0)])
    o.uploadPointSequences()
    o.insertNewPointSequencesInRollbuffer()
    with pytest.raises(OracleError):
        o.rollPointSequenceRollbufferCPU(5, 0)


def test_ros_time_minus():
    assert ros_time_minus(1000, 0, 1.0) == (999, 0)
    assert ros_time_minus(1000, 100, 0.25) == (999, 750000100)
    # the float param 0.1f is 0.10000000149 s -> Duration(0, 100000001 ns)
    assert ros_time_minus(1000, 0, np.float32(0.1)) == (999, 899999999)
    assert ros_time_minus(0, 5, 1.0) is None                # ros::Time would throw


def test_stable_sort_matches_numpy():
    rng = np.random.default_rng(3)
    for keys in [rng.integers(0, 2 ** 22, 100003), rng.integers(0, 5, 5000),
                 np.zeros(17, np.int64), np.arange(1000)[::-1], np.array([], np.int64),
                 rng.integers(0, 2 ** 32, 4097, dtype=np.uint64)]:
        k = keys.astype(np.uint32)
        idx, sk = stable_sort_keys(k)
        exp = np.argsort(k, kind="stable")
        np.testing.assert_array_equal(idx, exp)
        np.testing.assert_array_equal(sk, k[exp])


def test_max_distance_square_threshold():
    """The kernels test max_distance as p·p > 100.00001f (0x42C80001) instead of
    sqrtf(p·p) > 10.0f: identical for every float around the threshold and far from it."""
    thr = np.uint32(0x42C80001).view(np.float32)
    v = np.arange(0x42C70000, 0x42C90000, dtype=np.uint32).view(np.float32)
    np.testing.assert_array_equal(np.sqrt(v) > np.float32(10.0), v > thr)
    rng = np.random.default_rng(5)
    w = (rng.random(1 << 20) * 400).astype(np.float32)
    np.testing.assert_array_equal(np.sqrt(w) > np.float32(10.0), w > thr)
