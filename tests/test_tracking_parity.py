"""objectTracking parity: gdf::object_tracking (include/gdf_objects.hpp, the
facade's restatement of src/gpu_depthmap_fusion.cpp:2579-2944 and filter/*.h) against the
independent Python restatement tests/tracking_ref.py, frame by frame, bit for bit: the number and
order of the tracks, each track's filtered box (center, size, angle), score, age and the label of
the object it last merged.

Object sequences:
* recorded from the engine's own grids: the oracle engine (oracle/gdf_oracle.c) fuses dense VGA
  frames of two cameras whose world pose turns 1.5 deg per frame about the vertical (so the
  scene's objects move through the grid), lifetime 1; every grid goes through the segmentation
  front end (oracle/seg_oracle.c: labels, contours, label merge) and createCCObjects' grouping
  (oracle.create_cc_objects); an object's top view is the world (x, y) of its components'
  contour points (fusion.cpp:2439-2537), its box the facade's MinShapes of them;
* hand-made boxes for the association branches the scene does not reach: two objects competing
  for one track, objects below min_area, a box turning by 90 degrees (best_roll != 0), tracks
  that die after their objects vanish, an object jumping beyond the 2.5 m gates.

The boxes themselves (minAreaRect of the top view, OpenCV) are parity-unpinned (no OpenCV here);
both sides track the SAME boxes (the driver prints the boxes it computed).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import tracking_ref as tr  # noqa: E402

MIN_AREA = 0.05


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    exe = tmp_path_factory.mktemp("trk") / "tracking_drive"
    subprocess.run(["g++", "-std=c++17", "-O2", "-ffp-contract=off", "-Wall",
                    "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "tracking_drive.cpp"), "-o", str(exe)], check=True)
    return str(exe)


def hx(v):
    return float(v).hex()


def run_driver(exe, frames, min_area=MIN_AREA):
    """frames: per frame a list of objects ("p", label, [(x, y), ...]) or ("b", label, (cx, cy,
    w, h, angle)).  Returns per frame (boxes, tracks) as floats."""
    lines = [f"min_area {hx(min_area)}", f"frames {len(frames)}"]
    for objs in frames:
        lines.append(f"objects {len(objs)}")
        for kind, label, data in objs:
            if kind == "p":
                flat = " ".join(f"{hx(x)} {hx(y)}" for x, y in data)
                lines.append(f"p {label} {len(data)} {flat}")
            else:
                lines.append(f"b {label} " + " ".join(hx(v) for v in data))
    r = subprocess.run([exe], input="\n".join(lines) + "\n", capture_output=True, text=True,
                       check=True)
    out, it = [], iter(r.stdout.split("\n"))
    for _ in frames:
        next(it)
        nb = int(next(it).split()[1])
        boxes = [[float.fromhex(v) for v in next(it).split()] for _ in range(nb)]
        nt = int(next(it).split()[1])
        tracks = []
        for _ in range(nt):
            v = next(it).split()
            tracks.append(tuple(float.fromhex(q) for q in v[:7]) + (int(v[7]),))
        out.append((boxes, tracks))
    return out


def compare(frames, got, min_area=MIN_AREA):
    """Run the restatement on the driver's boxes and compare every frame's tracks exactly."""
    tracks = []
    ntracks = []
    for f, (objs, (boxes, want)) in enumerate(zip(frames, got)):
        assert len(boxes) == len(objs)
        objects = [{"box": tr.RRect(*b), "label": o[1]} for b, o in zip(boxes, objs)]
        tr.object_tracking(objects, tracks, min_area)
        mine = [tr.track_state(t) for t in tracks]
        assert len(mine) == len(want), f"frame {f}: {len(mine)} tracks vs {len(want)}"
        for i, (a, b) in enumerate(zip(mine, want)):
            fa = [float(v) for v in a[:7]]
            assert fa == list(b[:7]) and a[7] == b[7], f"frame {f} track {i}: {a} vs {b}"
        ntracks.append(len(mine))
    return ntracks


# ---- object sequences from the engine's grids ------------------------------------------------------
def engine_object_frames(nframes=14, W=640, H=480):
    from oracle import OracleFusion, create_cc_objects, object_segmentation_front
    from ros_gpu_depthmap_fusion_amd import synth
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams
    p = ComponentParams()
    p.occupancy_lifetime = 1
    orc = OracleFusion(threads=8)
    cams = [synth.make_camera(k, W, H) for k in (0, 2)]
    lo = np.array(p.voxel_min, np.float32)
    cs = np.array(p.voxel_size, np.float32)
    frames = []
    for f in range(nframes):
        R = np.eye(4, dtype=np.float64)
        R[:3, :3] = synth.yaw(1.5 * f)
        orc.clear()
        for k, c in zip((0, 2), cams):
            Tw = (R @ c.T_world.astype(np.float64)).astype(np.float32)
            orc.addDepthmap(synth.dense_frame(c, k, f), *c.intrinsics(), Tw, Tw)
        orc.processFrame(p)
        gx, gy, gz = orc.grid_size()
        grid = orc.downloadVoxelOccupancyGrid().reshape(gz, gy, gx)
        front = object_segmentation_front(grid)
        cols, order = create_cc_objects(front, lo, cs)
        nl = front["num_labels"].astype(np.int64)
        layer = np.repeat(np.arange(len(nl)), nl)
        # per layer: contour c -> its points (the flat arrays of seg_oracle)
        cpl = front["contours_per_layer"].astype(np.int64)
        sizes = front["contour_sizes"].astype(np.int64)
        starts = np.concatenate([[0], np.cumsum(sizes)])
        first_contour = np.concatenate([[0], np.cumsum(cpl)])
        objs = []
        for i in range(len(cols["label"])):
            a = int(cols["first_component"][i])
            pts = []
            for idx in order[a:a + int(cols["num_components"][i])]:
                c = int(front["labels_to_contours"][idx])
                if c < 0:
                    continue
                z = int(layer[idx])
                g = first_contour[z] + c
                for x, y in front["contour_points"][starts[g]:starts[g + 1]]:
                    # voxelCoordToWorldCoord (fusion.cpp:1720-1730): x * cs + lb in f32
                    wx = np.float32(np.float32(x) * cs[0]) + lo[0]
                    wy = np.float32(np.float32(y) * cs[1]) + lo[1]
                    pts.append((np.float32(wx), np.float32(wy)))
            objs.append(("p", int(cols["label"][i]), pts))
        frames.append(objs)
    return frames


def test_tracking_parity_engine_grids(driver):
    frames = engine_object_frames()
    assert min(len(o) for o in frames) > 5, "the grids hold objects"
    got = run_driver(driver, frames)
    n = compare(frames, got)
    assert max(n) > 3, n  # tracks exist ...
    merged = sum(1 for _, tracks in got for t in tracks if t[6] >= 1.0)
    assert merged > 0, "... and objects merged into them over the frames"


def box(label, cx, cy, w, h, a):
    return ("b", label, (cx, cy, w, h, a))


def test_tracking_parity_association_branches(driver):
    bg = box(0, 0, 0, 0, 0, 0)
    frames = []
    for f in range(40):
        objs = [bg]
        if f < 25:  # a box moving along x
            objs.append(box(1, 1.0 + 0.05 * f, 2.0, 1.0, 0.6, -20.0))
        if f < 30:  # a square turning; its box swaps width / height at -90 -> 0 (best_roll 1)
            ang = -80.0 + 3.0 * f
            w, h = (0.8, 1.2) if ang < 0 else (1.2, 0.8)
            objs.append(box(2, -3.0, 1.0 + 0.02 * f, w, h, ang if ang < 0 else ang - 90.0))
        if 5 <= f < 12:  # two objects close to one another: both want the same track
            objs.append(box(3, 5.0 + 0.01 * f, -2.0, 0.9, 0.9, -45.0))
            objs.append(box(4, 5.1 + 0.01 * f, -2.05, 0.85, 0.95, -40.0))
        if 8 <= f < 20:  # below min_area: ignored
            objs.append(box(5, 0.0, -4.0, 0.1, 0.2, -10.0))
        if f in (15, 16):  # an object jumping by 3 m between two frames (beyond the gates)
            objs.append(box(6, -6.0 + 3.0 * (f - 15), 5.0, 0.7, 0.7, -30.0))
        if 18 <= f < 22:  # a large box whose area halves (area_diff gate)
            s = 2.0 if f < 20 else 1.2
            objs.append(box(7, 8.0, 6.0, s, s, -60.0))
        frames.append(objs)
    got = run_driver(driver, frames)
    n = compare(frames, got)
    assert max(n) >= 4 and n[-1] < max(n), n  # tracks were created and later died
