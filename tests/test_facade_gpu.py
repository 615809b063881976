"""The C++ facade (include/gdf_fusion.hpp) driven on the GPU in the reference component's exact
call order (tests/facade_component.cpp, component.cpp:92-300): m_points, m_voxelCoords,
m_points_voxelized and m_occupancyGrid after each of three frames (depth map + point sequence)
equal the oracle's outputs committed in tests/golden/facade bit for bit, and objectSegmentation's
labels / stats / contours / merged labels equal the oracle's on that grid."""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ros_gpu_depthmap_fusion_amd", "lib")
FIX = os.path.join(ROOT, "tests", "golden", "facade")

pytestmark = pytest.mark.gpu


def build_component(out):
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "facade_component.cpp"), "-L", LIB, "-lgdf",
           "-Wl,-rpath," + LIB, "-Wl,--allow-shlib-undefined", "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_facade_component_sequence_on_gpu(tmp_path, gpu_engine_factory):
    gpu_engine_factory  # (builds libgdf.so, checks a GPU is visible)
    exe = tmp_path / "facade_component"
    build_component(exe)
    outd = tmp_path / "out"
    outd.mkdir()
    r = subprocess.run([str(exe), FIX, str(outd)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    frames = int(open(os.path.join(FIX, "manifest.txt")).readline().split()[1])
    for f in range(frames):
        for name, dt in (("points", "<u4"), ("coords", "<u4"), ("voxelized", "<u4"),
                         ("grid", "u1")):
            want = np.fromfile(os.path.join(FIX, f"{name}{f}.bin"), dt)
            got = np.fromfile(outd / f"{name}{f}.bin", dt)
            assert len(want) > 0 and np.array_equal(got, want), f"frame {f} {name}"
        # objectSegmentation front end (labelVoxels + mergeLabelsAcrossLayers) on that grid
        import oracle
        gx, gy, gz = (int(v) for v in open(outd / f"gridsize{f}.txt").read().split())
        grid = np.fromfile(os.path.join(FIX, f"grid{f}.bin"), "u1").reshape(gz, gy, gx)
        o = oracle.object_segmentation_front(grid)
        for name, dt, key in (("labels", "<u2", "labels"), ("stats", "<i4", "stats"),
                              ("merged", "<u4", "merged"), ("l2c", "<i4", "labels_to_contours"),
                              ("contours", "<i4", "contour_points")):
            got = np.fromfile(outd / f"{name}{f}.bin", dt)
            assert np.array_equal(got, o[key].reshape(-1)), f"frame {f} {name}"
        objs, _ = oracle.create_cc_objects(o, (-10, -20, -1), (0.1, 0.1, 0.12))
        got = np.fromfile(outd / f"objmin{f}.bin", "<i4")
        assert np.array_equal(got, objs["min_voxel"].reshape(-1)), f"frame {f} objects"
