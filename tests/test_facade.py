"""The C++ facade (include/gdf_fusion.hpp) compiles against the reference component's call
sequence and links against libgdf.so (CPU-only check: nothing is run)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "ros_gpu_depthmap_fusion_amd", "lib")


def test_facade_compiles_and_links(tmp_path):
    if not os.path.exists(os.path.join(LIB, "libgdf.so")):
        pytest.skip("libgdf.so not built")
    out = tmp_path / "facade_example"
    cmd = ["g++", "-std=c++17", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "facade_example.cpp"), "-L", LIB, "-lgdf",
           "-Wl,--allow-shlib-undefined", "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
