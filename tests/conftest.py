"""Test configuration: the `gpu` marker, import paths, and on-demand oracle build.

`-m "not gpu"` tests run in the build container (no GPU): oracle KATs, reference-radix pinning,
golden fixtures, host logic, ABI exports, multi-process gloo tests.  `-m gpu` tests are the
parity tests proper; they call libgdf.so through the C-ABI and compare with the oracle.
"""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libgdf.so)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True,
                       capture_output=True)


def gpu_available() -> bool:
    try:
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        n = ctypes.c_int(0)
        return hip.hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False


@pytest.fixture(scope="session")
def gpu_engine_factory():
    if not gpu_available():
        pytest.fail("-m gpu test run without a visible GPU")
    from ros_gpu_depthmap_fusion_amd import build_library
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    build_library()
    return GPUDepthmapFusion
