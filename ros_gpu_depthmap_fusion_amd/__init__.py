"""MI355X-native depth-map fusion hot path (drop-in for gpu_depthmap_fusion's GPUDepthmapFusion).

The compute path is libgdf.so (HIP kernels for gfx950 behind the C-ABI of include/gdf.h);
`gdf.GPUDepthmapFusion` is the Python mirror of the reference engine over that ABI.
"""
from .build import build_library, LIB_PATH  # noqa: F401

__all__ = ["build_library", "LIB_PATH"]
