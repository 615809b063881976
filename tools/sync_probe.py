"""The component-equivalent synchronous loop of bench.py (run_component_sync) alone, for a
timeline under rocprofv3 (--kernel-trace --memory-copy-trace): one host VGA frame at a time,
gdf_download_frame after every frame.  Prints the per-frame latency median."""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
from ros_gpu_depthmap_fusion_amd import build_library, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion  # noqa: E402

build_library()
p = ComponentParams()
cam = synth.make_camera(0, 640, 480)
ring = [synth.dense_frame(cam, 0, f) for f in range(8)]
pc = p.to_c(None, None, False)
eng = GPUDepthmapFusion(0)
lat = []
for i in range(int(sys.argv[1]) if len(sys.argv) > 1 else 200):
    t0 = time.perf_counter()
    eng.clear()
    eng.addDepthmap(ring[i % 8], *cam.intrinsics(), cam.T_world, cam.T_crop)
    t1 = time.perf_counter()
    eng.processFramePrepared(pc)
    t2 = time.perf_counter()
    out = eng.download_frame()
    t3 = time.perf_counter()
    lat.append((t1 - t0, t2 - t1, t3 - t2, t3 - t0))
a = np.array(lat[20:]) * 1e3
print("median ms: add %.4f process %.4f download %.4f total %.4f" % tuple(np.median(a, 0)))
