#!/usr/bin/env python3
"""H2D path probe: pointer attributes of pinned / pageable host memory, host read speed of the
pinned buffer, and per-frame time of gdf_run_host_stream (pinned, pageable) vs device frames."""
import ctypes as C
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion  # noqa: E402


class Attr(C.Structure):
    _fields_ = [("type", C.c_int), ("device", C.c_int), ("devicePointer", C.c_void_p),
                ("hostPointer", C.c_void_p), ("isManaged", C.c_int), ("flags", C.c_uint)]


def attrs(p):
    a = Attr()
    rc = hiprt.hip().hipPointerGetAttributes(C.byref(a), C.c_void_p(p))
    return rc, a.type, a.hostPointer is not None, a.flags


build_library()
cam = synth.make_camera(0, 640, 480)
frames = [synth.dense_frame(cam, 0, f) for f in range(8)]
pin = [hiprt.PinnedArray.from_numpy(f) for f in frames]
pag = [f.copy() for f in frames]
print("pinned attrs", attrs(pin[0].ptr), "pageable attrs", attrs(pag[0].ctypes.data), flush=True)
t0 = time.perf_counter()
for _ in range(20):
    s = int(pin[0].array.sum())
print("host read of a pinned frame: %.1f us" % ((time.perf_counter() - t0) / 20 * 1e6), flush=True)
dev = [hiprt.DeviceArray.from_numpy(f) for f in frames]
p = ComponentParams()
for name, ptrs, host in (("device", [d.ptr for d in dev], False),
                         ("pinned", [h.ptr for h in pin], True),
                         ("pageable", [h.ctypes.data for h in pag], True)):
    for depth in (1, 3):
        eng = GPUDepthmapFusion(0)
        eng.set_pipeline_depth(depth)
        sc = eng.make_stream_camera(ptrs, 640, 480, *cam.intrinsics(), cam.T_world, cam.T_crop)
        pc = p.to_c(None, None, False, False)
        run = eng.run_host_stream if host else eng.run_depth_stream
        run([sc], pc, 0, 20)
        eng.synchronize()
        t0 = time.perf_counter()
        run([sc], pc, 20, 200)
        eng.synchronize()
        dt = (time.perf_counter() - t0) / 200
        print(f"{name:9s} depth {depth}: {dt * 1e6:8.1f} us/frame", flush=True)
        eng.close()
