"""Host-side cost per frame of the Python binding + C engine (diagnostics).

Times, per frame, (a) ComponentParams.to_c, (b) clear + addDepthmapDevice, (c) the
gdf_process_frame call (asynchronous launches), with the GPU drained every 32 frames outside
the timed sections so the launch queue never fills."""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, FrameResult, GPUDepthmapFusion  # noqa: E402


def main():
    W, H = 640, 480
    build_library()
    cam = synth.make_camera(0, W, H)
    dframes = [hiprt.DeviceArray.from_numpy(synth.depth_frame(cam, 0, f)) for f in range(4)]
    eng = GPUDepthmapFusion(0)
    params = ComponentParams()
    prof = "prof" in sys.argv[1:]
    depth = int(next((a[6:] for a in sys.argv[1:] if a.startswith("depth=")), "1"))
    eng.set_pipeline_depth(depth)
    t = {"to_c": 0.0, "clear_add": 0.0, "process": 0.0}
    n = 0
    for i in range(2000):
        if i % 32 == 0:
            eng.synchronize()
        if i == 200:
            if prof:
                eng.set_profiling(True)
            t = {k: 0.0 for k in t}
            n = 0
        t0 = time.perf_counter()
        p = params.to_c(None, None, False, False)
        t1 = time.perf_counter()
        eng.clear()
        eng.addDepthmapDevice(dframes[i % 4].ptr, W, H, *cam.intrinsics(), cam.T_world, cam.T_crop)
        t2 = time.perf_counter()
        r = FrameResult()
        eng._check(eng._lib.gdf_process_frame(eng._h, C.byref(p), C.byref(r)))
        t3 = time.perf_counter()
        t["to_c"] += t1 - t0
        t["clear_add"] += t2 - t1
        t["process"] += t3 - t2
        n += 1
    eng.synchronize()
    print(json.dumps({k: round(v / n * 1e6, 2) for k, v in t.items()} | {"profiling": prof, "depth": depth}))


if __name__ == "__main__":
    main()
