"""Per-kernel timing sweep of the fused frame path over filter parameters (diagnostics)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402

from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion  # noqa: E402


def run(eng, dframes, cam, W, H, p, steps=100):
    def step(i):
        eng.clear()
        eng.addDepthmapDevice(dframes[i % len(dframes)].ptr, W, H, *cam.intrinsics(), cam.T_world,
                              cam.T_crop)
        eng.processFrame(p, synchronous=False)
    for i in range(10):
        step(i)
    eng.synchronize()
    eng.set_profiling(True)
    for i in range(steps):
        step(i)
    kt = eng.kernel_times()
    return {k: round(v[0] * 1e3 / max(v[1], 1), 2) for k, v in kt.items() if v[1]}


def main():
    W, H = (int(x) for x in (sys.argv[1:3] if len(sys.argv) > 2 else (640, 480)))
    build_library()
    cam = synth.make_camera(0, W, H)
    dframes = [hiprt.DeviceArray.from_numpy(synth.depth_frame(cam, 0, f)) for f in range(4)]
    eng = GPUDepthmapFusion(0)
    out = {}
    for F, rot in [(0, False), (1, False), (2, False), (4, False), (4, True)]:
        p = ComponentParams()
        p.flying_filter_size, p.flying_rot45 = F, rot
        out[f"F{F}{'r' if rot else ''}"] = run(eng, dframes, cam, W, H, p)
    p = ComponentParams()
    p.enable_voxel_filter = False
    out["novoxel"] = run(eng, dframes, cam, W, H, p)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
