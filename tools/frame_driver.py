"""Runs one fused-frame configuration for N frames (profiling driver for rocprofv3 / PMC).

    python tools/frame_driver.py W H F ROT45(0/1) [frames] [dense|stress]
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion  # noqa: E402


def main():
    W, H, F, rot = (int(x) for x in sys.argv[1:5])
    frames = int(sys.argv[5]) if len(sys.argv) > 5 else 50
    gen = synth.WORKLOADS[sys.argv[6] if len(sys.argv) > 6 else "stress"]
    build_library()
    cam = synth.make_camera(0, W, H)
    dframes = [hiprt.DeviceArray.from_numpy(gen(cam, 0, f)) for f in range(2)]
    eng = GPUDepthmapFusion(0)
    p = ComponentParams()
    p.flying_filter_size, p.flying_rot45 = F, bool(rot)
    pc = p.to_c(None, None, False, False)
    for i in range(frames):
        eng.clear()
        eng.addDepthmapDevice(dframes[i % 2].ptr, W, H, *cam.intrinsics(), cam.T_world, cam.T_crop)
        eng.processFramePrepared(pc)
    eng.synchronize()


if __name__ == "__main__":
    main()
