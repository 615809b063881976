"""Runs one fused-frame configuration for N steps, one at a time (profiling driver for rocprofv3 /
PMC: per-kernel durations without frames in flight overlapping).

    python tools/frame_driver.py W H F ROT45(0/1) [steps] [dense|stress] [batch]

A step is one frame, or `batch` frames through one launch chain (nextFrameInBatch, as the
headline C2 line's 8-frame batches)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion  # noqa: E402


def make(W, H, F, rot, workload, lib_path=None):
    gen = synth.WORKLOADS[workload]
    cam = synth.make_camera(0, W, H)
    ring = 8
    dframes = [hiprt.DeviceArray.from_numpy(gen(cam, 0, f)) for f in range(ring)]
    eng = GPUDepthmapFusion(0, lib_path=lib_path) if lib_path else GPUDepthmapFusion(0)
    p = ComponentParams()
    p.flying_filter_size, p.flying_rot45 = F, bool(rot)
    pc = p.to_c(None, None, False, False)

    def step(i, batch=1):
        eng.clear()
        for j in range(batch):
            if j:
                eng.nextFrameInBatch()
            eng.addDepthmapDevice(dframes[(i * batch + j) % ring].ptr, W, H, *cam.intrinsics(),
                                  cam.T_world, cam.T_crop)
        eng.processFramePrepared(pc)
    return eng, step


def main():
    W, H, F, rot = (int(x) for x in sys.argv[1:5])
    steps = int(sys.argv[5]) if len(sys.argv) > 5 else 50
    workload = sys.argv[6] if len(sys.argv) > 6 else "stress"
    batch = int(sys.argv[7]) if len(sys.argv) > 7 else 1
    build_library()
    eng, step = make(W, H, F, rot, workload)
    for i in range(steps):
        step(i, batch)
    eng.synchronize()


if __name__ == "__main__":
    main()
