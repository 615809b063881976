"""Host issue time vs wall time per frame of the C2 stream loop (diagnostics): is the frame rate
bound by the host (launch issue) or by the GPU?

    python tools/issue_rate.py [frames] [pipeline] [graphs 0/1]
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    depth = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    graphs = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    W, H = 640, 480
    build_library()
    cam = synth.make_camera(0, W, H)
    dframes = [hiprt.DeviceArray.from_numpy(synth.depth_frame(cam, 0, f)) for f in range(8)]
    eng = GPUDepthmapFusion(0)
    eng.set_graphs(bool(graphs))
    eng.set_pipeline_depth(depth)
    sc = [eng.make_stream_camera([d.ptr for d in dframes], W, H, *cam.intrinsics(), cam.T_world,
                                 cam.T_crop)]
    pc = ComponentParams().to_c(None, None, False, False)
    eng.run_depth_stream(sc, pc, 0, 50)
    eng.synchronize()
    t0 = time.perf_counter()
    eng.run_depth_stream(sc, pc, 50, n)
    t1 = time.perf_counter()
    eng.synchronize()
    t2 = time.perf_counter()
    print(f"depth={depth} graphs={graphs} issue {1e6 * (t1 - t0) / n:.2f} us/frame, "
          f"wall {1e6 * (t2 - t0) / n:.2f} us/frame")


if __name__ == "__main__":
    main()
