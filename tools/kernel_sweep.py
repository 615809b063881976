"""Per-kernel timing sweep of the fused frame path over filter parameters (diagnostics).

    python tools/kernel_sweep.py [W H [cameras]]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth  # noqa: E402
from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion  # noqa: E402


def run(eng, scams, p, steps=100):
    pc = p.to_c(None, None, False, False)
    eng.run_depth_stream(scams, pc, 0, 10)
    eng.synchronize()
    eng.set_profiling(True)
    eng.run_depth_stream(scams, pc, 10, steps)
    kt = eng.kernel_times()
    eng.set_profiling(False)
    return {k: round(v[0] * 1e3 / max(v[1], 1), 2) for k, v in kt.items() if v[1]}


def main():
    W, H = (int(x) for x in (sys.argv[1:3] if len(sys.argv) > 2 else (640, 480)))
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 1
    build_library()
    cams = synth.cameras(K, W, H)
    dframes = [[hiprt.DeviceArray.from_numpy(synth.depth_frame(c, k, f)) for f in range(4)]
               for k, c in enumerate(cams)]
    eng = GPUDepthmapFusion(0)
    scams = [eng.make_stream_camera([d.ptr for d in dframes[k]], W, H, *c.intrinsics(),
                                    c.T_world, c.T_crop) for k, c in enumerate(cams)]
    out = {"W": W, "H": H, "cameras": K}
    for F, rot in [(0, False), (1, False), (2, False), (4, False), (4, True)]:
        p = ComponentParams()
        p.flying_filter_size, p.flying_rot45 = F, rot
        out[f"F{F}{'r' if rot else ''}"] = run(eng, scams, p)
    p = ComponentParams()
    p.enable_voxel_filter = False
    out["novoxel"] = run(eng, scams, p)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
