"""Per-group timings of the voxel-sum kernel (k_group_runs_big) from the diagnostic build
libgdf_trace.so (built here by `python tools/group_trace.py --build`, run on the GPU box):

    python tools/group_trace.py W H F [dense|stress] [frames_per_batch]
    python tools/group_trace.py --c3 WINDOW      (720p depth + a WINDOW-sequence rollbuffer)

prints the kernel's span, the longest groups (points, chunks, cycles at barriers / LDS stores /
fetch issue / sums) and how the groups' start times spread."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ros_gpu_depthmap_fusion_amd.build import TRACE_LIB_PATH, build_library  # noqa: E402
import frame_driver  # noqa: E402

SLOTS = 1 << 16


def make_c3(window):
    """bench_c3's frames (720p depth + rollbuffer of `window` 720p sequences) on the trace build."""
    from ros_gpu_depthmap_fusion_amd import hiprt, synth
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion
    W, H = 1280, 720
    cam, lidar = synth.make_camera(0, W, H), synth.make_camera(1, W, H)
    depth = [hiprt.DeviceArray.from_numpy(synth.dense_frame(cam, 0, f)) for f in range(2)]
    seqs = []
    for f in range(2):
        xyz = synth.back_project(lidar, synth.dense_frame(lidar, 1, f))
        seqs.append(hiprt.DeviceArray.from_numpy(
            np.ascontiguousarray(np.concatenate([xyz, np.ones((len(xyz), 1), np.float32)], 1))))
    p = ComponentParams()
    p.ps_timespan = (window - 0.5) / 30.0
    pc = p.to_c(lidar.T_world, lidar.T_crop, False, False)
    eng = GPUDepthmapFusion(0, lib_path=TRACE_LIB_PATH)

    def step(k, batch=1):
        s_, ns = synth.sequence_time(k)
        eng.addPointSequenceDevice(seqs[k % 2].ptr, W * H, 16, s_, ns, synth.move_transform(k))
        eng.clear()
        eng.addDepthmapDevice(depth[k % 2].ptr, W, H, *cam.intrinsics(), cam.T_world, cam.T_crop)
        eng.processFramePrepared(pc)
    return eng, step


def main():
    if sys.argv[1] == "--build":
        print(build_library(trace=True))
        return
    if sys.argv[1] == "--c3":
        eng, step = make_c3(int(sys.argv[2]))
        nsteps, batch = int(sys.argv[2]) + 2, 1
    else:
        W, H, F = (int(x) for x in sys.argv[1:4])
        workload = sys.argv[4] if len(sys.argv) > 4 else "dense"
        batch = int(sys.argv[5]) if len(sys.argv) > 5 else 1
        eng, step = frame_driver.make(W, H, F, 0, workload, TRACE_LIB_PATH)
        nsteps = 4
    lib = eng._lib
    for i in range(nsteps):
        if i == nsteps - 1:
            eng.synchronize()
            assert lib.gdf_debug_group_trace_clear() == 0
        step(i, batch)
    eng.synchronize()
    buf = np.zeros((SLOTS, 8), np.uint64)
    assert lib.gdf_debug_group_trace(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
    print(f"queue: normal {int(buf[-1, 1])}  huge-first {int(buf[-1, 2])}  capacity {int(buf[-1, 3])}")
    buf[-1] = 0
    used = buf[:, 0] != 0
    g = buf[used]
    slots = np.flatnonzero(used)
    if len(g) == 0:
        print("no queued groups (every group summed in k_group_runs)")
        return
    w0, w1 = g[:, 0].astype(np.int64), g[:, 1].astype(np.int64)
    t0 = w0.min()
    npts = (g[:, 2] >> np.uint64(32)).astype(np.int64)
    chunks = (g[:, 2] & np.uint64(0xFFFFFFFF)).astype(np.int64)
    tot = g[:, 3].astype(np.int64)
    bar, sto, fet = g[:, 4].astype(np.int64), g[:, 5].astype(np.int64), g[:, 6].astype(np.int64)
    sm = (g[:, 7] & np.uint64((1 << 40) - 1)).astype(np.int64)
    hw = ((g[:, 7] >> np.uint64(40)) & np.uint64(0xFFFF)).astype(np.int64)
    xcc = ((g[:, 7] >> np.uint64(56)) & np.uint64(0xF)).astype(np.int64)
    print(f"groups {len(g)}  points {npts.sum()}  span {(w1.max() - t0) / 100:.1f} us (wall clock 100 MHz)")
    print(f"start offsets us: p50 {np.median(w0 - t0) / 100:.1f} p99 {np.percentile(w0 - t0, 99) / 100:.1f} max {(w0 - t0).max() / 100:.1f}")
    order = np.argsort(-(w1 - t0))[:12]
    print("slot   pts  chunks  start_us  end_us  cycles  barrier  stores  fetch   sum  cyc/chunk  xcc cu simd")
    for i in order:
        print(f"{slots[i]:5d} {npts[i]:6d} {chunks[i]:5d} {(w0[i] - t0) / 100:8.1f} {(w1[i] - t0) / 100:7.1f} "
              f"{tot[i]:7d} {bar[i]:7d} {sto[i]:7d} {fet[i]:6d} {sm[i]:6d} {tot[i] / max(chunks[i], 1):8.0f} "
              f" {xcc[i]} {(hw[i] >> 8) & 15} {(hw[i] >> 4) & 3}")
    wave = (bar == 0) & (sto == 0) & (fet == 0)
    print(f"block-mode groups {int((~wave).sum())} ({int(npts[~wave].sum())} points), wave-mode groups "
          f"{int(wave.sum())} ({int(npts[wave].sum())} points)")
    cyc = tot.sum()
    print(f"all groups: cycles {cyc}  barrier {bar.sum() / cyc:.2f}  stores {sto.sum() / cyc:.2f}  "
          f"fetch {fet.sum() / cyc:.2f}  sum {sm.sum() / cyc:.2f}  per chunk {cyc / chunks.sum():.0f}")


if __name__ == "__main__":
    main()
