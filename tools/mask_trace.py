"""Per-block phase timings of k_mask_px (the 1-row kernel) from the diagnostic build
libgdf_trace.so (`python tools/group_trace.py --build` builds it), on one isolated batch:

    python tools/mask_trace.py W H BATCH [dense|stress]

prints the launch's span, how the blocks' start times spread (the generations of resident blocks),
and wave 0's cycles per phase - segment geometry and camera, band loads landed, LDS stores +
barrier, the filter, ballots + publish barrier, the scan tail.  Each phase is closed by a wait for
the wave's outstanding memory operations, which the product kernel does not do: the phases are
upper bounds of what each costs, and the span is longer than the product kernel's."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ros_gpu_depthmap_fusion_amd.build import TRACE_LIB_PATH  # noqa: E402
import frame_driver  # noqa: E402

SLOTS = 1 << 14
PHASES = ("geometry+camera", "band loads", "LDS stores+barrier", "filter", "ballots+publish",
          "scan tail")


def main():
    W, H, B = (int(x) for x in sys.argv[1:4])
    workload = sys.argv[4] if len(sys.argv) > 4 else "dense"
    eng, step = frame_driver.make(W, H, 4, 0, workload, TRACE_LIB_PATH)
    for i in range(4):
        step(i, B)
    eng.synchronize()
    step(4, B)  # alone on the GPU
    eng.synchronize()
    buf = np.zeros((SLOTS, 8), np.uint64)
    assert eng._lib.gdf_debug_mask_trace(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
    g = buf[buf[:, 0] != 0]
    w0, w1 = g[:, 0].astype(np.int64), g[:, 1].astype(np.int64)
    t0 = w0.min()
    print(f"blocks {len(g)}  span {(w1.max() - t0) / 100:.1f} us  block life p50 "
          f"{np.median(w1 - w0) / 100:.2f} us p90 {np.percentile(w1 - w0, 90) / 100:.2f} us (wall clock 100 MHz)")
    st = (w0 - t0) / 100
    print("block starts us: " + "  ".join(f"p{q} {np.percentile(st, q):.1f}" for q in (10, 25, 50, 75, 90, 100)))
    ph = g[:, 2:8].astype(np.int64)
    tot = ph.sum(1)
    print(f"wave 0 cycles per block: mean {tot.mean():.0f}")
    for k, n in enumerate(PHASES):
        print(f"  {n:22s} mean {ph[:, k].mean():8.0f}  p50 {np.median(ph[:, k]):8.0f}  p90 "
              f"{np.percentile(ph[:, k], 90):8.0f}  share {ph[:, k].sum() / tot.sum():.2f}")


if __name__ == "__main__":
    main()
