#!/usr/bin/env python3
"""Per-tile phase timings of k_group_runs from the diagnostic build libgdf_trace.so
(`python tools/group_trace.py --build`; run this on the GPU box):

    python tools/gruns_trace.py W H F [frames_per_batch] [pipeline]   (default: 640 480 4 8 1)

prints the launch span (first block entry to last tile end), when the tiles start, and each
phase of a tile: run records + block scans, the tile's offset and last-group end, the staged sums,
the queue appends."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from ros_gpu_depthmap_fusion_amd.build import TRACE_LIB_PATH  # noqa: E402
import frame_driver  # noqa: E402

SLOTS = 1 << 14


def pct(x):
    return f"mean {x.mean():6.2f}  p50 {np.median(x):6.2f}  p90 {np.percentile(x, 90):6.2f}  max {x.max():6.2f}"


def main():
    W, H, F = (int(x) for x in sys.argv[1:4]) if len(sys.argv) > 3 else (640, 480, 4)
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    pipe = int(sys.argv[5]) if len(sys.argv) > 5 else 1
    eng, step = frame_driver.make(W, H, F, 0, "dense", TRACE_LIB_PATH)
    eng.set_pipeline_depth(pipe)
    lib = eng._lib
    nsteps = 6
    for i in range(nsteps):
        if i == nsteps - 1:
            eng.synchronize()
            assert lib.gdf_debug_runs_trace_clear() == 0
        step(i, batch)
    eng.synchronize()
    buf = np.zeros((SLOTS, 8), np.uint64)
    assert lib.gdf_debug_runs_trace(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
    used = buf[:, 5] != 0
    t = buf[used].astype(np.int64)
    if len(t) == 0:
        print("no k_group_runs tiles traced")
        return
    t0 = t[:, 0].min()
    span = (t[:, 5].max() - t0) / 100.0
    print(f"tiles {len(t)}  span {span:.1f} us (first block entry to last tile end)")
    st = np.sort((t[:, 1] - t0) / 100.0)
    print(f"  tile starts: p10 {np.percentile(st, 10):.1f}  p50 {np.median(st):.1f}  p90 {np.percentile(st, 90):.1f}  last {st[-1]:.1f} us")
    en = np.sort((t[:, 5] - t0) / 100.0)
    print(f"  tile ends:   p10 {np.percentile(en, 10):.1f}  p50 {np.median(en):.1f}  p90 {np.percentile(en, 90):.1f}  last {en[-1]:.1f} us")
    ph = np.diff(t[:, 1:6], axis=1) / 100.0
    tot = (t[:, 5] - t[:, 1]) / 100.0
    print(f"  tile time {pct(tot)}")
    for k, name in enumerate(("records+scans", "offset+end", "staged sums", "appends")):
        print(f"    {name:14s} {pct(ph[:, k])}  share {ph[:, k].sum() / tot.sum():.3f}")
    ent = np.sort((t[:, 1] - t[:, 0]) / 100.0)
    print(f"  block entry to tile start {pct(ent)}")
    blk = t[:, 7]
    print(f"  blocks with a tile {len(np.unique(blk))}, tiles per block max {np.bincount(blk.astype(np.int64)).max()}")


if __name__ == "__main__":
    main()
