#!/usr/bin/env python3
"""Per-tile phase timings of k_sel (the C3 window pass) from the diagnostic build libgdf_trace.so
(`python tools/group_trace.py --build` builds it here; run this on the GPU box):

    python tools/sel_trace.py WINDOW      (720p depth + a WINDOW-sequence rollbuffer, as bench_c3)

prints the launch span, each phase's share of a tile (ticket, counting pass, look-back, store
pass), and the gaps between consecutive tiles of one CU (block dispatch)."""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from group_trace import make_c3  # noqa: E402

SLOTS = 1 << 16


def pct(x):
    return f"mean {x.mean():7.2f}  p50 {np.median(x):7.2f}  p90 {np.percentile(x, 90):7.2f}  p99 {np.percentile(x, 99):7.2f}"


def main():
    window = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    eng, step = make_c3(window)
    lib = eng._lib
    nsteps = window + 2
    for i in range(nsteps):
        if i == nsteps - 1:
            eng.synchronize()
            assert lib.gdf_debug_sel_trace_clear() == 0
        step(i)
    eng.synchronize()
    buf = np.zeros((SLOTS, 8), np.uint64)
    assert lib.gdf_debug_sel_trace(buf.ctypes.data_as(C.c_void_p), C.c_size_t(buf.nbytes)) == 0
    used = buf[:, 4] != 0
    t = buf[used].astype(np.int64)
    if len(t) == 0:
        print("no k_sel tiles traced")
        return
    t0 = t[:, 0].min()
    span = (t[:, 4].max() - t0) / 100.0
    ph = np.diff(t[:, 0:5], axis=1) / 100.0  # us: ticket, counting pass, look-back, store pass
    tot = (t[:, 4] - t[:, 0]) / 100.0
    print(f"tiles {len(t)}  span {span:.1f} us  tile time {pct(tot)}")
    for k, name in enumerate(("ticket", "counting pass", "look-back", "store pass")):
        print(f"  {name:13s} {pct(ph[:, k])}  share {ph[:, k].sum() / tot.sum():.3f}")
    hw = t[:, 5]
    cu = ((hw >> 16) & 0xF) * 1000 + ((hw >> 13) & 0x7) * 100 + ((hw >> 12) & 0x1) * 20 + ((hw >> 8) & 0xF)
    gaps, busy, per = [], 0.0, []
    for c in np.unique(cu):
        r = t[cu == c]
        r = r[np.argsort(r[:, 0])]
        busy += ((r[:, 4] - r[:, 0]) / 100.0).sum()
        per.append(len(r))
        if len(r) > 1:
            gaps.extend(((r[1:, 0] - r[:-1, 4]) / 100.0).tolist())
    gaps = np.array(gaps)
    print(f"CUs {len(per)}  tiles per CU {np.mean(per):.1f} (min {min(per)} max {max(per)})  "
          f"busy {busy / (len(per) * span):.3f} of the span")
    if len(gaps):
        print(f"  gap between a CU's tiles {pct(gaps)}  (negative: two blocks overlapped on a CU)")
    first = np.sort((t[:, 0] - t0) / 100.0)
    print(f"  tile starts: first 256 by {first[min(255, len(first) - 1)]:.1f} us, last at {first[-1]:.1f} us")


if __name__ == "__main__":
    main()
