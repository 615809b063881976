#!/usr/bin/env python3
"""Dispatch timeline of a rocprofv3 --kernel-trace --output-format csv run: for a window of
dispatches, the queue, start (µs from the window start), duration and idle gap before each, and
the mean wall time per frame (counting k_mask dispatches).

    python tools/timeline.py gpurun_out/tl/kernel_trace.csv --skip 2000 --count 60
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--skip", type=int, default=0)
    ap.add_argument("--count", type=int, default=60)
    a = ap.parse_args()
    rows = []
    with open(a.path) as f:
        for r in csv.DictReader(f):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gdf::", ""),
                         int(r["Start_Timestamp"]), int(r["End_Timestamp"]), q))
    rows.sort(key=lambda r: r[1])
    rows = rows[a.skip:]
    frames = [r for r in rows if r[0].startswith("k_mask")]
    if len(frames) > 2:
        print("frames %d, mean frame period %.2f us" % (
            len(frames), (frames[-1][1] - frames[0][1]) / 1e3 / (len(frames) - 1)))
    busy_end = rows[0][1]
    t0 = rows[0][1]
    for n, s, e, q in rows[:a.count]:
        gap = (s - busy_end) / 1e3
        print("%-28s q=%-4s start %9.2f dur %7.2f gap %7.2f" % (n[:28], q, (s - t0) / 1e3,
                                                               (e - s) / 1e3, gap))
        busy_end = max(busy_end, e)


if __name__ == "__main__":
    main()
