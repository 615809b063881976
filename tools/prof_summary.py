#!/usr/bin/env python3
"""Per-kernel summary (calls, avg/min/max µs, share) of a rocprofv3 result: a rocpd SQLite
database (*_results.db) or a --output-format csv kernel_trace.csv.  Optionally the mean
host-visible gap between consecutive dispatches of the last N calls.

    python tools/prof_summary.py gpurun_out/prof/run_results.db [--skip-first N]
"""
import argparse
import collections
import csv
import sqlite3
import sys


def load(path):
    rows = []  # (name, start_ns, end_ns)
    if path.endswith(".db"):
        c = sqlite3.connect(path)
        for name, s, e in c.execute("select name, start, end from kernels order by start"):
            rows.append((name, int(s), int(e)))
    else:
        with open(path) as f:
            for r in csv.DictReader(f):
                rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
        rows.sort(key=lambda r: r[1])
    return rows


def short(name):
    n = name.split("(")[0]
    return n.replace("void ", "").replace("gdf::", "")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("path")
    ap.add_argument("--skip-first", type=int, default=0, help="drop the first N dispatches")
    args = ap.parse_args()
    rows = load(args.path)[args.skip_first:]
    st = collections.OrderedDict()
    for name, s, e in rows:
        st.setdefault(short(name), []).append((e - s) / 1e3)
    total = sum(sum(v) for v in st.values())
    print(f"{'kernel':40s} {'calls':>7s} {'avg_us':>9s} {'min_us':>9s} {'max_us':>9s} {'pct':>6s}")
    for k, v in sorted(st.items(), key=lambda kv: -sum(kv[1])):
        print(f"{k[:40]:40s} {len(v):7d} {sum(v)/len(v):9.2f} {min(v):9.2f} {max(v):9.2f} "
              f"{100*sum(v)/total:6.1f}")
    if len(rows) > 1:
        span = (rows[-1][2] - rows[0][1]) / 1e3
        print(f"dispatches {len(rows)}, busy {total:.0f} us of span {span:.0f} us "
              f"({100*total/span:.1f}% kernel-busy)")


if __name__ == "__main__":
    sys.exit(main())
