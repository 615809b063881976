"""Concurrency of a pipelined kernel trace (rocprofv3 --kernel-trace csv): over the steady-state
window (the last `frac` of the trace), per kernel family: launches, mean duration, the share of
wall time it is running, and the mean number of kernels running alongside it; plus the wall time
with 0, 1, 2, 3+ kernels running.  python3 tools/r5/concurrency.py <run_kernel_trace.csv> [frac]"""
import csv
import re
import sys


def fam(name):
    n = re.sub(r"\(.*", "", name).replace("void ", "").replace("gdf::", "")
    return n


def load(path):
    if path.endswith(".db"):  # rocprofv3's default (rocpd) output: the `kernels` view
        import sqlite3
        c = sqlite3.connect(path)
        return [(int(s), int(e), fam(n), int(gx) // max(int(wx), 1), int(q)) for s, e, n, gx, wx, q in
                c.execute("select start, end, name, grid_x, workgroup_x, queue_id from kernels")]
    r = [x for x in csv.DictReader(open(path)) if x["Kind"] == "KERNEL_DISPATCH"]
    return [(int(x["Start_Timestamp"]), int(x["End_Timestamp"]), fam(x["Kernel_Name"]),
             int(x["Grid_Size_X"]) // max(int(x["Workgroup_Size_X"]), 1), int(x["Queue_Id"])) for x in r]


def main(path, frac=0.5):
    ev = load(path)
    ev.sort()
    t0, t1 = ev[0][0], max(e[1] for e in ev)
    lo = t1 - (t1 - t0) * frac
    ev = [e for e in ev if e[0] >= lo]
    lo = ev[0][0]
    pts = sorted([(e[0], 1) for e in ev] + [(e[1], -1) for e in ev])
    hist = {}
    cur, last = 0, pts[0][0]
    for t, d in pts:
        hist[min(cur, 3)] = hist.get(min(cur, 3), 0) + (t - last)
        cur += d
        last = t
    wall = last - lo
    print(f"window {wall / 1e3:.1f} us, {len(ev)} launches, queues {sorted(set(e[4] for e in ev))}")
    print("running kernels: " + ", ".join(f"{k}{'+' if k == 3 else ''}: {v / wall:.2f}" for k, v in sorted(hist.items())))
    fams = {}
    for s, e, f, g, q in ev:
        d = fams.setdefault(f, [0, 0, 0, 0])
        d[0] += 1
        d[1] += e - s
        d[3] += g
    # mean concurrency seen by each family (other kernels overlapping its launches)
    for f, d in sorted(fams.items(), key=lambda kv: -kv[1][1]):
        ov = 0
        for s, e, ff, g, q in ev:
            if ff != f:
                continue
            for s2, e2, f2, g2, q2 in ev:
                if s2 >= e:
                    break
                if e2 > s and (s2, e2, f2) != (s, e, ff):
                    ov += min(e, e2) - max(s, s2)
        print(f"{f[:40]:40s} n={d[0]:5d} mean={d[1] / d[0] / 1e3:7.2f} us  wall share={d[1] / wall:5.2f}"
              f"  overlap={ov / max(d[1], 1):4.2f}  blocks={d[3] // d[0]}")


if __name__ == "__main__":
    main(sys.argv[1], float(sys.argv[2]) if len(sys.argv) > 2 else 0.5)
