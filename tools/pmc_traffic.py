#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 PMC passes -> profiles/pmc_traffic.json.

Inputs: the *_counter_collection.csv of a FETCH_SIZE pass and of a WRITE_SIZE pass (separate
rocprofv3 runs, MI355X_MICROARCH.md "rocprofv3 PMC slots": the two cannot share a pass).
FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (same guide, "HBM"): FETCH_SIZE counts
128-B requests as 64 B for wide coalesced streaming reads, so it is doubled; WRITE_SIZE is
taken as is.  Both are calibrated only for 16-B-per-lane streams: narrower access widths (the
2-B depth loads of k_mask) are reported with the same rule and flagged as uncalibrated.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv --workload 640x480/dense/b8 [--out profiles/pmc_traffic.json]

The output maps workload -> kernel slot -> bytes per launch (bench.py reads the entry of its
own workload; a launch of a multi-frame batch covers the batch).
"""
import argparse
import collections
import csv
import json

SLOT = {"k_mask": "mask", "k_mask_px": "mask", "k_emit": "emit", "k_sort_pass": "sort", "k_group": "group",
        "k_group_runs": "group", "k_group_big": "group_big", "k_group_runs_big": "group_big",
        "k_scan_counts": "scan", "k_grid_u8": "grid", "k_grid_u32": "grid", "k_sel": "sel",
        "k_sort_hist": "sort_hist", "k_group_count": "group_count"}


def per_kernel(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gdf::", "")
        base = name.split("<")[0]
        if base in SLOT:
            acc[SLOT[base]].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    a = ap.parse_args()
    fetch = per_kernel(a.fetch_csv, "FETCH_SIZE")
    write = per_kernel(a.write_csv, "WRITE_SIZE")
    try:
        allw = json.load(open(a.out))
        if not all(isinstance(v, dict) and "workload" not in v for v in allw.values()):
            allw = {}  # (round-1 layout: one workload at top level)
    except (OSError, ValueError):
        allw = {}
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k, 0.0) * 1024 * 2
        w = write.get(k, 0.0) * 1024
        out[k] = {"hbm_bytes_per_launch": round(f + w),
                  "fetch_bytes": round(f), "write_bytes": round(w),
                  "note": "FETCH_SIZE x2 (gfx950 wide-read rule), WRITE_SIZE as is; "
                          "uncalibrated for sub-16-B accesses"}
    allw[a.workload] = out
    json.dump(allw, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
