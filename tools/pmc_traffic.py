#!/usr/bin/env python3
"""Per-kernel HBM traffic from rocprofv3 PMC passes -> profiles/pmc_traffic.json.

Inputs: the *_counter_collection.csv of a FETCH_SIZE pass and of a WRITE_SIZE pass (separate
rocprofv3 runs, MI355X_MICROARCH.md "rocprofv3 PMC slots": the two cannot share a pass) of
`bench.py --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1`.  FETCH_SIZE /
WRITE_SIZE are in KiB.  gfx950 correction (same guide, "HBM"): FETCH_SIZE counts 128-B requests
as 64 B for wide coalesced streaming reads, so it is doubled; WRITE_SIZE is taken as is.  Both
are calibrated only for 16-B-per-lane streams: narrower access widths (the 2-B depth loads of
k_mask) are reported with the same rule and flagged as uncalibrated.

Attribution: kernels are kept apart by their FULL name (template arguments
included), so the timed batch kernels (k_mask_px<2, 256>, k_emit_px2<256>, k_sort_pass<8, ...>)
are never averaged with the single-frame variants of bench.py's synchronous count pass
(k_mask<false, 4u>, k_emit, k_sort_pass<4, 256>).  The steady phase starts at the first dispatch
of the most-dispatched compaction kernel (the count pass precedes it); a slot's entry averages its
variants' launches inside that phase, and "_step" is every byte the phase moved (all
kernels, copies included) per launch of that compaction kernel, i.e. per bench step.

    python tools/pmc_traffic.py FETCH.csv WRITE.csv --workload 640x480/dense/b8 [--out profiles/pmc_traffic.json]
"""
import argparse
import collections
import csv
import json

# slot of bench.py's roofline (SINGLE_SLOTS) per kernel base name
SLOT = {"k_mask": "mask", "k_mask_px": "mask", "k_mask_px_o8": "mask", "k_emit": "emit", "k_emit_px2": "emit",
        "k_sort_pass": "sort", "k_group": "group", "k_group_runs": "group",
        "k_group_big": "group_big", "k_group_runs_big": "group_big", "k_scan_counts": "scan",
        "k_scan_reduce": "scan_reduce", "k_grid_u8": "grid", "k_grid_u32": "grid",
        "k_grid_u8_batch": "grid", "k_sel": "sel", "k_sort_hist": "sort_hist",
        "k_group_count": "group_count", "k_ps_filter_insert": "ps_insert"}


def kname(raw):
    return raw.split("(")[0].replace("void ", "").replace("gdf::", "").strip()


def load(path, counter):
    """[(dispatch_id, kernel full name, KiB)] in dispatch order."""
    rows = []
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        rows.append((int(r["Dispatch_Id"]), kname(r["Kernel_Name"]), float(r["Counter_Value"])))
    rows.sort()
    return rows


def steady(rows):
    """Dispatches from the first one of the most-dispatched compaction (mask) kernel on, and the
    name of that kernel."""
    cnt = collections.Counter(n for _, n, _ in rows if n.split("<")[0] in ("k_mask", "k_mask_px", "k_mask_px_o8"))
    if not cnt:
        return rows, None
    mk = cnt.most_common(1)[0][0]
    first = next(i for i, (_, n, _) in enumerate(rows) if n == mk)
    return rows[first:], mk


def per_variant(rows, scale):
    acc = collections.defaultdict(list)
    for _, n, v in rows:
        acc[n].append(v * 1024 * scale)
    return {n: (sum(v) / len(v), len(v)) for n, v in acc.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch_csv")
    ap.add_argument("write_csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", default="profiles/pmc_traffic.json")
    ap.add_argument("--last", type=int, default=0,
                    help="only the last N steps (from the N-th last compaction dispatch on): runs "
                         "whose early frames differ, e.g. the C3 window filling up")
    a = ap.parse_args()
    fr, mk = steady(load(a.fetch_csv, "FETCH_SIZE"))
    wr, mk2 = steady(load(a.write_csv, "WRITE_SIZE"))
    if a.last:
        def tail(rows, k):
            idx = [i for i, (_, n, _) in enumerate(rows) if n == k]
            return rows[idx[-a.last]:] if len(idx) >= a.last else rows
        fr, wr = tail(fr, mk), tail(wr, mk2)
    fv, wv = per_variant(fr, 2.0), per_variant(wr, 1.0)
    out = {}
    by_slot = collections.defaultdict(list)
    for n in set(fv) | set(wv):
        base = n.split("<")[0]
        if base in SLOT:
            by_slot[SLOT[base]].append(n)
    for slot, names in sorted(by_slot.items()):
        # every variant of the slot inside the steady phase (e.g. the 8- and 9-bit radix passes of
        # one sort): bytes per launch averaged over their launches, as bench.py's event timing
        # averages the slot's launch durations
        fb = sum(fv.get(q, (0.0, 0))[0] * fv.get(q, (0.0, 0))[1] for q in names)
        wb = sum(wv.get(q, (0.0, 0))[0] * wv.get(q, (0.0, 0))[1] for q in names)
        nf = sum(fv.get(q, (0.0, 0))[1] for q in names)
        nw = sum(wv.get(q, (0.0, 0))[1] for q in names)
        f, w = fb / max(nf, 1), wb / max(nw, 1)
        out[slot] = {"kernels": sorted(names), "hbm_bytes_per_launch": round(f + w),
                     "fetch_bytes": round(f), "write_bytes": round(w), "dispatches": max(nf, nw)}
    nsteps = sum(1 for _, n, _ in fr if n == mk) if mk else 0
    if nsteps:
        fb = sum(v for _, _, v in fr) * 1024 * 2.0
        wb = sum(v for _, _, v in wr) * 1024
        out["_step"] = {"hbm_bytes_per_step": round((fb + wb) / nsteps),
                        "fetch_bytes_per_step": round(fb / nsteps),
                        "write_bytes_per_step": round(wb / nsteps), "steps": nsteps,
                        "step_kernel": mk,
                        "note": "every dispatch of the steady phase (from the first %s on) per "
                                "launch of it = per bench step" % mk}
    out["_note"] = ("FETCH_SIZE x2 (gfx950 wide-read rule), WRITE_SIZE as is; uncalibrated for "
                    "sub-16-B accesses; one batch in flight (--pipeline 1)" +
                    ("; the last %d steps" % a.last if a.last else ""))
    try:
        allw = json.load(open(a.out))
    except (OSError, ValueError):
        allw = {}
    allw[a.workload] = out
    json.dump(allw, open(a.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
