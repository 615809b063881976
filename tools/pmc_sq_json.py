#!/usr/bin/env python3
"""SQ counter CSV (rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY) -> profiles/pmc_sq.json per-wave ratios of the
hot kernels for one workload key (bench.py reads the "mask" entry for roofline.valu).

    python tools/pmc_sq_json.py run_counter_collection.csv --workload 640x480/dense/b8
"""
import argparse
import collections
import csv
import json

# full kernel names (template arguments included): the timed batch kernels only, never averaged
# with the single-frame variants of the bench's synchronous count pass
SLOT = {"k_mask": ("mask", 64), "k_mask_px<2, 256>": ("mask", 128), "k_mask_px_o8<2, 256>": ("mask", 128), "k_mask_px<4, 256>": ("mask", 256),
        "k_mask_px<2, 640>": ("mask", 128), "k_emit_px2<256>": ("emit", 128), "k_emit": ("emit_1px", 64),
        "k_sort_pass<8, 256>": ("sort", 64), "k_sort_pass<8, 512>": ("sort_wide", 64),
        "k_group_runs<2048, 2>": ("group", 0), "k_sel<16u>": ("sel", 1024), "k_sel<8u>": ("sel", 512),
        "k_group_runs_big<16, false>": ("group_big", 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--workload", required=True)
    ap.add_argument("--out", default="profiles/pmc_sq.json")
    ap.add_argument("--source", default=None, help="where the committed CSV lives (recorded)")
    args = ap.parse_args()
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(args.csv)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gdf::", "")
        k = "k_mask" if k.startswith("k_mask<") else k
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = {}
    for k, c in tot.items():
        if k not in SLOT or not c.get("SQ_WAVES") or not c.get("SQ_WAVE_CYCLES"):
            continue
        w, wc = c["SQ_WAVES"], c["SQ_WAVE_CYCLES"]
        slot, ppw = SLOT[k]
        out[slot] = {"kernel": k, "pixels_per_wave": ppw,
                     "valu_per_wave": round(c["SQ_INSTS_VALU"] / w, 1),
                     "salu_per_wave": round(c["SQ_INSTS_SALU"] / w, 1),
                     "lds_per_wave": round(c["SQ_INSTS_LDS"] / w, 1),
                     "active_frac": round(c["SQ_ACTIVE_INST_ANY"] / wc, 3),
                     "wait_frac": round(c["SQ_WAIT_ANY"] / wc, 3),
                     "wait_inst_frac": round(c["SQ_WAIT_INST_ANY"] / wc, 3),
                     "dispatches": len(disp[k])}
    try:
        doc = json.load(open(args.out))
    except FileNotFoundError:
        doc = {}
    doc["_note"] = ("rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES "
                    "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY of `python3 bench.py --steps 10 "
                    "--warmup 2 --no-secondary --no-cpu-baseline --no-kernel-timing --pipeline 1` "
                    "(C2) / `tools/bench_c3.py --steps 3 --profile-steps 1` (C3), tools/pmc_sq_json.py; "
                    "per-wave ratios (the SQ counters sample a subset of the chip's waves; ratios only)")
    out["_source"] = args.source or args.csv
    doc[args.workload] = out
    json.dump(doc, open(args.out, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
