"""Summarise a rocprofv3 --pmc counter_collection.csv per kernel (sum over dispatches, and per
dispatch averages) - the SQ instruction / wait mix of the hot kernels.

usage: python tools/pmc_sq.py <run_counter_collection.csv> [kernel-substring ...]
"""
import csv
import sys
from collections import defaultdict


def load(path):
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"]
        k = k.split("(")[0].replace("void ", "").replace("gdf::", "")
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return tot, disp


def main():
    tot, disp = load(sys.argv[1])
    want = sys.argv[2:]
    for k in sorted(tot, key=lambda q: -tot[q].get("SQ_WAVE_CYCLES", tot[q].get("GRBM_GUI_ACTIVE", 0))):
        if want and not any(w in k for w in want):
            continue
        n = len(disp[k])
        c = tot[k]
        line = [f"{k[:34]:34s} n={n:4d}"]
        for name, v in sorted(c.items()):
            line.append(f"{name.replace('SQ_', '')}={v / n:.4g}")
        waves = c.get("SQ_WAVES")
        if waves:
            if "SQ_INSTS_VALU" in c:
                line.append(f"valu/wave={c['SQ_INSTS_VALU'] / waves:.1f}")
            if "SQ_WAVE_CYCLES" in c:
                wc = c["SQ_WAVE_CYCLES"]
                line.append(f"active={c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} wait={c.get('SQ_WAIT_ANY', 0) / wc:.2f} "
                            f"waitinst={c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f}")
        print(" ".join(line))


if __name__ == "__main__":
    main()
