#!/usr/bin/env python3
"""Per-kernel average of each counter in rocprofv3 *_counter_collection.csv files (to keep the
committed profiles small): prints CSV kernel,counter,dispatches,average,unit-note."""
import collections
import csv
import sys


def main(paths):
    acc = collections.defaultdict(list)
    for p in paths:
        for r in csv.DictReader(open(p)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            acc[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    print("kernel,counter,dispatches,average")
    for (k, c), v in sorted(acc.items()):
        print(f"{k},{c},{len(v)},{sum(v) / len(v):.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
