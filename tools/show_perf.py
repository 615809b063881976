"""Summarise a tools/gpu_perf_groups.sh run: python tools/show_perf.py gpurun_out/<dir>"""
import csv
import json
import os
import sys

d = sys.argv[1]
for sub in ("t4k", "s4k", "sc2", "tc3"):
    f = os.path.join(d, sub, "run_kernel_stats.csv")
    if os.path.exists(f):
        for r in list(csv.DictReader(open(f)))[:8]:
            print(f"{sub:4s} {r['Name'][:44]:44s} {int(r['Calls']):6d} {float(r['AverageNs']) / 1000:9.1f} us {r['Percentage'][:5]}")
f = os.path.join(d, "bench_20_5.json")
if os.path.exists(f):
    b = json.load(open(f))
    print("C2", b["value"], b["roofline"]["per_kernel_us"])
    s = b["secondary"]
    print("4K", s["4k"]["value"], s["4k"]["roofline"]["per_kernel_us"])
    print("720p", s["720p"]["value"], "vga1", s["vga_single_frame"]["value"])
    print("C3", s["c3"]["value"], "group", s["c3"]["roofline"]["per_kernel"]["group"])
for f in ("trace4k.txt", "t.log"):
    p = os.path.join(d, f)
    if os.path.exists(p):
        print(open(p).read()[-2500:])
