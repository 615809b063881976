#!/usr/bin/env python3
"""Copy a tools/r4_final.sh result directory into profiles/r04/final and refresh the committed
counter files: profiles/pmc_traffic.json (FETCH / WRITE passes, tools/pmc_traffic.py),
profiles/pmc_sq.json (SQ pass, tools/pmc_sq_json.py), the per-kernel counter summaries and the
per-step kernel table of the C2 trace (one batch in flight).

    python tools/r4_collect.py gpurun_out/r4final3 [--dst profiles/r04/final]
"""
import argparse
import csv
import json
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)


def run(args, out_path=None):
    r = subprocess.run([sys.executable, *args], cwd=ROOT, capture_output=True, text=True, check=True)
    if out_path:
        with open(out_path, "w") as f:
            f.write(r.stdout)
    return r.stdout


def kernel_table(stats_csv, out_txt):
    rows = list(csv.DictReader(open(stats_csv)))
    nb = max(int(r["Calls"]) for r in rows if "k_mask_px" in r["Name"])
    lines = ["rocprofv3 --kernel-trace --stats of python3 bench.py --steps 50 --warmup 5 --no-secondary "
             "--no-cpu-baseline --no-kernel-timing --pipeline 1",
             f"(one 8-frame VGA batch in flight; per-step = total / {nb} steps incl. the settle + warm-up steps)",
             "kernel                               calls     avg_us    us/step"]
    for r in rows:
        name = r["Name"].split("(")[0].replace("void ", "").replace("gdf::", "")
        calls, avg = int(r["Calls"]), float(r["AverageNs"]) / 1e3
        if calls * avg / nb >= 0.15:
            lines.append("%-36s %6d %10.2f %10.2f" % (name[:36], calls, avg, calls * avg / nb))
    with open(out_txt, "w") as f:
        f.write("\n".join(lines) + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--dst", default=os.path.join(ROOT, "profiles", "r04", "final"))
    a = ap.parse_args()
    s, d = a.src, a.dst
    os.makedirs(d, exist_ok=True)
    for f in ("pytest_gpu.log", "smoke.log", "bench_default.json", "bench_20_5.json", "bench_300.json",
              "dist_n1.json", "c3.json"):
        if os.path.exists(os.path.join(s, f)):
            shutil.copy(os.path.join(s, f), os.path.join(d, f))
    for sub, name in (("trace", "c2_p1_kernel_stats.csv"), ("t4k", "4k_kernel_stats.csv"),
                      ("tdist", "dist_n1_kernel_stats.csv")):
        shutil.copy(os.path.join(s, sub, "run_kernel_stats.csv"), os.path.join(d, name))
    kernel_table(os.path.join(d, "c2_p1_kernel_stats.csv"), os.path.join(d, "c2_p1_kernel_summary.txt"))
    fetch = os.path.join(s, "fetch", "run_counter_collection.csv")
    write = os.path.join(s, "write", "run_counter_collection.csv")
    sq = os.path.join(s, "sq", "run_counter_collection.csv")
    run([os.path.join(HERE, "pmc_summary.py"), fetch, write], os.path.join(d, "c2_p1_pmc_hbm_summary.csv"))
    run([os.path.join(HERE, "pmc_summary.py"), sq], os.path.join(d, "c2_p1_pmc_sq_summary.csv"))
    t = run([os.path.join(HERE, "pmc_traffic.py"), fetch, write, "--workload", "640x480/dense/b8"])
    json.dump(json.loads(t), open(os.path.join(d, "pmc_traffic_c2.json"), "w"), indent=1)
    q = run([os.path.join(HERE, "pmc_sq_json.py"), sq, "--workload", "640x480/dense/b8"])
    json.dump(json.loads(q), open(os.path.join(d, "pmc_sq_c2.json"), "w"), indent=1)
    print(open(os.path.join(d, "c2_p1_kernel_summary.txt")).read())


if __name__ == "__main__":
    main()
