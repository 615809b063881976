"""Time the GPU segmentation front end (include/gdf_segment.h) on the occupancy grid the C2
workload produces (dense VGA frames through the engine, launch-default 400 x 400 x 21 grid),
next to the oracle's CPU time on the same grid.  Prints one JSON line.

    python tools/bench_seg.py [--frames 16] [--reps 50] [--json out.json]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def run_seg(frames=16, reps=50, cameras=4, cpu=True):
    """The segmentation front end on the C2-style grid: ms per call for the label/stat pass, with
    the connection matrices, and with contours; the oracle's single-thread CPU time beside it."""
    import torch
    from ros_gpu_depthmap_fusion_amd import build_library, synth
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion, Segmenter
    build_library()
    eng = GPUDepthmapFusion(0)
    p = ComponentParams()
    for f in range(frames):
        eng.clear()
        for k in range(cameras):
            cam = synth.make_camera(k, 640, 480)
            eng.addDepthmap(synth.dense_frame(cam, f, k), *cam.intrinsics(), cam.T_world,
                            cam.T_crop)
        eng.processFrame(p)
    grid = eng.downloadVoxelOccupancyGrid()
    gs, nc = eng.grid_size()
    seg = Segmenter(0)
    out = {"workload": f"occupancy grid after {frames} frames of {cameras} dense VGA cameras "
                       f"(launch defaults, grid {gs[0]}x{gs[1]}x{gs[2]})",
           "occupied_cells": int((grid > 0).sum())}
    for name, flags in (("labels_stats", 0), ("labels_stats_connections", 2), ("all", 3)):
        for _ in range(3):
            seg.label_engine_grid(eng, flags)
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            seg.label_engine_grid(eng, flags)
        torch.cuda.synchronize()
        out[f"ms_{name}"] = round((time.perf_counter() - t0) / reps * 1e3, 4)
    # the label merge alone (k_cc_merge_layers + the merged ids' D2H), and every output to the
    # host (labels 2 B per cell, stats, contours, connections, merge) after a fresh labelling
    tm, td = [], []
    for _ in range(max(3, reps // 2)):
        seg.label_engine_grid(eng, 2)  # (no contours: counts() then reads no contour records)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        seg.merge_labels()
        tm.append(time.perf_counter() - t0)
        seg.label_engine_grid(eng, 3)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        r = seg.results()
        td.append(time.perf_counter() - t0)
    out["ms_merge"] = round(float(np.median(tm)) * 1e3, 4)
    out["ms_download_all"] = round(float(np.median(td)) * 1e3, 4)
    out["download_all_bytes"] = int(sum(np.asarray(v).nbytes for v in r.values()
                                        if isinstance(v, np.ndarray)))
    c = seg.counts()
    out.update(total_labels=int(c.total_labels), contours=int(c.total_contours),
               contour_points=int(c.total_contour_points),
               connection_bytes=int(c.connection_bytes), objects=int(r["num_objects"]))
    if cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle  # the checker / CPU baseline only
        g3 = grid.reshape(gs[2], gs[1], gs[0])
        t0 = time.perf_counter()
        o = oracle.object_segmentation_front(g3)
        out["cpu_baseline"] = {"ms": round((time.perf_counter() - t0) * 1e3, 3), "threads": 1,
                               "kind": "port", "sample": "the same grid through oracle/seg_oracle.c"}
        same = all(np.array_equal(np.nan_to_num(np.asarray(r[k])),
                                  np.nan_to_num(np.asarray(o[k]))) for k in r)
        out["bit_exact_vs_oracle"] = bool(same)
    seg.close()
    eng.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cameras", type=int, default=4)
    ap.add_argument("--json", default=None)
    a = ap.parse_args()
    out = run_seg(a.frames, a.reps, a.cameras)
    line = json.dumps(out)
    print(line)
    if a.json:
        with open(a.json, "w") as fh:
            fh.write(line + "\n")


if __name__ == "__main__":
    main()
