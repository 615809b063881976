#!/usr/bin/env python3
"""C3 workload (BASELINE.json configs[2]): 1280x720 depth, 1 MI355X, rollbuffer timespan select +
radix compaction over a 256-frame window.

Per frame (GPUDepthmapFusionComponent::processDepthmaps, component.cpp:92-300): one new point
sequence (a back-projected 720p frame, 921 600 points, device-resident PointCloud2 records fed
through gdf_add_point_sequence_device) is filtered and inserted into the rollbuffer, the window
is rolled to the last `window` sequences (timespan (window - 0.5)/30 s at 30 fps stamps), all of
them are selected, transformed (T_world_move / T_crop_move = the lidar's camera transforms, so the
points land in the crop box like the depth camera's) and fused with the 720p depth frame:
compaction, voxel keys, occupancy marks, GPU voxelize (radix sort over every surviving point),
historic grid.  SURVEY.md §8(d) byte model + C3 additions.

    python tools/bench_c3.py [--window 256] [--steps 20] [--json out.json]

Prints one JSON line.  Not the driver's bench (that is bench.py, configs[1]); this reports the
C3 configuration with the same fields (value, roofline of the dominant kernel).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0


def run_c3(width=1280, height=720, window=256, steps=20, ring=4, profile_steps=5, corners=False,
           workload="dense"):
    """The C3 line as a dict (bench.py puts it into its "secondary" results)."""
    import numpy as np
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion

    build_library()
    W, H = width, height
    P = W * H
    gen = synth.WORKLOADS[workload]
    cam = synth.make_camera(0, W, H)        # depth camera
    lidar = synth.make_camera(1, W, H)      # the point-sequence source (another view)
    t0 = time.perf_counter()
    depth = [hiprt.DeviceArray.from_numpy(gen(cam, 0, f)) for f in range(ring)]
    seqs = []
    for f in range(ring):
        xyz = synth.back_project(lidar, gen(lidar, 1, f))
        rec = np.concatenate([xyz, np.ones((len(xyz), 1), np.float32)], 1)  # step 16
        seqs.append(hiprt.DeviceArray.from_numpy(np.ascontiguousarray(rec)))
    gen_s = time.perf_counter() - t0

    p = ComponentParams()
    p.ps_timespan = (window - 0.5) / 30.0
    p.voxel_average = not corners
    eng = GPUDepthmapFusion(0)
    pc_async = p.to_c(lidar.T_world, lidar.T_crop, False, False)
    pc_sync = p.to_c(lidar.T_world, lidar.T_crop, True, False)
    k = 0

    def frame(pc):
        nonlocal k
        s, ns = synth.sequence_time(k)
        eng.addPointSequenceDevice(seqs[k % ring].ptr, P, 16, s, ns, synth.move_transform(k))
        eng.clear()
        eng.addDepthmapDevice(depth[k % ring].ptr, W, H, *cam.intrinsics(), cam.T_world,
                              cam.T_crop)
        r = eng.processFramePrepared(pc)
        k += 1
        return r

    # fill the window (untimed), then one synchronous frame for the counts
    t0 = time.perf_counter()
    for i in range(window + 1):
        frame(pc_async)
        if i % 32 == 0:
            eng.synchronize()
            print(f"# c3 fill {i}/{window} {time.perf_counter() - t0:.1f}s", file=sys.stderr,
                  flush=True)
    eng.synchronize()
    r = frame(pc_sync)
    st = eng.rollbuffer_state()
    S, N, G = st.selection_point_count, r.num_points, r.num_voxelized
    NS, runs = eng.last_sort_items()  # what the voxelize sorts: runs of equal keys, or points
    # survivors of the depth part alone (a frame with the depth map only, no selection)
    (gx, gy, gz), ncells = eng.grid_size()
    probe = GPUDepthmapFusion(0)
    probe.clear()
    probe.addDepthmapDevice(depth[(k - 1) % ring].ptr, W, H, *cam.intrinsics(), cam.T_world,
                            cam.T_crop)
    N_depth = probe.processFrame(p).num_points
    probe.close()
    N_sel = N - N_depth
    _, gsz = np.unique(eng.downloadVoxelCoords(), return_counts=True)  # points per voxel
    group_sizes = {"max": int(gsz.max()), "p50": int(np.percentile(gsz, 50)),
                   "p99": int(np.percentile(gsz, 99)),
                   "points_in_groups_over_4096": int(gsz[gsz > 4096].sum())}

    for _ in range(3):  # every graph / buffer of the steady state in place
        frame(pc_async)
    eng.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        frame(pc_async)
    eng.synchronize()
    elapsed = time.perf_counter() - t0

    eng.set_profiling(True)
    for _ in range(profile_steps):
        frame(pc_async)
    eng.synchronize()
    kt = eng.kernel_times()
    eng.set_profiling(False)
    eng.close()

    ms = elapsed / steps * 1e3
    items = P + S
    seg = 1024
    # algorithmic HBM bytes per launch (SURVEY §8(d) + C3 terms)
    model = {
        "mask": 3.0 * P,                                         # depth in, stage bits out
        "emit": 1.0 * P + 22.0 * N_depth,                        # depth survivors: point + key
        # selected ring points in once, survivors (point + key) written once at their place
        "sel": 16.0 * S + 20.0 * N_sel,
        "sort": (12.0 * NS + 16.0 * NS * 2 + 2.0 * ncells) / 3.0,
        "group": (16.0 * N + 16.0 * NS if runs else 24.0 * N) + 16.0 * G,
        "ps_insert": 32.0 * P,                                   # new sequence in, ring out
        "scan": 8.0 * (items / seg),
    }
    per = {}
    for name in ("mask", "scan", "emit", "sel", "sort", "group", "ps_insert"):
        tot, n = kt[name]
        if n:
            per[name] = {"avg_us": round(tot * 1e3 / n, 2), "launches_per_frame":
                         round(n / profile_steps, 2),
                         "GBps": round(model[name] / (tot / 1e3 / n) / 1e9, 1)}
    dom = max(per, key=lambda q: per[q]["avg_us"] * per[q]["launches_per_frame"]) if per else None
    achieved = per[dom]["GBps"] if per else 0.0
    # PMC traffic per launch (profiles/pmc_traffic.json, tools/r5/pmc_secondary.sh) against the model
    pmc_key = "c3/%dx%d/w%d/%s" % (W, H, window, workload)
    try:
        rec = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json"))).get(pmc_key, {})
    except (OSError, ValueError):
        rec = {}
    from bench import slot_pmc  # (a timed slot's bytes: every kernel it brackets, bench.SLOT_PMC)
    for name, d in per.items():
        r = slot_pmc(rec, name)
        if r:
            d["model_bytes"] = round(model[name])
            d["pmc_bytes"] = r["hbm_bytes_per_launch"]
            d["pmc_kernels"] = r["kernels"]
            d["traffic_ratio"] = round(r["hbm_bytes_per_launch"] / max(model[name], 1), 3)
    # SURVEY §8(d) B_alg for C3: depth 2P + 24N + 9C, plus 24 n_new + 24 n_sel + 32 n_sel
    survey = 2.0 * P + 24.0 * N + 9.0 * ncells + 24.0 * P + 56.0 * S
    return {
        "metric": "Mpoints/s depth pixels (C3: 720p + %d-sequence rollbuffer window)" % window,
        "value": round(P / (elapsed / steps) / 1e6, 3),
        "unit": "Mpoints/s", "n_gpus": 1, "steps": steps, "ms_per_step": round(ms, 4),
        "points_per_frame_total": items,
        "total_points_Mps": round(items / (elapsed / steps) / 1e6, 1),
        "step_survey_bytes": round(survey),
        "step_survey_frac": round(survey / (elapsed / steps) / 1e9 / HBM_PEAK_GBPS, 4),
        "dtype": "f32", "data": "synthetic (ray-cast scene, %s frames; %d device-resident frames "
                                "and sequences reused round-robin)" % (workload, ring),
        "config": {"workload": "C3: %dx%d depth + rollbuffer window of %d sequences of %d "
                               "points (timespan select, transform, crop, compaction, voxelize, "
                               "grid %dx%dx%d)" % (W, H, window, P, gx, gy, gz),
                   "selected_points": S, "points_after_crop": N, "voxels": G,
                   "sorted_items": NS, "sorted_items_are_runs": runs,
                   "depth_points_after_crop": N_depth,
                   "points_per_voxel": group_sizes,
                   "grid_cells": ncells},
        "roofline": {"bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "traffic": per.get(dom, {}).get("pmc_bytes"),
                     "traffic_src": "profiles/pmc_traffic.json[%s]" % pmc_key,
                     "per_kernel": per},
        "setup_s": round(gen_s, 1),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--width", type=int, default=1280)
    ap.add_argument("--height", type=int, default=720)
    ap.add_argument("--window", type=int, default=256)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ring", type=int, default=4, help="distinct device-resident sequences/frames")
    ap.add_argument("--profile-steps", type=int, default=5)
    ap.add_argument("--workload", choices=("dense", "stress"), default="dense")
    ap.add_argument("--json", default=None)
    ap.add_argument("--corners", action="store_true",
                    help="voxelize without averaging (voxel corners; diagnostics)")
    args = ap.parse_args()
    out = run_c3(args.width, args.height, args.window, args.steps, args.ring, args.profile_steps,
                 args.corners, args.workload)
    line = json.dumps(out)
    print(line)
    if args.json:
        with open(args.json, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
