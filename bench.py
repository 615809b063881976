#!/usr/bin/env python3
"""Benchmark of the depth -> points -> flying-pixel -> crop -> voxel-occupancy hot path.

Workload (BASELINE.json configs[1], "C2"): one 640x480 16-bit synthetic depth stream per GPU,
launch-file defaults (flying-pixel F=4, thr 0.3; crop = voxel bounds -10..30 x -20..20 x -1..1.5,
cells 0.1/0.1/0.12 -> 400x400x21 = 3.36 M cells; voxelize with averaging; lifetime 10).
A step = one full frame of GPUDepthmapFusionComponent::processDepthmaps on the GPU: fused
convert+flying+crop+ordered compaction+voxel keys+occupancy marks, GPU voxelize (radix sort +
ordered means), historic-grid update.  Frames are device-resident (a ring of distinct frames
generated once and uploaded before timing).

N > 1 (torchrun, one rank per GPU over RCCL): rank k owns camera k (weak scaling).  The shared
voxel grid needs one real exchange per frame: the per-rank occupancy marks (1 bit per cell) are
all-gathered and OR-merged before every rank's identical historic-grid update.  Frames stay
pipelined on every rank; the marks of `--exchange-batch` frames travel in one all-gather and the
grid updates then run in frame order (the grids after every frame equal the per-frame exchange's).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpoints/s end-to-end depth→fused voxel grid @1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--ring", type=int, default=8, help="distinct device-resident frames")
    ap.add_argument("--cameras", type=int, default=1,
                    help="cameras per GPU (one frame = one depth map of each; camera ids "
                         "rank*cameras + k)")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="frames in flight on one GPU (engine slots, gdf_set_pipeline_depth); "
                         "N > 1 runs on torch's stream with depth 1")
    ap.add_argument("--exchange-batch", type=int, default=16,
                    help="N > 1: frames per occupancy-mark all-gather (multi.BatchedMarkExchange; "
                         "1 = one collective per frame on torch's stream, no pipelining)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="do not bracket launches with HIP events (for rocprofv3 runs)")
    return ap.parse_args()


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist = None
    rank, local_rank = 0, 0
    if args.gpus > 1 or world > 1:
        import torch
        import torch.distributed as dist
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        world = dist.get_world_size()
    import numpy as np
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt, synth
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion

    build_library()
    hiprt.set_device(local_rank)
    W, H = args.width, args.height
    K = args.cameras
    P = W * H * K
    cams = [synth.make_camera(rank * K + k, W, H) for k in range(K)]
    frames = [[synth.depth_frame(c, rank * K + k, f) for f in range(args.ring)]
              for k, c in enumerate(cams)]
    dframes = [[hiprt.DeviceArray.from_numpy(f) for f in fr] for fr in frames]
    params = ComponentParams()
    eng = GPUDepthmapFusion(local_rank)

    batched = dist is not None and args.exchange_batch > 1
    if dist is not None and not batched:
        import torch
        stream = torch.cuda.current_stream()
        eng.set_stream(stream.cuda_stream)

    def add(i):
        eng.clear()
        for k, c in enumerate(cams):
            eng.addDepthmapDevice(dframes[k][i % args.ring].ptr, W, H, *c.intrinsics(), c.T_world,
                                  c.T_crop)

    # per-frame point counts (for the algorithmic byte model), one synchronous pass over the ring
    npts, nvox = [], []
    for i in range(args.ring):
        add(i)
        r = eng.processFrame(params, synchronous=True)
        npts.append(r.num_points)
        nvox.append(r.num_voxelized)
    (gx, gy, gz), ncells = eng.grid_size()

    depth = 1
    if dist is not None and not batched:
        from ros_gpu_depthmap_fusion_amd.multi import DeviceMarkExchange
        marks = DeviceMarkExchange(eng, ncells, world)
    else:
        depth = max(1, min(4, args.pipeline))
        eng.set_pipeline_depth(depth)
        if batched:
            from ros_gpu_depthmap_fusion_amd.multi import BatchedMarkExchange
            marks = BatchedMarkExchange(eng, ncells, world, args.exchange_batch)

    pc_plain = params.to_c(None, None, False, False)
    pc_defer = params.to_c(None, None, False, True)

    # the component's per-frame loop runs in C++ (gdf_run_depth_stream: clear + addDepthmapDevice
    # + gdf_process_frame per frame), as the ROS component would drive the engine
    scam = [eng.make_stream_camera([d.ptr for d in dframes[k]], W, H, *c.intrinsics(),
                                   c.T_world, c.T_crop) for k, c in enumerate(cams)]

    def run(first, count):
        if dist is None:
            eng.run_depth_stream(scam, pc_plain, first, count)
            return
        for i in range(first, first + count):
            eng.run_depth_stream(scam, pc_defer, i, 1)
            if batched:  # occupancy union over RCCL, `exchange_batch` frames per all-gather
                marks.take()
                if marks.full():
                    marks.flush(params.occupancy_lifetime)
            else:  # one all-gather per frame (multi.py)
                marks.exchange()
                eng.voxelOccupancyGrid(params.occupancy_lifetime)
        if batched:
            marks.flush(params.occupancy_lifetime)

    def barrier_sync():
        eng.synchronize()
        if dist is not None:
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    run(0, args.warmup)
    barrier_sync()
    t0 = time.perf_counter()
    run(args.warmup, args.steps)
    barrier_sync()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    # per-kernel durations: a separate pass over the same frames with an HIP event pair around
    # every launch on the engine stream (kept out of the timed region: the extra event records
    # cost host time)
    ktimes = None
    if not args.no_kernel_timing:
        kt_steps = min(args.steps, 200)
        if dist is None or batched:
            eng.set_pipeline_depth(1)  # one frame in flight: launch durations without overlap
        eng.set_profiling(True)
        run(args.warmup, kt_steps)
        barrier_sync()
        ktimes = eng.kernel_times()
        eng.set_profiling(False)

    ms_per_step = elapsed / args.steps * 1e3
    value = world * P * args.steps / elapsed / 1e6
    # frames used in the timed region, for the byte model
    idx = [(args.warmup + i) % args.ring for i in range(args.steps)]
    n_avg = float(np.mean([npts[i] for i in idx]))
    g_avg = float(np.mean([nvox[i] for i in idx]))
    tiles = (P + 255) // 256
    # algorithmic HBM bytes per launch of each kernel (DESIGN.md "Kernels and their rooflines"):
    # the bytes the algorithm must move once, not the cache traffic of an implementation
    model_bytes = {
        "mask": 3.0 * P,                           # u16 depth in, u8 stage bits out
        "scan": 8.0 * tiles,
        "emit": 1.0 * P + 22.0 * n_avg,            # stage in, depth of kept px, xyzw + key out
        # 3 radix passes (key only in, key+index out; then key+index both ways) + the grid
        # update carried by the first pass, averaged per launch
        "sort": (12.0 * n_avg + 16.0 * n_avg * 2 + 2.0 * ncells) / 3.0,
        # sorted keys + indices + gathered points in, means out
        "group": 24.0 * n_avg + 16.0 * g_avg,
        "grid": 2.0 * ncells,
    }
    survey_bytes = 2.0 * P + 24.0 * n_avg + 9.0 * ncells  # SURVEY.md §8(d) B_alg per frame

    roofline = None
    if ktimes:
        singles = [k for k in ("mask", "scan", "emit", "sort", "group", "grid")
                   if ktimes[k][1]]
        per_step = {k: ktimes[k][0] / kt_steps for k in singles}  # ms per step
        slot = max(singles, key=lambda k: per_step[k])
        ms, n = ktimes[slot]
        # An event pair costs stream time of its own.  An empty pair (slot event_floor, recorded
        # over the same frames) spans two record packets, a bracketed kernel carries one of them:
        # half the empty-pair time is subtracted (calibrated against rocprofv3 kernel-trace
        # durations of the same command, profiles/r01/).
        fl_ms, fl_n = ktimes.get("event_floor", (0.0, 0))
        floor_s = fl_ms / 1e3 / fl_n if fl_n else 0.0
        raw_s = ms / 1e3 / max(n, 1)
        avg_s = max(raw_s - 0.5 * floor_s, 1e-9)
        achieved = model_bytes[slot] / avg_s / 1e9
        traffic = None
        pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
        if os.path.exists(pmc):
            try:
                rec = json.load(open(pmc)).get(slot)
                if rec and rec.get("workload") == f"{W}x{H}":
                    traffic = rec.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        roofline = {
            "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
            "kernel": slot, "avg_launch_us": round(avg_s * 1e6, 3),
            "event_raw_us": round(raw_s * 1e6, 3), "event_floor_us": round(floor_s * 1e6, 3),
            "launches_per_step": round(n / kt_steps, 3),
            "bytes_per_launch": round(model_bytes[slot]),
            "per_kernel_us": {k: round(ktimes[k][0] * 1e3 / ktimes[k][1], 3) for k in singles},
            "step_survey_bytes": round(survey_bytes),
            "step_survey_GBps": round(survey_bytes * args.steps / elapsed / 1e9, 2),
        }

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        from oracle import OracleFusion  # cpu_baseline leg only
        threads = min(16, os.cpu_count() or 1)
        orc = OracleFusion(threads=threads)
        done, t_cpu = 0, 0.0
        for i in range(2):  # warm-up
            orc.clear()
            for k, c in enumerate(cams):
                orc.addDepthmap(frames[k][i % args.ring], *c.intrinsics(), c.T_world, c.T_crop)
            orc.processFrame(params)
        tc0 = time.perf_counter()
        while True:
            orc.clear()
            for k, c in enumerate(cams):
                orc.addDepthmap(frames[k][done % args.ring], *c.intrinsics(), c.T_world,
                                c.T_crop)
            orc.processFrame(params)
            done += 1
            t_cpu = time.perf_counter() - tc0
            if t_cpu >= args.cpu_seconds or done >= 2000:
                break
        cpu = {"value": round(done * P / t_cpu / 1e6, 3), "unit": "Mpoints/s", "cores": threads,
               "kind": "port",
               "sample": f"{done} frames of the same {W}x{H} C2 workload through the C "
                         f"restatement (oracle/gdf_oracle.c, OpenMP {threads} threads), "
                         f"{t_cpu:.1f} s"}

    if rank == 0:
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Mpoints/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (ray-cast analytic scene, counter-hash noise/holes; "
                    "device-resident ring of %d frames)" % args.ring,
            "config": {"workload": "C2: %dx%d u16 depth stream per GPU, launch defaults "
                                   "(F=4 thr 0.3, crop/voxel -10..30/-20..20/-1..1.5, "
                                   "cells 0.1/0.1/0.12 -> %dx%dx%d, voxelize average, "
                                   "lifetime 10)" % (W, H, gx, gy, gz),
                       "cameras_per_gpu": K, "points_per_frame_after_crop": round(n_avg),
                       "voxels_per_frame": round(g_avg), "grid_cells": ncells,
                       "frames_in_flight": depth,
                       "exchange": ("sparse mark pairs (cap %d words/frame), %d dense-fallback "
                                    "batches" % (marks.cap, marks.dense_batches)
                                    if batched else None),
                       "parallelism": ("camera-per-GPU x%d, occupancy-mark all-gather every %d "
                                       "frame(s)" % (world, args.exchange_batch if batched else 1))
                       if dist is not None else "single GPU"},
            "roofline": roofline,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
