#!/usr/bin/env python3
"""Benchmark of the depth -> points -> flying-pixel -> crop -> voxel-occupancy hot path.

Workload (BASELINE.json configs[1], "C2"): one 640x480 16-bit synthetic depth stream per GPU,
launch-file defaults (flying-pixel F=4, thr 0.3; crop = voxel bounds -10..30 x -20..20 x -1..1.5,
cells 0.1/0.1/0.12 -> 400x400x21 = 3.36 M cells; voxelize with averaging; lifetime 10).
A step = one full frame of GPUDepthmapFusionComponent::processDepthmaps on the GPU: fused
convert+flying+crop+ordered compaction+voxel keys+occupancy marks, GPU voxelize (radix sort +
ordered means), historic-grid update.  Frames are device-resident (a ring of distinct frames
generated once and uploaded before timing).  The default frames are the realistic-density set
(synth.dense_frame: ~65 % of the pixels survive the flying-pixel filter); `--workload stress` is
round 1's independent-noise set.

Before the timed region every engine slot has captured its frame graph (`prime`, independent of
--warmup), so the steady state does not depend on --steps / --warmup.

N = 1 also reports, in "secondary", the same line for 720p and 4K depth, the stress frames, the
C2 frame with a host-resident depth map (pinned, H2D overlapped: `value_h2d`), and C3 (720p +
256-sequence rollbuffer window, tools/bench_c3.py) - each with the roofline of its dominant kernel.

N > 1 (torchrun, one rank per GPU over RCCL): rank k owns camera k (weak scaling).  The shared
voxel grid needs one real exchange per frame: the per-rank occupancy marks (1 bit per cell) are
all-gathered and OR-merged before every rank's identical historic-grid update.  `--exchange-batch
1` (default) exchanges every frame, as the reference component updates and downloads the grid per
frame (component.cpp:297,306); B > 1 is the deferred-grid mode (the grid is brought up to date
every B frames, labelled as such in `config`).

Prints ONE JSON line (rank 0).
"""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpoints/s end-to-end depth→fused voxel grid @1/2/4/8 GPU; % HBM roofline"
HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
SINGLE_SLOTS = ("mask", "scan", "emit", "sort", "group", "grid", "sel")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--workload", choices=("dense", "stress"), default="dense")
    ap.add_argument("--ring", type=int, default=32, help="distinct device-resident frames")
    ap.add_argument("--batch", type=int, default=8,
                    help="frames per launch chain (gdf_next_frame_in_batch); a step is one "
                         "batch, value counts every frame's pixels")
    ap.add_argument("--cameras", type=int, default=1,
                    help="cameras per GPU (one frame = one depth map of each; camera ids "
                         "rank*cameras + k)")
    ap.add_argument("--pipeline", type=int, default=3,
                    help="frames in flight on one GPU (engine slots, gdf_set_pipeline_depth); "
                         "N > 1 runs on torch's stream with depth 1")
    ap.add_argument("--multi-mode", choices=("fused", "marks"), default="fused",
                    help="N > 1: fused = the reference's output over all cameras (halo, mark "
                         "union, key-range all-to-all + voxelize); marks = occupancy union only")
    ap.add_argument("--exchange-batch", type=int, default=1,
                    help="N > 1: frames per occupancy-mark all-gather (1 = every frame, the "
                         "reference's per-frame grid; B > 1 = deferred grid, B frames per "
                         "all-gather)")
    ap.add_argument("--dist-backend", choices=("nccl", "gloo"), default="nccl",
                    help="N > 1: RCCL (default) or gloo with host-staged tensors (smoke runs of "
                         "several ranks on one GPU)")
    ap.add_argument("--dist", action="store_true",
                    help="the multi-GPU (torch.distributed) path even at one rank (RCCL at world 1)")
    ap.add_argument("--fused-impl", choices=("native", "python"), default="native",
                    help="RCCL fused mode: the step in C++ with libgdf's own RCCL calls "
                         "(gdf_fused_*, default) or multi.FusedCloudRank's torch collectives")
    ap.add_argument("--publish", action="store_true",
                    help="fused mode: gather the fused voxel cloud to rank 0 every step (the "
                         "component publishes it every frame)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="per CPU run (5 runs)")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="do not bracket launches with HIP events (for rocprofv3 runs)")
    ap.add_argument("--h2d-only", action="store_true",
                    help="only the host-depth-map (H2D-inclusive) line, as JSON")
    ap.add_argument("--no-secondary", action="store_true",
                    help="N = 1: skip the 720p / 4K / stress / H2D / C3 lines")
    ap.add_argument("--c3-window", type=int, default=256)
    ap.add_argument("--transport", choices=("rccl", "local"), default="rccl",
                    help="N > 1 fused mode: rccl = one process per GPU (torchrun, or started by "
                         "this script); local = N ranks of the C++ step in THIS process on one "
                         "GPU (gdf_fused_local: one engine + host thread per rank, device copies "
                         "as the collectives) - exercises the multi-rank step, not a scaling run")
    ap.add_argument("--rb-shard", action="store_true",
                    help="with --rb-window (C++ step): the window sharded over the ranks "
                         "(gdf_fused_set_rollbuffer_shard) instead of held by the last rank")
    ap.add_argument("--rb-window", type=int, default=0,
                    help="N > 1 fused mode: the last rank also runs a rollbuffer of this many "
                         "720p point sequences, one new sequence per step (C5 with its rollbuffer)")
    return ap.parse_args()


def radix_passes(ncells, B=1):
    """Radix passes of the voxelize sort (gdf_device.hpp radix_passes): the voxel-key bits plus
    the frame bits of a batch, 8-bit digits, a 9-bit last digit when that saves a pass (<= 25)."""
    bits = max(int(ncells - 1).bit_length(), 0) + (int(B - 1).bit_length() if B > 1 else 0)
    if bits == 0:
        return 1
    if bits <= 25:
        return 1 if bits <= 9 else (bits + 6) // 8
    return (bits + 7) // 8


def grid_update_bytes(ncells, B=1, snap_bytes=0.0):
    """Algorithmic bytes of one (batched) grid update: the u8 grid read and written once, each
    frame's 1-bit marks read, and the sparse snapshots of the frames but the last (4-B index +
    32 B per non-zero 32-cell group) - not dense per-frame grids."""
    return 2.0 * ncells + B * ncells / 8.0 + snap_bytes


def model_bytes(P, n_avg, g_avg, ncells, B=1, s_avg=None, runs=False, snap_bytes=0.0):
    """Algorithmic HBM bytes per launch of each kernel: the bytes the algorithm
    must move once, not the cache traffic of an implementation.  A launch of a B-frame batch
    processes B frames (P, n, g per frame); its grid update (carried by the first radix pass)
    reads and writes the grid once, reads the B frames' marks and writes the sparse snapshots of
    the B - 1 intermediate grids (snap_bytes, counted from the frames' grids).  s_avg: the items
    the voxelize sorts per frame - the points, or (runs) the runs of equal voxel keys, which the
    sort and the group phase then move instead of points."""
    P, n_avg, g_avg = B * P, B * n_avg, B * g_avg
    s_items = B * (s_avg if s_avg is not None else n_avg / B)
    tiles = (P + 255) // 256
    npass = radix_passes(ncells, B)
    grid = grid_update_bytes(ncells, B, snap_bytes)
    return {
        "mask": 3.0 * P,                           # u16 depth in, u8 stage bits out
        "scan": 8.0 * tiles,
        # stage in, depth of kept px, xyzw + key out (+ key and first point of each run)
        "emit": 1.0 * P + 22.0 * n_avg + (8.0 * s_items if runs else 0.0),
        # radix passes over the sorted items (key only in, key+index out; then key+index both
        # ways) + the grid update carried by the first pass, averaged per launch
        "sort": (12.0 * s_items + 16.0 * s_items * (npass - 1) + grid) / npass,
        # sorted keys + indices (+ the runs' point ranges) in, points in, means out
        "group": (16.0 * n_avg + 16.0 * s_items if runs else 24.0 * n_avg) + 16.0 * g_avg,
        "grid": grid,
    }


def roofline_from(ktimes, kt_steps, mb, pmc_key):
    """The dominant kernel (largest total time per step) of an event-timed pass, its average
    launch duration and algorithmic bytes per launch."""
    singles = [k for k in SINGLE_SLOTS if ktimes[k][1] and k in mb]
    per_step = {k: ktimes[k][0] / kt_steps for k in singles}
    slot = max(singles, key=lambda k: per_step[k])
    ms, n = ktimes[slot]
    # An event pair costs stream time of its own.  An empty pair (slot event_floor, recorded over
    # the same frames) spans two record packets, a bracketed kernel carries one of them: half the
    # empty-pair time is subtracted (calibrated against rocprofv3 kernel-trace durations of the
    # same command, profiles/).
    fl_ms, fl_n = ktimes.get("event_floor", (0.0, 0))
    floor_s = fl_ms / 1e3 / fl_n if fl_n else 0.0
    raw_s = ms / 1e3 / max(n, 1)
    avg_s = max(raw_s - 0.5 * floor_s, 1e-9)
    achieved = mb[slot] / avg_s / 1e9
    traffic, traffic_src = None, None
    allrec = pmc_record(pmc_key)
    rec = slot_pmc(allrec, slot)
    if rec:
        traffic = rec["hbm_bytes_per_launch"]
        traffic_src = {"kernels": rec["kernels"], "dispatches": rec["dispatches"],
                       "source": "profiles/pmc_traffic.json[%s]" % pmc_key}
    # every timed slot's PMC traffic against its byte model (profiles/pmc_traffic.json, one
    # batch in flight): > 1 = bytes the model does not count (partial-sector writes, re-reads)
    pk_traffic = {}
    for k in singles:
        r = slot_pmc(allrec, k)
        if r and mb.get(k):
            pk_traffic[k] = {"model_bytes": round(mb[k]), "pmc_bytes": r["hbm_bytes_per_launch"],
                             "ratio": round(r["hbm_bytes_per_launch"] / mb[k], 3),
                             "kernels": r["kernels"]}
    valu = None
    sq = os.path.join(ROOT, "profiles", "pmc_sq.json")
    if slot == "mask" and os.path.exists(sq):
        # k_mask is bound by neither HBM nor MFMA: its VALU issue rate beside the HBM fraction.
        # VALU instructions per wave from the committed SQ counters of this workload
        # (profiles/pmc_sq.json), one wave per 64 x (pixels per thread) pixels of the launch
        # (mb["mask"] = 3 B per pixel), a wave64 VALU instruction issues in 2 cycles on a SIMD
        # (MI355X_MICROARCH.md), 1024 SIMDs at 2.4 GHz.
        try:
            rec = json.load(open(sq)).get(pmc_key, {}).get("mask")
        except Exception:
            rec = None
        if rec:
            waves = mb["mask"] / 3.0 / rec.get("pixels_per_wave", 64)
            issue = waves * rec["valu_per_wave"] * 2.0 / (1024 * 2.4e9 * avg_s)
            valu = {"insts_per_wave": rec["valu_per_wave"], "waves_per_launch": round(waves),
                    "issue_frac": round(issue, 4), "wait_frac": rec["wait_frac"],
                    "source": "profiles/pmc_sq.json"}
    return {
        "valu": valu,
        "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS,
        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 5), "traffic": traffic,
        "traffic_src": traffic_src,
        "kernel": slot, "avg_launch_us": round(avg_s * 1e6, 3),
        "event_raw_us": round(raw_s * 1e6, 3), "event_floor_us": round(floor_s * 1e6, 3),
        "launches_per_step": round(n / kt_steps, 3),
        "bytes_per_launch": round(mb[slot]),
        "per_kernel_us": {k: round(ktimes[k][0] * 1e3 / ktimes[k][1], 3) for k in singles},
        "per_kernel_traffic": pk_traffic or None,
    }


# the kernels an event-timed slot brackets (the engine's HookScope in gdf_kernels.hip): the group
# slot is the whole group phase - the tile count, the staged groups and the queued long groups
SLOT_PMC = {"group": ("group", "group_count", "group_big"), "scan": ("scan", "scan_reduce")}


def slot_pmc(allrec, slot):
    """PMC bytes per launch of a timed SLOT: the bytes of every kernel the slot brackets, per
    dispatch of its main kernel ({} when none was recorded)."""
    base = allrec.get(slot)
    if not base or not base.get("dispatches"):
        return {}
    tot, kernels = 0.0, []
    for k in SLOT_PMC.get(slot, (slot,)):
        r = allrec.get(k)
        if r and r.get("dispatches"):
            tot += r["hbm_bytes_per_launch"] * r["dispatches"]
            kernels += r.get("kernels") or [k]
    return {"hbm_bytes_per_launch": round(tot / base["dispatches"]), "kernels": kernels,
            "dispatches": base["dispatches"]}


def pmc_record(pmc_key):
    """The committed PMC traffic of a workload (tools/pmc_traffic.py): {slot: record, "_step":
    bytes per bench step}; {} when none was recorded."""
    pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        return json.load(open(pmc)).get(pmc_key, {}) or {}
    except (OSError, ValueError):
        return {}


class DepthStream:
    """One GPU's camera stream: device-resident frames, the engine, the component loop."""

    def __init__(self, eng, W, H, K, rank, workload, ring, host_frames=False):
        import numpy as np
        from ros_gpu_depthmap_fusion_amd import hiprt, synth
        self.W, self.H, self.K, self.ring = W, H, K, ring
        self.P = W * H * K
        self.eng = eng
        gen = synth.WORKLOADS[workload]
        self.cams = [synth.make_camera(rank * K + k, W, H) for k in range(K)]
        self.frames = [[gen(c, rank * K + k, f) for f in range(ring)]
                       for k, c in enumerate(self.cams)]
        self.dframes = [[hiprt.DeviceArray.from_numpy(f) for f in fr] for fr in self.frames]
        self.host = None
        if host_frames:  # pinned host copies: the H2D-inclusive path
            self.host = [[hiprt.PinnedArray.from_numpy(f) for f in fr] for fr in self.frames]
        self.scam = [eng.make_stream_camera(
            [d.ptr for d in (self.host[k] if host_frames else self.dframes[k])], W, H,
            *c.intrinsics(), c.T_world, c.T_crop) for k, c in enumerate(self.cams)]
        self.np = np

    def counts(self, params):
        """Per-frame point / voxel counts (byte model), one synchronous pass over the ring."""
        npts, nvox = [], []
        for i in range(self.ring):
            self.eng.clear()
            for k, c in enumerate(self.cams):
                self.eng.addDepthmapDevice(self.dframes[k][i].ptr, self.W, self.H,
                                           *c.intrinsics(), c.T_world, c.T_crop)
            r = self.eng.processFrame(params, synchronous=True)
            npts.append(r.num_points)
            nvox.append(r.num_voxelized)
        return npts, nvox

    def sort_items(self, params, batch):
        """Items one batch's voxelize sorts per frame (runs of equal keys in run mode), from one
        synchronous batched frame, and whether they are runs."""
        self.eng.clear()
        for j in range(batch):
            if j:
                self.eng.nextFrameInBatch()
            for k, c in enumerate(self.cams):
                self.eng.addDepthmapDevice(self.dframes[k][j % self.ring].ptr, self.W, self.H,
                                           *c.intrinsics(), c.T_world, c.T_crop)
        self.eng.processFrame(params, synchronous=True)
        items, runs = self.eng.last_sort_items()
        # the batch's sparse grid snapshots (frames but the last): 36 B per non-zero 32-cell group
        np = self.np
        snap = 0
        for f in range(batch - 1):
            g = self.eng.downloadBatchVoxelOccupancyGrid(f)
            pad = (-len(g)) % 32
            g32 = np.concatenate([g, np.zeros(pad, np.uint8)]).reshape(-1, 32)
            snap += 36 * int(np.count_nonzero(g32.any(axis=1)))
        return items / batch, runs, snap

    def run(self, pc, first, count, batch=1):
        """`count` steps of `batch` frames from frame `first * batch` on."""
        if batch > 1:
            self.eng.run_depth_stream_batched(self.scam, pc, first * batch, count, batch,
                                              self.host is not None)
        elif self.host is not None:
            self.eng.run_host_stream(self.scam, pc, first, count)
        else:
            self.eng.run_depth_stream(self.scam, pc, first, count)


SETTLE_S = 0.25


def settle(eng, run_some, seconds=SETTLE_S):
    """Untimed steps for `seconds` of wall time before the warm-up: the GPU's clocks and power
    state ramp up under sustained load, and a short timed region (the driver's 20 steps of a
    batch are ~2 ms) must not start on a GPU that was idle a moment ago."""
    t = time.perf_counter()
    while time.perf_counter() - t < seconds:
        run_some()
    eng.synchronize()


def time_single(st, params, steps, warmup, depth, kernel_timing, pmc_key, batch=1):
    """Steady-state single-GPU line of one DepthStream: prime (every slot's graph captured),
    warm-up, K timed steps (a step = one batch of `batch` frames), then the event-timed pass for
    the roofline."""
    import numpy as np
    eng = st.eng
    npts, nvox = st.counts(params)
    (gx, gy, gz), ncells = eng.grid_size()
    eng.set_pipeline_depth(depth)
    pc = params.to_c(None, None, False, False)
    # prime: a slot captures its graph on its second steady frame; 2 rounds over the slots + 1
    prime = 2 * depth + 2
    st.run(pc, 0, prime, batch)
    settle(eng, lambda: st.run(pc, 0, 2 * depth + 2, batch))
    st.run(pc, prime, warmup, batch)
    eng.synchronize()
    t0 = time.perf_counter()
    st.run(pc, prime + warmup, steps, batch)
    eng.synchronize()
    elapsed = time.perf_counter() - t0
    idx = [((prime + warmup + i) * batch + j) % st.ring for i in range(steps) for j in range(batch)]
    n_avg = float(np.mean([npts[i] for i in idx]))
    g_avg = float(np.mean([nvox[i] for i in idx]))
    s_avg, runs, snap = st.sort_items(params, batch)
    mb = model_bytes(st.P, n_avg, g_avg, ncells, batch, s_avg, runs, snap)
    roof = None
    if kernel_timing:
        kt_steps = min(steps, 200)
        eng.set_pipeline_depth(1)  # one frame in flight: launch durations without overlap
        eng.set_profiling(True)
        st.run(pc, prime + warmup, kt_steps, batch)
        eng.synchronize()
        kt = eng.kernel_times()
        eng.set_profiling(False)
        roof = roofline_from(kt, kt_steps, mb, pmc_key)
    # SURVEY.md §8(d) B_alg per frame, times the frames of a step
    survey = batch * (2.0 * st.P + 24.0 * n_avg + 9.0 * ncells)
    # bytes the step actually moves (PMC FETCH x2 + WRITE of every kernel of a steady step, one
    # batch in flight, profiles/pmc_traffic.json) over the measured step time
    step_pmc = pmc_record(pmc_key).get("_step", {}).get("hbm_bytes_per_step")
    pmc_line = {}
    if step_pmc:
        gbps = step_pmc * steps / elapsed / 1e9
        pmc_line = {"step_pmc_bytes": step_pmc, "step_pmc_GBps": round(gbps, 2),
                    "step_pmc_frac": round(gbps / HBM_PEAK_GBPS, 4)}
    return {
        "value": round(st.P * batch * steps / elapsed / 1e6, 3),
        "ms_per_step": round(elapsed / steps * 1e3, 5),
        "frames_per_step": batch, "ms_per_frame": round(elapsed / steps / batch * 1e3, 5),
        "steps": steps, "warmup": warmup, "prime": prime,
        "points_per_frame_after_crop": round(n_avg), "voxels_per_frame": round(g_avg),
        "survival_after_crop": round(n_avg / st.P, 4),
        "grid": [gx, gy, gz], "grid_cells": ncells, "frames_in_flight": depth,
        "step_survey_bytes": round(survey),
        "step_survey_GBps": round(survey * steps / elapsed / 1e9, 2),
        "step_survey_frac": round(survey * steps / elapsed / 1e9 / HBM_PEAK_GBPS, 4),
        "step_survey_note": "SURVEY 8(d) B_alg (counts a u32 history this build never moves)",
        **pmc_line,
        "model_bytes_per_launch": {k: round(v) for k, v in mb.items()},
        "roofline": roof,
    }


def cgroup_cpu_quota():
    """CPUs this process may use per the cgroup v2 cpu.max (None: unlimited / unknown)."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def cpu_baseline(st, params, seconds):
    """The C restatement (oracle/gdf_oracle.c, OpenMP) on the host's cores: median of 5 runs of
    `seconds` each over the same frames (SURVEY.md §8(d) protocol)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    from oracle import OracleFusion  # cpu_baseline leg only
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    env_t = os.environ.get("OMP_NUM_THREADS")
    threads = min(affinity, int(env_t)) if env_t and env_t.isdigit() else affinity
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    orc = OracleFusion(threads=threads)

    def frame(i):
        orc.clear()
        for k, c in enumerate(st.cams):
            orc.addDepthmap(st.frames[k][i % st.ring], *c.intrinsics(), c.T_world, c.T_crop)
        orc.processFrame(params)

    for i in range(3):  # warm-up
        frame(i)
    rates, total_frames = [], 0
    for run in range(5):
        done, t0 = 0, time.perf_counter()
        while True:
            frame(done)
            done += 1
            t = time.perf_counter() - t0
            if t >= seconds or done >= 4000:
                break
        rates.append(done * st.P / t / 1e6)
        total_frames += done
    out = {"value": round(statistics.median(rates), 3), "unit": "Mpoints/s", "cores": threads,
           "kind": "port", "threads": threads, "nproc": os.cpu_count(),
           "affinity_cpus": affinity, "cpu_model": model,
           "runs_Mpoints_s": [round(r, 2) for r in rates],
           "min": round(min(rates), 3), "max": round(max(rates), 3),
           "spread": round((max(rates) - min(rates)) / max(statistics.median(rates), 1e-9), 3),
            "sample": f"median of 5 runs x {seconds:.0f} s ({total_frames} frames) of the same "
                      f"{st.W}x{st.H} frames through the C restatement (oracle/gdf_oracle.c, "
                      f"-O3 -ffp-contract=off, OpenMP {threads} threads = the pool's "
                      f"OMP_NUM_THREADS share of this GPU's host)"}
    # one thread, one run: a per-core figure that does not depend on the host's other tenants
    # sharing the thread pool's CPUs (the multi-thread median moved 49.5 -> 85 Mpoints/s between
    # rounds on the same pool)
    orc.set_threads(1)
    frame(0)
    done, t0 = 0, time.perf_counter()
    while True:
        frame(done)
        done += 1
        t = time.perf_counter() - t0
        if t >= seconds or done >= 4000:
            break
    out["single_thread_Mpoints_s"] = round(done * st.P / t / 1e6, 3)
    orc.set_threads(threads)
    quota = cgroup_cpu_quota()
    if quota is not None:
        out["cgroup_cpu_quota"] = round(quota, 2)
    if quota is not None and quota < affinity and quota <= threads * 1.05:
        # the CPUs beyond the quota only time-slice it (a 256-thread run under a 16-CPU quota
        # measured 0.41 Mpoints/s, 160x below the 16-thread run)
        out["all_cpus"] = {"skipped": "cgroup cpu.max quota of %.1f CPUs: the %d-thread run "
                                      "already uses this host's whole CPU allowance" % (quota, threads)}
    elif affinity > threads:  # and every CPU of the host (nproc), a short sample
        orc.set_threads(affinity)
        frame(0)
        rates_all = []
        for run in range(3):
            done, t0 = 0, time.perf_counter()
            while True:
                frame(done)
                done += 1
                t = time.perf_counter() - t0
                if t >= 1.0 or done >= 4000:
                    break
            rates_all.append(done * st.P / t / 1e6)
        out["all_cpus"] = {"value": round(statistics.median(rates_all), 3), "threads": affinity,
                           "runs_Mpoints_s": [round(r, 2) for r in rates_all],
                           "sample": "median of 3 runs x 1 s, OpenMP %d threads" % affinity}
    return out


def workload_name(W, H, K, wl):
    cams = "" if K == 1 else f"{K}x"
    return (f"{cams}{W}x{H} u16 depth ({wl} frames), launch defaults (F=4 thr 0.3, crop/voxel "
            f"-10..30/-20..20/-1..1.5, cells 0.1/0.1/0.12, voxelize average, lifetime 10)")


_JSON_FD = None  # the process's original stdout (the one JSON line goes there)


def emit(obj):
    os.write(_JSON_FD if _JSON_FD is not None else 1, (json.dumps(obj) + "\n").encode())


def launch_ranks(args) -> int:
    """`--gpus N` without a launcher: start N rank processes of this script under
    torch.distributed.run (127.0.0.1 rendezvous) as CHILDREN - before this process touches a GPU -
    and return their exit status (rank 0 prints the JSON line)."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           "--nproc-per-node=%d" % args.gpus, "--master-addr", "127.0.0.1",
           "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "4"))
    return subprocess.run(cmd, env=env).returncode


def main():
    # Library chatter on stdout (RCCL's version banner at communicator creation, ...) would break
    # the one-JSON-line contract: fd 1 points at stderr for the run, the line goes to the original.
    global _JSON_FD
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ and args.transport == "rccl":
        sys.exit(launch_ranks(args))  # (no GPU call has been made in this process)
    sys.stdout.flush()
    _JSON_FD = os.dup(1)
    os.dup2(2, 1)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    dist = None
    rank, local_rank = 0, 0
    if args.transport == "local" and args.gpus > 1:
        emit(time_local(args))
        return
    if args.gpus > 1 or world > 1 or args.dist:
        import torch
        import torch.distributed as dist
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if args.dist_backend == "gloo":  # (host-staged collectives: a smoke run of N ranks on
            local_rank %= max(1, torch.cuda.device_count())  # fewer GPUs)
            torch.cuda.set_device(local_rank)
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local_rank)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
        world = dist.get_world_size()
        if world != max(1, args.gpus):
            raise SystemExit("bench: %d ranks started for --gpus %d" % (world, args.gpus))
    import numpy as np
    from ros_gpu_depthmap_fusion_amd import build_library, hiprt
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion

    build_library()
    hiprt.set_device(local_rank)
    W, H, K = args.width, args.height, args.cameras
    params = ComponentParams()
    if args.h2d_only:
        emit(run_h2d(args, params, args.steps, args.warmup))
        return
    eng = GPUDepthmapFusion(local_rank)
    st = DepthStream(eng, W, H, K, rank, args.workload, args.ring)
    P = st.P
    pmc_key = f"{W}x{H}/{args.workload}" + (f"/b{args.batch}" if args.batch > 1 else "")

    if dist is None:
        line = time_single(st, params, args.steps, args.warmup, max(1, min(4, args.pipeline)),
                           not args.no_kernel_timing, pmc_key, max(1, args.batch))
        cfg_extra = {"parallelism": "single GPU", "exchange": None}
    else:
        line, cfg_extra = time_multi(args, st, params, dist, world, pmc_key)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(st, params, args.cpu_seconds)

    secondary = None
    if rank == 0 and world == 1 and not args.no_secondary:
        secondary = run_secondary(args, params)

    if rank == 0:
        roof = line.pop("roofline")
        out = {
            "metric": METRIC, "value": line.pop("value"), "unit": "Mpoints/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": line.pop("ms_per_step"),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (ray-cast analytic scene, %s frames; device-resident ring of %d "
                    "frames)" % (args.workload, args.ring),
            "config": dict({"workload": "C2: " + workload_name(W, H, K, args.workload) + (
                                "; a step = a batch of %d frames through one launch chain "
                                "(every frame's points, voxel means and grid)" % args.batch
                                if args.batch > 1 and (dist is None or args.multi_mode == "fused")
                                else ""),
                            "cameras_per_gpu": K}, **line, **cfg_extra),
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if secondary is not None:
            out["secondary"] = secondary
        emit(out)
    if dist is not None:
        eng.close()  # (the engine's streams before the process group: DESIGN.md §6, teardown)
        dist.barrier()
        dist.destroy_process_group()


def time_multi(args, st, params, dist, world, pmc_key):
    """N > 1: every rank runs its camera.  Mode "fused" (default): the reference's output over
    all cameras - camera k-1's depth tail as halo (all-gather), occupancy-mark union (all-gather
    + OR, every rank the same grid), key-range all-to-all of the (point, key) lists and the
    voxelize of each rank's range (multi.FusedCloudRank).  Mode "marks": only the occupancy union
    (voxel means per camera), `--exchange-batch` frames per all-gather."""
    import numpy as np
    import torch
    eng = st.eng
    npts, nvox = st.counts(params)
    (gx, gy, gz), ncells = eng.grid_size()
    depth = 1
    fused = args.multi_mode == "fused"
    rb = None
    native = False
    if fused:
        from ros_gpu_depthmap_fusion_amd import synth
        from ros_gpu_depthmap_fusion_amd.multi import (FusedCloudRank, NativeFusedRank,
                                                       gather_fused_cloud)
        rank = dist.get_rank()
        cams = [synth.make_camera(k, st.W, st.H) for k in range(world)]
        cuda = args.dist_backend == "nccl"
        native = cuda and args.fused_impl == "native"
        # pipelined steps (RCCL): `--pipeline` batches in the engine's slots, a step's points
        # exchange finished while the next step computes
        if native:
            fr = NativeFusedRank(eng, cams, rank, world, params, depth=max(1, min(4, args.pipeline)))
        else:
            fr = FusedCloudRank(eng, cams, rank, world, params, dev="cuda" if cuda else "cpu",
                                depth=max(1, min(4, args.pipeline)) if cuda else 1)
        depth = fr.depth
        n = st.W * st.H
        B = max(1, args.batch)
        if args.rb_window:
            if B != 1:
                raise SystemExit("--rb-window: frames carrying point sequences run one per step "
                                 "(--batch 1)")
            if args.rb_shard:
                if not native:
                    raise SystemExit("--rb-shard: the C++ step (--fused-impl native, nccl)")
                # blocks of ceil((window - 1) / (world - 1)) sequences: the window spans at most
                # `world` blocks, one per rank (include/gdf_fused.h)
                fr.shard_rollbuffer(max(1, -(-(args.rb_window - 1) // max(world - 1, 1))))
            rb = RollbufferFeed(eng, args.rb_window, params) if fr.has_rollbuffer else None
            params.ps_timespan = (args.rb_window - 0.5) / 30.0
            fr.p = params
            fr.pc = params.to_c(None, None, False, True, True)
            fr._pc_move.clear()

        def ptrs(i):
            return [st.dframes[0][(i * B + j) % st.ring].ptr for j in range(B)]

        ring = [d.ptr for d in st.dframes[0]]

        def run(first, count):
            if native and rb is None and not args.publish:  # the C++ step loop (gdf_fused_run)
                fr.run_stream(ring, first, count, B)
                return
            fr.run(count, lambda i: ptrs(first + i),
                   lambda i: [d + 2 * (n - fr.Lmax) for d in ptrs(first + i)],
                   move_of=(lambda i: rb.feed(first + i)) if rb is not None else None,
                   on_finish=(lambda j: gather_fused_cloud(fr, root=0)) if args.publish else None)
    else:
        batched = args.exchange_batch > 1
        if batched:
            from ros_gpu_depthmap_fusion_amd.multi import BatchedMarkExchange
            depth = max(1, min(4, args.pipeline))
            eng.set_pipeline_depth(depth)
            marks = BatchedMarkExchange(eng, ncells, world, args.exchange_batch)
        else:
            from ros_gpu_depthmap_fusion_amd.multi import DeviceMarkExchange
            eng.set_stream(torch.cuda.current_stream().cuda_stream)
            marks = DeviceMarkExchange(eng, ncells, world)
        pc_defer = params.to_c(None, None, False, True)

        def run(first, count):
            for i in range(first, first + count):
                st.run(pc_defer, i, 1)
                if batched:
                    marks.take()
                    if marks.full():
                        marks.flush(params.occupancy_lifetime)
                else:
                    marks.exchange()
                    eng.voxelOccupancyGrid(params.occupancy_lifetime)
            if batched:
                marks.flush(params.occupancy_lifetime)

    def barrier_sync():
        eng.synchronize()
        torch.cuda.synchronize()
        dist.barrier()
        torch.cuda.synchronize()

    prime = 2 * depth + 2
    if rb is not None:
        rb.fill()  # the window's sequences before the first timed step
    run(0, prime)
    # (the settle of time_single, as a fixed step count: every rank must run the same number of
    # exchanges)
    run(0, 200)
    run(prime, args.warmup)
    barrier_sync()
    t0 = time.perf_counter()
    run(prime + args.warmup, args.steps)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    t = torch.tensor([elapsed], dtype=torch.float64,
                     device="cuda" if args.dist_backend == "nccl" else "cpu")
    allt = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(allt, t)
    per_rank = [round(float(x.item()) / args.steps * 1e3, 5) for x in allt]
    elapsed = max(float(x.item()) for x in allt)  # (the max over ranks)
    fpb = max(1, args.batch) if fused else 1  # frames per step
    idx = [((prime + args.warmup + i) * fpb + j) % st.ring for i in range(args.steps)
           for j in range(fpb)]
    n_avg = float(np.mean([npts[i] for i in idx]))
    g_avg = float(np.mean([nvox[i] for i in idx]))
    line = {
        "value": round(world * st.P * fpb * args.steps / elapsed / 1e6, 3),
        "frames_per_step": fpb,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5), "prime": prime,
        "points_per_frame_after_crop": round(n_avg), "voxels_per_frame": round(g_avg),
        "grid": [gx, gy, gz], "grid_cells": ncells, "frames_in_flight": depth,
        "ms_per_step_per_rank": per_rank,
        "roofline": None,
    }
    if rb is not None or (fused and args.rb_window):
        line["rollbuffer"] = {"window_sequences": args.rb_window,
                              "rank": "all (sharded)" if args.rb_shard else world - 1,
                              "sequence_points": RollbufferFeed.POINTS,
                              "note": "sharded: every rank holds ~1/N of the window" if args.rb_shard
                                      else "the last rank holds the rollbuffer (SURVEY 8(e))",
                              "balance": "gpu_ms_per_step_per_rank: each rank's event-timed GPU "
                                         "work per step"}
    if not args.no_kernel_timing:
        kt_steps = min(args.steps, 100)
        if depth > 1:
            eng.synchronize()
            eng.set_pipeline_depth(1)
            if fused:
                fr.depth = 1
        eng.set_profiling(True)
        run(prime + args.warmup, kt_steps)
        barrier_sync()
        kt = eng.kernel_times()
        eng.set_profiling(False)
        line["roofline"] = roofline_from(kt, kt_steps, model_bytes(st.P, n_avg, g_avg, ncells, fpb),
                                         pmc_key)
        # each rank's GPU work per step (its event-timed launches): the load (im)balance that the
        # barrier-to-barrier times above hide
        g = torch.tensor([sum(ms for ms, _ in kt.values()) / kt_steps], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        allg = [torch.zeros_like(g) for _ in range(world)]
        dist.all_gather(allg, g)
        line["gpu_ms_per_step_per_rank"] = [round(float(x.item()), 5) for x in allg]
    transport_ranks = dist.get_world_size()
    if fused and native:
        transport_ranks = fr.info()[2]  # (ncclCommCount of the step's points communicator)
    if fused:
        fr.close()  # (its communicators / slot tensors, before the engine and the process group)
    if fused:
        cfg = {"parallelism": "camera-per-GPU x%d; per step of %d frames (one launch chain): "
                              "depth-tail halo all-gather, occupancy-mark all-gather + batched "
                              "grid update, key-range all-to-all of the (point, frame | key) "
                              "lists, voxelize per key range (fused cloud = one engine over all "
                              "cameras, per frame)%s%s" % (
                                  world, fpb, "; fused cloud gathered to rank 0 every step"
                                  if args.publish else "",
                                  "; the step in C++ (gdf_fused_run), RCCL called from libgdf on "
                                  "the slots' streams, two communicators" if native else
                                  "; torch.distributed collectives (multi.FusedCloudRank)"),
               "exchange": "per step of %d frames: halo %d px + %d-word marks per frame, one "
                           "points all-to-all" % (fpb, fr.Lmax, (ncells + 31) // 32),
               "transport_ranks": transport_ranks}
    else:
        cfg = {"parallelism": "camera-per-GPU x%d, occupancy-mark all-gather %s (voxel means per "
                              "camera)" % (world, "every frame" if not batched else
                                           "every %d frames (deferred grid)" % args.exchange_batch),
               "exchange": ("sparse mark pairs (cap %d words/frame), %d dense-fallback batches" %
                            (marks.cap, marks.dense_batches)) if batched else "bitmask per frame",
               "transport_ranks": transport_ranks}
    return line, cfg


def time_local(args):
    """`--transport local --gpus N`: N ranks of the C++ fused step (gdf_fused_run) in this process on
    ONE GPU - one engine, one host thread and one camera each, the collectives as device copies
    (multi.LocalFusedWorld).  The ranks share the GPU, so the rate is the step's throughput with N
    cameras on one device, not a scaling number (n_gpus: 1)."""
    import numpy as np
    from ros_gpu_depthmap_fusion_amd import build_library, synth
    from ros_gpu_depthmap_fusion_amd.gdf import ComponentParams, GPUDepthmapFusion
    from ros_gpu_depthmap_fusion_amd.multi import LocalFusedWorld, NativeFusedRank
    build_library()
    N, W, H, B = args.gpus, args.width, args.height, max(1, args.batch)
    params = ComponentParams()
    depth = max(1, min(4, args.pipeline))
    lw = LocalFusedWorld(N)
    cams = [synth.make_camera(k, W, H) for k in range(N)]
    streams = [DepthStream(GPUDepthmapFusion(0), W, H, 1, r, args.workload, args.ring)
               for r in range(N)]
    ranks = [NativeFusedRank(st.eng, cams, r, N, params, depth=depth, local=lw)
             for r, st in enumerate(streams)]
    info = ranks[0].info()
    rings = [[d.ptr for d in st.dframes[0]] for st in streams]

    def run(first, count):
        lw.run(lambda r: ranks[r].run_stream(rings[r], first, count, B))
        for st in streams:
            st.eng.synchronize()

    prime = 2 * depth + 2
    run(0, prime + 100)
    run(prime, args.warmup)
    t0 = time.perf_counter()
    run(prime + args.warmup, args.steps)
    elapsed = time.perf_counter() - t0
    for fr in ranks:
        fr.close()
    lw.close()
    P = W * H
    return {
        "metric": METRIC, "value": round(N * P * B * args.steps / elapsed / 1e6, 3),
        "unit": "Mpoints/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 5), "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "data": "synthetic (ray-cast analytic scene, %s frames)" % args.workload,
        "config": {"workload": "%d ranks x %s, a step = a batch of %d frames per rank" % (
                       N, workload_name(W, H, 1, args.workload), B),
                   "parallelism": "%d ranks of the C++ fused step (gdf_fused_run) in one process "
                                  "on one GPU, in-process transport (%s, %d ranks)" % (
                                      N, info[3], info[2]),
                   "ranks": N, "frames_in_flight": depth,
                   "note": "diagnostic: N cameras' fused step sharing ONE GPU, not a scaling run"},
        "roofline": None, "cpu_baseline": None,
    }


class RollbufferFeed:
    """The point-sequence stream of the rollbuffer rank (C5 "full rollbuffer"): C3's sequences -
    a 720p lidar frame back-projected, 921 600 points, T_move(k) = 0.01 k m along x, 30 per
    second - device-resident PointCloud2 records (two, alternated) added one per step; fill()
    ingests a full window first."""
    POINTS = 1280 * 720

    def __init__(self, eng, window, params):
        import numpy as np
        from ros_gpu_depthmap_fusion_amd import hiprt, synth
        self.eng, self.window, self.synth = eng, window, synth
        self.lidar = synth.make_camera(1, 1280, 720)
        recs = [np.concatenate([synth.back_project(self.lidar, synth.dense_frame(self.lidar, 1, f)),
                                np.ones((self.POINTS, 1), np.float32)], 1) for f in range(2)]
        self.dev = [hiprt.DeviceArray.from_numpy(r) for r in recs]
        self.k = 0

    def _add(self):
        s, ns = self.synth.sequence_time(self.k)
        self.eng.addPointSequenceDevice(self.dev[self.k % 2].ptr, self.POINTS, 16, s, ns,
                                        self.synth.move_transform(self.k))
        self.k += 1

    def fill(self):
        for _ in range(self.window - 1):
            self._add()

    def feed(self, i):
        """Step i: one new sequence, and the move transforms of the frame."""
        self._add()
        return (self.lidar.T_world, self.lidar.T_crop)


def run_alternating(args, params, steps, warm):
    """C2 batches with two parameter sets alternating step by step: graphs on (per-slot graph
    cache) vs direct launches (graphs off)."""
    import copy
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    p2 = copy.copy(params)
    p2.flying_threshold = params.flying_threshold + 0.01
    pcs = [params.to_c(None, None, False, False), p2.to_c(None, None, False, False)]
    batch = 1  # the component's frame-by-frame flow (batches take direct launches anyway)
    r = {"workload": "C2 single VGA frames (3 in flight), flying threshold %.2f / %.2f alternating "
                     "every frame" % (params.flying_threshold, p2.flying_threshold)}
    for graphs in (True, False):
        eng = GPUDepthmapFusion(0)
        st = DepthStream(eng, args.width, args.height, 1, 0, args.workload, args.ring)
        st.counts(params)
        eng.set_graphs(graphs)
        depth = max(1, min(4, args.pipeline))
        eng.set_pipeline_depth(depth)
        prime = 4 * depth + 4
        c0 = eng.graph_stats()
        eng.run_depth_stream_alternating(st.scam, pcs, 0, prime + warm, batch)
        eng.synchronize()
        t0 = time.perf_counter()
        eng.run_depth_stream_alternating(st.scam, pcs, prime + warm, steps, batch)
        eng.synchronize()
        el = time.perf_counter() - t0
        key = "graph_cache" if graphs else "direct_launches"
        r[key] = {"value": round(st.P * batch * steps / el / 1e6, 3),
                  "ms_per_step": round(el / steps * 1e3, 5)}
        if graphs:
            c1 = eng.graph_stats()
            r[key]["graph_captures_replays"] = [c1[0] - c0[0], c1[1] - c0[1]]
        del st
        eng.close()
    r["value"] = r["graph_cache"]["value"]
    r["ms_per_step"] = r["graph_cache"]["ms_per_step"]
    return r


def run_component_sync(args, params, frames=300, warm=20):
    """The reference component's per-frame sequence, synchronous, one frame at a time
    (GPUDepthmapFusionComponent::processDepthmaps, component.cpp:92-306): a host depth image
    (cv_bridge) -> addDepthmap -> the frame (uploadDepthmaps ... voxelOccupancyGrid) -> the
    downloads the component makes every frame: downloadPoints, downloadVoxelCoords, the voxelized
    points (published as out/Points, component.cpp:389-461) and downloadVoxelOccupancyGrid.  The
    latency per frame (median, p99) and the rate of one such stream."""
    import numpy as np
    from ros_gpu_depthmap_fusion_amd import synth
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    W, H = args.width, args.height
    cam = synth.make_camera(0, W, H)
    ring = [synth.WORKLOADS[args.workload](cam, 0, f) for f in range(8)]
    pc = params.to_c(None, None, False)  # (the frame's wait is the download's)

    def stream(per_call):
        eng = GPUDepthmapFusion(0)
        lat = []
        for i in range(warm + frames):
            t0 = time.perf_counter()
            eng.clear()
            eng.addDepthmap(ring[i % len(ring)], *cam.intrinsics(), cam.T_world, cam.T_crop)
            if per_call:  # downloadPoints / downloadVoxelCoords / ... one call (and wait) each
                eng.processFrame(params, synchronous=True)
                out = [eng.downloadPoints(), eng.downloadVoxelCoords(),
                       eng.downloadVoxelizedPoints(), eng.downloadVoxelOccupancyGrid()]
            else:  # gdf_download_frame: the four copies into pinned mirrors, one wait
                eng.processFramePrepared(pc)
                out = list(eng.download_frame().values())
            if i >= warm:
                lat.append(time.perf_counter() - t0)
        nbytes = int(sum(a.nbytes for a in out))
        eng.close()
        return np.array(lat), nbytes

    lat, nbytes = stream(False)
    lat_pc, _ = stream(True)
    return {"workload": "C2 component-equivalent: one %dx%d host depth frame at a time, "
                        "synchronous, with the per-frame downloads (points, voxel coords, "
                        "voxelized points, u8 grid) through gdf_download_frame" % (W, H),
            "value": round(W * H * len(lat) / lat.sum() / 1e6, 3),
            "latency_ms_median": round(float(np.median(lat)) * 1e3, 4),
            "latency_ms_p99": round(float(np.percentile(lat, 99)) * 1e3, 4),
            "frames": len(lat),
            "download_bytes_per_frame": nbytes,
            "per_call_downloads": {
                "latency_ms_median": round(float(np.median(lat_pc)) * 1e3, 4),
                "latency_ms_p99": round(float(np.percentile(lat_pc, 99)) * 1e3, 4),
                "note": "the same frames with the four per-call downloads (one wait each, "
                        "pageable destinations)"}}


def run_h2d(args, params, steps, warm):
    """C2 from HOST depth maps: each frame's map is copied into the slot's pinned staging by
    GDF_H2D_THREADS host threads and DMA'd on the slot's stream, overlapped with the kernels of the
    frames in flight."""
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    eng = GPUDepthmapFusion(0)
    st = DepthStream(eng, args.width, args.height, 1, 0, args.workload, args.ring,
                     host_frames=True)
    r = time_single(st, params, steps, warm, max(1, min(4, args.pipeline)), False, "", args.batch)
    r["workload"] = "C2 with host (pinned) depth maps: " + workload_name(
        args.width, args.height, 1, args.workload)
    r["value_h2d"] = r.pop("value")
    r["h2d_threads"] = int(os.environ.get("GDF_H2D_THREADS", "4"))  # (the engine default)
    r["h2d_GBps"] = round(2.0 * args.width * args.height * args.batch / (r["ms_per_step"] / 1e3) / 1e9, 2)
    del st
    eng.close()
    return r


def run_secondary(args, params):
    """N = 1 only: the other single-GPU configurations, each with its own roofline."""
    from ros_gpu_depthmap_fusion_amd.gdf import GPUDepthmapFusion
    out = {}
    # (at least 200 steps: a 50-step single-frame line times ~2 ms and moves by tens of % with
    # host launch jitter)
    steps = max(args.steps, 200)
    warm = max(args.warmup, 10)
    kt = not args.no_kernel_timing
    for name, (W, H, wl, ring, st_steps, B) in {
            "vga_single_frame": (640, 480, "dense", 8, steps, 1),
            "vga_batch4": (640, 480, "dense", 32, steps, 4),
            "720p": (1280, 720, "dense", 4, steps, 4),
            "720p_single_frame": (1280, 720, "dense", 4, steps, 1),
            "4k": (3840, 2160, "dense", 2, max(20, steps // 4), 1),
            "vga_stress": (640, 480, "stress", 8, steps, args.batch)}.items():
        eng = GPUDepthmapFusion(0)
        st = DepthStream(eng, W, H, 1, 0, wl, ring)
        r = time_single(st, params, st_steps, warm, max(1, min(4, args.pipeline)), kt,
                        f"{W}x{H}/{wl}" + (f"/b{B}" if B > 1 else ""), B)
        r["workload"] = workload_name(W, H, 1, wl)
        out[name] = r
        del st
        eng.close()
    # runtime parameter changes (component.cpp:970-990): two flying-pixel thresholds alternating
    # every step - one cached graph per (slot, set) - and the same stream with graphs off
    out["vga_alternating_params"] = run_alternating(args, params, steps, warm)
    out["vga_h2d"] = run_h2d(args, params, steps, warm)
    out["component_sync"] = run_component_sync(args, params)
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        from bench_c3 import run_c3
        out["c3"] = run_c3(window=args.c3_window, steps=20, ring=4, profile_steps=5)
    except Exception as exc:  # reported, not hidden
        out["c3"] = {"error": repr(exc)}
    try:  # objectSegmentation front end on the grid of the C2-style stream
        from bench_seg import run_seg
        out["segmentation"] = run_seg(frames=16, reps=20)
    except Exception as exc:
        out["segmentation"] = {"error": repr(exc)}
    return out


if __name__ == "__main__":
    main()
