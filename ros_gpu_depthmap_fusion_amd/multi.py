"""Multi-GPU exchange of the shared occupancy grid (one camera per rank).

The path shards per camera with no data exchange until the shared voxel grid.  The one real
exchange step is the occupancy union of a frame: every rank exports its occupancy marks as a
bitmask (cell c -> bit c % 32 of word c // 32, the layout of k_export_marks), the masks are
all-gathered, and every rank ORs all of them back into its engine before the identical
historic-grid update (voxel_grid_occupancy_of_points + decrement/max passes of the reference,
src/gpu_depthmap_fusion.cpp:1757-1823).  Occupancy is an idempotent union, so every rank's grid
equals the grid of one engine that saw all the cameras' points.

`torch.distributed` is the transport: backend "nccl" (RCCL over xGMI) for device tensors on the
GPU box, "gloo" for the CPU tests.
"""
from __future__ import annotations

import os

import numpy as np


def words_for(ncells: int) -> int:
    return (int(ncells) + 31) // 32


def pack_marks(marks: np.ndarray) -> np.ndarray:
    """bool/uint8 per cell -> uint32 words (bit c % 32 of word c // 32)."""
    m = np.asarray(marks).reshape(-1).astype(bool)
    pad = words_for(m.size) * 32 - m.size
    bits = np.packbits(np.concatenate([m, np.zeros(pad, bool)]).reshape(-1, 32)[:, ::-1],
                       axis=1, bitorder="big")
    return bits.view(">u4").astype(np.uint32).reshape(-1)


def unpack_marks(words: np.ndarray, ncells: int) -> np.ndarray:
    """inverse of pack_marks: bool per cell."""
    w = np.asarray(words, dtype=np.uint32).reshape(-1)
    bits = (w[:, None] >> np.arange(32, dtype=np.uint32)[None, :]) & 1
    return bits.reshape(-1)[:ncells].astype(bool)


def all_gather_or(words, group=None):
    """OR of every rank's mark words (a torch tensor of int32 words; CPU for gloo, device for
    nccl).  Returns a tensor of the same shape on every rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [torch.empty_like(words) for _ in range(world)]
    dist.all_gather(parts, words, group=group)
    out = parts[0].clone()
    for p in parts[1:]:
        out |= p
    return out


def historic_update(hist: np.ndarray, marks: np.ndarray, lifetime: int) -> np.ndarray:
    """The reference's per-frame grid update on a host u32 history: max(sat_dec(h), occ·L)
    (decrement_uints.glsl:31-51 + max_with_uints_times_scalar.glsl:36-46)."""
    dec = np.where(hist > 0, hist - 1, 0).astype(np.uint32)
    return np.maximum(dec, marks.astype(np.uint32) * np.uint32(lifetime)).astype(np.uint32)


class DeviceMarkExchange:
    """Per-frame exchange for GPU engines: export -> all-gather (RCCL) -> OR-import.

    Buffers are torch device tensors of the rank's GPU; the engine must run on the same stream
    as torch (GPUDepthmapFusion.set_stream(torch.cuda.current_stream().cuda_stream)) so the
    collective is ordered after the export and before the import."""

    def __init__(self, engine, ncells: int, world: int):
        import torch
        self.eng = engine
        self.words = words_for(ncells)
        self.world = world
        self.local = torch.zeros(self.words, dtype=torch.int32, device="cuda")
        self.gathered = torch.zeros(world * self.words, dtype=torch.int32, device="cuda")

    def exchange(self):
        import torch.distributed as dist
        self.eng.export_marks(self.local.data_ptr(), self.words)
        dist.all_gather_into_tensor(self.gathered, self.local)
        self.eng.import_marks(self.gathered.data_ptr(), self.words, self.world)


class BatchedMarkExchange:
    """The same exchange for `batch` frames per collective, with the engine's frames pipelined
    (gdf_set_pipeline_depth) instead of serialised behind a per-frame all-gather.

    Per frame (processed with defer_occupancy_grid): take() moves the frame's marks into slot i of
    a [batch, words] buffer and clears them in the engine.  flush(lifetime): one all-gather of the
    [batch, words] buffers of all ranks ([rank, batch, words]), then the batch's grid updates in
    ONE pass, frame after frame in registers (union of frame i: the masks at stride
    batch * words) - the grid equals that of the per-frame exchange."""

    def __init__(self, engine, ncells: int, world: int, batch: int, sparse_cap: int = -1):
        import torch
        self.eng = engine
        self.words = words_for(ncells)
        self.world = world
        self.batch = batch
        self.local = torch.zeros(batch * self.words, dtype=torch.int32, device="cuda")
        self.gathered = torch.zeros(world * batch * self.words, dtype=torch.int32, device="cuda")
        # sparse records: the non-zero mark words as (index, word) pairs (gdf_take_occupancy_marks
        # _sparse); the bitmasks travel only when some rank's frame has more than `cap`
        self.cap = max(1024, self.words // 16) if sparse_cap < 0 else sparse_cap
        self.rec = 1 + 2 * self.cap
        if self.cap:
            self.pairs = torch.zeros(batch * self.rec, dtype=torch.int32, device="cuda")
            self.gpairs = torch.zeros(world * batch * self.rec, dtype=torch.int32, device="cuda")
            self.union = torch.zeros(batch * self.words, dtype=torch.int32, device="cuda")
        self.n = 0
        self.dense_batches = 0

    def take(self):
        dst = self.local.data_ptr() + 4 * self.n * self.words
        if self.cap:
            self.eng.take_marks_sparse(dst, self.words,
                                       self.pairs.data_ptr() + 4 * self.n * self.rec, self.cap)
        else:
            self.eng.take_marks(dst, self.words)
        self.n += 1

    def full(self) -> bool:
        return self.n == self.batch

    def flush(self, lifetime: int):
        import torch
        import torch.distributed as dist
        if self.n == 0:
            return
        self.eng.synchronize()  # the takes (engine streams) before the collective (torch stream)
        dense = not self.cap
        if self.cap:
            dist.all_gather_into_tensor(self.gpairs, self.pairs)
            counts = self.gpairs.view(self.world, self.batch, self.rec)[:, :self.n, 0]
            dense = bool((counts > self.cap).any().item())  # same answer on every rank
        if dense:
            self.dense_batches += 1
            dist.all_gather_into_tensor(self.gathered, self.local)
            torch.cuda.current_stream().synchronize()  # the collective before the update
            self.eng.voxelOccupancyGridBatch(self.gathered.data_ptr(), self.words, self.world,
                                             self.n, self.words, self.batch * self.words,
                                             lifetime)
        else:
            torch.cuda.current_stream().synchronize()
            # only the n live frames of the (possibly partial) batch; records at stride batch
            self.eng.union_pairs(self.union.data_ptr(), self.words, self.gpairs.data_ptr(),
                                 self.world, self.n, self.rec, frames_per_rank=self.batch)
            self.eng.voxelOccupancyGridBatch(self.union.data_ptr(), self.words, 1, self.n,
                                             self.words, self.batch * self.words, lifetime)
        self.n = 0


# ---- fused voxel cloud across ranks -----------------------------------------
# The reference voxelizes the points of ALL cameras in one stable sort
# (src/gpu_depthmap_fusion.cpp:1743-1756, cameras concatenated at :1583-1626).  With one camera
# per rank the equal result is reached by one all-to-all of the compacted (point, key) lists by
# voxel-key range (gdf_partition_points): rank j receives the points of keys
# [ceil(j C / N), ceil((j+1) C / N)) from every rank, in rank order = camera order, pixel order
# inside each camera - the stable order of the single sort restricted to its key range - and
# voxelizes them (gdf_voxelize_points).  Each point crosses the fabric once (all-to-all), not N-1
# times (the all-gather the north star names).  The F-row halo: rank k's flying-pixel filter
# reads the last F rows + F pixels of camera k-1 at its top border; the ranks
# all-gather those tails (F*W + F depth values each) before the frame.

def part_slice_words(nparts: int, ncells: int) -> int:
    """Occupancy-mark words per key range: ceil(ceil(ncells / 32) / nparts)."""
    return ((ncells + 31) // 32 + nparts - 1) // nparts


def part_of_keys(keys: np.ndarray, nparts: int, ncells: int) -> np.ndarray:
    """Key-range owner of each key: min((key // 32) // S, nparts - 1), S = part_slice_words
    (k_part_count's rule: whole mark words per rank, so rank j's voxels mark exactly slice j of
    each frame's occupancy bitmask)."""
    S = np.uint64(part_slice_words(nparts, ncells))
    return np.minimum((keys.astype(np.uint64) >> np.uint64(5)) // S, nparts - 1).astype(np.int64)


def halo_pixels(F: int, width: int) -> int:
    """Depth values of camera k-1 that camera k's filter reads: F rows + F pixels."""
    return int(F) * int(width) + int(F)


def all_gather_tails(tail, group=None):
    """Every rank's depth tail (equal sizes) -> list indexed by rank."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    parts = [torch.empty_like(tail) for _ in range(world)]
    dist.all_gather(parts, tail, group=group)
    return parts


def exchange_points(send_pts, send_keys, counts, group=None):
    """All-to-all of part-major (point, key) send buffers: counts[j] items go to rank j.
    Returns (recv_pts [n, 4] float32, recv_keys [n] int32, recv_counts) in source-rank order.
    Tensors live on the collective's device (cuda for nccl, cpu for gloo)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = send_pts.device
    c = torch.as_tensor(counts, dtype=torch.int64, device=dev)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, c, group=group)
    rcounts = [int(x) for x in rc.cpu().tolist()]
    scounts = [int(x) for x in c.cpu().tolist()]
    n = sum(rcounts)
    rp = torch.empty((n, 4), dtype=torch.float32, device=dev)
    rk = torch.empty(n, dtype=torch.int32, device=dev)
    m = sum(scounts)
    dist.all_to_all_single(rp, send_pts[:m], output_split_sizes=rcounts,
                           input_split_sizes=scounts, group=group)
    dist.all_to_all_single(rk, send_keys[:m], output_split_sizes=rcounts,
                           input_split_sizes=scounts, group=group)
    return rp, rk, rcounts


def exchange_runs(send_pts, send_run_keys, send_run_starts, counts, runs, group=None):
    """exchange_points for the run form (gdf_partition_runs): counts[j] points and runs[j] runs
    go to rank j.  Returns (points, run keys, run starts, points per source, runs per source)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    mine = torch.tensor([[int(counts[j]), int(runs[j])] for j in range(world)], dtype=torch.int64)
    got = torch.zeros_like(mine)
    dist.all_to_all_single(got, mine, group=group)
    rc = [int(x) for x in got[:, 0].tolist()]
    rr = [int(x) for x in got[:, 1].tolist()]
    sc = [int(x) for x in counts]
    sr = [int(x) for x in runs]
    rp = torch.empty((sum(rc), 4), dtype=torch.float32)
    rk = torch.empty(sum(rr), dtype=torch.int32)
    rs = torch.empty(sum(rr), dtype=torch.int32)
    dist.all_to_all_single(rp, send_pts[:sum(sc)], output_split_sizes=rc, input_split_sizes=sc,
                           group=group)
    dist.all_to_all_single(rk, send_run_keys[:sum(sr)], output_split_sizes=rr,
                           input_split_sizes=sr, group=group)
    dist.all_to_all_single(rs, send_run_starts[:sum(sr)], output_split_sizes=rr,
                           input_split_sizes=sr, group=group)
    return rp, rk, rs, rc, rr


def exchange_points_dev(send_pts, send_keys, send_counts, group=None):
    """exchange_points for device tensors with the send counts still on the device (the
    partition's output): the counts' all-to-all runs on the device and ONE host read brings both
    the send and the receive split sizes (one synchronisation of the stream per exchange)."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    dev = send_pts.device
    c = send_counts.to(torch.int64)
    rc = torch.empty(world, dtype=torch.int64, device=dev)
    dist.all_to_all_single(rc, c, group=group)
    both = torch.cat([c, rc]).cpu().tolist()  # the one host synchronisation
    scounts, rcounts = [int(x) for x in both[:world]], [int(x) for x in both[world:]]
    n, m = sum(rcounts), sum(scounts)
    rp = torch.empty((n, 4), dtype=torch.float32, device=dev)
    rk = torch.empty(n, dtype=torch.int32, device=dev)
    dist.all_to_all_single(rp, send_pts[:m], output_split_sizes=rcounts,
                           input_split_sizes=scounts, group=group)
    dist.all_to_all_single(rk, send_keys[:m], output_split_sizes=rcounts,
                           input_split_sizes=scounts, group=group)
    return rp, rk, rcounts, scounts


class _SlotExchange:
    """Device / pinned buffers of the batch in flight on one engine slot (RCCL path): kept for the
    rank's lifetime so a collective on the slot's stream never reads memory the caching allocator
    handed to someone else; grown (after the slot's stream drained) when a batch needs more."""

    def __init__(self, world: int):
        import torch
        self.world = world
        self.cap = 0          # send capacity (points)
        self.rcap = 0         # receive capacity (points)
        self.mcap = 0         # mark words
        self.tcap = 0         # halo tail bytes
        # split sizes: (points, runs) per part - sent [world, 2], received [world, 2]
        self.cnt = torch.zeros(2 * world, dtype=torch.int32, device="cuda")
        self.c64 = torch.zeros((world, 2), dtype=torch.int64, device="cuda")
        self.rc = torch.zeros((world, 2), dtype=torch.int64, device="cuda")
        self.host = torch.zeros(4 * world, dtype=torch.int64, pin_memory=True)
        self.ev = torch.cuda.Event()
        self.pending = False

    def ensure(self, stream, n_send=0, n_recv=0, mark_words=0, tail_bytes=0):
        import torch
        grow = (n_send > self.cap or n_recv > self.rcap or mark_words > self.mcap or
                tail_bytes > self.tcap)
        if not grow:
            return
        stream.synchronize()  # the slot's previous batch no longer reads the old buffers
        if n_send > self.cap:
            self.cap = max(n_send, self.cap + self.cap // 2)
            self.sp = torch.empty((self.cap, 4), dtype=torch.float32, device="cuda")
            self.srk = torch.empty(self.cap, dtype=torch.int32, device="cuda")  # run keys
            self.srs = torch.empty(self.cap, dtype=torch.int32, device="cuda")  # run starts
        if n_recv > self.rcap:
            self.rcap = max(n_recv, self.rcap + self.rcap // 2)
            self.rp = torch.empty((self.rcap, 4), dtype=torch.float32, device="cuda")
            self.rrk = torch.empty(self.rcap, dtype=torch.int32, device="cuda")
            self.rrs = torch.empty(self.rcap + 1, dtype=torch.int32, device="cuda")
        if mark_words > self.mcap:
            self.mcap = mark_words
            self.local = torch.empty(mark_words, dtype=torch.int32, device="cuda")
            self.gathered = torch.empty(self.world * mark_words, dtype=torch.int32, device="cuda")
        if tail_bytes > self.tcap:
            self.tcap = tail_bytes
            self.tail = torch.empty(tail_bytes, dtype=torch.uint8, device="cuda")
            self.tails = torch.empty(self.world * tail_bytes, dtype=torch.uint8, device="cuda")


class FusedCloudRank:
    """One rank of the multi-GPU frame with the reference's fused output, over a GPU engine.

    Per step (one frame, or a batch of B frames through one launch chain): (halo) all-gather of
    the depth tails -> the rank's camera with camera k-1's tail as halo -> compaction + keys +
    marks (defer_voxelize, deferred grid) -> occupancy-mark union (all-gather) and the identical
    batched grid update on every rank -> key-range partition -> all-to-all -> voxelize of the
    rank's key range (the received list's runs of equal keys).  Collectives run on torch tensors
    of `dev` ("cuda": RCCL; "cpu": gloo, staged through host copies).

    RCCL path, pipelined (start / finish): the engine keeps `depth` batches in its pipeline slots,
    each slot's work and collectives on the slot's own stream.  start() runs a batch up to the
    all-to-all of its split sizes and queues their copy to pinned memory; finish() - called after
    the NEXT batch was started, so the GPU is busy while the host reads the sizes - runs the
    points all-to-all and the voxelize on the batch's slot.  The points travel on a second
    communicator (its own RCCL stream), so batch b's exchange never queues behind batch b + 1's
    mark / count collectives."""

    def __init__(self, engine, cams, rank: int, world: int, params, dev: str = "cuda",
                 depth: int = 1, mark_slices: bool = False, engine_streams: bool = False):
        import torch
        import torch.distributed as dist
        from . import hiprt
        self.eng, self.cams, self.rank, self.world, self.p = engine, cams, rank, world, params
        self.dev = dev
        self.hiprt = hiprt
        self.depth = max(1, int(depth)) if dev == "cuda" else 1
        self.streams = None
        self.engine_streams = False
        if dev == "cuda":
            engine.set_pipeline_depth(self.depth)
            # The slots' streams: torch streams by default (torch's allocator and the collectives
            # issued on them see streams that live as long as the process), or the engine's own
            # (engine_streams) wrapped as torch ExternalStreams.  Either way the slot tensors -
            # allocated by torch's caching allocator ON those streams - must be released before
            # the streams go: close() (then the engine's close) before destroy_process_group.
            # Round 4's teardown SIGSEGV was exactly that order reversed: the rank's __dict__
            # dropped the engine first (gdf_destroy: hipStreamDestroy of the slot streams), then
            # the slot tensors, whose free path in the caching allocator used the destroyed
            # streams (no Python frame on the faulthandler trace: a C-level tensor dealloc).
            self.engine_streams = bool(engine_streams)
            if not engine_streams:
                self.streams = [torch.cuda.Stream() for _ in range(self.depth)]
                engine.set_slot_streams([st.cuda_stream for st in self.streams])
            self.slots = {}
            # the points' communicator: its own RCCL stream (see the class docstring)
            self.pg_points = dist.new_group(list(range(world))) if world > 1 else None
        self.F = params.flying_filter_size
        # every rank sends the same number of tail values: the deepest read of any camera
        self.Lmax = max(halo_pixels(self.F, cams[k].width) for k in range(world))
        if any(cams[k].width * cams[k].height < self.Lmax for k in range(world)):
            raise ValueError("fused multi-GPU frames need cameras taller than F rows")
        self.pc = params.to_c(None, None, False, True, True)
        # The rollbuffer (point sequences, SURVEY §8(e): a single stream) lives on the LAST rank:
        # the reference appends the selected rollbuffer points after every camera's pixels, at
        # offset sum(P) (fusion.cpp:1509-1581, offsets :1525 / :1559), and sorts them together
        # with the depth points in one voxelize (:1743-1756).  The last rank compacts [its camera's
        # pixels, then the selected rollbuffer points] and partitions that list stably by key
        # range, so every key-range owner receives, in rank order, [camera 0 .. camera N-1 pixels,
        # rollbuffer points] - the reference's buffer order restricted to its range.
        self.rollbuffer_rank = world - 1
        self.has_rollbuffer = rank == self.rollbuffer_rank
        self._pc_move = {}  # to_c of the frames with move transforms (rollbuffer rank)
        self._staged = {}   # gloo path: the host-staged lists of a started batch
        self._keep = []
        # gloo path: the occupancy union as the C++ step builds it (gdf_fused.cpp) - no compaction
        # marks; the key-range voxelize marks its voxels (whole mark words per range,
        # part_of_keys) and the ranks all-gather those slices, not their full bitmasks
        self.mark_slices = bool(mark_slices) and dev != "cuda"
        if hasattr(engine, "set_partition_marks"):  # (the CPU tests' oracle stand-in has none)
            engine.set_partition_marks(not self.mark_slices)

    def _slot_stream(self, k):
        """Slot k's stream as a torch stream (the engine's slot k is the addressed slot)."""
        import torch
        if self.engine_streams:
            return torch.cuda.ExternalStream(self.eng.stream())
        return self.streams[k]

    def close(self):
        """Releases the slots' torch tensors (after their streams drained) and the streams, BEFORE
        the engine (and the process group) go - see __init__.  The engine stays."""
        import torch
        if self.dev == "cuda":
            self.eng.synchronize()
            torch.cuda.synchronize()
            self.slots = {}
            self._keep = []
            self._staged = {}
            self.streams = None

    def frame_params(self, move=None):
        """The frame's gdf_frame_params: `move` = (T_world_move, T_crop_move) when the component's
        tf lookup of the move frame succeeded (component.cpp:192-197) - used by the rollbuffer
        rank only (the other ranks hold no point sequences)."""
        if move is None or not self.has_rollbuffer:
            return self.pc
        key = tuple(np.asarray(move[0], np.float32).ravel()) + tuple(np.asarray(move[1], np.float32).ravel())
        pc = self._pc_move.get(key)
        if pc is None:
            if len(self._pc_move) > 64:
                self._pc_move.clear()
            pc = self._pc_move[key] = self.p.to_c(move[0], move[1], False, True, True)
        return pc

    # ---- one step, synchronous -------------------------------------------------------------------
    def frame(self, depth_ptr: int, tail_src_ptr: int, move=None):
        """One frame: depth_ptr = this rank's depth map (device), tail_src_ptr = its last
        Lmax depth values (device, the halo the next rank needs).  On the rollbuffer rank the
        point sequences added to the engine since the last frame (addPointSequence[Device]) are
        ingested, rolled and - with `move` - selected, transformed, cropped and compacted behind
        the camera's points.  Returns the send counts per rank."""
        return self.finish(self.start([depth_ptr], [tail_src_ptr], move))

    def batch(self, depth_ptrs, tail_src_ptrs):
        """B frames through one launch chain and ONE exchange: every rank's B tails in one
        all-gather (frame j's halo before frame j's depth map), the batch's compaction, the B
        frames' marks in one all-gather and one batched grid update (frame by frame in order),
        the (point, frame | key) lists partitioned by voxel-key range and exchanged once, and one
        voxelize of the rank's range - frame f's voxels of this range are
        eng.batch_ranges()[1][f:f+2]."""
        return self.finish(self.start(depth_ptrs, tail_src_ptrs))

    # ---- pipelined halves ---------------------------------------------------------------------
    def _slot(self, k):
        if k not in self.slots:
            self.slots[k] = _SlotExchange(self.world)
        return self.slots[k]

    def start(self, depth_ptrs, tail_src_ptrs, move=None):
        """Starts a step (1 frame or a batch) on the engine's next slot: everything up to the
        split sizes of the points all-to-all.  Returns the slot for finish()."""
        import torch
        import torch.distributed as dist
        h = self.hiprt
        eng, c = self.eng, self.cams[self.rank]
        B = len(depth_ptrs)
        L2 = 2 * self.Lmax
        halo = self.F > 0 and self.world > 1
        eng.clear()
        k = eng.slot() if self.dev == "cuda" else 0
        if self.dev == "cuda":
            S = self._slot(k)
            if S.pending:
                raise RuntimeError("FusedCloudRank.start: the slot's previous step is unfinished")
            st = self._slot_stream(k)
            S.ensure(st, tail_bytes=B * L2 if halo else 0)
            ctx = torch.cuda.stream(st)
        else:
            S, st, ctx = None, None, _nullctx()
        with ctx:
            halo_ptr = None
            if halo:
                # all ranks send Lmax values (the tail of their camera); rank k uses rank k-1's
                # (bytes: gloo has no 16-bit integer collectives)
                if self.dev == "cuda":
                    for j, src in enumerate(tail_src_ptrs):
                        h.copy_async(S.tail.data_ptr() + j * L2, src, L2, h.D2D, st.cuda_stream)
                    dist.all_gather_into_tensor(S.tails[:self.world * B * L2], S.tail[:B * L2])
                    if self.rank > 0:
                        halo_ptr = S.tails.data_ptr() + (self.rank - 1) * B * L2
                else:
                    tail = torch.from_numpy(np.concatenate(
                        [_d2h(h, src, np.uint8, L2) for src in tail_src_ptrs]))
                    parts = all_gather_tails(tail)
                    if self.rank > 0:
                        dh = h.DeviceArray.from_numpy(parts[self.rank - 1].numpy())
                        self._keep = [dh]
                        halo_ptr = dh.ptr
            for j in range(B):
                if j:
                    eng.nextFrameInBatch()
                if halo_ptr is not None:
                    pc_ = self.cams[self.rank - 1]
                    take = min(self.Lmax, pc_.width * pc_.height)
                    # the received tail holds camera k-1's last Lmax values (or all of a smaller one)
                    eng.addHaloDepthmapDevice(halo_ptr + j * L2 + 2 * (self.Lmax - take), take,
                                              pc_.width, pc_.height, *pc_.intrinsics(),
                                              pc_.T_world, pc_.T_crop)
                eng.addDepthmapDevice(depth_ptrs[j], c.width, c.height, *c.intrinsics(), c.T_world,
                                      c.T_crop)
            pc = self.frame_params(move) if B == 1 else self.pc
            # the send lists, written by the compaction itself (gdf_set_emit_partition): every
            # pixel of the step, and on the rollbuffer rank every point the window can select
            want = B * c.width * c.height
            if self.has_rollbuffer and B == 1 and pc.move_transform_available:
                want += (eng.rollbuffer_state().num_points +
                         eng.numCollectedPointSequencePoints())
            if self.dev == "cuda":
                S.ensure(st, n_send=max(want, 1))
                eng.set_emit_partition(self.world, S.sp.data_ptr(), S.srk.data_ptr(),
                                       S.srs.data_ptr(), S.cap, S.cnt.data_ptr())
            else:
                dsp, drk, drs = (h.DeviceArray(max(want, 1) * 16), h.DeviceArray(max(want, 1) * 4),
                                 h.DeviceArray(max(want, 1) * 4))
                dcnt = h.DeviceArray(2 * self.world * 4)
                eng.set_emit_partition(self.world, dsp.ptr, drk.ptr, drs.ptr, max(want, 1), dcnt.ptr)
            res = eng.processFramePrepared(pc)
            _, ncells = eng.grid_size()
            words = words_for(ncells)
            if self.dev == "cuda":
                S.ensure(st, mark_words=B * words)
                # occupancy union: the B frames' marks of every rank, one batched grid update
                eng.take_marks(S.local.data_ptr(), B * words)
                dist.all_gather_into_tensor(S.gathered[:self.world * B * words], S.local[:B * words])
                eng.voxelOccupancyGridBatch(S.gathered.data_ptr(), words, self.world, B, words,
                                            B * words, self.p.occupancy_lifetime)
                # the split sizes (points, runs) per part to the host without a stream sync
                S.c64.copy_(S.cnt.view(2, self.world).t())
                dist.all_to_all_single(S.rc, S.c64)
                S.host[:2 * self.world].copy_(S.c64.view(-1), non_blocking=True)
                S.host[2 * self.world:].copy_(S.rc.view(-1), non_blocking=True)
                S.ev.record(st)
                S.pending = True
            elif self.mark_slices:  # (the union after the voxelize: finish)
                eng.synchronize()
                self._staged[k] = ((B, words, ncells), dsp, drk, drs, dcnt)
            else:
                dl = h.DeviceArray(B * words * 4)
                eng.take_marks(dl.ptr, B * words)
                eng.synchronize()
                local = torch.from_numpy(dl.to_numpy(np.int32, B * words))
                parts = [torch.empty_like(local) for _ in range(self.world)]
                dist.all_gather(parts, local)
                dg = h.DeviceArray.from_numpy(torch.cat(parts).numpy())
                eng.voxelOccupancyGridBatch(dg.ptr, words, self.world, B, words, B * words,
                                            self.p.occupancy_lifetime)
                eng.synchronize()
                self._staged[k] = (dg, dsp, drk, drs, dcnt)
        return k

    def finish(self, k):
        """The points all-to-all and the voxelize of the step started on slot k.  Returns the
        send counts per rank."""
        import torch
        import torch.distributed as dist
        h = self.hiprt
        eng = self.eng
        if self.dev == "cuda":
            eng.select_slot(k)
            S = self.slots[k]
            if not S.pending:
                raise RuntimeError("FusedCloudRank.finish: no step in flight on this slot")
            st = self._slot_stream(k)
            S.ev.synchronize()  # (the slot's split sizes; the later slots keep the GPU busy)
            both = [int(x) for x in S.host.tolist()]
            W = self.world
            scounts, sruns = both[0:2 * W:2], both[1:2 * W:2]
            rcounts, rruns = both[2 * W::2], both[2 * W + 1::2]
            n, m, R, M = sum(rcounts), sum(scounts), sum(rruns), sum(sruns)
            S.ensure(st, n_recv=max(n, 1))
            with torch.cuda.stream(st):
                if self.world > 1 or n:
                    g = self.pg_points
                    dist.all_to_all_single(S.rp[:n], S.sp[:m], output_split_sizes=rcounts,
                                           input_split_sizes=scounts, group=g)
                    dist.all_to_all_single(S.rrk[:R], S.srk[:M], output_split_sizes=rruns,
                                           input_split_sizes=sruns, group=g)
                    dist.all_to_all_single(S.rrs[:R], S.srs[:M], output_split_sizes=rruns,
                                           input_split_sizes=sruns, group=g)
                eng.voxelize_runs(S.rp.data_ptr(), S.rrk.data_ptr(), S.rrs.data_ptr(),
                                  np.cumsum([0] + rcounts), np.cumsum([0] + rruns),
                                  self.p.voxel_average)
            S.pending = False
            return scounts
        dg, dsp, drk, drs, dcnt = self._staged.pop(k)
        c = dcnt.to_numpy(np.uint32, 2 * self.world).tolist()
        counts, runs = c[:self.world], c[self.world:]
        m, M = int(sum(counts)), int(sum(runs))
        sp = torch.from_numpy(dsp.to_numpy(np.float32, 4 * max(m, 1))[:4 * m].reshape(m, 4))
        srk = torch.from_numpy(drk.to_numpy(np.int32, max(M, 1))[:M])
        srs = torch.from_numpy(drs.to_numpy(np.int32, max(M, 1))[:M])
        rp, rrk, rrs, rc, rr = exchange_runs(sp, srk, srs, counts, runs)
        n, R = int(sum(rc)), int(sum(rr))
        drp = h.DeviceArray.from_numpy(rp.numpy()) if n else None
        drk2 = h.DeviceArray.from_numpy(rrk.numpy()) if R else None
        drs2 = h.DeviceArray.from_numpy(np.concatenate([rrs.numpy(), np.zeros(1, np.int32)]))
        if not self.mark_slices:
            eng.voxelize_runs(drp.ptr if n else 0, drk2.ptr if R else 0, drs2.ptr,
                              np.cumsum([0] + rc), np.cumsum([0] + rr), self.p.voxel_average)
            eng.synchronize()
            self._keep = [dg, drp, drk2, drs2]
            return counts
        B, words, ncells = dg
        Sw = part_slice_words(self.world, ncells)
        stride = Sw * self.world
        dmk = h.DeviceArray.from_numpy(np.zeros(B * stride, np.uint32))
        eng.voxelize_runs_marked(drp.ptr if n else 0, drk2.ptr if R else 0, drs2.ptr,
                                 np.cumsum([0] + rc), np.cumsum([0] + rr), dmk.ptr, stride,
                                 self.p.voxel_average)
        eng.synchronize()
        mk = dmk.to_numpy(np.uint32, B * stride).reshape(B, stride)
        mine = torch.from_numpy(np.ascontiguousarray(
            mk[:, self.rank * Sw:(self.rank + 1) * Sw]).view(np.int32))
        parts = [torch.empty_like(mine) for _ in range(self.world)]
        dist.all_gather(parts, mine)  # (each rank's slice of every frame)
        union = np.concatenate([q.numpy().view(np.uint32) for q in parts], axis=1)
        du = h.DeviceArray.from_numpy(np.ascontiguousarray(union))
        eng.voxelOccupancyGridBatch(du.ptr, words, 1, B, stride, B * stride, self.p.occupancy_lifetime)
        eng.synchronize()
        self._keep = [du, dmk, drp, drk2, drs2]
        return counts

    def run(self, steps, depth_ptrs_of, tail_ptrs_of, move_of=None, on_finish=None):
        """`steps` steps through the pipeline: step i's inputs from depth_ptrs_of(i) /
        tail_ptrs_of(i) (/ move_of(i)); up to `depth` steps in flight: step i - depth + 1 is
        finished right after step i started (the GPU computes the later steps while the host waits
        for the oldest one's split sizes).
        on_finish(i) runs after step i's finish (e.g. publishing its cloud)."""
        pending = []
        depth = self.depth if self.dev == "cuda" else 1
        for i in range(steps):
            k = self.start(depth_ptrs_of(i), tail_ptrs_of(i), move_of(i) if move_of else None)
            pending.append((i, k))
            if len(pending) >= depth:  # (`depth` steps in flight; the oldest one's slot is next)
                j, kk = pending.pop(0)
                self.finish(kk)
                if on_finish:
                    on_finish(j)
        for j, kk in pending:
            self.finish(kk)
            if on_finish:
                on_finish(j)


class LocalFusedWorld:
    """`world` ranks of the C++ fused step in ONE process (include/gdf_fused.h gdf_fused_local):
    one engine and one host thread per rank, the step's collectives as device copies on the ranks'
    streams.  The multi-rank C++ step on one GPU (RCCL refuses two ranks on one device); a rank is
    NativeFusedRank(..., local=this)."""

    def __init__(self, world: int, lib=None):
        import ctypes as C
        from .gdf import load_library
        self._lib = lib or load_library()
        self.world = world
        h = C.c_void_p()
        rc = self._lib.gdf_fused_local_create(world, C.byref(h))
        if rc:
            raise RuntimeError("gdf_fused_local_create: %d" % rc)
        self.handle = h

    def run(self, fn, timeout: float = 600.0):
        """fn(rank) on `world` threads (ctypes drops the GIL inside the library calls); returns
        their results in rank order, re-raises the first failure."""
        import threading
        out, err = [None] * self.world, [None] * self.world

        def body(r):
            try:
                out[r] = fn(r)
            except BaseException as e:  # noqa: BLE001 - handed to the caller
                err[r] = e

        ts = [threading.Thread(target=body, args=(r,), daemon=True) for r in range(self.world)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout)
        if any(t.is_alive() for t in ts):
            raise TimeoutError("local fused ranks still running after %.0f s" % timeout)
        for e in err:
            if e is not None:
                raise e
        return out

    def close(self):
        if getattr(self, "handle", None):
            rc = self._lib.gdf_fused_local_destroy(self.handle)
            if rc:
                raise RuntimeError("gdf_fused_local_destroy: %d (ranks still alive)" % rc)
            self.handle = None


def rccl_library_path() -> str:
    """The librccl torch loaded (torch/lib/librccl.so), so the C++ rank and torch share one RCCL."""
    import torch
    p = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return p if os.path.exists(p) else "librccl.so"


class NativeFusedRank:
    """FusedCloudRank's RCCL path with the step in C++ (include/gdf_fused.h, csrc/gdf_fused.cpp):
    the halo / mark / split-size all-gathers, the grid update, the partition and the grouped
    send / recv of the (point, key) lists issued by libgdf on the engine slots' streams over two
    RCCL communicators of its own (ids broadcast over the default process group) - no Python,
    torch op or host copy between the launches of a step.  Same start / finish / run / frame /
    batch interface and results as FusedCloudRank(dev="cuda")."""

    def __init__(self, engine, cams, rank: int, world: int, params, depth: int = 1, local=None):
        """local: a LocalFusedWorld - the rank is one of `world` ranks of THIS process (one host
        thread and one engine each) exchanging through device copies (gdf_fused_create_local);
        None: one rank per process over RCCL (ids broadcast over the default process group)."""
        import ctypes as C
        from . import hiprt
        from .gdf import StreamCamera
        self.eng, self.cams, self.rank, self.world, self.p = engine, cams, rank, world, params
        self.dev, self.hiprt = "cuda", hiprt
        self.depth = max(1, min(4, int(depth)))
        self._lib = engine._lib
        self.F = params.flying_filter_size
        sc = (StreamCamera * world)()
        for k in range(world):
            c = cams[k]
            sc[k].ring, sc[k].width, sc[k].height = 0, c.width, c.height
            sc[k].depth_scale, sc[k].fx, sc[k].fy, sc[k].cx, sc[k].cy = c.intrinsics()
            sc[k].T_world[:] = np.asarray(c.T_world, np.float32).ravel().tolist()
            sc[k].T_crop[:] = np.asarray(c.T_crop, np.float32).ravel().tolist()
        self._cams_c = sc
        h = C.c_void_p()
        engine.set_pipeline_depth(self.depth)
        self.local = local
        if local is not None:
            engine._check(self._lib.gdf_fused_create_local(engine.handle, local.handle, rank, world,
                                                           sc, self.F, C.byref(h)))
        else:
            import torch.distributed as dist
            path = rccl_library_path().encode()
            ids = (C.c_uint8 * 256)()
            if rank == 0:
                engine._check(self._lib.gdf_fused_unique_id(path, ids))
            obj = [bytes(ids)]
            dist.broadcast_object_list(obj, src=0)
            ids = (C.c_uint8 * 256).from_buffer_copy(obj[0])
            engine._check(self._lib.gdf_fused_create(engine.handle, path, ids, rank, world, sc,
                                                     self.F, C.byref(h)))
        self._h = h
        L = C.c_uint32()
        engine._check(self._lib.gdf_fused_halo_pixels(h, C.byref(L)))
        self.Lmax = L.value
        self.pc = params.to_c(None, None, False, True, True)
        self.rollbuffer_rank = world - 1
        self.has_rollbuffer = rank == self.rollbuffer_rank
        self._pc_move = {}

    def shard_rollbuffer(self, block: int):
        """gdf_fused_set_rollbuffer_shard: the rollbuffer window spread over the ranks - every
        rank is given EVERY point sequence and keeps those of blocks (k // block) % world == rank;
        every rank's steps then carry its share of the selection (before the first sequence)."""
        self.eng._check(self._lib.gdf_fused_set_rollbuffer_shard(self._h, int(block)))
        self.has_rollbuffer = block > 0 or self.rank == self.rollbuffer_rank
        self.shard_block = int(block)

    def info(self):
        """(rank, world, the rank count the transport reports, transport name)."""
        import ctypes as C
        r, w, n, k = C.c_int(), C.c_int(), C.c_int(), C.c_char_p()
        self.eng._check(self._lib.gdf_fused_info(self._h, C.byref(r), C.byref(w), C.byref(n),
                                                 C.byref(k)))
        return r.value, w.value, n.value, k.value.decode()

    frame_params = FusedCloudRank.frame_params

    def close(self):
        """Destroys the C++ rank (its communicators, buffers); the engine stays."""
        if getattr(self, "_h", None):
            self._lib.gdf_fused_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def start(self, depth_ptrs, tail_src_ptrs=None, move=None):
        """gdf_fused_start (the halo tails are the depth maps' last Lmax values: tail_src_ptrs is
        accepted for FusedCloudRank's signature and not read)."""
        import ctypes as C
        arr = (C.c_void_p * len(depth_ptrs))(*depth_ptrs)
        k = C.c_int()
        p = self.frame_params(move) if len(depth_ptrs) == 1 else self.pc
        self.eng._check(self._lib.gdf_fused_start(self._h, arr, len(depth_ptrs), C.byref(p),
                                                  C.byref(k)))
        return k.value

    def finish(self, k):
        import ctypes as C
        sc = (C.c_uint32 * self.world)()
        n = C.c_uint32()
        self.eng._check(self._lib.gdf_fused_finish(self._h, k, sc, C.byref(n)))
        return list(sc)

    def frame(self, depth_ptr: int, tail_src_ptr: int = 0, move=None):
        return self.finish(self.start([depth_ptr], None, move))

    def batch(self, depth_ptrs, tail_src_ptrs=None):
        return self.finish(self.start(depth_ptrs))

    run = FusedCloudRank.run

    def run_stream(self, frame_ptrs, first: int, steps: int, batch: int):
        """gdf_fused_run: `steps` pipelined steps of `batch` frames from the device ring
        frame_ptrs (step s takes frames (first + s) * batch + j), no Python per step."""
        import ctypes as C
        from .gdf import StreamCamera
        c = self.cams[self.rank]
        sc = StreamCamera()
        arr = (C.c_void_p * len(frame_ptrs))(*frame_ptrs)
        sc.frames = C.cast(arr, C.POINTER(C.c_void_p))
        sc.ring, sc.width, sc.height = len(frame_ptrs), c.width, c.height
        sc.depth_scale, sc.fx, sc.fy, sc.cx, sc.cy = c.intrinsics()
        sc.T_world[:] = np.asarray(c.T_world, np.float32).ravel().tolist()
        sc.T_crop[:] = np.asarray(c.T_crop, np.float32).ravel().tolist()
        self.eng._check(self._lib.gdf_fused_run(self._h, C.byref(sc), C.byref(self.pc), first,
                                                steps, batch, self.depth))


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def gather_fused_cloud(rank_obj, root: int = 0):
    """The fused voxel cloud on rank `root`: every rank's voxels (its key range of the frame's -
    or the batch's - m_points_voxelized) concatenated in rank order, which is ascending key order,
    i.e. the reference's single voxelize over all cameras (fusion.cpp:1743-1756) as the component
    publishes it (component.cpp:389-461).  Returns an (n, 4) float32 tensor on root (device for
    "cuda", host for "cpu"), None elsewhere.  One count all-gather (one host read) + one gather
    of the padded voxel lists."""
    import torch
    import torch.distributed as dist
    eng, world, dev = rank_obj.eng, rank_obj.world, rank_obj.dev
    h = rank_obj.hiprt
    rank = dist.get_rank()
    if dev == "cuda":
        n = eng.voxelized_count()  # (reads the engine's count: the stream has run voxelize)
        cnt = torch.tensor([n], dtype=torch.int64, device="cuda")
        allc = torch.empty(world, dtype=torch.int64, device="cuda")
        dist.all_gather_into_tensor(allc, cnt)
        counts = [int(x) for x in allc.cpu().tolist()]
        mx = max(max(counts), 1)
        mine = torch.zeros((mx, 4), dtype=torch.float32, device="cuda")
        if n:
            vptr = eng.device_results()[2]
            h.copy_async(mine.data_ptr(), vptr, 16 * n, h.D2D, torch.cuda.current_stream().cuda_stream)
    else:
        vox = eng.downloadVoxelizedPoints()
        n = len(vox)
        allc = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(allc, torch.tensor([n], dtype=torch.int64))
        counts = [int(x.item()) for x in allc]
        mx = max(max(counts), 1)
        mine = torch.zeros((mx, 4), dtype=torch.float32)
        mine[:n] = torch.from_numpy(vox)
    parts = [torch.empty_like(mine) for _ in range(world)] if rank == root else None
    dist.gather(mine, parts, dst=root)
    if rank != root:
        return None
    return torch.cat([parts[r][:counts[r]] for r in range(world)])


def _d2h(h, ptr, dtype, count):
    out = np.empty(count, dtype)
    h.check(h.hip().hipMemcpy(out.ctypes.data, ptr, out.nbytes, h.D2H), "D2H")
    return out
