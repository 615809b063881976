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

def part_of_keys(keys: np.ndarray, nparts: int, ncells: int) -> np.ndarray:
    """Key-range owner of each key: floor(key * nparts / ncells) (k_part_count's rule)."""
    return np.minimum((keys.astype(np.uint64) * np.uint64(nparts)) // np.uint64(ncells),
                      nparts - 1).astype(np.int64)


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


class FusedCloudRank:
    """One rank of the multi-GPU frame with the reference's fused output, over a GPU engine.

    Per frame: (halo) all-gather of the depth tails -> the rank's camera with camera k-1's tail
    as halo -> compaction + keys + marks (defer_voxelize, deferred grid) -> occupancy-mark union
    (all-gather + OR) and the identical grid update on every rank -> key-range partition ->
    all-to-all -> voxelize of the rank's key range.  Collectives run on torch tensors of `dev`
    ("cuda": RCCL, the engine on torch's stream; "cpu": gloo, staged through host copies)."""

    def __init__(self, engine, cams, rank: int, world: int, params, dev: str = "cuda"):
        import torch
        from . import hiprt
        self.eng, self.cams, self.rank, self.world, self.p = engine, cams, rank, world, params
        self.dev = dev
        self.hiprt = hiprt
        if dev == "cuda":
            engine.set_stream(torch.cuda.current_stream().cuda_stream)
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

    def frame(self, depth_ptr: int, tail_src_ptr: int, move=None):
        """One frame: depth_ptr = this rank's depth map (device), tail_src_ptr = its last
        Lmax depth values (device, the halo the next rank needs).  On the rollbuffer rank the
        point sequences added to the engine since the last frame (addPointSequence[Device]) are
        ingested, rolled and - with `move` - selected, transformed, cropped and compacted behind
        the camera's points."""
        import numpy as np
        import torch
        import torch.distributed as dist
        h = self.hiprt
        eng, c = self.eng, self.cams[self.rank]
        halo = None
        if self.F > 0 and self.world > 1:
            # all ranks send Lmax values (the tail of their camera); rank k uses rank k-1's
            # (bytes: gloo has no 16-bit integer collectives)
            if self.dev == "cuda":
                tail = torch.empty(2 * self.Lmax, dtype=torch.uint8, device="cuda")
                h.copy_async(tail.data_ptr(), tail_src_ptr, 2 * self.Lmax, h.D2D,
                             torch.cuda.current_stream().cuda_stream)
                parts = all_gather_tails(tail)
                halo = parts[self.rank - 1] if self.rank > 0 else None
                halo_ptr = halo.data_ptr() if halo is not None else 0
            else:
                tail = torch.from_numpy(_d2h(h, tail_src_ptr, np.uint8, 2 * self.Lmax))
                parts = all_gather_tails(tail)
                if self.rank > 0:
                    halo = h.DeviceArray.from_numpy(parts[self.rank - 1].numpy())
                    halo_ptr = halo.ptr
        eng.clear()
        if self.rank > 0 and halo is not None:
            pc = self.cams[self.rank - 1]
            n = pc.width * pc.height
            take = min(self.Lmax, n)
            # the received tail holds camera k-1's last Lmax values (or all of a smaller camera)
            eng.addHaloDepthmapDevice(halo_ptr + 2 * (self.Lmax - take), take, pc.width,
                                      pc.height, *pc.intrinsics(), pc.T_world, pc.T_crop)
        eng.addDepthmapDevice(depth_ptr, c.width, c.height, *c.intrinsics(), c.T_world, c.T_crop)
        res = eng.processFramePrepared(self.frame_params(move))
        _, ncells = eng.grid_size()
        words = words_for(ncells)
        # occupancy union (every rank the same grid)
        if self.dev == "cuda":
            local = torch.empty(words, dtype=torch.int32, device="cuda")
            gathered = torch.empty(self.world * words, dtype=torch.int32, device="cuda")
            eng.export_marks(local.data_ptr(), words)
            dist.all_gather_into_tensor(gathered, local)
            eng.import_marks(gathered.data_ptr(), words, self.world)
        else:
            dl = h.DeviceArray(words * 4)
            eng.export_marks(dl.ptr, words)
            eng.synchronize()
            local = torch.from_numpy(dl.to_numpy(np.int32, words))
            parts = [torch.empty_like(local) for _ in range(self.world)]
            dist.all_gather(parts, local)
            dg = h.DeviceArray.from_numpy(torch.cat(parts).numpy())
            eng.import_marks(dg.ptr, words, self.world)
        eng.voxelOccupancyGrid(self.p.occupancy_lifetime)
        # key-range partition + all-to-all + voxelize of this rank's range (send buffers for the
        # frame's depth pixels + selected rollbuffer points)
        n_total = max(int(res.num_points_total), 1)
        if self.dev == "cuda":
            sp = torch.empty((n_total, 4), dtype=torch.float32, device="cuda")
            sk = torch.empty(n_total, dtype=torch.int32, device="cuda")
            cnt = torch.empty(self.world, dtype=torch.int32, device="cuda")
            eng.partition_points(self.world, sp.data_ptr(), sk.data_ptr(), n_total, cnt.data_ptr())
            rp, rk, rc, counts = exchange_points_dev(sp, sk, cnt)
            eng.voxelize_points(rp.data_ptr(), rk.data_ptr(), int(sum(rc)), self.p.voxel_average)
            self._keep = (rp, rk)
        else:
            dsp, dsk, dcnt = h.DeviceArray(n_total * 16), h.DeviceArray(n_total * 4), h.DeviceArray(64)
            eng.partition_points(self.world, dsp.ptr, dsk.ptr, n_total, dcnt.ptr)
            eng.synchronize()
            counts = dcnt.to_numpy(np.uint32, self.world).tolist()
            m = int(sum(counts))
            sp = torch.from_numpy(dsp.to_numpy(np.float32, 4 * max(m, 1))[:4 * m].reshape(m, 4))
            sk = torch.from_numpy(dsk.to_numpy(np.int32, max(m, 1))[:m])
            rp, rk, rc = exchange_points(sp, sk, counts)
            n = int(sum(rc))
            drp = h.DeviceArray.from_numpy(rp.numpy()) if n else None
            drk = h.DeviceArray.from_numpy(rk.numpy()) if n else None
            eng.voxelize_points(drp.ptr if n else 0, drk.ptr if n else 0, n, self.p.voxel_average)
            eng.synchronize()
            self._keep = (drp, drk)
        return counts


    def batch(self, depth_ptrs, tail_src_ptrs):
        """B frames through one launch chain and ONE exchange (the bench's batched steps): every
        rank's B tails in one all-gather (frame j's halo before frame j's depth map), the batch's
        compaction, the B frames' marks in one all-gather and one batched grid update
        (gdf_voxel_occupancy_grid_batch: frame by frame in order), the (point, frame | key)
        lists partitioned by voxel-key range and exchanged once, and one voxelize of the rank's
        range - frame f's voxels of this range are eng.batch_ranges()[1][f:f+2]."""
        import numpy as np
        import torch
        import torch.distributed as dist
        h = self.hiprt
        eng, c = self.eng, self.cams[self.rank]
        B = len(depth_ptrs)
        L2 = 2 * self.Lmax
        halo_ptr = None
        keep = []
        if self.F > 0 and self.world > 1:
            if self.dev == "cuda":
                tail = torch.empty(B * L2, dtype=torch.uint8, device="cuda")
                stream = torch.cuda.current_stream().cuda_stream
                for j, src in enumerate(tail_src_ptrs):
                    h.copy_async(tail.data_ptr() + j * L2, src, L2, h.D2D, stream)
                parts = all_gather_tails(tail)
                if self.rank > 0:
                    keep.append(parts[self.rank - 1])
                    halo_ptr = parts[self.rank - 1].data_ptr()
            else:
                tail = torch.from_numpy(np.concatenate(
                    [_d2h(h, src, np.uint8, L2) for src in tail_src_ptrs]))
                parts = all_gather_tails(tail)
                if self.rank > 0:
                    dh = h.DeviceArray.from_numpy(parts[self.rank - 1].numpy())
                    keep.append(dh)
                    halo_ptr = dh.ptr
        eng.clear()
        for j in range(B):
            if j:
                eng.nextFrameInBatch()
            if halo_ptr is not None:
                pc = self.cams[self.rank - 1]
                take = min(self.Lmax, pc.width * pc.height)
                eng.addHaloDepthmapDevice(halo_ptr + j * L2 + 2 * (self.Lmax - take), take,
                                          pc.width, pc.height, *pc.intrinsics(), pc.T_world,
                                          pc.T_crop)
            eng.addDepthmapDevice(depth_ptrs[j], c.width, c.height, *c.intrinsics(), c.T_world,
                                  c.T_crop)
        eng.processFramePrepared(self.pc)
        _, ncells = eng.grid_size()
        words = words_for(ncells)
        if self.dev == "cuda":
            local = torch.empty(B * words, dtype=torch.int32, device="cuda")
            gathered = torch.empty(self.world * B * words, dtype=torch.int32, device="cuda")
            eng.take_marks(local.data_ptr(), B * words)
            dist.all_gather_into_tensor(gathered, local)
            eng.voxelOccupancyGridBatch(gathered.data_ptr(), words, self.world, B, words,
                                        B * words, self.p.occupancy_lifetime)
            keep.append(gathered)
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
            keep.append(dg)
        n_total = max(B * c.width * c.height, 1)
        if self.dev == "cuda":
            sp = torch.empty((n_total, 4), dtype=torch.float32, device="cuda")
            sk = torch.empty(n_total, dtype=torch.int32, device="cuda")
            cnt = torch.empty(self.world, dtype=torch.int32, device="cuda")
            eng.partition_points(self.world, sp.data_ptr(), sk.data_ptr(), n_total, cnt.data_ptr())
            rp, rk, rc, counts = exchange_points_dev(sp, sk, cnt)
            eng.voxelize_points(rp.data_ptr(), rk.data_ptr(), int(sum(rc)), self.p.voxel_average)
            keep += [rp, rk]
        else:
            dsp, dsk, dcnt = h.DeviceArray(n_total * 16), h.DeviceArray(n_total * 4), h.DeviceArray(64)
            eng.partition_points(self.world, dsp.ptr, dsk.ptr, n_total, dcnt.ptr)
            eng.synchronize()
            counts = dcnt.to_numpy(np.uint32, self.world).tolist()
            m = int(sum(counts))
            sp = torch.from_numpy(dsp.to_numpy(np.float32, 4 * max(m, 1))[:4 * m].reshape(m, 4))
            sk = torch.from_numpy(dsk.to_numpy(np.int32, max(m, 1))[:m])
            rp, rk, rc = exchange_points(sp, sk, counts)
            n = int(sum(rc))
            drp = h.DeviceArray.from_numpy(rp.numpy()) if n else None
            drk = h.DeviceArray.from_numpy(rk.numpy()) if n else None
            eng.voxelize_points(drp.ptr if n else 0, drk.ptr if n else 0, n, self.p.voxel_average)
            eng.synchronize()
            keep += [drp, drk]
        self._keep = keep
        return counts


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
