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
