// gdf_kernels.hpp — host-side launchers of the gfx950 kernels (gdf_kernels.hip).
#pragma once

#include "gdf.h"

// occupancy-mark words per key range of an nparts-way partition (the last range may be shorter):
// the key-range rule of the multi-GPU exchange (gdf_kernels.hip part_of)
__host__ __device__ inline uint32_t part_slice_words(uint32_t nparts, uint64_t ncells) {
    return (uint32_t)(((ncells + 31) / 32 + nparts - 1) / nparts);
}
#include "gdf_device.hpp"

#include <string>

namespace gdf {

// the calling thread's gdf_last_error() message (gdf_engine.cpp), for the other C-ABI sources
void set_last_error(const std::string& msg);

// Optional per-launch callbacks (the engine records HIP event pairs when profiling).
struct LaunchHook {
    virtual void begin(int slot) = 0;
    virtual void end(int slot) = 0;
    virtual ~LaunchHook() = default;
};

struct VoxelParams {
    float vlo[3], vcs[3], gmax[3];
    uint32_t gs[3];
    float vrcs[3];  // RN(1 / vcs)
};

// per-camera ray factors xn[u] = (u - cx)/fx, yn[v] = (v - cy)/fy
hipError_t launch_tables(uint32_t W, uint32_t H, float fx, float fy, float cx, float cy, float* xn,
                         float* yn, hipStream_t s);

// fused depth + rollbuffer compaction (convert, flying, crop, transform_indirect, apply,
// optional voxel keys + occupancy marks); needs no memset (epoch-tagged look-back, tickets)
hipError_t launch_frame(const FrameArgs& a, hipStream_t s, LaunchHook* hook = nullptr);
// the seg_offsets buffer also holds the chunk partials of the multi-block count scan:
// [scan_partials_offset(segs), + ceil(segs / 4096)) words
inline uint32_t scan_partials_offset(uint32_t segs) { return (segs + 63u) & ~63u; }
inline size_t seg_offsets_words(uint32_t segs) {
    return scan_partials_offset(segs) + (segs + 4095u) / 4096u + 1u;
}
// the compaction kernels (0: k_mask, 1: k_emit, 2/4/5: k_sel<8/4/16>, 3: none) as launched for
// `rot45` and flying-pixel rings F (0: no filter) (graph node lookup)
const void* frame_kernel(int which, int rot45, uint32_t F = 0);
bool sel_key_lds_allowed(uint32_t bytes);  // k_sel's key stash fits (and is enabled) at `bytes`
const void* mask_kernel(const FrameArgs& a);  // the compaction pass-1 kernel launch_frame uses
const void* emit_kernel(const FrameArgs& a);  // the compaction pass-2 kernel launch_frame uses
bool emit_partition_kernels(const FrameArgs& a);

// filter_point_sequence + insert into the rollbuffer ring (w = mask): new points
// [src0, src0 + cnt) (all by default) of the n uploaded, their filter neighbours over all n
hipError_t launch_ps_filter_insert(const float4* new_pts, uint32_t n, int do_filter, float thr,
                                   uint32_t F, float4* ring, uint64_t cap, uint64_t first,
                                   hipStream_t s, uint32_t src0 = 0, uint32_t cnt = 0xFFFFFFFFu);
// device-resident PointCloud2 records (x, y, z at byte offsets 0/4/8, step % 4 == 0) -> float4 w=1
hipError_t launch_gather_records(const void* rec, uint32_t n, uint32_t step, float4* out,
                                 hipStream_t s);

// sparse per-frame u8 grid snapshots of a batch (the non-zero 32-cell groups of the grid after
// each frame but the last), written by the batched grid update; layout per update launch of
// `nblocks` 256-thread blocks: snap_dims (W wave segments of `seg` entries per frame), entry e =
// (word index idx[e], 32 bytes data[2e], data[2e + 1]), counts cnt[f * W + w]
struct SnapArgs {
    uint32_t* idx;
    uint4* data;
    uint32_t* cnt;
};
void snap_dims(uint64_t ncells, uint32_t nblocks, uint32_t* waves, uint32_t* seg);
// blocks of the grid update that the first sort pass carries (for the snapshot layout), at `wpt`
// mark words per thread (Tuning::grid_wpt)
uint32_t fused_grid_blocks(uint64_t ncells, uint32_t wpt);
// blocks of k_grid_u8_batch
uint32_t batch_grid_blocks(uint64_t ncells);
// frame `frame`'s snapshot expanded into a dense u8 grid (out: padded to 32 bytes)
hipError_t launch_snap_expand(const SnapArgs& sn, uint32_t frame, uint32_t nblocks,
                              uint64_t ncells, uint8_t* out, hipStream_t s);

// historic grid update from the frame's mark bitmask (cleared on the way): u8 grid = history for
// lifetime <= 255; the general u32 history with a separate u8 output grid beyond
// (q: engine order of grid updates across streams, see GridSeq)
hipError_t launch_grid_u8(uint8_t* grid, uint32_t* marks, uint64_t ncells, uint32_t lifetime,
                          const GridSeq& q, hipStream_t s);
hipError_t launch_grid_u8_batch(uint8_t* grid, const uint32_t* bits, uint64_t ncells,
                                uint32_t nranks, uint32_t nframes, uint64_t frame_stride,
                                uint64_t rank_stride, uint32_t lifetime, const GridSeq& q,
                                const SnapArgs& snap, hipStream_t s);
hipError_t launch_grid_u32(uint32_t* hist, uint32_t* marks, uint8_t* out8, uint64_t ncells,
                           uint32_t lifetime, const GridSeq& q, hipStream_t s);
hipError_t launch_widen_grid(const uint8_t* grid8, uint32_t* hist, uint64_t ncells,
                             const GridSeq& q, hipStream_t s);

// standalone voxel keys over the compacted points (count read on the device)
hipError_t launch_coords(const float4* pts, const uint32_t* count, uint32_t nmax,
                         uint32_t* coords, const VoxelParams& v, hipStream_t s);
// occupancy marks (bitmask) from voxel keys
hipError_t launch_scatter(const uint32_t* coords, const uint32_t* count, uint32_t nmax,
                          uint32_t* marks, hipStream_t s);

// GPU voxelize: stable LSD radix sort of (key, index) + ordered per-voxel mean
struct VoxelizeArgs {
    const uint32_t* keys;       // voxel keys [N]
    const float4* pts;          // compacted points [N]
    const uint32_t* count;      // N on the device
    uint32_t nmax;              // capacity bound for launch sizing
    uint32_t key_bits;          // bit width of (num_cells - 1)
    int average;
    int hist_ready;             // the key histogram was already accumulated (fused k_frame)
    VoxelParams vp;
    // workspace
    uint32_t *keys_a, *keys_b, *vals_a, *vals_b;
    uint32_t* hist;                 // [kHistReps][4*256] zero on entry, left zero on exit
    unsigned long long* status;     // [sort tiles * 256] epoch granules
    unsigned long long* sgstatus;   // [sort tile groups * 256]
    unsigned long long* gstatus;    // [group tiles] epoch granules
    unsigned long long* ggstatus;   // [group tiles / 64 + 1]
    unsigned long long* ctrs;       // [kCtrSlots] self-resetting tile tickets (low 32 bits)
    int sort_pt;                    // keys per thread of a sort tile (4, 8 or 16)
    // optional fused historic-grid update (u8 grid, lifetime <= 255), run by extra blocks of the
    // first sort pass: it only needs the occupancy marks, which the compaction already wrote
    uint8_t* grid8;
    uint32_t* marks;
    uint32_t* group_marks;          // optional: k_group sets the occupancy mark of every voxel
    uint64_t group_mark_stride;     // k_group_runs: frame f's marks at f * stride words (0: one bitmask)
    uint32_t* group_counts;         // [group tiles] group starts per tile (large frames)
    uint32_t* group_offsets;        // [seg_offsets_words(group tiles)] their scan
    // [group tiles] the first group start of each tile (0xFFFFFFFF: none), written by
    // k_group_count: k_group_runs finds the end of a tile's last group from these, not from the
    // run keys past the tile
    uint32_t* group_first;
    // optional: the scan inside k_group_count (arrive_and_scan, no scan launches) - arrival
    // counters [group tiles / kScanGroup] (self-resetting) and group totals [same]
    uint32_t* group_done;
    uint32_t* group_gtot;
    uint4* bigq;                    // [group blocks * tiles per block] long voxels (large frames)
    uint32_t bigq_cap;              // run mode: one queue of bigq_cap groups (kCtrRunQueue counts)
    uint32_t* bigcnt;               // [group blocks] queued per block
    GridSeq gseq;                   // engine order of the fused grid update (frame pipelining)
    // multi-frame batch: keys of frame f (points [frame_pt_start[f], frame_pt_start[f+1])) sort
    // as key | f << frame_shift; k_group writes the first voxel of each frame (frame_vox_start,
    // nframes + 1 entries); the grid update applies the frames' marks (stride mark_words) in
    // order and writes the sparse snapshots of the grid after each frame but the last (snap)
    uint32_t nframes;
    uint32_t frame_shift;
    const uint32_t* frame_pt_start;
    uint32_t* frame_vox_start;
    uint64_t mark_words;
    SnapArgs snap;
    // runs of equal keys: keys / count are the run keys / run count, the sort orders runs and
    // k_group_runs groups them (run r = points run_start[r] .. run_start[r+1]-1; point_count:
    // the points)
    const uint32_t* run_start;
    const uint32_t* point_count;
    // the engine's own runs (<= 64 points each): the first radix pass packs each run's length into
    // key bits 26..31 and sorts its first point as the value (sort keys of <= 25 bits)
    int pack_runs;
    uint64_t ncells;
    uint32_t lifetime;
    uint32_t* err;
    // outputs
    float4* out;
    uint32_t* out_count;
    const Tuning* tune;  // the engine's launch shapes (sort / group grids, group-phase forms)
    // the stream gate of the grid update carried by the first radix pass (direct launches): wait
    // for grid_wait before that pass, record grid_rec after it - or, grid_rec_early, right before
    // it: the next update then waits until this one is next in its stream (dispatchable), not
    // done (null: none, e.g. graph capture)
    hipEvent_t grid_wait, grid_rec;
    int grid_rec_early;
    // > 0: k_group_runs_big's grid capped at this many blocks (batches of small frames: their
    // queue is almost always empty, and the launch of a resident grid is chain time - C2 +1 %)
    uint32_t big_cap;
};
hipError_t launch_voxelize(const VoxelizeArgs& a, hipStream_t s, LaunchHook* hook = nullptr);
size_t voxelize_status_words(uint32_t nmax, uint32_t key_bits);
size_t voxelize_group_tiles(uint32_t nmax);

// orphan shaders: mask_dilate (F <= kDilateMaxF) and single-matrix transform_points
hipError_t launch_mask_dilate(const uint32_t* in, uint32_t* out, uint32_t W, uint32_t H,
                              uint32_t F, int as_written, hipStream_t s);
struct Mat4 {
    float m[16];
};
hipError_t launch_transform_points(const float4* in, const uint32_t* mask, float4* out, uint32_t n,
                                   const float* T, hipStream_t s);

// multi-GPU fused cloud: stable partition of (points, keys)[*count] into nparts key ranges,
// part-major into out_pts / out_keys; part_counts[p] = items of part p (device).  A batch
// (fstart: the frames' point starts): the sent keys carry the frame index above bit fshift.  Workspace:
// counts [nparts * part_tiles(nmax)], offsets [seg_offsets_words(nparts * part_tiles(nmax))],
// total [1].
// With out_run_keys (runs mode): also the part-major runs of equal sent keys (run keys, run
// starts relative to the part's first point), part_counts[nparts + p] = runs of part p, counts /
// offsets twice as long (points' tile counts, then the runs'); out_keys may be null.
// splits (device words, optional): nsplit + 1 <= kMaxSegs SEGMENTS cut at the items splits[0] <=
// splits[stride] <= ... (stride 0: every cut at the one word splits[0]) - a frame's depth points,
// then its rollbuffer points in pieces (a sharded window: one piece per stretch of the selection
// this rank holds) - buckets b = part * nseg + segment take the place of the parts (bucket-major
// output, part_counts [nseg nparts points | nseg nparts runs], run starts relative to the bucket's
// first point, a run never crossing a cut); nparts * nseg <= kMaxBuckets, workspace sized for
// nseg nparts.
uint32_t part_tiles(uint32_t nmax);
hipError_t launch_partition(const float4* pts, const uint32_t* keys, const uint32_t* count,
                            uint32_t nmax, uint32_t nparts, uint64_t ncells, uint32_t* counts,
                            uint32_t* offsets, uint32_t* total, float4* out_pts,
                            uint32_t* out_keys, uint32_t* part_counts, hipStream_t s,
                            const uint32_t* fstart = nullptr, uint32_t nframes = 1,
                            uint32_t fshift = 0, uint32_t* out_run_keys = nullptr,
                            uint32_t* out_run_start = nullptr,
                            const uint32_t* splits = nullptr, uint32_t nsplit = 0,
                            uint32_t split_stride = 0);

// gdf_download_frame's prefetch: a single-frame launch chain ends with ONE kernel that writes the
// frame's downloads - the small counters, the points, voxel coords, voxelized points and the grid
// delta, each of the size the counters name - straight into pinned (host-mapped) mirrors, so the
// host waits once for the stream instead of reading the counts, then queueing the copies, then
// waiting again.
struct DlArgs {
    const uint32_t* misc;
    uint32_t misc_words, i_count, i_vox, i_delta;  // counter words: points, voxels, delta groups
    const uint4* pts;
    const uint32_t* coords;
    const uint4* vox;
    const uint32_t* didx;
    const uint4* ddata;  // 2 per group
    uint32_t pts_cap, vox_cap, delta_cap;
    uint32_t* h_misc;
    uint4* h_pts;
    uint32_t* h_coords;
    uint4* h_vox;
    uint32_t* h_didx;
    uint4* h_ddata;
    uint32_t parts;  // DL_* bits: which of the above this launch writes
};
enum : uint32_t { DL_MISC = 1, DL_POINTS = 2, DL_VOX = 4, DL_DELTA = 8 };
hipError_t launch_download(const DlArgs& d, hipStream_t s);

// gdf_voxelize_runs: nsrc received segments, source q's points from point_base[q] and runs from
// run_base[q] (q <= nsrc: the totals)
constexpr uint32_t kMaxOwnSources = 4;  // sources still in the caller's send lists (one rank's buckets)
struct RebaseArgs {
    uint32_t point_base[kMaxSources + 1];
    uint32_t run_base[kMaxSources + 1];
    uint32_t nsrc;
    // the multi-GPU step's own buckets, read from its send lists in the same pass (no device
    // copies first): source own_src[k]'s points, run keys and run starts (relative to the source)
    uint32_t n_own;
    uint32_t own_src[kMaxOwnSources];
    const float4* own_pts[kMaxOwnSources];
    const uint32_t* own_run_keys[kMaxOwnSources];
    const uint32_t* own_run_starts[kMaxOwnSources];
    float4* pts;          // the received list (the own sources' points are written here)
    uint32_t* run_keys;   // (the own sources' run keys are written here)
    // mark words cleared in the same pass: zero_rows rows of zero_row_words at zero_stride
    uint32_t* zero;
    uint64_t zero_row_words, zero_stride;
    uint32_t zero_rows;
};
hipError_t launch_run_rebase(uint32_t* run_start, const RebaseArgs& r, uint32_t* n_points,
                             uint32_t* n_runs, hipStream_t s);

// runs of equal keys in an external key list of *count (<= nmax) keys (the multi-GPU receive
// buffer): run_keys[r], run_start[r] (first item; run_start[R] = n), *run_total = R.  Workspace:
// tcounts [xrun_tiles(nmax)], offsets [seg_offsets_words(xrun_tiles(nmax))].
uint32_t xrun_tiles(uint32_t nmax);
hipError_t launch_xruns(const uint32_t* keys, const uint32_t* count, uint32_t nmax,
                        uint32_t* tcounts, uint32_t* offsets, uint32_t* run_keys,
                        uint32_t* run_start, uint32_t* run_total, hipStream_t s);

// multi-GPU occupancy marks: export = copy of the mark bitmask, import = OR of nranks masks
hipError_t launch_export_marks(const uint32_t* marks, uint64_t words, uint32_t* bits, hipStream_t s);
hipError_t launch_take_marks(uint32_t* marks, uint64_t words, uint32_t* bits, hipStream_t s);
hipError_t launch_take_marks_sparse(uint32_t* marks, uint64_t words, uint32_t* bits,
                                    uint32_t* pairs, uint32_t cap, hipStream_t s);
hipError_t launch_union_pairs(uint32_t* uni, uint64_t words, const uint32_t* pairs,
                              uint32_t nranks, uint32_t nframes, uint32_t frames_per_rank,
                              uint64_t rec_words, hipStream_t s);
// nranks masks of `words` words, mask r at bits + r * stride
hipError_t launch_import_marks(uint32_t* marks, uint64_t words, const uint32_t* bits,
                               uint32_t nranks, uint64_t stride, hipStream_t s);

}  // namespace gdf
