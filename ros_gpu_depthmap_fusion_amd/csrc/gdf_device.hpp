// gdf_device.hpp — data layout and float semantics shared by the gfx950 kernels.
//
// Float contract: binary32, correctly rounded / and sqrt
// (-fhip-fp32-correctly-rounded-divide-sqrt), no FMA contraction (-ffp-contract=off), explicit
// summation order — the same order the reference GLSL writes and the oracle restates, so
// masks, voxel keys and occupancy come out bit-identical.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gdf {

constexpr int kMaxCams = 16;          // GDF_MAX_CAMERAS
constexpr int kFrameThreads = 256;    // k_mask / k_emit block: 4 waves, 4 items per thread
constexpr int kArgCams = 8;           // camera descriptors passed in the kernel arguments
constexpr int kHalo = 8;              // band rows/columns staged around a segment: min(F, 8)
constexpr uint32_t kSegItems = 1024;  // items per compaction segment (max)
constexpr uint32_t kFusedPrefixSegs = 4096;  // up to this many segments k_emit sums the counts
constexpr uint32_t kScanGroup = 64;          // segments per group of the in-kernel group scan
constexpr uint32_t kMaxScanGroups = 4096;    // k_emit sums at most this many group totals
constexpr uint32_t kMaxGroupScanTiles = 65536;  // group phase: in-kernel scan up to this many tiles
constexpr uint32_t kSelSegs = 8;      // rollbuffer points per k_sel thread (default; 4, 8, 16)
constexpr uint32_t kSelThreads = 512; // k_sel block (default): a tile is segs * threads points
constexpr int kSortThreads = 256;
constexpr int kSortGroup = 8;         // radix tiles per look-back group (group granules: tiles / 8)
// the voxel-key digit histogram is accumulated into kHistReps replicas of [4 passes][256 digits]
// (block b adds into replica b % kHistReps): same-address atomics from hundreds of blocks
// serialise at the memory-side atomic unit; the sort pass sums the replicas of its digit
constexpr int kHistReps = 16;
constexpr int kHistWords = kHistReps * 4 * 256;

// Radix passes over a key of `bits` bits: 8-bit digits, except that up to 25 bits the LAST pass
// takes a 9-bit digit when that saves a pass (25 = 22 voxel-key bits + 3 frame bits of an 8-frame
// batch: 3 passes instead of 4; 17 and 9 likewise).  Pass p's histogram lives at [p*256, ...):
// the 9-bit last digit of pass 2 fills [512, 1024), still inside a replica's 1024 words.
__host__ __device__ constexpr uint32_t radix_passes(uint32_t bits) {
    return bits == 0 ? 1u : bits <= 25 ? (bits <= 9 ? 1u : (bits + 6) / 8) : (bits + 7) / 8;
}
__host__ __device__ constexpr bool radix_wide_last(uint32_t bits) {
    return bits >= 9 && bits <= 25 && bits % 8 == 1;
}
// digit of pass p (of np passes): a 9-bit mask on the last of <= 3 passes is exact for every key
// (an 8-bit last digit has bit 8 clear: the key has no bits there)
__host__ __device__ constexpr uint32_t radix_digit(uint32_t key, uint32_t p, uint32_t np) {
    return (key >> (8u * p)) & ((p + 1u == np && np <= 3u) ? 0x1FFu : 0xFFu);
}
// histogram words a producer clears / flushes for np passes
__host__ __device__ constexpr uint32_t radix_hist_span(uint32_t np) {
    return np <= 3u ? (np + 1u) * 256u : 1024u;
}
constexpr int kGroupThreads = 256;
constexpr int kSumChunk = 128;                               // points per wave gather chunk
constexpr uint32_t kSpinLimit = 1u << 26;                   // bounded look-back spins
constexpr uint32_t kDilateMaxF = 16;                        // mask_dilate window radius limit
constexpr uint32_t kMaxParts = 16;                          // ranks of the fused-cloud partition
constexpr uint32_t kMaxBuckets = 2 * kMaxParts;             // parts x segments, <= 32 (wave ballots)
constexpr uint32_t kMaxSegs = 4;                            // segments [depth | <= 3 rollbuffer pieces]
constexpr uint32_t kMaxSources = 2 * kMaxParts;             // received segments of gdf_voxelize_runs

// Device-wide counters: monotonically increasing tile tickets (the host passes each launch's
// base, so no per-launch memset) and the global digit histogram of the voxel keys.
// per-stream device counters (u64 words, low 32 bits used): tile tickets, look-back epoch
enum CounterSlot { kCtrSel = 0, kCtrSort0 = 1, kCtrGroup = 5, kCtrEpoch = 6,
                   kCtrRunQueue = 7,  // run-group queue: appends, draws, huge appends (u32 each,
                                      // over words 7 and 8)
                   kCtrSlots = 9 };

// engine-order of historic-grid updates across streams (grid_seq_enter / grid_seq_leave)
struct GridSeq {
    uint32_t* ctl;         // [0] updates completed, [1] blocks finished of the running one
    const uint32_t* fptr;  // the update's sequence number on the device (or nullptr: use f)
    uint32_t f;
    uint32_t* err;
    // optional delta of a single-frame u8 update (gdf_download_frame's grid): every 32-cell
    // group whose bytes changed, as (word index, new 32 bytes) appended at *dcnt (zeroed before)
    uint32_t* dcnt;
    uint32_t* didx;
    uint4* ddata;
};

// A halo camera (emit == 0, multi-GPU sharding) sits at a negative offset: its pixels are only
// read as flying-pixel neighbours, exactly where the reference's uint index arithmetic lands in
// the previous camera of the concatenated buffer.
// xn[u] = (u - cx) / fx and yn[v] = (v - cy) / fy are the per-column / per-row factors of
// sh/convert_depthmap_to_points.glsl:64-73 (the same f32 divisions, computed once per camera).
struct CamDesc {
    int64_t off;            // first index in the concatenated point space
    const uint16_t* depth;  // device pointer to pixel 0 of this camera
    const float* xn;        // [W]
    const float* yn;        // [H]
    uint64_t wmagic;        // ceil(2^40 / W): exact local / W for local < 2^24, W < 2^16
    uint32_t W, H, n;
    uint32_t emit;          // 1: pixels are processed; 0: halo camera, only read as neighbours
    float scale;
    uint32_t nchunk;        // segments per row: ceil(W / 1024)
    uint32_t seg0;          // first segment of this camera (emitting cameras)
    uint32_t nseg;          // H * nchunk
    uint32_t segw;          // pixels per segment (a multiple of 64, <= 1024)
    uint32_t frame;         // frame of a multi-frame batch (neighbour reads stay inside it)
    float Tw[16];           // row-major T_world
    float Tc[16];           // row-major T_crop
};
static_assert(sizeof(CamDesc) % 16 == 0, "CamDesc must stay 16-byte sized");

// Launch-shape choices of one engine (host-side; the kernels never read it).  None changes a
// result: each alternative is parity-tested against the oracle (test_gpu_round3/4/5).  An engine
// takes its snapshot at gdf_create - a GDF_* variable when set, the default otherwise - and its
// launches read only that snapshot, so engines created under other environments (other threads,
// the in-process world's ranks) never retune it; gdf_create logs every value that differs from
// its default.
struct Tuning {
    uint32_t mask_px2 = 2;            // GDF_MASK_PX: pixels per k_mask thread (2, or 1: k_mask)
    uint32_t mask_occ8 = 1;           // GDF_MASK_OCC8: k_mask_px at 8 waves per SIMD
    uint32_t emit_px2 = 1;            // GDF_EMIT_PX2: two pixels per k_emit thread
    uint32_t grid_wpt = 2;            // GDF_GRID_WPT: mark words per thread of the grid update (1..8)
    uint32_t sort_blocks = 2048;      // GDF_SORT_BLOCKS: radix grid cap
    uint32_t group_blocks = 2048;     // GDF_GROUP_BLOCKS: group-phase grid cap
    uint32_t group_scan_tiles = 1024; // GDF_GROUP_SCAN_TILES: tiles above which k_group counts + scans
    uint32_t group_first = 1;         // GDF_GROUP_FIRST: tile ends from k_group_count's first starts
    uint32_t run_stage = 2048;        // GDF_RUN_STAGE: staged points per k_group_runs tile (512 / 2048)
    uint32_t run_inblock = 1024;      // GDF_RUN_INBLOCK: in-block group size limit
    uint32_t run_wave = 2;            // GDF_RUN_WAVE: staged long groups 0 queued, 1 a wave, 2 4 lanes
    uint32_t small_group = 32;        // GDF_SMALL_GROUP: thread-summed group size
    uint32_t points_lane = 0;         // GDF_POINTS_LANE: k_group's long staged groups by 4-lane chains
    uint32_t run_wave_mode = 1;       // GDF_RUN_WAVE_MODE: queued groups 0 block, 1 by queue, 2 wave
    uint32_t run_big_occ4 = 0;        // GDF_RUN_BIG_OCC4: k_group_runs_big at 4 waves per SIMD
    uint32_t run_big_blocks = 1024;   // GDF_RUN_BIG_BLOCKS: k_group_runs_big grid cap
    uint32_t run_q16 = 2;             // GDF_RUN_Q16: chunks of 1 K points 0 never, 1 always, 2 single frames
};

// Arguments of the compaction launches, passed by value.  Up to kArgCams camera descriptors
// travel in the kernel arguments (kernel-argument bytes cost launch latency); more cameras are
// read from a device copy.
struct FrameArgs {
    CamDesc cams[kArgCams];
    const CamDesc* cams_dev;    // all descriptors when ncams > kArgCams
    int32_t ncams;
    uint32_t depth_total;       // ΣP of emitting cameras' index space
    uint32_t depth_segs;        // segments over the depth pixels
    uint32_t total_segs;        // segments of the two-pass (depth) compaction: depth_segs
    // flying-pixel filter (sh/filter_flying_pixels.glsl)
    int32_t do_flying;
    uint32_t F;
    float thr;
    int32_t rot45;
    // crop (sh/crop_points.glsl)
    int32_t do_crop;
    float lo[3], hi[3];
    // selected rollbuffer points (insertSelected + transform_points_indirect)
    uint32_t sel_count;
    const float4* ring;
    uint64_t ring_cap;
    uint64_t ring_first;        // physical index of logical point sel_point_start
    uint32_t nseg;
    // > 0: seg_start[k] = k * sel_uniform - sel_off for k >= 1 (equal sequences): the sequence of
    // selected point i is (i + sel_off) / sel_uniform, no search
    uint32_t sel_uniform, sel_off;
    const uint32_t* seg_start;  // relative first point of each covered sequence (ascending)
    const uint32_t* seg_tf;     // transform index of that sequence
    const float* tfw;           // row-major T_world_move·T_move per selected sequence
    const float* tfc;
    // rollbuffer compaction (k_sel): tiles of kSelSegs * kSelThreads points in ticket order, their
    // survivors placed behind the depth points by decoupled look-backs over the tiles
    uint32_t sel_tiles;
    uint32_t sel_tile;          // points per tile = sel_segs * k_sel block size
    uint32_t sel_segs;
    unsigned long long* sel_status;  // look-back granules: 2 channels (points, runs) x
                                     // 2 * (tiles + tiles / 64 + 2) words (tiles, then groups)
    uint32_t* sel_ctr;          // tile tickets
    uint32_t* epoch_word;       // look-back epoch (shared with the voxelize launches)
    uint32_t* final_count;      // depth + rollbuffer survivors (out_count then holds the depth part)
    // the partition's segment cuts (sharded windows: the pieces of the selection this rank holds):
    // sel_splits[0] = depth survivors, sel_splits[1 + c] = survivors before selected item
    // sel_cut_at[c] (c < sel_ncuts), the frame's total for the unused cuts (kMaxSegs - 1 words)
    uint32_t* sel_splits;
    uint32_t sel_ncuts;
    uint32_t sel_cut_at[kMaxSegs - 2];
    // run mode: bytes of dynamic LDS where k_sel keeps each item's voxel key from the run
    // detection for the store pass (0: the store pass recomputes them)
    uint32_t sel_key_lds;
    // voxel keys + occupancy marks (compute_voxel_coords + voxel_grid_occupancy_of_points)
    int32_t do_voxel;
    float vlo[3], vcs[3], gmax[3];
    float vrcs[3];              // RN(1 / vcs) (voxel_key's fast quotient)
    uint32_t gs[3];
    uint32_t* marks;            // occupancy mark bitmask (cell c -> bit c % 32 of word c / 32)
    uint32_t* key_hist;         // optional [npasses*256] digit histogram of the keys
    uint32_t npasses;
    // outputs
    float4* out_pts;
    uint32_t* out_count;
    uint32_t* out_coords;
    // reduce-then-scan compaction state
    unsigned long long* vbits;  // [total_segs * 16] validity bitmask
    uint32_t* seg_counts;       // [total_segs] valid items per segment
    uint32_t* seg_offsets;      // [total_segs] (k_scan_counts path)
    int32_t fused_prefix;       // k_emit sums the preceding segment counts itself
    uint32_t band_rowb;         // bytes per staged band row (16-B chunks)
    uint32_t band_lds;          // dynamic LDS of k_mask: band rows + column ray factors (+ hist)
    uint32_t hist_lds;          // k_mask_px: byte offset of the run-key digit histogram in it
    uint32_t seg_threads;       // block size of k_mask / k_emit (>= every segment, 64-multiple)
    uint8_t* dbg;               // optional per-item stage bits
    uint32_t* err;
    uint32_t* grid_seq_out;     // optional: k_mask stores grid_seq here (the fused grid update's
    uint32_t grid_seq;          // sequence number, read by the first sort pass of the frame)
    // multi-frame batch (depth-only frames through one launch chain): frame f's points are
    // [frame_pt_start[f], frame_pt_start[f + 1]) of the compacted output, its occupancy marks at
    // marks + f * mark_words, its sort key = voxel key | f << frame_shift
    uint32_t nframes;           // 1: a single frame
    uint32_t frame_shift;       // bit width of the voxel keys (the frame index sits above)
    uint64_t mark_words;        // words of one frame's mark bitmask
    uint32_t* frame_pt_start;   // [nframes + 1], written by k_emit
    // runs of equal voxel keys (depth-only frames): k_mask counts the runs among the kept pixels
    // of each wave (a run = consecutive kept lanes with one key; the voxelize then sorts runs,
    // not points), k_emit writes each run's sort key and first point
    int32_t run_mode;
    uint32_t* wave_runs;        // [total_segs * 16] runs per (segment, wave)
    uint32_t* run_keys;         // [runs] key | frame << frame_shift
    uint32_t* run_start;        // [runs + 1] first point of each run; [runs] = points
    uint32_t* run_count;        // runs of the frame (device)
    uint32_t* scan_total;       // scratch total of the segment-count scan
    uint32_t* run_total;        // runs of depth + rollbuffer points (k_sel's last tile)
    // group scan (no scan launch, kFusedPrefixSegs < segments <= kScanGroup * kMaxScanGroups):
    // the last k_mask block to finish in each group of kScanGroup segments scans the group's
    // counts into group-local offsets (seg_offsets) and the group totals (grp_tot: point totals,
    // then run totals); k_emit adds the totals of the groups before its own
    uint32_t* grp_done;         // [groups] arrival counters (self-resetting)
    uint32_t* grp_tot;          // [2 * groups]
    int32_t mask_packed;        // k_mask_px<2>: both pixels of a thread in packed f32 ops
    // emit partition (multi-GPU fused cloud, gdf_set_emit_partition): the compaction writes the
    // key-range partition itself - k_mask_px counts each segment's kept points and runs per part
    // (seg_counts [2 * nparts][total_segs], one scan), k_emit_px2 writes every kept point and run
    // record straight to its part: points part-major, run keys (with the frame) and run starts
    // relative to the part's first point; no compaction-order points, keys or runs
    uint32_t nparts;            // 0: off
    uint64_t part_ncells;       // part of voxel key k: floor(k * nparts / part_ncells)
    float4* part_pts;
    uint32_t* part_run_keys;
    uint32_t* part_run_starts;
    uint32_t* part_counts;      // [2 * nparts]: points, then runs per part (device)
    // > 1: the counts in the nseg-segment layout [points of (part p, segment s) at nseg p + s |
    // runs at nseg P + nseg p + s] with segments 1.. (a selection's rollbuffer pieces) empty - a
    // frame without one
    uint32_t part_nseg;
    // > 0: every camera emits with this many segments, camera k's from segment k * seg_uniform
    // (a batch of equal frames): a segment's camera is s / seg_uniform, no descriptor load
    uint32_t seg_uniform;
    const Tuning* tune;         // (host) the engine's launch shapes: mask_kernel / emit_kernel
};
static_assert(sizeof(FrameArgs) <= 4096, "kernel arguments are limited to 4 KiB");

// ---- canonical float helpers (mirror oracle/gdf_oracle.c) ----------------------------------
__device__ __forceinline__ float dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return (ax * bx + ay * by) + az * bz;
}

// out = M·p, ((m0·x + m1·y) + m2·z) + m3·w per row
template <class P>  // const float* or a global-address-space pointer
__device__ __forceinline__ float mrow(P m, float x, float y, float z, float w) {
    return ((m[0] * x + m[1] * y) + m[2] * z) + m[3] * w;
}

// GLSL normalize(v) = v / length(v)
__device__ __forceinline__ void normalize3(float& x, float& y, float& z) {
    float l = sqrtf(dot3(x, y, z, x, y, z));
    x = x / l;
    y = y / l;
    z = z / l;
}

// sh/convert_depthmap_to_points.glsl:64-81 (u = idx mod W, v = idx / W):
// p = ((u-cx)/fx · z, (v-cy)/fy · z, z) with z = f32(d)·scale
__device__ __forceinline__ uint32_t div_w(const CamDesc& c, uint32_t local) {
    return (uint32_t)(((unsigned long long)local * c.wmagic) >> 40);
}

__device__ __forceinline__ void cam_point(const CamDesc& c, uint32_t local, uint32_t d, float& x,
                                          float& y, float& z) {
    const uint32_t v = div_w(c, local);
    const uint32_t u = local - v * c.W;
    const float zz = (float)d * c.scale;
    x = c.xn[u] * zz;
    y = c.yn[v] * zz;
    z = zz;
}

// sh/compute_voxel_coords.glsl:44-53: clamp-then-floor per axis, x fastest, of the correctly
// rounded quotient (p - lo) / cs.  Only the floor of the clamped quotient matters, so the
// quotient is first taken as (p - lo) * rcp(cs) (rcs = RN(1/cs), host-computed): its relative
// error is <= 3 * 2^-24, and unless it lies within 2^-20 (relative) of an integer - where the
// exact quotient could floor (or clamp, at the integers 0 and gs - 1) differently - the floor is
// the same.  Those rare lanes (wave-uniform branch) divide exactly.
__device__ __forceinline__ float voxel_axis(float p, float lo, float cs, float rcs) {
    const float d = p - lo;
    const float q = d * rcs;
    const float r = rintf(q);
    if (__builtin_expect(fabsf(q - r) <= fabsf(q) * 9.5367431640625e-07f, 0))  // 2^-20
        return d / cs;
    return q;
}

__device__ __forceinline__ uint32_t voxel_key(float px, float py, float pz, const float* vlo,
                                              const float* vcs, const float* vrcs,
                                              const float* gmax, const uint32_t* gs) {
    float fx = voxel_axis(px, vlo[0], vcs[0], vrcs[0]);
    float fy = voxel_axis(py, vlo[1], vcs[1], vrcs[1]);
    float fz = voxel_axis(pz, vlo[2], vcs[2], vrcs[2]);
    fx = fminf(fmaxf(fx, 0.0f), gmax[0]);
    fy = fminf(fmaxf(fy, 0.0f), gmax[1]);
    fz = fminf(fmaxf(fz, 0.0f), gmax[2]);
    uint32_t ux = (uint32_t)floorf(fx), uy = (uint32_t)floorf(fy), uz = (uint32_t)floorf(fz);
    return ux + uy * gs[0] + uz * gs[0] * gs[1];
}

}  // namespace gdf
