/*
 * gdf.h — C-ABI of the MI355X-native depth-map fusion hot path.
 *
 * Drop-in boundary for the `GPUDepthmapFusion` engine of xaedes/ros_gpu_depthmap_fusion
 * (include/gpu_depthmap_fusion/gpu_depthmap_fusion.h:159-526, src/gpu_depthmap_fusion.cpp).
 * Every entry point below names the reference method it replaces (file:line, paths relative to
 * the reference root).  The ROS component (src/gpu_depthmap_fusion_component.cpp) keeps calling the
 * same method sequence through the C++ facade in include/gdf_fusion.hpp, which forwards here.
 *
 * Conventions
 *   - plain pointers and sizes only; no C++/torch/OpenCV types cross this boundary;
 *   - every function returns an int status (GDF_OK == 0, negative on error) and never throws;
 *     the message of the last error on the calling thread is returned by gdf_last_error();
 *   - 4x4 matrices are 16 floats, ROW-major, i.e. the memory of a cv::Matx44f
 *     (the reference uploads them with transpose=false and multiplies `point * M` in GLSL, which
 *     is M·p for the row-major matrix, include/gpu_depthmap_fusion/program_uniform.h:197-209);
 *   - points are float4 {x, y, z, w} (16 bytes), the layout of the reference's vec4 buffers;
 *   - an engine is bound to one HIP device and one HIP stream; frame calls must be serialised by
 *     the caller (the reference holds m_mutexCallbackN, component.cpp:95);
 *     gdf_add_point_sequence is internally locked and may be called from another thread
 *     (the reference's m_mutexCallbackPointSequence, component.cpp:162,997).
 */
#ifndef GDF_H_
#define GDF_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version: gdf_frame_params and the signatures below are exactly those of this version; a
 * caller checks gdf_version() against the header it was built with (the Python binding and the
 * C++ facade do).  0.2: gdf_frame_params.defer_voxelize, frames_per_rank of
 * gdf_union_occupancy_pairs; 0.3: batched take / sparse per-frame grids; 0.4: slot selection
 * (gdf_get_slot / gdf_select_slot), build provenance (gdf_build_info). */
#define GDF_VERSION_MAJOR 0
#define GDF_VERSION_MINOR 4

#define GDF_MAX_CAMERAS 16

enum gdf_status_code {
    GDF_OK = 0,
    GDF_ERR_ARG = -1,       /* invalid argument (null pointer, bad size, bad grid bounds)      */
    GDF_ERR_STATE = -2,     /* call out of order, or rollbuffer bookkeeping would underflow    */
    GDF_ERR_HIP = -3,       /* HIP runtime error                                               */
    GDF_ERR_NOMEM = -4,     /* device or host allocation failed                                */
    GDF_ERR_CAPACITY = -5,  /* a caller-provided output buffer is too small                    */
    GDF_ERR_TIME = -6,      /* ROS time arithmetic out of range (ros::Time would throw)        */
    GDF_ERR_DEVICE = -7     /* a kernel reported an internal error (bounded spin expired)      */
};

typedef struct gdf_engine gdf_engine;

/* Rollbuffer bookkeeping, the public m_rollBuffer* members of the reference
 * (gpu_depthmap_fusion.h:345-354). */
typedef struct gdf_rollbuffer_state {
    uint32_t num_points;                /* m_rollBufferNumPoints              */
    uint32_t num_seqs;                  /* m_rollBufferNumSeqs                */
    uint32_t selection_point_start;     /* m_rollBufferSelectionPointStart    */
    uint32_t selection_point_count;     /* m_rollBufferSelectionPointCount    */
    uint32_t selection_sequence_start;  /* m_rollBufferSelectionSequenceStart */
    uint32_t selection_sequence_count;  /* m_rollBufferSelectionSequenceCount */
    uint32_t earliest_time_sec;         /* m_rollBufferEarliestTimeSec        */
    uint32_t earliest_time_nsec;        /* m_rollBufferEarliestTimeNSec       */
    uint32_t last_time_sec;             /* m_rollBufferLastTimeSec            */
    uint32_t last_time_nsec;            /* m_rollBufferLastTimeNSec           */
} gdf_rollbuffer_state;

/* Parameters of one depth-fusion frame: the GPUDepthmapFusionComponent parameters read in
 * onInit (src/gpu_depthmap_fusion_component.cpp:1115-1187) plus the move-frame transforms
 * looked up per frame (component.cpp:192-197). */
typedef struct gdf_frame_params {
    /* point-sequence (lidar) chain, component.cpp:158-211 */
    float ps_filter_threshold;          /* point_sequence_flying_pixel_filter_threshold */
    uint32_t ps_filter_size;            /* point_sequence_flying_pixel_filter_size      */
    float ps_timespan;                  /* point_sequence_aggregation_timespan [s]      */
    int32_t move_transform_available;   /* canTransform(world, move) && canTransform(crop, move) */
    float T_world_move[16];
    float T_crop_move[16];
    /* depth chain, component.cpp:228-300 */
    uint32_t flying_filter_size;        /* flyingpixels_filter_size        */
    float flying_threshold;             /* flyingpixels_filter_threshold   */
    int32_t flying_rot45;               /* flyingpixels_filter_enable_rot45 */
    float crop_min[3];
    float crop_max[3];
    int32_t enable_voxel_filter;        /* enable_voxel_filter              */
    float voxel_min[3];
    float voxel_max[3];
    float voxel_size[3];
    int32_t voxel_average;              /* voxel_filter_enable_average       */
    uint32_t occupancy_lifetime;        /* voxel_occupancy_lifetime          */
    int32_t defer_occupancy_grid;       /* 1: stop after the voxel keys / occupancy marks / voxelize;
                                           the caller merges marks across ranks and then calls
                                           gdf_voxel_occupancy_grid (multi-GPU exchange step)  */
    int32_t synchronous;                /* 1: wait for the frame and fill the host mirrors
                                           (m_points / m_points_voxelized / m_occupancyGrid),
                                           0: enqueue only (results stay on the device)      */
    int32_t defer_voxelize;             /* 1: compute the voxel keys and occupancy marks but no
                                           voxelize: the caller exchanges the (point, key) lists
                                           across ranks and voxelizes them with
                                           gdf_voxelize_points (multi-GPU fused cloud)        */
} gdf_frame_params;

/* What gdf_process_frame produced (counts are only valid when synchronous != 0). */
typedef struct gdf_frame_result {
    int32_t processed;                  /* 0 when there was nothing to do (no depth, no points) */
    uint32_t num_depth_points;          /* m_depthmapsTotalElements            */
    uint32_t num_points_total;          /* m_numPointsTotal (depth + selected) */
    uint32_t num_points;                /* m_numItemsAfterMask                 */
    uint32_t num_voxelized;             /* m_points_voxelized.size()           */
    uint32_t latest_time_sec;           /* header stamp chosen by the component (overallLatestTime) */
    uint32_t latest_time_nsec;
} gdf_frame_result;

/* ---- lifetime ------------------------------------------------------------------------- */
/* GPUDepthmapFusion() + init(shaderPath) (gpu_depthmap_fusion.cpp:16-128): allocates the
 * device arena on HIP device `device` and creates the engine's stream. */
int gdf_create(int device, gdf_engine** out_engine);
int gdf_destroy(gdf_engine* engine);
const char* gdf_last_error(void);
int gdf_version(int* major, int* minor);
/* Build provenance (no reference counterpart): "source_sha=<digest of the sources the library
 * was compiled from>;built_on=<host>;built_at=<UTC time>" - which build a process loaded. */
const char* gdf_build_info(void);
/* Use a caller-owned hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL restores
 * the engine's own stream. */
int gdf_set_stream(gdf_engine* engine, void* hip_stream);
int gdf_synchronize(gdf_engine* engine);
/* The stream the engine's current frame is enqueued on (for consumers ordered after it). */
int gdf_get_stream(gdf_engine* engine, void** out_stream);
/* Frame pipelining (1..4, default 1): gdf_clear starts a frame on the next of `depth` slots,
 * each with its own stream and per-frame buffers, so a frame's compaction overlaps the previous
 * frame's sort / grouping.  Shared state stays ordered: grid updates run in frame order, frames
 * that touch the rollbuffer or rebuild camera tables wait for the previous frame.  Results of a
 * frame are read (downloads, gdf_get_device_results) before the next gdf_clear.  Call between
 * frames; not available with gdf_set_stream. */
int gdf_set_pipeline_depth(gdf_engine* engine, int depth);
/* The slot the engine's calls address (after gdf_clear: the new frame's), and its re-selection:
 * the follow-up calls of a frame still resident in its slot (gdf_take_occupancy_marks,
 * gdf_partition_points, gdf_voxelize_points, downloads) after later frames were started on other
 * slots - the multi-GPU exchange finishes batch b while batch b + 1 computes.  gdf_get_stream then
 * names that slot's stream.  The next gdf_clear continues the rotation after the most recently
 * cleared slot, whatever slot is selected.  (No reference counterpart: the reference runs one
 * frame at a time.) */
int gdf_get_slot(gdf_engine* engine, int* slot);
/* The pipeline slots' streams from the caller (e.g. torch streams, so the caller's allocator and
 * collectives share them): slot i runs on streams[i] (i < n; the others keep the engine's own);
 * the engine synchronises but never destroys them.  n = 0 restores the engine's streams.  Not
 * with gdf_set_stream. */
int gdf_set_slot_streams(gdf_engine* engine, void* const* streams, int n);
int gdf_select_slot(gdf_engine* engine, int slot);
/* Steady-state frames of gdf_process_frame as HIP graphs (default on; env GDF_NO_GRAPHS turns
 * the default off): when a slot's frame repeats the launch arguments of its previous frame (all
 * but the depth pointers and the grid ticket) the frame's launches are captured once and then
 * replayed - one graph launch per frame instead of six kernel launches.  Results are identical;
 * not used while profiling, with stage-mask debugging, gdf_set_stream or more than 4 cameras. */
int gdf_set_graphs(gdf_engine* engine, int enable);
/* voxel_group_size parameter (component.cpp:1149); kept for interface parity, it only tuned
 * the reference's CPU radix sort and does not change results. */
int gdf_set_voxel_group_size(gdf_engine* engine, int group_size);

/* ---- per-frame inputs ------------------------------------------------------------------ */
/* GPUDepthmapFusion::clear() (gpu_depthmap_fusion.cpp:725-732). */
int gdf_clear(gdf_engine* engine);
/* addDepthmap (gpu_depthmap_fusion.cpp:798-816).  `depth` is a HOST pointer to width*height
 * uint16 depth values; like the reference it is borrowed (not copied) until
 * gdf_upload_depthmaps returns. */
int gdf_add_depthmap(gdf_engine* engine, const uint16_t* depth, uint32_t width, uint32_t height,
                     float depth_scale, float fx, float fy, float cx, float cy,
                     const float T_world[16], const float T_crop[16]);
/* Multi-GPU (one camera per rank): the camera that precedes this engine's first camera in the
 * reference's concatenated buffer (rank k-1's camera), of which only the last `tail_pixels`
 * depth values are given (device memory; >= F rows + F pixels of this engine's first camera).
 * The flying-pixel reads of the first camera's top rows land there exactly as in the
 * reference's single buffer; the halo camera emits no points.  Call after
 * gdf_clear, before the depth maps; borrowed like gdf_add_depthmap_device's pointer. */
int gdf_add_halo_depthmap_device(gdf_engine* engine, const uint16_t* tail_device,
                                 uint32_t tail_pixels, uint32_t width, uint32_t height,
                                 float depth_scale, float fx, float fy, float cx, float cy,
                                 const float T_world[16], const float T_crop[16]);
/* Same, for a depth map already resident in device memory of this engine's GPU (no copy). */
int gdf_add_depthmap_device(gdf_engine* engine, const uint16_t* depth_device, uint32_t width,
                            uint32_t height, float depth_scale, float fx, float fy, float cx,
                            float cy, const float T_world[16], const float T_crop[16]);
/* addPointSequence (gpu_depthmap_fusion.cpp:747-796): copies x,y,z (float32 at byte offsets
 * 0, 4, 8 of each point_step record, the PointCloud2 layout) with w = 1 into the collect
 * buffer.  Thread-safe with respect to the frame calls. */
int gdf_add_point_sequence(gdf_engine* engine, const void* records, uint32_t num_points,
                           uint32_t point_step, uint32_t time_sec, uint32_t time_nsec,
                           const float T_move[16]);
/* Same, for PointCloud2 records already resident in device memory of this engine's GPU
 * (point_step a multiple of 4, records 4-byte aligned): borrowed like gdf_add_depthmap's pointer,
 * valid until the next gdf_upload_point_sequences / gdf_process_frame, which gathers x,y,z on the
 * device (no host copy, no PCIe). */
int gdf_add_point_sequence_device(gdf_engine* engine, const void* records_device,
                                  uint32_t num_points, uint32_t point_step, uint32_t time_sec,
                                  uint32_t time_nsec, const float T_move[16]);
/* numCollectedPointSequencePoints() (gpu_depthmap_fusion.h:356). */
int gdf_num_collected_point_sequence_points(gdf_engine* engine, uint32_t* out_count);

/* ---- point-sequence rollbuffer chain --------------------------------------------------- */
int gdf_upload_point_sequences(gdf_engine* engine);                      /* :819-857   */
int gdf_filter_new_point_sequences(gdf_engine* engine, float threshold,
                                   uint32_t filter_size);                /* :928-976   */
int gdf_insert_new_point_sequences(gdf_engine* engine);                  /* :979-1087  */
int gdf_roll_rollbuffer(gdf_engine* engine, uint32_t min_sec,
                        uint32_t min_nsec);                               /* :1098-1217 */
int gdf_select_timespan(gdf_engine* engine, uint32_t min_sec, uint32_t min_nsec,
                        uint32_t max_sec, uint32_t max_nsec);             /* :1358-1416 */
int gdf_prepare_point_and_mask_buffers(gdf_engine* engine);              /* :1497-1508 */
int gdf_insert_selected_point_sequence(gdf_engine* engine, const float T_world_move[16],
                                       const float T_crop_move[16]);     /* :1509-1553 */
int gdf_transform_point_sequence(gdf_engine* engine);                    /* :1555-1581 */
int gdf_get_rollbuffer_state(gdf_engine* engine, gdf_rollbuffer_state* out);

/* Rollbuffer sharding (not in the reference: the multi-GPU window, include/gdf_fused.h).  Every
 * shard is given EVERY point sequence (same order, same frames); sequence k (the k-th inserted
 * since this call) keeps its points on shard (k / block) % nshards only, and enters the other
 * shards' rollbuffers as a header without points.  So every shard rolls and selects the same
 * sequences by time (rollPointSequenceRollbufferCPU / selectPointSequenceTimespanCPU depend only
 * on the headers, fusion.cpp:1098-1217, 1358-1416) and holds ~1/nshards of the window; the shards'
 * selected points, placed piece by piece in gdf_get_rollbuffer_pieces' order, are the unsharded
 * selection (the point filter still sees every new point: its neighbours cross sequences).  The
 * rollbuffer state then counts the shard's own points.  Set before the first sequence is
 * inserted; nshards = 1: off. */
int gdf_set_rollbuffer_shard(gdf_engine* engine, uint32_t shard, uint32_t nshards, uint32_t block);
/* The pieces of the selected window in the selection's order (after the frame's selection): a
 * piece is a maximal stretch of selected sequences with points held by one shard; owners[i] = the
 * shard holding piece i.  *count = the number of pieces (GDF_ERR_CAPACITY when it exceeds
 * capacity).  A shard's rollbuffer points are its pieces in this order; with a window spanning
 * more than nshards blocks a shard holds several (the fused step cuts them apart, gdf_fused.h).
 * Unsharded: one piece, owner 0. */
int gdf_get_rollbuffer_pieces(gdf_engine* engine, uint32_t* owners, uint32_t capacity, uint32_t* count);

/* ---- depth chain ------------------------------------------------------------------------ */
int gdf_upload_depthmaps(gdf_engine* engine);                            /* :1583-1593 */
int gdf_convert_depthmaps(gdf_engine* engine);                           /* :1595-1628 */
int gdf_filter_flying_pixels(gdf_engine* engine, uint32_t filter_size, float threshold,
                             int enable_rot45);                          /* :1629-1648 */
int gdf_crop_points(gdf_engine* engine, const float lower[3],
                    const float upper[3]);                               /* :1649-1660 */
/* applyPointMask (:1661-1678): ordered compaction (pixel order, cameras in add order, selected
 * rollbuffer points after the depth points).  Writes the count when out_count != NULL (this
 * waits for the device, like the reference's blocking count download). */
int gdf_apply_point_mask(gdf_engine* engine, uint32_t* out_count);
int gdf_compute_voxel_coords(gdf_engine* engine, const float lower[3], const float upper[3],
                             const float cell_size[3]);                  /* :1680-1711 */
/* voxelize (:1743-1756): stable radix sort of the voxel keys + per-voxel mean (average != 0)
 * or voxel lower corner (average == 0), on the GPU. */
int gdf_voxelize(gdf_engine* engine, int average_voxels);
/* voxelOccupancyGrid (:1757-1823): decaying occupancy with `lifetime`. */
int gdf_voxel_occupancy_grid(gdf_engine* engine, uint32_t lifetime);

/* ---- results (device -> host) ----------------------------------------------------------- */
int gdf_get_point_count(gdf_engine* engine, uint32_t* out_count);        /* m_numItemsAfterMask */
/* downloadPoints (:2946-2951): compacted world points, float4[count]. */
int gdf_download_points(gdf_engine* engine, float* out_xyzw, uint32_t capacity,
                        uint32_t* out_count);
/* downloadVoxelCoords (:1712-1718): voxel index per compacted point. */
int gdf_download_voxel_coords(gdf_engine* engine, uint32_t* out, uint32_t capacity,
                              uint32_t* out_count);
/* m_points_voxelized after voxelize. */
int gdf_download_voxelized_points(gdf_engine* engine, float* out_xyzw, uint32_t capacity,
                                  uint32_t* out_count);
/* downloadVoxelOccupancyGrid (:1824-1839): uint8 per cell, x fastest, then y, then z. */
int gdf_download_occupancy_grid(gdf_engine* engine, uint8_t* out, uint64_t capacity);
/* VoxelGridMeta (gpu_depthmap_fusion.h:507): grid size per axis and cell count. */
int gdf_get_grid_size(gdf_engine* engine, uint32_t grid_size[3], uint64_t* num_cells);
/* Device pointers of the results (valid until the next frame call), for zero-copy consumers. */
int gdf_get_device_results(gdf_engine* engine, const float** points, const uint32_t** coords,
                           const float** voxelized, const uint8_t** occupancy);

/* All of a frame's host-side outputs at once (the component downloads points, voxel coords, the
 * voxelized cloud and the u8 grid every frame, component.cpp:297-401): the copies run on the
 * frame's stream into engine-owned pinned host mirrors of the addressed slot, with one wait for
 * them all; the pointers stay valid until the slot's next gdf_download_frame (or gdf_destroy):
 * frames processed in between write their prefetched downloads into a second set of mirrors, never
 * into the set last handed out.  Memory: the mirrors are pinned host memory sized to the largest
 * frame downloaded - 36 B per point (points 16, coords 4, voxelized 16, the latter per voxel at
 * most) plus the grid's cells - and a slot holds two sets once frames are downloaded while others
 * run: ~72 B per point per slot (a rollbuffer window of 10^8 surviving points: ~7 GB per slot);
 * download only the members needed (`what`) for such windows.
 * `what` is a mask of GDF_DL_*; members not asked for are NULL / 0.  (No single reference
 * counterpart: it replaces downloadPoints + downloadVoxelCoords + the voxelized download +
 * downloadVoxelOccupancyGrid, fusion.cpp:1712-1718, 1824-1839, 2946-2951.) */
#define GDF_DL_POINTS 1u
#define GDF_DL_COORDS 2u
#define GDF_DL_VOXELIZED 4u
#define GDF_DL_GRID 8u
typedef struct gdf_host_frame {
    const float* points;            /* float4[num_points]  (m_points)            */
    const uint32_t* voxel_coords;   /* uint32[num_points]  (m_voxelCoords)       */
    uint32_t num_points;
    const float* voxelized;         /* float4[num_voxelized] (m_points_voxelized) */
    uint32_t num_voxelized;
    const uint8_t* occupancy;       /* uint8[num_cells]    (m_occupancyGrid)     */
    uint64_t num_cells;
} gdf_host_frame;
int gdf_download_frame(gdf_engine* engine, uint32_t what, gdf_host_frame* out);

/* ---- whole frame -------------------------------------------------------------------------- */
/* The per-frame sequence of GPUDepthmapFusionComponent::processDepthmaps
 * (component.cpp:92-300) from uploadPointSequences through downloadVoxelOccupancyGrid, for the
 * depth maps added since gdf_clear.  Runs the fused kernels (one compaction launch for depth +
 * rollbuffer points with voxel keys and occupancy marks, one grid launch, the GPU voxelize). */
int gdf_process_frame(gdf_engine* engine, const gdf_frame_params* params,
                      gdf_frame_result* out_result);

/* Instrumentation (no reference counterpart): frame-graph captures and replays so far (every slot;
 * each slot keeps the graphs of up to 4 launch-argument sets, least recently used evicted). */
int gdf_get_graph_stats(gdf_engine* engine, uint64_t* captures, uint64_t* replays);
/* Instrumentation (no reference counterpart): the items the last synchronous gdf_process_frame's
 * voxelize sorted - runs of equal voxel keys (*runs = 1) or points (*runs = 0). */
int gdf_last_sort_items(gdf_engine* engine, uint32_t* items, int* runs);

/* ---- orphan shaders of the reference (device buffers, the engine's stream) ------------------ */
/* mask_dilate (shader/mask_dilate.glsl:40-67; never dispatched by the reference): for every pixel
 * of a width x height u32 mask, a zero in the (2F+1)^2 window clipped to the image writes 0;
 * as_written != 0 reproduces line 67 (the other pixels are written 0 too), as_written == 0 is the
 * intended erosion (they keep their value).  F <= 16; in and out must not alias. */
int gdf_mask_dilate(gdf_engine* engine, const uint32_t* in_mask_device, uint32_t* out_mask_device,
                    uint32_t width, uint32_t height, uint32_t filter_size, int as_written);
/* transform_points (shader/transform_points.glsl:37-54; orphan sibling of the indirect form the
 * rollbuffer uses): out[i] = T * in[i] for i < num_items with mask[i] != 0 (float4 points,
 * T row-major); other outputs are left unwritten. */
int gdf_transform_points(gdf_engine* engine, const float* in_points_device,
                         const uint32_t* mask_device, float* out_points_device, uint32_t num_items,
                         const float T[16]);

/* ---- multi-frame batches ------------------------------------------------------------------- */
/* Several depth-only frames through ONE launch chain (the per-frame sequence of
 * GPUDepthmapFusionComponent::processDepthmaps, component.cpp:92-300, applied to each frame; a
 * throughput mode for streams whose frames are launch-latency bound on the GPU, e.g. VGA).
 * After gdf_clear and the depth maps of frame 0, gdf_next_frame_in_batch starts frame 1 of the
 * same batch, and so on (<= 16 frames, each with >= 1 depth map); gdf_process_frame then runs
 * every frame: each frame's points, voxel keys, voxel means and grid update are exactly those of
 * processing the frames one by one (flying-pixel neighbour reads stay inside their frame, the
 * grid updates apply in frame order).  Results: the compacted points / keys / voxel means of all
 * frames back to back, frame f at [point_start[f], point_start[f+1]) and
 * [voxel_start[f], voxel_start[f+1]) (gdf_get_batch_ranges, nframes + 1 entries each); the u8
 * grid after frame f from gdf_download_batch_occupancy_grid (the batch's grid update keeps the
 * frames' grids as sparse snapshots).  Not with point sequences; the grid update is the fused
 * one (lifetime <= 255), or - deferred voxelize + deferred grid, the multi-GPU exchange -
 * gdf_voxel_occupancy_grid_batch after gdf_take_occupancy_marks, whose u32 history branch
 * (lifetime > 255) keeps no per-frame grids (their download fails with GDF_ERR_STATE). */
int gdf_next_frame_in_batch(gdf_engine* engine);
int gdf_get_batch_ranges(gdf_engine* engine, uint32_t* point_start, uint32_t* voxel_start,
                         uint32_t capacity, uint32_t* out_frames);
int gdf_download_batch_occupancy_grid(gdf_engine* engine, uint32_t frame, uint8_t* out,
                                      uint64_t capacity);

/* ---- multi-GPU (one camera per rank) ------------------------------------------------------- */
/* Per-frame occupancy marks of this rank as a bitmask of ceil(num_cells/32) uint32 words, and
 * the merge of all ranks' masks (bitwise OR of `num_ranks` masks laid out back to back, as
 * produced by an all-gather) back into this engine before gdf_voxel_occupancy_grid. */
int gdf_export_occupancy_marks(gdf_engine* engine, uint32_t* device_bitmask, uint64_t words);
int gdf_import_occupancy_marks(gdf_engine* engine, const uint32_t* device_bitmasks,
                               uint64_t words, uint32_t num_ranks);
/* Batched exchange (several frames per collective, frames pipelined): gdf_take_occupancy_marks
 * exports the marks of the frame just processed (defer_occupancy_grid = 1) AND clears them, so
 * the engine can run the next frames; once the masks of a batch are all-gathered, each frame's
 * union is imported in frame order - mask r of that frame at device_bitmasks + r *
 * rank_stride_words - and followed by its gdf_voxel_occupancy_grid.  Same grids as the per-frame
 * exchange.  A multi-frame batch (gdf_next_frame_in_batch) takes every frame's marks at once -
 * frame f at device_bitmask + f * words - and needs words >= num_frames * ceil(num_cells/32)
 * (GDF_ERR_CAPACITY otherwise: a partial take would leave frames' marks set). */
int gdf_take_occupancy_marks(gdf_engine* engine, uint32_t* device_bitmask, uint64_t words);
int gdf_import_occupancy_marks_strided(gdf_engine* engine, const uint32_t* device_bitmasks,
                                       uint64_t words, uint32_t num_ranks,
                                       uint64_t rank_stride_words);
/* The grid updates of `num_frames` such frames in ONE pass (voxelOccupancyGrid applied frame
 * after frame in registers): frame f's union is the OR over ranks r of the masks at
 * device_bitmasks + r * rank_stride_words + f * frame_stride_words.  Equals num_frames
 * import + gdf_voxel_occupancy_grid pairs; call after taking every frame's marks. */
/* Sparse form of the take (the marks are ~1-2 % of the cells): besides the bitmask, the
 * non-zero words as (index, word) pairs in `pairs` (device, 1 + 2 * cap words): pairs[0] = their
 * number (> cap: only the bitmask is complete, exchange the bitmasks), then the pairs.
 * gdf_union_occupancy_pairs ORs nranks x nframes such records - record (r, f) at
 * pairs + (r * frames_per_rank + f) * record_words, f < nframes <= frames_per_rank (a partial
 * batch of an all-gathered [rank, batch, record] buffer), each read up to its cap
 * (record_words - 1) / 2 - into union_bits[f * words + i] (zeroed first), the input of
 * gdf_voxel_occupancy_grid_batch with one rank.  Single frames only (GDF_ERR_STATE for a
 * multi-frame batch: take its marks with gdf_take_occupancy_marks). */
int gdf_take_occupancy_marks_sparse(gdf_engine* engine, uint32_t* device_bitmask, uint64_t words,
                                    uint32_t* device_pairs, uint32_t cap);
int gdf_union_occupancy_pairs(gdf_engine* engine, uint32_t* device_union_bitmasks, uint64_t words,
                              const uint32_t* device_pairs, uint32_t num_ranks,
                              uint32_t num_frames, uint32_t frames_per_rank,
                              uint64_t record_words);
int gdf_voxel_occupancy_grid_batch(gdf_engine* engine, const uint32_t* device_bitmasks,
                                   uint64_t words, uint32_t num_ranks, uint32_t num_frames,
                                   uint64_t frame_stride_words, uint64_t rank_stride_words,
                                   uint32_t lifetime);

/* Fused voxel cloud across ranks (the reference voxelizes the points of ALL cameras in one
 * stable sort, fusion.cpp:1743-1756): gdf_partition_points splits the frame's compacted
 * (point, key) list (gdf_process_frame with defer_voxelize = 1) by voxel-key range - part
 * p = min(floor(key / 32) / S, nparts - 1), S = ceil(ceil(num_cells / 32) / nparts): whole
 * 32-cell occupancy-mark words per part - into part-major send buffers (device, >= the frame's
 * points), stable inside each part, with part_counts[p] (device, nparts words).  After an
 * all-to-all (rank r receives part r of every rank, in rank order = camera order) each rank
 * calls gdf_voxelize_points on what it received: its key range of m_points_voxelized, equal to
 * the single-engine result over all cameras (gdf_download_voxelized_points). */
int gdf_partition_points(gdf_engine* engine, uint32_t nparts, float* send_points_device,
                         uint32_t* send_keys_device, uint32_t capacity,
                         uint32_t* part_counts_device);
int gdf_voxelize_points(gdf_engine* engine, const float* points_device,
                        const uint32_t* keys_device, uint32_t count, int average_voxels);
/* The same exchange with RUNS instead of per-point keys: gdf_partition_runs writes the part-major
 * points plus each part's runs of equal keys - consecutive points of one voxel (of one frame of a
 * batch: the run keys carry the frame above the voxel key, as gdf_partition_points' keys) - as run
 * keys and run starts relative to the part's first point; part_counts (device, 2 * nparts words):
 * points per part, then runs per part.  A rank that received nsources such segments, concatenated
 * in rank order (points of source q from point_base[q], its runs from run_base[q]; host arrays of
 * nsources + 1 entries, the last the totals), calls gdf_voxelize_runs: the run starts are rebased
 * in place (run_starts needs run_base[nsources] + 1 entries) and the voxelize sorts the runs - the
 * same voxel means as gdf_voxelize_points over the same points. */
int gdf_partition_runs(gdf_engine* engine, uint32_t nparts, float* send_points_device,
                       uint32_t* send_run_keys_device, uint32_t* send_run_starts_device,
                       uint32_t capacity, uint32_t* part_counts_device);
/* gdf_partition_runs' send lists written by the next frame's compaction itself: arm before a
 * gdf_process_frame with defer_voxelize (capacity >= that frame's pixels + selected points); that
 * frame's k_mask / k_emit count and place every kept point and run per part (no compaction-order
 * points, keys or runs: the frame's point / coords downloads are not available), or - frames the
 * fused kernels do not cover (rollbuffer points, other segment shapes) - compact and then
 * partition.  The same send lists and part_counts either way; disarmed after that frame
 * (nparts = 0 disarms explicitly). */
int gdf_set_emit_partition(gdf_engine* engine, uint32_t nparts, float* send_points_device,
                           uint32_t* send_run_keys_device, uint32_t* send_run_starts_device,
                           uint32_t capacity, uint32_t* part_counts_device);
/* nseg (1..4, nparts * nseg <= 32) for the armed frame: each part is cut into nseg buckets,
 * [the frame's depth points | the pieces of the selection this engine holds, in order] (bucket
 * b = part * nseg + segment, bucket-major send lists, run starts relative to the bucket's first
 * point, part_counts [nseg nparts points | nseg nparts runs]; a sharded window's shard holding
 * more pieces than nseg - 1 fails the frame with GDF_ERR_STATE, on every shard alike): the
 * multi-GPU step places the ranks' rollbuffer pieces behind every rank's depth points, in the
 * selection's order (the reference's buffer order, fusion.cpp:1509-1581).  A frame without a
 * selection keeps this layout with every rollbuffer bucket empty (the compaction writes the counts
 * so).  Disarmed (1) with the emit partition. */
int gdf_set_partition_segments(gdf_engine* engine, uint32_t nseg);
/* Whether a deferred frame armed with gdf_set_emit_partition sets its occupancy marks (default 1).
 * 0: a caller that builds the union from gdf_voxelize_runs_marked skips the compaction's marks
 * (and their clear) - the frame then has no marks to take. */
int gdf_set_partition_marks(gdf_engine* engine, int enabled);
int gdf_voxelize_runs(gdf_engine* engine, const float* points_device,
                      const uint32_t* run_keys_device, uint32_t* run_starts_device,
                      uint32_t nsources, const uint32_t* point_base, const uint32_t* run_base,
                      int average_voxels);
/* gdf_voxelize_runs that also ORs every voxel's occupancy mark into marks_device (device; frame f
 * of a batch at f * frame_stride_words, >= the grid's mark words; the caller zeroes it).  With the
 * word-range parts above, rank j's voxels mark exactly words [j S, (j + 1) S) of each frame, so an
 * in-place all-gather of those slices is the union of every rank's marks (gdf_fused.cpp: 1 / W of
 * the full bitmasks' all-gather volume), ready for gdf_voxel_occupancy_grid_batch. */
int gdf_voxelize_runs_marked(gdf_engine* engine, const float* points_device,
                             const uint32_t* run_keys_device, uint32_t* run_starts_device,
                             uint32_t nsources, const uint32_t* point_base, const uint32_t* run_base,
                             int average_voxels, uint32_t* marks_device, uint64_t frame_stride_words);
/* The multi-GPU step's receive side (include/gdf_fused.h) with its fixed work folded into the
 * rebase pass: as gdf_voxelize_runs_marked, where `own` names up to 4 sources that are still in
 * THIS rank's send lists (its own buckets: read from there - run starts rebased, points and run
 * keys written into pts / run_keys at their place - instead of device copies first) and mark
 * words to clear before the voxelize marks its voxels (clear_rows rows of clear_row_words at
 * clear_stride_words: the key range's slice of each frame). */
typedef struct gdf_recv_own {
    uint32_t count;
    uint32_t source[4];
    const float* points[4];
    const uint32_t* run_keys[4];
    const uint32_t* run_starts[4];
    uint32_t* clear;
    uint64_t clear_row_words, clear_stride_words;
    uint32_t clear_rows;
} gdf_recv_own;
int gdf_voxelize_runs_recv(gdf_engine* engine, float* points, uint32_t* run_keys,
                           uint32_t* run_starts, uint32_t nsources, const uint32_t* point_base,
                           const uint32_t* run_base, int average, uint32_t* marks,
                           uint64_t frame_stride_words, const gdf_recv_own* own);

/* ---- live kernel timing (HIP events on the engine stream) ------------------------------------ */
enum gdf_kernel_slot {
    GDF_KERNEL_FRAME = 0,      /* k_frame: fused convert/flying/crop/transform/compaction(+keys) */
    GDF_KERNEL_GRID = 1,       /* k_grid_u8 / k_grid_u32: historic occupancy update              */
    GDF_KERNEL_VOXELIZE = 2,   /* radix sort passes + group mean                                  */
    GDF_KERNEL_PS_INSERT = 3,  /* point-sequence filter + rollbuffer insert                      */
    /* single kernels inside the groups above (one launch each) */
    GDF_KERNEL_MASK = 4,       /* k_mask: convert + flying-pixel + crop stage bits, tile counts   */
    GDF_KERNEL_SCAN = 5,       /* k_scan_counts (frames over 1 Mi items only)                     */
    GDF_KERNEL_EMIT = 6,       /* k_emit: ordered compaction + voxel keys + marks + digit hist    */
    GDF_KERNEL_SORT = 7,       /* k_sort_pass: one radix pass (the first also updates the grid)   */
    GDF_KERNEL_GROUP = 8,      /* k_group: voxel groups of the sorted keys + ordered per-voxel means */
    GDF_KERNEL_SEL = 9,        /* k_sel + k_sel_place: single-pass rollbuffer compaction      */
    GDF_KERNEL_EVENT_FLOOR = 10, /* an event pair around no launch: the timing method's own cost    */
    GDF_KERNEL_SLOTS = 11
};
/* enable: record an event pair around every launch of each slot; reset clears the sums */
int gdf_set_profiling(gdf_engine* engine, int enable);
/* sum of event-measured milliseconds and number of launches per slot since the last reset
 * (synchronises the engine stream) */
int gdf_get_kernel_times(gdf_engine* engine, double* ms_sum, uint64_t* launches, int slots);

/* The tuning variables (GDF_* launch-shape knobs, none of which changes a result) the engine was
 * created under, as "NAME=value NAME=value" ("" when none: every built-in default).  Each engine
 * keeps the snapshot taken at gdf_create - engines created under other environments never retune
 * it - and gdf_create logs a non-empty one to stderr. */
int gdf_get_tuning(gdf_engine* engine, char* buf, uint32_t capacity);

/* ---- debug / parity hooks ------------------------------------------------------------------ */
/* Keep per-point stage masks of the next compaction launch: bit0 = valid after convert
 * (depth != 0 or rollbuffer mask != 0), bit1 = after the flying-pixel filter, bit2 = after crop. */
int gdf_set_debug(gdf_engine* engine, int enable);
int gdf_debug_stage_masks(gdf_engine* engine, uint8_t* out, uint32_t capacity,
                          uint32_t* out_count);
/* The rollbuffer in the reference's logical layout (the B buffers after a roll): points,
 * mask (0/1) and sequence index per point; sequence headers (sec, nsec, start, numPoints). */
int gdf_debug_rollbuffer(gdf_engine* engine, float* points_xyzw, uint32_t* mask,
                         uint32_t* seq_idx, uint32_t capacity, uint32_t* header_sec_nsec_start_num,
                         uint32_t header_capacity);
/* The historic occupancy grid as uint32 per cell (m_bufHistoricVoxelOccupancyA). */
int gdf_debug_historic_grid(gdf_engine* engine, uint32_t* out, uint64_t capacity);

#ifdef __cplusplus
}
#endif

#endif /* GDF_H_ */
