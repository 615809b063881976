/*
 * gdf_oracle.h — CPU restatement of the reference's depth-fusion hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this; the product (ros_gpu_depthmap_fusion_amd/) never links or calls it.
 *
 * The oracle keeps the reference's logical buffers (MaskA/MaskB, PointsA/B/C, the rollbuffer
 * A/B arrays, the u32 historic occupancy grid) and runs the reference's kernels one stage at a
 * time, each function citing the GLSL shader / host method it restates.  Floating-point
 * semantics are pinned as SURVEY.md Appendix A: IEEE-754 binary32, correctly rounded / and
 * sqrt, no FMA contraction (-ffp-contract=off), explicit summation order.
 *
 * Parity pinning: the radix sort + grouping is checked against the reference's own
 * include/gpu_depthmap_fusion/radix_grouper.h + radix_sort.h compiled into oracle/_ref
 * (oracle/Makefile), and against tests/golden/ fixtures generated from it.  The GLSL stages
 * cannot execute in this container (no GL 4.3 context, no EGL/OSMesa, no GPU)
 * and the reference ships no tests or golden vectors, so for those stages parity is
 * "unpinned": the oracle restates the shader source line by line and is pinned by the
 * hand-computed known-answer tests in tests/test_oracle_kat.py.
 */
#ifndef GDF_ORACLE_H_
#define GDF_ORACLE_H_

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_state orc_state;

orc_state* orc_create(void);
void orc_destroy(orc_state* s);
void orc_set_threads(orc_state* s, int nthreads);

void orc_clear(orc_state* s);
int orc_add_depthmap(orc_state* s, const uint16_t* depth, uint32_t width, uint32_t height,
                     float depth_scale, float fx, float fy, float cx, float cy,
                     const float T_world[16], const float T_crop[16]);
int orc_add_point_sequence(orc_state* s, const void* records, uint32_t num_points,
                           uint32_t point_step, uint32_t sec, uint32_t nsec,
                           const float T_move[16]);
uint32_t orc_num_collected_point_sequence_points(orc_state* s);

int orc_upload_point_sequences(orc_state* s);
int orc_filter_new_point_sequences(orc_state* s, float threshold, uint32_t filter_size);
int orc_insert_new_point_sequences(orc_state* s);
int orc_roll_rollbuffer(orc_state* s, uint32_t min_sec, uint32_t min_nsec);
int orc_select_timespan(orc_state* s, uint32_t min_sec, uint32_t min_nsec, uint32_t max_sec,
                        uint32_t max_nsec);
int orc_prepare_point_and_mask_buffers(orc_state* s);
int orc_insert_selected_point_sequence(orc_state* s, const float T_world_move[16],
                                       const float T_crop_move[16]);
int orc_transform_point_sequence(orc_state* s);

int orc_upload_depthmaps(orc_state* s);
int orc_convert_depthmaps(orc_state* s);
int orc_filter_flying_pixels(orc_state* s, uint32_t filter_size, float threshold, int rot45);
int orc_crop_points(orc_state* s, const float lower[3], const float upper[3]);
int orc_apply_point_mask(orc_state* s, uint32_t* out_count);
int orc_compute_voxel_coords(orc_state* s, const float lower[3], const float upper[3],
                             const float cell_size[3]);
int orc_voxelize(orc_state* s, int average);
int orc_voxel_occupancy_grid(orc_state* s, uint32_t lifetime);

/* frame driver: GPUDepthmapFusionComponent::processDepthmaps (component.cpp:92-300) */
typedef struct orc_frame_params {
    float ps_filter_threshold;
    uint32_t ps_filter_size;
    float ps_timespan;
    int32_t move_transform_available;
    float T_world_move[16];
    float T_crop_move[16];
    uint32_t flying_filter_size;
    float flying_threshold;
    int32_t flying_rot45;
    float crop_min[3];
    float crop_max[3];
    int32_t enable_voxel_filter;
    float voxel_min[3];
    float voxel_max[3];
    float voxel_size[3];
    int32_t voxel_average;
    uint32_t occupancy_lifetime;
    int32_t synchronous;
} orc_frame_params;
int orc_process_frame(orc_state* s, const orc_frame_params* p, int32_t* processed,
                      uint32_t* latest_sec, uint32_t* latest_nsec);

/* ros::Time(sec,nsec) - ros::Duration(seconds) as in roscpp_core; returns -1 if ros would throw */
int orc_ros_time_minus(uint32_t sec, uint32_t nsec, double seconds, uint32_t* out_sec,
                       uint32_t* out_nsec);

/* accessors (pointers stay valid until the next call that resizes them) */
uint32_t orc_num_points_total(orc_state* s);        /* n = depth + selected */
uint32_t orc_num_depth_points(orc_state* s);
uint32_t orc_num_points(orc_state* s);              /* after compaction */
const uint32_t* orc_mask_a(orc_state* s);
const uint32_t* orc_mask_b(orc_state* s);
const float* orc_points_a(orc_state* s);
const float* orc_points_b(orc_state* s);
const float* orc_points_c(orc_state* s);
const uint32_t* orc_voxel_coords(orc_state* s);
const float* orc_voxelized(orc_state* s, uint32_t* count);
const uint8_t* orc_occupancy(orc_state* s, uint64_t* num_cells);
const uint32_t* orc_historic(orc_state* s, uint64_t* num_cells);
void orc_grid_size(orc_state* s, uint32_t gs[3]);
const uint32_t* orc_new_ps_mask(orc_state* s, uint32_t* count);
void orc_rollbuffer_state(orc_state* s, uint32_t out[10]);
/* rollbuffer B (post-roll) logical arrays */
uint32_t orc_rollbuffer_b(orc_state* s, const float** pts, const uint32_t** mask,
                          const uint32_t** seq_idx, const uint32_t** headers, uint32_t* nseq);

/* standalone primitives for tests */
/* sh/mask_dilate.glsl:40-67 (orphan in the reference: never dispatched).  For every pixel of a
 * width x height mask (u32 per pixel, at in_mask / out_mask):  the (2F+1)^2 window clipped to the
 * image (the GLSL's `pixel.x + dx < 0` is unsigned arithmetic: never true, but a negative sum
 * wraps to >= width and is skipped by the second check, so the clip is exact);  a zero in the
 * window writes 0 and returns (:58-63).  as_written != 0: line 67 writes 0 for the pixels that
 * pass too (the mask is cleared everywhere); as_written == 0: the intended erosion, the pixel
 * keeps its input value. */
void orc_mask_dilate(const uint32_t* in_mask, uint32_t* out_mask, uint32_t width,
                     uint32_t height, uint32_t filter_size, int as_written);
/* sh/transform_points.glsl:37-54 (orphan sibling of transform_points_indirect): for i < n with
 * mask[i] != 0, out[i] = T * in[i] (T row-major, the reference's `point * transform`); other
 * outputs are left unwritten. */
void orc_transform_points(const float* in_points, const uint32_t* mask, float* out_points,
                          uint32_t n, const float T[16]);
void orc_stable_sort_keys(const uint32_t* keys, uint32_t n, uint32_t* out_sorted_idx,
                          uint32_t* out_sorted_keys);

#ifdef __cplusplus
}
#endif

#endif /* GDF_ORACLE_H_ */
