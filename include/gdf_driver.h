/* gdf_driver.h — the depth-stream loop of GPUDepthmapFusionComponent in C++, over the C-ABI.
 *
 * Not a reference interface: this is the host side of the component's per-frame callback
 * (GPUDepthmapFusionComponent::processDepthmaps, src/gpu_depthmap_fusion_component.cpp:92-300:
 * clear -> addDepthmap per camera -> the processing chain) for a stream of frames already in
 * device memory, written against include/gdf.h only (gdf_clear, gdf_add_depthmap_device,
 * gdf_process_frame).  The ROS component is C++; this loop is what it costs per frame on the host
 * without an interpreter in between.  bench.py drives the timed frames through it.
 */
#ifndef GDF_DRIVER_H
#define GDF_DRIVER_H

#include "gdf.h"

#ifdef __cplusplus
extern "C" {
#endif

/* One camera of the stream: a ring of `ring` device depth maps (width*height uint16 each) with
 * the camera's intrinsics and row-major transforms (the arguments of gdf_add_depthmap_device). */
typedef struct gdf_stream_camera {
    const uint16_t* const* frames;  /* host array of `ring` DEVICE (host: gdf_run_host_stream) pointers */
    uint32_t ring;
    uint32_t width, height;
    float depth_scale, fx, fy, cx, cy;
    float T_world[16];
    float T_crop[16];
} gdf_stream_camera;

/* Runs frames first .. first+count-1: for frame i, camera k contributes
 * frames[(i) % ring]; every frame is clear + add + gdf_process_frame(params).  Returns the first
 * non-zero status (gdf_last_error describes it).  Asynchronous like gdf_process_frame: call
 * gdf_synchronize to wait for the last frame. */
int gdf_run_depth_stream(gdf_engine* engine, const gdf_stream_camera* cameras,
                         uint32_t num_cameras, const gdf_frame_params* params, uint64_t first,
                         uint64_t count);

/* The same loop for HOST depth maps (frames[] are host pointers, gdf_add_depthmap): each frame's
 * maps (pinned or pageable alike) are copied into the frame slot's pinned staging by a few host
 * threads and sent to the device on the slot's stream, overlapping the kernels of the frames in flight
 * (gdf_set_pipeline_depth).  The H2D-inclusive form of gdf_run_depth_stream. */
int gdf_run_host_stream(gdf_engine* engine, const gdf_stream_camera* cameras,
                        uint32_t num_cameras, const gdf_frame_params* params, uint64_t first,
                        uint64_t count);

/* `batches` multi-frame batches of `batch` frames each (gdf_next_frame_in_batch, include/gdf.h):
 * batch b holds frames first + b*batch .. first + (b+1)*batch - 1; host != 0 reads host depth
 * maps like gdf_run_host_stream. */
int gdf_run_depth_stream_batched(gdf_engine* engine, const gdf_stream_camera* cameras,
                                 uint32_t num_cameras, const gdf_frame_params* params,
                                 uint64_t first, uint64_t batches, uint32_t batch, int host);

/* gdf_run_depth_stream_batched with the parameter set changing every step: step b of the call
 * uses params[(first + b) % nparams] (a component whose runtime config topics change the
 * filter parameters between frames, component.cpp:970-990; measures the graph cache). */
int gdf_run_depth_stream_alternating(gdf_engine* engine, const gdf_stream_camera* cameras,
                                     uint32_t num_cameras, const gdf_frame_params* params,
                                     uint32_t nparams, uint64_t first, uint64_t batches,
                                     uint32_t batch);

#ifdef __cplusplus
}
#endif

#endif /* GDF_DRIVER_H */
