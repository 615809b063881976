/*
 * gdf_segment.h — C-ABI of the GPU object-segmentation front end.
 *
 * Replaces the first half of GPUDepthmapFusion::objectSegmentation
 * (src/gpu_depthmap_fusion.cpp:2552-2575): labelVoxels (:1872-2011, OpenCV on the CPU in the
 * reference), uploadVoxelLabels (:2013-2073), prepareLayersConnections (:2075-2151),
 * computeLayersConnections (:2200-2214, shader/layers_connections.glsl:96-122) and
 * downloadLayersConnections (:2215-2241), plus mergeLabelsAcrossLayers (:2243-2361, host).
 * createCCObjects (:2364-2550) without its OpenCV shapes, and objectTracking (:2727-2944), stay out
 * of scope; gdf_seg_create_objects gives the objects' aggregate fields.
 *
 * Input: a device u8 occupancy grid of `layers` z-layers of height x width cells, x fastest
 * (m_occupancyGrid; layer i is the cv::Mat_<uint8_t>(height, width) view m_occupancyLayers[i],
 * fusion.cpp:1824-1839); a cell is foreground when non-zero.  Outputs, all with the reference's
 * layouts (flat, layer after layer):
 *   labels            u16 [layers][height][width]        m_ccLabeledLayersData
 *   num_labels        u32 [layers] (background included)  m_ccNumLabelsPerLayer
 *   stats             i32 [total_labels][5]               m_ccStatsData {LEFT, TOP, WIDTH, HEIGHT, AREA}
 *   centroids         f64 [total_labels][2]               m_ccCentroidsData
 *   labels_to_contours i32 [total_labels]                 m_labelsToContoursPerLayer (-1: none)
 *   contours          per layer, findContours order       m_contoursPerLayer (points x, y)
 *   connections       u8 [sum numA*numB] + starts         m_ccLayersConnectionsData / ...DataStarts
 *   merged            u32 [total_labels]                  m_ccLabelsMerged
 * Label numbering follows OpenCV's default 8-connectivity labelling (components ranked by their
 * first 2x2 block in block-raster order), contours follow findContours(RETR_EXTERNAL,
 * CHAIN_APPROX_NONE) — see DESIGN.md §9 for the restated semantics (parity unpinned: OpenCV is
 * absent from the reference tree and from this image).
 */
#ifndef GDF_SEGMENT_H_
#define GDF_SEGMENT_H_

#include <stdint.h>

#include "gdf.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gdf_segmenter gdf_segmenter;

typedef struct gdf_seg_counts {
    uint32_t width, height, layers;
    uint32_t total_labels;          /* sum of num_labels                    */
    uint32_t total_contours;        /* sum over layers of contours          */
    uint64_t total_contour_points;  /* points of all contours               */
    uint64_t connection_bytes;      /* sum over layer pairs of numA * numB  */
} gdf_seg_counts;

/* flags of gdf_seg_label_layers */
#define GDF_SEG_CONTOURS 1u     /* run findContours + labelsToContours (labelVoxels :1935-1952) */
#define GDF_SEG_CONNECTIONS 2u  /* build the layer connection matrices (:2075-2214)            */
#define GDF_SEG_ALL 3u

int gdf_seg_create(int device, gdf_segmenter** out);
int gdf_seg_destroy(gdf_segmenter* seg);
/* a caller-owned hipStream_t (NULL: the segmenter's own stream) */
int gdf_seg_set_stream(gdf_segmenter* seg, void* hip_stream);

/* objectSegmentation front end (fusion.cpp:2554-2567) on a device grid.  Synchronises the stream
 * once, after the per-layer label counts (they size the stats and the connection matrices, as
 * in the reference, fusion.cpp:2085-2093); the rest is enqueued. */
int gdf_seg_label_layers(gdf_segmenter* seg, const uint8_t* grid_device, uint32_t width,
                         uint32_t height, uint32_t layers, uint32_t flags);
/* the same on an engine's current u8 occupancy grid, on the engine's stream */
int gdf_seg_label_engine_grid(gdf_segmenter* seg, gdf_engine* engine, uint32_t flags);

int gdf_seg_get_counts(gdf_segmenter* seg, gdf_seg_counts* out);
/* downloads (synchronise); capacities in elements of the output type */
int gdf_seg_download_labels(gdf_segmenter* seg, uint16_t* out, uint64_t capacity);
int gdf_seg_download_num_labels(gdf_segmenter* seg, uint32_t* out, uint32_t capacity);
int gdf_seg_download_stats(gdf_segmenter* seg, int32_t* stats5, double* centroids2,
                           uint32_t capacity_labels);
int gdf_seg_download_connections(gdf_segmenter* seg, uint8_t* out, uint64_t capacity,
                                 uint64_t* starts, uint32_t starts_capacity);
/* contours in findContours order, layer after layer: contours_per_layer[layers],
 * sizes[total_contours] (points per contour), points_xy[2 * total_contour_points] */
int gdf_seg_download_contours(gdf_segmenter* seg, int32_t* labels_to_contours,
                              uint32_t* contours_per_layer, uint32_t* sizes, int32_t* points_xy,
                              uint64_t points_capacity);
/* mergeLabelsAcrossLayers (fusion.cpp:2243-2361): merged[label of layer i at
 * sum(num_labels[<i]) + label] and the number of merged objects (background objects included,
 * as in m_ccLabelsMergedGrouper); needs GDF_SEG_CONNECTIONS */
int gdf_seg_merge_labels(gdf_segmenter* seg, uint32_t* merged, uint32_t capacity,
                         uint32_t* num_objects);
/* createCCObjects (fusion.cpp:2364-2550) without the OpenCV shapes (minAreaRect /
 * minEnclosingCircle of the contours, SURVEY §8(f) rank 4, out of scope): one record per merged
 * object, in merged-label order (background objects included, as m_ccObjects), with the
 * reference's float/int arithmetic; `components` receives every object's global label indices in
 * grouped order (UIntGrouper: ascending index), object i's at [first_component,
 * first_component + num_components).  lower / cell_size: the grid's GridMeta lower bound and
 * cell size (voxelCoordToWorldCoord, fusion.cpp:1720-1730).  Needs gdf_seg_merge_labels' inputs
 * (GDF_SEG_CONNECTIONS) and GDF_SEG_CONTOURS for the contour point counts. */
typedef struct gdf_cc_object {
    uint32_t label, num_components, num_layers, first_component;
    float centroid[2];                        /* mean of the components' centroids (cv::Point2f) */
    int32_t min_voxel[3], max_voxel[3], aabb_voxel[3];
    float center_voxel[3], center_world[3], min_world[3], max_world[3], aabb_world[3];
    uint32_t num_contour_points;              /* points of the components' external contours */
} gdf_cc_object;
int gdf_seg_create_objects(gdf_segmenter* seg, const float lower[3], const float cell_size[3],
                           gdf_cc_object* objects, uint32_t capacity, uint32_t* components,
                           uint32_t components_capacity, uint32_t* num_objects);
/* device pointers of the results (valid until the next gdf_seg_label_*) */
int gdf_seg_get_device_results(gdf_segmenter* seg, const uint16_t** labels, const int32_t** stats5,
                               const double** centroids2, const uint8_t** connections);

#ifdef __cplusplus
}
#endif

#endif /* GDF_SEGMENT_H_ */
