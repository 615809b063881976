// gdf_fusion.hpp — header-only C++ facade with the interface of the reference engine class
// `GPUDepthmapFusion` (include/gpu_depthmap_fusion/gpu_depthmap_fusion.h:159-526 of
// xaedes/ros_gpu_depthmap_fusion), forwarding to the C-ABI in gdf.h.
//
// The ROS component (src/gpu_depthmap_fusion_component.cpp) calls the engine through exactly
// these method names and reads the same public members; INTEGRATION.md shows the swap.
// No OpenCV / glm / ROS headers are needed here: the overloads taking cv::Mat_<uint16_t>,
// cv::Matx44f, glm::vec3 and sensor_msgs::PointCloud2 are templates that only touch the members
// those types have (`data`/`cols`/`rows`, `val[16]`, `x`/`y`/`z`, `data`/`width`/`height`/
// `point_step`).  Errors of the C-ABI are thrown as std::runtime_error.
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "gdf.h"
#include "gdf_objects.hpp"
#include "gdf_segment.h"

// The component calls glMemoryBarrier(GL_ALL_BARRIER_BITS) between the engine calls
// (component.cpp:164-309, 12 sites); ordering is the HIP stream's here, so they are no-ops
// (SURVEY.md §8(b) "GL leakage into caller").  The no-op lives in namespace gdf; a build without
// any GL header defines GDF_GL_BARRIER_STUB before including this header to also get the global
// glMemoryBarrier / GL_* names the component's source uses (a GL header, when present, provides
// them itself - no clash whatever the include order).
namespace gdf {
constexpr unsigned int kAllBarrierBits = 0xFFFFFFFFu;
inline void glMemoryBarrier(unsigned int) {}
}  // namespace gdf
#if defined(GDF_GL_BARRIER_STUB) && !defined(GL_ALL_BARRIER_BITS)
#define GL_ALL_BARRIER_BITS 0xFFFFFFFFu
#define GL_SHADER_STORAGE_BARRIER_BIT 0x00002000u
using gdf::glMemoryBarrier;
#endif

namespace gdf {

struct vec4 {  // memory layout of glm::vec4 / the reference's vec4 buffers
    float x, y, z, w;
};

// the component calls m_measureTime.beginFrame()/endFrame() around addDepthmap
// (component.cpp:105,155); per-kernel timing lives in gdf_set_profiling / gdf_get_kernel_times
struct MeasureTime {
    void beginFrame() {}
    void endFrame() {}
    void print(const char*) const {}
};

class GPUDepthmapFusion {
public:
    explicit GPUDepthmapFusion(int device = 0) : device_(device) {
        int major = -1, minor = -1;  // the library's ABI is the one this header describes
        gdf_version(&major, &minor);
        if (major != GDF_VERSION_MAJOR || minor != GDF_VERSION_MINOR)
            throw std::runtime_error("gdf: libgdf ABI " + std::to_string(major) + "." +
                                     std::to_string(minor) + " differs from gdf.h");
        check(gdf_create(device, &h_));
    }
    ~GPUDepthmapFusion() {
        if (seg_) gdf_seg_destroy(seg_);
        gdf_destroy(h_);
    }
    GPUDepthmapFusion(const GPUDepthmapFusion&) = delete;
    GPUDepthmapFusion& operator=(const GPUDepthmapFusion&) = delete;

    // gpu_depthmap_fusion.cpp:16-128 loads and compiles the GLSL programs here; the HIP kernels
    // are part of libgdf.so, so there is nothing to load.
    void init(const std::string& /*shaderPath*/) {}

    void clear() { check(gdf_clear(h_)); }  // :725-732

    // addDepthmap (:798-816); the depth image is borrowed until uploadDepthmaps, as in the
    // reference (the component keeps the cv_bridge image alive for the frame)
    template <class DepthMat, class Matx44>
    void addDepthmap(const DepthMat& depthmap, float depthScale, float fx, float fy, float cx,
                     float cy, const Matx44& transform_world, const Matx44& transform_crop) {
        addDepthmap(reinterpret_cast<const uint16_t*>(depthmap.data), (uint32_t)depthmap.cols,
                    (uint32_t)depthmap.rows, depthScale, fx, fy, cx, cy, transform_world.val,
                    transform_crop.val);
    }
    void addDepthmap(const uint16_t* depth, uint32_t width, uint32_t height, float depthScale,
                     float fx, float fy, float cx, float cy, const float T_world[16],
                     const float T_crop[16]) {
        check(gdf_add_depthmap(h_, depth, width, height, depthScale, fx, fy, cx, cy, T_world,
                               T_crop));
    }
    void addDepthmapDevice(const uint16_t* depth_device, uint32_t width, uint32_t height,
                           float depthScale, float fx, float fy, float cx, float cy,
                           const float T_world[16], const float T_crop[16]) {
        check(gdf_add_depthmap_device(h_, depth_device, width, height, depthScale, fx, fy, cx,
                                      cy, T_world, T_crop));
    }

    // addPointSequence (:747-796): x, y, z float32 at byte offsets 0/4/8 of each record
    template <class PointCloud2, class Matx44>
    void addPointSequence(const PointCloud2& pointcloud, uint32_t timestampSec,
                          uint32_t timestampNSec, const Matx44& transform_move) {
        check(gdf_add_point_sequence(h_, pointcloud.data.data(),
                                     (uint32_t)(pointcloud.width * pointcloud.height),
                                     (uint32_t)pointcloud.point_step, timestampSec,
                                     timestampNSec, transform_move.val));
    }
    // the same for records already in device memory (e.g. a GPU lidar driver's buffer):
    // borrowed until the next uploadPointSequences, gathered on the device
    void addPointSequenceDevice(const void* records_device, uint32_t num_points,
                                uint32_t point_step, uint32_t timestampSec, uint32_t timestampNSec,
                                const float transform_move[16]) {
        check(gdf_add_point_sequence_device(h_, records_device, num_points, point_step,
                                            timestampSec, timestampNSec, transform_move));
    }
    uint32_t numCollectedPointSequencePoints() {
        uint32_t n = 0;
        check(gdf_num_collected_point_sequence_points(h_, &n));
        return n;
    }

    // ---- point-sequence rollbuffer chain (:819-1581) ----
    void uploadPointSequences() { check(gdf_upload_point_sequences(h_)); }
    void filterNewPointSequences(float threshold, uint32_t filter_size) {
        check(gdf_filter_new_point_sequences(h_, threshold, filter_size));
    }
    void insertNewPointSequencesInRollbuffer() {
        check(gdf_insert_new_point_sequences(h_));
        syncRollbuffer();
    }
    void rollPointSequenceRollbufferCPU(uint32_t minSec, uint32_t minNSec) {
        check(gdf_roll_rollbuffer(h_, minSec, minNSec));
        syncRollbuffer();
    }
    // the reference's GPU variant (:1218-1356) is dead code with the same intended result
    void rollPointSequenceRollbuffer(uint32_t minSec, uint32_t minNSec) {
        rollPointSequenceRollbufferCPU(minSec, minNSec);
    }
    void selectPointSequenceTimespanCPU(uint32_t minSec, uint32_t minNSec, uint32_t maxSec,
                                        uint32_t maxNSec) {
        check(gdf_select_timespan(h_, minSec, minNSec, maxSec, maxNSec));
        syncRollbuffer();
    }
    void selectPointSequenceTimespan(uint32_t minSec, uint32_t minNSec, uint32_t maxSec,
                                     uint32_t maxNSec) {
        selectPointSequenceTimespanCPU(minSec, minNSec, maxSec, maxNSec);
    }
    void preparePointAndMaskBuffers() { check(gdf_prepare_point_and_mask_buffers(h_)); }
    template <class Matx44>
    void insertSelectedPointSequence(const Matx44& tf_world_move, const Matx44& tf_crop_move) {
        check(gdf_insert_selected_point_sequence(h_, tf_world_move.val, tf_crop_move.val));
    }
    void transformPointSequence() { check(gdf_transform_point_sequence(h_)); }

    // ---- depth chain (:1583-1839) ----
    void uploadDepthmaps() { check(gdf_upload_depthmaps(h_)); }
    void convertDepthmaps() { check(gdf_convert_depthmaps(h_)); }
    void filterFlyingPixels(uint32_t filter_size, float threshold, bool enable_rot45) {
        check(gdf_filter_flying_pixels(h_, filter_size, threshold, enable_rot45 ? 1 : 0));
    }
    template <class Vec3>
    void cropPoints(const Vec3& lower_bound, const Vec3& upper_bound) {
        const float lo[3] = {lower_bound.x, lower_bound.y, lower_bound.z};
        const float hi[3] = {upper_bound.x, upper_bound.y, upper_bound.z};
        check(gdf_crop_points(h_, lo, hi));
    }
    void applyPointMask() {
        uint32_t n = 0;
        check(gdf_apply_point_mask(h_, &n));
        m_numPoints = (int)n;
    }
    template <class Vec3>
    void computeVoxelCoords(const Vec3& lower_bound, const Vec3& upper_bound,
                            const Vec3& cell_size) {
        const float lo[3] = {lower_bound.x, lower_bound.y, lower_bound.z};
        const float hi[3] = {upper_bound.x, upper_bound.y, upper_bound.z};
        const float cs[3] = {cell_size.x, cell_size.y, cell_size.z};
        check(gdf_compute_voxel_coords(h_, lo, hi, cs));
        for (int i = 0; i < 3; ++i) {  // GridMeta (grid_meta.h:140-158): sorted bounds
            lo_[i] = lo[i] < hi[i] ? lo[i] : hi[i];
            cs_[i] = cs[i];
        }
    }
    void downloadVoxelCoords() {
        uint32_t n = count();
        m_voxelCoords.resize(n);
        check(gdf_download_voxel_coords(h_, m_voxelCoords.data(), n, &n));
        m_voxelCoords.resize(n);
    }
    // voxelize (:1743-1756): on the GPU; m_points_voxelized is filled like the reference's
    void voxelize(bool average_voxels) {
        check(gdf_voxelize(h_, average_voxels ? 1 : 0));
        uint32_t n = count();
        m_points_voxelized.resize(n);
        check(gdf_download_voxelized_points(h_, reinterpret_cast<float*>(m_points_voxelized.data()),
                                            n, &n));
        m_points_voxelized.resize(n);
    }
    void voxelOccupancyGrid(uint32_t lifetime) { check(gdf_voxel_occupancy_grid(h_, lifetime)); }
    void downloadVoxelOccupancyGrid() {
        uint32_t gs[3];
        uint64_t cells = 0;
        check(gdf_get_grid_size(h_, gs, &cells));
        m_occupancyGrid.resize(cells);
        check(gdf_download_occupancy_grid(h_, m_occupancyGrid.data(), cells));
        for (int i = 0; i < 3; ++i) gridSize_[i] = gs[i];
    }
    // m_occupancyLayers[z] of the reference is a (gy x gx) uint8 view of layer z
    const uint8_t* occupancyLayer(uint32_t z) const {
        return m_occupancyGrid.data() + (size_t)z * gridSize_[0] * gridSize_[1];
    }
    void downloadPoints() {
        uint32_t n = count();
        m_points.resize(n);
        check(gdf_download_points(h_, reinterpret_cast<float*>(m_points.data()), n, &n));
        m_points.resize(n);
    }
    // the mapped variant (fusion.cpp:2952-2966): the points in host memory until unmap
    void* downloadPoints(int& count_out) {
        downloadPoints();
        count_out = (int)m_points.size();
        return m_points.data();
    }
    void unmap() {}
    // voxelCoordToWorldCoord / worldCoordToVoxelCoord (gpu_depthmap_fusion.cpp:1720-1741): the
    // lower corner of voxel (x, y, z), and back (glm::vec3 arithmetic in f32)
    vec3 voxelCoordToWorldCoord(float x, float y, float z) const {
        return vec3(x * cs_[0] + lo_[0], y * cs_[1] + lo_[1], z * cs_[2] + lo_[2]);
    }
    vec3 worldCoordToVoxelCoord(float x, float y, float z) const {
        return vec3((x - lo_[0]) / cs_[0], (y - lo_[1]) / cs_[1], (z - lo_[2]) / cs_[2]);
    }

    // the component's whole per-frame sequence as one call (gdf_process_frame)
    gdf_frame_result processFrame(const gdf_frame_params& params) {
        gdf_frame_result r{};
        check(gdf_process_frame(h_, &params, &r));
        if (params.synchronous) m_numPoints = (int)r.num_points;
        syncRollbuffer();
        return r;
    }

    // ---- object segmentation front end (fusion.cpp:1872-2361) on the GPU ----------------------
    // labelVoxels (:1872-2011): labels, stats, centroids, contours and labelsToContours of every
    // z-layer of the current occupancy grid (the grid stays on the device; downloadVoxel-
    // OccupancyGrid is not needed for it) + the layer connection matrices (:2075-2214)
    void labelVoxels() {
        if (!seg_) check(gdf_seg_create(device_, &seg_));
        check(gdf_seg_label_engine_grid(seg_, h_, GDF_SEG_ALL));
        gdf_seg_counts c{};
        check(gdf_seg_get_counts(seg_, &c));
        const uint32_t L = c.layers, T = c.total_labels;
        m_ccLabeledLayersData.resize((size_t)c.width * c.height * L);
        check(gdf_seg_download_labels(seg_, m_ccLabeledLayersData.data(), m_ccLabeledLayersData.size()));
        m_ccNumLabelsPerLayer.resize(L);
        check(gdf_seg_download_num_labels(seg_, m_ccNumLabelsPerLayer.data(), L));
        m_ccStatsData.resize((size_t)T * 5);
        m_ccCentroidsData.resize((size_t)T * 2);
        check(gdf_seg_download_stats(seg_, m_ccStatsData.data(), m_ccCentroidsData.data(), T));
        m_ccStatsDataStarts.resize(L);
        m_ccCentroidsDataStarts.resize(L);
        m_ccLabelsLayerStarts.resize(L);
        for (uint32_t i = 0, t = 0; i < L; t += m_ccNumLabelsPerLayer[i++]) {
            m_ccLabelsLayerStarts[i] = t;
            m_ccStatsDataStarts[i] = 5 * (int)t;
            m_ccCentroidsDataStarts[i] = 2 * (int)t;
        }
        std::vector<int32_t> l2c(T), pts(2 * c.total_contour_points);
        std::vector<uint32_t> per(L), sizes(c.total_contours);
        check(gdf_seg_download_contours(seg_, l2c.data(), per.data(), sizes.data(), pts.data(),
                                        c.total_contour_points));
        m_labelsToContoursPerLayer.assign(L, {});
        m_contoursPerLayer.assign(L, {});
        size_t q = 0, k = 0;
        for (uint32_t i = 0; i < L; ++i) {
            const uint32_t t0 = m_ccLabelsLayerStarts[i];
            m_labelsToContoursPerLayer[i].assign(l2c.begin() + t0,
                                                 l2c.begin() + t0 + m_ccNumLabelsPerLayer[i]);
            m_contoursPerLayer[i].resize(per[i]);
            for (uint32_t j = 0; j < per[i]; ++j, ++k)
                for (uint32_t n = 0; n < sizes[k]; ++n, ++q)
                    m_contoursPerLayer[i][j].push_back(Point{pts[2 * q], pts[2 * q + 1]});
        }
        m_ccLayersConnectionsData.resize(c.connection_bytes);
        m_ccLayersConnectionsDataStarts.resize(L ? L - 1 : 0);
        check(gdf_seg_download_connections(seg_, m_ccLayersConnectionsData.data(),
                                           m_ccLayersConnectionsData.size(),
                                           m_ccLayersConnectionsDataStarts.data(),
                                           (uint32_t)m_ccLayersConnectionsDataStarts.size()));
        // the cv::Mat_ views of the reference (fusion.cpp:1915, 2004-2010, 2108-2111)
        m_ccLabeledLayers.resize(L);
        m_ccStats.resize(L);
        m_ccCentroids.resize(L);
        for (uint32_t i = 0; i < L; ++i) {
            m_ccLabeledLayers[i] = Mat_<uint16_t>((int)c.height, (int)c.width,
                                                  m_ccLabeledLayersData.data() + (size_t)i * c.width * c.height);
            const int nl = (int)m_ccNumLabelsPerLayer[i];
            m_ccStats[i] = Mat_<int32_t>(nl, 5, m_ccStatsData.data() + m_ccStatsDataStarts[i]);
            m_ccCentroids[i] = Mat_<double>(nl, 2, m_ccCentroidsData.data() + m_ccCentroidsDataStarts[i]);
        }
        m_ccLayersConnections.resize(L ? L - 1 : 0);
        for (uint32_t i = 0; i + 1 < L; ++i)
            m_ccLayersConnections[i] = Mat_<uint8_t>(
                (int)m_ccNumLabelsPerLayer[i], (int)m_ccNumLabelsPerLayer[i + 1],
                m_ccLayersConnectionsData.data() + m_ccLayersConnectionsDataStarts[i]);
    }
    // the label upload, connection-matrix preparation and the layers_connections dispatch are
    // part of labelVoxels here (the labels never leave the device)
    void uploadVoxelLabels() {}
    void prepareLayersConnections() {}
    void computeLayersConnections() {}
    void downloadLayersConnections() {}
    // checkAllPointSequenceBuffers (fusion.cpp:859-926; its call sites :856, :975, :1086, :1216 are
    // commented out): the reference downloads every rollbuffer buffer into function statics for a
    // debugger.  Here the rollbuffer in the reference's logical B layout (points, mask, sequence
    // index per point; headers sec / nsec / start / numPoints) lands in the m_check* members.
    void checkAllPointSequenceBuffers() {
        syncRollbuffer();
        const uint32_t R = m_rollBufferNumPoints, S = m_rollBufferNumSeqs;
        m_checkPoints.resize((size_t)R * 4);
        m_checkPointsMask.resize(R);
        m_checkSeqIdcs.resize(R);
        m_checkSequences.resize((size_t)S * 4);
        check(gdf_debug_rollbuffer(h_, m_checkPoints.data(), m_checkPointsMask.data(), m_checkSeqIdcs.data(),
                                   R, m_checkSequences.data(), S));
    }
    std::vector<float> m_checkPoints;
    std::vector<uint32_t> m_checkPointsMask, m_checkSeqIdcs, m_checkSequences;

    // computeLayersConnectionsCPU (fusion.cpp:2153-2197, uncalled in the reference): the same
    // matrices from the downloaded labels on the host - zero each numLabels[i] x numLabels[i + 1]
    // matrix, then connection(labelA, labelB) = 1 for every cell (background label 0 included).
    // Rewrites m_ccLayersConnections' storage with what labelVoxels' device pass already produced.
    void computeLayersConnectionsCPU() {
        for (size_t i = 0; i < m_ccLayersConnections.size(); ++i) {
            Mat_<uint8_t>& mat = m_ccLayersConnections[i];
            const Mat_<uint16_t>& A = m_ccLabeledLayers[i];
            const Mat_<uint16_t>& B = m_ccLabeledLayers[i + 1];
            for (int a = 0; a < (int)m_ccNumLabelsPerLayer[i]; ++a)
                for (int b = 0; b < (int)m_ccNumLabelsPerLayer[i + 1]; ++b) mat.template at<uint8_t>(a, b) = 0;
            for (int y = 0; y < A.rows; ++y)
                for (int x = 0; x < A.cols; ++x)
                    mat.template at<uint8_t>(A.template at<uint16_t>(y, x), B.template at<uint16_t>(y, x)) = 1;
        }
    }
    // mergeLabelsAcrossLayers (:2243-2361): m_ccLabelsMerged / Layer / Local per global label
    void mergeLabelsAcrossLayers() {
        const size_t T = m_ccStatsData.size() / 5;
        m_ccLabelsMerged.resize(T);
        uint32_t nobj = 0;
        check(gdf_seg_merge_labels(seg_, m_ccLabelsMerged.data(), (uint32_t)T, &nobj));
        m_ccLabelsLayer.resize(T);
        m_ccLabelsLocal.resize(T);
        for (uint32_t i = 0, t = 0; i < m_ccNumLabelsPerLayer.size(); ++i)
            for (uint32_t k = 0; k < m_ccNumLabelsPerLayer[i]; ++k, ++t) {
                m_ccLabelsLayer[t] = i;
                m_ccLabelsLocal[t] = k;
            }
        m_ccNumObjects = nobj;
    }
    // createCCObjects (:2364-2550): the objects' aggregate fields and their components (global
    // label indices, grouped) from the GPU (gdf_seg_create_objects), then on the host each
    // component's contour in voxel and world coordinates, the per-layer and top-view point sets
    // and the minimal shapes (gdf_objects.hpp) of components, layers and top view
    void createCCObjects() {
        uint32_t n = 0;
        check(gdf_seg_create_objects(seg_, lo_, cs_, nullptr, 0, nullptr, 0, &n));
        m_ccObjectRecords.resize(n);
        m_ccObjectComponents.resize(m_ccLabelsMerged.size());
        check(gdf_seg_create_objects(seg_, lo_, cs_, m_ccObjectRecords.data(), n,
                                     m_ccObjectComponents.data(),
                                     (uint32_t)m_ccObjectComponents.size(), &n));
        m_ccObjects.assign(n, CCObject());
        for (uint32_t i = 0; i < n; ++i) build_object(m_ccObjectRecords[i], m_ccObjects[i]);
    }
    // objectSegmentation (:2552-2575)
    void objectSegmentation() {
        labelVoxels();
        mergeLabelsAcrossLayers();
        createCCObjects();
    }
    // objectTracking (:2727-2944): associates m_ccObjects with m_ccObjectTracks
    void objectTracking(float min_area) { object_tracking(m_ccObjects, m_ccObjectTracks, min_area); }

    gdf_rollbuffer_state rollbufferState() {
        gdf_rollbuffer_state s{};
        check(gdf_get_rollbuffer_state(h_, &s));
        return s;
    }
    gdf_engine* handle() const { return h_; }

    // public members the component reads (gpu_depthmap_fusion.h:318-362)
    int m_voxelGroupSize = 8;
    std::vector<uint8_t> m_occupancyGrid;
    std::vector<vec4> m_points;
    std::vector<vec4> m_points_voxelized;
    std::vector<uint32_t> m_voxelCoords;
    int m_numPoints = 0;
    MeasureTime m_measureTime;
    // m_rollBuffer* (gpu_depthmap_fusion.h:345-354), refreshed after every rollbuffer call
    uint32_t m_rollBufferNumPoints = 0, m_rollBufferNumSeqs = 0;
    uint32_t m_rollBufferSelectionPointStart = 0, m_rollBufferSelectionPointCount = 0;
    uint32_t m_rollBufferSelectionSequenceStart = 0, m_rollBufferSelectionSequenceCount = 0;
    uint32_t m_rollBufferEarliestTimeSec = 0, m_rollBufferEarliestTimeNSec = 0;
    uint32_t m_rollBufferLastTimeSec = 0, m_rollBufferLastTimeNSec = 0;
    // segmentation members (gpu_depthmap_fusion.h:328-341, 511-518), flat like their *Data
    // storage; cv::Mat_ views of them are (rows, cols, pointer) over these vectors
    std::vector<uint16_t> m_ccLabeledLayersData;
    std::vector<uint32_t> m_ccNumLabelsPerLayer;
    std::vector<int32_t> m_ccStatsData;
    std::vector<double> m_ccCentroidsData;
    std::vector<int> m_ccStatsDataStarts, m_ccCentroidsDataStarts;
    std::vector<std::vector<int>> m_labelsToContoursPerLayer;
    std::vector<std::vector<std::vector<Point>>> m_contoursPerLayer;
    std::vector<uint8_t> m_ccLayersConnectionsData;
    std::vector<uint64_t> m_ccLayersConnectionsDataStarts;
    std::vector<uint32_t> m_ccLabelsMerged, m_ccLabelsLayer, m_ccLabelsLocal, m_ccLabelsLayerStarts;
    uint32_t m_ccNumObjects = 0;
    // cv::Mat_ views over the *Data vectors (gpu_depthmap_fusion.h:328-333), valid until the next
    // labelVoxels
    std::vector<Mat_<uint16_t>> m_ccLabeledLayers;
    std::vector<Mat_<int32_t>> m_ccStats;
    std::vector<Mat_<double>> m_ccCentroids;
    std::vector<Mat_<uint8_t>> m_ccLayersConnections;
    std::vector<CCObject> m_ccObjects;            // (gpu_depthmap_fusion.h:342)
    std::vector<CCObjectTrack> m_ccObjectTracks;  // (gpu_depthmap_fusion.h:343)
    std::vector<gdf_cc_object> m_ccObjectRecords;  // the GPU's aggregates behind m_ccObjects
    std::vector<uint32_t> m_ccObjectComponents;

private:
    // one CCObject from the GPU record + the contours (fusion.cpp:2371-2537)
    void build_object(const gdf_cc_object& R, CCObject& obj) const {
        obj.centroid = Point2f(R.centroid[0], R.centroid[1]);
        obj.label = R.label;
        obj.num_components = R.num_components;
        obj.num_layers = R.num_layers;
        obj.min_coord.voxel = ivec3(R.min_voxel[0], R.min_voxel[1], R.min_voxel[2]);
        obj.max_coord.voxel = ivec3(R.max_voxel[0], R.max_voxel[1], R.max_voxel[2]);
        obj.aabb_size.voxel = ivec3(R.aabb_voxel[0], R.aabb_voxel[1], R.aabb_voxel[2]);
        obj.center_coord.voxel = vec3(R.center_voxel[0], R.center_voxel[1], R.center_voxel[2]);
        obj.center_coord.world = vec3(R.center_world[0], R.center_world[1], R.center_world[2]);
        obj.min_coord.world = vec3(R.min_world[0], R.min_world[1], R.min_world[2]);
        obj.max_coord.world = vec3(R.max_world[0], R.max_world[1], R.max_world[2]);
        obj.aabb_size.world = vec3(R.aabb_world[0], R.aabb_world[1], R.aabb_world[2]);
        obj.components.assign(R.num_components, CCObject::Component());
        obj.layers.assign(R.num_layers, CCObject::Layer());
        for (uint32_t k = 0; k < R.num_components; ++k) {
            const uint32_t idx = m_ccObjectComponents[R.first_component + k];
            const uint32_t layer = m_ccLabelsLayer[idx], local = m_ccLabelsLocal[idx];
            const int ci = m_labelsToContoursPerLayer[layer][local];
            if (ci < 0) continue;
            const std::vector<Point>& contour = m_contoursPerLayer[layer][ci];
            CCObject::Component& cmp = obj.components[k];
            CCObject::Layer& ly = obj.layers[layer - (uint32_t)obj.min_coord.voxel.z];
            for (const Point& p : contour) {
                const vec3 w = voxelCoordToWorldCoord((float)p.x, (float)p.y, (float)layer);
                cmp.contour3d.voxel.push_back(vec3((float)p.x, (float)p.y, (float)layer));
                cmp.contour3d.world.push_back(w);
                cmp.contour2d.voxel.push_back(Point2f((float)p.x, (float)p.y));
                cmp.contour2d.world.push_back(Point2f(w.x, w.y));
                ly.points2d.voxel.push_back(cmp.contour2d.voxel.back());
                ly.points2d.world.push_back(cmp.contour2d.world.back());
                obj.topview.points2d.world.push_back(cmp.contour2d.world.back());
                obj.topview.points2d.voxel.push_back(cmp.contour2d.voxel.back());
            }
            cmp.shapes.voxel = CCObject::MinShapes(cmp.contour2d.voxel);
            cmp.shapes.world = CCObject::MinShapes(cmp.contour2d.world);
        }
        for (CCObject::Layer& ly : obj.layers) {
            ly.shapes.voxel = CCObject::MinShapes(ly.points2d.voxel);
            ly.shapes.world = CCObject::MinShapes(ly.points2d.world);
        }
        obj.topview.shapes.voxel = CCObject::MinShapes(obj.topview.points2d.voxel);
        obj.topview.shapes.world = CCObject::MinShapes(obj.topview.points2d.world);
    }
    void syncRollbuffer() {
        const gdf_rollbuffer_state r = rollbufferState();
        m_rollBufferNumPoints = r.num_points;
        m_rollBufferNumSeqs = r.num_seqs;
        m_rollBufferSelectionPointStart = r.selection_point_start;
        m_rollBufferSelectionPointCount = r.selection_point_count;
        m_rollBufferSelectionSequenceStart = r.selection_sequence_start;
        m_rollBufferSelectionSequenceCount = r.selection_sequence_count;
        m_rollBufferEarliestTimeSec = r.earliest_time_sec;
        m_rollBufferEarliestTimeNSec = r.earliest_time_nsec;
        m_rollBufferLastTimeSec = r.last_time_sec;
        m_rollBufferLastTimeNSec = r.last_time_nsec;
    }
    static void check(int rc) {
        if (rc != GDF_OK) throw std::runtime_error(std::string("gdf: ") + gdf_last_error());
    }
    uint32_t count() {
        uint32_t n = 0;
        check(gdf_get_point_count(h_, &n));
        return n;
    }
    gdf_engine* h_ = nullptr;
    gdf_segmenter* seg_ = nullptr;
    int device_ = 0;
    float lo_[3] = {0, 0, 0}, cs_[3] = {1, 1, 1};
    uint32_t gridSize_[3] = {0, 0, 0};
};

}  // namespace gdf
