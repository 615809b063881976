// Compile check of include/gdf_fusion.hpp: the component's call sequence
// (src/gpu_depthmap_fusion_component.cpp:158-300 of the reference) written against the facade
// with minimal stand-ins for the OpenCV / glm / ROS types it accepts.  Built (and linked against
// libgdf.so) by tests/test_facade.py; never run there (no GPU on the test host).
#include <cstdint>
#include <vector>

#define GDF_GL_BARRIER_STUB  // no GL header in this build: the component's barrier lines compile as no-ops
#include "gdf_fusion.hpp"

namespace cv {
template <class T>
struct Mat_ {
    unsigned char* data;
    int rows, cols;
};
struct Matx44f {
    float val[16];
};
}  // namespace cv
namespace glm {
struct vec3 {
    float x, y, z;
};
}  // namespace glm
namespace sensor_msgs {
struct PointCloud2 {
    uint32_t height, width, point_step;
    std::vector<uint8_t> data;
};
}  // namespace sensor_msgs

int run_component_frame(gdf::GPUDepthmapFusion& f, const cv::Mat_<uint16_t>& depth,
                        const sensor_msgs::PointCloud2& cloud, const cv::Matx44f& T) {
    f.init("shader/");
    f.m_measureTime.beginFrame();
    f.addPointSequence(cloud, 5000u, 0u, T);
    f.clear();
    f.addDepthmap(depth, 0.001f, 384.f, 384.f, 320.f, 240.f, T, T);
    f.uploadPointSequences();
    f.filterNewPointSequences(0.05f, 1);
    f.insertNewPointSequencesInRollbuffer();
    f.rollPointSequenceRollbufferCPU(f.m_rollBufferLastTimeSec - 1u, f.m_rollBufferLastTimeNSec);
    f.selectPointSequenceTimespanCPU(4999u, 0u, 5000u, 0u);
    f.preparePointAndMaskBuffers();
    f.insertSelectedPointSequence(T, T);
    f.transformPointSequence();
    f.uploadDepthmaps();
    f.convertDepthmaps();
    f.filterFlyingPixels(4, 0.3f, false);
    f.cropPoints(glm::vec3{-10, -20, -1}, glm::vec3{30, 20, 1.5f});
    f.applyPointMask();
    f.computeVoxelCoords(glm::vec3{-10, -20, -1}, glm::vec3{30, 20, 1.5f},
                         glm::vec3{0.1f, 0.1f, 0.12f});
    f.voxelize(true);
    f.voxelOccupancyGrid(10);
    f.downloadVoxelOccupancyGrid();
    f.downloadPoints();
    const gdf::vec3 c = f.voxelCoordToWorldCoord(1, 2, 3);
    const gdf::vec3 v = f.worldCoordToVoxelCoord(c[0], c[1], c[2]);
    // the segmentation / tracking members the component reads (component.cpp:313-342, 541-632,
    // 731-962)
    f.objectSegmentation();
    f.objectTracking(0.1f);
    int acc = 0;
    for (size_t i = 0; i < f.m_ccCentroids.size(); ++i)
        for (int k = 1; k < f.m_ccCentroids[i].rows; ++k)
            acc += (int)f.voxelCoordToWorldCoord((float)f.m_ccCentroids[i](k, 0),
                                                 (float)f.m_ccCentroids[i](k, 1), (float)i)[0];
    if (!f.m_ccLayersConnections.empty() && f.m_ccLayersConnections[0].rows > 0)
        acc += f.m_ccLayersConnections[0].at<uint8_t>(0, 0);
    for (const auto& obj : f.m_ccObjects) {
        gdf::Point2f p[4];
        obj.topview.shapes.world.box.points(p);
        acc += (int)obj.label + (int)obj.min_coord.world.z + (int)obj.max_coord.world.z +
               (int)p[0].x + (int)obj.components.size();
        for (const auto& cmp : obj.components) acc += (int)cmp.contour3d.world.size();
    }
    for (const auto& t : f.m_ccObjectTracks)
        acc += (int)(t.score_filter.values[0] + gdf::norm(t.rrect_filter.rrect.center) +
                     t.lastObject.max_coord.world.z);
    return f.m_numPoints + (int)f.m_points_voxelized.size() + (int)f.m_occupancyGrid.size() +
           (int)c.x + (int)v.z + acc + (int)f.rollbufferState().num_seqs;
}

int main() { return 0; }
