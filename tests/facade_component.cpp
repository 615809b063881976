// The reference component's per-frame sequence (GPUDepthmapFusionComponent::processDepthmaps,
// src/gpu_depthmap_fusion_component.cpp:92-300, and the point-sequence callback :158-165) run on
// the GPU through the C++ facade include/gdf_fusion.hpp, with minimal stand-ins for the OpenCV /
// glm / ROS types the facade accepts.  Reads the fixture of tests/golden/facade (manifest.txt +
// raw .bin inputs), writes what the component reads from the engine after each frame
// (m_points, m_voxelCoords, m_points_voxelized, m_occupancyGrid) into <out_dir>/*.bin;
// tests/test_facade_gpu.py compares them with the oracle's outputs bit for bit.
//
//   facade_component <fixture_dir> <out_dir>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
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
    vec3(float a, float b, float c) : x(a), y(b), z(c) {}
};
}  // namespace glm
namespace sensor_msgs {
struct PointCloud2 {
    uint32_t height = 1, width = 0, point_step = 12;
    std::vector<uint8_t> data;
};
}  // namespace sensor_msgs

// ros::Time - ros::Duration(double) (roscpp_core: DurationBase::fromSec, normalizeSecNSec*)
static void ros_time_minus(uint32_t sec, uint32_t nsec, double seconds, uint32_t* os,
                           uint32_t* ons) {
    int64_t dsec = (int64_t)std::floor(seconds);
    int64_t dnsec = (int64_t)std::llround((seconds - (double)dsec) * 1e9);
    dsec += dnsec / 1000000000LL;
    dnsec %= 1000000000LL;
    int64_t s = (int64_t)sec - dsec, n = (int64_t)nsec - dnsec;
    while (n < 0) { n += 1000000000LL; --s; }
    *os = (uint32_t)s;
    *ons = (uint32_t)n;
}

template <class T>
static std::vector<T> read_bin(const std::string& path) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) throw std::runtime_error("cannot read " + path);
    const size_t n = (size_t)f.tellg() / sizeof(T);
    std::vector<T> v(n);
    f.seekg(0);
    f.read(reinterpret_cast<char*>(v.data()), (std::streamsize)(n * sizeof(T)));
    return v;
}

template <class T>
static void write_bin(const std::string& path, const T* p, size_t n) {
    std::ofstream f(path, std::ios::binary);
    f.write(reinterpret_cast<const char*>(p), (std::streamsize)(n * sizeof(T)));
}

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s <fixture_dir> <out_dir>\n", argv[0]);
        return 2;
    }
    const std::string dir = argv[1], out = argv[2];
    std::map<std::string, std::vector<double>> m;
    {
        std::ifstream f(dir + "/manifest.txt");
        std::string line;
        while (std::getline(f, line)) {
            std::istringstream ss(line);
            std::string key;
            ss >> key;
            double x;
            while (ss >> x) m[key].push_back(x);
        }
    }
    auto mat = [&](const std::string& k) {
        cv::Matx44f M;
        for (int i = 0; i < 16; ++i) M.val[i] = (float)m.at(k)[i];
        return M;
    };
    const int frames = (int)m.at("frames")[0];
    const int W = (int)m.at("depth_size")[0], H = (int)m.at("depth_size")[1];
    const auto& pr = m.at("params");
    const float psThr = (float)pr[0], psTimespan = (float)pr[2], flyThr = (float)pr[4];
    const uint32_t psSize = (uint32_t)pr[1], flySize = (uint32_t)pr[3];
    const bool rot45 = pr[5] != 0;
    const auto& cr = m.at("crop");
    const auto& vx = m.at("voxel");
    const bool average = m.at("voxel_average")[0] != 0;
    const uint32_t lifetime = (uint32_t)m.at("lifetime")[0];
    const auto& in = m.at("intrinsics");
    const cv::Matx44f Tw = mat("T_world"), Tc = mat("T_crop");
    const cv::Matx44f Twm = mat("T_world_move"), Tcm = mat("T_crop_move");

    gdf::GPUDepthmapFusion fusion(0);
    gdf::GPUDepthmapFusion* m_fusion = &fusion;
    m_fusion->init("shader/");
    for (int f = 0; f < frames; ++f) {
        // point-sequence callback (component.cpp:158-165): addPointSequence under its lock
        const auto& st = m.at("stamp" + std::to_string(f));
        sensor_msgs::PointCloud2 cloud;
        const std::vector<float> xyz = read_bin<float>(dir + "/cloud" + std::to_string(f) + ".bin");
        cloud.width = (uint32_t)(xyz.size() / 3);
        cloud.data.resize(xyz.size() * 4);
        std::memcpy(cloud.data.data(), xyz.data(), cloud.data.size());
        cv::Matx44f Tm;
        for (int i = 0; i < 16; ++i) Tm.val[i] = (float)st[2 + i];
        m_fusion->addPointSequence(cloud, (uint32_t)st[0], (uint32_t)st[1], Tm);

        // processDepthmaps (component.cpp:92-300)
        std::vector<uint16_t> depth = read_bin<uint16_t>(dir + "/depth" + std::to_string(f) + ".bin");
        cv::Mat_<uint16_t> img{reinterpret_cast<unsigned char*>(depth.data()), H, W};
        m_fusion->clear();
        m_fusion->m_measureTime.beginFrame();
        int numAdded = 0;
        m_fusion->addDepthmap(img, (float)in[0], (float)in[1], (float)in[2], (float)in[3],
                              (float)in[4], Tw, Tc);
        ++numAdded;
        m_fusion->m_measureTime.endFrame();
        if ((numAdded > 0) || (m_fusion->numCollectedPointSequencePoints() > 0)) {
            m_fusion->uploadPointSequences();
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->filterNewPointSequences(psThr, psSize);
            m_fusion->insertNewPointSequencesInRollbuffer();
            uint32_t ls = 0, ln = 0, es = 0, en = 0;
            if (m_fusion->m_rollBufferLastTimeSec != 0 || m_fusion->m_rollBufferLastTimeNSec != 0) {
                ls = m_fusion->m_rollBufferLastTimeSec;
                ln = m_fusion->m_rollBufferLastTimeNSec;
                ros_time_minus(ls, ln, (double)psTimespan, &es, &en);
            }
            m_fusion->rollPointSequenceRollbufferCPU(es, en);
            m_fusion->selectPointSequenceTimespanCPU(es, en, ls, ln);
            m_fusion->preparePointAndMaskBuffers();
            m_fusion->insertSelectedPointSequence(Twm, Tcm);
            m_fusion->transformPointSequence();
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->uploadDepthmaps();
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->convertDepthmaps();
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->filterFlyingPixels(flySize, flyThr, rot45);
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->cropPoints(glm::vec3((float)cr[0], (float)cr[1], (float)cr[2]),
                                 glm::vec3((float)cr[3], (float)cr[4], (float)cr[5]));
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->applyPointMask();
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->computeVoxelCoords(glm::vec3((float)vx[0], (float)vx[1], (float)vx[2]),
                                         glm::vec3((float)vx[3], (float)vx[4], (float)vx[5]),
                                         glm::vec3((float)vx[6], (float)vx[7], (float)vx[8]));
            m_fusion->downloadVoxelCoords();
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->downloadPoints();
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->voxelize(average);
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->voxelOccupancyGrid(lifetime);
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->downloadVoxelOccupancyGrid();
            glMemoryBarrier(GL_ALL_BARRIER_BITS);
            m_fusion->objectSegmentation();  // component.cpp:313-323
            m_fusion->objectTracking(0.1f);
            // the two uncalled reference methods: the CPU layer connections equal the device's,
            // and the rollbuffer check downloads the state the members report
            const std::vector<uint8_t> dev_conn = m_fusion->m_ccLayersConnectionsData;
            m_fusion->computeLayersConnectionsCPU();
            if (m_fusion->m_ccLayersConnectionsData != dev_conn) {
                std::fprintf(stderr, "frame %d: computeLayersConnectionsCPU differs from the device\n", f);
                return 3;
            }
            m_fusion->checkAllPointSequenceBuffers();
            uint32_t masked = 0;
            for (uint32_t m : m_fusion->m_checkPointsMask) masked += m;
            if (m_fusion->m_checkPoints.size() != 4 * (size_t)m_fusion->m_rollBufferNumPoints ||
                m_fusion->m_checkSequences.size() != 4 * (size_t)m_fusion->m_rollBufferNumSeqs ||
                (m_fusion->m_rollBufferNumPoints && !masked)) {
                std::fprintf(stderr, "frame %d: checkAllPointSequenceBuffers\n", f);
                return 4;
            }
        }
        const std::string s = std::to_string(f);
        write_bin(out + "/points" + s + ".bin", reinterpret_cast<const float*>(m_fusion->m_points.data()),
                  m_fusion->m_points.size() * 4);
        write_bin(out + "/coords" + s + ".bin", m_fusion->m_voxelCoords.data(),
                  m_fusion->m_voxelCoords.size());
        std::vector<float> vox;
        for (const gdf::vec4& v : m_fusion->m_points_voxelized) {
            vox.push_back(v.x);
            vox.push_back(v.y);
            vox.push_back(v.z);
        }
        write_bin(out + "/voxelized" + s + ".bin", vox.data(), vox.size());
        write_bin(out + "/grid" + s + ".bin", m_fusion->m_occupancyGrid.data(),
                  m_fusion->m_occupancyGrid.size());
        uint32_t gs[3];
        uint64_t cells = 0;
        if (gdf_get_grid_size(m_fusion->handle(), gs, &cells) == GDF_OK) {
            FILE* fh = std::fopen((out + "/gridsize" + s + ".txt").c_str(), "w");
            std::fprintf(fh, "%u %u %u\n", gs[0], gs[1], gs[2]);
            std::fclose(fh);
        }
        write_bin(out + "/labels" + s + ".bin", m_fusion->m_ccLabeledLayersData.data(),
                  m_fusion->m_ccLabeledLayersData.size());
        write_bin(out + "/stats" + s + ".bin", m_fusion->m_ccStatsData.data(),
                  m_fusion->m_ccStatsData.size());
        write_bin(out + "/merged" + s + ".bin", m_fusion->m_ccLabelsMerged.data(),
                  m_fusion->m_ccLabelsMerged.size());
        std::vector<int32_t> objmin;
        for (const gdf::CCObject& o : m_fusion->m_ccObjects)
            for (int i = 0; i < 3; ++i) objmin.push_back(o.min_coord.voxel[i]);
        write_bin(out + "/objmin" + s + ".bin", objmin.data(), objmin.size());
        std::vector<int32_t> l2c;
        for (const auto& v : m_fusion->m_labelsToContoursPerLayer) l2c.insert(l2c.end(), v.begin(), v.end());
        write_bin(out + "/l2c" + s + ".bin", l2c.data(), l2c.size());
        std::vector<int32_t> cpts;
        for (const auto& layer : m_fusion->m_contoursPerLayer)
            for (const auto& c : layer)
                for (const auto& p : c) {
                    cpts.push_back(p.x);
                    cpts.push_back(p.y);
                }
        write_bin(out + "/contours" + s + ".bin", cpts.data(), cpts.size());
        std::printf("frame %d: %d points, %zu voxels, rollbuffer %u points\n", f,
                    m_fusion->m_numPoints, m_fusion->m_points_voxelized.size(),
                    m_fusion->m_rollBufferNumPoints);
    }
    return 0;
}
