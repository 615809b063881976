// gdf_driver.cpp — the component's per-frame depth loop in C++, written against the C-ABI only
// (include/gdf_driver.h).  Mirrors GPUDepthmapFusionComponent::processDepthmaps
// (src/gpu_depthmap_fusion_component.cpp:92-300): clear (:128), addDepthmap per camera (:137),
// then the processing chain, here as the one gdf_process_frame call.
#include "gdf_driver.h"

namespace {

int run_stream(gdf_engine* e, const gdf_stream_camera* cams, uint32_t ncams,
               const gdf_frame_params* p, uint64_t first, uint64_t count, bool host) {
    if (!e || !p || (ncams && !cams)) return GDF_ERR_ARG;
    for (uint32_t k = 0; k < ncams; ++k)
        if (!cams[k].frames || cams[k].ring == 0) return GDF_ERR_ARG;
    for (uint64_t i = first; i < first + count; ++i) {
        int rc = gdf_clear(e);
        if (rc) return rc;
        for (uint32_t k = 0; k < ncams; ++k) {
            const gdf_stream_camera& c = cams[k];
            rc = (host ? gdf_add_depthmap : gdf_add_depthmap_device)(
                e, c.frames[i % c.ring], c.width, c.height, c.depth_scale, c.fx, c.fy, c.cx, c.cy,
                c.T_world, c.T_crop);
            if (rc) return rc;
        }
        rc = gdf_process_frame(e, p, nullptr);
        if (rc) return rc;
    }
    return GDF_OK;
}

}  // namespace

extern "C" int gdf_run_depth_stream(gdf_engine* e, const gdf_stream_camera* cams, uint32_t ncams,
                                    const gdf_frame_params* p, uint64_t first, uint64_t count) {
    return run_stream(e, cams, ncams, p, first, count, false);
}

extern "C" int gdf_run_host_stream(gdf_engine* e, const gdf_stream_camera* cams, uint32_t ncams,
                                   const gdf_frame_params* p, uint64_t first, uint64_t count) {
    return run_stream(e, cams, ncams, p, first, count, true);
}
