// gdf_driver.cpp — the component's per-frame depth loop in C++, written against the C-ABI only
// (include/gdf_driver.h).  Mirrors GPUDepthmapFusionComponent::processDepthmaps
// (src/gpu_depthmap_fusion_component.cpp:92-300): clear (:128), addDepthmap per camera (:137),
// then the processing chain, here as the one gdf_process_frame call.
#include "gdf_driver.h"

namespace {

// `count` calls of gdf_process_frame, each over `batch` consecutive frames (gdf_next_frame_in_batch
// between them); frame i takes frames[i % ring] of every camera
// (step b takes parameter set p[(first + b) % nparams])
int run_stream(gdf_engine* e, const gdf_stream_camera* cams, uint32_t ncams,
               const gdf_frame_params* p, uint64_t first, uint64_t count, bool host,
               uint32_t batch, uint32_t nparams = 1) {
    if (!e || !p || (ncams && !cams) || batch == 0 || nparams == 0) return GDF_ERR_ARG;
    for (uint32_t k = 0; k < ncams; ++k)
        if (!cams[k].frames || cams[k].ring == 0) return GDF_ERR_ARG;
    for (uint64_t b = 0; b < count; ++b) {
        int rc = gdf_clear(e);
        if (rc) return rc;
        for (uint32_t j = 0; j < batch; ++j) {
            const uint64_t i = first + b * batch + j;
            if (j && (rc = gdf_next_frame_in_batch(e))) return rc;
            for (uint32_t k = 0; k < ncams; ++k) {
                const gdf_stream_camera& c = cams[k];
                rc = (host ? gdf_add_depthmap : gdf_add_depthmap_device)(
                    e, c.frames[i % c.ring], c.width, c.height, c.depth_scale, c.fx, c.fy, c.cx,
                    c.cy, c.T_world, c.T_crop);
                if (rc) return rc;
            }
        }
        rc = gdf_process_frame(e, p + (first + b) % nparams, nullptr);
        if (rc) return rc;
    }
    return GDF_OK;
}

}  // namespace

extern "C" int gdf_run_depth_stream(gdf_engine* e, const gdf_stream_camera* cams, uint32_t ncams,
                                    const gdf_frame_params* p, uint64_t first, uint64_t count) {
    return run_stream(e, cams, ncams, p, first, count, false, 1);
}

extern "C" int gdf_run_host_stream(gdf_engine* e, const gdf_stream_camera* cams, uint32_t ncams,
                                   const gdf_frame_params* p, uint64_t first, uint64_t count) {
    return run_stream(e, cams, ncams, p, first, count, true, 1);
}

extern "C" int gdf_run_depth_stream_batched(gdf_engine* e, const gdf_stream_camera* cams,
                                            uint32_t ncams, const gdf_frame_params* p,
                                            uint64_t first, uint64_t batches, uint32_t batch,
                                            int host) {
    return run_stream(e, cams, ncams, p, first, batches, host != 0, batch);
}

extern "C" int gdf_run_depth_stream_alternating(gdf_engine* e, const gdf_stream_camera* cams,
                                                uint32_t ncams, const gdf_frame_params* params,
                                                uint32_t nparams, uint64_t first,
                                                uint64_t batches, uint32_t batch) {
    return run_stream(e, cams, ncams, params, first, batches, false, batch, nparams);
}
