"""Shared drivers for parity tests: replay GPUDepthmapFusionComponent::processDepthmaps
(src/gpu_depthmap_fusion_component.cpp:92-300) on either engine — the GPU engine
(ros_gpu_depthmap_fusion_amd.gdf.GPUDepthmapFusion) or the CPU oracle (oracle.OracleFusion) —
through their common method names, and compare the results.
"""
import numpy as np

from oracle import ros_time_minus


def stagewise_frame(eng, cams, params, T_world_move=None, T_crop_move=None):
    """The component's per-frame call sequence, one engine method per reference method."""
    eng.clear()
    for c in cams:
        eng.addDepthmap(*c)
    if not (len(cams) > 0 or eng.numCollectedPointSequencePoints() > 0):
        return False
    eng.uploadPointSequences()
    eng.filterNewPointSequences(params.ps_filter_threshold, params.ps_filter_size)
    eng.insertNewPointSequencesInRollbuffer()
    st = eng.rollbuffer_state()
    st = st.as_tuple() if hasattr(st, "as_tuple") else st
    last = (st[8], st[9])
    latest = earliest = (0, 0)
    if last != (0, 0):
        latest = last
        earliest = ros_time_minus(last[0], last[1], float(np.float32(params.ps_timespan)))
        assert earliest is not None
    eng.rollPointSequenceRollbufferCPU(*earliest)
    if T_world_move is not None:
        eng.selectPointSequenceTimespanCPU(earliest[0], earliest[1], latest[0], latest[1])
        eng.preparePointAndMaskBuffers()
        eng.insertSelectedPointSequence(T_world_move, T_crop_move)
        eng.transformPointSequence()
    else:
        eng.preparePointAndMaskBuffers()
    eng.uploadDepthmaps()
    eng.convertDepthmaps()
    eng.filterFlyingPixels(params.flying_filter_size, params.flying_threshold, params.flying_rot45)
    eng.cropPoints(params.crop_min, params.crop_max)
    eng.applyPointMask()
    if params.enable_voxel_filter:
        eng.computeVoxelCoords(params.voxel_min, params.voxel_max, params.voxel_size)
        eng.voxelize(params.voxel_average)
        eng.voxelOccupancyGrid(params.occupancy_lifetime)
    return True


def bits(a):
    a = np.ascontiguousarray(a, np.float32)
    return a.view(np.uint32)


def compare_results(gpu, orc, voxel=True, exact_points=True, tag=""):
    pg, po = gpu.downloadPoints(), orc.downloadPoints()
    assert len(pg) == len(po), f"{tag} point count gpu {len(pg)} oracle {len(po)}"
    if exact_points:
        bad = np.flatnonzero((bits(pg) != bits(po)).any(axis=1))
        assert len(bad) == 0, f"{tag} {len(bad)} points differ, first {bad[:5]}: {pg[bad[:3]]} vs {po[bad[:3]]}"
    else:
        np.testing.assert_allclose(pg[:, :3], po[:, :3], atol=1e-5, rtol=0)
    if not voxel:
        return
    cg, co = gpu.downloadVoxelCoords(), orc.downloadVoxelCoords()
    np.testing.assert_array_equal(cg, co, err_msg=f"{tag} voxel coords")
    vg, vo = gpu.downloadVoxelizedPoints(), orc.downloadVoxelizedPoints()
    assert len(vg) == len(vo), f"{tag} voxelized count gpu {len(vg)} oracle {len(vo)}"
    bad = np.flatnonzero((bits(vg[:, :3]) != bits(vo[:, :3])).any(axis=1))
    assert len(bad) == 0, f"{tag} {len(bad)} voxel means differ: {vg[bad[:3]]} vs {vo[bad[:3]]}"
    gg, go = gpu.downloadVoxelOccupancyGrid(), orc.downloadVoxelOccupancyGrid()
    assert gg.shape == go.shape
    nd = np.count_nonzero(gg != go)
    assert nd == 0, f"{tag} occupancy grid: {nd} cells differ"
    hg, ho = gpu.historic_grid(), orc.historic_grid()
    np.testing.assert_array_equal(hg, ho, err_msg=f"{tag} historic grid")
