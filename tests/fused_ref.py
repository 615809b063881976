"""Host-side pieces of the multi-GPU fused-cloud protocol used by the tests: the oracle as a
rank's engine (camera k with camera k-1 in front of it, i.e. the halo), the stable key-range
partition (k_part_count / k_part_scatter's rule) and the reference voxelize over a received list
(stable sort + sequential f32 sum in stable order, inc/voxelize.h:9-48).  TEST INFRASTRUCTURE."""
import numpy as np

from ros_gpu_depthmap_fusion_amd import multi, synth


def rank_points(orc, cams, rank, frame, params, halo: bool, gen=synth.dense_frame, move=None):
    """Compacted (points, keys) of camera `rank` as one rank of the fused layout produces them:
    the oracle runs camera rank-1 in front (its top-row reads) and drops its points.
    On the rollbuffer rank (`move` = (T_world_move, T_crop_move)) the point sequences added to
    `orc` are ingested too and their selected points follow the camera's (offset sum(P),
    fusion.cpp:1525/:1559)."""
    orc.clear()
    ks = [rank - 1, rank] if (halo and rank > 0) else [rank]
    for k in ks:
        c = cams[k]
        orc.addDepthmap(gen(c, k, frame), *c.intrinsics(), c.T_world, c.T_crop)
    if move is None:
        orc.processFrame(params)
    else:
        orc.processFrame(params, T_world_move=move[0], T_crop_move=move[1])
    pts, keys = orc.downloadPoints(), orc.downloadVoxelCoords()
    if len(ks) == 2:
        n_prev = cams[rank - 1].width * cams[rank - 1].height
        nh = int(np.count_nonzero(orc.stage_arrays()["maskA"][:n_prev]))
        pts, keys = pts[nh:], keys[nh:]
    return pts, keys


def partition(pts, keys, nparts, ncells):
    part = multi.part_of_keys(keys, nparts, ncells)
    order = np.argsort(part, kind="stable")
    return pts[order], keys[order], np.bincount(part, minlength=nparts).tolist()


def voxelize(pts, keys):
    """Voxel means in ascending key order, x/y/z = sequential f32 sum / f32 count."""
    if len(keys) == 0:
        return np.zeros((0, 3), np.float32)
    order = np.argsort(keys, kind="stable")
    k, p = keys[order], pts[order]
    starts = np.flatnonzero(np.r_[True, k[1:] != k[:-1]])
    ends = np.r_[starts[1:], len(k)]
    out = np.empty((len(starts), 3), np.float32)
    for g, (a, b) in enumerate(zip(starts, ends)):
        s = np.cumsum(p[a:b, :3], axis=0, dtype=np.float32)[-1]
        out[g] = s / np.float32(b - a)
    return out


# ---- the rollbuffer leg (point sequences on the last rank) ---------------------------------------
def lidar_camera(width: int, height: int):
    """The point-sequence source of the tests: a lidar-like camera (yaw 45 deg) whose dense depth
    frames are back-projected into PointCloud2 records (x, y, z, 1) - SURVEY §8(d) C3's sequences."""
    return synth.make_camera(1, width, height)


def sequence_records(lidar, k: int) -> np.ndarray:
    """Records of point sequence k: (n, 4) float32, x/y/z at byte offsets 0/4/8."""
    pts = synth.back_project(lidar, synth.dense_frame(lidar, 1, k % 2))
    return np.ascontiguousarray(np.concatenate([pts, np.ones((len(pts), 1), np.float32)], 1))


def schedule(first: int, frames: int):
    """Sequences ingested before each frame: `first` at once, then one per frame (the window then
    rolls the oldest out once it is full)."""
    out, k = [], 0
    for f in range(frames):
        nb = first if f == 0 else 1
        out.append(list(range(k, k + nb)))
        k += nb
    return out
