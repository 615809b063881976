"""multi.gather_fused_cloud on CPU (gloo, world 2 and 3): every rank's key range of voxels -
different lengths, one rank empty - arrives on the publishing rank concatenated in rank order
(= ascending voxel key, the order of the reference's single voxelize, fusion.cpp:1743-1756), the
other ranks get None.  The engine is a stub holding each rank's voxel list (the device path is
tests/test_gpu_multi.py::test_rccl_fused_cloud_world1)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def voxels_of(rank):
    n = [5, 0, 17][rank % 3]
    return (np.arange(4 * n, dtype=np.float32).reshape(n, 4) + 1000 * rank).astype(np.float32)


class _StubEngine:
    def __init__(self, rank):
        self.rank = rank

    def downloadVoxelizedPoints(self):
        return voxels_of(self.rank)


class _StubRank:
    def __init__(self, rank, world):
        self.eng, self.world, self.dev, self.hiprt = _StubEngine(rank), world, "cpu", None


def _rank(rank, world, port, root, out_dir):
    import torch.distributed as dist
    from ros_gpu_depthmap_fusion_amd import multi
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = multi.gather_fused_cloud(_StubRank(rank, world), root=root)
    if rank == root:
        np.save(os.path.join(out_dir, "pub.npy"), got.numpy())
    else:
        assert got is None
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("world,root", [(2, 0), (3, 0), (3, 2)])
def test_gather_fused_cloud_gloo(tmp_path, world, root):
    mp.start_processes(_rank, args=(world, _free_port(), root, str(tmp_path)), nprocs=world,
                       join=True, start_method="spawn")
    want = np.concatenate([voxels_of(r) for r in range(world)])
    np.testing.assert_array_equal(np.load(tmp_path / "pub.npy"), want)
