"""Generate tests/golden/radix_ref.npz from the REFERENCE's own radix sort (oracle/_ref).

Run in the build container (where /root/reference exists):  python tests/golden/make_golden.py
The fixture holds inputs and the reference's outputs only (RadixGrouper::group of
include/gpu_depthmap_fusion/radix_grouper.h:22-64 over radix_sort.h:107-289), so the GPU box, which
has no reference, can still pin the oracle and the GPU voxelize against it.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
from oracle import RefRadix, build  # noqa: E402


def cases():
    rng = np.random.default_rng(20261015)
    yield "rand22", rng.integers(0, 1 << 22, 3000).astype(np.uint32)
    yield "dups", rng.integers(0, 40, 2500).astype(np.uint32)
    yield "voxelish", (rng.integers(0, 400, 2000) + 400 * rng.integers(0, 400, 2000)
                       + 160000 * rng.integers(0, 21, 2000)).astype(np.uint32)
    yield "full32", rng.integers(0, 1 << 32, 1500, dtype=np.uint64).astype(np.uint32)
    yield "sorted_desc", np.arange(777, dtype=np.uint32)[::-1].copy()
    yield "all_equal", np.full(333, 12345, np.uint32)
    yield "single", np.array([7], np.uint32)
    yield "ragged_tiles", rng.integers(0, 1 << 16, 4097 + 5).astype(np.uint32)


def main():
    build()
    ref = RefRadix()
    out = {}
    for name, keys in cases():
        for gsz in (8, 1024):
            si, sk, gs, gz, gv = ref.group(keys, gsz)
            if gsz == 8:
                out[name + "_keys"] = keys
                out[name + "_sorted_idx"] = si
                out[name + "_group_starts"] = gs
                out[name + "_group_sizes"] = gz
                out[name + "_group_values"] = gv
            else:  # group size must not change the result
                assert np.array_equal(si, out[name + "_sorted_idx"]), name
    np.savez_compressed(os.path.join(HERE, "radix_ref.npz"), **out)
    print("wrote", os.path.join(HERE, "radix_ref.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
