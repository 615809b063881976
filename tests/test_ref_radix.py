"""Pin the oracle's stable sort + grouping (the observable result of the reference's CPU voxel
radix sort, inc/radix_sort.h:107-289 + radix_grouper.h:22-64) against the reference itself:
the committed fixture tests/golden/radix_ref.npz (made by tests/golden/make_golden.py from
oracle/_ref) and, where oracle/_ref is built, fresh random inputs."""
import os

import numpy as np
import pytest

from oracle import RefRadix, stable_sort_keys

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "radix_ref.npz")


def groups_of(sorted_keys):
    n = len(sorted_keys)
    if n == 0:
        return np.zeros(0, np.uint32), np.zeros(0, np.uint32), np.zeros(0, np.uint32)
    starts = np.flatnonzero(np.r_[True, sorted_keys[1:] != sorted_keys[:-1]]).astype(np.uint32)
    sizes = np.diff(np.r_[starts, n]).astype(np.uint32)
    return starts, sizes, sorted_keys[starts]


def test_oracle_matches_reference_golden_vectors():
    g = np.load(GOLDEN)
    names = sorted({k.rsplit("_keys", 1)[0] for k in g.files if k.endswith("_keys")})
    assert len(names) >= 8
    for name in names:
        keys = g[name + "_keys"]
        idx, sk = stable_sort_keys(keys)
        np.testing.assert_array_equal(idx, g[name + "_sorted_idx"], err_msg=name)
        st, sz, gv = groups_of(sk)
        np.testing.assert_array_equal(st, g[name + "_group_starts"], err_msg=name)
        np.testing.assert_array_equal(sz, g[name + "_group_sizes"], err_msg=name)
        np.testing.assert_array_equal(gv, g[name + "_group_values"], err_msg=name)


@pytest.mark.skipif(not RefRadix.available(), reason="oracle/_ref not built (no reference sources)")
@pytest.mark.parametrize("n,hi,gsz", [(0, 10, 8), (1, 10, 8), (100003, 1 << 22, 8),
                                      (50000, 7, 1024), (65537, 1 << 32, 8), (4096, 1 << 12, 3)])
def test_oracle_matches_reference_radix_live(n, hi, gsz):
    rng = np.random.default_rng(n + gsz)
    keys = rng.integers(0, hi, n, dtype=np.uint64).astype(np.uint32)
    si, sk, gs, gz, gv = RefRadix().group(keys, gsz)
    idx, k2 = stable_sort_keys(keys)
    np.testing.assert_array_equal(idx, si)
    np.testing.assert_array_equal(k2, sk)
    st, sz, vv = groups_of(k2)
    if n:
        np.testing.assert_array_equal(st, gs)
        np.testing.assert_array_equal(sz, gz)
        np.testing.assert_array_equal(vv, gv)
