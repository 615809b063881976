"""Known-answer tests of the oracle's restatement of the reference's orphan shaders
(shader/mask_dilate.glsl:40-67, shader/transform_points.glsl:37-54), against hand-computed
answers and an independent pure-Python loop restatement."""
import numpy as np

from oracle import mask_dilate, transform_points


def py_dilate(m, F, as_written):
    """mask_dilate.glsl:45-67 literally: x = idx mod W, y = idx / W, dx outer, dy inner, unsigned
    x + dx (a negative sum wraps past W and is skipped), first zero writes 0 and returns."""
    H, W = m.shape
    flat = m.reshape(-1)
    out = np.empty_like(flat)
    for idx in range(W * H):
        x, y = idx % W, idx // W
        res = None
        for dx in range(-F, F + 1):
            if (x + dx) % 2**32 >= W:
                continue
            for dy in range(-F, F + 1):
                if (y + dy) % 2**32 >= H:
                    continue
                if flat[idx + dx + dy * W] == 0:
                    res = 0
                    break
            if res is not None:
                break
        out[idx] = res if res is not None else (0 if as_written else flat[idx])
    return out.reshape(H, W)


def test_mask_dilate_hand_computed():
    m = np.ones((4, 5), np.uint32) * 3
    m[1, 2] = 0
    m[3, 4] = 0
    want = np.array([[3, 0, 0, 0, 3],
                     [3, 0, 0, 0, 3],
                     [3, 0, 0, 0, 0],
                     [3, 3, 3, 0, 0]], np.uint32)
    np.testing.assert_array_equal(mask_dilate(m, 1), want)
    np.testing.assert_array_equal(mask_dilate(m, 0), m)          # 1x1 window: identity
    assert not mask_dilate(m, 1, as_written=True).any()          # line 67 writes 0
    np.testing.assert_array_equal(mask_dilate(m, 9), np.zeros_like(m))  # window > image


def test_mask_dilate_matches_literal_loop():
    rng = np.random.default_rng(3)
    for (H, W) in [(1, 1), (1, 9), (7, 1), (11, 13), (20, 33)]:
        m = (rng.random((H, W)) < 0.93) * rng.integers(1, 2**32, (H, W), dtype=np.uint64)
        m = m.astype(np.uint32)
        for F in (0, 1, 2, 5):
            for aw in (False, True):
                np.testing.assert_array_equal(mask_dilate(m, F, aw), py_dilate(m, F, aw),
                                              err_msg=f"{H}x{W} F={F} as_written={aw}")


def test_transform_points_known_answer():
    T = np.array([[0, 0, 1, 2], [-1, 0, 0, 3], [0, -1, 0, 4], [0, 0, 0, 1]], np.float32)
    pts = np.array([[1, 2, 3, 1], [4, 5, 6, 1], [7, 8, 9, 0.5]], np.float32)
    mask = np.array([1, 0, 7], np.uint32)
    out = np.full((3, 4), -9.0, np.float32)
    got = transform_points(pts, mask, T, out)
    np.testing.assert_array_equal(got[0], [5, 2, 2, 1])
    np.testing.assert_array_equal(got[1], [-9, -9, -9, -9])      # mask 0: not written
    np.testing.assert_array_equal(got[2], [9 + 1.0, -7 + 1.5, -8 + 2.0, 0.5])
