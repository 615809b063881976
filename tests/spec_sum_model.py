"""Model of the GPU voxel sum (gdf_kernels.hip: spec_try / spec_finish / row_sum4) - TEST
INFRASTRUCTURE: a numpy restatement of the kernel's stretch algorithm, lane for lane, so its
exactness can be checked on the CPU against the reference's sequential f32 chain
(inc/voxelize.h:29-35) on adversarial inputs.

A row of 64 terms x_b..x_{nv-1} is added to s:
  * s not admissible (zero, |s| < 2^-104, inf, NaN): one ordinary f32 add, next term;
  * else u = ulp(s) = 2^(ex - 150), m = s / u, y_k = x_k / u, t_k = rint(y_k),
    P_k = m + t_b + ... + t_k (int), and lane k is valid when y_k is not a tie, |y_k| <= 2^24 and
    either y_k is integral with |P_k| <= 2^24, or 2^23 < |P_k| < 2^24;
  * the first invalid lane L: s = P_{L-1} u, s = fl(s + x_L), continue at L + 1.
"""
import numpy as np

f32 = np.float32


def _bits(v):
    return int(np.array([v], f32).view(np.uint32)[0])


def _float(b):
    return np.array([b], np.uint32).view(f32)[0]


def admissible(s):
    ex = (_bits(s) >> 23) & 255
    return 24 <= ex != 255


def row_sum(s, x, stats=None):
    """s + x[0] + ... + x[len(x)-1] in order (x: float32 array of <= 64 terms)."""
    s = f32(s)
    nv = len(x)
    b = 0
    while b < nv:
        if not admissible(s):
            with np.errstate(all="ignore"):
                s = f32(s + x[b])
            b += 1
            if stats is not None:
                stats["single"] += 1
            continue
        ex = (_bits(s) >> 23) & 255
        scale = _float((277 - ex) << 23)
        u = _float((ex - 23) << 23)
        m = int(f32(s * scale))
        with np.errstate(invalid="ignore", over="ignore"):
            y = (x[b:] * scale).astype(f32)
            r = np.rint(y).astype(f32)
            ok = (np.abs(y) <= f32(16777216.0)) & (np.abs(y - r) != f32(0.5))
        t = np.where(ok, r, 0).astype(np.int64)
        P = m + np.cumsum(t)
        aP = np.abs(P)
        exact = y == r
        ok &= np.where(exact, aP <= 16777216, (aP >= 8388609) & (aP <= 16777215))
        bad = np.flatnonzero(~ok)
        L = int(bad[0]) if len(bad) else len(y)
        if stats is not None:
            stats["stretches"] += 1
        if L > 0:
            s = f32(f32(P[L - 1]) * u)
        if L == len(y):
            break
        with np.errstate(all="ignore"):
            s = f32(s + x[b + L])
        b += L + 1
    return s


def group_sum(x, stats=None):
    s = f32(0.0)
    for r0 in range(0, len(x), 64):
        s = row_sum(s, x[r0:r0 + 64], stats)
    return s


def sequential_sum(x):
    """The reference's chain: float32 accumulate, one rounding per term."""
    if len(x) == 0:
        return f32(0.0)
    with np.errstate(all="ignore"):
        acc = np.add.accumulate(np.concatenate([[f32(0.0)], np.asarray(x, f32)]), dtype=f32)
    return f32(acc[-1])
