"""Model of the GPU voxel sum (gdf_voxsum.hpp: comp_stretch_sum, rows_chunk_sum) - TEST
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


def cursor_sum(x, R=4, stats=None):
    """The GPU's form (gdf_voxsum.hpp comp_stretch_sum): attempts over up to 64 R values from a
    cursor, every step checked as a rounding step (|P| in [2^23 + 1, 2^24 - 1]), terms clamped to
    +-2^25, ties and NaN caught by |y - t| >= 1/2; the first failing value j: prefix committed,
    x_j added by one f32 add, next attempt at j + 1; an attempt failing within its first 32 R values
    is followed by 1, 2, 4 .. 32 rows of the plain chain (reset by any attempt getting further), a
    zero / tiny sum takes one chain row, an inf / NaN sum the plain chain to the end."""
    x = np.asarray(x, f32)
    s = f32(0.0)
    pos, n = 0, len(x)
    streak = ser = 0  # the kernel's backoff: chain rows after attempts failing early
    while pos < n:
        ex = (_bits(s) >> 23) & 255
        if ser or (ex < 24 and pos < n):
            ser = max(ser - 1, 0)
            with np.errstate(all="ignore"):
                for v in x[pos:pos + 64]:
                    s = f32(s + v)
            pos += 64
            if stats is not None:
                stats["single"] += 1
            continue
        if ex == 255:
            with np.errstate(all="ignore"):
                for v in x[pos:]:
                    s = f32(s + v)
            return s
        if stats is not None:
            stats["stretches"] += 1
        scale = _float((277 - ex) << 23)
        u = _float((ex - 23) << 23)
        O = int(f32(s * scale))
        seg = x[pos:pos + 64 * R]
        with np.errstate(all="ignore"):
            y = (seg * scale).astype(f32)
            r = np.clip(np.rint(y), f32(-33554432.0), f32(33554432.0)).astype(f32)
            d = (y - r).astype(f32)
            bad = ~(np.abs(d) < f32(0.5))  # (NaN: not < 0.5)
        t = np.where(bad, 0, r).astype(np.int64)  # (values past a failure are never used)
        P = O + np.cumsum(t)
        aP = np.abs(P)
        bad |= (aP < 8388609) | (aP > 16777215)
        f = np.flatnonzero(bad)
        if len(f) == 0:
            s = f32(f32(P[-1]) * u)
            pos += len(seg)
            streak = 0
            continue
        j = int(f[0])
        pre = O if j == 0 else int(P[j - 1])
        with np.errstate(all="ignore"):
            s = f32(f32(f32(pre) * u) + seg[j])
        pos += j + 1
        if j < 32 * R:
            ser = 1 << min(streak, 5)
            streak += 1
        else:
            streak = 0
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


def rows_sum(x, NR=16, stats=None):
    """The GPU's row form (gdf_voxsum.hpp rows_chunk_sum): chunks of NR rows of 64 values; per row
    a predicted binade (the f32 sum s plus the rows up to it, summed loosely - a guess, checked;
    non-finite for a row holding or following a NaN / inf term),
    its integer terms t = rint(x / u) clamped to +-2^24, the row total T and the min / max of the
    row's running prefix, and whether any |x / u - t| >= 1/2 (tie / NaN).  Then, from the exact s,
    row after row while the binade of s equals the row's guess and every running value
    |O + P_k| stays in [2^23 + 1, 2^24 - 1], s moves on by T u exactly; the first row failing
    that is added by the plain chain (64 f32 adds), as is any row while s is zero, tiny, inf or
    NaN."""
    x = np.asarray(x, f32)
    s = f32(0.0)
    A, B = 8388609, 16777215
    CH = 64 * NR
    for c0 in range(0, len(x), CH):
        seg = x[c0:c0 + CH]
        nrows = (len(seg) + 63) // 64
        rows = np.full((nrows, 64), f32(-0.0), f32)
        rows.reshape(-1)[:len(seg)] = seg
        with np.errstate(all="ignore"):
            rsum = rows.sum(axis=1, dtype=f32)
            pred = (s + np.cumsum(rsum, dtype=f32)).astype(f32)
        exr = (pred.view(np.uint32) >> 23) & 255
        info = []
        for r in range(nrows):
            e = min(max(int(exr[r]), 24), 254)
            scale = _float((277 - e) << 23)
            with np.errstate(all="ignore"):
                y = (rows[r] * scale).astype(f32)
                t = np.clip(np.rint(y), f32(-16777216.0), f32(16777216.0)).astype(f32)
                d = np.abs((y - t).astype(f32))
            fail = not bool(np.all(d[np.isfinite(rows[r])] < f32(0.5)))  # (NaN / inf: the guess)
            P = np.cumsum(np.where(np.isfinite(t), t, 0).astype(np.int64))
            info.append((int(exr[r]), fail, int(P[-1]), int(P.min()), int(P.max())))
        r = 0
        while r < nrows:
            ex = (_bits(s) >> 23) & 255
            ok = 24 <= ex != 255
            if ok:
                ex_r, fail, T, mn, mx = info[r]
                scale = _float((277 - ex) << 23)
                O = int(f32(s * scale))
                if O > 0:
                    ok = ex_r == ex and not fail and O + mn >= A and O + mx <= B
                else:
                    ok = ex_r == ex and not fail and O + mx <= -A and O + mn >= -B
            if ok:
                s = f32(f32(O + T) * _float((ex - 23) << 23))
                if stats is not None:
                    stats["rows"] = stats.get("rows", 0) + 1
            else:
                with np.errstate(all="ignore"):
                    for v in rows[r]:
                        s = f32(s + v)
                if stats is not None:
                    stats["chain_rows"] = stats.get("chain_rows", 0) + 1
            r += 1
    return s
