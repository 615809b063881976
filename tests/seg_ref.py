"""Second, independent pure-Python restatement of the segmentation front end (small images only)
— TEST INFRASTRUCTURE.  Cross-checks oracle/seg_oracle.c the way tests/shader_ref.py checks the
GLSL restatement: same published algorithms, written separately and structured differently
(dictionary union-find over pixels, explicit 8-direction tables, Python ints).

OpenCV (absent here) semantics restated — see oracle/seg_oracle.c's header:
  labels:   8-connected components numbered by their first 2x2 block in block-raster order
  stats:    [LEFT, TOP, WIDTH, HEIGHT, AREA]; centroids = mean x, mean y
  contours: findContours(RETR_EXTERNAL, CHAIN_APPROX_NONE), reverse discovery order
"""
from __future__ import annotations

import numpy as np

# icvCodeDeltas: code -> (dx, dy)
CODE = [(1, 0), (1, -1), (0, -1), (-1, -1), (-1, 0), (-1, 1), (0, 1), (1, 1)]


def components(img: np.ndarray):
    """(labels, num_labels) of one layer."""
    H, W = img.shape
    parent = {}

    def find(a):
        while parent[a] != a:
            a = parent[a]
        return a

    def union(a, b):
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)

    fg = [(y, x) for y in range(H) for x in range(W) if img[y, x]]
    for p in fg:
        parent[p] = p
    for (y, x) in fg:
        for dy, dx in ((-1, -1), (-1, 0), (-1, 1), (0, -1)):
            q = (y + dy, x + dx)
            if q in parent:
                union((y, x), q)
    # first 2x2 block of every component, in block-raster order
    first = {}
    for (y, x) in fg:
        r = find((y, x))
        key = ((y // 2), (x // 2))
        if r not in first or key < first[r]:
            first[r] = key
    order = sorted(first, key=lambda r: first[r])
    rank = {r: i + 1 for i, r in enumerate(order)}
    lab = np.zeros((H, W), np.uint16)
    for p in fg:
        lab[p] = rank[find(p)]
    return lab, len(order) + 1


def stats(lab: np.ndarray, n: int):
    H, W = lab.shape
    st = np.zeros((n, 5), np.int64)
    ce = np.zeros((n, 2), np.float64)
    for l in range(n):
        ys, xs = np.nonzero(lab == l)
        if len(xs) == 0:
            st[l] = [2**31 - 1, 2**31 - 1, -(2**31) - (2**31 - 1) + 1, -(2**31) - (2**31 - 1) + 1, 0]
            ce[l] = [np.nan, np.nan]
            continue
        st[l] = [xs.min(), ys.min(), xs.max() - xs.min() + 1, ys.max() - ys.min() + 1, len(xs)]
        ce[l] = [float(int(xs.sum())) / len(xs), float(int(ys.sum())) / len(xs)]
    st = ((st + 2**31) % 2**32 - 2**31).astype(np.int32)  # int32 wrap of an empty label
    return st, ce


def external_contours(img: np.ndarray):
    """findContours(img, RETR_EXTERNAL, CHAIN_APPROX_NONE): list of (k, 2) int arrays."""
    H, W = img.shape
    Hp, Wp = H + 2, W + 2
    a = [[0] * Wp for _ in range(Hp)]
    for y in range(H):
        for x in range(W):
            a[y + 1][x + 1] = 1 if img[y, x] else 0

    def nz(x, y, s):
        dx, dy = CODE[s & 7]
        return a[y + dy][x + dx] != 0

    def fetch(x0, y0):
        pts = []
        s = None
        for c in (3, 2, 1, 0, 7, 6, 5):  # clockwise from code 3 (code 4 is the zero predecessor)
            if nz(x0, y0, c):
                s = c
                break
        if s is None:
            a[y0][x0] = -126
            return [(x0 - 1, y0 - 1)]
        x1, y1 = x0 + CODE[s][0], y0 + CODE[s][1]
        x3, y3 = x0, y0
        while True:
            s_end = s
            k = 1
            while not nz(x3, y3, s_end + k):
                k += 1
            s = (s_end + k) & 7
            x4, y4 = x3 + CODE[s][0], y3 + CODE[s][1]
            if 1 <= s <= s_end:  # (unsigned)(s - 1) < (unsigned)s_end: the east pixel was passed
                a[y3][x3] = -126
            elif a[y3][x3] == 1:
                a[y3][x3] = 2
            pts.append((x3 - 1, y3 - 1))
            if (x4, y4) == (x0, y0) and (x3, y3) == (x1, y1):
                break
            x3, y3 = x4, y4
            s = (s + 4) & 7
        return pts

    found = []
    for y in range(1, Hp - 1):
        prev, lnbd, x = 0, 0, 1
        while x < Wp - 1:
            p = a[y][x]
            if p == prev:
                x += 1
                continue
            if prev == 0 and p == 1:
                if a[y][lnbd] <= 0:
                    found.append(np.array(fetch(x, y), np.int32).reshape(-1, 2))
                    prev = a[y][x]
                    x += 1
                    continue
            elif p == 0 and prev >= 1 and (prev & -2):
                lnbd = x - 1
            prev = p
            if prev & -2:
                lnbd = x
            x += 1
    return found[::-1]


def front_end(grid: np.ndarray) -> dict:
    """The flat result dictionary of oracle.object_segmentation_front for a small grid."""
    L, H, W = grid.shape
    labs, nl, sts, ces, l2cs, ncont, sizes, pts = [], [], [], [], [], [], [], []
    for z in range(L):
        lab, n = components(grid[z])
        st, ce = stats(lab, n)
        cs = external_contours(grid[z])
        l2c = np.full(n, -1, np.int32)
        for j, c in enumerate(cs):
            l2c[lab[c[0, 1], c[0, 0]]] = j
        labs.append(lab); nl.append(n); sts.append(st); ces.append(ce); l2cs.append(l2c)
        ncont.append(len(cs)); sizes += [len(c) for c in cs]; pts += list(cs)
    conn, starts = [], []
    off = 0
    for z in range(L - 1):
        m = np.zeros((nl[z], nl[z + 1]), np.uint8)
        m[labs[z].ravel(), labs[z + 1].ravel()] = 1
        starts.append(off)
        off += m.size
        conn.append(m.ravel())
    # mergeLabelsAcrossLayers
    starts_l = np.cumsum([0] + nl[:-1])
    g = list(range(sum(nl)))
    for z in range(L - 1):
        m = conn[z].reshape(nl[z], nl[z + 1])
        for b in range(nl[z + 1]):
            for a_ in range(nl[z]):
                if (a_ == 0) != (b == 0) or not m[a_, b]:
                    continue
                g[starts_l[z + 1] + b] = min(g[starts_l[z + 1] + b], g[starts_l[z] + a_])
    for i in range(L - 1):
        za, zb = L - 2 - i, L - 1 - i
        m = conn[za].reshape(nl[za], nl[zb])
        for a_ in range(nl[za]):
            for b in range(nl[zb]):
                if (a_ == 0) != (b == 0) or not m[a_, b]:
                    continue
                g[starts_l[za] + a_] = min(g[starts_l[za] + a_], g[starts_l[zb] + b])
    ids = {v: i for i, v in enumerate(sorted(set(g)))}
    return dict(
        labels=np.stack(labs), num_labels=np.array(nl, np.uint32),
        stats=np.concatenate(sts), centroids=np.concatenate(ces),
        labels_to_contours=np.concatenate(l2cs), contours_per_layer=np.array(ncont, np.uint32),
        contour_sizes=np.array(sizes, np.uint32),
        contour_points=(np.concatenate(pts) if pts else np.zeros((0, 2), np.int32)),
        connections=(np.concatenate(conn) if conn else np.zeros(0, np.uint8)),
        connection_starts=np.array(starts, np.uint64),
        merged=np.array([ids[v] for v in g], np.uint32), num_objects=len(ids))
