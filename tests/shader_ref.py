"""Second, independent restatement of the reference shaders in pure Python with float32 scalar
arithmetic, for tiny inputs only (TEST INFRASTRUCTURE).  It pins the C oracle: both are written
from the GLSL sources (shader/*.glsl of the reference) and must agree bit for bit.
"""
import math

import numpy as np

f32 = np.float32


def _mrow(M, r, p):
    m = M[4 * r: 4 * r + 4]
    return f32(f32(f32(f32(m[0] * p[0]) + f32(m[1] * p[1])) + f32(m[2] * p[2])) + f32(m[3] * p[3]))


def mat_vec(M, p):
    M = [f32(x) for x in np.asarray(M, np.float32).reshape(16)]
    return [_mrow(M, r, p) for r in range(4)]


def dot3(a, b):
    return f32(f32(f32(a[0] * b[0]) + f32(a[1] * b[1])) + f32(a[2] * b[2]))


def normalize3(a):
    l = f32(np.sqrt(dot3(a, a)))
    with np.errstate(all="ignore"):
        return [f32(a[0] / l), f32(a[1] / l), f32(a[2] / l)]


def cross3(a, b):
    return [f32(f32(a[1] * b[2]) - f32(a[2] * b[1])), f32(f32(a[2] * b[0]) - f32(a[0] * b[2])),
            f32(f32(a[0] * b[1]) - f32(a[1] * b[0]))]


def cam_point(idx, d, W, scale, fx, fy, cx, cy):
    """convert_depthmap_to_points.glsl:64-73 + rectify :75-81"""
    u = f32(idx % W)
    v = f32(idx // W)
    z = f32(f32(d) * f32(scale))
    with np.errstate(all="ignore"):
        x = f32(f32(u - f32(cx)) / f32(fx))
        y = f32(f32(v - f32(cy)) / f32(fy))
    return [f32(x * z), f32(y * z), z, f32(1.0)]


def convert(cams):
    """cams: list of (depth[H,W] u16, scale, fx, fy, cx, cy, Tw, Tc) -> maskA, A, B, C"""
    n = sum(c[0].size for c in cams)
    maskA = [0] * n
    A = [[f32(0)] * 4 for _ in range(n)]
    B = [[f32(0)] * 4 for _ in range(n)]
    Cc = [[f32(0)] * 4 for _ in range(n)]
    off = 0
    for (depth, scale, fx, fy, cx, cy, Tw, Tc) in cams:
        H, W = depth.shape
        flat = depth.reshape(-1)
        for idx in range(H * W):
            g = off + idx
            d = int(flat[idx])
            if d == 0:
                continue
            p = cam_point(idx, d, W, scale, fx, fy, cx, cy)
            maskA[g] = 1
            A[g] = p
            B[g] = mat_vec(Tw, p)
            Cc[g] = mat_vec(Tc, p)
        off += H * W
    return maskA, A, B, Cc


def flying(cams, maskA, A, F, thr, rot45):
    """filter_flying_pixels.glsl:43-165, OOB (wrapped) reads -> 0"""
    n = len(maskA)
    maskB = [0] * n
    thr = f32(thr)

    def m(gi):
        return maskA[gi] if 0 <= gi < n else 0

    off = 0
    for (depth, *_rest) in cams:
        H, W = depth.shape
        for idx in range(H * W):
            g = off + idx
            mv = maskA[g]
            if mv == 0:
                continue
            out = mv
            p = A[g][:3]
            if f32(np.sqrt(dot3(p, p))) > f32(10.0):
                continue
            x, y = idx % W, idx // W
            for i in range(1, F + 1):
                for variant in ([False, True] if rot45 else [False]):
                    ok = True
                    if x + i > W - 1 or y + i > H - 1:
                        ok = False
                    else:
                        iw = i * W
                        if not variant:
                            up, down, left, right = g - iw, g + iw, g - i, g + i
                        else:
                            up, down, left, right = g - iw - i, g + iw + i, g + iw - i, g - iw + i
                        if m(g) == 0 or m(up) == 0 or m(down) == 0 or m(left) == 0 or m(right) == 0:
                            ok = False
                        else:
                            pu, pd, pl, pr = A[up], A[down], A[left], A[right]
                            dx = [f32(pr[k] - pl[k]) for k in range(3)]
                            dy = [f32(pd[k] - pu[k]) for k in range(3)]
                            nrm = normalize3(cross3(dy, dx))
                            npv = normalize3(p)
                            nn = [f32(-npv[0]), f32(-npv[1]), f32(-npv[2])]
                            cv = dot3(nrm, nn)
                            if cv < thr:
                                ok = False
                    if not ok:
                        out = 0
            maskB[g] = out
        off += H * W
    return maskB


def crop(maskB, Cc, lo, hi):
    lo = [f32(v) for v in lo]
    hi = [f32(v) for v in hi]
    out = []
    for g, mv in enumerate(maskB):
        if mv == 0:
            out.append(0)
            continue
        p = Cc[g]
        if (p[0] < lo[0] or p[0] > hi[0] or p[1] < lo[1] or p[1] > hi[1] or p[2] < lo[2]
                or p[2] > hi[2]):
            out.append(0)
        else:
            out.append(mv)
    return out


def apply_mask(maskA, B):
    return [B[g] for g in range(len(maskA)) if maskA[g] > 0]


def voxel_coords(points, lo, hi, cs):
    gs = [int(math.ceil(f32(f32(f32(hi[a]) - f32(lo[a])) / f32(cs[a])))) for a in range(3)]
    out = []
    for p in points:
        u = []
        for a in range(3):
            with np.errstate(all="ignore"):
                f = f32(f32(p[a] - f32(lo[a])) / f32(cs[a]))
            f = f32(0.0) if np.isnan(f) else f
            f = min(max(f, f32(0.0)), f32(gs[a] - 1))
            u.append(int(np.floor(f)))
        out.append((u[0] + u[1] * gs[0] + u[2] * gs[0] * gs[1]) & 0xFFFFFFFF)
    return out, gs


def occupancy_step(hist, coords, lifetime):
    occ = [0] * len(hist)
    for c in coords:
        occ[c] = 1
    new = []
    for c, h in enumerate(hist):
        hb = h - 1 if h >= 1 else 0
        m = (occ[c] * lifetime) & 0xFFFFFFFF
        new.append(max(hb, m))
    return new, [v & 0xFF for v in new]


def ps_filter(points, thr, F):
    """filter_point_sequence.glsl:78-122 over one array of (x,y,z) points"""
    n = len(points)
    thr = f32(thr)
    out = []
    for g in range(n):
        p = [f32(v) for v in points[g][:3]]
        if f32(np.sqrt(dot3(p, p))) < f32(1e-3):
            out.append(0)
            continue
        inv = False
        for i in range(F):
            for j in (g + i - 1, g + i + 1):
                j &= 0xFFFFFFFF
                if j < n and not inv:
                    q = [f32(v) for v in points[j][:3]]
                    dvec = normalize3([f32(q[k] - p[k]) for k in range(3)])
                    npv = normalize3(p)
                    nn = [f32(-npv[0]), f32(-npv[1]), f32(-npv[2])]
                    c = f32(abs(dot3(dvec, nn)))
                    if f32(f32(1.0) - c) < thr:
                        inv = True
        out.append(0 if inv else 1)
    return out
