"""Deterministic synthetic depth frames and point sequences (SURVEY.md §8(d) "Synthetic inputs").

There is no network and no dataset: frames are ray-cast from an analytic scene (ground plane,
room walls, boxes, a sphere) with a counter-hash RNG, h = splitmix64(seed ^ cam<<48 ^ frame<<32 ^
pixel), for ±1 % multiplicative depth noise and 3 % zero holes.  Depth is uint16 millimetres in
[300, 12000]; further returns are dropped (0), so some points exceed the 10 m max_distance of the
flying-pixel filter and some leave the crop box.

Camera k: fx = fy = 0.6 W, cx = W/2, cy = H/2, depth_scale 0.001, T_world = yaw(45°·k) ·
optical→world rotation [[0,0,1],[-1,0,0],[0,-1,0]] with the camera 1 m above the ground
(the crop frame is the world frame, launch/gpu_depthmap_fusion.launch:71).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Tuple

import numpy as np

SEED_BASE = 0x5EED0000
_M1 = np.uint64(0x9E3779B97F4A7C15)
_M2 = np.uint64(0xBF58476D1CE4E5B9)
_M3 = np.uint64(0x94D049BB133111EB)


def splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = (x + _M1).astype(np.uint64)
        z = (z ^ (z >> np.uint64(30))) * _M2
        z = (z ^ (z >> np.uint64(27))) * _M3
        return z ^ (z >> np.uint64(31))


def uniform01(h: np.ndarray) -> np.ndarray:
    return (h >> np.uint64(11)).astype(np.float64) * (1.0 / 9007199254740992.0)


@dataclass
class Camera:
    width: int
    height: int
    fx: float
    fy: float
    cx: float
    cy: float
    depth_scale: float
    T_world: np.ndarray  # 4x4 float32 row-major
    T_crop: np.ndarray

    def intrinsics(self):
        return self.depth_scale, self.fx, self.fy, self.cx, self.cy


OPT_TO_WORLD = np.array([[0, 0, 1], [-1, 0, 0], [0, -1, 0]], np.float64)


def yaw(deg: float) -> np.ndarray:
    a = np.deg2rad(deg)
    c, s = np.cos(a), np.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]], np.float64)


def make_camera(k: int, width: int, height: int) -> Camera:
    R = yaw(45.0 * k) @ OPT_TO_WORLD
    T = np.eye(4, dtype=np.float64)
    T[:3, :3] = R
    T[:3, 3] = (0.0, 0.0, 1.0)
    T = T.astype(np.float32)
    return Camera(width, height, float(np.float32(0.6 * width)), float(np.float32(0.6 * width)),
                  float(width / 2), float(height / 2), 0.001, T, T.copy())


# scene: (lo, hi) boxes in world metres
BOXES = [((3.0, -1.5, 0.0), (4.0, -0.5, 1.2)),
         ((5.5, 1.0, 0.0), (6.5, 2.5, 2.0)),
         ((-4.0, 3.0, 0.0), (-2.5, 4.0, 0.8)),
         ((1.5, -5.0, 0.0), (2.5, -3.5, 1.6))]
SPHERE = ((2.5, 1.0, 0.6), 0.6)
ROOM = ((-7.0, -7.0), (8.0, 7.0))  # x/y extent of the room walls
CEILING = 3.0


def _raycast(origin: np.ndarray, dirs: np.ndarray) -> np.ndarray:
    """Smallest positive ray parameter t (dirs have optical z = 1, so t = optical depth)."""
    n = dirs.shape[0]
    t = np.full(n, np.inf)
    dx, dy, dz = dirs[:, 0], dirs[:, 1], dirs[:, 2]
    with np.errstate(divide="ignore", invalid="ignore"):
        tg = np.where(dz < 0, -origin[2] / dz, np.inf)  # ground z = 0
        t = np.minimum(t, tg)
        tc = np.where(dz > 0, (CEILING - origin[2]) / dz, np.inf)  # ceiling
        t = np.minimum(t, tc)
        for ax, (lo, hi) in ((0, (ROOM[0][0], ROOM[1][0])), (1, (ROOM[0][1], ROOM[1][1]))):
            d = dirs[:, ax]
            tw = np.where(d > 0, (hi - origin[ax]) / d, np.where(d < 0, (lo - origin[ax]) / d, np.inf))
            t = np.minimum(t, np.where(tw > 0, tw, np.inf))
        for lo, hi in BOXES:
            lo = np.asarray(lo); hi = np.asarray(hi)
            t0 = (lo[None, :] - origin[None, :]) / dirs
            t1 = (hi[None, :] - origin[None, :]) / dirs
            tmin = np.nanmax(np.minimum(t0, t1), axis=1)
            tmax = np.nanmin(np.maximum(t0, t1), axis=1)
            hit = (tmax >= tmin) & (tmax > 0)
            tb = np.where(hit, np.where(tmin > 0, tmin, np.inf), np.inf)
            t = np.minimum(t, tb)
        c, r = np.asarray(SPHERE[0]), SPHERE[1]
        oc = origin - c
        a = np.sum(dirs * dirs, axis=1)
        b = 2 * dirs @ oc
        cc = oc @ oc - r * r
        disc = b * b - 4 * a * cc
        ts = np.where(disc >= 0, (-b - np.sqrt(np.maximum(disc, 0))) / (2 * a), np.inf)
        t = np.minimum(t, np.where(ts > 0, ts, np.inf))
    return t


def depth_frame(cam: Camera, k: int, frame: int, seed: int = SEED_BASE + 2,
                hole_frac: float = 0.03, noise: float = 0.01) -> np.ndarray:
    """uint16 [H, W] depth in millimetres for camera k at `frame`."""
    H, W = cam.height, cam.width
    v, u = np.mgrid[0:H, 0:W].astype(np.float64)
    ro = np.stack([(u - cam.cx) / cam.fx, (v - cam.cy) / cam.fy, np.ones_like(u)], -1).reshape(-1, 3)
    R = cam.T_world[:3, :3].astype(np.float64)
    dirs = ro @ R.T
    origin = cam.T_world[:3, 3].astype(np.float64)
    t = _raycast(origin, dirs)
    pix = np.arange(H * W, dtype=np.uint64)
    key = np.uint64(seed) ^ (np.uint64(k) << np.uint64(48)) ^ (np.uint64(frame) << np.uint64(32))
    h1 = splitmix64(key ^ pix)
    h2 = splitmix64(h1)
    nz = 1.0 + noise * (2.0 * uniform01(h1) - 1.0)
    d = np.where(np.isfinite(t), t * 1000.0 * nz, 0.0)
    d = np.rint(d)
    d = np.where((d < 300) | (d > 12000), 0, d)
    d = np.where(uniform01(h2) < hole_frac, 0, d)
    return d.astype(np.uint16).reshape(H, W)


def _value_noise(W: int, H: int, cells: int, key: np.uint64) -> np.ndarray:
    """Smooth value noise in [-1, 1] over an H x W image: random values on a lattice of `cells`
    cells across the image width (square cells, so the structure has the same angular size at
    every resolution), smoothstep-interpolated."""
    step = W / float(cells)
    gx, gy = cells + 2, int(np.ceil(H / step)) + 2
    node = np.arange(gx * gy, dtype=np.uint64)
    lat = (2.0 * uniform01(splitmix64(key ^ node)) - 1.0).reshape(gy, gx)
    fu = (np.arange(W, dtype=np.float64) + 0.5) / step
    fv = (np.arange(H, dtype=np.float64) + 0.5) / step
    iu, iv = np.floor(fu).astype(np.int64), np.floor(fv).astype(np.int64)
    su, sv = fu - iu, fv - iv
    su, sv = su * su * (3 - 2 * su), sv * sv * (3 - 2 * sv)
    a = lat[iv][:, iu]
    b = lat[iv][:, iu + 1]
    c = lat[iv + 1][:, iu]
    d = lat[iv + 1][:, iu + 1]
    top = a + (b - a) * su[None, :]
    bot = c + (d - c) * su[None, :]
    return top + (bot - top) * sv[:, None]


def dense_frame(cam: Camera, k: int, frame: int, seed: int = SEED_BASE + 2) -> np.ndarray:
    """uint16 [H, W] depth in millimetres with sensor-like, spatially correlated errors: the
    realistic-density workload of the benchmark (VERDICT r1 "What's weak" 4).

    `depth_frame` draws independent ±1 % noise and 3 % holes per pixel; at 4K 1 % of the depth is
    ~20x the lateral pixel spacing, every surface normal is noise and the flying-pixel filter
    (filter_flying_pixels.glsl:135-165, F=4 thr 0.3) removes ~99.97 % of the pixels.  Here the
    errors have a size in the image (fractions of the field of view), not in pixels:
      - a smooth depth bias of ±0.2 % (value noise, 32 cells across the image);
      - ±0.5 mm dither before the rounding to whole millimetres (the u16 quantisation);
      - holes as blobs (value noise over 48 cells above a threshold, ~2 % of the image) plus a
        0.02 % per-pixel dropout.
    With the same analytic scene about 60-70 % of the pixels survive the launch-default filter at
    VGA, 720p and 4K alike (tests/test_synth.py states the measured fractions)."""
    H, W = cam.height, cam.width
    v, u = np.mgrid[0:H, 0:W].astype(np.float64)
    ro = np.stack([(u - cam.cx) / cam.fx, (v - cam.cy) / cam.fy, np.ones_like(u)], -1).reshape(-1, 3)
    R = cam.T_world[:3, :3].astype(np.float64)
    dirs = ro @ R.T
    origin = cam.T_world[:3, 3].astype(np.float64)
    t = _raycast(origin, dirs).reshape(H, W)
    key = np.uint64(seed) ^ (np.uint64(k) << np.uint64(48)) ^ (np.uint64(frame) << np.uint64(32))
    bias = _value_noise(W, H, 32, key ^ np.uint64(0xB1A5 << 16))
    blobs = _value_noise(W, H, 48, key ^ np.uint64(0x401E << 16))
    pix = np.arange(H * W, dtype=np.uint64)
    h1 = splitmix64(key ^ pix).reshape(H, W)
    h2 = splitmix64(h1)
    dither = uniform01(h1) - 0.5
    d = np.where(np.isfinite(t), t * 1000.0 * (1.0 + 0.002 * bias) + dither, 0.0)
    d = np.rint(d)
    d = np.where((d < 300) | (d > 12000), 0, d)
    d = np.where((blobs > 0.80) | (uniform01(h2) < 2e-4), 0, d)
    return d.astype(np.uint16)


WORKLOADS = {"dense": dense_frame, "stress": depth_frame}


def uniform_frame(cam: Camera, k: int, frame: int, seed: int = SEED_BASE + 9) -> np.ndarray:
    """Stress frame: uniform random u16 depth (flying pixels everywhere)."""
    pix = np.arange(cam.height * cam.width, dtype=np.uint64)
    key = np.uint64(seed) ^ (np.uint64(k) << np.uint64(48)) ^ (np.uint64(frame) << np.uint64(32))
    h = splitmix64(key ^ pix)
    return (h & np.uint64(0xFFFF)).astype(np.uint16).reshape(cam.height, cam.width)


def back_project(cam: Camera, depth: np.ndarray) -> np.ndarray:
    """Camera-frame points (n, 3) float32 of every pixel (zero depth -> origin), as a lidar-like
    point sequence (a 720p frame back-projected)."""
    H, W = depth.shape
    v, u = np.mgrid[0:H, 0:W].astype(np.float32)
    z = depth.astype(np.float32) * np.float32(cam.depth_scale)
    x = (u - np.float32(cam.cx)) / np.float32(cam.fx) * z
    y = (v - np.float32(cam.cy)) / np.float32(cam.fy) * z
    return np.stack([x, y, z], -1).reshape(-1, 3).astype(np.float32)


def sequence_time(k: int, fps: int = 30) -> Tuple[int, int]:
    return 1000 + k // fps, (k % fps) * (1000000000 // fps)


def move_transform(k: int) -> np.ndarray:
    T = np.eye(4, dtype=np.float32)
    T[0, 3] = np.float32(0.01 * k)
    return T


def cameras(n: int, width: int, height: int) -> List[Camera]:
    return [make_camera(k, width, height) for k in range(n)]


RESOLUTIONS = {"vga": (640, 480), "720p": (1280, 720), "4k": (3840, 2160)}
