"""Deterministic synthetic RGB-D sequences (SURVEY.md §8d "Synthetic inputs").

The reference's bundled dataset is not in the checkout, so every
test and benchmark runs on an analytic scene rendered here: a back wall, a
floor, a side wall, three spheres and a box inside the TSDF volume, seen by a
pinhole camera moving along a smooth, bounded trajectory (<= ~1 cm and ~0.5
deg per frame, cf. doc/poses.txt max 2.4 cm / 1.5 deg).

Coordinates follow the reference: camera frame x right, y down, z forward; the
world frame is the camera frame of frame 0 (kinectfusion.cpp:84-93 integrates
frame 1 at the identity pose).  Depth is uint16 millimetres like the dataset's
PNGs (depth_sensor.cpp:191), colour is BGR8.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


@dataclass
class Intrinsics:
    width: int = 640
    height: int = 480
    fx: float = 525.0
    fy: float = 525.0
    cx: float = 319.5
    cy: float = 239.5

    @staticmethod
    def vga() -> "Intrinsics":
        return Intrinsics(640, 480, 525.0, 525.0, 319.5, 239.5)

    @staticmethod
    def hd720() -> "Intrinsics":
        return Intrinsics(1280, 720, 920.0, 920.0, 639.5, 359.5)

    @staticmethod
    def qvga() -> "Intrinsics":
        return Intrinsics(320, 240, 262.5, 262.5, 159.5, 119.5)

    @staticmethod
    def qqvga() -> "Intrinsics":
        return Intrinsics(160, 120, 131.25, 131.25, 79.5, 59.5)


@dataclass
class Scene:
    """Analytic scene sized for a cubic volume of edge L metres whose pose is
    translate(-L/2, -L/2, 0.5) (kinectfusion.cpp:184)."""

    L: float = 2.048
    planes: list = field(default_factory=list)   # (normal(3), offset): n.x = c
    spheres: list = field(default_factory=list)  # (centre(3), radius)
    boxes: list = field(default_factory=list)    # (lo(3), hi(3))

    @staticmethod
    def default(L: float = 2.048) -> "Scene":
        z0 = 0.5
        s = Scene(L=L)
        s.planes = [
            (np.array([0.0, 0.0, 1.0]), z0 + 0.9 * L),   # back wall z = const
            (np.array([0.0, 1.0, 0.0]), 0.33 * L),       # floor y = const (y down)
            (np.array([1.0, 0.0, 0.0]), -0.42 * L),      # left wall
        ]
        s.spheres = [
            (np.array([-0.22 * L, 0.08 * L, z0 + 0.45 * L]), 0.10 * L),
            (np.array([0.20 * L, 0.12 * L, z0 + 0.62 * L]), 0.13 * L),
            (np.array([0.02 * L, -0.16 * L, z0 + 0.72 * L]), 0.08 * L),
        ]
        s.boxes = [
            (np.array([0.05 * L, 0.12 * L, z0 + 0.30 * L]), np.array([0.22 * L, 0.33 * L, z0 + 0.42 * L])),
        ]
        return s

    @staticmethod
    def plane(depth_m: float) -> "Scene":
        s = Scene(L=2.0)
        s.planes = [(np.array([0.0, 0.0, 1.0]), depth_m)]
        return s


def _rot(axis: str, ang: float) -> np.ndarray:
    c, s = math.cos(ang), math.sin(ang)
    if axis == "x":
        return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])
    if axis == "y":
        return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def trajectory(n_frames: int, seed: int = 7, amp_t: float = 0.08, amp_r_deg: float = 6.0,
               period: float = 120.0) -> np.ndarray:
    """Camera-to-world poses (n, 4, 4) float64, pose[0] = I.  Smooth sums of
    sines with seeded phases-free frequencies; per-frame motion stays below
    ~7 mm and ~0.4 deg for the defaults."""
    rng = np.random.default_rng(seed)
    w = 2.0 * math.pi / period
    fr = rng.uniform(0.7, 1.3, size=6)
    poses = np.zeros((n_frames, 4, 4))
    for k in range(n_frames):
        t = np.array([amp_t * math.sin(w * fr[0] * k),
                      0.5 * amp_t * math.sin(w * fr[1] * k),
                      0.6 * amp_t * math.sin(w * fr[2] * k)])
        yaw = math.radians(amp_r_deg) * math.sin(w * fr[3] * k)
        pitch = math.radians(0.6 * amp_r_deg) * math.sin(w * fr[4] * k)
        roll = math.radians(0.3 * amp_r_deg) * math.sin(w * fr[5] * k)
        R = _rot("y", yaw) @ _rot("x", pitch) @ _rot("z", roll)
        poses[k, :3, :3] = R
        poses[k, :3, 3] = t
        poses[k, 3, 3] = 1.0
    return poses


def render(scene: Scene, intr: Intrinsics, pose: np.ndarray, noise_seed: int | None = None,
           dropout: float = 0.0, max_depth_m: float = 6.5) -> tuple[np.ndarray, np.ndarray]:
    """Ray-cast the analytic scene.  Returns (bgr uint8 HxWx3, depth uint16 HxW mm).

    Depth is the camera-frame z of the nearest hit (un-normalised pinhole ray
    (u-cx)/fx, (v-cy)/fy, 1, so the ray parameter is z)."""
    H, W = intr.height, intr.width
    u, v = np.meshgrid(np.arange(W, dtype=np.float64), np.arange(H, dtype=np.float64))
    d_cam = np.stack([(u - intr.cx) / intr.fx, (v - intr.cy) / intr.fy, np.ones_like(u)], -1)
    R = pose[:3, :3]
    o = pose[:3, 3]
    d = d_cam @ R.T                                   # world directions (H, W, 3)
    best = np.full((H, W), np.inf)
    prim = np.full((H, W), -1, dtype=np.int32)
    pid = 0
    for n, c in scene.planes:
        nd = d @ n
        with np.errstate(divide="ignore", invalid="ignore"):
            t = (c - o @ n) / nd
        ok = (t > 1e-6) & (t < best)
        best = np.where(ok, t, best)
        prim = np.where(ok, pid, prim)
        pid += 1
    for ce, r in scene.spheres:
        oc = o - ce
        a = np.einsum("hwk,hwk->hw", d, d)
        b = 2.0 * (d @ oc)
        cc = oc @ oc - r * r
        disc = b * b - 4 * a * cc
        with np.errstate(invalid="ignore"):
            t = (-b - np.sqrt(disc)) / (2 * a)
        ok = (disc >= 0) & (t > 1e-6) & (t < best)
        best = np.where(ok, t, best)
        prim = np.where(ok, pid, prim)
        pid += 1
    for lo, hi in scene.boxes:
        with np.errstate(divide="ignore", invalid="ignore"):
            inv = 1.0 / d
            t0 = (lo - o) * inv
            t1 = (hi - o) * inv
        tmin = np.nanmax(np.minimum(t0, t1), axis=-1)
        tmax = np.nanmin(np.maximum(t0, t1), axis=-1)
        ok = (tmax >= tmin) & (tmin > 1e-6) & (tmin < best)
        best = np.where(ok, tmin, best)
        prim = np.where(ok, pid, prim)
        pid += 1
    depth = np.where(np.isfinite(best) & (best < max_depth_m), best, 0.0)
    if noise_seed is not None:
        rng = np.random.default_rng(noise_seed)
        sigma = 0.0012 + 0.0019 * (depth - 0.4) ** 2
        depth = np.where(depth > 0, depth + rng.normal(size=depth.shape) * sigma, 0.0)
        if dropout > 0:
            drop = rng.random(depth.shape) < dropout
            depth = np.where(drop, 0.0, depth)
    depth_mm = np.clip(np.rint(depth * 1000.0), 0, 65535).astype(np.uint16)
    # procedural checker colour by world position, tinted per primitive
    p = o + d * np.where(np.isfinite(best), best, 0.0)[..., None]
    chk = ((np.floor(p[..., 0] / 0.1) + np.floor(p[..., 1] / 0.1) + np.floor(p[..., 2] / 0.1)) % 2)
    tint = np.array([[200, 180, 160], [90, 140, 200], [120, 200, 120], [60, 60, 220],
                     [220, 120, 60], [180, 60, 180], [40, 200, 220], [160, 160, 40]], dtype=np.float64)
    base = tint[np.clip(prim, 0, len(tint) - 1) % len(tint)]
    col = base * (0.65 + 0.35 * chk)[..., None]
    col = np.where((prim >= 0)[..., None], col, 0.0)
    bgr = np.clip(np.rint(col), 0, 255).astype(np.uint8)
    return bgr, depth_mm


def sequence(n_frames: int, intr: Intrinsics | None = None, L: float = 2.048, noise: bool = False,
             seed: int = 42, traj_seed: int = 7, dropout: float = 0.0, **traj_kw):
    """Render n frames.  Returns (bgr (n,H,W,3) u8, depth (n,H,W) u16 mm,
    gt poses (n,4,4) f64)."""
    intr = intr or Intrinsics.vga()
    scene = Scene.default(L)
    poses = trajectory(n_frames, seed=traj_seed, **traj_kw)
    bgr = np.empty((n_frames, intr.height, intr.width, 3), np.uint8)
    dep = np.empty((n_frames, intr.height, intr.width), np.uint16)
    for k in range(n_frames):
        b, dm = render(scene, intr, poses[k], noise_seed=(seed + k) if noise else None,
                       dropout=dropout)
        bgr[k] = b
        dep[k] = dm
    return bgr, dep, poses


def ping_pong(n_unique: int, n_total: int) -> list[int]:
    """Frame order that walks 0..n-1..0.. so a looped sequence stays continuous."""
    if n_unique <= 1:
        return [0] * n_total
    cyc = list(range(n_unique)) + list(range(n_unique - 2, 0, -1))
    return [cyc[i % len(cyc)] for i in range(n_total)]
