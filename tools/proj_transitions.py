#!/usr/bin/env python3
"""how often does a voxel's projected pixel change along a
column?  Within a column segment where vc is an arithmetic progression the
rounded projection (u, v) is a step function of z, so an incremental scheme
could reuse (iu, iv) and the depth gather between transitions and run the exact
division sequence only at transitions.  This counts, over the voxels integrate
visits (frustum + frame max depth, identity camera at the volume pose
translate(-L/2, -L/2, 0.5)), the fraction whose (u, v) differs from the
previous voxel's, for C2, C3 and C5.  usage: python3 tools/proj_transitions.py"""
import numpy as np

CASES = {  # name: (W, H, f, dims, L)
    "C2": (640, 480, 525.0, 512, 2.048),
    "C3": (640, 480, 525.0, 1024, 2.048),
    "C5": (1280, 720, 920.0, 2048, 4.096),
}
rng = np.random.default_rng(1)
for name, (W, H, f, n, L) in CASES.items():
    cx, cy = (W - 1) / 2, (H - 1) / 2
    vs = L / n
    zmax = 0.5 + 0.9 * L  # the scene's back wall: the frame max depth bounds the visited range
    cols = rng.integers(0, n, size=(20000, 2))
    z = np.arange(1, n)
    tot_vis, tot_tr, tot_tr_u, tot_tr_v = 0, 0, 0, 0
    for x, y in cols:
        X = x * vs - L / 2
        Y = y * vs - L / 2
        Z = z * vs + 0.5
        u = np.rint(X / Z * f + cx)
        v = np.rint(Y / Z * f + cy)
        vis = (u >= 0) & (u < W) & (v >= 0) & (v < H) & (Z <= zmax)
        if vis.sum() < 2:
            continue
        iv = np.flatnonzero(vis)
        du = u[iv[1:]] != u[iv[:-1]]
        dv = v[iv[1:]] != v[iv[:-1]]
        tot_vis += len(iv)
        tot_tr += int((du | dv).sum())
        tot_tr_u += int(du.sum())
        tot_tr_v += int(dv.sum())
    print(f"{name}: visited voxels sampled {tot_vis}, pixel transitions per voxel {tot_tr / tot_vis:.3f} "
          f"(u {tot_tr_u / tot_vis:.3f}, v {tot_tr_v / tot_vis:.3f}); build threshold: <= 0.333")
    # what a wave (8x8 column tile, lanes in lockstep over z in batches of 4
    # voxels) would see: the fraction of batches in which NO lane's pixel
    # changes (only those could skip the exact projection for the whole wave)
    quiet, batches = 0, 0
    for tx, ty in rng.integers(0, n // 8, size=(800, 2)):
        xs = tx * 8 + np.arange(8)
        ys = ty * 8 + np.arange(8)
        X = (xs[None, :, None] * vs - L / 2)
        Y = (ys[:, None, None] * vs - L / 2)
        Z = z[None, None, :] * vs + 0.5
        u = np.rint(X / Z * f + cx)
        v = np.rint(Y / Z * f + cy)
        vis = (u >= 0) & (u < W) & (v >= 0) & (v < H) & (Z <= zmax)
        ch = np.zeros_like(vis)
        ch[:, :, 1:] = ((u[:, :, 1:] != u[:, :, :-1]) | (v[:, :, 1:] != v[:, :, :-1])) & vis[:, :, 1:] & vis[:, :, :-1]
        any_vis = vis.reshape(64, -1).any(0)
        any_ch = ch.reshape(64, -1).any(0)
        for b in range(0, len(z) - 3, 4):
            if any_vis[b:b + 4].any():
                batches += 1
                quiet += not any_ch[b:b + 4].any()
    print(f"    wave batches (4 voxels x 64 lanes) with no lane changing pixel: {quiet / max(batches, 1):.4f} of {batches}")
