#!/usr/bin/env python3
"""Phase timing of the persistent ICP kernel on a VGA 512^3 run (GPU box; a trace
build: tools/variants.sh trace -DKFX_ICP_TRACE, then KFX_LIB_PATH=.../lib/var_trace/libkfx.so);
`icp_trace.py hd720`: 1280x720 frames (C5's size) on a 512^3 volume of C5's
4.096 m extent."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-kinectfusion_amd"))
import kfx  # noqa: E402
from kfx import synth  # noqa: E402
from kfx.abi import default_params  # noqa: E402

hd = len(sys.argv) > 1 and sys.argv[1] == "hd720"
intr = synth.Intrinsics.hd720() if hd else synth.Intrinsics.vga()
L = 4.096 if hd else 2.048
kf = kfx.KinectFusion(intr, default_params(dims=512, range_m=L))
# the benchmark's regime: frames staged in HBM, overlapped launches (the
# next frame's preprocess runs beside this frame's ICP), 25 frames
bgr, dep, _ = synth.sequence(25, intr, L=L)
kf.stage_frames(bgr, dep.astype(np.float32))
for k in range(len(dep)):
    kf.pipeline_staged(k)
kf.synchronize()
tr = kf.icp_trace().astype(np.int64)
t0 = tr[0, 0]
print("iter  start  b0_arrive  last_arrive  release  solved   (us from frame ICP start; 100 MHz)")
for i, r in enumerate(tr):
    f = lambda v: (v - t0) / 100.0
    print(f"{i:3d} {f(r[0]):7.2f} {f(r[1]):9.2f} {f(r[4]):11.2f} {f(r[2]):8.2f} {f(r[3]):7.2f}")
print("per-iteration (release-start):", np.round((tr[:, 2] - tr[:, 0]) / 100.0, 2))
print("lane (load+gather+products):", np.round((tr[:, 8] - tr[:, 0]) / 100.0, 2))
print("block reduce:", np.round((tr[:, 9] - tr[:, 8]) / 100.0, 2))
print("atomics:", np.round((tr[:, 10] - tr[:, 9]) / 100.0, 2))
print("arrive:", np.round((tr[:, 1] - tr[:, 10]) / 100.0, 2))
print("sums read:", np.round((tr[:, 5] - tr[:, 2]) / 100.0, 2))
print("solve:", np.round((tr[:, 6] - tr[:, 5]) / 100.0, 2))
print("post-solve:", np.round((tr[:, 3] - tr[:, 6]) / 100.0, 2))
