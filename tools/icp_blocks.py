#!/usr/bin/env python3
"""Per-block ICP phase stamps (debug library built with -DKFX_ICP_BLOCK_TRACE):
for each iteration, the spread of block lane-phase starts and arrivals (us,
relative to block 0's start), and which blocks arrive last.
usage: KFX_LIB_PATH=<debug lib> python3 tools/icp_blocks.py [hd720]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "slam-kinectfusion_amd"))
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
buf = (C.c_uint64 * (19 * 1024))()
n = kfx.lib().kfx_debug_icp_blocks(kf._h, buf, 19)
a = np.frombuffer(buf, np.uint64)[: n * 1024].reshape(n, 512, 2).astype(np.int64)
for s in range(n):
    st, ar = a[s, :, 0], a[s, :, 1]
    used = st > 0
    t0 = st[0]
    sts, ars = (st[used] - t0) / 100.0, (ar[used] - t0) / 100.0
    lane = ars - sts
    last = np.argsort(-ar[used])[:5]
    print(f"it {s:2d} blocks {used.sum():3d} start spread {sts.min():6.2f}..{sts.max():6.2f}  "
          f"arrive {ars.min():6.2f}..{ars.max():6.2f}  phase med {np.median(lane):5.2f} "
          f"p90 {np.percentile(lane, 90):5.2f} p99 {np.percentile(lane, 99):5.2f} max {lane.max():5.2f}  "
          f"last {list(np.nonzero(used)[0][last])}")
