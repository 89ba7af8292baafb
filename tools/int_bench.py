#!/usr/bin/env python3
"""Stage-level timing of k_integrate on a fixed C2 volume state (run it under
rocprofv3 --kernel-trace --stats): the bench's synthetic sequence runs
`frames` frames, the volume is snapshotted, then the next frame is integrated
`reps` times, the snapshot re-uploaded before each, so every timed launch
sees the same state (transient after ~10 frames, saturated after ~100).
usage: [KFX_LIB_PATH=...] python3 tools/int_bench.py [frames] [reps]"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "slam-kinectfusion_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "oracle"))
import kfx  # noqa: E402
from kfx import synth  # noqa: E402
from kfx.abi import Intrinsics, Pose, default_params  # noqa: E402
import oracle as O  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 10
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 8
intr = synth.Intrinsics.vga()
I = Intrinsics.from_any(intr)
p = default_params(dims=512, range_m=2.048)
bgr, dep, _ = synth.sequence(48, intr, L=2.048, noise=True, traj_seed=7, dropout=0.005)
order = synth.ping_pong(48, frames + 1)
kf = kfx.KinectFusion(I, p)
kf.stage_frames(bgr, dep.astype(np.float32))
for i in order[:frames]:
    kf.pipeline_staged(int(i))
kf.synchronize()
snap = kf.download_tsdf()
k = int(order[frames])
pose = Pose.from_matrix(kf.pose_record[-1])
vol2cam = O.pose_mul(O.pose_inv(pose), p.volu_pose)
kf.stage_preprocess(bgr[k], dep[k].astype(np.float32))
for r in range(reps):
    kf.upload_tsdf(snap)
    nu, nc = kf.stage_integrate(vol2cam, counts=(r == 0))
    if r == 0:
        print(f"frames {frames}: updated {nu} coloured {nc}")
kf.close()
