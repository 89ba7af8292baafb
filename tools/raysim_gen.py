#!/usr/bin/env python3
"""Volume + pose for tools/raysim (CPU model of k_raycast's march schedule).

Runs the serial oracle over the frames tools/ray_trace.py drives on the GPU
(C2: 640x480, 512^3 @ 4 mm, the bench's synthetic sequence in ping-pong order)
and dumps the x-fastest int16 tsdf plus the last frame's cam2vol pose, so the
march schedule of every wave can be counted on the CPU against the same volume
the GPU traces saw (the oracle is bit-identical to the GPU pipeline).
usage: python3 tools/raysim_gen.py [frames] [out_dir]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-kinectfusion_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402  (test infrastructure: an analysis tool, not the product)
from kfx import synth  # noqa: E402
from kfx.abi import Intrinsics, Pose, default_params  # noqa: E402

nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 25
out = sys.argv[2] if len(sys.argv) > 2 else "/tmp/raysim"
dims = int(os.environ.get("RAYSIM_DIMS", "512"))
os.makedirs(out, exist_ok=True)
intr = synth.Intrinsics.vga()
p = default_params(dims=dims, range_m=2.048)
bgr, dep, _ = synth.sequence(48, intr, L=2.048, noise=True, traj_seed=7, dropout=0.005)
order = synth.ping_pong(48, nfr)
pipe = O.Pipeline(Intrinsics.from_any(intr), p)
for k, i in enumerate(order):
    assert pipe.process(bgr[i], dep[i].astype(np.float32)) == 0
    print(f"frame {k + 1}/{nfr}", flush=True)
t, w, c = pipe.volume()
t.astype(np.int16).tofile(os.path.join(out, "tsdf.bin"))
pose = Pose.from_matrix(pipe.poses()[-1].astype(np.float32))
c2v = O.pose_mul(O.pose_inv(p.volu_pose), pose)
m = c2v.matrix().astype(np.float32)
np.array([dims, 640, 480], np.int32).tofile(os.path.join(out, "dims.bin"))
np.concatenate([m[:3, :3].ravel(), m[:3, 3]]).astype(np.float32).tofile(os.path.join(out, "c2v.bin"))
print("wrote", out)
