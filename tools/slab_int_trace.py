#!/usr/bin/env python3
"""Per-wave timeline of one Z-slab member's k_integrate (debug library built
with -DKFX_INT_TRACE): the C4 / C5 split held as an in-process group on one GPU
(kfx_pipeline_group), a few frames, then each listed member integrates the last
frame once more alone (kfx_stage_integrate at the last tracked pose) with the
trace on; prints the wave-duration spread, the resident fraction over time and
how much of the span is the tail.
usage: KFX_LIB_PATH=<trace lib> python3 tools/slab_int_trace.py c4|c5 [ranks, e.g. 0,7] [frames]"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-kinectfusion_amd"))
sys.path.insert(0, ROOT)
import kfx  # noqa: E402
from kfx import synth  # noqa: E402
from kfx.abi import Intrinsics, Pose, default_params  # noqa: E402
from bench import CONFIGS, intrinsics  # noqa: E402

cfg = sys.argv[1] if len(sys.argv) > 1 else "c4"
ranks = [int(r) for r in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 7]
nfr = int(sys.argv[3]) if len(sys.argv) > 3 else 6
W, H, n, L = CONFIGS[cfg]
intr = intrinsics(W, H)
p = default_params(dims=n, range_m=L)
bgr, dep, gt = synth.sequence(16, intr, L=L, noise=True, traj_seed=7, dropout=0.005)
dep = dep.astype(np.float32)
I = Intrinsics.from_any(intr)
probe = kfx.KinectFusion(I, p, slab=(0, n // 16))
work = np.mean([probe.slice_work_at(bgr[i], dep[i], gt[i])[0] for i in (0, 5, 10, 15)], axis=0).round().astype(np.int64)
probe.close()
cuts = kfx.slab_balance(work, 8)
members = [kfx.KinectFusion(I, p, slab=(r, 8), cuts=cuts) for r in range(8)]
order = synth.ping_pong(16, nfr)
for i in order:
    assert kfx.pipeline_group(members, bgr[i], dep[i]) == kfx.KFX_OK
lib = kfx.lib()
print(f"{cfg} cuts {list(cuts)}")
for r in ranks:
    m = members[r]
    vol2cam = Pose.from_matrix(np.linalg.inv(m.pose_record[-1].astype(np.float64)) @ p.volu_pose.matrix())
    m.stage_integrate(vol2cam, counts=False)
    buf = (C.c_uint64 * (4 * (1 << 20)))()
    nw = lib.kfx_debug_integrate_trace(buf, 1 << 20)
    a = np.frombuffer(buf, dtype=np.uint64)[: 4 * nw].reshape(nw, 4).astype(np.int64)
    live = a[:, 1] > 0
    a = a[live]
    t0 = a[:, 0].min()
    st, en = (a[:, 0] - t0) * 10, (a[:, 1] - t0) * 10
    dur = en - st
    span = en.max()
    print(f"rank {r}: waves launched {nw}, recorded {len(a)}; span {span / 1e3:.1f} us; wave dur us med "
          f"{np.median(dur) / 1e3:.1f} p90 {np.percentile(dur, 90) / 1e3:.1f} max {dur.max() / 1e3:.1f}; "
          f"start spread {st.max() / 1e3:.1f} us")
    for q in (50, 90, 99, 100):
        print(f"   {q:3d}% of waves done by {np.percentile(en, q) / 1e3:7.1f} us")
    for k in range(10):
        t = span * (k + 0.5) / 10
        print(f"   t={t / 1e3:6.1f} us resident {((st <= t) & (en > t)).sum() / 8192:5.2f}")
    short = dur < 3000
    print(f"   waves under 3 us (empty intervals): {short.sum()}  ({short.mean():.2f})")
for m in members:
    m.close()
