#!/usr/bin/env python3
"""Per-wave timeline of k_raycast (debug library built with -DKFX_RAY_TRACE):
runs the C2 bench workload, dumps the last raycast's wave records and prints
the wave-duration spread and how it relates to the skip lookups / batches.
usage: KFX_LIB_PATH=<trace lib> python3 tools/ray_trace.py [frames]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "slam-kinectfusion_amd"))
import kfx  # noqa: E402
from kfx import synth  # noqa: E402
from kfx.abi import Intrinsics, default_params  # noqa: E402

nfr = int(sys.argv[1]) if len(sys.argv) > 1 else 30
intr = synth.Intrinsics.vga()
params = default_params(dims=512, range_m=2.048)
bgr, dep, _ = synth.sequence(48, intr, L=2.048, noise=True, traj_seed=7, dropout=0.005)
order = synth.ping_pong(48, nfr)
kf = kfx.KinectFusion(Intrinsics.from_any(intr), params, device=0)
kf.set_graph_mode(False)
kf.set_frame_overlap(False)
kf.stage_frames(bgr, dep.astype(np.float32))
for i in order:
    kf.pipeline_staged(int(i))
kf.synchronize()
lib = kfx.lib()
buf = (C.c_uint64 * (8 * 65536))()
n = lib.kfx_debug_raycast_trace(buf, 65536)
a = np.frombuffer(buf, dtype=np.uint64)[: 8 * n].reshape(n, 8).astype(np.int64)
a = a[a[:, 1] > 0]
t0 = a[:, 0].min()
st, en = (a[:, 0] - t0) * 10, (a[:, 1] - t0) * 10  # ns
dur = en - st
lk, bt = a[:, 3] >> 32, a[:, 3] & 0xffffffff
print(f"waves {len(a)}  kernel span {en.max() / 1e3:.1f} us  start spread {st.max() / 1e3:.1f} us  wave dur us: min {dur.min() / 1e3:.1f} "
      f"med {np.median(dur) / 1e3:.1f} p90 {np.percentile(dur, 90) / 1e3:.1f} max {dur.max() / 1e3:.1f}")
for q in (10, 25, 50, 75, 90, 99, 100):
    print(f"  {q:3d}% of waves done by {np.percentile(en, q) / 1e3:7.1f} us")
print(f"max-lane lookups per wave: med {np.median(lk):.0f} p90 {np.percentile(lk, 90):.0f} max {lk.max()}")
print(f"max-lane batches per wave: med {np.median(bt):.0f} p90 {np.percentile(bt, 90):.0f} max {bt.max()}")
for name, x in (("lookups", lk), ("batches", bt)):
    c = np.corrcoef(x, dur)[0, 1]
    print(f"corr(dur, {name}) = {c:.2f}")
tm = (a[:, 4] - a[:, 0]) * 10
tn = np.where(a[:, 5] > 0, a[:, 5] - a[:, 4], a[:, 6] - a[:, 4]) * 10
tnd = np.where(a[:, 5] > 0, a[:, 6] - a[:, 5], 0) * 10
tend = (a[:, 1] - a[:, 6]) * 10
for name, x in (("setup", tm), ("march to first normal pass", tn), ("normal pass(es) + rest of loop", tnd), ("stores+resize", tend)):
    print(f"  phase {name:32s} us: med {np.median(x) / 1e3:6.2f} p90 {np.percentile(x, 90) / 1e3:6.2f} max {x.max() / 1e3:6.2f}")
h = np.stack([(a[:, 7] >> (16 * k)) & 0xffff for k in range(4)], 1)
tot = h.sum(1)
print("march-loop iterations per wave by live lanes (1 | 2-4 | 5-16 | 17-64): "
      f"all waves {h.sum(0).tolist()}")
slow20 = np.argsort(dur)[-max(1, len(a) // 50):]
print(f"  slowest 2% of waves: {h[slow20].sum(0).tolist()}  iterations med {np.median(tot[slow20]):.0f} max {tot.max()}")
print(f"  median waves: iterations med {np.median(tot):.0f}")
slow = np.argsort(dur)[-8:]
print("slowest waves: dur us / lookups / batches / live hist", [(round(dur[i] / 1e3, 1), int(lk[i]), int(bt[i]), h[i].tolist()) for i in slow])
try:
    ib = (C.c_uint64 * (34 * 65536))()
    ni = lib.kfx_debug_raycast_iters(ib, 65536)
    it = np.frombuffer(ib, dtype=np.uint64)[: 34 * ni].reshape(ni, 34).astype(np.int64)
    valid = np.frombuffer(buf, dtype=np.uint64)[: 8 * n].reshape(n, 8)[:, 1] > 0
    it = it[:n][valid]
    print("per-iteration records of the 8 slowest waves (lookup-phase us / batch-phase us / live / lookups / replayed max-lane samples):")
    for i in slow:
        k = int(it[i, 0])
        rows = []
        for j in range(min(k, 16)):
            a, b = int(it[i, 2 + 2 * j]), int(it[i, 3 + 2 * j])
            rows.append((round((a >> 32) / 2400, 2), round((a & 0xffffffff) / 2400, 2), b & 0xff, (b >> 8) & 0xff, b >> 16))
        tot = sum(((int(it[i, 2 + 2 * j]) >> 32) + (int(it[i, 2 + 2 * j]) & 0xffffffff)) for j in range(min(k, 16)))
        print(f"    (clock check: {tot} cycles over the march phase's {tn[i] / 1e3:.1f} us = {tot / max(tn[i], 1) * 1e3:.0f} MHz)")
        print(f"  wave {i}: dur {dur[i] / 1e3:.1f} us, setup {tm[i] / 1e3:.1f} us, {k} iterations:", rows)
    # all waves: mean cycles per lookup and per batch phase
    lk_c, bt_c, nlk = [], [], []
    for i in range(len(it)):
        for j in range(min(int(it[i, 0]), 16)):
            a, b = int(it[i, 2 + 2 * j]), int(it[i, 3 + 2 * j])
            nl = (b >> 8) & 0xff
            if nl:
                lk_c.append((a >> 32) / nl)
            bt_c.append(a & 0xffffffff)
    print(f"all waves: lookup round (per lookup) us med {np.median(lk_c) / 2400:.2f} p90 {np.percentile(lk_c, 90) / 2400:.2f};"
          f" batch phase us med {np.median(bt_c) / 2400:.2f} p90 {np.percentile(bt_c, 90) / 2400:.2f}")
except AttributeError:
    print("(library without kfx_debug_raycast_iters)")
kf.close()
