#!/usr/bin/env python3
"""Per-wave timeline of k_integrate (debug library built with -DKFX_INT_TRACE):
runs the C2 bench workload for a few frames, dumps the last integrate's wave
records and prints the SIMD/CU occupancy over time and the wave-duration spread.
usage: KFX_LIB_PATH=<trace lib> python3 tools/int_trace.py [out.npy|-] [frames]"""
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "slam-kinectfusion_amd"))
import kfx  # noqa: E402
from kfx import synth  # noqa: E402
from kfx.abi import Intrinsics, default_params  # noqa: E402

intr = synth.Intrinsics.vga()
params = default_params(dims=512, range_m=2.048)
bgr, dep, _ = synth.sequence(48, intr, L=2.048, noise=True, traj_seed=7, dropout=0.005)
order = synth.ping_pong(48, int(sys.argv[2]) if len(sys.argv) > 2 else 200)
kf = kfx.KinectFusion(Intrinsics.from_any(intr), params, device=0)
kf.set_graph_mode(False)
kf.set_frame_overlap(False)
kf.stage_frames(bgr, dep.astype(np.float32))
for i in order:
    kf.pipeline_staged(int(i))
kf.synchronize()
lib = kfx.lib()
buf = (C.c_uint64 * (4 * 65536))()
n = lib.kfx_debug_integrate_trace(buf, 65536)
a = np.frombuffer(buf, dtype=np.uint64)[: 4 * n].reshape(n, 4).astype(np.int64)
launched = n
a = a[a[:, 1] > 0]
print(f"launched waves {launched}  with work {len(a)}  empty {launched - len(a)} "
      f"({(launched - len(a)) / max(launched, 1):.3f})")
t0 = a[:, 0].min()
st, en = (a[:, 0] - t0) * 10, (a[:, 1] - t0) * 10  # ns
dur = en - st
print(f"waves {len(a)}  kernel span {en.max() / 1e3:.1f} us  wave dur us: min {dur.min() / 1e3:.1f} "
      f"med {np.median(dur) / 1e3:.1f} p90 {np.percentile(dur, 90) / 1e3:.1f} max {dur.max() / 1e3:.1f}")
hw = a[:, 2] & 0xffffffff
cu = ((a[:, 2] >> 32) << 8) | ((hw >> 12) & 0xF) << 4 | ((hw >> 8) & 0xF)  # xcc, se, cu
simd = (cu << 2) | ((hw >> 4) & 3)
print("distinct SIMDs", len(np.unique(simd)), "CUs", len(np.unique(cu)))
# SIMD busy: last end per SIMD
last = {}
for s_, e in zip(simd, en):
    last[s_] = max(last.get(s_, 0), e)
le = np.array(list(last.values())) / 1e3
print(f"SIMD last-wave end us: min {le.min():.1f} p10 {np.percentile(le, 10):.1f} med {np.median(le):.1f} max {le.max():.1f}")
for q in (10, 25, 50, 75, 90, 100):
    t = np.percentile(en, q) / 1e3
    print(f"  {q:3d}% of waves done by {t:7.1f} us")
# resident waves over time (fraction of the 8192 slots of 8 waves x 1024 SIMDs)
span = en.max()
for k in range(20):
    t = span * (k + 0.5) / 20
    print(f"  t={t / 1e3:6.1f} us resident {((st <= t) & (en > t)).sum() / 8192:5.2f}")
print(f"wave-time / (span x 8192 slots) = {dur.sum() / (span * 8192):.3f}")
chunk = a[:, 3] >> 32
for c in np.unique(chunk):
    m = chunk == c
    print(f"  chunk {c}: waves {m.sum():5d} start med {np.median(st[m]) / 1e3:6.1f} dur med {np.median(dur[m]) / 1e3:6.1f} "
          f"p90 {np.percentile(dur[m], 90) / 1e3:6.1f} max {dur[m].max() / 1e3:6.1f} us; ends after 90% of span: "
          f"{(m & (en > 0.9 * span)).sum()}")
if len(sys.argv) > 1 and sys.argv[1] != "-":
    np.save(sys.argv[1], a)
kf.close()
