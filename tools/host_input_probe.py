#!/usr/bin/env python3
"""Where does the host-input path (kfx_pipeline_async) lose time against staged
frames?  C2 frames fed four ways, each timed over the same frame sequence:
  staged   kfx_pipeline_staged (device-resident input: the bench's `value` path)
  ring     kfx_pipeline_async from plain host memory (copy into the pinned ring)
  direct   kfx_pipeline_async from kfx_register_host_buffer'ed memory (no host copy)
Prints per-mode frames/s, ms/frame and the host time spent inside the calls.
usage: python3 tools/host_input_probe.py [--frames 200]"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-kinectfusion_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=25)
    a = ap.parse_args()
    import kfx
    from kfx import synth
    from kfx.abi import Intrinsics, default_params
    intr = synth.Intrinsics.vga()
    bgr, dep, _ = synth.sequence(48, intr)
    dep = dep.astype(np.float32)
    p = default_params(dims=512, range_m=2.048)
    kf = kfx.KinectFusion(Intrinsics.from_any(intr), p, device=0)
    kf.stage_frames(bgr, dep)
    order = synth.ping_pong(len(dep), a.warmup + 4 * a.frames)
    for i in range(a.warmup):
        kf.pipeline_staged(order[i])
    kf.synchronize()
    hb = np.ascontiguousarray(bgr)
    hd = np.ascontiguousarray(dep)
    res = {}
    pos = a.warmup

    def run(name, call):
        nonlocal pos
        kf.synchronize()
        seq = order[pos:pos + a.frames]
        pos += a.frames
        host = 0.0
        t0 = time.perf_counter()
        for i in seq:
            c0 = time.perf_counter()
            call(i)
            host += time.perf_counter() - c0
        st = kf.synchronize()
        dt = time.perf_counter() - t0
        res[name] = {"frames_per_s": round(len(seq) / dt, 1), "ms_per_frame": round(1e3 * dt / len(seq), 4),
                     "host_ms_in_calls_per_frame": round(1e3 * host / len(seq), 4), "status": st}
        print(name, res[name], flush=True)

    run("staged", lambda i: kf.pipeline_staged(i))
    run("ring", lambda i: kf.pipeline_async(hb[i], hd[i]))
    kf.register_host_buffer(hb)
    kf.register_host_buffer(hd)
    run("direct", lambda i: kf.pipeline_async(hb[i], hd[i]))
    run("staged_again", lambda i: kf.pipeline_staged(i))
    kf.unregister_host_buffer(hb)
    kf.unregister_host_buffer(hd)
    kf.close()


if __name__ == "__main__":
    main()
