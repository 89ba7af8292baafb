#!/usr/bin/env python3
"""KinectFusion hot-path benchmark (BASELINE.json metric: frames/sec at
640x480, 512^3 TSDF; per-stage ms).

Workload (BASELINE config C2): synthetic 640x480 depth + BGR frames of the
analytic scene (kfx.synth), 512^3 TSDF @ 4 mm, 3-level ICP {10,5,4}.  A "step"
is one kf::kinectfusion::pipeline() frame: preprocess, 19 ICP iterations,
integrate, raycast, resize.  Frames are staged in HBM before the timed region
(kfx_stage_frames); every timed frame then runs the captured per-frame hipGraph
on its staged input.

Multi-GPU (`torchrun --nproc-per-node N`), one process per GPU:
  --mode replicas (default for N > 1): every rank runs an independent
      KinectFusion stream on its own camera trajectory (weak scaling, no
      collective on the data path); value = frames of all ranks / max wall time.
  --mode slab: ONE stream whose volume is Z-slab sharded over the N ranks
      (kfx_create_slab + RCCL combine; strong scaling); value =
      frames of the stream / max wall time.
  With --mode replicas and N > 1 the JSON line also carries "zslab": the same
  C2 stream Z-slab sharded over the N ranks, timed after the main measurement.

The JSON line also carries:
  stage_ms      per-stage device ms (HIP events on the pipeline stream)
  roofline      integrate kernel: algorithmic bytes (8*N_upd + 8*N_col + 7*W*H,
                SURVEY.md §8d; N counted on the device) / its event-timed
                duration vs 8 TB/s HBM; traffic = HBM bytes per launch from the
                committed rocprofv3 PMC summary (profiles/integrate_pmc.json)
  cpu_baseline  the serial C++ oracle running the same pipeline on host cores
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "slam-kinectfusion_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
REF_MS_PER_FRAME = 18.0  # README.md:8-9 (GTX 1650 Ti, 640x480, 512^3)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--dims", type=int, default=512)
    ap.add_argument("--range", type=float, default=2.048)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--height", type=int, default=480)
    ap.add_argument("--unique", type=int, default=48, help="distinct frames rendered (played ping-pong)")
    ap.add_argument("--profile-frames", type=int, default=20)
    ap.add_argument("--cpu-frames", type=int, default=8, help="oracle frames timed for cpu_baseline (0 = skip)")
    ap.add_argument("--host-frames", type=int, default=200,
                    help="frames fed from host memory through kfx_pipeline_async for host_input (0 = skip)")
    ap.add_argument("--c1-frames", type=int, default=100,
                    help="oracle frames of the C1 record (128^3, same frames; 0 = skip)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r02_integrate_pmc.json"),
                    help="integrate PMC traffic record; attached only when it was measured on this command's "
                         "workload and step counts")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--sample-every", type=int, default=8,
                    help="time kernels on every k-th timed frame with HIP events (0 = off)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="single-stream frames (no preprocess/ICP overlap across frames)")
    ap.add_argument("--mode", choices=["auto", "replicas", "slab"], default="auto")
    ap.add_argument("--zslab", type=int, default=1, help="with replicas at N>1: also time the Z-slab stream")
    ap.add_argument("--zslab-timeout", type=float, default=240.0)
    return ap.parse_args()


def intrinsics(w, h):
    from kfx import synth
    if (w, h) == (640, 480):
        return synth.Intrinsics.vga()
    if (w, h) == (1280, 720):
        return synth.Intrinsics.hd720()
    s = w / 640.0
    return synth.Intrinsics(w, h, 525.0 * s, 525.0 * s, (w - 1) / 2.0, (h - 1) / 2.0)


class pinned_to_one_core:
    """Run the serial CPU baseline on one host core (taskset -c <first allowed
    core> semantics for this process), restoring the affinity afterwards."""

    def __enter__(self):
        self.prev = os.sched_getaffinity(0)
        self.core = min(self.prev)
        os.sched_setaffinity(0, {self.core})
        return self

    def __exit__(self, *exc):
        os.sched_setaffinity(0, self.prev)


def cpu_baseline(intr, params, bgr, dep, order, n):
    """Serial oracle (TEST INFRASTRUCTURE, used here only as the reported CPU
    baseline) on a bounded sample, pinned to one core: the first frame of
    `order` bootstraps untimed, the next n are timed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    from kfx.abi import Intrinsics
    pipe = oracle.Pipeline(Intrinsics.from_any(intr), params)
    with pinned_to_one_core() as pin:
        pipe.process(bgr[order[0]], dep[order[0]].astype(np.float32))
        t0 = time.perf_counter()
        for k in order[1:n + 1]:
            assert pipe.process(bgr[k], dep[k].astype(np.float32)) == 0
        dt = time.perf_counter() - t0
    return {"value": round(n / dt, 4), "unit": "frames/s", "cores": 1, "kind": "port",
            "ms_per_frame": round(1000.0 * dt / n, 1),
            "sample": f"{n} frames after a bootstrap frame of the same synthetic sequence "
                      f"({intr.width}x{intr.height}, {params.volu_dims[0]}^3), full pipeline "
                      f"(preprocess+ICP+integrate+raycast), single thread pinned to core {pin.core}, "
                      f"oracle/kfx_oracle.cpp -O2",
            "host_cpus": os.cpu_count(), "cpu": _cpu_model()}


def raycast_roofline(work, ms, W, H, ms_source):
    """B_ray = 2 N_uniq + 24 W H, N_uniq = the distinct voxels
    the reference raycast (no skipping) reads, counted on the device on the
    last frame's state (kfx_raycast_stats, pinned against the oracle's count).
    The empty-space skipping kernel reads far fewer: `kernel_tsdf_reads`
    estimates its 2-B sample loads (14 per marched batch + the carried sample
    after each skip run + 48 normal corners per hit candidate)."""
    if not work or not work.get("ref_uniq_voxels") or not ms == ms:
        return None
    b = 2 * work["ref_uniq_voxels"] + 24 * W * H
    achieved = b / (ms * 1e-3) / 1e9
    return {"kernel": "k_raycast", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "algorithmic_bytes_per_launch": int(b), "avg_launch_ms": round(ms, 4), "launch_ms_source": ms_source,
            "ref_uniq_voxels": work["ref_uniq_voxels"], "ref_tsdf_reads": work["ref_reads"],
            "kernel_tsdf_reads": int(14 * work["batches"] + work["blocked_lookups"] + 48 * work["normal_candidates"])}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


class Dist:
    """torch.distributed wrapper (None-safe for the single-process case)."""

    def __init__(self, world, local):
        self.world = world
        self.dist = None
        if world > 1:
            import torch
            import torch.distributed as dist
            backend = "nccl" if torch.cuda.is_available() else "gloo"
            if backend == "nccl":
                torch.cuda.set_device(local)
            dist.init_process_group(backend=backend)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch
        dev = "cuda" if self.dist.get_backend() == "nccl" else "cpu"
        t = torch.tensor([x], dtype=torch.float64, device=dev)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def bcast_bytes(self, b: bytes | None, src: int = 0) -> bytes:
        if self.dist is None:
            return b
        obj = [b]
        self.dist.broadcast_object_list(obj, src=src)
        return obj[0]

    def close(self):
        if self.dist is not None:
            self.dist.destroy_process_group()


def timed_frames(kf, order, lo, hi, D):
    """W/K contract: barrier + device sync on both sides, max over ranks; a
    frame dropped by a tracking failure fails the run."""
    import kfx
    kf.synchronize()
    D.barrier()
    t0 = time.perf_counter()
    for i in range(lo, hi):
        kf.pipeline_staged(order[i])
    st = kf.synchronize()
    elapsed = time.perf_counter() - t0
    if st != kfx.KFX_OK:
        raise SystemExit("bench: a timed frame lost tracking (KFX_TRACKING_LOST)")
    elapsed = D.max(elapsed)
    D.barrier()
    return elapsed


def zslab_stream(a, intr, params, D, rank, world, local):
    """One C2 stream Z-slab sharded over the ranks (RCCL combine); frames/s."""
    import kfx
    from kfx import synth
    from kfx.abi import Intrinsics
    bgr, dep, _ = synth.sequence(a.unique, intr, L=a.range, noise=True, traj_seed=7, dropout=0.005)
    order = synth.ping_pong(a.unique, a.warmup + a.steps)
    kf = kfx.KinectFusion(Intrinsics.from_any(intr), params, device=local, slab=(rank, world))
    uid = D.bcast_bytes(kfx.comm_unique_id() if rank == 0 else None)
    kf.comm_init(uid)
    kf.set_graph_mode(not a.no_graph)
    kf.set_frame_overlap(not a.no_overlap)
    kf.stage_frames(bgr, dep.astype(np.float32))
    for i in range(a.warmup):
        kf.pipeline_staged(order[i])
    elapsed = timed_frames(kf, order, a.warmup, a.warmup + a.steps, D)
    poses = kf.pose_record.shape[0]
    zb, zn, o0, o1 = kf.slab_info()
    kf.close()
    return {"value": round(a.steps / elapsed, 3), "unit": "frames/s", "scaling": "strong",
            "ms_per_step": round(1000.0 * elapsed / a.steps, 4), "n_gpus": world,
            "slab_slices": o1 - o0, "stored_slices": zn, "poses": int(poses),
            "note": "one C2 stream, volume Z-slab sharded over the ranks, raycast combined by "
                    "RCCL all-reduce MIN(key)+MAX(bits) per frame, ICP replicated"}


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    D = Dist(world, local)
    mode = a.mode if a.mode != "auto" else ("replicas" if world > 1 else "single")

    import kfx
    from kfx import synth
    from kfx.abi import Intrinsics, default_params

    intr = intrinsics(a.width, a.height)
    params = default_params(dims=a.dims, range_m=a.range)
    W, H = intr.width, intr.height
    slab_main = mode == "slab"
    seed = 7 if (slab_main or world == 1) else 7 + rank
    bgr, dep, gt = synth.sequence(a.unique, intr, L=a.range, noise=True, traj_seed=seed, dropout=0.005)
    order = synth.ping_pong(a.unique, a.warmup + a.steps + a.profile_frames)

    if slab_main:
        kf = kfx.KinectFusion(Intrinsics.from_any(intr), params, device=local, slab=(rank, world))
        kf.comm_init(D.bcast_bytes(kfx.comm_unique_id() if rank == 0 else None))
    else:
        kf = kfx.KinectFusion(Intrinsics.from_any(intr), params, device=local)
    kf.set_graph_mode(not a.no_graph)
    kf.set_frame_overlap(not a.no_overlap)
    kf.stage_frames(bgr, dep.astype(np.float32))

    for i in range(a.warmup):
        kf.pipeline_staged(order[i])
    kf.synchronize()
    n_before = kf.pose_record.shape[0]
    # kernel durations over the timed region: every 8th frame bracketed by HIP
    # events on the stream the kernels run on
    if a.sample_every > 0:
        kf.set_kernel_timing(a.sample_every, a.steps // a.sample_every + 2)
    elapsed = timed_frames(kf, order, a.warmup, a.warmup + a.steps, D)
    ktime = kf.kernel_timing() if a.sample_every > 0 else None
    kf.set_kernel_timing(0)
    tracked = kf.pose_record.shape[0] - n_before  # frames that appended a pose
    if tracked != a.steps:  # a dropped frame (tracking reset) invalidates the measurement
        raise SystemExit(f"bench: {a.steps - tracked} of {a.steps} timed frames were not tracked")

    # host-input throughput (not `value`): the same frames from host memory
    # through kfx_pipeline_async (pinned ring, H2D overlapped with the previous
    # frame), PCIe included, f32 depth as the reference's pipeline() takes it
    host_in = None
    if a.host_frames > 0:
        hb = [np.ascontiguousarray(bgr[i]) for i in range(a.unique)]
        hd = [np.ascontiguousarray(dep[i].astype(np.float32)) for i in range(a.unique)]
        ho = synth.ping_pong(a.unique, a.host_frames)
        kf.synchronize()
        D.barrier()
        t0 = time.perf_counter()
        for i in ho:
            kf.pipeline_async(hb[i], hd[i])
        st_h = kf.synchronize()
        dt_h = D.max(time.perf_counter() - t0)
        host_in = {"value": round(len(ho) * (world if not slab_main else 1) / dt_h, 3), "unit": "frames/s",
                   "ms_per_step": round(1000.0 * dt_h / len(ho), 4), "frames": len(ho),
                   "status": "ok" if st_h == kfx.KFX_OK else "tracking lost",
                   "bytes_per_frame_h2d": W * H * 7,
                   "path": "kfx_pipeline_async: host frame -> pinned 4-slot ring -> H2D on a copy stream "
                           "overlapped with the previous frame; f32 depth mm + BGR8"}

    # per-stage device ms + integrate roofline on further frames (profiled, eager)
    kf.set_profiling(True)
    stages = {k: [] for k in ("preprocess", "icp", "integrate", "raycast", "total")}
    int_bytes, int_ms, int_work = [], [], []
    for i in range(a.warmup + a.steps, a.warmup + a.steps + a.profile_frames):
        kf.pipeline_staged(order[i])
        ms = kf.stage_ms()
        for k in stages:
            stages[k].append(ms[k])
        wk = kf.integrate_stats()
        nu, nc = wk["updated"], wk["colored"]
        int_work.append(wk)
        int_bytes.append(8 * nu + 8 * nc + 7 * W * H)
        int_ms.append(ms["integrate"])
    kf.set_profiling(False)
    ray_work = kf.raycast_stats() if a.profile_frames else None
    kf.synchronize()
    kf.close()
    ray_ms = float(ktime["raycast"]) if ktime and ktime["samples"] > 0 else (
        float(statistics.median(stages["raycast"])) if stages["raycast"] else float("nan"))
    stage_med = {k: round(statistics.median(v), 4) for k, v in stages.items()} if a.profile_frames else {}
    avg_bytes = float(np.mean(int_bytes)) if int_bytes else 0.0
    # the integrate launch duration of the roofline: the HIP-event samples of
    # the timed region (fallback: the profiled frames after it)
    if ktime and ktime["samples"] > 0:
        avg_ms, ms_source = float(ktime["integrate"]), f"timed region, {ktime['samples']} event-bracketed frames"
    else:
        avg_ms, ms_source = (float(np.mean(int_ms)) if int_ms else float("nan")), "profiled frames"
    achieved = avg_bytes / (avg_ms * 1e-3) / 1e9 if avg_ms == avg_ms else 0.0
    # HBM traffic of the integrate launch from a rocprofv3 FETCH_SIZE/WRITE_SIZE
    # record (tools/prof.sh), attached only when that record was measured on
    # this workload with the same step counts (the same saturation regime)
    traffic, traffic_src = None, "none: no PMC record of this workload and step count"
    try:
        rec = json.load(open(a.traffic))
        if (not slab_main and rec.get("workload") == [a.dims, W, H] and rec.get("steps") == a.steps
                and rec.get("warmup") == a.warmup):
            traffic = rec.get("hbm_bytes_per_launch")
            traffic_src = f"{os.path.relpath(a.traffic, ROOT)}: {rec.get('command')} ({rec.get('regime')})"
    except (OSError, ValueError):
        pass

    cpu = c1 = None
    if rank == 0 and world == 1 and a.cpu_frames > 0:
        cpu = cpu_baseline(intr, params, bgr, dep, synth.ping_pong(a.unique, a.cpu_frames + 1), a.cpu_frames)
    if rank == 0 and world == 1 and a.c1_frames > 0 and (W, H) == (640, 480):
        # BASELINE C1: 128^3 TSDF (16 mm) on the same 640x480 frames, serial oracle
        c1 = cpu_baseline(intr, default_params(dims=128, range_m=a.range), bgr, dep,
                          synth.ping_pong(a.unique, a.c1_frames + 1), a.c1_frames)
        c1["config"] = "C1: 128^3 TSDF @ 16 mm, 640x480 synthetic frames (the bundled dataset is absent)"

    frames = a.steps if slab_main else a.steps * world
    value = frames / elapsed
    out = {
        "metric": "frames/sec at 640×480, 512³ TSDF; per-stage ms (ICP/integrate/raycast)",
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1000.0 * elapsed / a.steps, 4),
        "higher_is_better": True,
        "scaling": "strong" if slab_main else "weak",
        "vs_baseline": round(value / (1000.0 / REF_MS_PER_FRAME), 3),
        "dtype": "f32",
        "data": "synthetic",
        "config": {
            "workload": f"C2: synthetic {W}x{H} depth+BGR, {a.dims}^3 TSDF @ "
                        f"{1000 * a.range / a.dims:.1f} mm, 3-level ICP {{10,5,4}}, full pipeline per frame",
            "width": W, "height": H, "volume_dims": a.dims, "volume_range_m": a.range,
            "frames_unique": a.unique, "graph": not a.no_graph, "overlap": not a.no_overlap,
            "parallelism": (f"zslab x{world}" if slab_main else
                            (f"replicas x{world} (independent streams)" if world > 1 else "single")),
            "tracked_frames": int(tracked),
            "reference_ms_per_frame": REF_MS_PER_FRAME,
        },
        "stage_ms": stage_med,
        "timed_region_kernel_ms": ({k: round(v, 4) if isinstance(v, float) else v for k, v in ktime.items()}
                                   if ktime else None),
        "integrate_voxels": ({k: int(np.mean([w[k] for w in int_work])) for k in int_work[0]}
                             if int_work else None),
        "raycast_work": ray_work,
        "roofline": {
            "kernel": "k_integrate",
            "bound": "hbm",
            "achieved": round(achieved, 1),
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": traffic,
            "traffic_source": traffic_src,
            "algorithmic_bytes_per_launch": int(avg_bytes),
            "avg_launch_ms": round(avg_ms, 4),
            "launch_ms_source": ms_source,
        },
        "roofline_raycast": raycast_roofline(ray_work, ray_ms, W, H, ms_source),
        "host_input": host_in,
        "cpu_baseline": cpu,
        "c1_record": c1,
    }

    if mode == "replicas" and a.zslab:
        # the main measurement is complete: a failure or hang in the Z-slab
        # side measurement must not lose it
        lock = threading.Lock()
        printed = []

        def emit(extra):
            with lock:
                if printed:
                    return
                printed.append(1)
                if rank == 0:
                    out["zslab"] = extra
                    print(json.dumps(out), flush=True)

        def on_timeout():
            emit({"error": f"timed out after {a.zslab_timeout:.0f} s"})
            os._exit(0)

        timer = threading.Timer(a.zslab_timeout, on_timeout)
        timer.daemon = True
        timer.start()
        try:
            extra = zslab_stream(a, intr, params, D, rank, world, local)
        except Exception as e:  # noqa: BLE001 — reported in the JSON line
            extra = {"error": f"{type(e).__name__}: {e}"[:300]}
        timer.cancel()
        emit(extra)
    elif rank == 0:
        print(json.dumps(out), flush=True)
    D.close()


if __name__ == "__main__":
    main()
