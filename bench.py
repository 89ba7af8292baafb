#!/usr/bin/env python3
"""KinectFusion hot-path benchmark (BASELINE.json metric: frames/sec at
640x480, 512^3 TSDF; per-stage ms).

Workload (BASELINE config C2): synthetic 640x480 depth + BGR frames of the
analytic scene (kfx.synth), 512^3 TSDF @ 4 mm, 3-level ICP {10,5,4}.  A "step"
is one kf::kinectfusion::pipeline() frame: preprocess, 19 ICP iterations,
integrate, raycast, resize.  Frames are staged in HBM before the timed region
(kfx_stage_frames); every timed frame then runs the captured per-frame hipGraph
on its staged input.

Configs (BASELINE.json configs[1..4], --config): c2 640x480 512^3 @ 4 mm (the
metric's config, default at N=1), c3 1024^3 @ 2 mm single GPU (recorded beside
the C2 line at N=1 as "c3_record"), c4 1024^3 @ 2 mm Z-slab sharded over the N
GPUs (default at N>1), c5 1280x720 2048^3 @ 2 mm.

Multi-GPU (`torchrun --nproc-per-node N`), one process per GPU:
  --mode slab (default for N > 1): ONE stream whose volume is Z-slab sharded
      over the N ranks (kfx_create_slab + RCCL combine; strong
      scaling); value = frames of the stream / max wall time; "per_rank" holds
      every rank's ICP / integrate / raycast / combine ms.  --icp allreduce
      shards the ICP sums too.  Independent replica streams are timed first
      ("replicas"); if the slab stream fails or hangs, they become the line.
  --mode replicas: every rank runs an independent stream (weak scaling, no
      collective on the data path); value = frames of all ranks / max time.

The JSON line also carries:
  stage_ms      per-stage device ms (HIP events on the pipeline stream)
  roofline      integrate kernel: algorithmic bytes (6*N_upd + 8*N_col + 7*W*H:
                SURVEY.md §8d with the u8 weight store; N counted on the device) / its event-timed
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
    ap.add_argument("--config", choices=["auto", "c2", "c3", "c4", "c5"], default="auto",
                    help="BASELINE config (auto: c2 at N=1, c4 at N>1)")
    ap.add_argument("--dims", type=int, default=None, help="override the config's volume dims")
    ap.add_argument("--range", type=float, default=None, help="override the config's volume range (m)")
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--unique", type=int, default=0,
                    help="distinct frames rendered, played ping-pong (0: 48, 16 above 640x480)")
    ap.add_argument("--profile-frames", type=int, default=20)
    ap.add_argument("--cpu-frames", type=int, default=8, help="oracle frames timed for cpu_baseline (0 = skip)")
    ap.add_argument("--host-frames", type=int, default=200,
                    help="frames fed from host memory through kfx_pipeline_async for host_input (0 = skip)")
    ap.add_argument("--c1-frames", type=int, default=100,
                    help="oracle frames of the C1 record (128^3, same frames; 0 = skip)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "r06_integrate_pmc.json"),
                    help="integrate PMC traffic record; attached only when it was measured on this command's "
                         "workload and step counts with the same libkfx.so (sha256)")
    ap.add_argument("--traffic-c3", default=os.path.join(ROOT, "profiles", "r06_c3_pmc.json"),
                    help="PMC record of the C3 workload (attached to c3_record under the same rule)")
    ap.add_argument("--traffic-c5", default=os.path.join(ROOT, "profiles", "r06_c5_pmc.json"),
                    help="PMC record of the C5 single-volume workload (attached to c5_record under the same rule)")
    ap.add_argument("--graph", choices=["auto", "0", "1", "2"], default="auto",
                    help="kfx_set_graph_mode of the timed frames: 0 eager, 1 the pyrDown+preprocess graph, 2 also "
                         "ICP+integrate+raycast (+RCCL combine) as a graph; auto: 2 for C5 (BASELINE names a "
                         "hipGraph-captured per-frame pipeline there), 1 otherwise")
    ap.add_argument("--no-graph", action="store_true", help="= --graph 0")
    ap.add_argument("--graph-full", action="store_true", help="= --graph 2")
    ap.add_argument("--sample-every", type=int, default=8,
                    help="time kernels on every k-th timed frame with HIP events (0 = off)")
    ap.add_argument("--no-overlap", action="store_true",
                    help="single-stream frames (no preprocess/ICP overlap across frames)")
    ap.add_argument("--mode", choices=["auto", "single", "replicas", "slab"], default="auto",
                    help="auto: single at N=1, slab at N>1")
    ap.add_argument("--icp", choices=["replicated", "allreduce"], default="replicated",
                    help="slab mode: every rank runs the full ICP, or its band with the partials all-reduced")
    ap.add_argument("--zslab", choices=["none", "c2", "c4", "c5"], default="c5",
                    help="N>1 with the replica line: also time ONE stream of this config Z-slab sharded over "
                         "the N GPUs (strong scaling, RCCL combine) as the `zslab` record; default c5, the "
                         "2048^3 volume north_star's integrate-scaling claim is about")
    ap.add_argument("--replicas", type=int, default=1,
                    help="slab mode at N>1: time independent replica streams first (the fallback line)")
    ap.add_argument("--zslab-timeout", type=float, default=300.0)
    ap.add_argument("--cuts", choices=["balanced", "first", "equal"], default="balanced",
                    help="slab mode: Z-slab cuts balanced on the mean per-slice work of 4 frames of the timed "
                         "run at their poses, on the first frame's alone, or equal slice ranges")
    ap.add_argument("--extract", type=int, default=1,
                    help="N=1: time point extraction and marching cubes on the final volume (0 = skip)")
    ap.add_argument("--c3-frames", type=int, default=20,
                    help="N=1, C2: timed frames of the C3 record (1024^3 @ 2 mm, same frames; 0 = skip)")
    ap.add_argument("--c5-frames", type=int, default=10,
                    help="N=1, C2: timed frames of the C5 single-volume record (1280x720, 2048^3 @ 2 mm: the "
                         "N=1 point of the zslab curve; 0 = skip)")
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


def raycast_roofline(work, ms, W, H, ms_source, traffic=None, traffic_src=None):
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
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": traffic_src or "none: no PMC record of this workload and step count",
            "algorithmic_bytes_per_launch": int(b), "avg_launch_ms": round(ms, 4), "launch_ms_source": ms_source,
            "ref_uniq_voxels": work["ref_uniq_voxels"], "ref_tsdf_reads": work["ref_reads"],
            "kernel_tsdf_reads": int(14 * work["batches"] + work["blocked_lookups"] + 48 * work["normal_candidates"])}


def file_sha256(path):
    import hashlib
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    except OSError:
        return None


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

    def gather(self, row):
        """Every rank's list of floats, in rank order (on every rank)."""
        if self.dist is None:
            return [list(row)]
        import torch
        dev = "cuda" if self.dist.get_backend() == "nccl" else "cpu"
        t = torch.zeros(self.world, len(row), dtype=torch.float64, device=dev)
        t[self.dist.get_rank()] = torch.tensor(row, dtype=torch.float64, device=dev)
        self.dist.all_reduce(t)
        return t.cpu().tolist()

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


CONFIGS = {  # BASELINE.json configs[1..4]: (width, height, volume dims, volume range m)
    "c2": (640, 480, 512, 2.048),
    "c3": (640, 480, 1024, 2.048),
    "c4": (640, 480, 1024, 2.048),
    "c5": (1280, 720, 2048, 4.096),
}


def graph_mode(a, cfg):
    """kfx_set_graph_mode for a stream of config cfg (--graph; auto: 2 for C5,
    whose BASELINE config names a hipGraph-captured per-frame pipeline)."""
    if a.no_graph:
        return 0
    if a.graph_full:
        return 2
    if a.graph != "auto":
        return int(a.graph)
    return 2 if cfg == "c5" else 1


def graph_parts(a, mode, effective=None, requested=1):
    """The part of each timed frame replayed as a captured graph (effective:
    kfx_get_graph_mode after the run, lowered where RCCL refused capture)."""
    if requested == 0 or effective == 0:
        return "none (eager)"
    if a.no_overlap:
        return "whole frame (single stream)"
    main = "ICP+integrate+raycast" + ("+RCCL combine" if mode == "slab" else "")
    if requested == 2 and effective in (None, 2):
        return f"pyrDown+preprocess graph and {main} graph (mode 2)"
    return f"pyrDown+preprocess graph; {main} eager (mode 1)" + (
        " (mode 2 requested: capture refused, fell back)" if requested == 2 else "")


def resolve(a, world):
    """Config and mode.  The line's workload is the metric's config (C2) at every
    N: one stream at N=1, N independent C2 streams (one per GPU, weak scaling)
    at N>1, so the per-N values form one curve; the Z-slab sharded stream (C4 by
    default, `--zslab`) is timed beside it as the `zslab` record.  An explicit
    --config c4 / c5 at N>1 makes the Z-slab stream itself the line."""
    name = a.config if a.config != "auto" else "c2"
    W, H, n, L = CONFIGS[name]
    over = [a.width, a.height, a.dims, a.range]
    if any(v is not None for v in over):
        W, H, n, L = [v if v is not None else d for v, d in zip(over, (W, H, n, L))]
        name = "custom" if (W, H, n, L) != CONFIGS[name] else name
    if a.mode != "auto":
        mode = a.mode
    elif world == 1:
        mode = "single"
    else:
        mode = "slab" if a.config in ("c4", "c5") else "replicas"
    return name, W, H, n, L, mode


CUTS_TEXT = {"balanced": "cuts balanced on the mean per-slice integrate work of 4 frames of the run at their poses",
             "first": "cuts balanced on the first frame's per-slice integrate work",
             "equal": "equal slice ranges"}


def workload_text(name, W, H, n, L, mode, world, icp_ar, cuts="balanced"):
    t = (f"{name.upper()}: synthetic {W}x{H} depth+BGR, {n}^3 TSDF @ {1000 * L / n:.1f} mm, "
         f"3-level ICP {{10,5,4}}, full pipeline per frame")
    if mode == "slab":
        t += (f"; one stream, volume Z-slab sharded over {world} GPUs ("
              f"{CUTS_TEXT[cuts]}), raycast combined per frame by RCCL "
              f"(MIN keys + MAX {{Ts, normal}} payload), ICP " + ("sharded (27 int64 partials all-reduced per "
                                                                   "iteration)" if icp_ar else "replicated"))
    elif mode == "replicas":
        t += f"; {world} independent streams, one per GPU (no collective)"
    return t


def run_stream(a, intr, params, frames, D, local, slab=None, icp_ar=False, timing=True, gmode=1):
    """Create a context, warm up, time a.steps staged frames (W/K contract).
    Returns the open context and the timed-region record; the caller closes it.
    gmode: kfx_set_graph_mode of the timed frames (graph_mode)."""
    import kfx
    from kfx.abi import Intrinsics
    bgr, dep, order, gt = frames  # gt: the trajectory's poses (slab cut calibration), or None
    cuts = None
    if slab is not None and a.cuts != "equal":
        if a.cuts == "first" or gt is None:
            calib = [order[0]]
        else:  # 4 frames spread over the timed run's distinct frames
            seen = sorted(set(order[a.warmup:a.warmup + a.steps]))
            calib = [seen[int(round(j * (len(seen) - 1) / 3))] for j in range(4)]
        cuts = balanced_cuts(intr, params, [(bgr[i], dep[i], None if gt is None else gt[i]) for i in calib], local,
                             slab[1])
    kf = kfx.KinectFusion(Intrinsics.from_any(intr), params, device=local, slab=slab, cuts=cuts)
    if slab is not None:
        kf.comm_init(D.bcast_bytes(kfx.comm_unique_id() if slab[0] == 0 else None))
        kf.set_icp_allreduce(icp_ar)
    kf.set_graph_mode(gmode)
    kf.set_frame_overlap(not a.no_overlap)
    kf.stage_frames(bgr, dep)
    for i in range(a.warmup):
        kf.pipeline_staged(order[i])
    kf.synchronize()
    n_before = kf.pose_record.shape[0]
    # kernel durations over the timed region: every k-th frame bracketed by HIP
    # events on the stream the kernels run on
    if timing and a.sample_every > 0:
        kf.set_kernel_timing(a.sample_every, a.steps // a.sample_every + 2)
    elapsed = timed_frames(kf, order, a.warmup, a.warmup + a.steps, D)
    ktime = kf.kernel_timing() if timing and a.sample_every > 0 else None
    kf.set_kernel_timing(0)
    tracked = kf.pose_record.shape[0] - n_before  # frames that appended a pose
    if tracked != a.steps:  # a dropped frame (tracking reset) invalidates the measurement
        raise SystemExit(f"bench: {a.steps - tracked} of {a.steps} timed frames were not tracked")
    if ktime is not None and not ktime["samples"]:
        ktime = None
    note = kf.graph_note() if hasattr(kf, "graph_note") else ""
    return kf, {"elapsed": elapsed, "ktime": ktime, "tracked": tracked, "graph_mode": kf.graph_mode(),
                "graph_requested": gmode, "graph_note": note}


def balanced_cuts(intr, params, calib, local, world):
    """Work-balanced Z-slab cuts: the mean per-slice integrate work of the
    calibration frames [(bgr, depth, camera pose)] (kfx_slice_work_at on a
    throw-away 16-slice slab context), then kfx_slab_balance.  Every rank
    computes the same cuts from the same frames.  The poses are the synthetic
    trajectory's (a live system would use its tracked poses)."""
    import kfx
    from kfx.abi import Intrinsics
    Z = int(params.volu_dims[2])
    probe = kfx.KinectFusion(Intrinsics.from_any(intr), params, device=local, slab=(0, Z // 16))
    work = np.mean([probe.slice_work_at(b, d, g)[0] for b, d, g in calib], axis=0).round().astype(np.int64)
    probe.close()
    return kfx.slab_balance(work, world)


def integrate_roofline(work, ms, W, H, ms_source, traffic=None, traffic_src=None):
    """SURVEY.md §8d's B_int = 8 N_upd + 8 N_col + 7 W H (N counted on the device)
    with the per-updated-voxel term of THIS storage format: int16 tsdf + u8 weight
    read and written = 6 B (the reference's int16 weight makes it 8 B;
    `achieved_ref_format` is the same time priced at the survey's 8 B)."""
    b = 6 * work["updated"] + 8 * work["colored"] + 7 * W * H
    b_ref = 8 * work["updated"] + 8 * work["colored"] + 7 * W * H
    ok = ms == ms and ms > 0
    achieved = b / (ms * 1e-3) / 1e9 if ok else 0.0
    achieved_ref = b_ref / (ms * 1e-3) / 1e9 if ok else 0.0
    return {"kernel": "k_integrate", "bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "traffic_source": traffic_src or "none: no PMC record of this workload and step count",
            "algorithmic_bytes_per_launch": int(b), "bytes_formula": "6*N_upd + 8*N_col + 7*W*H (u8 weight store)",
            "achieved_ref_format": round(achieved_ref, 1), "avg_launch_ms": round(ms, 4), "launch_ms_source": ms_source}


def extract_record(kf, n):
    """Surface extraction off the per-frame path (C5 names the
    marching-cubes extract): kfx_extract_points (FullScan6 zero crossings,
    tsdf_volume.cu:307-481) and kfx_extract_mesh on the volume the timed frames
    built; device ms of the volume pass, the offset scan and the pool copy
    (passes = 1: the volume is read once) or the emit pass (passes = 2), HIP
    events.  Roofline on the reference's bytes: its FullScan6 reads every
    voxel's int16 tsdf + u8 weight once (3 B; neighbours come from cache) and
    writes 12 B per point (36 B per triangle for the mesh).  The kernels skip
    the waves whose brick the occupancy map proves empty, so `achieved` is the
    full-scan-equivalent rate."""
    vox = n * n * (n - 1)  # z = 0 .. Z-2 (the +z neighbour must exist)
    out = {"voxels_scanned": vox, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "bytes_basis": "one full-volume pass of 3 B/voxel + the outputs (the reference's FullScan6); "
                          "clear bricks are skipped, so achieved is the full-scan-equivalent rate"}
    for name, fn, per in (("points", kf.extract_points, 12), ("mesh", kf.extract_mesh, 36)):
        items = fn(cap=50_000_000)
        ms = kf.extract_ms()
        b = 3 * vox + per * len(items)
        t = ms["count"] + ms["scan"] + ms["emit"]
        out[name] = {"items": int(len(items)), "passes": ms["passes"], "count_ms": round(ms["count"], 4),
                     "scan_ms": round(ms["scan"], 4), "copy_or_emit_ms": round(ms["emit"], 4),
                     "total_ms": round(t, 4), "algorithmic_bytes": int(b),
                     "achieved": round(b / (t * 1e-3) / 1e9, 1) if t > 0 else None,
                     "frac": round(b / (t * 1e-3) / 1e9 / HBM_PEAK_GBS, 4) if t > 0 else None}
        del items
    return out


def round_ms(d):
    return {k: round(v, 4) if isinstance(v, float) else v for k, v in d.items()} if d else None


def pmc_record(path, workload, steps, warmup, lib_hash):
    """A committed rocprofv3 PMC record (tools/prof.sh + tools/traffic.py
    --commit) for this workload [dims, W, H] and step counts, measured on this
    very library (sha256): (traffic bytes per integrate launch, raycast bytes,
    SQ issue records, source text), or Nones with the reason."""
    try:
        rec = json.load(open(path))
    except (OSError, ValueError):
        return None, None, None, None
    same_run = (rec.get("workload") == list(workload) and rec.get("steps") == steps and rec.get("warmup") == warmup)
    rel = os.path.relpath(path, ROOT)
    if same_run and rec.get("lib_sha256") == lib_hash:
        sq = {"integrate": rec.get("integrate_sq"), "raycast": rec.get("raycast_sq")}
        src = (f"{rel}: {rec.get('command')} ({rec.get('regime')}); "
               f"libkfx.so sha256 {lib_hash[:16]} (commit {rec.get('commit')})")
        return rec.get("hbm_bytes_per_launch"), rec.get("raycast_hbm_bytes_per_launch"), sq, src
    if same_run:
        return None, None, None, (f"none: {rel} was measured on libkfx.so sha256 {str(rec.get('lib_sha256'))[:16]}, "
                                  f"this run loaded {str(lib_hash)[:16]}")
    return None, None, None, None


def issue_figures(sq, kernel):
    q = (sq or {}).get(kernel)
    if not q:
        return None
    # valu_busy_frac_bounds: VALU issue cycles / SIMD-cycles, bracketed by the
    # calibration of SQ_INSTS_VALU / SQ_ACTIVE_INST_VALU (tools/traffic.py
    # sq_issue, profiles/r06_valu_calib.json); records measured before it carry
    # none (their valu_active_frac is not a fraction of the SIMD's cycles)
    return {k: q.get(k) for k in ("valu_issue_frac_2cyc", "valu_busy_frac_bounds", "valu_insts_per_wave",
                                  "wave_cycles_split", "kernel_cycles") if k in q}


def single_record(a, name, intr, n, L, frames, D, local, traffic_path=None):
    """A side measurement of one more single-GPU config (C3 / C5 at N=1):
    frames/s over the same W/K contract, kernel ms, integrate roofline (with
    the PMC traffic of a committed record of this workload and library)."""
    import kfx
    from kfx.abi import default_params
    params = default_params(dims=n, range_m=L)
    gm = graph_mode(a, name)
    kf, r = run_stream(a, intr, params, frames, D, local, gmode=gm)
    wk = kf.integrate_stats()
    kf.close()
    kt = r["ktime"]
    W, H = intr.width, intr.height
    lib_hash = file_sha256(kfx.LIB_PATH)
    traffic, _, sq, src = pmc_record(traffic_path, [n, W, H], a.steps, a.warmup, lib_hash) if traffic_path else (
        None, None, None, None)
    roof = integrate_roofline(wk, kt["integrate"] if kt else float("nan"), W, H,
                              "timed region, HIP-event-bracketed frames", traffic, src)
    roof["lib_sha256"] = lib_hash
    if issue_figures(sq, "integrate"):
        roof["issue"] = issue_figures(sq, "integrate")
    return {"config": workload_text(name, W, H, n, L, "single", 1, False),
            "graph": graph_parts(a, "single", r["graph_mode"], r["graph_requested"]),
            "value": round(a.steps / r["elapsed"], 3), "unit": "frames/s",
            "ms_per_step": round(1000.0 * r["elapsed"] / a.steps, 4), "steps": a.steps, "warmup": a.warmup,
            "tracked_frames": r["tracked"], "timed_region_kernel_ms": round_ms(kt), "integrate_voxels": wk,
            "roofline": roof}


def main():
    a = parse()
    # stdout carries only the JSON line: library banners (RCCL prints its
    # version there) and any other output go to stderr
    json_fd = os.dup(1)
    sys.stdout.flush()
    os.dup2(2, 1)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    D = Dist(world, local)
    name, W, H, n, L, mode = resolve(a, world)
    icp_ar = a.icp == "allreduce"

    import kfx
    from kfx import synth
    from kfx.abi import default_params

    intr = intrinsics(W, H)
    params = default_params(dims=n, range_m=L)
    unique = a.unique if a.unique else (16 if W * H > 640 * 480 else 48)
    # one camera trajectory for every rank: the slab ranks share one stream, and
    # replica streams are independent whatever frames they replay
    bgr, dep, gt = synth.sequence(unique, intr, L=L, noise=True, traj_seed=7, dropout=0.005)
    dep = dep.astype(np.float32)
    order = synth.ping_pong(unique, a.warmup + a.steps + a.profile_frames)
    frames = (bgr, dep, order, gt)

    # N>1: the replica streams first (no collective), so that a failing or hung
    # Z-slab stream still leaves a measured line
    replicas = None
    if mode == "slab" and world > 1 and a.replicas:
        kf, r = run_stream(a, intr, params, frames, D, local, timing=False, gmode=graph_mode(a, name))
        kf.close()
        replicas = {"value": round(a.steps * world / r["elapsed"], 3), "unit": "frames/s", "scaling": "weak",
                    "ms_per_step": round(1000.0 * r["elapsed"] / a.steps, 4),
                    "config": workload_text(name, W, H, n, L, "replicas", world, False)}

    lock = threading.Lock()
    printed = []

    def emit(line, extra=None):
        """Print the line once; `extra` is merged into a copy taken under the lock
        (a watchdog thread never changes the main thread's dict)."""
        with lock:
            if printed:
                return
            printed.append(1)
            if extra:
                line = dict(line, **extra)
            if rank == 0:
                os.write(json_fd, (json.dumps(line) + "\n").encode())

    def fallback(err):
        """The replicas measurement as the line, the slab failure recorded."""
        line = base_line(a, world, replicas["value"], float(replicas["ms_per_step"]), "weak",
                         {"workload": replicas["config"], "parallelism": f"replicas x{world}"})
        line["zslab"] = {"error": err}
        return line

    timer = None
    if replicas is not None:
        def on_timeout():  # the line is printed, but a hang is a failure: exit 3
            emit(fallback(f"timed out after {a.zslab_timeout:.0f} s"))
            os._exit(3)
        timer = threading.Timer(a.zslab_timeout, on_timeout)
        timer.daemon = True
        timer.start()
    try:
        out = measure_main(a, name, intr, params, frames, D, rank, world, local, mode, icp_ar)
    except Exception as e:  # noqa: BLE001 -- a failed slab stream falls back to the replicas line
        if replicas is None:
            raise
        out = fallback(f"{type(e).__name__}: {e}"[:300])
    if timer is not None:
        timer.cancel()
    if replicas is not None and "zslab" not in out:
        out["replicas"] = replicas
    # N>1 replica line: one Z-slab sharded stream beside it, under
    # its own time limit, so that a failing or hung collective still leaves the line
    if mode == "replicas" and (world > 1 or a.mode == "replicas") and a.zslab != "none":
        def on_zslab_timeout():  # the replica line stands, the hang exits 3
            emit(out, {"zslab": {"error": f"timed out after {a.zslab_timeout:.0f} s"}})
            os._exit(3)
        zt = threading.Timer(a.zslab_timeout, on_zslab_timeout)
        zt.daemon = True
        zt.start()
        try:
            out["zslab"] = zslab_record(a, intr, frames, D, rank, world, local, icp_ar, (W, H, L))
        except Exception as e:  # noqa: BLE001 -- recorded, the replica line stands
            out["zslab"] = {"error": f"{type(e).__name__}: {e}"[:300]}
        zt.cancel()
    # N=1: the C3 record (1024^3 @ 2 mm on the same frames) beside the C2 line
    if world == 1 and mode == "single" and a.c3_frames and name == "c2":
        import copy
        b = copy.copy(a)
        b.steps = a.c3_frames
        W3, H3, n3, L3 = CONFIGS["c3"]
        f3 = (bgr, dep, synth.ping_pong(len(bgr), b.warmup + b.steps), None)
        out["c3_record"] = single_record(b, "c3", intr, n3, L3, f3, D, local, a.traffic_c3)
    # N=1: the C5 single volume (1280x720, 2048^3 @ 2 mm), the N=1 point of the
    # zslab curve the driver's N>1 runs record
    if world == 1 and mode == "single" and a.c5_frames and name == "c2":
        import copy
        b = copy.copy(a)
        b.steps = a.c5_frames
        W5, H5, n5, L5 = CONFIGS["c5"]
        i5 = intrinsics(W5, H5)
        u5 = 16
        bgr5, dep5, _ = synth.sequence(u5, i5, L=L5, noise=True, traj_seed=7, dropout=0.005)
        f5 = (bgr5, dep5.astype(np.float32), synth.ping_pong(u5, b.warmup + b.steps), None)
        out["c5_record"] = single_record(b, "c5", i5, n5, L5, f5, D, local, a.traffic_c5)
        del bgr5, dep5, f5
    emit(out)
    D.close()


def base_line(a, world, value, ms, scaling, config):
    return {
        "metric": "frames/sec at 640×480, 512³ TSDF; per-stage ms (ICP/integrate/raycast)",
        "value": round(value, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": scaling,
        "vs_baseline": round(value / (1000.0 / REF_MS_PER_FRAME), 3),
        "dtype": "f32",
        "data": "synthetic",
        "config": config,
    }


def zslab_record(a, intr, frames, D, rank, world, local, icp_ar, geom):
    """ONE stream of config a.zslab, its volume Z-slab sharded over the N ranks
    (work-balanced cuts, RCCL combine of the raycast, ICP replicated or
    all-reduced): frames/s of the stream (strong scaling) and every rank's
    kernel ms, integrate work and slab extent (the W/K contract of the line)."""
    from kfx import synth
    from kfx.abi import default_params
    W, H, n, L = CONFIGS[a.zslab]
    params = default_params(dims=n, range_m=L)
    if (W, H, L) == geom:
        zintr, zframes = intr, frames
    else:
        zintr = intrinsics(W, H)
        unique = 16 if W * H > 640 * 480 else 48
        bgr, dep, gt = synth.sequence(unique, zintr, L=L, noise=True, traj_seed=7, dropout=0.005)
        zframes = (bgr, dep.astype(np.float32), synth.ping_pong(unique, a.warmup + a.steps), gt)
    kf, r = run_stream(a, zintr, params, zframes, D, local, slab=(rank, world), icp_ar=icp_ar,
                       gmode=graph_mode(a, a.zslab))
    kt = r["ktime"] or {}
    work = kf.integrate_stats()
    zb, zn, o0, o1 = kf.slab_info()
    kf.close()
    row = [kt.get("icp", float("nan")), kt.get("integrate", float("nan")), kt.get("raycast_local", float("nan")),
           kt.get("combine", float("nan")), float(work["updated"]), float(o1 - o0), float(zn)]
    rows = D.gather(row)
    per_rank = [{"rank": k, "icp_ms": round(x[0], 4), "integrate_ms": round(x[1], 4), "raycast_ms": round(x[2], 4),
                 "combine_ms": round(x[3], 4), "integrate_updated": int(x[4]), "owned_slices": int(x[5]),
                 "stored_slices": int(x[6])} for k, x in enumerate(rows)]
    return {"workload": workload_text(a.zslab, W, H, n, L, "slab", world, icp_ar, a.cuts),
            "graph": graph_parts(a, "slab", r["graph_mode"], r["graph_requested"]) +
                     (f" [{r['graph_note']}]" if r.get("graph_note") else ""),
            "value": round(a.steps / r["elapsed"], 3), "unit": "frames/s", "scaling": "strong",
            "ms_per_step": round(1000.0 * r["elapsed"] / a.steps, 4), "steps": a.steps, "warmup": a.warmup,
            "tracked_frames": int(r["tracked"]), "per_rank": per_rank,
            "integrate_ms_per_rank": [p["integrate_ms"] for p in per_rank],
            "integrate_imbalance_max_over_mean": imbalance([p["integrate_ms"] for p in per_rank])}


def imbalance(xs):
    """max / mean of the per-rank values (1.0 = perfectly balanced; None when
    any rank has no sample)."""
    xs = [float(x) for x in xs]
    if not xs or any(x != x for x in xs) or sum(xs) <= 0:
        return None
    return round(max(xs) / (sum(xs) / len(xs)), 4)


def measure_main(a, name, intr, params, frames, D, rank, world, local, mode, icp_ar):
    import kfx
    from kfx import synth
    from kfx.abi import default_params
    bgr, dep, order, _ = frames
    W, H = intr.width, intr.height
    n, L = params.volu_dims[0], params.volu_range[0]
    slab = (rank, world) if mode == "slab" else None
    kf, r = run_stream(a, intr, params, frames, D, local, slab=slab, icp_ar=icp_ar, gmode=graph_mode(a, name))
    elapsed, ktime, tracked, gmode = r["elapsed"], r["ktime"], r["tracked"], r["graph_mode"]
    ms_source = (f"timed region, {ktime['samples']} HIP-event-bracketed frames" if ktime else "profiled frames")

    # per-stage device ms on further frames (profiled, eager; single volume)
    stages = {k: [] for k in ("preprocess", "icp", "integrate", "raycast", "total")}
    int_ms, int_work = [], []
    nprof = a.profile_frames if mode != "slab" else 0
    if nprof:
        kf.set_profiling(True)
        for i in range(a.warmup + a.steps, a.warmup + a.steps + nprof):
            kf.pipeline_staged(order[i])
            ms = kf.stage_ms()
            for k in stages:
                stages[k].append(ms[k])
            int_work.append(kf.integrate_stats())
            int_ms.append(ms["integrate"])
        kf.set_profiling(False)
    else:
        int_work.append(kf.integrate_stats())  # the last timed frame's integrate work
    ray_work = kf.raycast_stats() if nprof else None
    # host-input throughput (not `value`; after the profiled frames, so that their
    # integrate work, the roofline's bytes, follows the timed frames directly): the
    # same frames from host memory
    # through kfx_pipeline_async (pinned ring, H2D overlapped with the previous
    # frame), PCIe included, f32 depth as the reference's pipeline() takes it
    host_in = None
    if a.host_frames > 0 and mode == "single":
        unique = len(bgr)
        hb = np.ascontiguousarray(bgr)
        hd = np.ascontiguousarray(dep)
        # zero copy: the frames' host memory is page-locked once, then every
        # frame is DMAed straight from it (no staging copy on the host)
        kf.register_host_buffer(hb)
        kf.register_host_buffer(hd)
        ho = synth.ping_pong(unique, a.host_frames)
        for i in ho[:8]:  # untimed: every ring slot used once (its graphs captured)
            kf.pipeline_async(hb[i], hd[i])
        kf.synchronize()
        D.barrier()
        t0 = time.perf_counter()
        for i in ho:
            kf.pipeline_async(hb[i], hd[i])
        st_h = kf.synchronize()
        dt_h = D.max(time.perf_counter() - t0)
        kf.unregister_host_buffer(hb)
        kf.unregister_host_buffer(hd)
        host_in = {"value": round(len(ho) * world / dt_h, 3), "unit": "frames/s",
                   "ms_per_step": round(1000.0 * dt_h / len(ho), 4), "frames": len(ho),
                   "status": "ok" if st_h == kfx.KFX_OK else "tracking lost",
                   "bytes_per_frame_h2d": W * H * 7,
                   "path": "kfx_pipeline_async from host buffers registered with kfx_register_host_buffer: "
                           "H2D straight from the caller's page-locked frames on a copy stream, overlapped with "
                           "the previous frame (no host copy); f32 depth mm + BGR8"}

    extract = extract_record(kf, n) if (mode == "single" and a.extract) else None
    zb, zn, o0, o1 = kf.slab_info()
    kf.synchronize()
    kf.close()
    stage_med = {k: round(statistics.median(v), 4) for k, v in stages.items()} if nprof else {}
    work = {k: int(np.mean([w[k] for w in int_work])) for k in int_work[0]}
    # the integrate launch duration of the roofline: the HIP-event samples of
    # the timed region (fallback: the profiled frames after it)
    if ktime:
        int_launch_ms = float(ktime["integrate"])
    else:
        int_launch_ms = float(np.mean(int_ms)) if int_ms else float("nan")
    ray_ms = float(ktime["raycast"]) if ktime else (
        float(statistics.median(stages["raycast"])) if stages["raycast"] else float("nan"))

    # per-rank kernel ms and integrate work (slab ranks integrate different slabs)
    kt = ktime or {}
    row = [kt.get("icp", float("nan")), kt.get("integrate", float("nan")), kt.get("raycast_local", float("nan")),
           kt.get("combine", float("nan")), float(kt.get("samples", 0)), float(work["updated"]),
           float(work["colored"]), float(o1 - o0), float(zn)]
    rows = D.gather(row)
    per_rank = [{"rank": k, "icp_ms": round(x[0], 4), "integrate_ms": round(x[1], 4),
                 "raycast_ms": round(x[2], 4), "combine_ms": round(x[3], 4), "samples": int(x[4]),
                 "integrate_updated": int(x[5]), "integrate_colored": int(x[6]), "owned_slices": int(x[7]),
                 "stored_slices": int(x[8])} for k, x in enumerate(rows)]

    # HBM traffic of the integrate launch from a rocprofv3 FETCH_SIZE/WRITE_SIZE
    # record (tools/prof.sh), attached only when that record was measured on
    # this workload with the same step counts (the same saturation regime)
    # and on the very library this process loaded (sha256 of libkfx.so)
    lib_hash = file_sha256(kfx.LIB_PATH)
    traffic, ray_traffic, sq, traffic_src = (None, None, None, None) if mode != "single" else pmc_record(
        a.traffic, [n, W, H], a.steps, a.warmup, lib_hash)
    if mode == "slab":
        # the critical path is the slowest rank's integrate
        k = max(range(len(per_rank)), key=lambda q: per_rank[q]["integrate_ms"])
        pr = per_rank[k]
        roof = integrate_roofline({"updated": pr["integrate_updated"], "colored": pr["integrate_colored"]},
                                  pr["integrate_ms"], W, H, ms_source + f", slowest rank ({k})")
    else:
        roof = integrate_roofline(work, int_launch_ms, W, H, ms_source, traffic, traffic_src)
        roof["lib_sha256"] = lib_hash
        if issue_figures(sq, "integrate"):
            roof["issue"] = issue_figures(sq, "integrate")

    cpu = c1 = None
    if rank == 0 and world == 1 and a.cpu_frames > 0:
        cpu = cpu_baseline(intr, params, bgr, dep, synth.ping_pong(len(bgr), a.cpu_frames + 1), a.cpu_frames)
    if rank == 0 and world == 1 and a.c1_frames > 0 and (W, H) == (640, 480):
        # BASELINE C1: 128^3 TSDF (16 mm) on the same 640x480 frames, serial oracle
        c1 = cpu_baseline(intr, default_params(dims=128, range_m=L), bgr, dep,
                          synth.ping_pong(len(bgr), a.c1_frames + 1), a.c1_frames)
        c1["config"] = "C1: 128^3 TSDF @ 16 mm, 640x480 synthetic frames (the bundled dataset is absent)"

    frames_done = a.steps * (world if mode == "replicas" else 1)
    value = frames_done / elapsed
    out = base_line(a, world, value, 1000.0 * elapsed / a.steps, "strong" if mode == "slab" else "weak", {
        "workload": workload_text(name, W, H, n, L, mode, world, icp_ar, a.cuts),
        "width": W, "height": H, "volume_dims": n, "volume_range_m": L,
        "frames_unique": len(bgr),
        # what the timed frames replay as graphs (kfx_set_graph_mode); the few
        # stage-timing sample frames launch eagerly with their events
        "graph": graph_parts(a, mode, gmode, r["graph_requested"]), "overlap": not a.no_overlap,
        "parallelism": (f"zslab x{world}" + (" + icp allreduce" if icp_ar else "") if mode == "slab" else
                        (f"replicas x{world} (independent streams)" if world > 1 else "single")),
        "collective": ("RCCL: raycast combine per frame" + (" + ICP partials per iteration" if icp_ar else "")
                       if mode == "slab" else
                       ("none: N independent C2 streams; this line is NOT the Z-slab sharded scaling "
                        "(that is the `zslab` record)" if world > 1 else "none (one GPU)")),
        "tracked_frames": int(tracked),
        "reference_ms_per_frame": REF_MS_PER_FRAME,
    })
    out.update({
        "stage_ms": stage_med,
        "timed_region_kernel_ms": round_ms(ktime),
        "per_rank": per_rank if world > 1 else None,
        "integrate_voxels": work,
        "raycast_work": ray_work,
        "roofline": roof,
        "roofline_raycast": raycast_roofline(ray_work, ray_ms, W, H, ms_source, ray_traffic,
                                             traffic_src if ray_traffic else None),
        "host_input": host_in,
        "extract": extract,
        "cpu_baseline": cpu,
        "c1_record": c1,
    })
    return out


if __name__ == "__main__":
    main()
