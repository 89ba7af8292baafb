#!/usr/bin/env python3
"""Multi-GPU readiness record on ONE GPU: the Z-slab split
of BASELINE C4 (1024^3 @ 2 mm, 640x480) or C5 (2048^3 @ 2 mm, 1280x720) over
8 slab contexts held in one process (kfx_pipeline_group), next to the single
volume on the same frames.  With kernel timing on, the group runs its members
one after another, each alone on the GPU as on a GPU of its own, and every
member reports its ICP / integrate / local raycast / combine ms (HIP events on
its stream) and its integrate work (kfx_integrate_stats: updated voxels of the
last frame).  The combine here is the in-process one (one reduction kernel
over the members' buffers + mask + expand + pyramid), not RCCL.

usage: python3 tools/slab_record.py c4|c5 [--world 8] [--frames 20] [--warmup 5] [--out FILE]"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "slam-kinectfusion_amd"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config", choices=["c4", "c5"])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--groups", default="equal,balanced,balanced_unbounded,calibrated",
                    help="cut sets to time (A/B runs: e.g. calibrated)")
    ap.add_argument("--rccl-us", type=float, default=25.0,
                    help="assumed latency of one 27 x int64 RCCL all-reduce over the ranks (not measured here: "
                         "one GPU), used to price the sharded ICP (19 all-reduces per frame)")
    a = ap.parse_args()
    import kfx
    from kfx import synth
    from kfx.abi import Intrinsics, default_params
    from bench import CONFIGS, intrinsics
    W, H, n, L = CONFIGS[a.config]
    intr = intrinsics(W, H)
    p = default_params(dims=n, range_m=L)
    unique = 16
    bgr, dep, gt = synth.sequence(unique, intr, L=L, noise=True, traj_seed=7, dropout=0.005)
    dep = dep.astype(np.float32)
    order = synth.ping_pong(unique, a.warmup + a.frames)
    I = Intrinsics.from_any(intr)
    rec = {"config": a.config, "width": W, "height": H, "volume_dims": n, "volume_range_m": L, "world": a.world,
           "frames_timed": a.frames, "warmup": a.warmup, "lib_sha256": None,
           "method": "8 slab contexts on one GPU (kfx_pipeline_group); timed members run alone, one after "
                     "another; HIP events on each member's stream; combine = shared in-process reductions, masks, resume passes + own expand + "
                     "pyramid (not RCCL)"}
    import hashlib
    rec["lib_sha256"] = hashlib.sha256(open(kfx.LIB_PATH, "rb").read()).hexdigest()

    # the single volume on the same host frames
    single = kfx.KinectFusion(I, p)
    for i in order[:a.warmup]:
        single.pipeline(bgr[i], dep[i])
    single.set_kernel_timing(1, a.frames + 2)
    t0 = time.perf_counter()
    for i in order[a.warmup:a.warmup + a.frames]:
        assert single.pipeline(bgr[i], dep[i]) == kfx.KFX_OK
    t_single = time.perf_counter() - t0
    ks = single.kernel_timing()
    ws = single.integrate_stats()
    rec["single"] = {"icp_ms": ks["icp"], "integrate_ms": ks["integrate"], "raycast_ms": ks["raycast"],
                     "integrate_updated": ws["updated"], "wall_ms_per_frame": 1e3 * t_single / a.frames}
    sp = single.pose_record
    single.close()

    def group(cuts, bound=1):
        members = [kfx.KinectFusion(I, p, slab=(r, a.world), cuts=cuts) for r in range(a.world)]
        for m in members:
            m.set_slab_bound(bound)
        for i in order[:a.warmup]:
            kfx.pipeline_group(members, bgr[i], dep[i])
        for m in members:
            m.set_kernel_timing(1, a.frames + 2)
        t0 = time.perf_counter()
        for i in order[a.warmup:a.warmup + a.frames]:
            assert kfx.pipeline_group(members, bgr[i], dep[i]) == kfx.KFX_OK
        t_group = time.perf_counter() - t0
        slabs = []
        for r, m in enumerate(members):
            k = m.kernel_timing()
            w = m.integrate_stats()
            zb, zn, o0, o1 = m.slab_info()
            slabs.append({"rank": r, "owned_slices": [o0, o1], "stored_slices": [zb, zb + zn],
                          "icp_ms": k["icp"], "integrate_ms": k["integrate"], "raycast_local_ms": k["raycast_local"],
                          "combine_ms": k["combine"], "integrate_updated": w["updated"], "samples": k["samples"]})
        if not os.environ.get("KFX_TIMING_ONLY"):  # (timing-only variants compute wrong values)
            assert all(np.array_equal(m.pose_record, sp) for m in members), "slab poses differ from the single volume"
        # the sharded ICP's per-rank device work (kfx_set_icp_allreduce: band r of
        # every level's rows, 19 k_icp_acc + k_icp_solve launches) on the last
        # frame's maps, without its 19 all-reduces (priced at --rccl-us)
        iters = int(sum(p.icp_iter_count[:3]))
        for r, (m, sl) in enumerate(zip(members, slabs)):
            sl["icp_banded_ms"] = m.debug_icp_band_ms(r, a.world, reps=5)
            sl["icp_sharded_ms_priced"] = sl["icp_banded_ms"] + iters * a.rccl_us * 1e-3
        full_launches = members[0].debug_icp_band_ms(0, 1, reps=5)
        for m in members:
            m.close()
        it = np.array([s["integrate_ms"] for s in slabs])
        up = np.array([s["integrate_updated"] for s in slabs], dtype=np.float64)
        # per-rank critical path of one frame at N GPUs (replicated ICP, RCCL not included)
        crit = [s["icp_ms"] + s["integrate_ms"] + s["raycast_local_ms"] for s in slabs]
        crit_c = [c + s["combine_ms"] for c, s in zip(crit, slabs)]
        rc = np.array([s["raycast_local_ms"] for s in slabs])
        crit_sh = [s["icp_sharded_ms_priced"] + s["integrate_ms"] + s["raycast_local_ms"] + s["combine_ms"]
                   for s in slabs]
        return {"cuts": cuts, "slab_bound": bound, "slabs": slabs,
                "icp_per_iteration_launches_whole_frame_ms": full_launches,
                "rccl_allreduce_us_assumed": a.rccl_us,
                "max_rank_crit_sharded_icp_ms": float(max(crit_sh)),
                "group_wall_ms_per_frame": 1e3 * t_group / a.frames,
                "max_slab_over_single_raycast": float(rc.max() / rec["single"]["raycast_ms"]),
                "max_rank_icp_integrate_raycast_combine_ms": float(max(crit_c)),
                "integrate_imbalance_max_over_mean": float(it.max() / it.mean()),
                "updated_imbalance_max_over_mean": float(up.max() / up.mean()),
                "max_slab_over_single_integrate": float(it.max() / rec["single"]["integrate_ms"]),
                "max_rank_icp_integrate_raycast_ms": float(max(crit))}

    rec["ideal"] = 1.0 / a.world
    rec["single_icp_integrate_raycast_ms"] = float(sum(rec["single"][k] for k in ("icp_ms", "integrate_ms",
                                                                                    "raycast_ms")))
    # per-slice work of the first frame (what bench.py balances on at N > 1)
    probe = kfx.KinectFusion(I, p, slab=(0, n // 16))
    work = probe.slice_work(bgr[order[0]], dep[order[0]])
    cover, upd = probe.slice_work_parts(bgr[order[0]], dep[order[0]])
    # the same estimate averaged over 4 frames of the timed run at their
    # ground-truth poses (bench.py --cuts balanced: cuts for the run)
    seen = sorted(set(order[a.warmup:a.warmup + a.frames]))
    calib = [seen[int(round(j * (len(seen) - 1) / 3))] for j in range(4)]
    parts = [probe.slice_work_at(bgr[i], dep[i], gt[i]) for i in calib]
    cw = np.mean([q[0] for q in parts], axis=0).round().astype(np.int64)
    ccov = np.mean([q[1] for q in parts], axis=0)  # visited slots per slice (the occlusion-clipped intervals)
    cupd = np.mean([q[2] for q in parts], axis=0)  # updated voxels per slice
    probe.close()
    rec["slice_cover_calibrated"] = [float(x) for x in ccov]
    rec["slice_updated_calibrated"] = [float(x) for x in cupd]
    rec["calibration_frames"] = [int(i) for i in calib]
    rec["slice_work_first_frame"] = [int(x) for x in work]
    rec["slice_work_calibrated"] = [int(x) for x in cw]
    rec["slice_cover_first_frame"] = [int(x) for x in cover]
    rec["slice_updated_first_frame"] = [int(x) for x in upd]
    gs = a.groups.split(",")
    if "equal" in gs:
        rec["equal_cuts"] = group(None)
    if "balanced" in gs:
        rec["balanced_cuts"] = group(kfx.slab_balance(work, a.world))
    # the same cuts with every slab ray marched to its end (no bound, no resume pass)
    if "balanced_unbounded" in gs:
        rec["balanced_cuts_unbounded"] = group(kfx.slab_balance(work, a.world), bound=0)
    if "calibrated" in gs:
        rec["calibrated_cuts_unbounded"] = group(kfx.slab_balance(cw, a.world), bound=0)
    # every timed slab's estimated work over its stored slices (the calibration
    # frames' mean): the inputs of the cost fit (tools/slab_fit.py)
    for k in ("equal_cuts", "balanced_cuts", "balanced_cuts_unbounded", "calibrated_cuts_unbounded"):
        for sl in rec.get(k, {}).get("slabs", []):
            z0, z1 = sl["stored_slices"]
            sl["est_cover"] = float(ccov[z0:z1].sum())
            sl["est_updated"] = float(cupd[z0:z1].sum())
            sl["stored_slots"] = float(n * n * (z1 - z0))
            # k_integrate's waves for this slab (kfx_kernels.hip integrate_chunks)
            tiles, zn = (n // 8) ** 2, z1 - z0
            nc = max(nc_min := (12288 + tiles - 1) // tiles, min((zn + 95) // 96, 4 * 12288 // tiles))
            sl["waves"] = float(tiles * max(1, min(8, max(nc, nc_min))))
    if not all(k in rec for k in ("equal_cuts", "balanced_cuts")):
        out = a.out or os.path.join(ROOT, "gpurun_out", f"slabs_{a.config}.json")
        os.makedirs(os.path.dirname(out), exist_ok=True)
        json.dump(rec, open(out, "w"), indent=1)
        for k in ("equal_cuts", "balanced_cuts", "balanced_cuts_unbounded", "calibrated_cuts_unbounded"):
            if k in rec:
                sl = rec[k]["slabs"]
                print(k, "integrate ms", [round(x["integrate_ms"], 3) for x in sl], "sum",
                      round(sum(x["integrate_ms"] for x in sl), 3), "crit",
                      round(rec[k]["max_rank_icp_integrate_raycast_combine_ms"], 3))
        return
    # integrate ms of a slab against its stored slices' estimated parts
    # (non-negative least squares, tools/slab_fit.py: this config alone)
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from slab_fit import fit
    rec["cost_fit"] = fit([rec])
    out = a.out or os.path.join(ROOT, "gpurun_out", f"slabs_{a.config}.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps({"config": rec["config"], "ideal": rec["ideal"],
                      **{f"{k}:{q}": rec[k][q] for k in ("equal_cuts", "balanced_cuts")
                         for q in ("integrate_imbalance_max_over_mean", "max_slab_over_single_integrate")},
                      **{f"{k}:{q}": rec[k][q] for k in ("balanced_cuts", "balanced_cuts_unbounded",
                                                          "calibrated_cuts_unbounded")
                         for q in ("max_slab_over_single_raycast", "max_rank_icp_integrate_raycast_combine_ms")},
                      "single_icp_integrate_raycast_ms": rec["single_icp_integrate_raycast_ms"],
                      "cost_fit": rec["cost_fit"]}))


if __name__ == "__main__":
    main()
