#!/usr/bin/env python3
"""Per-launch HBM traffic of the kfx kernels from rocprofv3 PMC passes.

Input: the directory tools/prof.sh writes (gpurun_out/prof):
  calib/{FETCH_SIZE,WRITE_SIZE}/**/counter_collection.csv  known-byte streams (tools/pmc_calib.hip)
  pmc/{FETCH_SIZE,WRITE_SIZE}/**/counter_collection.csv    the bench run
  stats/**/*kernel_stats.csv                               rocprofv3 --stats summary

FETCH_SIZE / WRITE_SIZE are converted to bytes with the calibration factors of
the 2-byte streams (the width of the tsdf/weight arrays that dominate integrate
and raycast): factor = counter value per dispatch / bytes the stream moved
(MI355X_MICROARCH.md: only 16-B/lane streams are calibrated there, other widths
must be calibrated on a known byte count).  The SQ pass (pmc/SQ) gives the
issue figures of integrate and raycast (VALU issue fraction, wave-cycle split).
Output: <dir>/traffic.json, and profiles/$PMC_RECORD (default
r04_integrate_pmc.json) when --commit is given: bench.py attaches it as
roofline.traffic only to a run that loaded the library it names by sha256.
"""
import collections
import csv
import glob
import json
import os
import sys

CALIB_BYTES = 512 << 20  # each calibration kernel streams 512 MiB once


def short(name):
    name = name.replace("void ", "")
    for p in ("kfx::(anonymous namespace)::", "kfx::"):
        name = name.replace(p, "")
    return name.split("(")[0].strip()


def per_kernel(root):
    agg = collections.defaultdict(list)
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r.get("Kernel_Name", "?"))].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def main():
    root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof"
    commit = "--commit" in sys.argv
    out = {"calibration": {}, "kernels": {}}
    fac = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        cal = per_kernel(f"{root}/calib/{c}")
        want = "k_read<unsigned short>" if c == "FETCH_SIZE" else "k_write<unsigned short>"
        for k, (v, n) in cal.items():
            out["calibration"][f"{c}:{k}"] = {"per_dispatch": v, "units_per_byte": v / CALIB_BYTES}
        hit = [v for k, (v, n) in cal.items() if k.startswith(want)]
        fac[c] = (hit[0] / CALIB_BYTES) if hit else None
    out["factor_units_per_byte"] = fac
    fetch = per_kernel(f"{root}/pmc/FETCH_SIZE")
    write = per_kernel(f"{root}/pmc/WRITE_SIZE")
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (None, 0))
        w, nw = write.get(k, (None, 0))
        rec = {"FETCH_SIZE": f, "WRITE_SIZE": w, "dispatches": max(nf, nw)}
        if f is not None and fac.get("FETCH_SIZE"):
            rec["read_bytes"] = f / fac["FETCH_SIZE"]
        if w is not None and fac.get("WRITE_SIZE"):
            rec["write_bytes"] = w / fac["WRITE_SIZE"]
        if "read_bytes" in rec and "write_bytes" in rec:
            rec["hbm_bytes_per_launch"] = rec["read_bytes"] + rec["write_bytes"]
        out["kernels"][k] = rec
    for k, r in out["kernels"].items():
        if k.startswith("k_"):
            print(f"{k:40s} n={r['dispatches']:5d} hbm/launch={r.get('hbm_bytes_per_launch', float('nan')) / 1e6:10.2f} MB")
    sq = {k: v for k, v in per_counter(f"{root}/pmc/SQ").items()}
    out["sq"] = sq
    json.dump(out, open(f"{root}/traffic.json", "w"), indent=1)
    if commit:  # profiles/<round>_integrate_pmc.json: what bench.py attaches as roofline.traffic
        integ = [r for k, r in out["kernels"].items()
                 if k.startswith("k_integrate<false") and "hbm_bytes_per_launch" in r]
        if integ:
            import shlex
            args = shlex.split(os.environ.get("PROF_ARGS", ""))

            def arg(name, default):
                return int(args[args.index(name) + 1]) if name in args else default
            steps, warmup = arg("--steps", 300), arg("--warmup", 20)
            # the workload [dims, W, H] of the named config (bench.py CONFIGS), --dims overriding
            cfg = args[args.index("--config") + 1] if "--config" in args else "c2"
            W, H, dims = {"c2": (640, 480, 512), "c3": (640, 480, 1024), "c4": (640, 480, 1024),
                          "c5": (1280, 720, 2048)}.get(cfg, (640, 480, 512))
            dims = arg("--dims", dims)
            r = max(integ, key=lambda r: r["dispatches"])
            # the single-volume raycast (32- or 64-bit index), not a slab or stats variant
            ray = sorted([rr for k, rr in out["kernels"].items() if k.startswith("k_raycast<") and
                          k.endswith(", false, false>") and "hbm_bytes_per_launch" in rr],
                         key=lambda rr: -rr["dispatches"])
            lib = os.environ.get("KFX_LIB_PATH") or os.path.join(REPO, "slam-kinectfusion_amd", "lib", "libkfx.so")
            rec = {"kernel": "k_integrate", "hbm_bytes_per_launch": int(r["hbm_bytes_per_launch"]),
                   "read_bytes": int(r["read_bytes"]), "write_bytes": int(r["write_bytes"]),
                   "dispatches": r["dispatches"], "factor_units_per_byte": fac,
                   "raycast_hbm_bytes_per_launch": int(ray[0]["hbm_bytes_per_launch"]) if ray and
                   "hbm_bytes_per_launch" in ray[0] else None,
                   "workload": [dims, W, H], "steps": steps, "warmup": warmup,
                   "command": "python3 bench.py " + " ".join(args),
                   "regime": ("mean over every dispatch of the run: %d warm-up + %d timed + profiled "
                              "frames%s" % (warmup, steps, " (unsaturated transient: < 64 frames)"
                                            if warmup + steps + 20 < 64 else "")),
                   "source": "tools/prof.sh FETCH_SIZE/WRITE_SIZE passes, 2-byte stream calibration",
                   # the library the counters were collected on: bench.py attaches this
                   # record only to a run that loaded the same file
                   "lib": os.path.relpath(lib, REPO), "lib_sha256": sha256(lib),
                   "commit": os.environ.get("KFX_COMMIT")}
            for pre, name in (("k_integrate<false,", "integrate_sq"), ("k_raycast<", "raycast_sq")):
                ks = sorted([k for k in sq if k.startswith(pre) and (name != "raycast_sq" or k.endswith(", false, false>"))],
                            key=lambda k: -sq[k].get("dispatches", 0))
                if ks:
                    rec[name] = sq_issue(sq[ks[0]])
            name = os.environ.get("PMC_RECORD", "r04_integrate_pmc.json")
            json.dump(rec, open(os.path.join(REPO, "profiles", name), "w"), indent=1)
            # a copy beside the counters (profiles/ does not come back from the GPU box)
            json.dump(rec, open(os.path.join(root, name), "w"), indent=1)


REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_SIMD = 1024  # 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)


def sha256(path):
    import hashlib
    try:
        return hashlib.sha256(open(path, "rb").read()).hexdigest()
    except OSError:
        return None


def per_counter(root):
    """{kernel: {counter: mean per dispatch, "dispatches": n}} over a pass directory."""
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{root}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r.get("Kernel_Name", "?"))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for k, d in agg.items():
        out[k] = {c: sum(v) / len(v) for c, v in d.items()}
        out[k]["dispatches"] = max(len(v) for v in d.values())
    return out


def sq_issue(d):
    """Issue figures of one kernel from the SQ pass (means per dispatch).
    GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs, so the dispatch spans
    GRBM_GUI_ACTIVE / 8 shader cycles on each of the 1024 SIMDs.  VALU issue
    cycles, calibrated on known instruction streams (tools/valu_calib.hip,
    profiles/r06_valu_calib.json): a wave64 v_add_f32 occupies its SIMD for 2
    cycles, v_pk_fma_f32 and v_mad_u32_u24 for 4, v_rcp_f32 for 8, and
    SQ_ACTIVE_INST_VALU (A) counts 1 for the first three, 2 for v_rcp, while
    SQ_INSTS_VALU (I) counts 1 each.  With n2 + n4 = 2I - A instructions of 2 or
    4 cycles and n8 = A - I of 8, the issue cycles lie in [6A - 4I, 4A]; their
    fraction of the SIMD-cycles is the bracket reported (never above 1: a
    SIMD issues at most one VALU instruction at a time).  The round-5 figure
    4A / SIMD-cycles (`valu_active_frac`) counted every 2-cycle instruction
    as 4 and read above 1 on C3 / C5."""
    cyc = d.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    rec = {c: d[c] for c in sorted(d) if c != "dispatches"}
    rec["dispatches"] = d.get("dispatches")
    if cyc > 0:
        rec["kernel_cycles"] = cyc
        I, A = d.get("SQ_INSTS_VALU"), d.get("SQ_ACTIVE_INST_VALU")
        if I is not None:
            rec["valu_issue_frac_2cyc"] = round(2.0 * I / (N_SIMD * cyc), 4)
        if I is not None and A is not None:
            lo = max(2.0 * I, 6.0 * A - 4.0 * I) / (N_SIMD * cyc)
            hi = 4.0 * A / (N_SIMD * cyc)
            rec["valu_busy_frac_bounds"] = [round(min(lo, 1.0), 4), round(min(hi, 1.0), 4)]
    if d.get("SQ_WAVES"):
        rec["valu_insts_per_wave"] = round(d.get("SQ_INSTS_VALU", 0.0) / d["SQ_WAVES"], 1)
    if d.get("SQ_WAVE_CYCLES"):
        w = d["SQ_WAVE_CYCLES"]
        rec["wave_cycles_split"] = {k: round(d.get(c, 0.0) / w, 4) for k, c in
                                    (("active_inst_any", "SQ_ACTIVE_INST_ANY"), ("wait_any", "SQ_WAIT_ANY"),
                                     ("wait_inst_any", "SQ_WAIT_INST_ANY"))}
    return rec

if __name__ == "__main__":
    main()
