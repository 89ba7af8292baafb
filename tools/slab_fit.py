#!/usr/bin/env python3
"""Slab integrate cost model: a slab's integrate ms against
its stored slices' estimated work, ms ~ c + a * cover + b * updated + s * slots
+ w * waves + p * cover / waves, minimising the largest relative error (cover: visited voxel slots of the occlusion-clipped column
intervals, updated: voxels passing the update test, slots: stored voxel slots,
waves: k_integrate's (tile, chunk) waves; the calibration
frames' means, tools/slab_record.py), fitted (non-negative weights, minimax relative error) over
every timed slab of the given records (C4 + C5; one constant c per config),
with per-slab residuals (non-negative weights: a linear program).  The per-slice part (a, b, s) is what
kfx_slab_balance balances (kfx_api.hip slice_cost); c is paid by every slab
of a config alike.
usage: python3 tools/slab_fit.py profiles/r05_c4_slabs.json profiles/r05_c5_slabs.json"""
import json
import sys

import numpy as np
from scipy.optimize import linprog, nnls

TERMS = ("cover", "updated", "slots", "waves", "per_wave")


def rows(recs):
    cfgs = sorted({r.get("config") for r in recs})
    out = []
    for rec in recs:
        onehot = [1.0 if rec.get("config") == c else 0.0 for c in cfgs]  # a per-slab constant per config
        for k in ("equal_cuts", "balanced_cuts", "balanced_cuts_unbounded", "calibrated_cuts_unbounded"):
            for sl in rec.get(k, {}).get("slabs", []):
                if "est_cover" not in sl:
                    continue
                waves = sl.get("waves", 0.0)
                # per_wave: visited slots per launched wave — the slab's waves are
                # few and long when one z-chunk covers its slices (its tail)
                out.append((rec.get("config"), k, sl["rank"],
                            onehot + [sl["est_cover"], sl["est_updated"], sl["stored_slots"], waves,
                                      sl["est_cover"] / waves if waves else 0.0],
                            sl["integrate_ms"]))
    return cfgs, out


def fit(recs):
    cfgs, rs = rows(recs)
    names = tuple(f"const_{c}" for c in cfgs) + TERMS
    if len(rs) < len(names):
        return None
    A = np.array([r[3] for r in rs], np.float64)
    y = np.array([r[4] for r in rs], np.float64)
    scale = A.max(axis=0)
    scale[scale == 0] = 1.0
    # the model is judged by its largest relative error over the slabs: a
    # minimax (Chebyshev) fit of the relative errors, non-negative weights, by
    # linear programming — minimise t with -t <= (A c - y) / y <= t, c >= 0;
    # relative least squares (NNLS of the rows divided by y) if that fails
    B = (A / scale) / y[:, None]
    nc = B.shape[1]
    cost = np.zeros(nc + 1)
    cost[-1] = 1.0
    ones = np.ones((len(y), 1))
    A_ub = np.vstack([np.hstack([B, -ones]), np.hstack([-B, -ones])])
    b_ub = np.concatenate([np.ones(len(y)), -np.ones(len(y))])
    res = linprog(cost, A_ub=A_ub, b_ub=b_ub, bounds=[(0, None)] * (nc + 1), method="highs")
    if res.status == 0:
        coef = res.x[:nc]
    else:
        coef, _ = nnls(B, np.ones(len(y)))
    coef = coef / scale
    pred = A @ coef
    rel = (pred - y) / y
    k = len(cfgs)
    return {"terms": {t: float(c) for t, c in zip(names, coef)},
            "per_slice_weights_over_cover": {t: (float(c / coef[k]) if coef[k] > 0 else None)
                                             for t, c in zip(TERMS[1:], coef[k + 1:])},
            "max_rel_err": float(np.max(np.abs(rel))), "rms_rel_err": float(np.sqrt(np.mean(rel ** 2))),
            "residuals": [{"config": r[0], "cuts": r[1], "rank": r[2], "ms": round(r[4], 4),
                           "fit_ms": round(float(p), 4), "rel_err": round(float(e), 4)} for r, p, e in zip(rs, pred, rel)]}


if __name__ == "__main__":
    recs = [json.load(open(f)) for f in sys.argv[1:]]
    res = fit(recs)
    print(json.dumps({k: v for k, v in res.items() if k != "residuals"}, indent=1))
    worst = sorted(res["residuals"], key=lambda r: -abs(r["rel_err"]))[:8]
    for r in worst:
        print(r)
