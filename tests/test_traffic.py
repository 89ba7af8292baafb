"""tools/traffic.py sq_issue: the VALU issue bracket [6A - 4I, 4A] of the SQ
counters (A = SQ_ACTIVE_INST_VALU, I = SQ_INSTS_VALU), calibrated on the known
instruction streams of tools/valu_calib.hip (profiles/r06_valu_calib.json):
for each calibration kernel the bracket contains the issue time measured
in-kernel, and no reported fraction exceeds 1 (CPU only)."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import traffic  # noqa: E402


def test_bracket_contains_the_calibrated_issue_time():
    rec = json.load(open(os.path.join(ROOT, "profiles", "r06_valu_calib.json")))
    for name, k in rec["kernels"].items():
        c = k["counters_per_dispatch"]
        q = traffic.sq_issue(dict(c, dispatches=1))
        lo, hi = q["valu_busy_frac_bounds"]
        assert 0.0 <= lo <= hi <= 1.0, (name, lo, hi)
        # the issue time the kernel measured (cycles per instruction x count);
        # its loop's scalar instructions (one s_add / s_cmp / s_cbranch per 16
        # VALU) inflate the in-kernel cycles per VALU instruction by a few %
        true = k["cycles_per_wave_instruction"]["med"] * c["SQ_INSTS_VALU"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8)
        assert lo <= min(true, 1.0) * 1.08 and min(true, 1.0) <= hi * 1.08, (name, lo, true, hi)


@pytest.mark.parametrize("I,A", [(100.0, 100.0), (100.0, 150.0), (100.0, 200.0)])
def test_bracket_from_instruction_classes(I, A):
    """I instructions of which A - I are 8-cycle transcendentals and the rest
    2- or 4-cycle: every mix's issue time lies in the bracket."""
    cyc = 1000.0
    d = {"SQ_INSTS_VALU": I * 1024, "SQ_ACTIVE_INST_VALU": A * 1024, "GRBM_GUI_ACTIVE": 8 * cyc, "dispatches": 1}
    lo, hi = traffic.sq_issue(d)["valu_busy_frac_bounds"]
    n8 = A - I
    for share4 in (0.0, 0.5, 1.0):
        n4 = (I - n8) * share4
        n2 = I - n8 - n4
        t = (2 * n2 + 4 * n4 + 8 * n8) / cyc
        assert lo - 1e-9 <= min(t, 1.0) <= hi + 1e-9
