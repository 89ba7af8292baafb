"""Exact fast-forward of repeated float adds (csrc/kfx_ffadd.h, CPU).

Integrate replays the reference's per-slice accumulation vc += zstep
(tsdf_volume.cu:53-55) to the first slice of a z-chunk or Z-slab; kfx::ff_add
does n of those adds in a few integer steps per binade.  It must equal the
plain loop bit for bit: tests/ffadd/ff_check.cpp compares them on random
columns, ties, zero crossings, fixed points, extreme exponents and non-finite
inputs, built once plain (-O2, no contraction) and once under UBSan."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "ffadd", "ff_check.cpp")
INC = os.path.join(ROOT, "slam-kinectfusion_amd", "csrc")


@pytest.mark.parametrize("flags", [["-O2"], ["-O1", "-g", "-fsanitize=undefined", "-fno-sanitize-recover=all"]],
                         ids=["O2", "ubsan"])
def test_ffadd_matches_plain_loop(tmp_path, flags):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    exe = str(tmp_path / "ff_check")
    subprocess.run(["g++", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", *flags, "-I", INC, SRC, "-o", exe],
                   check=True)
    for seed in (1, 2):
        r = subprocess.run([exe, str(seed), "60000"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and r.stdout.strip() == "bad 0", (r.stdout[-2000:], r.stderr[-2000:])
