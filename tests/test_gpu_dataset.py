"""Dataset front-end end to end on the GPU: a synthetic sequence written as the
reference's dataset layout (color/, depth/ 16-bit PNG, intr.txt) runs through
examples/kfx_run (main.cpp's loop over the C-ABI, separate process) and through
the Python binding on the frames kfx.Dataset decodes; both must write the same
poses.txt bytes as the binding fed the original arrays."""
import os
import subprocess

import numpy as np
import pytest
from PIL import Image

import kfx
from kfx import synth
from kfx.abi import Intrinsics, default_params

pytestmark = pytest.mark.gpu
RUNNER = os.path.join(os.path.dirname(kfx.LIB_PATH), "kfx_run")


def _write(root, bgr, dep, intr):
    os.makedirs(os.path.join(root, "color"))
    os.makedirs(os.path.join(root, "depth"))
    for k in range(len(dep)):
        Image.fromarray(np.ascontiguousarray(bgr[k][:, :, ::-1])).save(os.path.join(root, "color", f"{k:06d}.png"))
        Image.fromarray(dep[k]).save(os.path.join(root, "depth", f"{k:06d}.png"))
    with open(os.path.join(root, "intr.txt"), "w") as f:
        f.write(f"{intr.fx} 0 {intr.cx}\n0 {intr.fy} {intr.cy}\n0 0 1\n")


def _poses(kf, path):
    kf.write_poses_txt(str(path))
    return open(path).read()


def test_dataset_runner_matches_binding(tmp_path):
    intr = synth.Intrinsics.qvga()
    bgr, dep, _ = synth.sequence(8, intr, noise=True, dropout=0.01)
    root = str(tmp_path / "ds")
    _write(root, bgr, dep, intr)
    p = default_params()  # the runner uses the reference defaults (512^3, 3 m)

    ref = kfx.KinectFusion(Intrinsics.from_any(intr), p)
    for k in range(len(dep)):
        ref.pipeline(bgr[k], dep[k].astype(np.float32))
    want = _poses(ref, tmp_path / "want.txt")
    ref.close()

    ds = kfx.Dataset(root)
    assert ds.has_intr and len(ds) == len(dep)
    kf = kfx.KinectFusion(ds.intrinsics, p)
    for k in range(len(ds)):
        c, d = ds.read(k)
        kf.pipeline(c, d)
    assert _poses(kf, tmp_path / "got.txt") == want
    kf.close()
    ds.close()

    out = tmp_path / "runner.txt"
    r = subprocess.run([RUNNER, root, str(out), str(tmp_path / "cloud.ply")], capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "end!" in r.stdout
    assert open(out).read() == want
    assert open(tmp_path / "cloud.ply").read().startswith("ply\nformat ascii 1.0\nelement vertex ")
