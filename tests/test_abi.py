"""C-ABI boundary checks that need no GPU: the library builds for gfx950,
loads, exports every entry point include/kfx.h declares, and its host-side
defaults match the reference's default_params (kinectfusion.cpp:167-190)."""
import ctypes as C
import os
import re

import numpy as np

import kfx
from kfx.abi import Params, default_params

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "kfx.h")


def declared_symbols():
    src = open(HDR).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(kfx_[a-z0-9_]+)\s*\(", src)))


def test_header_and_binding_agree():
    assert declared_symbols() == sorted(kfx.EXPORTS)


def test_library_exports_every_declared_symbol(kfx_lib):
    L = C.CDLL(kfx_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert kfx_lib.lib().kfx_abi_version() == 2


def test_library_is_gfx950_code_object(kfx_lib):
    data = open(kfx_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data
    assert b"k_integrate" in data and b"k_raycast" in data and b"k_icp_acc" in data


def test_default_params_match_reference(kfx_lib):
    p = Params()
    assert kfx_lib.lib().kfx_default_params(C.byref(p)) == 0
    q = default_params(dims=512, range_m=3.0)
    assert bytes(p) == bytes(q)
    assert p.pyramid_height == 3 and list(p.icp_iter_count)[:3] == [4, 5, 10]
    assert np.float32(p.volu_trun_dist) == np.float32(2.1) * np.float32(3.0) / np.float32(512)


def test_create_rejects_bad_arguments(kfx_lib):
    from kfx.abi import Intrinsics
    h = C.c_void_p()
    p = default_params(dims=64)
    bad = Intrinsics(321, 240, 1.0, 1.0, 0.0, 0.0)
    assert kfx_lib.lib().kfx_create(C.byref(bad), C.byref(p), 0, C.byref(h)) == -1
    p2 = default_params(dims=60)
    good = Intrinsics(320, 240, 262.5, 262.5, 159.5, 119.5)
    assert kfx_lib.lib().kfx_create(C.byref(good), C.byref(p2), 0, C.byref(h)) == -1
    assert b"multiples of 8" in kfx_lib.lib().kfx_last_error()


def test_product_build_refuses_experiment_macros():
    """make ARCH=gfx950 with -DKFX_* macros is refused for the product library
    (experiments build into lib/var_<name>), and the shipped kernel source holds
    none of the dropped experiment switches."""
    import subprocess
    pkg = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "slam-kinectfusion_amd")
    r = subprocess.run(["make", "-n", "-C", pkg, "ARCH=gfx950", "EXTRA=-DKFX_INT_CERT=1"],
                       capture_output=True, text=True)
    assert r.returncode != 0 and "var_" in (r.stdout + r.stderr)
    src = open(os.path.join(pkg, "csrc", "kfx_kernels.hip")).read()
    for m in ("KFX_INT_ZCLASS", "KFX_INT_CERT", "KFX_INT_DEDUP", "KFX_INT_LEAN", "KFX_INT_PLAN", "KFX_INT_PRIO",
              "KFX_RAY_PRIO", "KFX_ICP_XCOARSE", "KFX_INT_EXP", "KFX_PLAN_EXP", "KFX_RAY_NOREPLAY",
              "KFX_RAY_NONORMAL", "KFX_RAY_PIPE", "KFX_RAY_FFREPLAY", "KFX_RAY_FF_MIN", "KFX_RAY_FAKE_REPLAY",
              "KFX_RAY_LDS", "wrong values"):
        assert m not in src, m


def test_adapter_header_compiles_and_links(tmp_path):
    """adapter/kinectfusion.h (the reference's kf::kinectfusion over the C-ABI)
    compiled with a main.cpp-like driver against stand-ins for the few OpenCV
    core types it uses (OpenCV is not in this image) and linked to libkfx.so.
    Without a GPU the program reports the missing device and exits 2."""
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    stub = os.path.join(root, "tests", "adapter_stub")
    lib = os.path.join(root, "slam-kinectfusion_amd", "lib")
    exe = str(tmp_path / "main_like")
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-I", stub,
                        "-I", os.path.join(root, "slam-kinectfusion_amd", "adapter"),
                        os.path.join(stub, "main_like.cpp"), "-o", exe, "-L", lib, "-lkfx",
                        f"-Wl,-rpath,{lib}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    import torch
    if not torch.cuda.is_available():
        p = subprocess.run([exe], capture_output=True, text=True, timeout=120)
        assert p.returncode == 2 and "kinectfusion:" in p.stderr
