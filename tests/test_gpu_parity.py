"""GPU-vs-oracle parity through the C-ABI (libkfx.so on an MI355X).

Bar: every stage is bit-identical to the CPU oracle on the
same inputs — float maps compared bit for bit (NaN positions equal), voxel
records / ICP sums / counts exactly equal.  The end-to-end pose tolerance is
stated where it is used (it is 0 when every stage is bit-exact).
"""
import os

import numpy as np
import pytest

import oracle as O
from kfx import KFX_FRAME_CUR, KFX_FRAME_PREV, KFX_OK, KFX_TRACKING_LOST, KfxError, KinectFusion, synth
from kfx.abi import Intrinsics, Pose, default_params

pytestmark = pytest.mark.gpu

L_VOL = 2.048


def feq(a, b):
    """Bit equality of float32 arrays with NaNs compared by position."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    z = np.float32(0)
    return np.array_equal(np.where(na, z, a).view(np.uint32), np.where(nb, z, b).view(np.uint32))


def mismatch(a, b):
    a = np.asarray(a, np.float32).ravel()
    b = np.asarray(b, np.float32).ravel()
    bad = ~((a == b) | (np.isnan(a) & np.isnan(b)))
    return int(bad.sum())


@pytest.fixture(scope="module")
def seq_qvga():
    return synth.sequence(10, synth.Intrinsics.qvga(), noise=True, dropout=0.01)


@pytest.fixture(scope="module")
def seq_vga():
    return synth.sequence(6, synth.Intrinsics.vga(), noise=True, dropout=0.01)


def make(intr, dims=128, **kw):
    p = default_params(dims=dims, range_m=L_VOL)
    for k, v in kw.items():
        setattr(p, k, v)
    return KinectFusion(Intrinsics.from_any(intr), p), p


@pytest.mark.parametrize("which", ["qvga", "vga"])
def test_preprocess_bit_exact(which, seq_qvga, seq_vga):
    bgr, dep, _ = seq_qvga if which == "qvga" else seq_vga
    intr = synth.Intrinsics.qvga() if which == "qvga" else synth.Intrinsics.vga()
    kf, p = make(intr, dims=64)
    I = Intrinsics.from_any(intr)
    for k in (0, 3):
        d = dep[k].astype(np.float32)
        kf.stage_preprocess(bgr[k], d)
        ds, vs, ns = O.preprocess(d, I, p)
        for l in range(3):
            gd, gv, gn = kf.frame_maps(KFX_FRAME_CUR, l)
            assert feq(gd, ds[l]), f"dmap level {l}: {mismatch(gd, ds[l])} px differ"
            assert feq(gv, vs[l]), f"vmap level {l}: {mismatch(gv, vs[l])} differ"
            assert feq(gn, ns[l]), f"nmap level {l}: {mismatch(gn, ns[l])} differ"
    kf.close()


def test_icp_accumulate_bit_exact(seq_vga):
    bgr, dep, gt = seq_vga
    intr = synth.Intrinsics.vga()
    I = Intrinsics.from_any(intr)
    kf, p = make(intr, dims=64)
    prev = O.preprocess(dep[1].astype(np.float32), I, p)
    kf.stage_preprocess(bgr[2], dep[2].astype(np.float32))
    cur = O.preprocess(dep[2].astype(np.float32), I, p)
    for l in range(3):
        kf.set_frame_maps(KFX_FRAME_PREV, l, prev[1][l], prev[2][l])
    rel = (np.linalg.inv(gt[1]) @ gt[2]).astype(np.float32)
    jitter = rel.copy()
    jitter[:3, 3] += [0.003, -0.002, 0.004]
    for pose_m in (np.eye(4, dtype=np.float32), rel, jitter):
        pose = Pose.from_matrix(pose_m)
        for l in range(3):
            g = kf.stage_icp_accumulate(l, pose)
            o = O.icp_accumulate(cur[1][l], cur[2][l], prev[1][l], prev[2][l], I.level(l), pose)
            assert np.array_equal(g, o), f"level {l}: {g - o}"
            assert g[0] > 0
    kf.close()


@pytest.mark.parametrize("dist,angle", [(None, None), (0.004, 8.0), (0.1, 60.0)])
def test_icp_track_matches_oracle(dist, angle, seq_vga):
    """Persistent ICP vs the oracle's kfo_icp_track; besides the defaults, a
    tight and a loose pair of thresholds (the kernel tests x <= sqrt_le_bound(t)
    where the reference tests sqrtf(x) <= t)."""
    import ctypes as C
    from kfx.abi import fptr
    bgr, dep, gt = seq_vga
    intr = synth.Intrinsics.vga()
    I = Intrinsics.from_any(intr)
    kw = {} if dist is None else {"icp_dist_threshold": dist, "icp_angle_threshold": angle}
    kf, p = make(intr, dims=64, **kw)
    prev = O.preprocess(dep[2].astype(np.float32), I, p)
    cur = O.preprocess(dep[3].astype(np.float32), I, p)
    kf.stage_preprocess(bgr[3], dep[3].astype(np.float32))
    for l in range(3):
        kf.set_frame_maps(KFX_FRAME_PREV, l, prev[1][l], prev[2][l])
    rc, gpose = kf.stage_icp()
    PA = C.POINTER(C.c_float) * 3
    opose = Pose()
    st = O.lib().kfo_icp_track(PA(*[fptr(a) for a in cur[1]]), PA(*[fptr(a) for a in cur[2]]),
                               PA(*[fptr(a) for a in prev[1]]), PA(*[fptr(a) for a in prev[2]]),
                               C.byref(I), C.byref(p), C.byref(opose))
    assert (rc == KFX_OK) == (st == 0), (rc, st)
    if dist is None:
        assert st == 0
    # the double cos/sin of the Rodrigues step are the only non-IEEE-basic ops
    if st == 0:
        assert np.abs(gpose.matrix() - opose.matrix()).max() == 0
    kf.close()


def test_icp_track_720p_strided_matches_oracle():
    """1280x720 (C5's frames): level 0 has more pixel groups than the persistent
    grid holds co-resident, so blocks take several groups (k_icp_track<true>);
    the int64 sums, and so the pose, still match the oracle's kfo_icp_track.
    The persistent kernel must be the one that ran (no per-iteration fallback)."""
    import ctypes as C
    from kfx.abi import fptr
    intr = synth.Intrinsics.hd720()
    bgr, dep, gt = synth.sequence(4, intr, noise=True, dropout=0.01)
    I = Intrinsics.from_any(intr)
    kf, p = make(intr, dims=64)
    prev = O.preprocess(dep[1].astype(np.float32), I, p)
    cur = O.preprocess(dep[2].astype(np.float32), I, p)
    kf.stage_preprocess(bgr[2], dep[2].astype(np.float32))
    for l in range(3):
        kf.set_frame_maps(KFX_FRAME_PREV, l, prev[1][l], prev[2][l])
    rc, gpose = kf.stage_icp()
    PA = C.POINTER(C.c_float) * 3
    opose = Pose()
    st = O.lib().kfo_icp_track(PA(*[fptr(a) for a in cur[1]]), PA(*[fptr(a) for a in cur[2]]),
                               PA(*[fptr(a) for a in prev[1]]), PA(*[fptr(a) for a in prev[2]]),
                               C.byref(I), C.byref(p), C.byref(opose))
    assert rc == KFX_OK and st == 0
    assert np.abs(gpose.matrix() - opose.matrix()).max() == 0
    assert kf.set_icp_persistent(False)  # True: the persistent path was the one in use
    kf.close()


def _vol_equal(kf, vol):
    t, w, c = kf.volume_soa()
    assert np.array_equal(t, vol.tsdf), f"tsdf: {(t != vol.tsdf).sum()} voxels differ"
    assert np.array_equal(w, vol.weight), f"weight: {(w != vol.weight).sum()} voxels differ"
    assert np.array_equal(c, vol.rgb), f"rgb: {(c != vol.rgb).sum()} bytes differ"


def test_integrate_bit_exact_128(seq_qvga):
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    I = Intrinsics.from_any(intr)
    kf, p = make(intr, dims=128)
    vol = O.Volume((128,) * 3, (L_VOL,) * 3)
    for k in (0, 1, 2):
        d = dep[k].astype(np.float32)
        kf.stage_preprocess(bgr[k], d)
        ds, _, _ = O.preprocess(d, I, p)
        cam = Pose.from_matrix(gt[k])
        vol2cam = O.pose_mul(O.pose_inv(cam), p.volu_pose)
        gu, gc = kf.stage_integrate(vol2cam)
        ou, oc = O.integrate(vol, p.volu_trun_dist, I, vol2cam, ds[0], bgr[k])
        assert (gu, gc) == (ou, oc)
        assert ou > 0 and oc > 0
        _vol_equal(kf, vol)
    kf.close()


@pytest.mark.parametrize("n", [512, 1024])
def test_integrate_512_column_spot_check(n, seq_vga):
    """Full BASELINE sizes (C2 512^3 @ 4 mm; C3 1024^3 @ 2 mm, 2^30 voxels on
    the 32-bit-offset path): GPU volume vs the oracle on 3000 sampled columns
    (the oracle restates any column independently)."""
    bgr, dep, gt = seq_vga
    intr = synth.Intrinsics.vga()
    I = Intrinsics.from_any(intr)
    kf, p = make(intr, dims=n)
    d = dep[0].astype(np.float32)
    kf.stage_preprocess(bgr[0], d)
    ds, _, _ = O.preprocess(d, I, p)
    vol2cam = p.volu_pose
    gu, gc = kf.stage_integrate(vol2cam)
    t, w, c = kf.volume_soa()
    rng = np.random.default_rng(5)
    cols = np.stack([rng.integers(0, n, 3000), rng.integers(0, n, 3000)], 1).astype(np.int32)
    cols = np.concatenate([cols, np.array([[n // 2, n // 2], [0, 0], [n - 1, n - 1], [n // 2 - 1, 300]], np.int32)])
    cols = np.unique(cols, axis=0)  # a repeated column would be integrated twice
    vol = O.Volume((n,) * 3, (L_VOL,) * 3)
    O.integrate(vol, p.volu_trun_dist, I, vol2cam, ds[0], bgr[0], cols=cols)
    idx = (cols[:, 0][None, :] + n * cols[:, 1][None, :] + n * n * np.arange(n, dtype=np.int64)[:, None]).ravel()
    assert np.array_equal(t[idx], vol.tsdf[idx])
    assert np.array_equal(w[idx], vol.weight[idx])
    c4 = c.reshape(-1, 4)
    assert np.array_equal(c4[idx], vol.rgb.reshape(-1, 4)[idx])
    assert (w[idx] > 0).sum() > 10000
    # counts: total over the volume equals the per-column oracle sum where computed in full
    assert gu > 0 and 0 < gc < gu
    kf.close()


def test_c3_pipeline_two_frames_match_oracle(seq_vga):
    """BASELINE C3 at full size (640x480, 1024^3 @ 2 mm, 2^30 voxels on the
    32-bit-offset path) through the whole pipeline: the bootstrap frame and one
    tracked frame (19 ICP iterations against the 1024^3 raycast), against the
    serial oracle's pipeline (8 GiB of host volume).  Poses, every level of the
    raycast model maps, and 3000 sampled columns of the volume."""
    bgr, dep, _ = seq_vga
    intr = synth.Intrinsics.vga()
    I = Intrinsics.from_any(intr)
    n = 1024
    kf, p = make(intr, dims=n)
    pipe = O.Pipeline(I, p)
    for k in range(2):
        d = dep[k].astype(np.float32)
        assert kf.pipeline(bgr[k], d) == pipe.process(bgr[k], d) == KFX_OK
    gp, op = kf.pose_record, pipe.poses()
    assert gp.shape == op.shape == (2, 4, 4)
    err = np.abs(gp - op).max()
    assert err == 0, err  # bit-exact: every stage, the Rodrigues cos/sin included
    for l in range(3):
        _, gv, gn = kf.frame_maps(KFX_FRAME_PREV, l)
        assert feq(gv, pipe.map(1, 1, l)), f"vmap level {l}: {mismatch(gv, pipe.map(1, 1, l))} differ"
        assert feq(gn, pipe.map(1, 2, l)), f"nmap level {l}"
    rng = np.random.default_rng(11)
    cols = np.unique(np.stack([rng.integers(0, n, 3000), rng.integers(0, n, 3000)], 1).astype(np.int32), axis=0)
    gt_, gw, gc = kf.download_columns(cols)
    ot, ow, oc = pipe.volume()
    idx = (cols[:, 0][:, None] + n * cols[:, 1][:, None] + n * n * np.arange(n, dtype=np.int64)[None, :])
    assert np.array_equal(gt_, ot[idx]) and np.array_equal(gw, ow[idx])
    assert np.array_equal(gc.reshape(-1, n, 4), oc.reshape(-1, 4)[idx])
    assert (gw > 0).sum() > 10000
    kf.close()


@pytest.mark.timeout(600)
def test_720p_pipeline_matches_oracle():
    """C5's frame size (1280x720) through the whole pipeline against the
    serial oracle: 512^3 @ 8 mm (L = 4.096 m, C5's volume extent), 4 frames.
    This pins the A2 ICP floor grid at 720p (rows 704 / 352 / 160 of 720 / 360
    / 180; rigid_icp.cu:135-139), the strided persistent ICP (k_icp_track<true>:
    level 0 has more pixel groups than the co-resident grid), and the 720p
    raycast + resize.  Poses identical, every level of the
    raycast model maps bit for bit, and the whole volume bit for bit."""
    intr = synth.Intrinsics.hd720()
    L = 4.096
    bgr, dep, _ = synth.sequence(4, intr, L=L, noise=True, dropout=0.01)
    I = Intrinsics.from_any(intr)
    p = default_params(dims=512, range_m=L)
    kf = KinectFusion(I, p)
    pipe = O.Pipeline(I, p)
    for k in range(len(dep)):
        d = dep[k].astype(np.float32)
        assert kf.pipeline(bgr[k], d) == pipe.process(bgr[k], d) == KFX_OK, k
    gp, op = kf.pose_record, pipe.poses()
    assert gp.shape == op.shape == (len(dep), 4, 4)
    err = float(np.abs(gp - op).max())
    assert err == 0, err
    assert np.abs(gp[-1] - np.eye(4)).max() > 1e-3  # the camera moved: ICP did work
    for l in range(3):
        _, gv, gn = kf.frame_maps(KFX_FRAME_PREV, l)
        assert feq(gv, pipe.map(1, 1, l)), f"vmap level {l}: {mismatch(gv, pipe.map(1, 1, l))} differ"
        assert feq(gn, pipe.map(1, 2, l)), f"nmap level {l}: {mismatch(gn, pipe.map(1, 2, l))} differ"
    t, w, c = kf.volume_soa()
    ot, ow, oc = pipe.volume()
    assert np.array_equal(t, ot), f"tsdf: {(t != ot).sum()} voxels differ"
    assert np.array_equal(w, ow), f"weight: {(w != ow).sum()} voxels differ"
    assert np.array_equal(c, oc), f"rgb: {(c != oc).sum()} bytes differ"
    assert (w > 0).sum() > 100000
    assert kf.set_icp_persistent(False)  # True: the (strided) persistent ICP was the path in use
    kf.close()


@pytest.mark.timeout(480)
def test_c4_geometry_pipeline_matches_oracle():
    """BASELINE C4's single volume (640x480, 1024^3 @ 2 mm: 2^30 voxels, the
    geometry the 8-slab split reproduces) through the whole pipeline against
    the serial oracle, 2 frames (bootstrap + one tracked: ICP over the 1024^3
    raycast maps): the tracked pose (identical), every level
    of the raycast model maps bit for bit, and 4000 volume columns bit for bit
    (the oracle's 8.6 GB volume is read in place).  The oracle takes about 30 s
    a frame at this size."""
    intr = synth.Intrinsics.vga()
    I = Intrinsics.from_any(intr)
    n = 1024
    bgr, dep, _ = synth.sequence(2, intr, L=L_VOL, noise=True, dropout=0.005)
    p = default_params(dims=n, range_m=L_VOL)
    kf = KinectFusion(I, p)
    pipe = O.Pipeline(I, p)
    for k in range(2):
        d = dep[k].astype(np.float32)
        assert kf.pipeline(bgr[k], d) == KFX_OK, k
        print(f"frame {k}: oracle", flush=True)
        assert pipe.process(bgr[k], d) == KFX_OK, k
    gp, op = kf.pose_record, pipe.poses()
    assert gp.shape == op.shape == (2, 4, 4)
    err = float(np.abs(gp - op).max())
    assert err == 0, err
    for l in range(3):
        _, gv, gn = kf.frame_maps(KFX_FRAME_PREV, l)
        assert feq(gv, pipe.map(1, 1, l)), f"vmap level {l}: {mismatch(gv, pipe.map(1, 1, l))} differ"
        assert feq(gn, pipe.map(1, 2, l)), f"nmap level {l}: {mismatch(gn, pipe.map(1, 2, l))} differ"
    rng = np.random.default_rng(5)
    cols = np.unique(np.stack([rng.integers(0, n, 4000), rng.integers(0, n, 4000)], 1).astype(np.int32), axis=0)
    gt_, gw, gc = kf.download_columns(cols)
    kf.close()
    ot = np.ctypeslib.as_array(O.lib().kfo_pipe_tsdf(pipe.h), shape=(pipe.nvox,))
    ow = np.ctypeslib.as_array(O.lib().kfo_pipe_weight(pipe.h), shape=(pipe.nvox,))
    oc = np.ctypeslib.as_array(O.lib().kfo_pipe_rgb(pipe.h), shape=(4 * pipe.nvox,)).reshape(-1, 4)
    idx = (cols[:, 0][:, None].astype(np.int64) + n * cols[:, 1][:, None].astype(np.int64)
           + n * n * np.arange(n, dtype=np.int64)[None, :])
    assert np.array_equal(gt_, ot[idx]), f"tsdf: {(gt_ != ot[idx]).sum()} differ"
    assert np.array_equal(gw, ow[idx]), f"weight: {(gw != ow[idx]).sum()} differ"
    assert np.array_equal(gc, oc[idx]), "rgb differs"
    assert (gw > 0).sum() > 10000


@pytest.mark.timeout(600)
def test_c5_geometry_poses_match_oracle():
    """BASELINE C5's single volume (1280x720, 2048^3 @ 2 mm: 2^33 voxels, the
    64-bit-index integrate and raycast) through the whole pipeline against the
    serial oracle (69 GB of host memory), 2 frames: the tracked pose computed
    by the GPU's own ICP over its own 2048^3 raycast (bit-exact) and every level of the raycast model maps bit for bit.  About
    140 s on the GPU box (the oracle), so opt-in: a silent test that long can
    pass for a hung one."""
    intr = synth.Intrinsics.hd720()
    I = Intrinsics.from_any(intr)
    L = 4.096
    bgr, dep, _ = synth.sequence(2, intr, L=L, noise=True, dropout=0.005)
    p = default_params(dims=2048, range_m=L)
    kf = KinectFusion(I, p)
    pipe = O.Pipeline(I, p)
    for k in range(2):
        d = dep[k].astype(np.float32)
        assert kf.pipeline(bgr[k], d) == KFX_OK, k
        print(f"frame {k}: oracle", flush=True)
        assert pipe.process(bgr[k], d) == KFX_OK, k
    gp, op = kf.pose_record, pipe.poses()
    assert gp.shape == op.shape == (2, 4, 4)
    err = float(np.abs(gp - op).max())
    assert err == 0, err
    for l in range(3):
        _, gv, gn = kf.frame_maps(KFX_FRAME_PREV, l)
        assert feq(gv, pipe.map(1, 1, l)), f"vmap level {l}: {mismatch(gv, pipe.map(1, 1, l))} differ"
        assert feq(gn, pipe.map(1, 2, l)), f"nmap level {l}: {mismatch(gn, pipe.map(1, 2, l))} differ"
    kf.close()
    del pipe  # the oracle's 69 GB volume


def test_raycast_bit_exact(seq_qvga):
    """The raycast against the oracle's (tsdf_volume.cu:210-260) at every map
    level."""
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    I = Intrinsics.from_any(intr)
    kf, p = make(intr, dims=128)
    vol = O.Volume((128,) * 3, (L_VOL,) * 3)
    for k in (0, 1, 2):
        d = dep[k].astype(np.float32)
        kf.stage_preprocess(bgr[k], d)
        ds, _, _ = O.preprocess(d, I, p)
        vol2cam = O.pose_mul(O.pose_inv(Pose.from_matrix(gt[k])), p.volu_pose)
        kf.stage_integrate(vol2cam, counts=False)
        O.integrate(vol, p.volu_trun_dist, I, vol2cam, ds[0], bgr[k])
    for k in (2, 4):
        cam2vol = O.pose_mul(O.pose_inv(p.volu_pose), Pose.from_matrix(gt[k]))
        Rinv = cam2vol.matrix()[:3, :3].T.copy()
        kf.stage_raycast(cam2vol, Rinv)
        ov, on = O.raycast(vol, I, cam2vol, Rinv)
        _, gv, gn = kf.frame_maps(KFX_FRAME_PREV, 0)
        assert feq(gv, ov), f"vmap: {mismatch(gv, ov)} differ"
        assert feq(gn, on), f"nmap: {mismatch(gn, on)} differ"
        assert (ov[..., 2] > 0).mean() > 0.5
        for l in (1, 2):
            ov, on = O.resize_points_normals(ov, on)
            _, gv, gn = kf.frame_maps(KFX_FRAME_PREV, l)
            assert feq(gv, ov) and feq(gn, on), f"level {l}"
    kf.close()


def _run_pipeline(kf, bgr, dep, u16=False):
    st = []
    for k in range(len(dep)):
        st.append(kf.pipeline(bgr[k], dep[k] if u16 else dep[k].astype(np.float32)))
    return st


@pytest.mark.parametrize("which", ["qvga", "vga"])
def test_pipeline_matches_oracle(which, seq_qvga, seq_vga):
    bgr, dep, gt = seq_qvga if which == "qvga" else seq_vga
    intr = synth.Intrinsics.qvga() if which == "qvga" else synth.Intrinsics.vga()
    I = Intrinsics.from_any(intr)
    kf, p = make(intr, dims=128)
    st = _run_pipeline(kf, bgr, dep)
    pipe = O.Pipeline(I, p)
    ost = [pipe.process(bgr[k], dep[k].astype(np.float32)) for k in range(len(dep))]
    assert st == ost == [KFX_OK] * len(dep)
    assert kf.frame_count == pipe.frame_count == len(dep) + 1
    gp, op = kf.pose_record, pipe.poses()
    assert gp.shape == op.shape == (len(dep), 4, 4)
    # bar: every stage bit-exact, so the poses are identical (0 difference)
    err = np.abs(gp - op).max()
    assert err == 0, err
    t, w, c = kf.volume_soa()
    ot, ow, oc = pipe.volume()
    assert np.array_equal(t, ot) and np.array_equal(w, ow) and np.array_equal(c, oc)
    for l in range(3):
        _, gv, gn = kf.frame_maps(KFX_FRAME_PREV, l)
        assert feq(gv, pipe.map(1, 1, l)) and feq(gn, pipe.map(1, 2, l))
    kf.close()


def test_pipeline_modes_and_inputs_identical(seq_qvga):
    """graph / eager / profiled launches, u16 / f32 / staged inputs (overlapped
    staged frames replayed as graphs or launched eagerly) and the persistent vs
    per-iteration ICP launches all give the same poses and volume."""
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    res = []
    for mode in ("graph", "eager", "profile", "u16", "staged", "staged_eager", "staged_full",
                 "staged_graph", "staged_mixed", "staged_per_iter", "icp_per_iter", "icp_coop",
                 "staged_coop", "staged_events", "staged_mixed_back", "async"):
        if mode == "staged_events":  # overlapped frames ordered by events, not the raycast start signal
            os.environ["KFX_STREAM_SIGNAL"] = "0"
        try:
            kf, p = make(intr, dims=64)
        finally:
            os.environ.pop("KFX_STREAM_SIGNAL", None)
        if mode == "staged_graph":  # staged frames without the two-stream overlap
            kf.set_frame_overlap(False)
        if mode in ("eager", "staged_eager"):  # staged_eager: overlapped frames launched eagerly
            kf.set_graph_mode(False)
        if mode == "staged_full":  # overlapped frames: ICP/integrate/raycast replayed as a graph too
            with pytest.raises(KfxError):
                kf.set_graph_mode(3)  # modes are 0, 1, 2
            kf.set_graph_mode(2)
        if mode in ("icp_per_iter", "staged_per_iter"):
            assert kf.set_icp_persistent(False)  # persistent path was the one in use
            kf.set_graph_mode(False)
        if mode in ("icp_coop", "staged_coop"):  # cooperative launch of the persistent ICP
            assert kf.set_icp_persistent(2)
        if mode == "profile":
            kf.set_profiling(True)
        if mode in ("staged", "staged_eager", "staged_full", "staged_graph", "staged_per_iter",
                    "staged_coop", "staged_events"):
            kf.stage_frames(bgr, dep.astype(np.float32))
            for k in range(len(dep)):
                kf.pipeline_staged(k)
            kf.synchronize()
        elif mode == "staged_mixed":  # overlapped frames, then single-stream host frames
            kf.stage_frames(bgr, dep.astype(np.float32))
            half = 5  # odd: the last overlapped frame used set 1, the host frames set 0
            for k in range(half):
                kf.pipeline_staged(k)
            for k in range(half, len(dep)):
                kf.pipeline(bgr[k], dep[k].astype(np.float32))
        elif mode == "staged_mixed_back":  # overlapped, single-stream, overlapped again
            kf.stage_frames(bgr, dep.astype(np.float32))
            for k in range(3):
                kf.pipeline_staged(k)
            for k in range(3, 6):
                kf.pipeline(bgr[k], dep[k].astype(np.float32))
            for k in range(6, len(dep)):
                kf.pipeline_staged(k)
            kf.synchronize()
        elif mode == "async":  # pipelined host input through the pinned ring
            for k in range(len(dep)):
                kf.pipeline_async(bgr[k], dep[k].astype(np.float32))
            kf.synchronize()
        else:
            _run_pipeline(kf, bgr, dep, u16=(mode == "u16"))
        if mode == "profile":
            ms = kf.stage_ms()
            assert ms["total"] > 0 and ms["integrate"] > 0
        res.append((kf.pose_record, kf.volume_soa()))
        kf.close()
    for poses, vol in res[1:]:
        assert np.array_equal(poses, res[0][0])
        for a, b in zip(vol, res[0][1]):
            assert np.array_equal(a, b)


def test_icp_watchdog_stall_switches_to_cooperative_launch(seq_qvga):
    """A persistent-ICP grid barrier that never completes (test hook: block 0
    withholds its first arrival) fires the watchdog: that frame reports an
    error and is dropped with a volume reset (as on a tracking loss); later
    frames run the persistent ICP through a cooperative launch and track again,
    with graphs and with staged overlapped frames."""
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    kf, p = make(intr, dims=64)
    assert kf.set_icp_persistent(True)
    for k in range(3):
        assert kf.pipeline(bgr[k], dep[k].astype(np.float32)) == KFX_OK
    kf.debug_force_icp_stall()
    with pytest.raises(KfxError, match="cooperative"):
        kf.pipeline(bgr[3], dep[3].astype(np.float32))
    n = kf.pose_record.shape[0]
    for k in range(4, 7):
        assert kf.pipeline(bgr[k], dep[k].astype(np.float32)) == KFX_OK
    kf.stage_frames(bgr, dep.astype(np.float32))
    for k in range(7, len(dep)):
        kf.pipeline_staged(k)
    assert kf.synchronize() == KFX_OK
    # the stalled frame is an ICP failure (reset, like the reference's failed
    # rigidTransform): the oracle with a failing (blank) frame 3 gives the same poses
    I = Intrinsics.from_any(intr)
    pipe = O.Pipeline(I, p)
    for k in range(len(dep)):
        d = dep[k].astype(np.float32) if k != 3 else np.zeros_like(dep[k], dtype=np.float32)
        pipe.process(bgr[k], d)
    op = pipe.poses()
    assert kf.pose_record.shape == op.shape and n == 1
    assert np.abs(kf.pose_record - op).max() == 0
    kf.close()


def test_tracking_failure_resets_like_reference(seq_qvga):
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    kf, p = make(intr, dims=64)
    assert kf.pipeline(bgr[0], dep[0].astype(np.float32)) == KFX_OK
    assert kf.pipeline(bgr[1], dep[1].astype(np.float32)) == KFX_OK
    blank = np.zeros_like(dep[2], dtype=np.float32)
    assert kf.pipeline(bgr[2], blank) == KFX_TRACKING_LOST
    assert kf.frame_count == 1
    assert kf.pose_record.shape == (1, 4, 4)
    t, w, c = kf.volume_soa()
    assert not t.any() and not w.any() and not c.any()
    # next frame bootstraps again (kinectfusion.cpp:84-93)
    assert kf.pipeline(bgr[3], dep[3].astype(np.float32)) == KFX_OK
    assert kf.frame_count == 2
    assert kf.volume_soa()[1].any()
    kf.close()


def test_staged_tracking_failure_reported_by_synchronize(seq_qvga):
    """Staged (device-input, overlapped) frames return without a host sync; the
    drop of a frame by a tracking failure is reported by kfx_synchronize
    (ADVICE r1), once, and the state equals the host-frame path's."""
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    frames = dep[:4].astype(np.float32).copy()
    frames[2] = 0.0  # no depth: ICP det check fails -> reset(), frame dropped
    kf, p = make(intr, dims=64)
    kf.stage_frames(bgr[:4], frames)
    assert kf.synchronize() == KFX_OK
    for k in range(4):
        kf.pipeline_staged(k)
    assert kf.synchronize() == KFX_TRACKING_LOST
    assert kf.synchronize() == KFX_OK  # reported once
    assert kf.frame_count == 2 and kf.pose_record.shape == (1, 4, 4)
    ref, _ = make(intr, dims=64)
    st = [ref.pipeline(bgr[k], frames[k]) for k in range(4)]
    assert st == [KFX_OK, KFX_OK, KFX_TRACKING_LOST, KFX_OK]
    for a, b in zip(kf.volume_soa(), ref.volume_soa()):
        assert np.array_equal(a, b)
    kf.close()
    ref.close()


@pytest.mark.parametrize("u16", [False, True])
def test_async_host_input_matches_staged(u16, seq_qvga):
    """kfx_pipeline_async (pinned ring + H2D on a copy stream, no per-frame host
    sync; more frames than ring slots, a dropped frame among them) gives the
    staged path's poses and volume bit for bit, and reports the drop once; with
    graph modes 1, 2 and 0 on the ring, registered and odd-address inputs."""
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    frames = dep.astype(np.uint16 if u16 else np.float32).copy()
    frames[6] = 0  # tracking failure: reset(), frame dropped
    kf, p = make(intr, dims=64)
    for k in range(len(frames)):
        kf.pipeline_async(bgr[k], frames[k])
    assert kf.synchronize() == KFX_TRACKING_LOST
    assert kf.synchronize() == KFX_OK
    # zero copy: the same frames uploaded straight from registered host buffers
    zc, _ = make(intr, dims=64)
    zc.set_graph_mode(2)  # the ring slots' frames replay both graphs (kf: preprocess graph)
    hb = np.ascontiguousarray(bgr)
    zc.register_host_buffer(hb)
    zc.register_host_buffer(frames)
    for k in range(len(frames)):
        zc.pipeline_async(hb[k], frames[k])
    assert zc.synchronize() == KFX_TRACKING_LOST
    zc.unregister_host_buffer(hb)
    with pytest.raises(KfxError):
        zc.unregister_host_buffer(hb)
    # registered colour frames at an odd address (the fetch kernel's byte path)
    raw = np.empty(hb.nbytes + 16, np.uint8)
    hu = raw[3:3 + hb.nbytes].reshape(hb.shape)
    hu[...] = hb
    un, _ = make(intr, dims=64)
    un.set_graph_mode(0)  # eager launches
    fu = frames.copy()  # (a page range is registered by one context at a time)
    un.register_host_buffer(hu)
    un.register_host_buffer(fu)
    for k in range(len(frames)):
        un.pipeline_async(hu[k], fu[k])
    assert un.synchronize() == KFX_TRACKING_LOST
    ref, _ = make(intr, dims=64)
    ref.stage_frames(bgr, frames.astype(np.float32))
    for k in range(len(frames)):
        ref.pipeline_staged(k)
    assert ref.synchronize() == KFX_TRACKING_LOST
    assert np.array_equal(kf.pose_record, ref.pose_record) and kf.frame_count == ref.frame_count
    assert np.array_equal(zc.pose_record, ref.pose_record) and zc.frame_count == ref.frame_count
    assert np.array_equal(un.pose_record, ref.pose_record) and un.frame_count == ref.frame_count
    for a, b, z, u in zip(kf.volume_soa(), ref.volume_soa(), zc.volume_soa(), un.volume_soa()):
        assert np.array_equal(a, b) and np.array_equal(z, b) and np.array_equal(u, b)
    kf.close()
    zc.close()
    un.close()
    ref.close()


def test_tsdf_record_export_roundtrip(seq_qvga):
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    kf, p = make(intr, dims=64)
    _run_pipeline(kf, bgr[:3], dep[:3])
    rec = kf.download_tsdf()
    t, w, c = kf.volume_soa()
    assert np.array_equal(rec["tsdf"], t) and np.array_equal(rec["weight"], w)
    assert np.array_equal(rec["rgb"], c.reshape(-1, 4)[:, :3]) and not rec["pad"].any()
    kf2, _ = make(intr, dims=64)
    kf2.upload_tsdf(rec)
    assert np.array_equal(kf2.download_tsdf().view(np.uint64), rec.view(np.uint64))
    kf.close()
    kf2.close()


def test_poses_txt_matches_oracle_writer(seq_qvga, tmp_path):
    bgr, dep, gt = seq_qvga
    kf, p = make(synth.Intrinsics.qvga(), dims=64)
    _run_pipeline(kf, bgr[:4], dep[:4])
    path = tmp_path / "poses.txt"
    kf.write_poses_txt(str(path))
    exp = "".join(O.format_pose(Pose.from_matrix(m)) for m in kf.pose_record)
    assert path.read_text() == exp
    kf.close()


def test_full_size_pipeline_512(seq_vga):
    """BASELINE C2 geometry (640x480, 512^3 @ 4 mm): GPU pipeline vs the oracle
    pipeline on the same frames (the oracle runs ~seconds per frame)."""
    bgr, dep, gt = seq_vga
    n = 4
    intr = synth.Intrinsics.vga()
    kf, p = make(intr, dims=512)
    st = _run_pipeline(kf, bgr[:n], dep[:n])
    assert st == [KFX_OK] * n
    pipe = O.Pipeline(Intrinsics.from_any(intr), p)
    for k in range(n):
        assert pipe.process(bgr[k], dep[k].astype(np.float32)) == 0
    gp, op = kf.pose_record, pipe.poses()
    assert np.abs(gp - op).max() == 0
    # A3 bias bounds accuracy to ~2 voxels (8 mm) against the analytic truth
    assert np.abs(gp[:, :3, 3] - gt[:n, :3, 3]).max() < 0.012
    kf.close()


def test_render_matches_oracle(seq_qvga):
    """getRenderMap(PHONG / NORMAL) on the device vs kfo_render on the same
    previous-frame maps: after frame 1 (the measured maps, NaN normals) and
    after tracking frames (raycast maps)."""
    bgr, dep, gt = seq_qvga
    intr = synth.Intrinsics.qvga()
    kf, p = make(intr, dims=64)
    for k in range(4):
        kf.pipeline(bgr[k], dep[k].astype(np.float32))
        _, v, n = kf.frame_maps(KFX_FRAME_PREV, 0)
        eye = kf.pose_record[-1][:3, 3].astype(np.float32)
        for kind in ("phong", "normal"):
            got = kf.render(kind)
            want = O.render(v, n, eye, kind)
            assert np.array_equal(got, want), (k, kind, int((got != want).sum()))
        assert (kf.render("phong") > 0).any()
    kf.close()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("which", ["qvga128", "vga512"])
def test_index64_kernels_match_oracle(which, seq_qvga, seq_vga):
    """The 64-bit-index kernels (k_integrate<.., false>, k_raycast<false, ..>:
    the path a volume of >= 2^31 stored voxels takes, A9 — the reference's
    int32 index overflows there, device_utils.cuh:31, tsdf_volume.cpp:24)
    forced at sizes the oracle runs (kfx_debug_force_index64): 128^3 QVGA and
    BASELINE C2 (640x480, 512^3 @ 4 mm) through the whole pipeline against
    O.Pipeline — poses, every level of the raycast model maps and the whole
    volume bit for bit.  Poses identical (0 difference, as everywhere)."""
    if which == "qvga128":
        bgr, dep, _ = seq_qvga
        intr, dims, n = synth.Intrinsics.qvga(), 128, 6
    else:
        bgr, dep, _ = seq_vga
        intr, dims, n = synth.Intrinsics.vga(), 512, 3
    I = Intrinsics.from_any(intr)
    kf, p = make(intr, dims=dims)
    kf.debug_force_index64(True)
    pipe = O.Pipeline(I, p)
    for k in range(n):
        d = dep[k].astype(np.float32)
        assert kf.pipeline(bgr[k], d) == pipe.process(bgr[k], d) == KFX_OK, k
    gp, op = kf.pose_record, pipe.poses()
    assert gp.shape == op.shape == (n, 4, 4)
    err = float(np.abs(gp - op).max())
    assert err == 0, err
    assert np.abs(gp[-1] - np.eye(4)).max() > 1e-3  # tracked frames: the raycast maps fed ICP
    for l in range(3):
        _, gv, gn = kf.frame_maps(KFX_FRAME_PREV, l)
        assert feq(gv, pipe.map(1, 1, l)), f"vmap level {l}: {mismatch(gv, pipe.map(1, 1, l))} differ"
        assert feq(gn, pipe.map(1, 2, l)), f"nmap level {l}: {mismatch(gn, pipe.map(1, 2, l))} differ"
    t, w, c = kf.volume_soa()
    ot, ow, oc = pipe.volume()
    assert np.array_equal(t, ot), f"tsdf: {(t != ot).sum()} voxels differ"
    assert np.array_equal(w, ow), f"weight: {(w != ow).sum()} voxels differ"
    assert np.array_equal(c, oc), f"rgb: {(c != oc).sum()} bytes differ"
    assert (w > 0).sum() > 10000
    # the switch is per context and reversible: the 32-bit kernels continue the same stream identically
    kf.debug_force_index64(False)
    d = dep[n].astype(np.float32)
    assert kf.pipeline(bgr[n], d) == pipe.process(bgr[n], d) == KFX_OK
    assert np.abs(kf.pose_record - pipe.poses()).max() == 0
    kf.close()
