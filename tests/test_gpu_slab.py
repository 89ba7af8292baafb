"""Z-slab sharding on the GPU: a stream split over N slab
contexts must reproduce the single-volume context bit for bit — poses, model
maps of every pyramid level, and every owned voxel record.

On the one-GPU test box the slabs run as an in-process group
(kfx_pipeline_group: the same kernels, the all-reduces done by one kernel over
the members' buffers); the RCCL path is exercised with a one-rank communicator
(the collectives and their stream capture run; multi-rank RCCL needs one GPU per
rank, see tests/test_slab_dist.py for the multi-process decomposition check).
"""
import numpy as np
import pytest

from kfx import KFX_FRAME_PREV, KFX_OK, KFX_TRACKING_LOST, KinectFusion, comm_unique_id, pipeline_group, synth
from kfx.abi import Intrinsics, default_params
import oracle as O

pytestmark = pytest.mark.gpu

L_VOL = 2.048


def bits_equal(a, b):
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.fixture(scope="module")
def seq_qvga():
    return synth.sequence(8, synth.Intrinsics.qvga(), noise=True, dropout=0.01)


def _single(intr, p, bgr, dep):
    kf = KinectFusion(Intrinsics.from_any(intr), p)
    st = [kf.pipeline(bgr[k], dep[k].astype(np.float32)) for k in range(len(dep))]
    return kf, st


def _compare(single, members, levels=3):
    ref_poses = single.pose_record
    t, w, c = single.volume_soa()
    ts, ws, cs = (np.zeros_like(t), np.zeros_like(w), np.zeros_like(c))
    slice_ = single.dims[0] * single.dims[1]
    covered = 0
    for m in members:
        assert np.array_equal(m.pose_record, ref_poses)
        assert m.frame_count == single.frame_count
        for l in range(levels):
            _, gv, gn = single.frame_maps(KFX_FRAME_PREV, l)
            _, mv, mn = m.frame_maps(KFX_FRAME_PREV, l)
            assert bits_equal(mv, gv), f"vmap level {l}: {(mv != gv).sum()} differ"
            assert bits_equal(mn, gn), f"nmap level {l}"
        zb, zn, o0, o1 = m.slab_info()
        mt, mw, mc = m.volume_soa()
        sl = slice(o0 * slice_, o1 * slice_)
        ts[sl], ws[sl] = mt[sl], mw[sl]
        cs[4 * o0 * slice_:4 * o1 * slice_] = mc[4 * o0 * slice_:4 * o1 * slice_]
        covered += o1 - o0
    assert covered == single.dims[2]
    assert np.array_equal(ts, t), f"tsdf: {(ts != t).sum()} voxels differ"
    assert np.array_equal(ws, w) and np.array_equal(cs, c)
    assert w.any()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_slab_group_matches_single_volume(world, seq_qvga):
    bgr, dep, _ = seq_qvga
    intr = synth.Intrinsics.qvga()
    p = default_params(dims=64, range_m=L_VOL)
    single, st = _single(intr, p, bgr, dep)
    members = [KinectFusion(Intrinsics.from_any(intr), p, slab=(r, world)) for r in range(world)]
    for r, m in enumerate(members):
        zb, zn, o0, o1 = m.slab_info()
        assert (zb, zn, o0, o1) == O.slab_bounds(64, r, world)
        assert zb == max(0, o0 - 4) and zb + zn == min(64, o1 + 4)
    gst = [pipeline_group(members, bgr[k], dep[k].astype(np.float32)) for k in range(len(dep))]
    assert gst == st == [KFX_OK] * len(dep)
    _compare(single, members)
    for m in members:
        m.close()
    single.close()


def test_slab_group_vga_128(seq_qvga):
    """640x480 against a 128^3 volume in 2 slabs (the slab boundary at z = 64
    crosses the scene: rays hit surfaces on both sides of it)."""
    bgr, dep, _ = synth.sequence(5, synth.Intrinsics.vga(), noise=True, dropout=0.01)
    intr = synth.Intrinsics.vga()
    p = default_params(dims=128, range_m=L_VOL)
    single, st = _single(intr, p, bgr, dep)
    members = [KinectFusion(Intrinsics.from_any(intr), p, slab=(r, 2)) for r in range(2)]
    gst = [pipeline_group(members, bgr[k], dep[k].astype(np.float32)) for k in range(len(dep))]
    assert gst == st
    _compare(single, members)
    for m in members:
        m.close()
    single.close()


def test_slab_group_tracking_failure(seq_qvga):
    bgr, dep, _ = seq_qvga
    intr = synth.Intrinsics.qvga()
    p = default_params(dims=64, range_m=L_VOL)
    members = [KinectFusion(Intrinsics.from_any(intr), p, slab=(r, 2)) for r in range(2)]
    assert pipeline_group(members, bgr[0], dep[0].astype(np.float32)) == KFX_OK
    assert pipeline_group(members, bgr[1], dep[1].astype(np.float32)) == KFX_OK
    blank = np.zeros_like(dep[2], dtype=np.float32)
    assert pipeline_group(members, bgr[2], blank) == KFX_TRACKING_LOST
    for m in members:
        assert m.frame_count == 1 and m.pose_record.shape == (1, 4, 4)
        t, w, c = m.volume_soa()
        assert not t.any() and not w.any()
        m.close()


@pytest.mark.parametrize("graph", [True, False])
def test_slab_rccl_single_rank_matches(graph, seq_qvga):
    """A one-rank RCCL communicator: the collectives of the slab combine run
    (captured into the per-frame graph when RCCL allows it)."""
    bgr, dep, _ = seq_qvga
    intr = synth.Intrinsics.qvga()
    p = default_params(dims=64, range_m=L_VOL)
    single, st = _single(intr, p, bgr, dep)
    m = KinectFusion(Intrinsics.from_any(intr), p, slab=(0, 1))
    m.comm_init(comm_unique_id())
    m.set_graph_mode(graph)
    gst = [m.pipeline(bgr[k], dep[k].astype(np.float32)) for k in range(len(dep))]
    assert gst == st
    _compare(single, [m])
    m.stage_frames(bgr, dep.astype(np.float32))
    single.stage_frames(bgr, dep.astype(np.float32))
    for k in range(len(dep)):
        m.pipeline_staged(k)
        single.pipeline_staged(k)
    m.synchronize()
    single.synchronize()
    _compare(single, [m])
    m.close()
    single.close()
