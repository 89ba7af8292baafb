"""Z-slab decomposition of the raycast on the CPU, against the
oracle's single-volume raycast (tsdf_volume.cu:210-260).

Each slab reads only its stored slices (the rest of its array is filled with
garbage, so a read outside the halo would show), ends rays only at owned
samples and reports the deciding sample's index; the combine is the GPU path's:
all-reduce MIN of the keys, clear the pixels a slab lost, all-reduce MAX of
the payload bits {Ts, nout}, rebuild the maps from the payload.  The
multi-process variant runs that combine over torch.distributed (gloo,
world_size 2) like bench.py's ranks do over RCCL, with libkfx's own host
build of the combine steps (kfx_slab_mask_payload, kfx_slab_expand: the code
the device combine runs, callable without a GPU).
"""
import os
import socket

import numpy as np
import pytest

import oracle as O
from kfx import slab_expand, slab_mask_payload, synth
from kfx.abi import Intrinsics, Pose, default_params

L_VOL = 2.048
DIMS = 64


def _scene():
    intr = synth.Intrinsics.qvga()
    I = Intrinsics.from_any(intr)
    bgr, dep, gt = synth.sequence(6, intr, noise=True, dropout=0.01)
    p = default_params(dims=DIMS, range_m=L_VOL)
    vol = O.Volume((DIMS,) * 3, (L_VOL,) * 3)
    for k in range(3):
        ds, _, _ = O.preprocess(dep[k].astype(np.float32), I, p)
        vol2cam = O.pose_mul(O.pose_inv(Pose.from_matrix(gt[k])), p.volu_pose)
        O.integrate(vol, p.volu_trun_dist, I, vol2cam, ds[0], bgr[k])
    poses = []
    for k in (2, 4, 5):
        cam2vol = O.pose_mul(O.pose_inv(p.volu_pose), Pose.from_matrix(gt[k]))
        poses.append((cam2vol, cam2vol.matrix()[:3, :3].T.copy()))
    return I, vol, poses


def _slab_view(vol, rank, world, seed):
    zb, zn, o0, o1 = O.slab_bounds(DIMS, rank, world)
    t = np.random.default_rng(seed).integers(-32767, 32768, vol.tsdf.size).astype(np.int16)
    s = DIMS * DIMS
    t[zb * s:(zb + zn) * s] = vol.tsdf[zb * s:(zb + zn) * s]
    return t, (zb, zn, o0, o1)


def _payload(ts, nmap):
    """A slab's combine payload: the [Ts | nx | ny | nz] u32 planes."""
    n = ts.size
    pay = np.zeros((4, n), np.uint32)
    pay[0] = ts.ravel().view(np.uint32)
    pay[1:] = nmap.reshape(n, 3).T.view(np.uint32)
    return pay


def _combine(parts, I, cam2vol, Rinv):
    keys = np.min(np.stack([p[0] for p in parts]), axis=0)
    pay = np.zeros((4, keys.size), np.uint32)
    for k, v, n, ts in parts:
        pay = np.maximum(pay, slab_mask_payload(k, keys, _payload(ts, n)))
    v, n = slab_expand(pay, I, cam2vol, Rinv)
    return keys, v, n


@pytest.fixture(scope="module")
def scene():
    return _scene()


def test_single_slab_equals_raycast(scene):
    I, vol, poses = scene
    cam2vol, Rinv = poses[0]
    k, v, n, ts = O.raycast_slab(vol.tsdf, vol, I, cam2vol, Rinv, 0, DIMS, 0, DIMS)
    rv, rn = O.raycast(vol, I, cam2vol, Rinv)
    assert np.array_equal(v.view(np.uint32), rv.view(np.uint32))
    assert np.array_equal(n.view(np.uint32), rn.view(np.uint32))
    hit = rv[..., 2] != 0
    assert hit.mean() > 0.5 and (k[hit] != np.uint32(0xFFFFFFFF)).all()
    # the payload path rebuilds the same maps (libkfx host combine)
    ev, en = slab_expand(_payload(ts, n), I, cam2vol, Rinv)
    assert np.array_equal(ev.view(np.uint32), rv.view(np.uint32))
    assert np.array_equal(en.view(np.uint32), rn.view(np.uint32))


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_slab_decomposition_serial(world, scene):
    I, vol, poses = scene
    for cam2vol, Rinv in poses:
        parts = []
        for r in range(world):
            t, b = _slab_view(vol, r, world, seed=r)
            parts.append(O.raycast_slab(t, vol, I, cam2vol, Rinv, *b))
        keys, v, n = _combine(parts, I, cam2vol, Rinv)
        rv, rn = O.raycast(vol, I, cam2vol, Rinv)
        assert np.array_equal(v.view(np.uint32), rv.view(np.uint32)), (v != rv).sum()
        assert np.array_equal(n.view(np.uint32), rn.view(np.uint32))
        # the decisive events really are spread over several slabs
        winners = [((p[0] == keys) & (keys != 0xFFFFFFFF)).sum() for p in parts]
        assert sum(1 for w in winners if w > 0) >= 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_main(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    I, vol, poses = _scene()
    ok = True
    for cam2vol, Rinv in poses:
        t, b = _slab_view(vol, rank, world, seed=100 + rank)
        k, v, n, ts = O.raycast_slab(t, vol, I, cam2vol, Rinv, *b)
        keys = torch.from_numpy(k.astype(np.int64))
        dist.all_reduce(keys, op=dist.ReduceOp.MIN)
        pay = slab_mask_payload(k, keys.numpy().astype(np.uint32), _payload(ts, n))  # libkfx host combine
        pb = torch.from_numpy(pay.astype(np.int64))
        dist.all_reduce(pb, op=dist.ReduceOp.MAX)
        gv, gn = slab_expand(pb.numpy().astype(np.uint32), I, cam2vol, Rinv)  # libkfx host combine
        rv, rn = O.raycast(vol, I, cam2vol, Rinv)
        ok &= np.array_equal(gv.view(np.uint32), rv.view(np.uint32))
        ok &= np.array_equal(gn.view(np.uint32), rn.view(np.uint32))
    dist.destroy_process_group()
    with open(os.path.join(out_dir, f"rank{rank}"), "w") as f:
        f.write("ok" if ok else "mismatch")


def test_slab_decomposition_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.spawn(_rank_main, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f"rank{r}").read() for r in range(2)] == ["ok", "ok"]
