"""Z-slab decomposition of the raycast on the CPU, against the
oracle's single-volume raycast (tsdf_volume.cu:210-260).

Each slab reads only its stored slices (the rest of its array is filled with
garbage, so a read outside the halo would show), ends rays only at owned
samples and reports the deciding sample's index; the combine is the GPU path's:
all-reduce MIN of the keys, clear the pixels a slab lost, all-reduce MAX of
the map bits.  The multi-process variant runs that combine over
torch.distributed (gloo, world_size 2) like bench.py's ranks do over RCCL.
"""
import os
import socket

import numpy as np
import pytest

import oracle as O
from kfx import synth
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


def _combine(parts):
    keys = np.min(np.stack([k for k, _, _ in parts]), axis=0)
    out_v = np.zeros_like(parts[0][1]).view(np.uint32)
    out_n = np.zeros_like(parts[0][2]).view(np.uint32)
    for k, v, n in parts:
        lost = (k != keys)[..., None]
        out_v = np.maximum(out_v, np.where(lost, 0, v.view(np.uint32)))
        out_n = np.maximum(out_n, np.where(lost, 0, n.view(np.uint32)))
    return keys, out_v.view(np.float32), out_n.view(np.float32)


@pytest.fixture(scope="module")
def scene():
    return _scene()


def test_single_slab_equals_raycast(scene):
    I, vol, poses = scene
    cam2vol, Rinv = poses[0]
    k, v, n = O.raycast_slab(vol.tsdf, vol, I, cam2vol, Rinv, 0, DIMS, 0, DIMS)
    rv, rn = O.raycast(vol, I, cam2vol, Rinv)
    assert np.array_equal(v.view(np.uint32), rv.view(np.uint32))
    assert np.array_equal(n.view(np.uint32), rn.view(np.uint32))
    hit = rv[..., 2] != 0
    assert hit.mean() > 0.5 and (k[hit] != np.uint32(0xFFFFFFFF)).all()


@pytest.mark.parametrize("world", [2, 3, 4, 8])
def test_slab_decomposition_serial(world, scene):
    I, vol, poses = scene
    for cam2vol, Rinv in poses:
        parts = []
        for r in range(world):
            t, b = _slab_view(vol, r, world, seed=r)
            parts.append(O.raycast_slab(t, vol, I, cam2vol, Rinv, *b))
        keys, v, n = _combine(parts)
        rv, rn = O.raycast(vol, I, cam2vol, Rinv)
        assert np.array_equal(v.view(np.uint32), rv.view(np.uint32)), (v != rv).sum()
        assert np.array_equal(n.view(np.uint32), rn.view(np.uint32))
        # the decisive events really are spread over several slabs
        winners = [((k == keys) & (keys != 0xFFFFFFFF)).sum() for k, _, _ in parts]
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
        k, v, n = O.raycast_slab(t, vol, I, cam2vol, Rinv, *b)
        keys = torch.from_numpy(k.astype(np.int64))
        dist.all_reduce(keys, op=dist.ReduceOp.MIN)
        lost = (k.astype(np.int64) != keys.numpy())[..., None]
        vb = torch.from_numpy(np.where(lost, 0, v.view(np.uint32)).astype(np.int64))
        nb = torch.from_numpy(np.where(lost, 0, n.view(np.uint32)).astype(np.int64))
        dist.all_reduce(vb, op=dist.ReduceOp.MAX)
        dist.all_reduce(nb, op=dist.ReduceOp.MAX)
        rv, rn = O.raycast(vol, I, cam2vol, Rinv)
        ok &= np.array_equal(vb.numpy().astype(np.uint32), rv.view(np.uint32))
        ok &= np.array_equal(nb.numpy().astype(np.uint32), rn.view(np.uint32))
    dist.destroy_process_group()
    with open(os.path.join(out_dir, f"rank{rank}"), "w") as f:
        f.write("ok" if ok else "mismatch")


def test_slab_decomposition_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    port = _free_port()
    mp.spawn(_rank_main, args=(2, port, str(tmp_path)), nprocs=2, join=True)
    assert [open(tmp_path / f"rank{r}").read() for r in range(2)] == ["ok", "ok"]
