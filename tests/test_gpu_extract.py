"""Point-cloud extraction (kfx_extract_points / kfx_save_pointcloud) against
the oracle's FullScan6 restatement (tsdf_volume.cu:307-481): identical point
arrays (bit for bit, canonical order), totals, capped prefixes, slab
concatenation and the PLY text of kinectfusion::savePointcloud."""
import numpy as np
import pytest

import oracle as O
from kfx import KinectFusion, pipeline_group, synth, write_ply
from kfx.abi import Intrinsics, default_params

pytestmark = pytest.mark.gpu

L_VOL = 2.048


@pytest.fixture(scope="module")
def fused():
    intr = synth.Intrinsics.qvga()
    bgr, dep, _ = synth.sequence(5, intr, noise=True, dropout=0.01)
    p = default_params(dims=128, range_m=L_VOL)
    kf = KinectFusion(Intrinsics.from_any(intr), p)
    for k in range(len(dep)):
        kf.pipeline(bgr[k], dep[k].astype(np.float32))
    yield kf, p, (bgr, dep, intr)
    kf.close()


def _oracle_points(kf, p, **kw):
    t, w, _ = kf.volume_soa()
    vol = O.Volume(kf.dims, (L_VOL,) * 3)
    return O.extract_points(vol, p.volu_pose, tsdf=t, weight=w, **kw)


def test_extract_matches_oracle(fused):
    kf, p, _ = fused
    g = kf.extract_points()
    o, n = _oracle_points(kf, p)
    assert n == len(o) > 10000
    assert g.shape == o.shape
    assert np.array_equal(g.view(np.uint32), o.view(np.uint32))


def test_extract_cap_prefix(fused):
    kf, p, _ = fused
    g = kf.extract_points(cap=777)
    o, _ = _oracle_points(kf, p, cap=777)
    assert len(g) == 777 and np.array_equal(g, o)


def test_save_pointcloud_text(fused, tmp_path):
    kf, p, _ = fused
    path = tmp_path / "cloud.ply"
    kf.save_pointcloud(str(path))
    o, _ = _oracle_points(kf, p)
    assert path.read_text() == O.ply_text(o)
    path2 = tmp_path / "w.ply"
    write_ply(str(path2), o[:10])
    assert path2.read_text() == O.ply_text(o[:10])


def test_slab_clouds_concatenate(fused):
    kf, p, (bgr, dep, intr) = fused
    members = [KinectFusion(Intrinsics.from_any(intr), p, slab=(r, 3)) for r in range(3)]
    for k in range(len(dep)):
        pipeline_group(members, bgr[k], dep[k].astype(np.float32))
    parts = [m.extract_points() for m in members]
    assert all(len(x) > 0 for x in parts)
    assert np.array_equal(np.concatenate(parts), kf.extract_points())
    for m in members:
        m.close()


def test_mesh_matches_oracle(fused, tmp_path):
    """Marching cubes on the device vs the oracle on the downloaded volume:
    identical triangle arrays (bit for bit, canonical order), capped prefix,
    slab meshes concatenating to the single volume's, and the PLY mesh text."""
    from kfx import write_ply_mesh
    kf, p, (bgr, dep, intr) = fused
    g = kf.extract_mesh()
    t, w, _ = kf.volume_soa()
    vol = O.Volume(kf.dims, (L_VOL,) * 3)
    o, n = O.extract_mesh(vol, p.volu_pose, tsdf=t, weight=w)
    assert n == len(o) > 10000 and g.shape == o.shape
    assert np.array_equal(g.view(np.uint32), o.view(np.uint32))
    assert np.array_equal(kf.extract_mesh(cap=999), o[:999])
    members = [KinectFusion(Intrinsics.from_any(intr), p, slab=(r, 2)) for r in range(2)]
    for k in range(len(dep)):
        pipeline_group(members, bgr[k], dep[k].astype(np.float32))
    parts = [m.extract_mesh() for m in members]
    assert all(len(x) > 0 for x in parts) and np.array_equal(np.concatenate(parts), g)
    for m in members:
        m.close()
    path = tmp_path / "mesh.ply"
    write_ply_mesh(str(path), o[:3])
    txt = path.read_text().splitlines()
    assert txt[:10] == ["ply", "format ascii 1.0", "element vertex 9", "property float x", "property float y",
                        "property float z", "element face 3", "property list uchar int vertex_indices",
                        "end_header", "%g %g %g" % tuple(float(v) for v in o[0, 0])]
    assert txt[-1] == "3 6 7 8"


@pytest.mark.parametrize("mesh", [False, True])
def test_single_pass_equals_two_pass(mesh, fused):
    """The one-read extraction (count + items into a pool, offset scan, pool
    copy in canonical order) gives the two-pass result (count pass, offset
    scan, emit pass) bit for bit, full and capped (a cap below the total
    overflows the pool and takes the emit pass), and the count-only total."""
    kf, p, _ = fused
    fn = kf.extract_mesh if mesh else kf.extract_points
    one = fn(cap=50_000_000)
    assert kf.extract_ms()["passes"] == 1  # one volume read (pool + copy)
    capped = fn(cap=1234)  # fewer slots than items: the pool overflows, the emit pass writes
    assert kf.extract_ms()["passes"] == 2
    kf.set_extract_passes(2)
    try:
        two = fn(cap=50_000_000)
        ms2 = kf.extract_ms()
        assert ms2["emit"] > 0 and ms2["passes"] == 2
        two_capped = fn(cap=1234)
    finally:
        kf.set_extract_passes(1)
    assert len(one) == kf.extract_count(mesh) > 1000
    assert np.array_equal(one.view(np.uint32), two.view(np.uint32))
    assert np.array_equal(capped.view(np.uint32), two_capped.view(np.uint32)) and len(capped) == 1234
