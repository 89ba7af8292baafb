"""Marching cubes (§8 f5) on the oracle, CPU: the derived triangle table
against its defining properties, and meshes of analytic SDF volumes against
topology (closed, consistently oriented, Euler characteristic) and geometry.
The reference has no mesh extraction, so these are the pins; the GPU kernel is
compared with this oracle bit for bit in tests/test_gpu_extract.py."""
import collections

import numpy as np
import pytest

import oracle as O
from kfx.abi import Pose

EDGES = [(c, c | (1 << a)) for a in range(3) for c in range(8) if not (c >> a) & 1]


def test_table_properties(oracle_lib):
    tab = O.mc_table()
    assert tab[0, 0] == 0 and tab[255, 0] == 0
    assert tab[:, 0].max() == 5
    for pat in range(256):
        inside = [(pat >> c) & 1 for c in range(8)]
        cut = {e for e, (u, v) in enumerate(EDGES) if inside[u] != inside[v]}
        n = tab[pat, 0]
        used = set(tab[pat, 1:1 + 3 * n].tolist())
        assert used == cut, pat
        # every cut edge is a vertex of the loop fan; loops of k edges give k-2 triangles
        tris = tab[pat, 1:1 + 3 * n].reshape(-1, 3)
        assert all(len(set(t)) == 3 for t in tris)


def _sdf_volume(n, centres, radius, trunc_vox=3.0):
    g = np.arange(n, dtype=np.float64) + 0.5
    z, y, x = np.meshgrid(g, g, g, indexing="ij")
    d = np.full(x.shape, np.inf)
    for cx, cy, cz in centres:
        d = np.minimum(d, np.sqrt((x - cx) ** 2 + (y - cy) ** 2 + (z - cz) ** 2) - radius)
    t = np.clip(d / trunc_vox, -1, 1)
    vol = O.Volume((n, n, n), (float(n),) * 3)  # 1 m voxels: positions in voxel units
    q = np.clip((t * 32767).astype(np.int32), -32767, 32767)
    q[q == 0] = 1  # a corner exactly on the level set puts several edge vertices at one point
    vol.tsdf[:] = q.ravel().astype(np.int16)
    vol.weight[:] = 1
    return vol


def _identity():
    p = Pose()
    p.R[0] = p.R[4] = p.R[8] = 1.0
    return p


def _topology(tris):
    key = {}
    vid = lambda p: key.setdefault(p.tobytes(), len(key))
    faces = [tuple(vid(t[k]) for k in range(3)) for t in tris]
    directed = collections.Counter()
    for a, b, c in faces:
        for u, v in ((a, b), (b, c), (c, a)):
            directed[(u, v)] += 1
    und = collections.Counter()
    for (u, v), m in directed.items():
        und[(min(u, v), max(u, v))] += m
    return len(key), len(und), len(faces), directed, und


@pytest.mark.parametrize("centres,chi", [([(16.3, 15.8, 16.1)], 2), ([(12.2, 12.4, 16.0), (36.1, 35.7, 32.2)], 4)])
def test_sphere_meshes_are_closed_and_oriented(oracle_lib, centres, chi):
    n, r = 48, 7.3
    vol = _sdf_volume(n, centres, r)
    tris, total = O.extract_mesh(vol, _identity())
    assert total == len(tris) > 100
    V, E, F, directed, und = _topology(tris)
    assert all(m == 2 for m in und.values())        # closed: every edge in two triangles
    assert all(m == 1 for m in directed.values())   # consistently oriented
    assert V - E + F == chi
    # vertices on the spheres (positions are voxel centres + 0.5 in voxel units)
    p = tris.reshape(-1, 3).astype(np.float64)
    d = np.min([np.linalg.norm(p - np.array(c), axis=1) for c in centres], axis=0)
    assert np.abs(d - r).max() < 0.6


def test_mesh_skips_unobserved_and_splits_by_slab(oracle_lib):
    vol = _sdf_volume(32, [(16.2, 16.1, 15.9)], 6.4)
    full, n = O.extract_mesh(vol, _identity())
    # z ranges concatenate (canonical order is chunk-major, chunks aligned to 8)
    a, na = O.extract_mesh(vol, _identity(), zlo=0, zhi=16)
    b, nb = O.extract_mesh(vol, _identity(), zlo=16, zhi=31)
    assert na + nb == n and np.array_equal(np.concatenate([a, b]), full)
    # cubes touching a weight-0 voxel are skipped
    vol.weight.reshape(32, 32, 32)[16, :, :] = 0
    part, m = O.extract_mesh(vol, _identity())
    assert 0 < m < n
