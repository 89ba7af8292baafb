"""Work-balanced Z-slab cuts (kfx_slab_balance, host code in libkfx; no GPU):
cuts run 0..Z on multiples of 8 with >= 8 slices per slab, and minimise the
largest slab's stored-range work (owned slices + 4 halo slices each side) —
checked against exhaustive search on small volumes and against the equal
split on frustum-shaped histograms."""
import itertools

import numpy as np
import pytest

import kfx

HALO = 4


def load(work, cuts):
    Z, world = len(work), len(cuts) - 1
    out = []
    for r in range(world):
        lo = max(0, cuts[r] - HALO) if world > 1 else 0
        hi = min(Z, cuts[r + 1] + HALO) if world > 1 else Z
        out.append(int(work[lo:hi].sum()))
    return out


def valid(cuts, Z, world):
    return (len(cuts) == world + 1 and cuts[0] == 0 and cuts[-1] == Z and
            all(b - a >= 8 for a, b in zip(cuts, cuts[1:])) and all(c % 8 == 0 for c in cuts[1:-1]))


def test_balance_is_optimal_on_small_volumes(kfx_lib):
    rng = np.random.default_rng(1)
    for Z, world in ((48, 2), (64, 3), (64, 4), (80, 3)):
        for _ in range(6):
            work = rng.integers(0, 1000, Z).astype(np.int64)
            cuts = kfx.slab_balance(work, world)
            assert valid(cuts, Z, world), cuts
            best = min(max(load(work, [0, *inner, Z]))
                       for inner in itertools.combinations(range(8, Z - 7, 8), world - 1)
                       if valid([0, *inner, Z], Z, world))
            assert max(load(work, cuts)) == best


def test_balance_beats_equal_split_on_a_frustum(kfx_lib):
    Z, world = 1024, 8
    z = np.arange(Z)
    work = np.minimum((0.3 + z / 400.0) ** 2, 6.0) * 1e5  # cross-section grows with depth
    work[900:] = 0  # behind the back wall
    work = work.astype(np.int64)
    cuts = kfx.slab_balance(work, world)
    assert valid(cuts, Z, world)
    equal = [0] + [Z * r // world // 8 * 8 for r in range(1, world)] + [Z]
    assert max(load(work, cuts)) < 0.75 * max(load(work, equal))
    lb = load(work, cuts)
    assert max(lb) / np.mean(lb) < 1.1


def test_balance_rejects_bad_input(kfx_lib):
    with pytest.raises(kfx.KfxError):
        kfx.slab_balance(np.ones(40, np.int64), 8)  # fewer than 8 slices per slab
