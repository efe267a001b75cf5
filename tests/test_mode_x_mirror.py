"""CPU: the Mode X mirror bounce (Material.reflectivity; DESIGN.md "Mode X") in the oracle and the
host plumbing.  The reference has no mirrors, so there is no reference vector to pin against: these
are property tests of the build-defined spec (parity unpinned against the reference by nature; the
GPU path is pinned bit for bit to this oracle in test_gpu_parity.py)."""
import ctypes

import numpy as np
import pytest

import oracle_util as U

gi = U.pkg()
S = U.scenes()


def _all_mirrors(sc, r):
    for e in sc.entities:
        if e.material is None:
            e.material = S.Material(tuple(e.args[-3:]) if e.kind == 1 else (1.0, 0.0, 0.0))
        e.material.reflectivity = r
    return sc


def test_reflectivity_scn_round_trip_and_default_digest():
    sc = S.named_scene("cornell_mirror")
    t = sc.to_scn()
    assert S.parse_scn(t).to_scn().split("\n", 1)[1] == t.split("\n", 1)[1]
    assert any(len(l.split()) == 9 for l in t.splitlines() if l.startswith("material"))
    plain = S.cornell_scene().to_scn()   # reflectivity 0 is not written: existing scene files unchanged
    assert all(len(l.split()) == 8 for l in plain.splitlines() if l.startswith("material"))


def test_entity_desc_carries_reflectivity():
    d = gi.EntityDesc()
    gi.ImpSphere((0.0, 0.0, 0.0), 1.0, (1, 0, 0))._desc(d)
    assert d.mat_reflectivity == 0.0
    e = gi.ImpSphere((0.0, 0.0, 0.0), 1.0, (1, 0, 0))
    e.material = gi.Material((1, 0, 0), reflectivity=0.25)
    e._desc(d)
    assert d.has_material == 1 and d.mat_reflectivity == 0.25
    assert ctypes.sizeof(gi.EntityDesc) == 8 + 11 * 8 + 3 * 8 + 3 * 8 + 8 + 8


def test_depth1_ignores_reflectivity():
    a = S.cornell_scene()
    b = _all_mirrors(S.cornell_scene(), 1.0)
    oa = U.oracle_render(a.to_scn(), 48, 32, mode=1, spp=2, depth=1, seed=3)
    ob = U.oracle_render(b.to_scn(), 48, 32, mode=1, spp=2, depth=1, seed=3)
    assert U.bits_equal(oa["rgb"], ob["rgb"]).all()


def test_perfect_mirrors_draw_no_bounce_randomness():
    """reflectivity 1 everywhere + spp 1 (no jitter): every bounce is a mirror bounce and no random
    number is drawn for it, so the frame does not depend on the seed; diffuse frames do."""
    m = _all_mirrors(S.cornell_scene(), 1.0).to_scn()
    f1 = U.oracle_render(m, 40, 30, mode=1, spp=1, depth=6, seed=1)
    f2 = U.oracle_render(m, 40, 30, mode=1, spp=1, depth=6, seed=2)
    assert U.bits_equal(f1["rgb"], f2["rgb"]).all()
    d = S.cornell_scene().to_scn()
    g1 = U.oracle_render(d, 40, 30, mode=1, spp=1, depth=6, seed=1)
    g2 = U.oracle_render(d, 40, 30, mode=1, spp=1, depth=6, seed=2)
    assert not U.bits_equal(g1["rgb"], g2["rgb"]).all()
    assert not U.bits_equal(f1["rgb"], g1["rgb"]).all()
    assert (f1["ncand"] != g1["ncand"]).any()   # other paths: rays leave through the open front


def test_mirror_ray_count_and_bad_reflectivity():
    sc = S.named_scene("cornell_mirror")
    o = U.oracle_render(sc.to_scn(), 32, 24, mode=1, spp=2, depth=5, seed=9)
    assert np.isfinite(o["rgb"]).all() and (o["rgb"] >= 0).all() and (o["rgb"] <= 1).all()
    bad = S.cornell_scene()
    bad.entities[0].material.reflectivity = 1.5
    with pytest.raises(RuntimeError, match="reflectivity"):
        U.oracle_render(bad.to_scn(), 8, 8, mode=1, spp=1, depth=2)
