"""CPU: pins the oracle (oracle/gi_oracle.cpp, this repo's restatement of the reference per-pixel
loop) against golden vectors produced by the COMPILED REFERENCE (tests/golden/make_golden.py).
Mode R is required to match bit for bit: radiance, hit entity, (u,v), candidate-list length and
node-test count.  Where oracle/_ref exists (build container), also re-checks live against it."""
import glob
import json
import os
import re

import numpy as np
import pytest

import oracle_util as U

S = U.scenes()
GOLD = U.GOLDEN


def _scene(name):
    return S.named_scene(name)


FRAMES = sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLD, "*.npz"))
                if re.search(r"_\d+x\d+", os.path.basename(p)))


def load_frame(name):
    z = np.load(os.path.join(GOLD, name + ".npz"))
    meta = json.loads(str(z["meta"]))
    return z, meta


def render_pixels(scn, w, h, xs, ys, **kw):
    """oracle at exactly the golden pixel set (bounding window, then gather)."""
    x0, x1, y0, y1 = xs.min(), xs.max() + 1, ys.min(), ys.max() + 1
    o = U.oracle_render(scn, w, h, window=(x0, y0, x1, y1), **kw)
    idx = (ys - y0) * (x1 - x0) + (xs - x0)
    return {k: v[idx] for k, v in o.items()}


def texel_ub_mask(hit, uv):
    """Pixels whose texture lookup reads outside the reference's 32x32 array (negative flat index
    (u%32)*32 + v%32, C remainder semantics; texture.h / entities.h).  The reference reads stack memory
    there (undefined behaviour), so those pixels carry no parity claim; the oracle and the device both
    wrap the flat index into the array instead.  See DESIGN.md, texture UB."""
    f = np.fmod(uv[:, 0], 32) * 32 + np.fmod(uv[:, 1], 32)
    return (hit >= 0) & ((f < 0) | (f >= 1024))


# pixels excluded as texel UB, exactly, per fixture (only the single-ExpSphere frame has any: its
# latitude coordinate goes negative below the equator, entities.h:549-571)
TEXEL_UB_PIXELS = {"only_expsphere_96x96": 154}


def test_frames_present():
    assert len(FRAMES) >= 6, FRAMES


@pytest.mark.parametrize("name", FRAMES)
def test_mode_r_bit_exact_vs_reference_golden(name):
    z, meta = load_frame(name)
    sc = _scene(meta["scene"])
    assert sc.digest() == meta["scene_sha256"], "scene generator drifted from the fixture"
    if meta["scene"] == "soup100000" and len(z["x"]) > 9000:
        pytest.skip("large")
    o = render_pixels(sc.to_scn(), meta["w"], meta["h"], z["x"], z["y"])
    ok = ~texel_ub_mask(z["hit"], z["uv"])
    assert int((~ok).sum()) == TEXEL_UB_PIXELS.get(name, 0), "texel-UB pixel count drifted"
    assert U.bits_equal(o["rgb"], z["rgb"])[ok].all(), "fp64 radiance differs from the reference"
    assert (o["hit"] == z["hit"]).all()
    assert (o["uv"] == z["uv"]).all()
    assert (o["ncand"] == z["ncand"]).all()
    assert (o["nnode"] == z["nnode"]).all()
    assert (o["q"] == z["q"])[ok].all()
    if "run_q" in z.files:   # RayTracer::run's own QImage (Qt) agrees with the restated quantisation
        q = z["q"].reshape(meta["h"], meta["w"], 3)
        okq = ok.reshape(meta["h"], meta["w"])
        assert (z["run_q"] == q)[okq].all()


def test_main_scene_checksum_anchor():
    # SURVEY Appendix B regression anchor: main.cpp scene 500x500 -> sum(3R+5G+7B) = 111049727
    o = U.oracle_render(S.main_scene().to_scn(), 500, 500)
    q = o["q"].astype(np.int64)
    assert int((3 * q[:, 0] + 5 * q[:, 1] + 7 * q[:, 2]).sum()) == 111049727
    assert int((q.sum(1) > 0).sum()) == 53182


@pytest.mark.parametrize("scene", ["main", "sphere", "cornell", "soup1000", "zoo"])
def test_octree_structure_vs_reference(scene):
    import hashlib
    st = json.load(open(os.path.join(GOLD, f"tree_{scene}.json")))
    dump = U.oracle_tree(_scene(scene).to_scn())
    assert hashlib.sha256(dump.encode()).hexdigest() == st["sha256"]


def test_cornell_tree_stats():
    st = json.load(open(os.path.join(GOLD, "tree_cornell.json")))
    # Cornell 81 nodes / 71 leaves / depth 4 / 22 of 34 reachable (A.6)
    assert (st["n_nodes"], st["n_leaves"], st["max_depth"], st["n_reachable"]) == (81, 71, 4, 22)


@pytest.mark.parametrize("scene", ["main", "cornell", "zoo"])
def test_entity_intersect_kat(scene):
    z = np.load(os.path.join(GOLD, f"rays_{scene}.npz"))
    sc = _scene(scene)
    o = U.oracle_rays(sc.to_scn(), z["rays"], len(sc.entities))
    assert (o["hit"] == z["hit"]).all()
    assert U.bits_equal(o["pn"], z["pn"]).all()
    assert (o["uv"] == z["uv"]).all()


def test_expbox_node_test_kat():
    z = np.load(os.path.join(GOLD, "boxes.npz"))
    assert (U.oracle_boxes(z["recs"]) == z["hit"]).all()


def test_main_cpp_kat_values():
    kat = json.load(open(os.path.join(GOLD, "kat.json")))
    # main.cpp:90-104 entity_test through the oracle's sphere routine (a sphere scene + one ray)
    s = S.Scene(entities=[])
    s.imp_sphere((2.0, 0.0, 0.0), 10, (0, 1, 0))
    o = U.oracle_rays(s.to_scn(), np.array([[-10.0, 0, 0, 1, 0.5, 0.5]]), 1)
    assert o["hit"][0, 0] == kat["entity_test.hit"][0]
    assert np.array_equal(o["pn"][0, 0, :3], kat["entity_test.point"])
    assert np.array_equal(o["pn"][0, 0, 3:], kat["entity_test.normal"])


def test_zoo_kat_covers_every_entity_kind():
    z = np.load(os.path.join(GOLD, "rays_zoo.npz"))
    kinds = [e.kind for e in S.zoo_scene().entities]
    assert sorted(set(kinds)) == list(range(1, 9))
    assert (z["hit"].sum(0) > 0).all(), "every zoo entity is hit by some KAT ray"


def test_soup_generator_digest():
    d = json.load(open(os.path.join(GOLD, "soup_digest.json")))
    assert S.soup_digest(1000, 2019) == d["soup1000_vertices_sha256"]


@pytest.mark.skipif(not U.have_ref(), reason="compiled reference only in the build container")
def test_live_reference_random_scene():
    # a seeded random scene of all supported entity kinds, compared live with the reference
    rng = np.random.default_rng(11)
    s = S.Scene(entities=[])
    for _ in range(6):
        s.imp_sphere(tuple(rng.uniform(-4, 8, 3)), float(rng.uniform(0.5, 3)), tuple(rng.integers(0, 2, 3)))
    for _ in range(20):
        c = rng.uniform(-3, 9, 3)
        v = c + rng.uniform(-2, 2, (3, 3))
        s.imp_triangle(tuple(v[0]), tuple(v[1]), tuple(v[2]), tuple(rng.integers(0, 2, 3)))
    s.exp_quad((1.0, 0.5, -0.5), 3, 2, 0.7, (1, 1, 0))
    s.exp_sphere(tuple(rng.uniform(-2, 4, 3)), 1.5, (1, 0, 1))
    s.exp_cube(tuple(rng.uniform(-2, 4, 3)), 1.0, 2.0, 1.5, (0, 1, 1))
    s.exp_cone(tuple(rng.uniform(-2, 4, 3)), (1.0, -0.5, 0.3), 3, 1.2, (1, 1, 0))
    scn = s.to_scn()
    r = U.ref_render(scn, 96, 96)
    o = U.oracle_render(scn, 96, 96)
    ok = ~texel_ub_mask(r["hit"], r["uv"])
    assert U.bits_equal(r["rgb"], o["rgb"])[ok].all()
    assert (r["hit"] == o["hit"]).all() and (r["nnode"] == o["nnode"]).all()
    assert U.ref_tree(scn) == U.oracle_tree(scn)


@pytest.mark.parametrize("scene,w,h,spp,depth,win", [
    ("soup1000", 64, 48, 2, 8, None), ("zoo", 48, 48, 2, 4, None), ("cornell", 48, 40, 3, 5, None),
    ("cornell_mirror", 40, 40, 2, 6, None), ("main", 40, 40, 2, 3, None),
    ("soup100000", 1920, 1080, 1, 8, (956, 956, 964, 964))])
def test_oracle_mode_x_bvh_equals_brute_force(scene, w, h, spp, depth, win):
    """The oracle's Mode X closest / shadow queries by its own BVH (used for the 100k-soup C4/C5
    checks) return exactly the brute-force answer over all primitives: same frames bit for bit and
    the same ray counts."""
    scn = S.named_scene(scene).to_scn()
    out = []
    try:
        for m in (0, 1):
            U.oracle_accel(m)
            out.append(U.oracle_render(scn, w, h, mode=1, spp=spp, depth=depth, seed=7, window=win))
    finally:
        U.oracle_accel(-1)
    assert U.bits_equal(out[0]["rgb"], out[1]["rgb"]).all()
    assert (out[0]["ncand"] == out[1]["ncand"]).all()
    assert (out[0]["hit"] == out[1]["hit"]).all()


def test_oracle_mode_x_sample_parallel_window_equals_pixel_loop():
    """Small windows with many samples run the samples of a pixel in parallel (summed in order
    afterwards): the same pixels as the pixel-parallel loop over a larger window."""
    scn = S.cornell_scene().to_scn()
    a = U.oracle_render(scn, 64, 48, mode=1, spp=33, depth=4, seed=5, window=(20, 20, 28, 28))    # 64 px: pixel loop
    b = U.oracle_render(scn, 64, 48, mode=1, spp=33, depth=4, seed=5, window=(22, 22, 25, 25))    # 9 px: sample loop
    aa = a["rgb"].reshape(8, 8, 3)[2:5, 2:5].reshape(-1, 3)
    assert U.bits_equal(aa, b["rgb"]).all()
    assert (a["ncand"].reshape(8, 8)[2:5, 2:5].reshape(-1) == b["ncand"]).all()
    assert (a["hit"].reshape(8, 8)[2:5, 2:5].reshape(-1) == b["hit"]).all()


@pytest.mark.parametrize("name", sorted(U.ANCHOR))
def test_reduced_mode_x_anchored_to_reference(name):
    """Mode X's shared stages (raygen, fp64 hit points, polynomial acos texture mapping, square-and-
    multiply Blinn-Phong) tied to the COMPILED REFERENCE's frames where the semantics coincide:
    depth 1, 1 spp, no shadow rays.  Excluded pixels are counted exactly by class (oracle_util.ANCHOR:
    A.1/A.6 entity choice, texel edges, fp32 sphere roots); all others within 1e-5 relative."""
    z, meta = load_frame(name)
    sc = _scene(meta["scene"])
    U.oracle_no_shadow(True)
    try:
        o = render_pixels(sc.to_scn(), meta["w"], meta["h"], z["x"], z["y"], mode=1, spp=1, depth=1)
    finally:
        U.oracle_no_shadow(False)
    ent, tex, far, exact, far_max = U.anchor_counts(o["rgb"], o["hit"], o["uv"], z)
    assert (ent, tex, far, exact) == U.ANCHOR[name]
    assert far_max <= U.ANCHOR_ABS


@pytest.mark.parametrize("scene,spp", [("cornell", 3), ("soup1000", 2), ("main", 1)])
def test_time_rows_pixels_equal_render(scene, spp):
    """gio_time_rows' per-pixel output (the whole-frame / strided-row GPU parity tests and bench.py's
    self-check compare against it) is gio_render's Mode X frame on those rows, bit for bit -- the
    background samples it resolves by its scene-box test add exactly +0."""
    sc = S.named_scene(scene)
    w, h, depth = 48, 40, 5
    full = U.oracle_render(sc.to_scn(), w, h, mode=1, spp=spp, depth=depth, seed=13)
    r = U.oracle_time_rows(sc.to_scn(), w, h, spp, depth, 13, 3, 7, 100, pixels=True)
    assert r["rows"] == list(range(3, h, 7))
    f = full["rgb"].reshape(h, w, 3)[r["rows"]]
    assert U.bits_equal(r["rgb"], f).all()
    assert (r["q"] == full["q"].reshape(h, w, 3)[r["rows"]]).all()
