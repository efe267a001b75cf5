"""Generates the golden fixtures in tests/golden/ from the COMPILED REFERENCE (oracle/_ref/, built
by `make -C oracle ref` from /root/reference's own headers).  Run in the build container:

    python tests/golden/make_golden.py

Fixtures are data only (inputs and the reference's outputs):
  kat.json              main.cpp:90-133 ad-hoc tests (entity_test, bbox_test, matrix_test)
  <scene>_<w>x<h>.npz   per-pixel fp64 radiance / hit entity / (u,v) / candidate & node-test counts /
                        RGB888 for a pixel set (full frame or window+stride), plus RayTracer::run's own
                        8-bit frame where it was run (ref_run, Qt-linked)
  tree_<scene>.json     octree statistics + sha256 of the `tree` dump (octree.h structure)
  rays_<scene>.npz      per-(ray, entity) intersect/getTextureCoord KAT on seeded random rays
  boxes.npz             ExpBox node-test KAT (entities.h:379-440) on seeded random boxes/rays
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))
import oracle_util as U  # noqa: E402

S = U.scenes()


def scene_by_name(name: str):
    return S.named_scene(name)


# (scene, w, h, window or None, stride, run RayTracer::run too)
FRAMES = [
    ("main", 200, 200, None, 1, True),
    ("sphere", 256, 256, None, 1, True),          # C1 at its config size
    ("cornell", 128, 128, None, 1, True),
    ("cornell", 512, 512, None, 61, False),       # C2 frame, sampled
    ("cornell", 1920, 1080, None, 509, False),    # C3 frame, sampled
    ("soup1000", 160, 160, None, 1, False),
    ("soup100000", 1920, 1080, (700, 600, 1220, 1080), 29, False),   # C4 frame: the soup's region
    ("zoo", 160, 160, None, 1, True),                                # every entity type (f1)
    ("only_expsphere", 96, 96, None, 1, False),
    ("only_expcube", 96, 96, None, 1, False),
    ("only_expcone", 96, 96, None, 1, False),
    ("only_exprectangle", 96, 96, None, 1, False),
    ("only_expbox", 96, 96, None, 1, False),
]


def frame_name(scene, w, h, window, stride):
    n = f"{scene}_{w}x{h}"
    if window is not None:
        n += "_win" + "-".join(map(str, window))
    if stride != 1:
        n += f"_s{stride}"
    return n


def ref_run_frame(scn: str, w: int, h: int) -> np.ndarray:
    with tempfile.TemporaryDirectory() as td:
        sp, op = os.path.join(td, "s.scn"), os.path.join(td, "o.rgb")
        open(sp, "w").write(scn)
        env = dict(os.environ, QT_QPA_PLATFORM="offscreen")
        subprocess.run([U.REF_RUN, sp, str(w), str(h), op], check=True, env=env)
        return np.frombuffer(open(op, "rb").read(), np.uint8).reshape(h, w, 3).copy()


def make_frames():
    for scene, w, h, window, stride, run in FRAMES:
        sc = scene_by_name(scene)
        scn = sc.to_scn()
        r = U.ref_render(scn, w, h, window=window, stride=stride)
        name = frame_name(scene, w, h, window, stride)
        extra = {}
        if run:
            extra["run_q"] = ref_run_frame(scn, w, h)
        np.savez_compressed(os.path.join(HERE, name + ".npz"), x=r["x"], y=r["y"], rgb=r["rgb"], hit=r["hit"],
                            uv=r["uv"], ncand=r["ncand"], nnode=r["nnode"], q=r["q"],
                            meta=np.array(json.dumps(dict(scene=scene, w=w, h=h, window=window, stride=stride,
                                                          scene_sha256=sc.digest()))), **extra)
        print(name, len(r["x"]), "px,", int((r["hit"] >= 0).sum()), "hits")


def tree_stats(dump: str) -> dict:
    nodes = [l.split() for l in dump.splitlines() if l.startswith("node")]
    leaves = [n for n in nodes if n[3] == "1"]
    reach = set()
    for n in leaves:
        reach.update(int(x) for x in n[11:])
    return dict(n_nodes=len(nodes), n_leaves=len(leaves), max_depth=max(int(n[1]) for n in nodes),
                n_reachable=len(reach), sha256=hashlib.sha256(dump.encode()).hexdigest())


def make_trees():
    for scene in ["main", "sphere", "cornell", "soup1000", "soup100000", "zoo"]:
        sc = scene_by_name(scene)
        st = tree_stats(U.ref_tree(sc.to_scn()))
        st["scene_sha256"] = sc.digest()
        json.dump(st, open(os.path.join(HERE, f"tree_{scene}.json"), "w"), indent=1)
        print("tree", scene, st)


def random_rays(rng, n, origin_box, target_box):
    o = rng.uniform(origin_box[0], origin_box[1], size=(n, 3))
    t = rng.uniform(target_box[0], target_box[1], size=(n, 3))
    return np.concatenate([o, t - o], axis=1)


def make_rays():
    rng = np.random.default_rng(2019)
    for scene, ob, tb in [("main", (-12, -8), (-3, 6)), ("cornell", (-12, 9), (-5, 10)), ("zoo", (-12, -8), (-6, 6))]:
        sc = scene_by_name(scene)
        rays = random_rays(rng, 4000, ob, tb)
        # plus axis-aligned and grazing rays (dir components exactly 0)
        ax = np.zeros((12, 6))
        ax[:, 0:3] = [-10, 0, 0]
        ax[0:3, 3:6] = np.eye(3)
        ax[3:6, 3:6] = -np.eye(3)
        ax[6:, 3:6] = rng.uniform(-1, 1, size=(6, 3))
        ax[6:, 4] = 0
        rays = np.concatenate([rays, ax])
        r = U.ref_rays(sc.to_scn(), rays, len(sc.entities))
        np.savez_compressed(os.path.join(HERE, f"rays_{scene}.npz"), rays=rays, **r)
        print("rays", scene, rays.shape[0], "hits", int(r["hit"].sum()))


def make_boxes():
    rng = np.random.default_rng(7)
    n = 6000
    lo = rng.uniform(-5, 5, size=(n, 3))
    ext = rng.uniform(0.05, 6, size=(n, 3))
    o = rng.uniform(-12, 12, size=(n, 3))
    tgt = lo + rng.uniform(-0.5, 1.5, size=(n, 3)) * ext
    recs = np.concatenate([lo, lo + ext, o, tgt - o], axis=1)
    # octree-shaped boxes seen from the config camera
    m = 2000
    lvl = rng.integers(1, 6, size=m)
    size = 40.0 / (2.0 ** lvl)
    cell = np.floor(rng.uniform(0, 1, size=(m, 3)) * (2 ** lvl)[:, None])
    bmin = -20 + cell * size[:, None]
    cam = np.tile([-10.0, 0, 0], (m, 1))
    d = np.concatenate([np.ones((m, 1)), rng.uniform(-1, 1, size=(m, 2))], axis=1)
    recs = np.concatenate([recs, np.concatenate([bmin, bmin + size[:, None], cam, d], axis=1)])
    hit = U.ref_boxes(recs)
    np.savez_compressed(os.path.join(HERE, "boxes.npz"), recs=recs, hit=hit)
    print("boxes", recs.shape[0], "hits", int(hit.sum()))


def make_kat():
    out = subprocess.run([U.REF_HARNESS, "kat"], check=True, capture_output=True, text=True).stdout
    kat = {}
    for line in out.splitlines():
        k, *v = line.split()
        kat[k] = [float(x) for x in v]
    json.dump(kat, open(os.path.join(HERE, "kat.json"), "w"), indent=1)
    print("kat", kat)


# Whole large Mode R frames: R-C3 (Cornell) and R-C4 (the 100k soup) at
# 1920x1080, every pixel through the compiled reference, in row bands over parallel processes.  The
# fixture is digests only: the sha256 of the whole RGB888 frame and of each RGB888 row (the exact bar),
# plus per row the fp64 radiance's channel sums over its non-NaN pixels and its NaN count (compared
# within 1e-5 relative: device acos / sin / pow may differ from libm by an ulp).
WHOLE = [("cornell", 1920, 1080), ("soup100000", 1920, 1080)]


def _band(args):
    scn, w, h, y0, y1 = args
    return y0, U.ref_render(scn, w, h, window=(0, y0, w, y1), stride=1)


def make_whole_frames(jobs: int = 8, band: int = 8):
    from multiprocessing import Pool
    for scene, w, h in WHOLE:
        sc = scene_by_name(scene)
        scn = sc.to_scn()
        rgb = np.zeros((h, w, 3), np.float64)
        q = np.zeros((h, w, 3), np.uint8)
        hits = 0
        with Pool(jobs) as pool:
            for y0, r in pool.imap_unordered(_band, [(scn, w, h, y, min(h, y + band)) for y in range(0, h, band)]):
                rgb[r["y"], r["x"]] = r["rgb"]
                q[r["y"], r["x"]] = r["q"].reshape(-1, 3)
                hits += int((r["hit"] >= 0).sum())
        d = U.whole_frame_digest(rgb, q)
        d.update(scene=scene, w=w, h=h, mode="R", scene_sha256=sc.digest(), hits=hits)
        json.dump(d, open(os.path.join(HERE, f"whole_{scene}_{w}x{h}.json"), "w"))
        print("whole", scene, w, h, d["rgb8_sha256"], int(sum(d["row_nan"])), "NaN pixels")


if __name__ == "__main__":
    if not U.have_ref():
        sys.exit("oracle/_ref/ref_harness missing: run `make -C oracle ref` where /root/reference exists")
    if sys.argv[1:] == ["whole"]:   # the whole 1080p Mode R frames only (minutes over 8 processes)
        make_whole_frames()
        sys.exit(0)
    json.dump({"soup100000_vertices_sha256": S.soup_digest(100000, 2019),
               "soup1000_vertices_sha256": S.soup_digest(1000, 2019)},
              open(os.path.join(HERE, "soup_digest.json"), "w"), indent=1)
    make_kat()
    make_trees()
    make_rays()
    make_boxes()
    make_frames()
