"""Scene I/O: the OBJ loader.  CPU: libgi's gi_obj_parse (C-ABI) against this
repo's Python restatement (scenes.load_obj) on the same text -- identical triangles, bit for bit --
and both against meshes whose triangles are known (a cube of quads, the Cornell box and the 1k
soup written out as OBJ).  GPU: a mesh loaded from OBJ renders the same frame as the same
triangles pushed one by one (no test here reads the reference: OBJ has no reference counterpart)."""
import ctypes
import math

import numpy as np
import pytest

import oracle_util as U

gi = U.pkg()
S = U.scenes()

CUBE = """# unit cube, quads, every reference form
mtllib cube.mtl
o cube
v 0 0 0
v 1 0 0
v 1 1 0
v 0 1 0 1.0
v 0 0 1
v 1 0 1 0.5 0.5 0.5
v 1 1 1
v 0 1 1
vt 0 0
vn 0 0 -1
usemtl white
s off
f 1 4 3 2
f 5/1 6/1 7/1 8/1
f 1//1 2//1 6//1 5//1
f 4/1/1 8/1/1 7/1/1 3/1/1
g side
f -8 -4 -1 -5   # x = 0, relative references
f 2 3 \\
  7 6
l 1 2
"""


def c_parse(text, material=None):
    """gi_obj_parse straight through the C-ABI: list of (kind, has_material, args[0:9], colour)."""
    L = gi.lib()
    data = text.encode()
    tmpl = None
    if material is not None:
        tmpl = gi.EntityDesc()
        tmpl.has_material = 1
        for i in range(3):
            tmpl.mat_color[i] = material[i]
            tmpl.mat_shader[i] = (0.1, 0.7, 1.0)[i]
        tmpl.mat_specular_power = 5.0
    n = ctypes.c_int64()
    rc = L.gi_obj_parse(data, len(data), tmpl, None, 0, ctypes.byref(n))
    if rc != 0:
        raise gi.GIError(L.gi_last_error().decode())
    arr = (gi.EntityDesc * max(1, n.value))()
    assert L.gi_obj_parse(data, len(data), tmpl, arr, n.value, ctypes.byref(n)) == 0
    return [(d.kind, d.has_material, tuple(d.args[0:9]), tuple(d.mat_color)) for d in arr[:n.value]]


def py_parse(text, material=None):
    m = None if material is None else S.Material(tuple(float(c) for c in material))
    s = S.load_obj(text, m)
    return [(e.kind, 0 if e.material is None else 1, e.args,
             (0.0, 0.0, 0.0) if e.material is None else e.material.color) for e in s.entities]


def test_cube_fan_triangulation():
    c, p = c_parse(CUBE), py_parse(CUBE)
    assert c == p
    assert len(c) == 12 and all(k == S.IMP_TRIANGLE for k, *_ in c)
    v = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]
    tri = lambda a, b, cc: tuple(float(x) for x in (*v[a], *v[b], *v[cc]))   # noqa: E731
    assert c[0][2] == tri(0, 3, 2) and c[1][2] == tri(0, 2, 1)              # f 1 4 3 2: (v0, v_k, v_k+1)
    assert c[8][2] == tri(0, 4, 7) and c[9][2] == tri(0, 7, 3)              # f -8 -4 -1 -5
    assert c[10][2] == tri(1, 2, 6) and c[11][2] == tri(1, 6, 5)            # continued face
    # every face of the closed cube: total area 6
    area = 0.0
    for _, _, a, _ in c:
        p0, p1, p2 = np.array(a[0:3]), np.array(a[3:6]), np.array(a[6:9])
        area += 0.5 * np.linalg.norm(np.cross(p1 - p0, p2 - p0))
    assert math.isclose(area, 6.0)


def test_material_template():
    c = c_parse(CUBE, (0.0, 1.0, 0.0))
    assert c == py_parse(CUBE, (0.0, 1.0, 0.0))
    assert all(h == 1 and col == (0.0, 1.0, 0.0) for _, h, _, col in c)
    ents = gi.obj_entities(CUBE, gi.Material((0, 1, 0)))
    assert len(ents) == 12 and ents[3].material.color == (0.0, 1.0, 0.0)
    assert [e._args for e in ents] == [a for _, _, a, _ in c]
    assert gi.obj_entities(CUBE)[0].material is None   # the reference's default ImpTriangle material


def to_obj(scene):
    """Each triangle of a scene as its own face (repr floats: every double round-trips)."""
    out = ["# written by tests/test_obj.py"]
    for e in scene.entities:
        a = e.args
        for k in range(3):
            out.append("v " + " ".join(repr(float(x)) for x in a[3 * k:3 * k + 3]))
        out.append("f -3 -2 -1")
    return "\r\n".join(out) + "\r\n"


@pytest.mark.parametrize("name", ["cornell", "soup1000"])
def test_scene_round_trip(name):
    sc = S.named_scene(name)
    text = to_obj(sc)
    c, p = c_parse(text), py_parse(text)
    assert c == p
    assert [a for _, _, a, _ in c] == [e.args for e in sc.entities]


@pytest.mark.parametrize("bad", ["v 1 2\n", "v 1 2 x\n", "v 1 2 nan\n", "v 0 0 0\nv 1 0 0\nf 1 2\n",
                                 "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 4\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 0 1 2\n",
                                 "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 -4\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 a/1\n",
                                 # one number grammar on both sides (gi_obj.cpp is_real): no hex floats,
                                 # inf / nan, digit separators, non-ASCII digits, bare '.' or exponent
                                 "v 0x1p3 0 0\n", "v 1_0 0 0\n", "v \u0661 0 0\n", "v inf 0 0\n", "v -Infinity 0 0\n",
                                 "v . 0 0\n", "v 1e 0 0\n", "v 1e+ 0 0\n", "v 1,5 0 0\n", "v +-1 0 0\n",
                                 "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 0x3\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 3_\n",
                                 "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 \u0663\n", "v 0 0 0\nv 1 0 0\nv 0 1 0\nf 1 2 +\n"])
def test_malformed_input_rejected(bad):
    with pytest.raises(gi.GIError, match="obj line"):
        c_parse(bad)
    with pytest.raises(ValueError, match="obj line"):
        py_parse(bad)


def test_number_forms_agree():
    """Every accepted number form parses to the same double on both sides."""
    text = ("v +1. .5 -0\nv 1E+2 -2.5e-3 007\nv 1e308 -4.9e-324 123456789012345678901234567890\n"
            "f +1 2/7 -1//3\n"
            "v 1e-400 -2e-324 0.000001e-330\nf 1 2 4\n")   # underflow to a signed zero on both sides
    c, p = c_parse(text), py_parse(text)
    assert c == p
    assert c[0][2] == (1.0, 0.5, -0.0, 100.0, -0.0025, 7.0, 1e308, -5e-324, 1.2345678901234568e29)
    v = c[1][2][6:9]
    assert v == (0.0, -0.0, 0.0) and [str(x) for x in v] == ["0.0", "-0.0", "0.0"]


def test_parse_ignores_c_locale(tmp_path):
    """the reference host is a Qt app (QApplication sets the C locale from the
    environment), so gi_obj_parse must not read "1.5" as 1 under a comma-decimal LC_NUMERIC.  A
    comma-decimal locale is compiled into tmp_path with localedef (the image ships none) and the
    parse runs in a child process with it in force."""
    import shutil
    import subprocess
    import sys
    if not shutil.which("localedef"):
        pytest.skip("localedef not available")
    (tmp_path / "comma").write_text('LC_NUMERIC\ndecimal_point "<U002C>"\nthousands_sep "<U002E>"\n'
                                    'grouping 3;3\nEND LC_NUMERIC\n')
    cm = ["<escape_char> /", "<comment_char> %", "<code_set_name> ASCIITEST", "<mb_cur_min> 1", "<mb_cur_max> 1",
          "CHARMAP"] + ["<U%04X> /x%02x C%d" % (i, i, i) for i in range(128)] + ["END CHARMAP"]
    (tmp_path / "ascii.cm").write_text("\n".join(cm) + "\n")
    subprocess.run(["localedef", "-c", "-i", str(tmp_path / "comma"), "-f", str(tmp_path / "ascii.cm"), "--no-archive",
                    str(tmp_path / "xxcomma")], capture_output=True)
    if not (tmp_path / "xxcomma" / "LC_NUMERIC").exists():
        pytest.skip("localedef could not build a test locale")
    child = f"""
import ctypes, locale, sys
sys.path.insert(0, {repr(__import__("os").path.join(U.ROOT, "tests"))})
import test_obj as T
locale.setlocale(locale.LC_NUMERIC, "xxcomma")
libc = ctypes.CDLL(None)
libc.strtod.restype = ctypes.c_double
assert libc.strtod(b"1.5", None) == 1.0, "the test locale is not comma-decimal"
print(repr(T.c_parse(T.CUBE.replace(" 1 1 1", " 1.5 0.25 1e-1"))))
"""
    env = dict(__import__("os").environ, LOCPATH=str(tmp_path))
    r = subprocess.run([sys.executable, "-c", child], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().splitlines()[-1] == repr(c_parse(CUBE.replace(" 1 1 1", " 1.5 0.25 1e-1")))


def test_error_line_numbers_agree():
    text = "# c\nv 0 0 0\nv 1 0 0\n\nv 0 1 0\nf 1 2 \\\n 9\n"
    with pytest.raises(gi.GIError, match="obj line 7:"):
        c_parse(text)
    with pytest.raises(ValueError, match="obj line 7:"):
        py_parse(text)


def test_empty_and_comment_only():
    assert c_parse("") == [] and py_parse("") == []
    assert c_parse("# nothing\n\n   \nvt 0 0\n") == []


@pytest.mark.gpu
def test_obj_mesh_renders_like_pushed_triangles():
    """The 1k soup loaded from OBJ (material = the soup's white) renders bit-identical Mode X and
    Mode R frames to the same triangles pushed one by one (scenes.soup_scene)."""
    import torch
    assert torch.cuda.is_available()
    sc = S.soup_scene(1000)
    o = gi.Octree(sc.octree_min, sc.octree_max)
    for e in gi.obj_entities(to_obj(sc), gi.Material((1.0, 1.0, 1.0))):
        o.push_back(e)
    a = gi.DeviceScene(o)
    b = gi.DeviceScene.from_scene(sc)
    cam = gi.Camera(sc.cam_pos, sc.cam_look, sc.focal)
    for kw in (dict(), dict(mode=gi.MODE_X, spp=2, depth=4, seed=3)):
        ra, qa = a.render(cam, sc.light, 96, 64, **kw)
        rb, qb = b.render(cam, sc.light, 96, 64, **kw)
        assert U.bits_equal(ra, rb).all() and (qa == qb).all()


def _demo():
    import os
    exe = os.path.join(U.ROOT, "integration", "_build", "dropin_demo")
    if not os.path.exists(exe):
        pytest.skip("integration/_build/dropin_demo not built (needs the reference tree)")
    return exe


def test_cpp_push_obj_candidates_match_oracle(tmp_path):
    """include/gi_dropin/obj.h's push_obj from the reference app's own classes (integration/
    dropin_demo.cpp, `obj:<path>`): the 1k soup read back from OBJ gives, on every pixel's primary
    ray, the candidate-list length (Octree::intersect, octree.h:46-68) the oracle computes for the
    scene built in Python -- the mesh arrived as the same ImpTriangles in the same push order."""
    import subprocess
    exe = _demo()
    sc = S.soup_scene(1000)
    path = tmp_path / "soup.obj"
    path.write_text(to_obj(sc))
    out = tmp_path / "c.bin"
    w, h = 64, 48
    subprocess.run([exe, str(w), str(h), str(out), f"obj:{path}", "cands"], check=True, timeout=120)
    c = np.fromfile(out, np.int32)
    o = U.oracle_render(sc.to_scn(), w, h)
    assert (c == o["ncand"]).all()


@pytest.mark.gpu
def test_cpp_push_obj_frame_matches_oracle(tmp_path):
    """RayTracer::run (the drop-in) over an OBJ-loaded mesh: the RGB888 frame equals the oracle's
    Mode R frame of the same triangles."""
    import os
    import subprocess
    exe = _demo()
    sc = S.soup_scene(1000)
    path = tmp_path / "soup.obj"
    path.write_text(to_obj(sc))
    out = tmp_path / "f.rgb"
    w, h = 64, 48
    subprocess.run([exe, str(w), str(h), str(out), f"obj:{path}"], check=True, timeout=120,
                   env=dict(os.environ, QT_QPA_PLATFORM="offscreen"))
    got = np.frombuffer(out.read_bytes(), np.uint8).reshape(-1, 3)
    o = U.oracle_render(sc.to_scn(), w, h)
    assert (got == o["q"]).all()
