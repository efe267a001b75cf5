"""Scene descriptions for the gi path (host side, no GPU).

A scene is exactly what the reference's app code builds by hand in ``main.cpp:24-48``: an
``Octree(min, max)`` (octree.h:14), a ``Camera(pos, lookAt, focal)`` (camera.h:8-10), a point
light, and a sequence of ``Octree::push_back(new Entity(...))`` calls (octree.h:20-43) whose
order defines the reference's candidate order.  Entity parameters are the reference
constructor arguments (entities.h:45, 138, 461, 581, 652, 823), optionally followed by a
``material`` override (``entity->material = Material(color[, shader])``, material.h:12-29).

The ``.scn`` text form is read by the oracle harness (oracle/ref_harness.cpp), by this repo's CPU
restatement (oracle/gi_oracle.cpp) and here; numbers are written with ``repr`` so every double
round-trips exactly.

Config scenes (BASELINE.json ``configs``):
  * ``main_scene``    — main.cpp:24-48 (ExpQuad + 2 ImpSpheres), the plumbing fixture;
  * ``sphere_scene``  — C1: one ImpSphere r=2 at the origin;
  * ``cornell_scene`` — C2/C3: 34 ImpTriangles (5 walls + 2 blocks), light (5,0,4.5);
  * ``soup_scene``    — C4/C5: N random ImpTriangles from splitmix64(seed=2019).
"""
from __future__ import annotations

import hashlib
import math
import re
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

Vec3 = Tuple[float, float, float]

# entity kinds; values are the C-ABI's gi_entity_kind (include/gi.h)
IMP_SPHERE = 1
IMP_TRIANGLE = 2
EXP_QUAD = 3
EXP_SPHERE = 4
EXP_CUBE = 5
EXP_CONE = 6
EXP_RECTANGLE = 7
EXP_BOX = 8

_KW = {
    IMP_SPHERE: "impsphere",
    IMP_TRIANGLE: "imptriangle",
    EXP_QUAD: "expquad",
    EXP_SPHERE: "expsphere",
    EXP_CUBE: "expcube",
    EXP_CONE: "expcone",
    EXP_RECTANGLE: "exprectangle",
    EXP_BOX: "expbox",
}
_KIND = {v: k for k, v in _KW.items()}
# number of ctor arguments per kind (after the keyword)
_NARGS = {IMP_SPHERE: 7, IMP_TRIANGLE: 9, EXP_QUAD: 9, EXP_SPHERE: 7, EXP_CUBE: 9, EXP_CONE: 11, EXP_RECTANGLE: 9,
          EXP_BOX: 6}


@dataclass
class Material:
    """``Material(color[, shader])`` (material.h:13-20) plus ``specular_power`` (material.h:29).
    ``reflectivity`` is Mode X only (no reference counterpart): the probability that a bounce is a
    mirror reflection; written to .scn as an 8th material value only when non-zero."""

    color: Vec3
    shader: Vec3 = (0.1, 0.7, 1.0)
    specular_power: float = 5.0
    reflectivity: float = 0.0


@dataclass
class Entity:
    kind: int
    args: Tuple[float, ...]            # reference ctor arguments, in ctor order
    material: Optional[Material] = None  # explicit override after construction


@dataclass
class Scene:
    octree_min: Vec3 = (-20.0, -20.0, -20.0)
    octree_max: Vec3 = (20.0, 20.0, 20.0)
    cam_pos: Vec3 = (-10.0, 0.0, 0.0)
    cam_look: Vec3 = (1.0, 0.0, 0.0)
    focal: float = 0.1
    light: Vec3 = (-10.0, 10.0, 10.0)
    entities: List[Entity] = field(default_factory=list)
    name: str = "scene"

    # -- builders mirroring the reference constructors --------------------------------------
    def imp_sphere(self, pos: Vec3, radius: float, color: Vec3) -> Entity:
        return self._add(IMP_SPHERE, (*pos, radius, *color))

    def imp_triangle(self, p1: Vec3, p2: Vec3, p3: Vec3, color: Optional[Vec3] = None) -> Entity:
        e = self._add(IMP_TRIANGLE, (*p1, *p2, *p3))
        if color is not None:
            e.material = Material(tuple(float(c) for c in color))
        return e

    def exp_quad(self, pos: Vec3, width: float, length: float, alpha: float, color: Vec3) -> Entity:
        return self._add(EXP_QUAD, (*pos, width, length, alpha, *color))

    def exp_sphere(self, pos: Vec3, radius: float, color: Vec3) -> Entity:
        return self._add(EXP_SPHERE, (*pos, radius, *color))

    def exp_cube(self, pos: Vec3, width: float, length: float, height: float, color: Vec3) -> Entity:
        return self._add(EXP_CUBE, (*pos, width, length, height, *color))

    def exp_cone(self, pos: Vec3, direction: Vec3, height: float, radius: float, color: Vec3) -> Entity:
        return self._add(EXP_CONE, (*pos, *direction, height, radius, *color))

    def exp_rectangle(self, p1: Vec3, p2: Vec3, p3: Vec3) -> Entity:
        return self._add(EXP_RECTANGLE, (*p1, *p2, *p3))

    def exp_box(self, mn: Vec3, mx: Vec3) -> Entity:
        return self._add(EXP_BOX, (*mn, *mx))

    def _add(self, kind: int, args: Sequence[float]) -> Entity:
        e = Entity(kind, tuple(float(a) for a in args))
        self.entities.append(e)
        return e

    # -- text form ------------------------------------------------------------------------------
    def to_scn(self) -> str:
        r = repr
        out = [f"# gi scene v1: {self.name}",
               "octree " + " ".join(r(float(v)) for v in (*self.octree_min, *self.octree_max)),
               "camera " + " ".join(r(float(v)) for v in (*self.cam_pos, *self.cam_look, self.focal)),
               "light " + " ".join(r(float(v)) for v in self.light)]
        for e in self.entities:
            out.append(_KW[e.kind] + " " + " ".join(r(a) for a in e.args))
            if e.material is not None:
                m = e.material
                vals = (*m.color, *m.shader, m.specular_power) + ((m.reflectivity,) if m.reflectivity else ())
                out.append("material " + " ".join(r(float(v)) for v in vals))
        return "\n".join(out) + "\n"

    def digest(self) -> str:
        return hashlib.sha256(self.to_scn().encode()).hexdigest()


def parse_scn(text: str) -> Scene:
    s = Scene(entities=[])
    for raw in text.splitlines():
        line = raw.split("#", 1)[0].strip()
        if not line:
            continue
        kw, *vals = line.split()
        v = [float(x) for x in vals]
        if kw == "octree":
            s.octree_min, s.octree_max = tuple(v[0:3]), tuple(v[3:6])
        elif kw == "camera":
            s.cam_pos, s.cam_look, s.focal = tuple(v[0:3]), tuple(v[3:6]), v[6]
        elif kw == "light":
            s.light = tuple(v[0:3])
        elif kw == "material":
            if not s.entities:
                raise ValueError("material before any entity")
            m = Material(tuple(v[0:3]))
            if len(v) >= 6:
                m.shader = tuple(v[3:6])
            if len(v) >= 7:
                m.specular_power = v[6]
            if len(v) >= 8:
                m.reflectivity = v[7]
            s.entities[-1].material = m
        elif kw in _KIND:
            k = _KIND[kw]
            if len(v) < _NARGS[k]:
                raise ValueError(f"{kw}: expected {_NARGS[k]} numbers, got {len(v)}")
            s.entities.append(Entity(k, tuple(v[: _NARGS[k]])))
        else:
            raise ValueError(f"unknown scene keyword {kw!r}")
    return s


# gi_obj.cpp's number grammar (is_real / parse_index), ASCII digits only: float() and int() alone
# would also take "1_0", "inf", "nan" and non-ASCII digits, which the C parser rejects
_OBJ_REAL = re.compile(r"[+-]?(?:[0-9]+(?:\.[0-9]*)?|\.[0-9]+)(?:[eE][+-]?[0-9]+)?", re.ASCII)
_OBJ_INT = re.compile(r"[+-]?[0-9]+", re.ASCII)


def load_obj(text: str, material: Optional[Material] = None, scene: Optional[Scene] = None) -> Scene:
    """Wavefront OBJ text -> ImpTriangle entities appended to `scene` (a new Scene if None), one per
    triangle of each face's fan (v0, v_k, v_k+1) in file order, each with `material` (None: the
    reference's default ImpTriangle material).  The same rules as libgi's gi_obj_parse
    (2019global_amd/csrc/gi_obj.cpp; tests compare the two): v (values after xyz ignored), f with
    i, i/t, i//n, i/t/n references (1-based, negative = relative to the last vertex), '#' comments,
    '\\' continuations; vt, vn, vp, o, g, s, usemtl, mtllib, l, p are skipped.  ValueError with the
    line number on a malformed v / f line or a vertex reference out of range."""
    s = scene if scene is not None else Scene(name="obj", entities=[])
    verts: List[Vec3] = []
    lines = text.split("\n")
    k = 0
    while k < len(lines):
        parts = []
        while True:   # one logical line: a physical line ending in '\' (before any comment) continues
            raw = lines[k].rstrip("\r")
            k += 1
            h = raw.find("#")
            body = raw if h < 0 else raw[:h]
            if h < 0 and raw.endswith("\\"):
                parts.append(raw[:-1])
                if k >= len(lines):
                    break
                continue
            parts.append(body)
            break
        lineno = k   # the logical line's last physical line, as gi_obj_parse reports it
        tok = " ".join(parts).replace("\t", " ").replace("\r", " ").split(" ")
        tok = [t for t in tok if t]
        if not tok:
            continue
        if tok[0] == "v":
            if len(tok) < 4:
                raise ValueError(f"obj line {lineno}: v needs 3 coordinates")
            if not all(_OBJ_REAL.fullmatch(t) for t in tok[1:4]):
                raise ValueError(f"obj line {lineno}: bad coordinate")
            xyz = tuple(float(t) for t in tok[1:4])
            if not all(math.isfinite(c) for c in xyz):
                raise ValueError(f"obj line {lineno}: bad coordinate")
            verts.append(xyz)
        elif tok[0] == "f":
            if len(tok) < 4:
                raise ValueError(f"obj line {lineno}: a face needs 3 vertices")
            idx = []
            for t in tok[1:]:
                ref = t.split("/", 1)[0]
                if not _OBJ_INT.fullmatch(ref):
                    raise ValueError(f"obj line {lineno}: bad vertex reference")
                r = int(ref, 10)
                if r == 0:
                    raise ValueError(f"obj line {lineno}: bad vertex reference")
                z = r - 1 if r > 0 else len(verts) + r
                if not 0 <= z < len(verts):
                    raise ValueError(f"obj line {lineno}: vertex {r} out of range")
                idx.append(z)
            for j in range(1, len(idx) - 1):
                e = s._add(IMP_TRIANGLE, (*verts[idx[0]], *verts[idx[j]], *verts[idx[j + 1]]))
                if material is not None:
                    e.material = Material(material.color, material.shader, material.specular_power,
                                          material.reflectivity)
    return s


# ---------------------------------------------------------------------------------------------
# Config scenes
# ---------------------------------------------------------------------------------------------

def main_scene() -> Scene:
    """main.cpp:24-48: camera (-10,0,0)->(1,0,0) f=0.1, light (-10,10,10), ExpQuad + 2 spheres."""
    s = Scene(name="main")
    s.exp_quad((0.0, 0.0, 0.0), 2, 3, 90.0 * math.pi / 180.0, (1, 2, 3))
    s.imp_sphere((3.0, 4.0, 4.0), 2, (1, 0, 0))
    s.imp_sphere((4.0, -4.0, 4.0), 2, (0, 0, 1))
    return s


def sphere_scene() -> Scene:
    """C1: single ImpSphere r=2 at the origin, colour (1,0,0), light (-10,10,10)."""
    s = Scene(name="sphere")
    s.imp_sphere((0.0, 0.0, 0.0), 2, (1, 0, 0))
    return s


def _quad(s: Scene, a: Vec3, b: Vec3, c: Vec3, d: Vec3, color: Vec3) -> None:
    s.imp_triangle(a, b, c, color)
    s.imp_triangle(a, c, d, color)


def _block(s: Scene, lo: Vec3, hi: Vec3, color: Vec3) -> None:
    x0, y0, z0 = lo
    x1, y1, z1 = hi
    _quad(s, (x0, y0, z0), (x1, y0, z0), (x1, y1, z0), (x0, y1, z0), color)  # bottom
    _quad(s, (x0, y0, z1), (x1, y0, z1), (x1, y1, z1), (x0, y1, z1), color)  # top
    _quad(s, (x0, y0, z0), (x1, y0, z0), (x1, y0, z1), (x0, y0, z1), color)  # y = y0
    _quad(s, (x0, y1, z0), (x1, y1, z0), (x1, y1, z1), (x0, y1, z1), color)  # y = y1
    _quad(s, (x0, y0, z0), (x0, y1, z0), (x0, y1, z1), (x0, y0, z1), color)  # x = x0
    _quad(s, (x1, y0, z0), (x1, y1, z0), (x1, y1, z1), (x1, y0, z1), color)  # x = x1


def cornell_scene() -> Scene:
    """C2/C3: Cornell box of 34 ImpTriangles; colours are 0/1 integers (A.7)."""
    s = Scene(name="cornell", light=(5.0, 0.0, 4.5))
    W, R, G = (1, 1, 1), (1, 0, 0), (0, 1, 0)
    _quad(s, (10, -5, -5), (10, 5, -5), (10, 5, 5), (10, -5, 5), W)   # back wall x=10
    _quad(s, (0, 5, -5), (10, 5, -5), (10, 5, 5), (0, 5, 5), R)       # left wall y=+5
    _quad(s, (0, -5, -5), (10, -5, -5), (10, -5, 5), (0, -5, 5), G)   # right wall y=-5
    _quad(s, (0, -5, -5), (10, -5, -5), (10, 5, -5), (0, 5, -5), W)   # floor z=-5
    _quad(s, (0, -5, 5), (10, -5, 5), (10, 5, 5), (0, 5, 5), W)       # ceiling z=+5
    _block(s, (5.0, -3.5, -5.0), (7.5, -1.0, -2.0), W)                 # short block
    _block(s, (6.5, 0.5, -5.0), (9.0, 3.0, 0.5), W)                    # tall block
    assert len(s.entities) == 34
    return s


def cornell_mirror_scene() -> Scene:
    """Mode X mirror-bounce coverage (Material.reflectivity, no reference counterpart; not a BASELINE
    config): the Cornell box with a perfect-mirror tall block, a half-mirror back wall and a
    mirror-like ImpSphere in front of the short block."""
    s = cornell_scene()
    s.name = "cornell_mirror"
    for e in s.entities[:2]:                       # back wall
        e.material.reflectivity = 0.5
    for e in s.entities[22:34]:                    # tall block
        e.material.reflectivity = 1.0
    sp = s.imp_sphere((4.0, -2.0, -3.5), 1.5, (1, 1, 0))
    sp.material = Material((1.0, 1.0, 0.0), reflectivity=0.8)
    return s


_GAMMA = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, n: int) -> np.ndarray:
    """First n outputs of splitmix64(seed) (state += gamma; mix)."""
    with np.errstate(over="ignore"):
        k = np.arange(1, n + 1, dtype=np.uint64)
        z = np.uint64(seed) + k * _GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def soup_vertices(n: int = 100_000, seed: int = 2019) -> np.ndarray:
    """(n, 3, 3) float64 vertices: centre x~U[0,10], y,z~U[-5,5]; vertex = centre + 0.15*U(-1,1)^3.

    Draw order per triangle: cx, cy, cz, then v1.xyz, v2.xyz, v3.xyz (12 draws)."""
    u = (splitmix64(seed, 12 * n) >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    u = u.reshape(n, 12)
    c = np.empty((n, 3))
    c[:, 0] = 10.0 * u[:, 0]
    c[:, 1] = -5.0 + 10.0 * u[:, 1]
    c[:, 2] = -5.0 + 10.0 * u[:, 2]
    off = 0.15 * (2.0 * u[:, 3:].reshape(n, 3, 3) - 1.0)
    return c[:, None, :] + off


def soup_scene(n: int = 100_000, seed: int = 2019) -> Scene:
    """C4/C5: n random white ImpTriangles, light (-10,10,10)."""
    s = Scene(name=f"soup{n}")
    v = soup_vertices(n, seed)
    white = Material((1.0, 1.0, 1.0))
    for t in v:
        e = s._add(IMP_TRIANGLE, (*t[0], *t[1], *t[2]))
        e.material = white
    return s


def soup_digest(n: int = 100_000, seed: int = 2019) -> str:
    """SHA-256 of the little-endian float64 vertex buffer (committed instead of the buffer)."""
    return hashlib.sha256(soup_vertices(n, seed).astype("<f8").tobytes()).hexdigest()


def zoo_scene() -> Scene:
    """Every entity type of entities.h in one frame: the commented-out scene
    objects of main.cpp:31-40 plus an ExpRectangle/ExpBox; not a BASELINE config."""
    s = Scene(name="zoo")
    s.exp_sphere((-2.0, 0.0, 0.0), 2, (0, 1, 0))                    # main.cpp:38
    s.exp_cube((0.0, 0.0, 0.0), 2, 2, 2, (1, 0, 0))                 # main.cpp:39
    s.exp_cone((0.0, 0.0, 2.0), (-1.0, 1.0, -3.0), 5, 3, (1, 1, 0))  # main.cpp:37
    s.exp_quad((0.0, 0.0, 0.0), 2, 3, 90.0 * math.pi / 180.0, (1, 2, 3))
    s.imp_sphere((3.0, 4.0, 4.0), 2, (1, 0, 0))
    s.imp_triangle((0.0, 3.0, 2.0), (3.0, 3.0, -4.0), (3.0, -3.0, -4.0), (0, 1, 1))   # main.cpp:36
    s.exp_rectangle((1.0, -6.0, -3.0), (1.0, -3.0, 0.0), (1.0, -6.0, 0.0))
    s.exp_box((2.0, 4.0, -5.0), (4.0, 6.0, -3.0))
    return s


def only_scene(kind_name: str) -> Scene:
    """One entity of the zoo alone, e.g. only_scene("expcone") (exercises its shading in frames)."""
    z = zoo_scene()
    s = Scene(name=f"only_{kind_name}")
    s.entities = [e for e in z.entities if _KW[e.kind] == kind_name]
    assert s.entities, kind_name
    return s


def named_scene(name: str) -> Scene:
    """Scene factory used by tests, goldens and bench: main, sphere, cornell, zoo, soupN, only_<kind>."""
    if name.startswith("soup"):
        return soup_scene(int(name[4:]))
    if name.startswith("only_"):
        return only_scene(name[5:])
    return CONFIG_SCENES[name]()


CONFIG_SCENES = {
    "main": main_scene,
    "sphere": sphere_scene,
    "cornell": cornell_scene,
    "zoo": zoo_scene,
    "cornell_mirror": cornell_mirror_scene,
}
