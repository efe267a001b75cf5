"""2019global_amd — MI355X-native (gfx950) per-pixel radiance path for preon7/2019global.

Host-side mirror of the reference's render API over the C-ABI in ``include/gi.h`` (``libgi.so``):

  reference (C++ header-only)                         here
  ---------------------------------------------------  ------------------------------------------
  Camera(pos, lookAt, focal)        camera.h:8-10      Camera(pos, look_at, focal)
  Octree(min, max) / push_back(e)   octree.h:14,20   Octree(min, max) / push_back(e)
  ImpSphere / ImpTriangle / ExpQuad entities.h:45,138,581  same names and constructor arguments
  Material(color[, shader]), .specular_power           Material(color, shader, specular_power)
  RayTracer(camera, light)          raytracer.h:18     RayTracer(camera, light)
    .setScene(octree) / .run(w, h) / .start() / .stop() / .running() / .getImage()

``RayTracer.run`` renders on the GPU through ``gi_render`` and returns when the frame is done (or
``stop()`` was called from another thread); ``getImage()`` returns the RGB888 frame the reference's
``Image`` would hold.  There is no CPU fallback: without ``libgi.so`` or a gfx950 device every
render raises ``GIError``.

Lower-level handles for benchmarks and multi-GPU: ``DeviceScene`` (a scene resident in HBM) with
``render_device`` into caller-owned device buffers on a HIP stream; ``MultiScene`` (several GPUs of
one process, RCCL gather; ``RayTracer`` uses it when ``GI_DEVICES`` lists more than one device);
``Octree.intersect`` (the reference's public candidate query, on the host).
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional, Sequence

import numpy as np

from . import scenes as _scenes

__all__ = [
    "GIError", "lib", "Camera", "Material", "Octree", "ImpSphere", "ImpTriangle", "ExpQuad",
    "ExpSphere", "ExpCube", "ExpCone", "ExpRectangle", "ExpBox",
    "RayTracer", "DeviceScene", "MODE_R", "MODE_X", "STAT_RAYS", "STAT_NODES", "STAT_PRIMS",
    "STAT_PIXELS", "TILE", "MultiScene", "devices_from_env", "obj_entities",
]

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("GI_LIB") or os.path.join(HERE, "libgi.so")   # GI_LIB: A/B builds

MODE_R, MODE_X = 0, 1
FLAG_STATS = 1
FLAG_R_DFS = 2   # Mode R: reverse-DFS over the whole reference octree (A/B against the default)
FLAG_TIME = 4    # HIP events around the dominant kernel; read with DeviceScene.kernel_ms()
FLAG_X_NO_SHADOW = 8   # Mode X, tests only: no shadow rays (reduces depth-1 Mode X to the reference's shading)
FLAG_X_WF = 16   # Mode X: the wavefront form (one launch per bounce over compacted path queues, gi_wf.hip)
FLAG_X_MEGA = 32   # Mode X: the persistent path-state kernel k_mode_x
FLAG_X_SEG = 64   # Mode X: the segment-synchronous persistent form k_seg (no form flag: chosen per launch)
X_FORMS = ("k_mode_x", "k_wf_bounce", "k_seg")   # gi_scene_x_form's values
R_KERNELS = ("k_mode_r", "k_rf_walk", "k_mode_r_batch")   # gi_scene_r_kernel's (1: the flat phases)
STAT_RAYS, STAT_NODES, STAT_PRIMS, STAT_PIXELS, STAT_X_PATH_MAX = 0, 1, 2, 3, 4
STAT_X_ITERS, STAT_X_TRAV, STAT_X_HANDLE, STAT_X_HLANES, STAT_X_HCLOSE, STAT_X_HSHADOW = 5, 6, 7, 8, 9, 10
STAT_X_CYC_TRAV, STAT_X_CYC_HIT, STAT_X_CYC_NEXT, STAT_X_CYC_ALL = 11, 12, 13, 14
STAT_X_RESOLVED = 15
STAT_X_IT_NODE, STAT_X_LN_NODE, STAT_X_IT_LEAF, STAT_X_LN_LEAF = 16, 17, 18, 19
STAT_X_IT_RS, STAT_X_LN_RS, STAT_X_IT_ST, STAT_X_LN_ST = 20, 21, 22, 23
STAT_R_PAIRS, STAT_R_OVF_TILES = 24, 25
STATS_N = 26
TILE = 8
ABI_VERSION = 10


class GIError(RuntimeError):
    pass


# ---- C structures (include/gi.h) -------------------------------------------------------------
class EntityDesc(ctypes.Structure):
    _fields_ = [("kind", ctypes.c_int32), ("has_material", ctypes.c_int32), ("args", ctypes.c_double * 11),
                ("mat_color", ctypes.c_double * 3), ("mat_shader", ctypes.c_double * 3),
                ("mat_specular_power", ctypes.c_double), ("mat_reflectivity", ctypes.c_double)]


class SceneDesc(ctypes.Structure):
    _fields_ = [("octree_min", ctypes.c_double * 3), ("octree_max", ctypes.c_double * 3),
                ("n_entities", ctypes.c_int32), ("entities", ctypes.POINTER(EntityDesc))]


class CameraDesc(ctypes.Structure):
    _fields_ = [("pos", ctypes.c_double * 3), ("up", ctypes.c_double * 3), ("forward", ctypes.c_double * 3),
                ("focal", ctypes.c_double)]


class Opts(ctypes.Structure):
    _fields_ = [("mode", ctypes.c_int32), ("spp", ctypes.c_int32), ("depth", ctypes.c_int32),
                ("shard_count", ctypes.c_int32), ("shard_index", ctypes.c_int32), ("band_rows", ctypes.c_int32),
                ("flags", ctypes.c_uint32), ("reserved", ctypes.c_int32), ("seed", ctypes.c_uint64),
                ("stats", ctypes.c_void_p), ("sample_begin", ctypes.c_int32), ("sample_end", ctypes.c_int32)]


class SceneInfo(ctypes.Structure):
    _fields_ = [("n_entities", ctypes.c_int32), ("n_nodes", ctypes.c_int32), ("n_leaves", ctypes.c_int32),
                ("max_depth", ctypes.c_int32), ("n_reachable", ctypes.c_int32), ("n_dropped", ctypes.c_int32),
                ("x_nodes", ctypes.c_int32), ("x_prims", ctypes.c_int32), ("device_bytes", ctypes.c_int64),
                ("x_node_bytes", ctypes.c_int32), ("x_lds_resident", ctypes.c_int32)]


class Hit(ctypes.Structure):
    _fields_ = [("entity", ctypes.c_int32), ("u", ctypes.c_int32), ("v", ctypes.c_int32),
                ("point", ctypes.c_double * 3), ("normal", ctypes.c_double * 3)]


TILE_CB = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.POINTER(ctypes.c_uint8),
                           ctypes.POINTER(ctypes.c_double))

EXPORTS = ["gi_abi_version", "gi_last_error", "gi_camera_init", "gi_scene_create", "gi_scene_destroy",
           "gi_scene_get_info", "gi_render", "gi_render_device", "gi_shard_tiles", "gi_unshard_device",
           "gi_trace_ray", "gi_kat_expbox", "gi_scene_kernel_ms", "gi_scene_x_form", "gi_scene_r_kernel", "gi_octree_create", "gi_octree_destroy",
           "gi_octree_intersect", "gi_multi_create", "gi_multi_destroy", "gi_multi_info", "gi_multi_render", "gi_device_count",
           "gi_device_list", "gi_build_id", "gi_obj_parse"]

_lib = None
_lock = threading.Lock()


def lib():
    """Load libgi.so (built in-tree by ``2019global_amd/build.py``).  torch, when importable, is
    imported first so that libgi binds to the same HIP runtime instance torch uses."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise GIError(f"{LIB_PATH} is missing: run `python 2019global_amd/build.py` (no CPU fallback)")
        try:
            import torch  # noqa: F401  (one HIP runtime per process)
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, dp = ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_double)
        L.gi_abi_version.restype = i32
        L.gi_last_error.restype = ctypes.c_char_p
        L.gi_camera_init.argtypes = [dp, dp, ctypes.c_double, ctypes.POINTER(CameraDesc)]
        L.gi_scene_create.argtypes = [ctypes.POINTER(SceneDesc), ctypes.POINTER(vp)]
        L.gi_scene_destroy.argtypes = [vp]
        L.gi_scene_destroy.restype = None
        L.gi_scene_get_info.argtypes = [vp, ctypes.POINTER(SceneInfo)]
        L.gi_render.argtypes = [vp, ctypes.POINTER(CameraDesc), dp, i32, i32, ctypes.POINTER(Opts), dp,
                                ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int), TILE_CB, vp]
        L.gi_render_device.argtypes = [vp, ctypes.POINTER(CameraDesc), dp, i32, i32, ctypes.POINTER(Opts), vp, vp, vp]
        L.gi_shard_tiles.argtypes = [i32, i32, i32]
        L.gi_shard_tiles.restype = ctypes.c_int64
        L.gi_unshard_device.argtypes = [i32, i32, i32, vp, vp, vp, vp, vp]
        L.gi_trace_ray.argtypes = [vp, dp, dp, dp, ctypes.POINTER(Hit), dp]
        L.gi_kat_expbox.argtypes = [i32, dp, ctypes.POINTER(ctypes.c_int32)]
        L.gi_scene_kernel_ms.argtypes = [vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int64)]
        L.gi_scene_x_form.argtypes = [vp, ctypes.POINTER(Opts), ctypes.POINTER(ctypes.c_int32)]
        L.gi_scene_r_kernel.argtypes = [vp, ctypes.POINTER(Opts), ctypes.POINTER(ctypes.c_int32)]
        L.gi_octree_create.argtypes = [ctypes.POINTER(SceneDesc), ctypes.POINTER(vp)]
        L.gi_octree_destroy.argtypes = [vp]
        L.gi_octree_destroy.restype = None
        L.gi_octree_intersect.argtypes = [vp, dp, dp, ctypes.POINTER(ctypes.c_int32), ctypes.c_int64,
                                          ctypes.POINTER(ctypes.c_int64)]
        L.gi_multi_create.argtypes = [ctypes.POINTER(SceneDesc), i32, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(vp)]
        L.gi_multi_destroy.argtypes = [vp]
        L.gi_multi_destroy.restype = None
        L.gi_multi_info.argtypes = [vp, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int),
                                    ctypes.POINTER(ctypes.c_int)]
        L.gi_multi_render.argtypes = [vp, ctypes.POINTER(CameraDesc), dp, i32, i32, ctypes.POINTER(Opts), dp,
                                      ctypes.POINTER(ctypes.c_uint8), ctypes.POINTER(ctypes.c_int), TILE_CB, vp]
        L.gi_device_list.argtypes = [ctypes.POINTER(ctypes.c_int32), i32]
        L.gi_build_id.restype = ctypes.c_char_p
        L.gi_obj_parse.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.POINTER(EntityDesc),
                                   ctypes.POINTER(EntityDesc), ctypes.c_int64, ctypes.POINTER(ctypes.c_int64)]
        if L.gi_abi_version() != ABI_VERSION:
            raise GIError(f"libgi ABI {L.gi_abi_version()} != {ABI_VERSION}")
        _lib = L
        return L


def build_id() -> str:
    """Source hash the loaded libgi was compiled from (build.py source_hash)."""
    return lib().gi_build_id().decode()


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise GIError(f"{what} failed ({rc}): {lib().gi_last_error().decode()}")


def _d3(v) -> ctypes.Array:
    return (ctypes.c_double * 3)(*[float(x) for x in v])


# ---- reference-shaped API ---------------------------------------------------------------------
class Material:
    """Material(color[, shader]) (material.h:13-20); specular_power (material.h:29).
    reflectivity: Mode X only (no reference counterpart) -- probability that a bounce is a mirror
    reflection instead of a diffuse sample; 0 = the reference's diffuse-only material."""

    def __init__(self, color, shader=(0.1, 0.7, 1.0), specular_power: float = 5.0, reflectivity: float = 0.0):
        self.color = tuple(float(c) for c in color)
        self.shader_parameters = tuple(float(c) for c in shader)
        self.specular_power = float(specular_power)
        self.reflectivity = float(reflectivity)


class _Entity:
    kind = 0

    def __init__(self, args: Sequence[float], material: Optional[Material]):
        self._args = tuple(float(a) for a in args)
        self._material = material   # explicit override (entity->material = ...)

    @property
    def material(self) -> Optional[Material]:
        return self._material

    @material.setter
    def material(self, m: Material) -> None:
        self._material = m

    def _desc(self, d: EntityDesc) -> None:
        d.kind = self.kind
        for i, a in enumerate(self._args):
            d.args[i] = a
        m = self._material
        d.has_material = 1 if m is not None else 0
        if m is not None:
            for i in range(3):
                d.mat_color[i] = m.color[i]
                d.mat_shader[i] = m.shader_parameters[i]
            d.mat_specular_power = m.specular_power
            d.mat_reflectivity = m.reflectivity


class ImpSphere(_Entity):
    """ImpSphere(pos, float radius, color) (entities.h:45)."""
    kind = _scenes.IMP_SPHERE

    def __init__(self, pos, radius, color):
        super().__init__((*pos, radius, *color), None)


class ImpTriangle(_Entity):
    """ImpTriangle(p1, p2, p3) (entities.h:138); default material red (entities.h:21)."""
    kind = _scenes.IMP_TRIANGLE

    def __init__(self, p1, p2, p3):
        super().__init__((*p1, *p2, *p3), None)


class ExpQuad(_Entity):
    """ExpQuad(pos, float width, float length, float alpha, color) (entities.h:581)."""
    kind = _scenes.EXP_QUAD

    def __init__(self, pos, width, length, alpha, color):
        super().__init__((*pos, width, length, alpha, *color), None)


class ExpSphere(_Entity):
    """ExpSphere(pos, float radius, color) (entities.h:461): 10x10 stack/sector triangle mesh."""
    kind = _scenes.EXP_SPHERE

    def __init__(self, pos, radius, color):
        super().__init__((*pos, radius, *color), None)


class ExpCube(_Entity):
    """ExpCube(pos, float width, float length, float height, color) (entities.h:652)."""
    kind = _scenes.EXP_CUBE

    def __init__(self, pos, width, length, height, color):
        super().__init__((*pos, width, length, height, *color), None)


class ExpCone(_Entity):
    """ExpCone(pos, dir, float height, float radius, color) (entities.h:823).  As in the reference,
    dir is kept but the mesh always points along (-1, 0, -10) (:825)."""
    kind = _scenes.EXP_CONE

    def __init__(self, pos, dir, height, radius, color):
        super().__init__((*pos, *dir, height, radius, *color), None)


class ExpRectangle(_Entity):
    """ExpRectangle(p1, p2, p3) (entities.h:310); requires (p1-p3).(p2-p3) == 0 (:312)."""
    kind = _scenes.EXP_RECTANGLE

    def __init__(self, p1, p2, p3):
        super().__init__((*p1, *p2, *p3), None)


class ExpBox(_Entity):
    """ExpBox(min, max) (entities.h:381); getTextureCoord is (0, 0)."""
    kind = _scenes.EXP_BOX

    def __init__(self, mn, mx):
        super().__init__((*mn, *mx), None)


def obj_entities(text, material: Optional[Material] = None) -> list:
    """A Wavefront OBJ mesh (text or bytes) as ImpTriangle entities (entities.h:138), one per
    triangle of each face's fan in file order, through libgi's gi_obj_parse (no device needed);
    push them onto an Octree like hand-built entities.  `material` is set on every triangle (None:
    the reference's default ImpTriangle material)."""
    L = lib()
    data = text.encode() if isinstance(text, str) else bytes(text)
    tmpl = None
    if material is not None:
        tmpl = EntityDesc()
        t = _Entity((), material)
        t._desc(tmpl)
    n = ctypes.c_int64()
    _check(L.gi_obj_parse(data, len(data), tmpl, None, 0, ctypes.byref(n)), "gi_obj_parse")
    arr = (EntityDesc * max(1, n.value))()
    _check(L.gi_obj_parse(data, len(data), tmpl, arr, n.value, ctypes.byref(n)), "gi_obj_parse")
    out = []
    for i in range(n.value):
        d = arr[i]
        e = ImpTriangle(tuple(d.args[0:3]), tuple(d.args[3:6]), tuple(d.args[6:9]))
        if material is not None:
            e.material = Material(material.color, material.shader_parameters, material.specular_power,
                                  material.reflectivity)
        out.append(e)
    return out


class Octree:
    """Octree(min, max) + push_back (octree.h:14-43).  The tree itself is built by libgi from the
    push order (gi_scene_create), exactly as the reference builds it."""

    def __init__(self, min=(-20, -20, -20), max=(20, 20, 20)):
        self.min = tuple(float(v) for v in min)
        self.max = tuple(float(v) for v in max)
        self.entities = []
        self.generation = 0       # bumped by push_back: a RayTracer re-uploads a changed scene
        self._host = None         # gi_octree for intersect(), rebuilt when the generation changes
        self._host_gen = -1

    def push_back(self, e: _Entity) -> None:
        self.entities.append(e)
        self.generation += 1

    def intersect(self, origin, direction) -> list:
        """Octree::intersect(Ray(origin, dir)) (octree.h:46-68 -> Node::intersect :132-155): the
        candidate list -- entities in DFS order over children 0..7, duplicates kept -- from libgi's
        host copy of the reference octree (gi_octree_intersect; no device needed).  `direction` is
        normalised first, as the reference's Ray constructor does (ray.h:6)."""
        L = lib()
        if self._host is None or self._host_gen != self.generation:
            self._close_host()
            d, keep = self._scene_desc()
            h = ctypes.c_void_p()
            _check(L.gi_octree_create(ctypes.byref(d), ctypes.byref(h)), "gi_octree_create")
            del keep
            self._host, self._host_gen = h, self.generation
        dv = np.asarray(direction, np.float64)
        dv = dv * (1.0 / np.sqrt((dv[0] * dv[0] + dv[1] * dv[1]) + dv[2] * dv[2]))   # glm::normalize
        n = ctypes.c_int64()
        _check(L.gi_octree_intersect(self._host, _d3(origin), _d3(dv), None, 0, ctypes.byref(n)), "gi_octree_intersect")
        out = (ctypes.c_int32 * max(1, n.value))()
        _check(L.gi_octree_intersect(self._host, _d3(origin), _d3(dv), out, n.value, ctypes.byref(n)),
               "gi_octree_intersect")
        return [self.entities[i] for i in out[:n.value]]

    def _close_host(self):
        if self._host is not None and self._host.value:
            lib().gi_octree_destroy(self._host)
        self._host = None

    def __del__(self):
        try:
            self._close_host()
        except Exception:
            pass

    @classmethod
    def from_scene(cls, s: "_scenes.Scene") -> "Octree":
        o = cls(s.octree_min, s.octree_max)
        for e in s.entities:
            ent = _Entity(e.args, None if e.material is None else
                          Material(e.material.color, e.material.shader, e.material.specular_power,
                                   e.material.reflectivity))
            ent.kind = e.kind
            o.push_back(ent)
        return o

    def _scene_desc(self):
        n = len(self.entities)
        arr = (EntityDesc * max(n, 1))()
        for i, e in enumerate(self.entities):
            e._desc(arr[i])
        d = SceneDesc()
        d.octree_min = _d3(self.min)
        d.octree_max = _d3(self.max)
        d.n_entities = n
        d.entities = ctypes.cast(arr, ctypes.POINTER(EntityDesc))
        return d, arr


class Camera:
    """Camera(pos, lookAt, focal) (camera.h:8-10): up = (0,0,1), forward = normalize(lookAt - pos)."""

    def __init__(self, pos, lookAt=(0.0, 0.0, 0.0), focal: float = 0.04):
        self._c = CameraDesc()
        _check(lib().gi_camera_init(_d3(pos), _d3(lookAt), float(focal), ctypes.byref(self._c)), "gi_camera_init")

    @property
    def pos(self):
        return tuple(self._c.pos)

    @property
    def up(self):
        return tuple(self._c.up)

    @property
    def forward(self):
        return tuple(self._c.forward)

    @property
    def focalDist(self):
        return self._c.focal


class DeviceScene:
    """A scene resident in HBM on the current HIP device (gi_scene_create)."""

    def __init__(self, octree: Octree):
        L = lib()
        d, keep = octree._scene_desc()
        h = ctypes.c_void_p()
        _check(L.gi_scene_create(ctypes.byref(d), ctypes.byref(h)), "gi_scene_create")
        self._h = h
        del keep

    @classmethod
    def from_scene(cls, s: "_scenes.Scene") -> "DeviceScene":
        return cls(Octree.from_scene(s))

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            lib().gi_scene_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def info(self) -> dict:
        i = SceneInfo()
        _check(lib().gi_scene_get_info(self._h, ctypes.byref(i)), "gi_scene_get_info")
        return {f: getattr(i, f) for f, _ in SceneInfo._fields_}

    @staticmethod
    def opts(mode=MODE_R, spp=1, depth=1, seed=0, shard_count=1, shard_index=0, band_rows=0, stats_ptr=0,
             flags=0, samples=None) -> Opts:
        """samples=(begin, end): a progressive pass of Mode X samples [begin, end) (gi.h gi_opts)."""
        o = Opts()
        o.mode, o.spp, o.depth, o.seed = mode, spp, depth, seed
        o.shard_count, o.shard_index, o.band_rows = shard_count, shard_index, band_rows
        o.flags = (FLAG_STATS if stats_ptr else 0) | flags
        o.stats = stats_ptr or None
        if samples is not None:
            o.sample_begin, o.sample_end = samples
        return o

    def render(self, cam: Camera, light, w: int, h: int, mode=MODE_R, spp=1, depth=1, seed=0, band_rows=0,
               cancel: Optional[ctypes.c_int] = None, callback=None, out=None, flags=0, samples=None):
        """Host-buffer render (gi_render).  Returns (rgb float64 [h,w,3], rgb8 uint8 [h,w,3]).
        out=(rgb, rgb8): caller-owned C-contiguous arrays to fill instead (either may be None:
        that output is not copied back).  samples=(begin, end): one progressive Mode X pass."""
        if out is None:
            rgb, rgb8 = np.zeros((h, w, 3), np.float64), np.zeros((h, w, 3), np.uint8)
        else:
            rgb, rgb8 = out
        for a, dt in ((rgb, np.float64), (rgb8, np.uint8)):
            if a is not None and (a.dtype != dt or a.size != w * h * 3 or not a.flags.c_contiguous):
                raise ValueError("render: out arrays must be C-contiguous [h, w, 3] float64 / uint8")
        cb = TILE_CB(callback) if callback is not None else TILE_CB()
        o = self.opts(mode, spp, depth, seed, band_rows=band_rows, flags=flags, samples=samples)
        _check(lib().gi_render(self._h, ctypes.byref(cam._c), _d3(light), w, h, ctypes.byref(o),
                               rgb.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if rgb is not None else None,
                               rgb8.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if rgb8 is not None else None,
                               ctypes.byref(cancel) if cancel is not None else None, cb, None), "gi_render")
        return rgb, rgb8

    def render_device(self, cam: Camera, light, w: int, h: int, d_rgb: int, d_rgb8: int = 0, stream: int = 0,
                      mode=MODE_R, spp=1, depth=1, seed=0, shard_count=1, shard_index=0, stats_ptr=0,
                      flags=0, samples=None) -> None:
        """Asynchronous render into device buffers (gi_render_device); pointers are ints."""
        o = self.opts(mode, spp, depth, seed, shard_count, shard_index, stats_ptr=stats_ptr, flags=flags,
                      samples=samples)
        _check(lib().gi_render_device(self._h, ctypes.byref(cam._c), _d3(light), w, h, ctypes.byref(o),
                                      d_rgb or None, d_rgb8 or None, stream or None), "gi_render_device")

    def x_form(self, mode=MODE_X, spp=1, depth=1, flags=0) -> str:
        """The Mode X form a render with these options would run: "k_mode_x" (persistent path-state
        kernel), "k_wf_bounce" (wavefront, one launch per bounce) or "k_seg" (segment-synchronous) --
        gi_scene_x_form."""
        o = self.opts(mode, spp, depth, 0, flags=flags)
        f = ctypes.c_int32()
        _check(lib().gi_scene_x_form(self._h, ctypes.byref(o), ctypes.byref(f)), "gi_scene_x_form")
        return X_FORMS[f.value]

    def r_kernel(self, flags=0) -> str:
        """The Mode R kernel a render would run: "k_mode_r" (one lane per pixel), "k_rf_walk" (the flat
        phases k_rf_*, their overflowed tiles by k_mode_r_batch) or "k_mode_r_batch" (the whole frame)
        -- gi_scene_r_kernel."""
        o = self.opts(MODE_R, 1, 1, 0, flags=flags)
        k = ctypes.c_int32()
        _check(lib().gi_scene_r_kernel(self._h, ctypes.byref(o), ctypes.byref(k)), "gi_scene_r_kernel")
        return R_KERNELS[k.value]

    def kernel_ms(self):
        """(average ms, launches) of the dominant kernel over the renders issued with FLAG_TIME since
        the previous call (gi_scene_kernel_ms; waits for the last one, then resets)."""
        ms, n = ctypes.c_float(), ctypes.c_int64()
        _check(lib().gi_scene_kernel_ms(self._h, ctypes.byref(ms), ctypes.byref(n)), "gi_scene_kernel_ms")
        return float(ms.value), int(n.value)

    def trace_ray(self, origin, direction, light):
        hit = Hit()
        rgb = (ctypes.c_double * 3)()
        _check(lib().gi_trace_ray(self._h, _d3(origin), _d3(direction), _d3(light), ctypes.byref(hit), rgb),
               "gi_trace_ray")
        return hit, tuple(rgb)


def devices_from_env(default=None):
    """GI_DEVICES="0,1,2,3" (device per shard; repeats allowed) or "all"; None when unset."""
    v = os.environ.get("GI_DEVICES")
    if not v:
        return default
    if v.strip() == "all":
        import torch
        return list(range(torch.cuda.device_count()))
    return [int(t) for t in v.split(",") if t.strip()]


class MultiScene:
    """RayTracer::run over several GPUs of this process (gi_multi_*): a scene replica per device,
    8x8 tiles dealt round-robin over the shards, packed tiles gathered to devices[0] by RCCL
    send/recv over xGMI, bit-identical to a one-device render."""

    def __init__(self, octree: Octree, devices: Sequence[int]):
        L = lib()
        d, keep = octree._scene_desc()
        devs = (ctypes.c_int * len(devices))(*[int(x) for x in devices])
        h = ctypes.c_void_p()
        _check(L.gi_multi_create(ctypes.byref(d), len(devices), devs, ctypes.byref(h)), "gi_multi_create")
        self._h = h
        del keep

    @classmethod
    def from_scene(cls, s: "_scenes.Scene", devices: Sequence[int]) -> "MultiScene":
        return cls(Octree.from_scene(s), devices)

    def info(self) -> dict:
        a, b, c = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _check(lib().gi_multi_info(self._h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)), "gi_multi_info")
        return {"shards": a.value, "devices": b.value, "rccl": bool(c.value)}

    def render(self, cam: Camera, light, w: int, h: int, mode=MODE_R, spp=1, depth=1, seed=0, band_rows=0,
               cancel: Optional[ctypes.c_int] = None, callback=None, out=None):
        """gi_multi_render into host arrays; out=(rgb, rgb8) as DeviceScene.render (either may be None)."""
        if out is None:
            rgb, rgb8 = np.zeros((h, w, 3), np.float64), np.zeros((h, w, 3), np.uint8)
        else:
            rgb, rgb8 = out
        for a, dt in ((rgb, np.float64), (rgb8, np.uint8)):
            if a is not None and (a.dtype != dt or a.size != w * h * 3 or not a.flags.c_contiguous):
                raise ValueError("render: out arrays must be C-contiguous [h, w, 3] float64 / uint8")
        cb = TILE_CB(callback) if callback is not None else TILE_CB()
        o = DeviceScene.opts(mode, spp, depth, seed, band_rows=band_rows)
        _check(lib().gi_multi_render(self._h, ctypes.byref(cam._c), _d3(light), w, h, ctypes.byref(o),
                                     rgb.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if rgb is not None else None,
                                     rgb8.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)) if rgb8 is not None else None,
                                     ctypes.byref(cancel) if cancel is not None else None, cb, None), "gi_multi_render")
        return rgb, rgb8

    def close(self) -> None:
        if getattr(self, "_h", None) and self._h.value:
            lib().gi_multi_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def kat_expbox(recs: np.ndarray) -> np.ndarray:
    """Device ExpBox node test over (min, max, origin, dir) records (gi_kat_expbox)."""
    recs = np.ascontiguousarray(recs, np.float64)
    out = np.zeros(recs.shape[0], np.int32)
    _check(lib().gi_kat_expbox(recs.shape[0], recs.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                               out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))), "gi_kat_expbox")
    return out


def shard_tiles(w: int, h: int, shard_count: int) -> int:
    return int(lib().gi_shard_tiles(w, h, shard_count))


def unshard_device(w, h, shard_count, d_packed, d_packed8, d_rgb, d_rgb8, stream=0) -> None:
    _check(lib().gi_unshard_device(w, h, shard_count, d_packed or None, d_packed8 or None, d_rgb or None,
                                   d_rgb8 or None, stream or None), "gi_unshard_device")


class Image:
    """What the reference's Image (image.h:7-29) holds after run(): RGB888 pixels."""

    def __init__(self, rgb8: np.ndarray, rgb: Optional[np.ndarray] = None):
        self.rgb8 = rgb8
        self.radiance = rgb

    def width(self) -> int:
        return self.rgb8.shape[1]

    def height(self) -> int:
        return self.rgb8.shape[0]

    def getPixel(self, x: int, y: int):
        p = self.rgb8[y, x]
        return (p[0] / 255.0, p[1] / 255.0, p[2] / 255.0)


class RayTracer:
    """RayTracer(camera, light) (raytracer.h:15-101) backed by the gfx950 kernels."""

    def __init__(self, camera: Camera, light):
        self._camera = camera
        self._light = tuple(float(v) for v in light)
        self._image = Image(np.zeros((0, 0, 3), np.uint8))
        self._scene: Optional[Octree] = None
        self._dev: Optional[DeviceScene] = None
        self._cancel = ctypes.c_int(1)   # _running = false (raytracer.h:96)
        self.band_rows = 64              # progressive granularity (reference: per pixel)

    def setScene(self, scene: Octree) -> None:
        self._scene = scene
        self._dev = None   # rebuilt lazily on the next run()
        self._dev_gen = -1

    def running(self) -> bool:
        return self._cancel.value == 0

    def stop(self) -> None:
        self._cancel.value = 1

    def start(self) -> None:
        self._cancel.value = 0

    def getImage(self) -> Image:
        return self._image

    def run(self, w: int, h: int) -> None:
        self._image = Image(np.zeros((h, w, 3), np.uint8), np.zeros((h, w, 3)))   # raytracer.h:25
        if self._scene is None:
            raise GIError("setScene() was not called")
        # the reference reads the live octree on every run (raytracer.h:45): re-upload after push_back
        if self._dev is None or getattr(self, "_dev_gen", -1) != self._scene.generation:
            devs = devices_from_env()
            self._dev = MultiScene(self._scene, devs) if devs and len(devs) > 1 else DeviceScene(self._scene)
            self._dev_gen = self._scene.generation
        img = self._image

        def on_band(_user, y0, rows, p8, pf):
            n = w * rows * 3
            img.rgb8[y0:y0 + rows] = np.ctypeslib.as_array(p8, shape=(n,)).reshape(rows, w, 3)
            img.radiance[y0:y0 + rows] = np.ctypeslib.as_array(pf, shape=(n,)).reshape(rows, w, 3)

        rgb = np.zeros((h, w, 3))
        rgb8 = np.zeros((h, w, 3), np.uint8)
        o = DeviceScene.opts(MODE_R, band_rows=self.band_rows)
        cb = TILE_CB(on_band)
        fn = lib().gi_multi_render if isinstance(self._dev, MultiScene) else lib().gi_render
        rc = fn(self._dev._h, ctypes.byref(self._camera._c), _d3(self._light), w, h, ctypes.byref(o),
                             rgb.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                             rgb8.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), ctypes.byref(self._cancel), cb, None)
        if rc not in (0, -4):   # -4: stopped, partial frame like the reference's loop exit
            _check(rc, "gi_render")
