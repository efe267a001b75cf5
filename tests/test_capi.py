"""CPU: the C-ABI library loads and exports every entry point include/gi.h declares; host-side logic
(scene text form, tile-shard layout) behaves; with no GPU the product fails loudly (no CPU
fallback)."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

import oracle_util as U

gi = U.pkg()
S = U.scenes()
HDR = os.path.join(U.ROOT, "include", "gi.h")


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|void|const char\*|int64_t)\s+(gi_\w+)\s*\(", txt, re.M)))


def test_library_built_and_exports_header_symbols():
    if not os.path.exists(gi.LIB_PATH):
        from importlib import import_module
        import_module("2019global_amd.build").build()
    out = subprocess.run(["nm", "-D", "--defined-only", gi.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (gi_\w+)", out))
    decl = declared_symbols()
    assert len(decl) >= 11
    missing = [s for s in decl if s not in exported]
    assert not missing, missing
    assert sorted(decl) == sorted(gi.EXPORTS)


def test_library_loads_and_abi_version():
    L = gi.lib()
    assert L.gi_abi_version() == gi.ABI_VERSION
    assert ctypes.sizeof(gi.EntityDesc) == 160
    assert ctypes.sizeof(gi.Opts) == 56   # ABI 10: + sample_begin, sample_end
    assert ctypes.sizeof(gi.CameraDesc) == 80


def test_loaded_library_built_from_this_tree():
    """Provenance: gi_build_id() of the libgi this process loaded equals the hash of
    the sources in the tree (build.py source_hash), so the suite -- here and in `pytest -m gpu` on
    the GPU box, which loads the same in-tree .so -- runs the kernels these sources define."""
    from importlib import import_module
    B = import_module("2019global_amd.build")
    assert gi.build_id() == B.source_hash()


def test_ctypes_layouts_match_header(tmp_path):
    """The Python mirror's structs against include/gi.h as the C compiler lays them out."""
    import subprocess
    src = tmp_path / "sz.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "gi.h"\n'
                   'int main(void) { printf("%zu %zu %zu %zu %zu\\n", sizeof(gi_entity_desc), '
                   'offsetof(gi_entity_desc, mat_reflectivity), sizeof(gi_opts), sizeof(gi_camera), '
                   'sizeof(gi_scene_desc)); return 0; }\n')
    exe = tmp_path / "sz"
    subprocess.run(["gcc", "-I", os.path.join(U.ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [ctypes.sizeof(gi.EntityDesc), gi.EntityDesc.mat_reflectivity.offset, ctypes.sizeof(gi.Opts),
                   ctypes.sizeof(gi.CameraDesc), ctypes.sizeof(gi.SceneDesc)]


def test_library_has_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", gi.LIB_PATH],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout


def test_camera_init_matches_oracle_basis():
    c = gi.Camera((-10, 0, 0), (1, 0, 0), 0.1)
    assert c.up == (0.0, 0.0, 1.0)
    assert c.forward == (1.0, 0.0, 0.0)
    c2 = gi.Camera((1, 2, 3), (4, -1, 7), 0.5)
    f = np.array([3.0, -3.0, 4.0])
    f = f * (1.0 / np.sqrt((f[0] * f[0] + f[1] * f[1]) + f[2] * f[2]))
    assert c2.forward == tuple(f)


def test_shard_tile_math():
    # 8x8 tiles, round-robin: every tile owned once, per-rank buffers padded to the same count
    for w, h, n in [(1920, 1080, 8), (512, 512, 3), (17, 9, 2), (256, 256, 1)]:
        tiles = ((w + 7) // 8) * ((h + 7) // 8)
        assert gi.shard_tiles(w, h, n) == -(-tiles // n)


def test_no_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(gi.GIError, match="device|HIP"):
        gi.DeviceScene.from_scene(S.sphere_scene())


def test_scene_text_roundtrip():
    for s in (S.main_scene(), S.cornell_scene(), S.soup_scene(50)):
        t = s.to_scn()
        s2 = S.parse_scn(t)
        assert s2.to_scn().split("\n", 1)[1] == t.split("\n", 1)[1]


def test_soup_vertex_generator():
    v = S.soup_vertices(1000, 2019)
    c = v.mean(axis=1)
    assert v.shape == (1000, 3, 3)
    assert (np.abs(v - c[:, None, :]) <= 0.3 + 1e-12).all()   # vertices within 0.15 of the drawn centre
    assert -0.15 <= c[:, 0].min() and c[:, 0].max() <= 10.15


def _primary_dirs(sc, w, xs, ys):
    """raytracer.h:26-30, 41-43 in fp64 with glm's operation order (same as the kernels' make_cam /
    primary_dir): the un-normalised primary directions of pixels (xs, ys)."""
    pos = np.array(sc.cam_pos, np.float64)
    look = np.array(sc.cam_look, np.float64)
    f = look - pos
    f = f * (1.0 / np.sqrt((f[0] * f[0] + f[1] * f[1]) + f[2] * f[2]))
    up = np.array([0.0, 0.0, 1.0])
    left = np.array([up[1] * f[2] - f[1] * up[2], up[2] * f[0] - f[2] * up[0], up[0] * f[1] - f[0] * up[1]])
    left = left * (1.0 / np.sqrt((left[0] * left[0] + left[1] * left[1]) + left[2] * left[2]))
    rx = ry = 0.0002
    tl = (((pos + sc.focal * f) + ((left * float(w)) * 0.5) * rx) + ((up * float(w)) * 0.5) * ry) - pos
    out = []
    for x, y in zip(xs, ys):
        out.append((tl - (left * float(x)) * rx) - (up * float(y)) * ry)
    return pos, out


@pytest.mark.parametrize("name", ["cornell_128x128", "zoo_160x160", "soup1000_160x160", "main_200x200"])
def test_octree_intersect_candidate_lists_match_reference(name):
    """Octree::intersect(const Ray&) (octree.h:46-68) through the C-ABI's host octree
    (gi_octree_intersect, no device): for every golden pixel, the candidate list has the length the
    compiled reference's list had (ncand) and contains the entity the reference chose (hit)."""
    import json
    z = np.load(os.path.join(U.GOLDEN, name + ".npz"))
    meta = json.loads(str(z["meta"]))
    sc = S.named_scene(meta["scene"])
    tree = gi.Octree.from_scene(sc)
    idx = np.arange(len(z["x"]))[::7]
    pos, dirs = _primary_dirs(sc, meta["w"], z["x"][idx], z["y"][idx])
    for i, d in zip(idx, dirs):
        cand = tree.intersect(pos, d)
        assert len(cand) == int(z["ncand"][i]), (int(z["x"][i]), int(z["y"][i]))
        if z["hit"][i] >= 0:
            assert tree.entities[int(z["hit"][i])] in cand


def test_error_paths_without_device():
    """gi_multi_create with no GPU fails with GI_ERR_DEVICE (no CPU fallback); argument errors are
    GI_ERR_ARG; gi_device_count is 0."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    L = gi.lib()
    assert L.gi_device_count() == 0
    assert L.gi_device_list(None, 0) == 0
    with pytest.raises(gi.GIError, match=r"\(-2\)"):
        gi.MultiScene.from_scene(S.sphere_scene(), [0, 0])
    h = ctypes.c_void_p()
    assert L.gi_multi_create(None, 1, None, ctypes.byref(h)) == -1
    assert L.gi_octree_create(None, ctypes.byref(h)) == -1


@pytest.mark.parametrize("scene,w,h", [("main", 200, 200), ("zoo", 160, 160)])
def test_cpp_dropin_octree_intersect_matches_reference(tmp_path, scene, w, h):
    """include/gi_dropin/octree.h's Octree::intersect(const Ray&) (octree.h:46-68), called from the
    reference app's own classes (integration/dropin_demo.cpp, built where the reference tree
    exists): candidate-list lengths equal the compiled reference's on every pixel's primary ray."""
    exe = U.dropin_demo()
    out = tmp_path / "c.bin"
    subprocess.run([exe, str(w), str(h), str(out), scene, "cands"], check=True, timeout=120)
    c = np.fromfile(out, np.int32)
    z = np.load(os.path.join(U.GOLDEN, f"{scene}_{w}x{h}.npz"))
    assert c.size == w * h
    assert (c[z["y"] * w + z["x"]] == z["ncand"]).all()


def test_allocation_failure_returns_nomem_not_abort(tmp_path):
    """No exception crosses the C-ABI (gi.h): a scene too large for the host memory the process may
    use makes gi_octree_create return GI_ERR_NOMEM (-5) instead of terminating the caller.  A child
    process under RLIMIT_AS = 8 GiB asks for 2^31 - 1 entities (the builder's first vector alone
    needs far more)."""
    import sys
    code = (
        "import ctypes, resource, sys\n"
        "resource.setrlimit(resource.RLIMIT_AS, (8 << 30, 8 << 30))\n"
        "sys.path.insert(0, %r)\n"
        "from importlib import import_module\n"
        "gi = import_module('2019global_amd')\n"
        "L = ctypes.CDLL(gi.LIB_PATH)\n"
        "L.gi_last_error.restype = ctypes.c_char_p\n"
        "d = gi.SceneDesc()\n"
        "one = (gi.EntityDesc * 1)()\n"
        "d.n_entities = 2**31 - 1\n"
        "d.entities = ctypes.cast(one, ctypes.POINTER(gi.EntityDesc))\n"
        "h = ctypes.c_void_p()\n"
        "rc = L.gi_octree_create(ctypes.byref(d), ctypes.byref(h))\n"
        "print('rc', rc, L.gi_last_error().decode())\n"
    ) % U.ROOT
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "rc -5 host memory exhausted" in r.stdout, r.stdout


def test_cpp_dropin_refuses_other_abi_loudly(tmp_path):
    """a drop-in build whose gi.h has another GI_ABI_VERSION than the loaded libgi
    refuses to render AND says so -- RayTracer::lastStatus() == GI_ERR_ABI, dropin_demo exits 3 --
    instead of leaving a black Image behind a zero exit.  (Built here, where the reference tree
    exists; the check runs before any device call, so no GPU is needed.)"""
    if not os.path.isdir("/root/reference/include"):
        pytest.skip("needs the reference tree to build the demo")
    hdr = open(HDR).read()
    m = re.search(r"#define GI_ABI_VERSION (\d+)", hdr)
    other = tmp_path / "inc"
    other.mkdir()
    (other / "gi.h").write_text(hdr.replace(m.group(0), "#define GI_ABI_VERSION %d" % (int(m.group(1)) - 1)))
    exe = tmp_path / "demo_other_abi"
    subprocess.run(["make", "-s", "-C", os.path.join(U.ROOT, "integration"), f"OUT={exe}", f"EXTRA_INC=-I{other}"],
                   check=True, timeout=300)
    env = dict(os.environ, QT_QPA_PLATFORM="offscreen",
               LD_LIBRARY_PATH=os.path.join(U.ROOT, "2019global_amd") + ":" + os.environ.get("LD_LIBRARY_PATH", ""))
    assert subprocess.run([str(exe), "--abi"], capture_output=True, text=True, check=True, env=env).stdout.strip() == \
        str(int(m.group(1)) - 1)
    r = subprocess.run([str(exe), "32", "32", str(tmp_path / "f.rgb")], capture_output=True, text=True, env=env,
                       timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr)
    assert "ABI" in r.stderr and "status -100" in r.stderr, r.stderr
    assert not (tmp_path / "f.rgb").exists()
