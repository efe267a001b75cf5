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
    assert ctypes.sizeof(gi.Opts) == 48
    assert ctypes.sizeof(gi.CameraDesc) == 80


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
