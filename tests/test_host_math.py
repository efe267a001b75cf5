"""CPU: the shared host/device math header (2019global_amd/csrc/gi_math.h) compiled by g++.
The triangle prefilter used by the gfx950 kernels must never change a reference triangle test."""
import os
import subprocess

import oracle_util as U


def test_prefilter_never_changes_triangle_result(tmp_path):
    exe = str(tmp_path / "pf")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I" + os.path.join(U.ROOT, "2019global_amd", "csrc"),
                    "-o", exe, os.path.join(U.ROOT, "tests", "cpp", "prefilter_stress.cpp")], check=True)
    out = subprocess.run([exe, "2000000"], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "mismatches 0" in out.stdout


def test_mode_x_acceleration_structure(tmp_path):
    """The Mode X 8-wide BVH (gi_bvh.cpp) and the SAT octree (gi_build.cpp), built by libgi's own host
    code: structural invariants, and the kernel's stackless traversal (restated in the checker)
    returns exactly the brute-force closest / any hit on random soups and the Cornell box."""
    exe = str(tmp_path / "xac")
    csrc = os.path.join(U.ROOT, "2019global_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-I" + csrc,
                    "-I" + os.path.join(U.ROOT, "include"), "-o", exe,
                    os.path.join(U.ROOT, "tests", "cpp", "xaccel_check.cpp"), os.path.join(csrc, "gi_build.cpp"),
                    os.path.join(csrc, "gi_bvh.cpp")], check=True)
    scn = tmp_path / "cornell.scn"
    scn.write_text(U.scenes().cornell_scene().to_scn())
    for env in ({}, {"GI_XLEAF_MAX": "1"}, {"GI_XACCEL": "octree"}):
        for args in (["4000"], ["4000", str(scn)]):
            out = subprocess.run([exe, *args], capture_output=True, text=True, env=dict(os.environ, **env))
            assert out.returncode == 0, (env, out.stdout)
            assert "mismatches 0" in out.stdout


def test_mode_r_candidate_reconstruction_equals_reverse_dfs(tmp_path):
    """Mode R's candidate reconstruction (line BVH + appearance ranks + leaf-path reachability, the
    kernel's default) and the reference-order reverse DFS, both restated on the host over libgi's
    scene builder: same hit entity and bit-identical point/normal on every ray -- random mixed scenes
    (spheres, triangles, ExpQuad/ExpRectangle/ExpBox) and the main, Cornell, zoo, 1k- and 100k-soup
    scenes."""
    exe = str(tmp_path / "rcc")
    csrc = os.path.join(U.ROOT, "2019global_amd", "csrc")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-I" + csrc,
                    "-I" + os.path.join(U.ROOT, "include"), "-o", exe,
                    os.path.join(U.ROOT, "tests", "cpp", "rcand_check.cpp"), os.path.join(csrc, "gi_build.cpp"),
                    os.path.join(csrc, "gi_bvh.cpp")], check=True)
    scns = []
    for name in ("main", "cornell", "zoo", "soup1000", "soup100000"):
        p = tmp_path / f"{name}.scn"
        p.write_text(U.scenes().named_scene(name).to_scn())
        scns.append(str(p))
    out = subprocess.run([exe, "3000", *scns], capture_output=True, text=True)
    assert out.returncode == 0, out.stdout
    assert "mismatches 0" in out.stdout
