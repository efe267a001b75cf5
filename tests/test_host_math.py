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
