"""Builds 2019global_amd/libgi.so in-tree (gfx950 only).

Host translation units (scene builder, C-ABI) are compiled by g++ and the kernels by hipcc, both
with ``-ffp-contract=off``: the Mode R parity contract is bit-level and the reference (x86-64,
no FMA) never contracts a*b+c.  Run ``python -m 2019global_amd.build`` or ``__graft_entry__.build()``.
"""
from __future__ import annotations

import glob
import hashlib
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
INCLUDE = os.path.join(ROOT, "include")
OUT = os.path.join(HERE, "libgi.so")
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
ARCH = "gfx950"

HOST_SRCS = ["gi_build.cpp", "gi_bvh.cpp", "gi_capi.cpp", "gi_multi.cpp", "gi_obj.cpp"]
DEV_SRCS = ["gi_kernels.hip", "gi_wf.hip"]
HEADERS = ["gi_math.h", "gi_scene.h", "gi_internal.h", "gi_dev.h"]

COMMON = ["-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math", f"-I{INCLUDE}", f"-I{CSRC}"]


def source_hash() -> str:
    """Provenance id of a build: sha256 (first 16 hex digits) over every source and header the
    library is compiled from.  Compiled into libgi as gi_build_id(); tests compare the loaded
    library's id with this hash of the tree, so a stale .so cannot pass unnoticed."""
    h = hashlib.sha256()
    for name in sorted(HOST_SRCS + DEV_SRCS + HEADERS):
        h.update(name.encode() + b"\0" + open(os.path.join(CSRC, name), "rb").read() + b"\0")
    h.update(b"gi.h\0" + open(os.path.join(INCLUDE, "gi.h"), "rb").read())
    return h.hexdigest()[:16]


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _stale(out, deps):
    if not os.path.exists(out):
        return True
    t = os.path.getmtime(out)
    return any(os.path.getmtime(d) > t for d in deps)


def build(verbose: bool = False, force: bool = False, variant: str = "", hip_defines=()) -> str:
    """Builds libgi.so; a named variant (tuning experiments: extra -D flags for the kernels) goes to
    2019global_amd/_variants/libgi_<variant>.so and is selected at run time with GI_LIB=<path>."""
    hipcc = shutil.which("hipcc") or os.path.join(ROCM, "bin", "hipcc")
    objdir = os.path.join(HERE, "_obj")
    out = OUT
    if variant:
        out = os.path.join(HERE, "_variants", f"libgi_{variant}.so")
        os.makedirs(os.path.dirname(out), exist_ok=True)
    os.makedirs(objdir, exist_ok=True)
    hdrs = [os.path.join(CSRC, h) for h in HEADERS] + [os.path.join(INCLUDE, "gi.h")]
    # the build id goes into gi_capi.o: recompiled whenever any source changed since its last build
    bid = source_hash()
    bid_file = os.path.join(objdir, "build_id")
    old_bid = open(bid_file).read().strip() if os.path.exists(bid_file) else ""
    objs = []
    for s in HOST_SRCS:
        src, obj = os.path.join(CSRC, s), os.path.join(objdir, s + ".o")
        defs = [f'-DGI_BUILD_ID="{bid}"'] if s == "gi_capi.cpp" else []
        if force or _stale(obj, [src] + hdrs) or (defs and old_bid != bid):
            _run(["g++", "-O2", *COMMON, *defs, "-D__HIP_PLATFORM_AMD__", f"-I{ROCM}/include", "-c", src, "-o", obj],
                 verbose)
        objs.append(obj)
    with open(bid_file, "w") as f:
        f.write(bid + "\n")
    jobs = []   # the kernel translation units compile in parallel
    for s in DEV_SRCS:
        src = os.path.join(CSRC, s)
        obj = os.path.join(objdir, s + (f".{variant}" if variant else "") + ".o")
        if force or _stale(obj, [src] + hdrs):
            # (A/B variants only: GI_VARIANT_FLAGS adds code-generation flags, e.g. -mllvm scheduler options)
            extra = os.environ.get("GI_VARIANT_FLAGS", "").split() if variant else []
            cmd = [hipcc, f"--offload-arch={ARCH}", "-O3", "-Wshadow", *COMMON, *[f"-D{d}" for d in hip_defines],
                   *extra, "-munsafe-fp-atomics", "-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            jobs.append((cmd, subprocess.Popen(cmd)))
        objs.append(obj)
    # wait for every job before reporting (a failed one must not leave the others writing objects that
    # a later build would take as up to date); a failed job's object is removed
    failed = [(cmd, p.returncode) for cmd, p in [(c, p) for c, p in jobs if p.wait() != 0]]
    for cmd, _ in failed:
        if os.path.exists(cmd[-1]):
            os.remove(cmd[-1])
    if failed:
        for cmd, rc in failed:
            print(f"build failed ({rc}): {' '.join(cmd)}", file=sys.stderr)
        raise subprocess.CalledProcessError(failed[0][1], failed[0][0])
    if force or _stale(out, objs):
        _run([hipcc, f"--offload-arch={ARCH}", "-shared", "-o", out, *objs, f"-L{ROCM}/lib", "-lamdhip64", "-ldl"], verbose)
    # hipcc's unbundling temporaries (libgi.so.<n>.hipv4-..., .host-...): removed on every build
    for leftover in glob.glob(out + ".[0-9]*.hipv4-*") + glob.glob(out + ".[0-9]*.host-*"):
        os.remove(leftover)
    return out


if __name__ == "__main__":
    # python build.py [--force] [--variant NAME DEFINE ...]
    args = sys.argv[1:]
    var, defs = "", []
    if "--variant" in args:
        i = args.index("--variant")
        var, defs = args[i + 1], [a for a in args[i + 2:] if not a.startswith("--")]
    build(verbose=True, force="--force" in args, variant=var, hip_defines=defs)
