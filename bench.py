#!/usr/bin/env python3
"""bench.py — Mray/s and ms/frame of the gfx950 radiance path on the BASELINE.json metric config.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload C3|C2|C4|C5|R-C4|R-main]

N > 1 is launched by the driver as `torch.distributed.run --nproc-per-node N bench.py --gpus N ...`:
one rank per GPU (RCCL over xGMI).  The frame's 8x8 pixel tiles are dealt round-robin to the
ranks (tile t -> rank t % N), each rank renders its tiles into a packed buffer in HBM, and one
ncclGather (torch.distributed.gather on the nccl backend) brings them to rank 0, which
reassembles the frame with gi_unshard_device.  A step = one whole frame: render + gather +
unshard of the RGB888 image (the reference's output, image.h:14-16; every rank also writes its
fp64 radiance, gathered once after the timed region for `frame_check`); the frame is fixed as N
grows ("scaling": "strong").

Default workload C3 (BASELINE.json configs[2]): Cornell box (34 ImpTriangles), 1920x1080,
depth 8, 64 spp, Mode X (the build-defined integrator: the reference itself renders depth 1 only).
`value` = rays traced (primary + bounce + shadow rays that reached the BVH, all ranks) per second,
inputs resident in HBM; `mray_s_all_rays` also counts the primary samples resolved
exactly without traversal.  The ray count per frame is exact: a counting launch (GI_FLAG_STATS) of the same
deterministic frame runs before the timed region.

roofline: the resource the dominant kernel (k_seg / k_mode_x; Mode R: the flat phases) uses.  Mode X:
the VALU pipe -- achieved = useful VALU lane-op slots per launch (PMC counters of the same workload,
profiles/rNN_<workload>_pmc.json: pipe-weighted VALU instructions x 64 lanes x lane utilisation) /
the kernel's average launch time from HIP events recorded directly around it on the launch stream
(GI_FLAG_TIME, read with gi_scene_kernel_ms), against 1,024 SIMDs x 32 lanes x 2.4 GHz; `binding`
names what holds it below (latency / valu / hbm).  Mode R: the FP64 vector peak.  The
algorithmic record bytes (Mode X: wide-node records x 256 B -- 128 B for the quantised nodes of
large HBM-resident scenes -- + primitive records x 80 B + 27 B/pixel output; Mode R: 64 B nodes +
144 B triangles) per launch / that time stay beside it as hbm_alg_frac, and traffic = the HBM bytes
the counters saw (hbm_counter_frac): the records live in LDS / L2, so the two differ 10-100x.
cpu_baseline: this repo's CPU port of the same integrator (oracle, test infrastructure), OpenMP over
the job's CPU share and on 1 thread, on full-width rows spread over the same frame (Mode X: those
rows also checked against the timed GPU frame, bit for bit); reference_cpu: the compiled reference itself (depth 1, the
only depth it has) on a strided sample of the same frame, when oracle/_ref is present.
"""
from __future__ import annotations

import argparse
import ctypes
import glob
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
NODE_BYTES = {0: 64, 1: 256}   # RNode / XWNode (8 child boxes) records; Mode X on large HBM-resident
                               # scenes: the quantised 128-B XCNode (gi_scene_info.x_node_bytes)
PRIM_BYTES = {0: 144, 1: 80}   # Mode R: TriRec (sphere/quad records are <= 160 B) / Mode X: XHot fp64 record

WORKLOADS = {
    # name: (scene, w, h, mode, spp, depth, description)
    "C3": ("cornell", 1920, 1080, 1, 64, 8, "Cornell box (34 tris), 1920x1080, depth=8, 64 spp (configs[2])"),
    "C2": ("cornell", 512, 512, 1, 1, 4, "Cornell box (34 tris), 512x512, depth=4 (configs[1])"),
    "C4": ("soup100000", 1920, 1080, 1, 1, 8, "100k-triangle random mesh + octree, 1920x1080, depth=8 (configs[3])"),
    "C5": ("soup100000", 3840, 2160, 1, 256, 8, "100k-triangle mesh, 3840x2160, depth=8, 256 spp (configs[4])"),
    "R-C4": ("soup100000", 1920, 1080, 0, 1, 1, "reference semantics (Mode R), 100k-triangle mesh, 1920x1080"),
    "R-C3": ("cornell", 1920, 1080, 0, 1, 1, "reference semantics (Mode R), Cornell box, 1920x1080"),
    "R-main": ("main", 500, 500, 0, 1, 1, "reference semantics (Mode R), main.cpp scene, 500x500"),
    # extra Mode X scenes (tuning / coverage; not BASELINE configs)
    "X-main": ("main", 1920, 1080, 1, 16, 8, "Mode X, main.cpp scene, 1920x1080, depth=8, 16 spp"),
    "X-zoo": ("zoo", 1920, 1080, 1, 16, 8, "Mode X, every entity type, 1920x1080, depth=8, 16 spp"),
    "X-soup1000": ("soup1000", 1920, 1080, 1, 16, 8, "Mode X, 1k-triangle soup, 1920x1080, depth=8, 16 spp"),
}


def make_scene(name):
    from importlib import import_module
    return import_module("2019global_amd.scenes").named_scene(name)


FP64_VALU_PEAK_TFS = 78.6     # MI355X FP64 vector peak (AMD spec; half the guide's 157.3 TF FP32 vector rate)
# VALU lane-op slots per second: 256 CUs x 4 SIMDs x 32 lanes per cycle (a wave64 instruction holds the
# SIMD's pipe 2 cycles, an f64 one 4) x 2.4 GHz -- the Mode X roofline (f64 instructions count twice)
VALU_LANE_PEAK_TOPS = 256 * 4 * 32 * 2.4e9 / 1e12
N_SIMDS = 1024                 # 256 CUs x 4 SIMDs


def pmc_summary(workload: str, kernel: str = ""):
    """The latest committed rocprofv3 PMC summary of this workload's dominant kernel
    (profiles/rNN[tag]_<workload>_pmc.json, written by profiles/summarize.py) whose kernel is the one
    this run launches (k_seg / k_mode_x / k_wf_bounce / k_mode_r...: A/B profiles of the other forms
    sit beside it), or None.  Latest = highest round number."""
    best = None
    for p in glob.glob(os.path.join(ROOT, "profiles", "r*_pmc.json")):
        try:
            d = json.load(open(p))
        except Exception:
            continue
        if d.get("workload") != workload or not d.get("counters_per_launch"):
            continue
        if kernel and kernel + "<" not in d.get("kernel", ""):   # (the flat Mode R summary names all its kernels)
            continue
        base = os.path.basename(p)
        # latest round first; within a round the plain rNN_ summary (the round's final evidence)
        # before tagged ones (rNNa_, rNNmega_, ...: mid-round or forced-form A/B profiles)
        rnd = (base[1:3], base[3:base.index("_")] == "")
        if best is None or rnd > best[0]:
            best = (rnd, os.path.relpath(p, ROOT), d)
    return best[1:] if best else None


def counter_ceilings(workload: str, kern_ms: float, kernel: str = ""):
    """What the dominant kernel meets, from the committed PMC summary of the same workload:
      * HBM: counter bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, gfx950 correction) / live kernel
        time / 8 TB/s -- the bytes that actually reach HBM;
      * VALU: issue share = SQ_INSTS_VALU x 4 cycles / (1,024 SIMDs x kernel cycles, GRBM_GUI_ACTIVE / 8)
        and lane utilisation = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU); their product is
        the fraction of the chip's VALU lane-slots doing work;
      * FP64 (Mode R): f64 VALU instructions / all VALU instructions, and the f64 FLOP
        rate (SQ_INSTS_VALU_FLOPS_FP64, a per-wave-instruction count, x 64 lanes x lane utilisation)
        against the 78.6 TF/s FP64 vector peak -- Mode R's roofline.
    `binding` names the tightest: valu when the VALU pipe is busy >= 75% of the cycles (2 cycles
    per wave64 instruction, 4 for f64), else hbm when counter traffic is >= 60% of peak, else latency
    (the waves wait on dependent instructions and memory)."""
    got = pmc_summary(workload, kernel)
    if got is None:
        return None
    src, d = got
    c = d["counters_per_launch"]
    out = {"pmc_source": src, "pmc_kernel_ms": round(d.get("avg_launch_ns", 0) / 1e6, 4)}
    hbm = d.get("hbm_bytes_per_launch")
    if hbm:
        out["hbm_counter_bytes"] = int(hbm)
        out["hbm_counter_frac"] = round(hbm / (kern_ms * 1e-3) / (HBM_PEAK_GBS * 1e9), 5)
    if c.get("GRBM_GUI_ACTIVE") and c.get("SQ_INSTS_VALU"):
        cycles = c["GRBM_GUI_ACTIVE"] / 8.0
        out["valu_issue_frac"] = round(c["SQ_INSTS_VALU"] * 4.0 / (N_SIMDS * cycles), 4)
        f64n = [c.get(k) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                                   "SQ_INSTS_VALU_TRANS_F64")]
        if all(v is not None for v in f64n):
            # the SIMD-32 pipe's busy share: a wave64 instruction occupies it 2 cycles (4 for f64, half
            # rate), so several waves can keep it full (MI355X_MICROARCH.md: one wave alone issues
            # every 4 cycles); valu_issue_frac above prices every instruction at 4 cycles
            n64 = sum(f64n)
            out["valu_pipe_frac"] = round(((c["SQ_INSTS_VALU"] - n64) * 2.0 + n64 * 4.0) / (N_SIMDS * cycles), 4)
            # VALU lane-op slots per launch at pipe weight (an f64 instruction holds the pipe twice as long,
            # so it counts twice): the useful ones are these x the lane utilisation (Mode X roofline)
            out["valu_lane_slots"] = int(((c["SQ_INSTS_VALU"] - n64) + 2.0 * n64) * 64.0)
    if c.get("SQ_ACTIVE_INST_VALU") and c.get("SQ_THREAD_CYCLES_VALU"):
        out["valu_lane_util"] = round(c["SQ_THREAD_CYCLES_VALU"] / (64.0 * c["SQ_ACTIVE_INST_VALU"]), 4)
    if "valu_issue_frac" in out and "valu_lane_util" in out:
        out["valu_frac"] = round(out["valu_issue_frac"] * out["valu_lane_util"], 4)
    if c.get("SQ_WAVE_CYCLES") and c.get("SQ_WAIT_ANY"):
        out["wait_share"] = round(c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"], 4)
    f64 = [c.get(k) for k in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64",
                              "SQ_INSTS_VALU_TRANS_F64")]
    if all(v is not None for v in f64) and c.get("SQ_INSTS_VALU"):
        out["f64_inst_share"] = round(sum(f64) / c["SQ_INSTS_VALU"], 4)
    # FP64 FLOP rate (Mode R's designated bound).  SQ_INSTS_VALU_FLOPS_FP64 counts per
    # wave instruction (it equals add + 2 fma + mul + trans of the f64 instruction counters exactly,
    # VERDICT r02), so the FLOPs are that count x 64 lanes x the fraction of lanes active -- the
    # kernel-wide VALU lane utilisation, applied to its f64 instructions
    if c.get("SQ_INSTS_VALU_FLOPS_FP64") is not None and "valu_lane_util" in out:
        flops = c["SQ_INSTS_VALU_FLOPS_FP64"] * 64.0 * out["valu_lane_util"]
        out["f64_flops_per_launch"] = int(flops)
        out["f64_tflops"] = round(flops / (kern_ms * 1e-3) / 1e12, 4)
        out["f64_valu_frac"] = round(out["f64_tflops"] / FP64_VALU_PEAK_TFS, 5)
    pipe = out.get("valu_pipe_frac", out.get("valu_issue_frac", 0))
    if pipe >= 0.75:
        out["binding"] = "valu"
    elif out.get("hbm_counter_frac", 0) >= 0.6:
        out["binding"] = "hbm"
    else:   # neither pipe is full: the waves wait on dependent instructions and memory
        out["binding"] = "latency"
    return out


def cpu_info():
    model = "?"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return model, os.cpu_count() or 1


def cpu_threads():
    """Threads for the CPU port: every CPU this job may use -- OMP_NUM_THREADS when set (the GPU box
    sets it to the job's CPU share, 16: the pool's rules size worker pools to that share, while
    os.cpu_count() there reports the whole machine), else the CPUs of the process's affinity mask."""
    v = os.environ.get("OMP_NUM_THREADS")
    if v and v.isdigit():
        return max(1, int(v))
    try:
        return max(1, len(os.sched_getaffinity(0)))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cpu_baseline(scn_text, w, h, mode, spp, depth, seed, target_s=16.0, target_1t_s=10.0, gpu_frame=None):
    """The oracle (this repo's CPU port, OpenMP) on a frame-representative sample of the same workload:
    full-width rows spread evenly over the frame (y = row0 + k * stride).  A probe of 8 rows sets the
    rate, then about `target_s` seconds of rows are timed on every CPU this job may use (`value`,
    `cores`), and about `target_1t_s` seconds on ONE thread (`value_1t`; the reference's own loop is
    single-threaded, raytracer.h:32-33).  Mode X `value` basis: rays that reach the
    scene -- primary samples whose ray misses the scene's bounding box add exactly +0 and are counted
    apart (the GPU's classify pass and root-box pretest resolve the same kind of sample apart from its
    `value`), so `value` here is traced rays per second like the GPU line's; `value_all_rays` counts
    them too.  gpu_frame (Mode X; (rgb (h, w, 3) fp64, rgb8 (h, w, 3)) of the timed GPU frame, N = 1):
    the sampled rows the oracle rendered are compared with it bit for bit (`gpu_rows_check`), so the
    bench checks its own frame.  Mode R: one ray per pixel over a centred window (the reference's
    only depth)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_util as U
    import numpy as np
    threads = cpu_threads()
    model, host_cores = cpu_info()
    if mode == 0:
        cx, cy, ww, wh = w // 2, h // 2, min(w, 512), min(h, 256)
        win = (max(0, cx - ww // 2), max(0, cy - wh // 2), min(w, cx - ww // 2 + ww), min(h, cy - wh // 2 + wh))
        t = time.perf_counter()
        U.oracle_render(scn_text, w, h, mode=0, window=win, threads=threads)
        dt = time.perf_counter() - t
        rays = (win[2] - win[0]) * (win[3] - win[1])
        # one thread on the window's middle rows (about a quarter of it)
        q = (win[3] - win[1]) // 4
        win1 = (win[0], win[1] + q, win[2], win[3] - q)
        t = time.perf_counter()
        U.oracle_render(scn_text, w, h, mode=0, window=win1, threads=1)
        dt1 = time.perf_counter() - t
        rays1 = (win1[2] - win1[0]) * (win1[3] - win1[1])
        return {"value": round(rays / dt / 1e6, 4), "unit": "Mray/s", "cores": threads, "kind": "port",
                "value_1t": round(rays1 / dt1 / 1e6, 4), "cores_1t": 1,
                "value_all": round(rays / dt / 1e6, 4), "cores_all": threads,
                "cpu_model": model, "host_cores": host_cores,
                "sample": f"Mode R window x[{win[0]},{win[2]}) y[{win[1]},{win[3]}), {rays} rays, {dt:.2f} s wall, "
                          f"OpenMP over {threads} threads; value_1t: rows y[{win1[1]},{win1[3]}) of it, {rays1} rays, "
                          f"{dt1:.2f} s on 1 thread"}

    def run(row0, stride, n_rows, nt, pixels=False):
        t = time.perf_counter()
        r = U.oracle_time_rows(scn_text, w, h, spp, depth, seed, row0, stride, n_rows, nt, pixels=pixels)
        return r, time.perf_counter() - t

    def sized(nt, target, pixels=False):
        n, stride = min(8, h), max(1, h // min(8, h))
        r, dt = run(stride // 2, stride, n, nt)
        for _ in range(3):   # rescale until the sample takes about target (whole frame at most)
            if dt >= 0.5 * target or n >= h:
                break
            n = int(max(1, min(h, n * target / max(dt, 1e-3))))
            stride = max(1, h // n)
            n = min(n, (h + stride - 1) // stride)
            r, dt = run(stride // 2, stride, n, nt, pixels)
        if pixels and "rgb" not in r:
            r, dt = run(stride // 2, stride, n, nt, pixels)
        return r, dt, stride

    r, dt, stride = sized(threads, target_s, pixels=gpu_frame is not None)
    traced = r["rays"] - r["resolved"]
    r1, dt1, stride1 = sized(1, target_1t_s)
    traced1 = r1["rays"] - r1["resolved"]
    v_all, v_1t = traced / dt / 1e6, traced1 / dt1 / 1e6
    extra = {}
    if gpu_frame is not None:
        g, g8 = gpu_frame
        same = U.bits_equal(g[r["rows"]], r["rgb"]).all(2) & (g8[r["rows"]] == r["q"]).all(2)
        extra["gpu_rows_check"] = (f"{len(r['rows'])} sampled rows ({r['pixels']} pixels) of the timed GPU frame "
                                   + ("bit-identical to the oracle" if same.all() else
                                      f"MISMATCH: {int((~same).sum())} pixels differ from the oracle"))
    return {"value": round(v_all, 4), "unit": "Mray/s", "cores": threads, "kind": "port",
            "value_all_rays": round(r["rays"] / dt / 1e6, 4),
            # VERDICT r05 item 6 / BASELINE.md: the port at 1 thread and at every CPU this job may use
            "value_1t": round(v_1t, 4), "cores_1t": 1,
            "value_all": round(v_all, 4), "cores_all": threads,
            "parallel_efficiency": round(v_all / (threads * v_1t), 3) if v_1t > 0 else None,
            # an UPPER bound for the whole host: perfect scaling of the 1-thread rate over every logical
            # CPU (no run may use them: the pool sizes a job's worker pools to its CPU share)
            "value_host_upper_bound": round(v_1t * host_cores, 2), "host_cores_note":
                f"the host has {host_cores} logical CPUs; this job's share is {threads} (OMP_NUM_THREADS / "
                f"affinity), the most any run here may use, so value_all is measured at {threads} and "
                f"value_host_upper_bound = value_1t x {host_cores} bounds an all-core run from above",
            "sample_1t": f"{r1['pixels'] // w} full-width rows y = {stride1 // 2} + k*{stride1}, {traced1} traced rays, "
                         f"{dt1:.2f} s wall, 1 thread",
            **extra,
            "cpu_model": model, "host_cores": host_cores,
            "value_basis": "rays that reach the scene (primary samples missing the scene's bounding box counted "
                           "apart, as the GPU's value does); value_all_rays includes them.  The two sides resolve "
                           "background samples by different conservative tests -- the oracle by its exact fp64 "
                           "test of the scene box, the GPU by a pixel-frustum test and an fp32 root-box pretest "
                           "(k_x_classify, wf_primary_misses) -- so the traced counts of a whole frame differ by a "
                           "few ppm (C3: 104,395,196 CPU against 104,395,779 GPU, 6 ppm); every such sample adds "
                           "exactly +0 on both sides, so the frames are identical",
            "sample": f"{r['pixels'] // w} full-width rows y = {stride // 2} + k*{stride} spread over the frame "
                      f"({r['pixels']} pixels x {spp} spp), {traced} traced rays + {r['resolved']} resolved samples, "
                      f"{dt:.2f} s wall, OpenMP over {threads} threads (OMP_NUM_THREADS; the host has {host_cores} "
                      f"logical CPUs); closest-hit queries by the oracle's own BVH above 256 primitives, brute force "
                      f"below"}


def reference_cpu(scn_text, w, h):
    """The compiled reference (oracle/_ref/ref_harness `time`: RayTracer::run's per-pixel body,
    depth 1, 1 thread) on a strided sample of the same frame."""
    exe = os.path.join(ROOT, "oracle", "_ref", "ref_harness")
    if not os.path.exists(exe):
        return None
    import tempfile
    with tempfile.TemporaryDirectory() as td:
        sp = os.path.join(td, "s.scn")
        open(sp, "w").write(scn_text)
        stride = max(1, (w * h) // 20000)
        try:
            out = subprocess.run([exe, "time", sp, str(w), str(h), str(stride)], capture_output=True, text=True,
                                 timeout=120, check=True).stdout
        except Exception as e:   # never fail the bench on the optional reference leg
            return {"error": str(e)[:200]}
    r = json.loads(out)
    model, host_cores = cpu_info()
    return {"value": round(r["mray_s"], 6), "unit": "Mray/s", "cores": 1, "kind": "reference",
            "cpu_model": model, "host_cores": host_cores,
            "sample": f"depth 1 (the reference's only depth), every {stride}th pixel, {r['rays']} rays"}


def host_path(gi, sc, dev, cam, light, w, h, mode, spp, depth, seed, reps=3):
    """gi_render with host buffers (the drop-in RayTracer's path): render + PCIe copy-back, ms per
    frame, and the same frame through gi_multi_render (the drop-in's GI_DEVICES route) on this one
    device: two tile shards on it, and one shard whose tiles travel through RCCL to itself
    (GI_MULTI_RCCL=1).  Reported beside `value`, never as it (inputs are not HBM-resident here)."""
    import numpy as np
    rgb = np.empty((h, w, 3), np.float64)
    rgb8 = np.empty((h, w, 3), np.uint8)
    res = {}

    def timed(name, fn, out, band):
        fn(cam, light, w, h, mode=mode, spp=spp, depth=depth, seed=seed, band_rows=band, out=out)   # warm
        t = time.perf_counter()
        for _ in range(reps):
            fn(cam, light, w, h, mode=mode, spp=spp, depth=depth, seed=seed, band_rows=band, out=out)
        res[name] = round((time.perf_counter() - t) / reps * 1e3, 3)

    for name, out, band in (("rgb8", (None, rgb8), 0), ("rgb8+fp64", (rgb, rgb8), 0),
                            ("rgb8_bands32", (None, rgb8), 32), ("rgb8+fp64_bands32", (rgb, rgb8), 32)):
        timed(name, dev.render, out, band)
    multi = {}
    try:
        m2 = gi.MultiScene.from_scene(sc, [0, 0])
        timed("multi_2shards_1dev_rgb8+fp64_bands32", m2.render, (rgb, rgb8), 32)
        m2.close()
        os.environ["GI_MULTI_RCCL"] = "1"   # read by gi_multi_create
        try:
            m1 = gi.MultiScene.from_scene(sc, [0])
        finally:
            del os.environ["GI_MULTI_RCCL"]
        if m1.info()["rccl"]:
            timed("multi_rccl_self_rgb8+fp64_bands32", m1.render, (rgb, rgb8), 32)
            timed("multi_rccl_self_rgb8+fp64", m1.render, (rgb, rgb8), 0)
        m1.close()
    except Exception as e:   # never fail the bench on this side measurement
        multi["error"] = str(e)[:200]
    return {"ms_per_frame": res, **multi,
            "note": "host buffers: PCIe copy-back included (rgb8 = the reference Image's RGB888; +fp64 "
                    "radiance; bands32 = 32-row progressive bands as the drop-in RayTracer::run uses; multi_* "
                    "= gi_multi_render, the drop-in's GI_DEVICES route, on this one device); not `value`"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", default="C3", choices=sorted(WORKLOADS))
    ap.add_argument("--seed", type=int, default=2019)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-host-path", action="store_true",
                    help="skip the host-buffer gi_render timings (profiling runs: only the timed frames launch)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (= RCCL over xGMI) for real runs; gloo rehearses N ranks sharing one GPU")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from importlib import import_module
    gi = import_module("2019global_amd")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    ndev = max(1, torch.cuda.device_count())
    dev_index = local % ndev   # one GPU per rank; ranks share a device only in a gloo rehearsal
    torch.cuda.set_device(dev_index)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group("gloo")

    scene_name, w, h, mode, spp, depth, desc = WORKLOADS[args.workload]
    sc = make_scene(scene_name)
    dev = gi.DeviceScene.from_scene(sc)
    cam = gi.Camera(sc.cam_pos, sc.cam_look, sc.focal)
    stream = torch.cuda.current_stream()
    sptr = stream.cuda_stream
    kw = dict(mode=mode, spp=spp, depth=depth, seed=args.seed, shard_count=world, shard_index=rank)

    shard = import_module("2019global_amd.shard")
    if world == 1:
        buf = torch.empty(w * h * 3, dtype=torch.float64, device="cuda")
        buf8 = torch.empty(w * h * 3, dtype=torch.uint8, device="cuda")
    else:
        fg = shard.FrameGather(torch, dist, w, h, world, rank, "cuda")
        buf, buf8 = fg.buf, fg.buf8
        if rank == 0:
            frame = torch.empty(w * h * 3, dtype=torch.float64, device="cuda")
            frame8 = torch.empty(w * h * 3, dtype=torch.uint8, device="cuda")

    # exact work counts of this rank's share of the frame (same deterministic frame, untimed)
    stats = torch.zeros(gi.STATS_N, dtype=torch.int64, device="cuda")
    dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), sptr, stats_ptr=stats.data_ptr(), **kw)
    torch.cuda.synchronize()
    if world > 1:
        if args.dist_backend == "gloo":
            cs = stats.cpu()
            dist.all_reduce(cs)
            stats.copy_(cs)
        else:
            dist.all_reduce(stats)
    st = stats.cpu().tolist()
    rays_frame = st[gi.STAT_RAYS]

    ev0 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ev1 = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]

    def step(i=None):
        if i is not None:
            ev0[i].record(stream)
        # GI_FLAG_TIME adds HIP events around the dominant kernel on the same stream (warmup steps
        # too: the event ring is created on first use, outside the timed region)
        dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), sptr,
                          **dict(kw, flags=kw.get("flags", 0) | gi.FLAG_TIME))
        if i is not None:
            ev1[i].record(stream)
        if world > 1:   # one ncclGather of the packed RGB888 tiles to rank 0, then reassembly on its GPU
            fg.gather(radiance=False)
            if rank == 0:
                gi.unshard_device(w, h, world, 0, fg.packed_all8.data_ptr(), 0, frame8.data_ptr(), sptr)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if args.warmup:
        dev.kernel_ms()   # drops the warmup launches' timings
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    # device time of the whole render call (classify + dominant kernel + reduce) and of the
    # dominant kernel alone (gi_scene_kernel_ms: the events recorded by GI_FLAG_TIME)
    render_ms = sum(a.elapsed_time(b) for a, b in zip(ev0, ev1)) / max(1, args.steps)
    kern_ms, kern_n = dev.kernel_ms()
    if kern_n != args.steps:
        raise RuntimeError(f"timed {kern_n} dominant-kernel launches, expected {args.steps}")
    if world > 1:
        t = torch.tensor([elapsed, kern_ms, render_ms], dtype=torch.float64,
                         device="cuda" if args.dist_backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, render_ms = t.tolist()

    frame_check = None
    if world > 1:   # after timing: the last frame's fp64 radiance too, for the check below
        fg.gather(radiance=True)
        if rank == 0:
            gi.unshard_device(w, h, world, fg.packed_all.data_ptr(), fg.packed_all8.data_ptr(), frame.data_ptr(),
                              frame8.data_ptr(), sptr)
    if world > 1 and rank == 0:   # the assembled frame against a whole frame rendered here alone
        ref = torch.empty(w * h * 3, dtype=torch.float64, device="cuda")
        ref8 = torch.empty(w * h * 3, dtype=torch.uint8, device="cuda")
        dev.render_device(cam, sc.light, w, h, ref.data_ptr(), ref8.data_ptr(), sptr,
                          **dict(kw, shard_count=1, shard_index=0))
        torch.cuda.synchronize()
        same = bool(torch.equal(ref.view(torch.int64), frame.view(torch.int64)) and torch.equal(ref8, frame8))
        frame_check = "bit-identical to the single-GPU frame" if same else "MISMATCH vs single-GPU frame"

    if rank == 0:
        ms_frame = elapsed / args.steps * 1e3
        resolved = st[gi.STAT_X_RESOLVED] if mode == 1 else 0
        # Mray/s = rays TRACED per second -- primary + bounce + shadow rays that
        # reached the acceleration structure; the primary samples the pixel-frustum classify and the
        # root-box pretest resolve without traversal (each adds exactly +0) are counted apart
        rays_traced = rays_frame - resolved
        form = dev.x_form(mode, spp, depth) if mode == 1 else None   # the Mode X form this launch ran
        rkern = dev.r_kernel() if mode == 0 else None                 # Mode R: its kernel (k_rf_walk: the flat phases)
        value = rays_traced * args.steps / elapsed / 1e6
        # algorithmic bytes per launch of the dominant kernel (this rank's launch; N=1: the frame)
        node_bytes = dev.info()["x_node_bytes"] if mode == 1 else NODE_BYTES[0]
        alg = (st[gi.STAT_NODES] * node_bytes + st[gi.STAT_PRIMS] * PRIM_BYTES[mode] +
               st[gi.STAT_PIXELS] * 27) / world
        achieved = alg / (kern_ms * 1e-3) / 1e9
        ceil = counter_ceilings(args.workload, kern_ms, form if mode == 1 else rkern) if world == 1 else None
        traffic = ceil.get("hbm_counter_bytes") if ceil else None
        out = {
            "metric": "Mray/s + ms/frame at 1920x1080, depth 8; %HBM roofline",
            "value": round(value, 3),
            "unit": "Mray/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_frame, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "value_basis": "rays traced per second (primary + bounce + shadow rays that reached the BVH, all "
                           "ranks; SURVEY §8(d)); mray_s_all_rays adds the primary samples resolved exactly "
                           "without traversal",
            "dtype": "f64",
            "data": "synthetic (procedural scene, no external data)",
            "config": {"workload": f"{args.workload}: {desc}", "mode": "X" if mode == 1 else "R", "width": w,
                       "height": h, "spp": spp, "depth": depth, "seed": args.seed,
                       "rays_per_frame": rays_frame, "primary_rays_per_frame": w * h * spp,
                       # rays that reached the BVH: rays_per_frame minus the primary samples resolved
                       # by the pixel-frustum classify and the root-box pretest (each adds exactly +0)
                       "rays_traced_per_frame": rays_traced,
                       "parallelism": f"tile-shard{world}"},
            # primary (w*h*spp) and total (primary + bounce + shadow) rays per second
            "mray_s_primary": round(w * h * spp * args.steps / elapsed / 1e6, 3),
            "mray_s_all_rays": round(rays_frame * args.steps / elapsed / 1e6, 3),
            "roofline": {"bound": "hbm", "kernel": (form if mode == 1 else rkern),
                         "achieved": round(achieved, 3), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": traffic, "alg_bytes_per_launch": int(alg),
                         "kernel_ms": round(kern_ms, 4), "render_call_ms": round(render_ms, 4),
                         "node_visits": st[gi.STAT_NODES], "prim_tests": st[gi.STAT_PRIMS],
                         "node_record_bytes": node_bytes,
                         "alg_bytes_note": "algorithmic record bytes (north_star's HBM roofline is met on these "
                                           "only: for LDS-resident scenes (C2/C3) they are served from LDS, for "
                                           "C4/C5 mostly from L2/MALL -- hbm_counter_frac is what reaches HBM)"},
        }
        if ceil:
            out["roofline"].update({k: v for k, v in ceil.items() if k != "hbm_counter_bytes"})
        if mode == 1 and ceil and ceil.get("valu_lane_slots") and "valu_lane_util" in ceil:
            # the headline roofline is the resource the kernel actually uses.  Mode X's
            # records live in LDS (C2/C3) or L2/MALL (C4/C5): counters show 1-9% of HBM, so HBM is not the
            # roofline.  Its instruction stream is VALU: achieved = the USEFUL VALU lane-op slots per launch
            # (PMC: pipe-weighted VALU instructions x 64 x lane utilisation, pmc_source) / live kernel time,
            # against the VALU lane peak -- frac = the pipe's busy share x its lane utilisation.  `binding`
            # says what holds it below that peak (latency: the pipe is not full, waves wait on dependent
            # fp64 chains and LDS/L2 reads).  The algorithmic-byte figure stays as hbm_alg_*.
            r = out["roofline"]
            hbm_part = {"hbm_alg_achieved_gbs": r.pop("achieved"), "hbm_peak_gbs": r.pop("peak"),
                        "hbm_alg_frac": r.pop("frac")}
            useful = ceil["valu_lane_slots"] * ceil["valu_lane_util"]
            ach = useful / (kern_ms * 1e-3) / 1e12
            r.update({"bound": "valu", "achieved": round(ach, 4), "peak": round(VALU_LANE_PEAK_TOPS, 3),
                      "unit": "Tlane-op/s", "frac": round(ach / VALU_LANE_PEAK_TOPS, 5),
                      "achieved_note": "useful VALU lane-op slots per launch (PMC: (VALU - f64 + 2 x f64 "
                                       "instructions) x 64 x valu_lane_util, pmc_source) / live kernel time; "
                                       "peak = 1,024 SIMDs x 32 lanes x 2.4 GHz; frac = valu_pipe_frac x "
                                       "valu_lane_util at the live kernel time", **hbm_part})
        if mode == 0 and ceil and "f64_tflops" in ceil:
            # Mode R is FP64-VALU bound by arithmetic intensity (the exact ExpBox node
            # test is ~20-40 fp64 ops per record byte): the roofline is the FP64 vector peak; the
            # algorithmic record bytes stay beside it as hbm_* fields
            r = out["roofline"]
            hbm_part = {"hbm_achieved_gbs": r.pop("achieved"), "hbm_peak_gbs": r.pop("peak"), "hbm_frac": r.pop("frac")}
            r.update({"bound": "fp64_valu", "achieved": ceil["f64_tflops"], "peak": FP64_VALU_PEAK_TFS,
                      "unit": "TFLOP/s", "frac": ceil["f64_valu_frac"],
                      "achieved_note": "f64 FLOPs per launch (PMC SQ_INSTS_VALU_FLOPS_FP64 x 64 lanes x VALU "
                                       "lane utilisation, pmc_source) / live kernel time", **hbm_part})
        if rkern == "k_rf_walk":   # the flat phases' candidate pairs and the tiles left to k_mode_r_batch
            out["roofline"]["kernel_note"] = "flat phases k_rf_walk/hit/scan/reach/shade + k_mode_r_batch over overflowed tiles"
            out["rf_pairs"] = st[gi.STAT_R_PAIRS]
            out["rf_overflow_tiles"] = st[gi.STAT_R_OVF_TILES]
        if frame_check is not None:
            out["frame_check"] = frame_check
            if args.dist_backend != "nccl":
                out["rehearsal"] = f"{args.dist_backend}: {world} ranks on {ndev} device(s)"
        if form == "k_seg" and st[gi.STAT_X_ITERS]:   # k_seg divergence profile (STATS launch)
            segs = max(1, st[gi.STAT_X_HANDLE])
            out["schedule"] = {
                "form": form, "wave_iterations": st[gi.STAT_X_ITERS], "wave_segments": st[gi.STAT_X_HANDLE],
                # lanes carrying a path when a segment starts / 64
                "segment_lane_fill": round(st[gi.STAT_X_HLANES] / (64.0 * segs), 4),
                # traversal loops: the wave's iterations (its slowest lane's steps) and the lanes' own steps
                "closest_trav": {"wave_iterations": st[gi.STAT_X_IT_LEAF],
                                 "lane_fill": round(st[gi.STAT_X_LN_LEAF] / (64.0 * max(1, st[gi.STAT_X_IT_LEAF])), 4)},
                "shadow_trav": {"wave_iterations": st[gi.STAT_X_IT_NODE],
                                "lane_fill": round(st[gi.STAT_X_LN_NODE] / (64.0 * max(1, st[gi.STAT_X_IT_NODE])), 4)},
                # wave clock shares: closest trace, shadow trace, shading + next direction, unit refill
                "cycle_share": {k: round(v / max(1, st[gi.STAT_X_CYC_ALL]), 4) for k, v in (
                    ("closest", st[gi.STAT_X_IT_RS]), ("shadow", st[gi.STAT_X_CYC_TRAV] - st[gi.STAT_X_IT_RS]),
                    ("shade", st[gi.STAT_X_CYC_HIT]), ("refill", st[gi.STAT_X_CYC_NEXT]))}}
        elif mode == 1 and st[gi.STAT_X_ITERS]:   # k_mode_x schedule (STATS launch; wave = 64 lanes)
            it, hd = st[gi.STAT_X_ITERS], max(1, st[gi.STAT_X_HANDLE])
            out["schedule"] = {"wave_iterations": it, "lane_trav_steps": st[gi.STAT_X_TRAV],
                               "trav_lane_fill": round(st[gi.STAT_X_TRAV] / (64.0 * it), 4),
                               "handler_runs": st[gi.STAT_X_HANDLE],
                               "handler_lane_fill": round(st[gi.STAT_X_HLANES] / (64.0 * hd), 4),
                               "handler_closest_lanes": st[gi.STAT_X_HCLOSE],
                               "handler_shadow_lanes": st[gi.STAT_X_HSHADOW],
                               "iterations_per_ray": round(it * 64.0 / max(1, rays_frame), 3),
                               # the longest sample path (primary ray to its end), device constant clock
                               "longest_path": {"ms": round((st[gi.STAT_X_PATH_MAX] >> 32) / 1e5, 4),
                                                "wave_iterations": (st[gi.STAT_X_PATH_MAX] >> 16) & 0xFFFF,
                                                "trav_steps": st[gi.STAT_X_PATH_MAX] & 0xFFFF},
                               # divergence profile: loop iterations that ran each block, and the
                               # lanes that used it (fill = lanes / (64 x iterations))
                               "blocks": {k: {"iterations": st[a], "lane_fill": round(st[b] / (64.0 * max(1, st[a])), 4)}
                                          for k, a, b in (("node_test", gi.STAT_X_IT_NODE, gi.STAT_X_LN_NODE),
                                                          ("leaf_test", gi.STAT_X_IT_LEAF, gi.STAT_X_LN_LEAF),
                                                          ("bounce_restart", gi.STAT_X_IT_RS, gi.STAT_X_LN_RS),
                                                          ("ray_start_pass", gi.STAT_X_IT_ST, gi.STAT_X_LN_ST))},
                               "cycle_share": {k: round(st[i] / max(1, st[gi.STAT_X_CYC_ALL]), 4) for k, i in
                                               (("traverse", gi.STAT_X_CYC_TRAV), ("consume", gi.STAT_X_CYC_HIT),
                                                ("next_ray", gi.STAT_X_CYC_NEXT))}}
        if world == 1 and not args.no_host_path:
            out["host_path"] = host_path(gi, sc, dev, cam, sc.light, w, h, mode, spp, depth, args.seed)
            # SURVEY §8(d) ms/frame: the end-to-end gi_render time with the framebuffer's D2H copy
            # (RGB888, the reference Image's content) included
            out["ms_per_frame_with_d2h"] = out["host_path"]["ms_per_frame"]["rgb8"]
        if not args.no_cpu_baseline and world == 1:
            scn = sc.to_scn()
            gf = None
            if mode == 1:   # the last timed frame (deterministic: every timed frame is this one)
                gf = (buf.cpu().numpy().reshape(h, w, 3), buf8.cpu().numpy().reshape(h, w, 3))
            out["cpu_baseline"] = cpu_baseline(scn, w, h, mode, spp, depth, args.seed, gpu_frame=gf)
            ref = reference_cpu(scn, w, h)
            if ref is not None:
                out["reference_cpu"] = ref
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
