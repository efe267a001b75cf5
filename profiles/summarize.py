#!/usr/bin/env python3
"""Summarise a profiles/run_profile.sh output directory (gpurun_out/prof_<tag>) into one JSON:

  * kernel-trace --stats: per-kernel calls / average ns (the dominant kernel's average launch time
    must agree with bench.py's HIP-event `kernel_ms`);
  * PMC passes: per-dispatch averages for the dominant kernel (timed launches, not the STATS one);
  * derived: VALU lane utilisation = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU), memory-
    wait share = SQ_WAIT_ANY / SQ_WAVE_CYCLES, L2 hit rate, HBM bytes per launch
    = (2 * FETCH_SIZE + WRITE_SIZE) * 1024 (FETCH_SIZE/WRITE_SIZE are KiB; gfx950 FETCH_SIZE counts
    half of the bytes of wide reads, MI355X_MICROARCH.md §HBM, so it is doubled — an upper bound
    for narrower access widths).

    python profiles/summarize.py gpurun_out/prof_c3 C3 k_mode_x profiles/r01_c3_pmc.json [frames]

kernel "auto": the dominant one (by total time) of k_mode_x / k_wf_bounce / k_seg / k_mode_r_batch /
k_mode_r and the flat Mode R pipeline (k_rf_walk, k_rf_hit, k_rf_scan, k_rf_reach, k_rf_shade and its
k_mode_r_batch launch over the overflowed tiles), whose figures are the sums
over its kernels per frame (frames = k_rf_walk's timed calls).  The wavefront form (k_wf_bounce)
launches once per bounce, so its figures are per FRAME too: `frames` (the bench's timed + warm-up
frames) given, avg_launch_ns and every counter are the sums over the frame's dispatches (per PMC
pass: sum over all dispatches / frames).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SINGLE = ("k_mode_x", "k_wf_bounce", "k_seg", "k_mode_r_batch", "k_mode_r")


def finish(workload, out, stats, name, launch_ns, per, avg):
    der = {}
    if "SQ_THREAD_CYCLES_VALU" in avg and avg.get("SQ_ACTIVE_INST_VALU"):
        der["valu_lane_utilisation"] = avg["SQ_THREAD_CYCLES_VALU"] / (64.0 * avg["SQ_ACTIVE_INST_VALU"])
    if avg.get("SQ_WAVE_CYCLES"):
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if k in avg:
                der[k.lower() + "_share"] = avg[k] / avg["SQ_WAVE_CYCLES"]
    if "TCC_HIT_sum" in avg:
        der["l2_hit_rate"] = avg["TCC_HIT_sum"] / max(1.0, avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"])
    hbm = None
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        hbm = (2.0 * avg["FETCH_SIZE"] + avg["WRITE_SIZE"]) * 1024.0
    res = {"workload": workload, "kernel": name, "avg_launch_ns": launch_ns, "per": per,
           "hbm_bytes_per_launch": hbm, "counters_per_launch": avg, "derived": der, "kernel_stats": stats}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("workload", "avg_launch_ns", "hbm_bytes_per_launch")}), json.dumps(der))


def pmc_sums(d, names, per):
    """Per PMC pass: the counters of the named kernels' dispatches, summed and divided by `per`
    (None: one value per dispatch); averaged over passes / dispatches."""
    ctr = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        run = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] in names:
                if per:
                    run[r["Counter_Name"]] += float(r["Counter_Value"]) / per
                else:
                    ctr[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in run.items():
            ctr[k].append(v)
    return {k: sum(v) / len(v) for k, v in ctr.items()}


def main(d, workload, kernel, out, frames=None):
    frames = int(frames) if frames else None
    stats = {}
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                            "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])}
    flat = [k for k in stats if ("k_rf_" in k or "k_mode_r_batch" in k) and "<false" in k]
    if kernel == "auto":
        tot = {kn: sum(v["total_ns"] for k, v in stats.items() if kn + "<false" in k) for kn in SINGLE}
        if any("k_rf_walk" in k for k in flat):
            tot["k_rf_"] = sum(stats[k]["total_ns"] for k in flat)
        kernel = max(tot, key=tot.get)
    if kernel == "k_rf_":   # the flat Mode R pipeline: every timed launch of it, per frame
        n_fr = sum(stats[k]["calls"] for k in flat if "k_rf_walk" in k)
        finish(workload, out, stats, " + ".join(sorted(flat)), sum(stats[k]["total_ns"] for k in flat) / n_fr,
               "frame (sum over the pipeline's kernels)", pmc_sums(d, flat, n_fr))
        return
    # the timed launches: STATS=false is the kernel's first template argument (k_mode_x<false, ...>)
    dom = [k for k in stats if kernel + "<false" in k] or [k for k in stats if kernel in k]
    dom_name = max(dom, key=lambda k: stats[k]["total_ns"])
    per_frame = frames is not None and "k_wf_bounce" in dom_name
    launch_ns = stats[dom_name]["total_ns"] / frames if per_frame else stats[dom_name]["avg_ns"]
    finish(workload, out, stats, dom_name, launch_ns,
           "frame (sum over the per-bounce dispatches)" if per_frame else "dispatch",
           pmc_sums(d, [dom_name], frames if per_frame else None))


if __name__ == "__main__":
    main(*sys.argv[1:6])
