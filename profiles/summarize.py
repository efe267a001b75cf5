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

kernel "auto": the dominant one of k_mode_x / k_wf_bounce / k_seg / k_mode_r_par / k_mode_r_split / k_mode_r (by
total time).  The wavefront
form (k_wf_bounce) launches once per bounce, so its figures are per FRAME: `frames` (the bench's
timed + warm-up frames) given, avg_launch_ns and every counter are the sums over the frame's
dispatches (per PMC pass: sum over all dispatches / frames).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(d, workload, kernel, out, frames=None):
    frames = int(frames) if frames else None
    stats = {}
    for r in csv.DictReader(open(os.path.join(d, "trace", "run_kernel_stats.csv"))):
        stats[r["Name"]] = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]),
                            "total_ns": float(r["TotalDurationNs"]), "pct": float(r["Percentage"])}
    if kernel == "auto":
        kernel = max(("k_mode_x", "k_wf_bounce", "k_seg", "k_mode_r_par", "k_mode_r_batch", "k_mode_r_split", "k_mode_r"),
                     key=lambda kn: sum(v["total_ns"] for k, v in stats.items() if kn + "<false" in k))
    # the timed launches: STATS=false is the kernel's first template argument (k_mode_x<false, ...>)
    dom = [k for k in stats if kernel + "<false" in k] or [k for k in stats if kernel in k]
    dom_name = max(dom, key=lambda k: stats[k]["total_ns"])
    per_frame = frames is not None and "k_wf_bounce" in dom_name
    ctr = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "pmc*", "run_counter_collection.csv"))):
        run = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r["Kernel_Name"] == dom_name:
                if per_frame:
                    run[r["Counter_Name"]] += float(r["Counter_Value"]) / frames
                else:
                    ctr[r["Counter_Name"]].append(float(r["Counter_Value"]))
        for k, v in run.items():
            ctr[k].append(v)
    avg = {k: sum(v) / len(v) for k, v in ctr.items()}
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
    launch_ns = stats[dom_name]["total_ns"] / frames if per_frame else stats[dom_name]["avg_ns"]
    res = {"workload": workload, "kernel": dom_name, "avg_launch_ns": launch_ns,
           "per": "frame (sum over the per-bounce dispatches)" if per_frame else "dispatch",
           "hbm_bytes_per_launch": hbm, "counters_per_launch": avg, "derived": der,
           "kernel_stats": stats}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: res[k] for k in ("workload", "avg_launch_ns", "hbm_bytes_per_launch")}), json.dumps(der))


if __name__ == "__main__":
    main(*sys.argv[1:6])
