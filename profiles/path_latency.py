#!/usr/bin/env python3
"""Latency of one sample path with the chip otherwise idle vs under a full frame's load: renders
C4's frame alone, then single 8x8 tiles of it (default: the soup's core, pixel rows 952-967) (tile t = rank t of a shard_count > n_tiles split),
and prints the longest path's duration, wave iterations and traversal steps (GI_STAT_X_PATH_MAX)
and the kernel time of each launch.

    python profiles/path_latency.py [--workload C4] [--tiles 16200,16201,...]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C4")
    ap.add_argument("--tiles", default="28920,28921,28680,29160")
    ap.add_argument("--top", type=int, default=0,
                    help="Mode R: also time every tile of the frame alone and print the N slowest")
    a = ap.parse_args()
    import torch
    from importlib import import_module
    import bench
    gi = import_module("2019global_amd")
    scene_name, w, h, mode, spp, depth, desc = bench.WORKLOADS[a.workload]
    sc = bench.make_scene(scene_name)
    dev = gi.DeviceScene.from_scene(sc)
    cam = gi.Camera(sc.cam_pos, sc.cam_look, sc.focal)
    s = torch.cuda.current_stream()
    buf = torch.empty(w * h * 3, dtype=torch.float64, device="cuda")
    buf8 = torch.empty(w * h * 3, dtype=torch.uint8, device="cuda")
    n_tiles = ((w + 7) // 8) * ((h + 7) // 8)
    split = 1 << (n_tiles - 1).bit_length()   # > n_tiles: rank t renders tile t alone
    cases = [("frame", 1, 0)] + [(f"tile{t}", split, t) for t in map(int, a.tiles.split(","))]
    for name, n, r in cases:
        kw = dict(mode=mode, spp=spp, depth=depth, seed=2019, shard_count=n, shard_index=r)
        stats = torch.zeros(gi.STATS_N, dtype=torch.int64, device="cuda")
        dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), s.cuda_stream, stats_ptr=stats.data_ptr(), **kw)
        torch.cuda.synchronize()
        st = stats.cpu().tolist()
        for _ in range(3):
            dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), s.cuda_stream, flags=gi.FLAG_TIME, **kw)
        torch.cuda.synchronize()
        kms, kn = dev.kernel_ms()
        p = st[gi.STAT_X_PATH_MAX]
        ms, it, steps = (p >> 32) / 1e5, (p >> 16) & 0xFFFF, p & 0xFFFF
        print(json.dumps({"case": name, "kernel_ms": round(kms, 4), "rays": st[gi.STAT_RAYS],
                          "longest_path_ms_stats": round(ms, 4), "iterations": it, "steps": steps,
                          "us_per_iteration": round(ms * 1e3 / max(1, it), 3),
                          "wave_iterations": st[gi.STAT_X_ITERS], "lane_trav_steps": st[gi.STAT_X_TRAV],
                          "handler_runs": st[gi.STAT_X_HANDLE], "nodes": st[gi.STAT_NODES], "prims": st[gi.STAT_PRIMS],
                          "clk_per_iter": round(st[gi.STAT_X_CYC_ALL] / max(1, st[gi.STAT_X_ITERS]), 1),
                          # (round 6's GI_X_STEPPROBE measurement build read slots 16-20 here; its data is
                          # profiles/r06_c4_stepprobe.jsonl and the build was removed after)
                          "clk_share": {k: round(st[i] / max(1, st[gi.STAT_X_CYC_ALL]), 3) for k, i in
                                        (("trav", gi.STAT_X_CYC_TRAV), ("shade", gi.STAT_X_CYC_HIT),
                                         ("next", gi.STAT_X_CYC_NEXT))}}), flush=True)
    if a.top:   # every tile alone: is the frame bound by a few tiles' serial work?
        evs = []
        for t in range(n_tiles):
            kw = dict(mode=mode, spp=spp, depth=depth, seed=2019, shard_count=split, shard_index=t)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), s.cuda_stream, **kw)
            e1.record(s)
            evs.append((t, e0, e1))
        torch.cuda.synchronize()
        ms = sorted(((e0.elapsed_time(e1), t) for t, e0, e1 in evs), reverse=True)
        tot = sum(m for m, _ in ms)
        print(json.dumps({"tiles": len(ms), "sum_ms": round(tot, 3), "median_ms": round(ms[len(ms) // 2][0], 4),
                          "slowest": [(t, round(m, 4)) for m, t in ms[:a.top]]}), flush=True)

if __name__ == "__main__":
    main()
