#!/usr/bin/env python3
"""k_rf_reach's chunks at N ranks (GI_RF_PROBE measurement build, GI_LIB=...): for rank 0 and rank
N-1 of each N, the slowest wave's time and node tests, the mean, and the largest per-lane work --
is the reach phase bound by a few heavy chunks?

    GI_LIB=2019global_amd/_variants/libgi_rfprobe.so python profiles/rf_probe.py [--workload R-C4] [--ns 1,8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="R-C4")
    ap.add_argument("--ns", default="1,8")
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
    for n in [int(x) for x in a.ns.split(",")]:
        for r in sorted({0, n - 1}):
            kw = dict(mode=mode, spp=spp, depth=depth, seed=2019, shard_count=n, shard_index=r)
            st = torch.zeros(gi.STATS_N, dtype=torch.int64, device="cuda")
            dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), s.cuda_stream, stats_ptr=st.data_ptr(), **kw)
            torch.cuda.synchronize()
            v = st.cpu().tolist()
            waves = max(1, v[7])
            print(json.dumps({"n": n, "rank": r, "waves_with_work": v[7], "chunks": v[12],
                              "slowest_wave_us": v[5] / 100.0, "mean_wave_us": round(v[6] / 100.0 / waves, 2),
                              "slowest_wave_node_tests": v[13] & 0xFFFFFFFF,
                              "max_lane_appearances": v[8], "max_lane_node_tests": v[9], "max_wave_node_tests": v[10],
                              "appearances": v[11], "node_tests": v[gi.STAT_NODES], "pairs": v[gi.STAT_R_PAIRS]}), flush=True)


if __name__ == "__main__":
    main()
