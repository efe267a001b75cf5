#!/usr/bin/env python3
"""Strong-scaling probe on ONE GPU: time the render of one rank's share of the frame for
shard_count N = 1, 2, 4, 8 (rank 0 and rank N-1 of N), i.e. the per-rank kernel time of an N-GPU
run without the gather.  ideal = t(1) / N; the ratio shows the load-balance tail at small shares.

    python profiles/shard_scaling.py [--workload C3] [--reps 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="C3")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ns", default="1,2,4,8")
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
    res = {"workload": a.workload}
    t1 = None
    for n in [int(x) for x in a.ns.split(",")]:
        for r in sorted({0, n - 1}):
            kw = dict(mode=mode, spp=spp, depth=depth, seed=2019, shard_count=n, shard_index=r)
            dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), s.cuda_stream, **kw)
            e0 = torch.cuda.Event(enable_timing=True)
            e1 = torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(a.reps):
                dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), s.cuda_stream,
                                  **dict(kw, flags=gi.FLAG_TIME))
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / a.reps
            kms, _ = dev.kernel_ms()   # the dominant kernel alone (k_mode_x)
            st_t = torch.zeros(gi.STATS_N, dtype=torch.int64, device="cuda")
            dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), s.cuda_stream,
                              stats_ptr=st_t.data_ptr(), **kw)
            st = st_t.cpu().tolist()
            it, rays = st[gi.STAT_X_ITERS], max(1, st[gi.STAT_RAYS])
            sched = {"rays": rays, "wave_iters_per_kray": round(it * 1e3 / rays, 3),
                     "trav_lane_fill": round(st[gi.STAT_X_TRAV] / max(1, 64.0 * it), 4),
                     "handler_lane_fill": round(st[gi.STAT_X_HLANES] / max(1, 64.0 * st[gi.STAT_X_HANDLE]), 4),
                     "longest_path_ms": round((st[gi.STAT_X_PATH_MAX] >> 32) / 1e5, 4),
                     "longest_path_iters": (st[gi.STAT_X_PATH_MAX] >> 16) & 0xFFFF}
            if n == 1:
                t1 = ms
            res[f"N{n}_rank{r}_ms"] = round(ms, 3)
            if t1:
                res[f"N{n}_rank{r}_speedup"] = round(t1 / ms, 3)
            print(json.dumps({"n": n, "rank": r, "ms": round(ms, 3), "kernel_ms": round(kms, 3),
                              "ideal_ms": round(t1 / n, 3) if t1 else None,
                              "speedup": round(t1 / ms, 3) if t1 else None, **sched}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
