#!/usr/bin/env python3
"""Frame-pipelining probe on ONE GPU: K frames rendered back to back on one
stream and scene handle (what bench.py does) against the same K frames alternating over two scene
handles on two streams, so that frame i+1's work fills frame i's ramp-down.  Reported for the whole
C3 frame and for one rank's share at N = 8.  Throughput only: each frame's latency is unchanged.

    python profiles/pipeline_probe.py [--frames 12]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=12)
    ap.add_argument("--workload", default="C3")
    a = ap.parse_args()
    import torch
    from importlib import import_module
    import bench
    gi = import_module("2019global_amd")
    scene_name, w, h, mode, spp, depth, _ = bench.WORKLOADS[a.workload]
    sc = bench.make_scene(scene_name)
    cam = gi.Camera(sc.cam_pos, sc.cam_look, sc.focal)
    scenes = [gi.DeviceScene.from_scene(sc) for _ in range(2)]
    streams = [torch.cuda.Stream() for _ in range(2)]
    for n in (1, 8):
        px = gi.shard_tiles(w, h, n) * gi.TILE * gi.TILE * 3
        bufs = [(torch.empty(px, dtype=torch.float64, device="cuda"), torch.empty(px, dtype=torch.uint8, device="cuda"))
                for _ in range(2)]
        kw = dict(mode=mode, spp=spp, depth=depth, seed=2019, shard_count=n, shard_index=0)
        res = {"workload": a.workload, "shard_count": n}
        for inflight in (1, 2):
            def frame(i):
                k = i % inflight
                scenes[k].render_device(cam, sc.light, w, h, bufs[k][0].data_ptr(), bufs[k][1].data_ptr(),
                                        streams[k].cuda_stream, **kw)
            for i in range(2 * inflight):   # warm both handles (work buffers are allocated on first use)
                frame(i)
            torch.cuda.synchronize()
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record(streams[0])
            streams[1].wait_event(ev0)
            for i in range(a.frames):
                frame(i)
            done = torch.cuda.Event()
            done.record(streams[1])
            streams[0].wait_event(done)
            ev1.record(streams[0])
            torch.cuda.synchronize()
            res[f"ms_per_frame_inflight{inflight}"] = round(ev0.elapsed_time(ev1) / a.frames, 4)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
