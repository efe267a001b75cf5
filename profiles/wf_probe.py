#!/usr/bin/env python3
"""A/B of the two Mode X forms on one GPU: the persistent path-state kernel (k_mode_x, FLAG_X_MEGA)
and the wavefront form (k_wf_bounce per bounce, FLAG_X_WF).  Per workload: both frames (fp64 bits
and RGB888 must be identical), the render-call time and the dominant pass's time (HIP events) of
each, K timed frames after W warm-up frames.  One JSON line per workload.

    python profiles/wf_probe.py [--steps K] [--warmup W] C3 C2 C4 ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seed", type=int, default=2019)
    ap.add_argument("--forms", default="mega,wf,seg")
    ap.add_argument("workloads", nargs="+")
    args = ap.parse_args()
    import torch
    from importlib import import_module
    gi = import_module("2019global_amd")
    bench = import_module("bench")
    torch.cuda.set_device(0)
    stream = torch.cuda.current_stream()
    forms = {"mega": gi.FLAG_X_MEGA, "wf": gi.FLAG_X_WF, "seg": gi.FLAG_X_SEG}
    for wl in args.workloads:
        scene_name, w, h, mode, spp, depth, desc = bench.WORKLOADS[wl]
        sc = bench.make_scene(scene_name)
        dev = gi.DeviceScene.from_scene(sc)
        cam = gi.Camera(sc.cam_pos, sc.cam_look, sc.focal)
        out = {"workload": wl}
        frames = {}
        for name in args.forms.split(","):
            fl = forms[name]
            buf = torch.empty(w * h * 3, dtype=torch.float64, device="cuda")
            buf8 = torch.empty(w * h * 3, dtype=torch.uint8, device="cuda")
            stats = torch.zeros(gi.STATS_N, dtype=torch.int64, device="cuda")
            kw = dict(mode=mode, spp=spp, depth=depth, seed=args.seed)
            dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), stream.cuda_stream,
                              stats_ptr=stats.data_ptr(), flags=fl, **kw)
            torch.cuda.synchronize()
            st = stats.cpu().tolist()
            for _ in range(args.warmup):
                dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), stream.cuda_stream,
                                  flags=fl | gi.FLAG_TIME, **kw)
            torch.cuda.synchronize()
            dev.kernel_ms()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), stream.cuda_stream,
                                  flags=fl | gi.FLAG_TIME, **kw)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            kms, n = dev.kernel_ms()
            frames[name] = (buf.view(torch.int64).clone(), buf8.clone())
            out[name] = {"ms_per_frame": round(ms, 4), "pass_ms": round(kms, 4), "rays": st[gi.STAT_RAYS],
                         "resolved": st[gi.STAT_X_RESOLVED], "nodes": st[gi.STAT_NODES], "prims": st[gi.STAT_PRIMS],
                         "pixels": st[gi.STAT_PIXELS]}
        names = list(frames)
        for nm in names[1:]:   # every form's frame against the first form's, bit for bit
            a, b = frames[names[0]], frames[nm]
            same = bool(torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]))
            out.setdefault("identical", True)
            out["identical"] = out["identical"] and same
            if not same:
                out["n_diff_" + nm] = int((a[0] != b[0]).sum().item())
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
