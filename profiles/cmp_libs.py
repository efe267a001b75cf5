"""Renders one Mode X frame with two libgi builds (GI_LIB paths) and reports bit differences.
   python profiles/cmp_libs.py <libA> <libB> [workload]"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r'''
import sys, os, numpy as np, torch
sys.path.insert(0, os.environ["ROOT"])
from importlib import import_module
gi = import_module("2019global_amd"); import bench
sc_name, w, h, mode, spp, depth, _ = bench.WORKLOADS[sys.argv[1]]
sc = bench.make_scene(sc_name)
d = gi.DeviceScene.from_scene(sc)
rgb, rgb8 = d.render(gi.Camera(sc.cam_pos, sc.cam_look, sc.focal), sc.light, w, h, mode=mode, spp=spp, depth=depth, seed=2019)
np.save(sys.argv[2], rgb)
'''
a, b = sys.argv[1], sys.argv[2]
wl = sys.argv[3] if len(sys.argv) > 3 else "C3"
outs = []
for i, lib in enumerate((a, b)):
    out = f"/tmp/cmp_{i}.npy"
    subprocess.run([sys.executable, "-c", CHILD, wl, out], check=True, env=dict(os.environ, GI_LIB=lib, ROOT=ROOT))
    outs.append(np.load(out))
x, y = outs
same = (x.view(np.int64) == y.view(np.int64)).all(-1)
print(json.dumps({"workload": wl, "pixels": int(same.size), "differing": int((~same).sum()),
                  "max_abs": float(np.nanmax(np.abs(x - y)))}))
