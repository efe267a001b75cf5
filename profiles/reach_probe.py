"""Probe of k_rf_reach's per-hit work and chunk timeline (R-C4), with the probe build: apply
profiles/r06_reach/reach_probe.patch to a scratch copy of the tree (it adds the per-hit / per-chunk
stores under GI_REACH_PROBE; the product source carries no probe code), then
`python 2019global_amd/build.py --variant reachprobe GI_REACH_PROBE` and select it with GI_LIB.

Per hitting pair: appearances walked and node tests; per chunk of 64 pairs: wall-clock start / end.
Prints, for the whole frame and for each eighth (shard_count 8), the distribution of per-hit work,
per-chunk lane maxima, chunk durations and the kernel's span.  Output: one JSON line per case."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from importlib import import_module  # noqa: E402

gi = import_module("2019global_amd")
S = import_module("2019global_amd.scenes")

name = sys.argv[1] if len(sys.argv) > 1 else "soup100000"
sc = S.named_scene(name)
dev = gi.DeviceScene.from_scene(sc)
cam = gi.Camera(sc.cam_pos, sc.cam_look, sc.focal)
w, h = 1920, 1080
buf = torch.empty(w * h * 3, dtype=torch.float64, device="cuda")
buf8 = torch.empty(w * h * 3, dtype=torch.uint8, device="cuda")
stats = torch.empty(64 << 20, dtype=torch.int64, device="cuda")
os.environ["GI_REACH_PROBE_PTR"] = str(stats.data_ptr())   # the production (non-STATS) kernels run
sptr = torch.cuda.current_stream().cuda_stream


def q(a, ps=(50, 90, 99, 99.9, 100)):
    return [float(np.percentile(a, p)) for p in ps] if len(a) else []


for shard_count, shard_index in [(1, 0)] + [(8, k) for k in range(8)]:
    for rep in range(2):   # the second render is measured (the first builds scratch)
        stats.fill_(-1)
        stats[:64].zero_()
        dev.render_device(cam, sc.light, w, h, buf.data_ptr(), buf8.data_ptr(), sptr, mode=gi.MODE_R,
                          shard_count=shard_count, shard_index=shard_index)
        torch.cuda.synchronize()
    s = stats.cpu().numpy()
    n_hits = int(s[63])
    per = s[64:64 + 2 * n_hits].reshape(-1, 2)
    napp, nn = per[:, 0], per[:, 1]
    g = int(os.environ.get("GI_RF_GROUP", "0"))   # k_rf_reach's lanes per hit: chunks of 64 / G hits
    G = g if g in (1, 4) else (4 if n_hits <= 40960 else 1)
    nch = (n_hits + 64 // G - 1) // (64 // G)
    ch3 = s[64 + 2 * n_hits:64 + 2 * n_hits + 3 * nch].reshape(-1, 3).astype(np.float64)
    ok = (ch3 >= 0).all(1)
    ch3 = ch3[ok]
    find_us = (ch3[:, 1] - ch3[:, 0]) / 100.0   # rf_find + the lanes' segment scan + memo clear
    ch = ch3[:, 1:]
    dur_us = (ch[:, 1] - ch[:, 0]) / 100.0   # s_memrealtime: 100 MHz
    span_us = (ch[:, 1].max() - ch3[:, 0].min()) / 100.0 if len(ch) else 0.0
    t_base = ch3[:, 0].min() if len(ch) else 0.0
    pad = np.zeros(nch * (64 // G), np.int64)
    pad[:n_hits] = nn
    lane_max = pad.reshape(-1, 64 // G).max(1)
    lane_mean = pad.reshape(-1, 64 // G).mean(1)
    # the chunks that end last: how long did they run and how much node work did they hold
    order = np.argsort(ch[:, 1])[-8:] if len(ch) else []
    out = {"scene": name, "shard": f"{shard_index}/{shard_count}", "n_hits": n_hits, "lanes_per_hit": G, "chunks": int(nch),
           "nodes_total": int(nn.sum()), "apps_total": int(napp.sum()),
           "nodes_per_hit_p50_90_99_999_max": q(nn), "apps_per_hit_p50_90_99_999_max": q(napp),
           "chunk_lane_max_nodes_p50_90_99_max": q(lane_max, (50, 90, 99, 100)),
           "chunk_fill": float(lane_mean.sum() / max(1, lane_max.sum())),
           "chunk_us_p50_90_99_max": q(dur_us, (50, 90, 99, 100)), "span_us": span_us,
           "find_us_p50_90_99_max": q(find_us, (50, 90, 99, 100)),
           "top_start_us_p50_90_99_max": q((ch3[:, 0] - t_base) / 100.0, (50, 90, 99, 100)),
           "last_chunks": [{"us": float(dur_us[i]), "lane_max_nodes": int(lane_max[np.flatnonzero(ok)[i]]),
                            "start_us": float((ch3[i, 0] - t_base) / 100.0), "find_us": float(find_us[i])} for i in order]}
    print(json.dumps(out), flush=True)
