# Diagnostic: Mode X cost of rays that all miss (raygen + handler + root cull only) vs the C3 frame.
import sys, time, torch
sys.path.insert(0, '.')
from importlib import import_module
gi = import_module("2019global_amd"); S = import_module("2019global_amd.scenes")
def run(sc, w, h, spp, depth, reps=3):
    d = gi.DeviceScene.from_scene(sc); cam = gi.Camera(sc.cam_pos, sc.cam_look, sc.focal)
    buf = torch.zeros(w*h*3, dtype=torch.float64, device='cuda'); st = torch.zeros(8, dtype=torch.int64, device='cuda')
    kw = dict(mode=gi.MODE_X, spp=spp, depth=depth, seed=1)
    d.render_device(cam, sc.light, w, h, buf.data_ptr(), stats_ptr=st.data_ptr(), **kw); torch.cuda.synchronize()
    t = time.time()
    for _ in range(reps): d.render_device(cam, sc.light, w, h, buf.data_ptr(), **kw)
    torch.cuda.synchronize(); dt = (time.time() - t) / reps
    rays = st[0].item(); print(f"rays {rays} ms {dt*1e3:.2f} Mray/s {rays/dt/1e6:.1f} ns/ray/CU {dt/rays*256*1e9:.1f}")
miss = S.Scene(entities=[]); miss.imp_sphere((0.0, 0.0, -500.0), 1, (1, 1, 1))
print("all-miss 1080p 64spp:", end=" "); run(miss, 1920, 1080, 64, 8)
print("C3:", end=" "); run(S.cornell_scene(), 1920, 1080, 64, 8)
print("C3 1spp depth1:", end=" "); run(S.cornell_scene(), 1920, 1080, 1, 1)
