import sys, time, torch
sys.path.insert(0, '.')
from importlib import import_module
gi = import_module("2019global_amd"); S = import_module("2019global_amd.scenes")
sc = S.cornell_scene(); d = gi.DeviceScene.from_scene(sc); cam = gi.Camera(sc.cam_pos, sc.cam_look, sc.focal)
mode = sys.argv[1]; w = int(sys.argv[2]); h = int(sys.argv[3])
buf = torch.zeros(w*h*3, dtype=torch.float64, device='cuda')
st = torch.zeros(8, dtype=torch.int64, device='cuda')
t = time.time()
kw = dict(mode=gi.MODE_X, spp=1, depth=4, seed=1)
if mode == 'stats': kw['stats_ptr'] = st.data_ptr()
if mode == 'stream': d.render_device(cam, sc.light, w, h, buf.data_ptr(), 0, torch.cuda.current_stream().cuda_stream, **kw)
else: d.render_device(cam, sc.light, w, h, buf.data_ptr(), **kw)
torch.cuda.synchronize(); print(mode, w, h, "ok %.3fs" % (time.time()-t), st.tolist(), flush=True)
