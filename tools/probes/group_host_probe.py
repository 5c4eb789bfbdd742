import importlib, sys, time
sys.path.insert(0, '/root/repo') if False else None
import os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
rtm = importlib.import_module("2018rustraytracer_amd")
sc = importlib.import_module("2018rustraytracer_amd.scenes")
w, h, k = 3840, 2160, 64
s, eye, sh = sc.scene_a_bench(100), sc.eye_camera(), sc.shadow_camera()
g = rtm.Group(n_devices=1)
out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
def t(f, n=10):
    f()
    t0 = time.perf_counter()
    for _ in range(n): f()
    return (time.perf_counter() - t0) / n * 1e3
def dev():
    g.render_async(s, eye, sh, w, h, k, 0, 0, 0, out.data_ptr()); g.synchronize(0)
host = np.empty((h, w, 4), np.float32)
print("group device-out ms", t(dev))
print("group host-out ms", t(lambda: g.render(s, eye, sh, w, h, k, 0, 0, out=host)))
print("render_ex host ms", t(lambda: rtm.render_frame_ex(s, eye, sh, w, h, k, 0, 0, out=host)))
with rtm.HostRegistration(host):
    print("group host-out registered ms", t(lambda: g.render(s, eye, sh, w, h, k, 0, 0, out=host)))
    print("render_ex registered ms", t(lambda: rtm.render_frame_ex(s, eye, sh, w, h, k, 0, 0, out=host)))
def hc():
    torch.cuda.synchronize(); 
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    assert hip.hipMemcpy(host.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(out.data_ptr()), ctypes.c_size_t(host.nbytes), 2) == 0
print("plain hipMemcpy D2H pageable ms", t(hc))
g.close()
