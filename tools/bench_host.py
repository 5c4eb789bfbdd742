"""Host-buffer rates (not the headline): rtm_render (whole frame into caller-owned
host memory, blocking: kernels + D2H copy over PCIe) and rtm_write_ppm (GPU
encode + text, D2H of the text).  Prints one JSON line.
Usage: python tools/bench_host.py [--config 3] [--frames 20]"""
import argparse
import importlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=3)
    ap.add_argument("--frames", type=int, default=20)
    a = ap.parse_args()
    import ctypes as C

    import torch  # noqa: F401  (one HIP runtime per process, see abi.load_library)
    rtm = importlib.import_module("2018rustraytracer_amd")
    sc = importlib.import_module("2018rustraytracer_amd.scenes")
    cfg = sc.CONFIGS[a.config]
    W, H, K = cfg["width"], cfg["height"], cfg["steps"]
    eye = cfg.get("eye", sc.eye_camera)()
    scene = cfg["scene"]()
    lib = rtm.load_library()
    sc_c, keep = scene.to_c()
    e_c, s_c = eye.to_c(), sc.shadow_camera().to_c()
    host = np.empty((H, W, 4), np.float32)  # pageable, as a plain caller would pass
    ptr = host.ctypes.data_as(C.POINTER(C.c_float))

    def render():
        rtm.abi.check(lib, lib.rtm_render(C.byref(sc_c), C.byref(e_c), C.byref(s_c), W, H, K, cfg["flags"], ptr),
                      "rtm_render")

    for _ in range(3):
        render()
    t0 = time.perf_counter()
    for _ in range(a.frames):
        render()
    dt = (time.perf_counter() - t0) / a.frames

    ctx = rtm.Context(0)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
    ctx.render_async(scene, eye, sc.shadow_camera(), W, H, K, cfg["flags"], out.data_ptr())
    ctx.synchronize()
    ctx.write_ppm(out.data_ptr(), W, H)
    n = max(3, a.frames // 4)
    t0 = time.perf_counter()
    for _ in range(n):
        txt = ctx.write_ppm(out.data_ptr(), W, H)
    dp = (time.perf_counter() - t0) / n
    print(json.dumps({
        "config_id": a.config, "width": W, "height": H,
        "rtm_render_host": {"ms_per_frame": round(dt * 1e3, 3), "mpix_per_s": round(W * H / dt / 1e6, 1),
                            "d2h_bytes": W * H * 16,
                            "note": "blocking frame into pageable host memory: kernels + PCIe D2H"},
        "write_ppm_host": {"ms": round(dp * 1e3, 3), "bytes": len(txt),
                           "note": "GPU encode + P3 text + D2H of the text into a Python buffer"},
    }))


if __name__ == "__main__":
    main()
