"""Time the writeColorImage kernels (BASELINE §8f-2) on one 4K frame.

encode_rgb8: 16 B read (RGBA f32) + 3 B written (RGB8) per pixel — HBM-bound.
write_ppm:   the whole call (encode + row lengths + scan + text + D2H copy).
Prints one JSON line.  Usage: python tools/bench_encode.py [--iters N]
"""
import argparse
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    a = ap.parse_args()
    import torch
    rtm = importlib.import_module("2018rustraytracer_amd")
    scenes = importlib.import_module("2018rustraytracer_amd.scenes")
    w, h = a.width, a.height
    ctx = rtm.Context(0)
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda:0")
    cfg = scenes.CONFIGS[3]
    ctx.render_async(cfg["scene"](), scenes.eye_camera(), scenes.shadow_camera(), w, h, cfg["steps"], cfg["flags"],
                     out.data_ptr())
    rgb = torch.empty(w * h * 3, dtype=torch.uint8, device="cuda:0")
    s = torch.cuda.ExternalStream(ctx.stream, device="cuda:0")  # events on the stream the kernel runs on
    for _ in range(10):
        ctx.encode_rgb8_async(out.data_ptr(), w * h, rgb.data_ptr())
    ctx.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(a.iters):
        ctx.encode_rgb8_async(out.data_ptr(), w * h, rgb.data_ptr())
    e1.record(s)
    e1.synchronize()
    enc_ms = e0.elapsed_time(e1) / a.iters
    ctx.write_ppm(out.data_ptr(), w, h)
    n_ppm = max(1, a.iters // 20)
    t0 = time.perf_counter()
    for _ in range(n_ppm):
        txt = ctx.write_ppm(out.data_ptr(), w, h)
    ppm_ms = (time.perf_counter() - t0) * 1e3 / n_ppm
    algo = 19 * w * h
    print(json.dumps(dict(
        kernel="encode_rgb8", width=w, height=h, avg_launch_ms=round(enc_ms, 5),
        mpix_per_s=round(w * h / enc_ms / 1e3, 1),
        roofline=dict(bound="hbm", achieved=round(algo / enc_ms / 1e6, 1), peak=8000.0, unit="GB/s",
                      frac=round(algo / enc_ms / 1e6 / 8000.0, 4), algorithmic_bytes_per_launch=algo),
        write_ppm_ms=round(ppm_ms, 3), ppm_bytes=len(txt),
        write_ppm_note="whole call incl. device->host copy of the text over PCIe")))


if __name__ == "__main__":
    main()
