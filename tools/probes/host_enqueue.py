"""Host-side cost of enqueueing frames (diagnostic): wall time of the
rtm_render_frames_async call itself (it returns once every launch is queued)
vs the GPU time of the same frames.  CFG env: bench config (default 2); N env: frames
(default 200; a short sequence, e.g. 24, measures the host cost without queue
back-pressure); outputs rotate over a ring of 48 frames, as in bench.py."""
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    rtm = importlib.import_module("2018rustraytracer_amd")
    sc = importlib.import_module("2018rustraytracer_amd.scenes")
    cfg = sc.CONFIGS[int(os.environ.get("CFG", "2"))]
    W, H, K = cfg["width"], cfg["height"], cfg["steps"]
    n = int(os.environ.get("N", "200"))
    ctx = rtm.Context(0)
    ctx.set_timing_capacity(1)
    ctx.set_timing_stride(1 << 30)  # only the first launch is timed
    ring = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in range(48)]
    cid = int(os.environ.get("CFG", "2"))
    scenes = [cfg["scene"]() if cid >= 5 else sc.scene_a_bench(100 + i) for i in range(n)]
    eye, sh = cfg.get("eye", sc.eye_camera)(), cfg.get("shadow", sc.shadow_camera)()
    prep = ctx.prepare_frames(scenes)
    res = {}
    for rep in range(3):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ctx.render_frames_async([0] * n, eye, sh, W, H, K, cfg["flags"], [ring[i % 48].data_ptr() for i in range(n)], prep)
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        res = {"frames": n, "lanes": ctx.last_lanes(), "batch": ctx.last_batch(),
               "enqueue_us_per_frame": (t1 - t0) / n * 1e6,
               "total_us_per_frame": (t2 - t0) / n * 1e6}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
