"""Concurrency probe (diagnostic): the same frame sequence rendered by one
context (one stream, one shadow map) vs split over C contexts on the same GPU
(C streams, C shadow maps, C output buffers), every context's frames enqueued
before any is waited on.  A 2-rank bench rehearsal on one GPU ran faster per
frame than one rank; this isolates whether in-process streams do the same.
CFG env: bench config (default 3); N env: frames (default 200)."""
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
    cfg = sc.CONFIGS[int(os.environ.get("CFG", "3"))]
    W, H, K = cfg["width"], cfg["height"], cfg["steps"]
    n = int(os.environ.get("N", "200"))
    eye, sh = cfg.get("eye", sc.eye_camera)(), sc.shadow_camera()
    scenes = [sc.scene_a_bench(100 + i) for i in range(n)]
    res = {}
    runs = [(nc, 1 << 30) for nc in (1, 2, 3, 4, 1, 2, 3)] + [(1, 10), (1, 50), (2, 10), (3, 10)]
    for nc, stride in runs:
        ctxs = [rtm.Context(0) for _ in range(nc)]
        for ctx in ctxs:
            ctx.set_timing_capacity(64)
            ctx.set_timing_stride(stride)  # 1 << 30: no per-frame timing events after launch 0
        outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0") for _ in range(nc)]
        parts = [scenes[c::nc] for c in range(nc)]
        preps = [ctx.prepare_frames(p) for ctx, p in zip(ctxs, parts)]
        best = None
        for rep in range(4):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for ctx, p, pr, o in zip(ctxs, parts, preps, outs):
                ctx.render_frames_async([0] * len(p), eye, sh, W, H, K, cfg["flags"], [o.data_ptr()] * len(p), pr)
            for ctx in ctxs:
                ctx.synchronize()
            dt = (time.perf_counter() - t0) / n * 1e6
            best = dt if best is None else min(best, dt)
        key = f"contexts_{nc}" + ("" if stride == 1 << 30 else f"_stride{stride}")
        res.setdefault(key, []).append(round(best, 2))
        for ctx in ctxs:
            ctx.close()
    print(json.dumps({"us_per_frame": res, "config": cfg["desc"], "frames": n}))


if __name__ == "__main__":
    main()
