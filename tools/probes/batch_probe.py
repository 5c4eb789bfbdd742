"""Host enqueue time vs wall time of rtm_render_frames_async per frames-per-launch
(rtm_ctx_set_batch) for a bench config: where a batched sequence spends its time."""
import argparse
import importlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=7)
    ap.add_argument("--frames", type=int, default=400)
    ap.add_argument("--batches", default="1,2,4,8,16")
    ap.add_argument("--lanes", default="1")
    a = ap.parse_args()
    import torch
    rtm = importlib.import_module("2018rustraytracer_amd")
    sc = importlib.import_module("2018rustraytracer_amd.scenes")
    cfg = sc.CONFIGS[a.config]
    W, H, K = cfg["width"], cfg["height"], cfg["steps"]
    eye, shadow = cfg.get("eye", sc.eye_camera)(), sc.shadow_camera()
    scenes = [cfg["scene"]() if a.config >= 5 else sc.scene_a_bench(100 + i) for i in range(a.frames)]
    ctx = rtm.Context(0)
    ctx.set_timing_capacity(0)
    ring = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(48)]
    outs = [ring[i % 48].data_ptr() for i in range(a.frames)]
    prep = ctx.prepare_frames(scenes)
    for fused in (0, rtm.abi.RTM_FLAG_FUSED_SHADOW):
        for L in [int(x) for x in a.lanes.split(",")]:
            for B in [int(x) for x in a.batches.split(",")]:
                ctx.set_batch(B)
                ctx.set_lanes(L)
                fl = cfg["flags"] | fused
                for rep in range(3):
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    ctx.render_frames_async([0] * a.frames, eye, shadow, W, H, K, fl, outs, prep)
                    t1 = time.perf_counter()
                    ctx.synchronize()
                    t2 = time.perf_counter()
                print(f"config {a.config} fused={bool(fused)} lanes={ctx.last_lanes()} batch={ctx.last_batch()}: "
                      f"enqueue {1e6 * (t1 - t0) / a.frames:.2f} us/frame, wall {1e6 * (t2 - t0) / a.frames:.2f} "
                      f"us/frame = {W * H * a.frames / (t2 - t0) / 1e9:.1f} Gpix/s", flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
