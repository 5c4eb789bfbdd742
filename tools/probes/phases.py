"""Per-wave phase timing (diagnostic, A/B builds only): renders one batched launch of a
config's frames on one lane with a library built with -DRTM_AB_PHASES
(tools/ab_lib.sh phases "-DRTM_AB_PHASES") and summarises the s_memtime stamps each
wave wrote at its program points (RTM_PHASE in rtm_kernels.hip): regions 0-2 = the
coded shadow tile PART 0/1/2, region 3 = the eye tile.
Run on the GPU box: RTM_LIB=$PWD/2018rustraytracer_amd/librtm_phases.so CFG=3 python tools/probes/phases.py"""
import ctypes as C
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

NAMES = {0: "shadow PART 0", 1: "shadow PART 1 (raster-free strips)", 2: "shadow PART 2 (sphere strips)", 3: "eye tile"}
POINTS = {0: ["entry", "records+LDS+barrier", "strip0 march", "strip0 raster", "strip0 stored", "all strips drained"],
          1: ["entry", "records+LDS+barrier", "strip0 march", "strip0 raster", "strip0 stored", "all strips drained"],
          2: ["entry", "records+LDS+barrier", "strip0 march", "strip0 raster", "strip0 stored", "all strips drained"],
          3: ["entry", "masks ready", "traced+shaded", "stored+drained"]}


def main():
    import torch
    lib_path = os.environ["RTM_LIB"]
    rtm = importlib.import_module("2018rustraytracer_amd")
    sc = importlib.import_module("2018rustraytracer_amd.scenes")
    rtm.load_library()
    diag = C.CDLL(lib_path)
    diag.rtm_diag_phase_region.restype = C.c_longlong
    R = int(diag.rtm_diag_phase_region())
    cfg_id = int(os.environ.get("CFG", "3"))
    cfg = sc.CONFIGS[cfg_id]
    W, H, K = cfg["width"], cfg["height"], cfg["steps"]
    eye, shadow = cfg.get("eye", sc.eye_camera)(), cfg.get("shadow", sc.shadow_camera)()
    buf = torch.zeros(4 * R * 8, dtype=torch.int64, device="cuda")
    assert diag.rtm_diag_set_phase_buffer(C.c_void_p(buf.data_ptr())) == 0
    ctx = rtm.Context(0)
    ctx.set_lanes(1)
    px = W * H
    F = max(1, min(64 if px < (1 << 20) else 32, (64 << 20) // px))  # one launch of the auto batch
    scenes = [sc.scene_a_bench(100 + i) if cfg_id in (2, 3, 4) else cfg["scene"]() for i in range(F)]
    outs = [torch.empty((H, W, 4), dtype=torch.float32, device="cuda") for _ in range(F)]
    ptrs = [o.data_ptr() for o in outs]
    for _ in range(5):
        ctx.render_frames_async(scenes, eye, shadow, W, H, K, cfg["flags"], ptrs)
    ctx.synchronize()
    buf.zero_()
    torch.cuda.synchronize()
    ctx.render_frames_async(scenes, eye, shadow, W, H, K, cfg["flags"], ptrs)
    ctx.synchronize()
    b = buf.cpu().numpy().reshape(4, R, 8)
    res = {"config": cfg_id, "frames_per_launch": F, "note": "s_memtime ticks; each stamp after s_waitcnt(0)"}
    for r in range(4):
        n = len(POINTS[r])
        rows = b[r][:, :n]
        live = rows[:, 0] != 0
        if not live.any():
            continue
        t = rows[live].astype(np.int64)
        done = (t != 0).all(axis=1)  # waves that reached every point (early-out waves skip some)
        t0 = t[:, 0].min()
        last = np.where(t != 0, t, 0).max(axis=1)
        life = last - t[:, 0]
        d = {"waves": int(live.sum()), "waves_all_points": int(done.sum()),
             "kernel_span_ticks": int(last.max() - t0),
             "lifetime_ticks": {"mean": float(life.mean()), "p50": float(np.median(life)),
                                "p90": float(np.percentile(life, 90))},
             "start_ticks_percentiles": [float(np.percentile(t[:, 0] - t0, q)) for q in (0, 25, 50, 75, 100)],
             "end_ticks_percentiles": [float(np.percentile(last - t0, q)) for q in (0, 25, 50, 75, 100)]}
        if done.any():
            ph = np.diff(t[done], axis=1)
            d["phase_mean_ticks"] = {f"{POINTS[r][i]} -> {POINTS[r][i + 1]}": float(ph[:, i].mean()) for i in range(n - 1)}
            d["phase_p50_ticks"] = {f"{POINTS[r][i]} -> {POINTS[r][i + 1]}": float(np.median(ph[:, i]))
                                    for i in range(n - 1)}
        res[NAMES[r]] = d
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
