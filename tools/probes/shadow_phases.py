"""Per-wave phase timing of the lean shadow tile (diagnostic).  Renders config-3
frames with RTM_DIAG_SHADOW=8 (s_memtime of lane 0 of every wave at six program
points, see RTM_PHASE in rtm_kernels.hip) and summarises: phase durations,
wave lifetimes, and how wave start/end times spread over the kernel.
Run on the GPU box: RTM_DIAG_SHADOW=8 python tools/probes/shadow_phases.py"""
import ctypes as C
import importlib
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    assert int(os.environ.get("RTM_DIAG_SHADOW", "0")) & 8, "set RTM_DIAG_SHADOW=8"
    import torch
    rtm = importlib.import_module("2018rustraytracer_amd")
    sc = importlib.import_module("2018rustraytracer_amd.scenes")
    cfg = sc.CONFIGS[int(os.environ.get("CFG", "3"))]
    W, H, K = cfg["width"], cfg["height"], cfg["steps"]
    ctx = rtm.Context(0)
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda:0")
    torch.cuda.synchronize()
    for f in range(5):
        ctx.render_async(cfg["scene"](), sc.eye_camera(), sc.shadow_camera(), W, H, K, cfg["flags"], out.data_ptr())
    ctx.synchronize()
    lib = rtm.load_library()
    n_waves = ((W + 127) // 128) * ((H + 15) // 16) * 4
    buf = np.zeros(n_waves * 8, np.uint64)
    assert lib.rtm_diag_shadow_phases(buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), int(buf.size)) == 0
    t = buf.reshape(n_waves, 8)[:, :6].astype(np.int64)
    t -= t[:, 0].min()
    ph = np.diff(t, axis=1)
    # coded tile (default; RTM_CODED=0: the lean tile's points): 0 loads issued, 1 raster
    # done + LDS written, 2 past the barrier, 3 march done, 4 stores issued, 5 drained
    names = (["loads+raster+LDS write", "barrier", "march", "stores issued", "stores drained"]
             if os.environ.get("RTM_CODED", "1") != "0" else
             ["fill-load+raster", "LDS write+barrier", "march", "stores issued", "stores drained"])
    res = {"waves": n_waves, "kernel_span_ticks": int(t[:, 5].max() - t[:, 0].min()),
           "lifetime_ticks": {"mean": float((t[:, 5] - t[:, 0]).mean()),
                              "p50": float(np.median(t[:, 5] - t[:, 0])),
                              "p99": float(np.percentile(t[:, 5] - t[:, 0], 99))},
           "phase_mean_ticks": {n: float(ph[:, i].mean()) for i, n in enumerate(names)},
           "phase_p99_ticks": {n: float(np.percentile(ph[:, i], 99)) for i, n in enumerate(names)},
           "start_ticks_percentiles": [float(np.percentile(t[:, 0], q)) for q in (0, 10, 50, 90, 100)],
           "end_ticks_percentiles": [float(np.percentile(t[:, 5], q)) for q in (0, 10, 50, 90, 100)],
           "note": "s_memtime ticks (the shader clock counter); waves of the last of 5 frames"}
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
