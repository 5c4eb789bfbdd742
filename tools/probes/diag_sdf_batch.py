"""Probe: the batched SDF frames with a materialised (all +INF) shadow viewport --
frames and the last decoded shadow map against the oracle, per frame count."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import importlib  # noqa: E402

rtm = importlib.import_module("2018rustraytracer_amd")
sc = importlib.import_module("2018rustraytracer_amd.scenes")
import oracle as O  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
W, H, K = 192, 132, 16
cases = {"sdf_persp": (sc.sdf_bench_scene(), sc.sdf_eye_camera()),
         "rt_persp": (sc.scene_r_bench(), sc.perspective_eye_camera())}
for name, (s, eye) in cases.items():
    want = O.render(s, eye, sc.shadow_camera(), W, H, K, 0, nthreads=8, want_shadow=True)
    for n in (1, 2, 3, 8):
        ctx = rtm.Context(0)
        outs = [torch.full((H, W, 4), -7.0, dtype=torch.float32, device="cuda") for _ in range(n)]
        torch.cuda.synchronize()
        ctx.render_frames_async([s] * n, eye, sc.shadow_camera(), W, H, K, 0, [o.data_ptr() for o in outs])
        ctx.synchronize()
        bad = []
        for i, o in enumerate(outs):
            g = o.cpu().numpy()
            d = np.argwhere(np.any(g.view(np.uint32) != want["rgba"].view(np.uint32), axis=-1))
            bad.append((i, len(d), tuple(d[0]) if len(d) else None))
        m = np.empty((H, W), np.float64)
        p = ctx.shadow_map_ptr()
        msg = ""
        if p and hip.hipMemcpy(m.ctypes.data, p, W * H * 8, 2) == 0:
            dm = np.argwhere(m.view(np.uint64) != want["shadow"].view(np.uint64))
            msg = f"map: {len(dm)} texels differ" + (f", first {tuple(dm[0])} got {m[tuple(dm[0])]} want "
                                                    f"{want['shadow'][tuple(dm[0])]}, rows {dm[:,0].min()}..{dm[:,0].max()} "
                                                    f"cols {dm[:,1].min()}..{dm[:,1].max()}" if len(dm) else "")
        print(f"{name} n={n} batch={ctx.last_batch()} texel_bytes={ctx.shadow_map_texel_bytes()} frames {bad} {msg}",
              flush=True)
        ctx.close()
