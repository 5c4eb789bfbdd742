#!/usr/bin/env python3
"""Per-band render cost of the tile-partitioned frame (VERDICT r02
item 4), on one GPU: for N in (2, 4, 8) bands of ceil(H/N) rows, each band
rendered alone with the fused shadow (what rank r renders in the multi-GPU
frame: rtm_render_rows_async, RTM_FLAG_FUSED_SHADOW), timed with HIP events on
the context's stream over `reps` frames after warm-up.  Reports ms per band,
max/mean, the cyclic 8-row-stripe alternative's balance (same band sizes,
modelled from a per-stripe profile at N = H/8, and measured: each rank's 8-row
stripes rendered by rtm_render_stripes_async), and the unbanded two-pass frame.

usage: python tools/band_balance.py [configs ...]   (default 3 4 5) -> JSON on stdout
"""
import ctypes as C
import importlib
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    rtm = importlib.import_module("2018rustraytracer_amd")
    sc = importlib.import_module("2018rustraytracer_amd.scenes")
    shard = importlib.import_module("2018rustraytracer_amd.shard")
    lib = rtm.load_library()
    cfgs = [int(a) for a in sys.argv[1:]] or [3, 4, 5]
    reps = int(os.environ.get("BAND_REPS", "8"))
    ctx = rtm.Context(0)
    stream = torch.cuda.ExternalStream(ctx.stream)
    out = {}
    for cfg in cfgs:
        c = sc.CONFIGS[cfg]
        W, H, K = c["width"], c["height"], c["steps"]
        scene = sc.scene_a_bench(100) if c["scene"] is sc.scene_a_bench else c["scene"]()
        s_c, keep = scene.to_c()
        e_c, sh_c = sc.eye_camera().to_c(), sc.shadow_camera().to_c()
        buf = torch.empty(W * H * 16, dtype=torch.uint8, device="cuda")

        def time_rows(r0, r1, flags):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for it in range(2 + reps):
                if it == 2:
                    ev0.record(stream)
                rc = lib.rtm_render_rows_async(ctx.handle, C.byref(s_c), C.byref(e_c), C.byref(sh_c), W, H, K,
                                               flags | c["flags"], 0, r0, r1, C.c_void_p(buf.data_ptr()))
                rtm.abi.check(lib, rc, "rtm_render_rows_async")
            ev1.record(stream)
            ev1.synchronize()
            return ev0.elapsed_time(ev1) / reps

        fused = rtm.abi.RTM_FLAG_FUSED_SHADOW
        res = {"width": W, "height": H, "steps": K, "frame_two_pass_ms": round(time_rows(0, H, 0), 4),
               "frame_fused_ms": round(time_rows(0, H, fused), 4)}
        # 8-row stripe profile (fused), for the cyclic-stripe model
        stripes = [time_rows(y, min(H, y + 8), fused) for y in range(0, H, 8)] if H <= 4320 else []
        def time_stripes(n, r, S, flags):
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for it in range(2 + reps):
                if it == 2:
                    ev0.record(stream)
                rc = lib.rtm_render_stripes_async(ctx.handle, C.byref(s_c), C.byref(e_c), C.byref(sh_c), W, H, K,
                                                  flags | c["flags"], 0, S, n, r, C.c_void_p(buf.data_ptr()))
                rtm.abi.check(lib, rc, "rtm_render_stripes_async")
            ev1.record(stream)
            ev1.synchronize()
            return ev0.elapsed_time(ev1) / reps

        for n in (2, 4, 8):
            bands = [time_rows(r0, r1, fused) for (r0, r1) in shard.row_bands(H, n)]
            mean = statistics.fmean(bands)
            entry = {"band_ms": [round(b, 4) for b in bands], "max_over_mean": round(max(bands) / mean, 4),
                     "sum_ms": round(sum(bands), 4)}
            st8 = [time_stripes(n, r, 8, fused) for r in range(n)]
            entry["stripes8_ms"] = [round(b, 4) for b in st8]
            entry["stripes8_max_over_mean"] = round(max(st8) / statistics.fmean(st8), 4)
            if stripes:
                # rank r of n takes stripes r, r+n, ...: its modelled cost is the sum of
                # those stripes' profiled times (launch overhead included per stripe, so
                # only the ratio is meaningful)
                cyc = [sum(stripes[i] for i in range(r, len(stripes), n)) for r in range(n)]
                entry["cyclic8_model_max_over_mean"] = round(max(cyc) / statistics.fmean(cyc), 4)
            res[f"n{n}"] = entry
        out[f"config{cfg}"] = res
        print(json.dumps({f"config{cfg}": res}), flush=True)
    ctx.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
