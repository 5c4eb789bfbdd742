#!/usr/bin/env python3
"""In-process A/B timing of kernel variants (interleaved rounds, one process,
cdna_hip_programming.md §5.4 rule 24).  Variants are selected by environment
variables read by librtm at launch, so each variant runs in a child process;
rounds interleave the children.  Prints median/min ms per frame per variant."""
import json
import os
import statistics
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes as C, importlib, json, os, sys, time
sys.path.insert(0, %(root)r)
import torch
torch.cuda.set_device(0)
rtm = importlib.import_module("2018rustraytracer_amd")
sc = importlib.import_module("2018rustraytracer_amd.scenes")
cfg = sc.CONFIGS[%(cfg)d]
W, H, K = cfg["width"], cfg["height"], cfg["steps"]
K = %(steps)d if %(steps)d >= 0 else K
flags = cfg["flags"] | %(flags)d
ctx = rtm.Context(0)
ctx.set_timing_capacity(%(events)d)
lib = rtm.load_library()
scenes = [sc.scene_a_bench(100 + i) if %(cfg)d in (2, 3, 4) else cfg["scene"]() for i in range(%(n)d)]
cs = [s.to_c() for s in scenes]
e, s_ = cfg.get("eye", sc.eye_camera)().to_c(), sc.shadow_camera().to_c()
out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
prep = ctx.prepare_frames(scenes)
def run(n):
    if %(pipe)d:
        ctx.render_frames_async(None, cfg.get("eye", sc.eye_camera)(), sc.shadow_camera(), W, H, K, flags, [out.data_ptr()] * n,
                                (prep[0], prep[1]) if n == len(scenes) else ctx.prepare_frames(scenes[:n]))
        return
    for i in range(n):
        rc = lib.rtm_render_async(ctx.handle, C.byref(cs[i][0]), C.byref(e), C.byref(s_), W, H, K, flags, 0, H,
                                  C.c_void_p(out.data_ptr()))
        assert rc == 0
run(10); torch.cuda.synchronize()
t0 = time.perf_counter(); run(%(n)d); torch.cuda.synchronize(); dt = time.perf_counter() - t0
res = {"ms_per_frame": dt / %(n)d * 1e3}
import hashlib
res["frame_sha"] = hashlib.sha256(out.cpu().numpy().tobytes()).hexdigest()[:12]
if %(events)d:
    sh, ey = ctx.kernel_ms_history(%(n)d + 1)
    res["shadow_ms"] = sum(sh) / len(sh); res["eye_ms"] = sum(ey) / len(ey)
print(json.dumps(res))
'''


def main():
    variants = json.loads(sys.argv[1])  # {"name": {"env": {...}, "flags": 0, "events": 200}}
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    cfg = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    res = {k: [] for k in variants}
    for _ in range(rounds):
        for name, v in variants.items():
            env = dict(os.environ)
            env.update({k: x.replace("__ROOT__", ROOT) for k, x in v.get("env", {}).items()})
            code = CHILD % dict(root=ROOT, cfg=cfg, flags=v.get("flags", 0), events=v.get("events", 200), n=200,
                               steps=v.get("steps", -1), pipe=1 if v.get("pipe") else 0)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(name, "FAILED", p.stderr[-2000:])
                sys.exit(1)
            res[name].append(json.loads(p.stdout.strip().splitlines()[-1]))
    for name, rs in res.items():
        summ = {k: (round(statistics.median(r[k] for r in rs), 5), round(min(r[k] for r in rs), 5))
                for k in rs[0] if k != "frame_sha"}
        summ["frame_sha"] = sorted({r["frame_sha"] for r in rs})
        print(name, json.dumps(summ))


if __name__ == "__main__":
    main()
