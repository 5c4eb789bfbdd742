"""The coded shadow map (rtm_kernels.h): the shadow pass stores
WHICH source won each texel (a march step k, a sphere, or +INF) in 1 or 2 bytes
instead of the 8-byte value, and the eye pass recomputes the value from the code
with the writer's operations.  The image and the decoded map (rtm_ctx_shadow_map)
must equal the oracle's bit for bit in every code width, for the lean tile, the
generic tile (general march), batched and laned sequences -- and equal the f64
map (RTM_SMAP=f64, read once per process, hence the subprocesses)."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes, importlib, sys
import numpy as np, torch
sys.path.insert(0, %(root)r)
sys.path.insert(0, %(root)r + "/oracle")
import oracle
rtm = importlib.import_module("2018rustraytracer_amd")
sc = importlib.import_module("2018rustraytracer_amd.scenes")
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
u = lambda a: np.ascontiguousarray(a).view(np.uint64 if a.dtype == np.float64 else np.uint32)
eye = sc.eye_camera()
ctx = rtm.Context(0)
F64 = %(f64)r

def smap(c, w, h):
    m = np.empty((h, w), np.float64)
    assert hip.hipMemcpy(m.ctypes.data, c.shadow_map_ptr(), w * h * 8, 2) == 0
    return m

# single frames: u8 codes (K=64, 33), u16 codes (K=500, 300 with 16 spheres), the
# generic tile (tilted sun), ragged sizes (partial 128 x 4 blocks)
cases = [(sc.scene_a_bench(100), sc.shadow_camera(), 640, 360, 64),
         (sc.scene_a_bench(130), sc.shadow_camera(), 333, 97, 33),
         (sc.closely_orbiting_sphere(100), sc.shadow_camera(), 512, 512, 500),
         (sc.CONFIGS[5]["scene"](), sc.shadow_camera(), 770, 203, 300),
         (sc.CONFIGS[5]["scene"](), sc.shadow_camera(), 257, 130, 240),
         (sc.scene_b(), sc.tilted_shadow_camera(), 400, 240, 128),
         (sc.scene_a_bench(100), sc.tilted_shadow_camera(), 129, 5, 600)]
for s, shc, w, h, k in cases:
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.render_async(s, eye, shc, w, h, k, 0, out.data_ptr())
    ctx.synchronize()
    expect = 8 if F64 else (1 if k + len(s.spherePrimitives) <= 254 else 2)
    assert ctx.shadow_map_texel_bytes() == expect, (ctx.shadow_map_texel_bytes(), expect, k)
    want = oracle.render(s, eye, shc, w, h, k, 0, nthreads=8, want_shadow=True)
    assert np.array_equal(u(out.cpu().numpy()), u(want["rgba"])), (w, h, k)
    assert np.array_equal(u(smap(ctx, w, h)), u(want["shadow"])), ("map", w, h, k)
# a sequence: batched (4 frames per launch) on 2 lanes, then the last frame's map
w, h, k = 480, 270, 64
frames = [sc.scene_a_bench(100 + 7 * i) for i in range(9)]
outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
ctx.set_batch(4)
ctx.set_lanes(2)
torch.cuda.synchronize()
ctx.render_frames_async(frames, eye, sc.shadow_camera(), w, h, k, 0, [o.data_ptr() for o in outs])
ctx.synchronize()
for s, o in zip(frames, outs):
    want = oracle.render(s, eye, sc.shadow_camera(), w, h, k, 0, nthreads=8, want_shadow=True)
    assert np.array_equal(u(o.cpu().numpy()), u(want["rgba"]))
assert np.array_equal(u(smap(ctx, w, h)), u(want["shadow"]))
print("smap ok")
'''


@pytest.mark.gpu
@pytest.mark.parametrize("fmt", ["coded", "f64"])
def test_shadow_map_formats_in_subprocess(fmt):
    env = dict(os.environ)
    env.pop("RTM_SMAP", None)
    if fmt == "f64":
        env["RTM_SMAP"] = "f64"
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT, "f64": fmt == "f64"}], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0 and "smap ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
