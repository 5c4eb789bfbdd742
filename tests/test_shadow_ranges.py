"""The coded shadow tile's sphere raster by depth ranges (rtm_kernels.hip,
shadow_tile_coded): a covered texel's BACK-face depth lies in [z, z + r]
(main.rs:236-246), coverage is s2 < 1, so with pairwise-disjoint ranges the nearest
covering sphere and the march's verdict against it need no square root unless the
march t falls inside the winner's range.  These frames drive each branch -- decided
by the range (scene A), t inside the range (a flat patch at the spheres' depth:
every covered texel takes the exact depth), overlapping ranges (spheres at equal
depth, spheres nested in depth), no march (t = +INF) -- in the split and the
single launch, and must equal the oracle's frame and shadow map bit for bit."""
import ctypes as C
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _scene(scenes, kind):
    S, L, B = scenes.PrimitiveSphere, scenes.Linear, scenes.Bilinear
    col = scenes.Shading(0.9, 0.2, 0.2)
    if kind == "inside":  # a flat patch at depth 0.6: t ~ 0.6 inside sphere 0's range [0.5, 0.7]
        s = scenes.scene_a_bench(100)
        s.patches = [B(L(0.6, 0.6), L(0.6, 0.6))]
        return s, 0
    if kind == "inside_tilted":  # t sweeps through both spheres' ranges across the frame
        s = scenes.scene_a_bench(100)
        s.patches = [B(L(0.3, 1.3), L(0.5, 1.5))]
        return s, 0
    if kind == "equal_depth":  # two spheres at the same depth: overlapping ranges
        return scenes.Scene([S(0, col, (0.0, 0.0, 0.5), 0.2), S(1, col, (0.15, 0.1, 0.5), 0.2),
                             S(2, col, (-0.3, -0.2, 0.9), 0.1)], [scenes.BENCH_PATCH]), 0
    if kind == "nested":  # one range inside another (big far sphere, small near one)
        return scenes.Scene([S(0, col, (0.0, 0.0, 0.6), 0.4), S(1, col, (0.05, 0.0, 0.7), 0.1)],
                            [scenes.BENCH_PATCH]), 0
    if kind == "no_march":
        return scenes.scene_a_bench(100), scenes.abi.RTM_FLAG_NO_MARCH
    if kind == "negative_radius":  # r < 0: the range's ends swap
        return scenes.Scene([S(0, col, (0.0, 0.0, 0.9), -0.2), S(1, col, (0.3, 0.0, 0.3), 0.1)],
                            [scenes.BENCH_PATCH]), 0
    raise ValueError(kind)


@pytest.mark.parametrize("split", ["split", "single"])
@pytest.mark.parametrize("kind", ["inside", "inside_tilted", "equal_depth", "nested", "no_march", "negative_radius"])
def test_sphere_ranges_match_oracle(rtm, oracle, scenes, split, kind):
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import ctypes as C, importlib, sys
import numpy as np, torch
sys.path.insert(0, %(root)r); sys.path.insert(0, %(root)r + "/tests"); sys.path.insert(0, %(root)r + "/oracle")
import oracle
from test_shadow_ranges import _scene
rtm = importlib.import_module("2018rustraytracer_amd")
sc = importlib.import_module("2018rustraytracer_amd.scenes")
s, flags = _scene(sc, %(kind)r)
ctx = rtm.Context(0)
hip = C.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
for w, h, k in ((1024, 768, 64), (901, 333, 40)):
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    ctx.render_async(s, sc.eye_camera(), sc.shadow_camera(), w, h, k, flags, out.data_ptr())
    ctx.synchronize()
    want = oracle.render(s, sc.eye_camera(), sc.shadow_camera(), w, h, k, flags, nthreads=%(nt)d, want_shadow=True)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want["rgba"].view(np.uint32)), (w, h)
    m = np.empty((h, w), np.float64)
    assert hip.hipMemcpy(m.ctypes.data, ctx.shadow_map_ptr(), h * w * 8, 2) == 0
    assert np.array_equal(m.view(np.uint64), want["shadow"].view(np.uint64)), ("map", w, h)
print("ranges ok")
''' % {"root": root, "kind": kind, "nt": NT}
    env = dict(os.environ)
    # the split launch for any sphere box (RTM_CODED_SPLIT_MAX=1) or never (0)
    env["RTM_CODED_SPLIT_MAX"] = "1.0" if split == "split" else "-1"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "ranges ok" in r.stdout, r.stdout[-3000:] + r.stderr[-3000:]
