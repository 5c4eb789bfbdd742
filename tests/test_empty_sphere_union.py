"""A shadow viewport that rasterizes (no RTM_FLAG_NO_SHADOW_RASTER) but whose
spheres cover nothing -- an empty union of sphere pixel ranges -- must still get
every texel of its map written.  Round 4 found the split shadow launch leaving
the top-left 128 x 16 texels unwritten there: the empty union (1, 0, 1, 0) "met"
any strip spanning row 0 and column 0, so the raster-free part left that strip
to the sphere part, which an empty union never launches.  The map then held
whatever the buffer held before.  These tests make "before" a frame whose big
sphere covers the whole map (so a stale texel is a finite depth, not +INF) and
compare the next, sphere-free frame's decoded map with the oracle's all-+INF map
-- one frame per launch and batched."""
import ctypes
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch
from test_bounds import oob

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _smap(ctx, w, h):
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    m = np.empty((h, w), np.float64)
    p = ctx.shadow_map_ptr()
    assert p, "no shadow map"
    assert hip.hipMemcpy(m.ctypes.data, p, w * h * 8, 2) == 0
    return m


def _scenes(scenes):
    big = scenes.Scene([scenes.PrimitiveSphere(0, scenes.Shading(0.5, 0.5, 0.5), (0.0, 0.0, 2.0), 3.0)], [])
    return big, scenes.Scene([], [])


@pytest.mark.parametrize("w,h", [(256, 100), (384, 64)])
@pytest.mark.parametrize("batched", [False, True], ids=["single", "batched"])
def test_sphere_free_frame_writes_every_texel(rtm, oracle, scenes, w, h, batched):
    import torch
    big, empty = _scenes(scenes)
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    k = 8
    want_big = oracle.render(big, eye, sh, w, h, k, 0, nthreads=NT, want_shadow=True)["shadow"]
    assert np.isfinite(want_big[:16, :128]).all()  # (the stale texels would be finite)
    want = oracle.render(empty, eye, sh, w, h, k, 0, nthreads=NT, want_shadow=True)
    assert np.isinf(want["shadow"]).all()
    ctx = rtm.Context(0)
    n = 2 if batched else 1
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(n)]
    try:
        torch.cuda.synchronize()
        assert oob(rtm, ctx) >= 0  # (clears the device-wide count)
        for s in (big, empty):
            if batched:
                ctx.render_frames_async([s] * n, eye, sh, w, h, k, 0, [o.data_ptr() for o in outs])
            else:
                ctx.render_async(s, eye, sh, w, h, k, 0, outs[0].data_ptr())
            ctx.synchronize()
        if batched:
            assert ctx.last_batch() == n, ctx.last_batch()
        got = _smap(ctx, w, h)
        assert bits_equal(got, want["shadow"]), first_mismatch(got, want["shadow"])
        assert oob(rtm, ctx) == 0  # no decode met a code outside the frame's spheres
        for o in outs:
            g = o.cpu().numpy()
            assert bits_equal(g, want["rgba"]), first_mismatch(g, want["rgba"])
    finally:
        del outs
        ctx.close()
