"""Frames without shadow raster and march (RTM_FLAG_NO_MARCH | NO_SHADOW_RASTER:
main()'s own scene, testscene_raytracingPlane0, main.rs:910-1046) have an all-+INF
shadow viewport.  The library skips their shadow pass and their eye pass
evaluates the +INF texels on demand (rtm_api.cpp trivial_shadow): the image must
stay the oracle's bit for bit, rtm_ctx_shadow_map_texel_bytes reports 0 (no map
stored), and rtm_ctx_shadow_map still returns the all-+INF f64 viewport."""
import ctypes
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _map(ctx, w, h):
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    m = np.empty((h, w), np.float64)
    p = ctx.shadow_map_ptr()
    assert p, "no shadow map"
    assert hip.hipMemcpy(m.ctypes.data, p, w * h * 8, 2) == 0
    return m


def test_single_frame_then_normal_frame(rtm, oracle, scenes):
    import torch
    fl = scenes.RAYTRACING_FLAGS
    eye, sh = scenes.perspective_eye_camera(), scenes.shadow_camera()
    ctx = rtm.Context(0)
    try:
        for (w, h, s) in ((512, 512, scenes.raytracing_plane0()), (333, 97, scenes.raytracing_plane0(True)),
                          (640, 360, scenes.scene_r_bench())):
            out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            ctx.render_async(s, eye, sh, w, h, 0, fl, out.data_ptr())
            ctx.synchronize()
            want = oracle.render(s, eye, sh, w, h, 0, fl, nthreads=NT, want_shadow=True)
            got = out.cpu().numpy()
            assert bits_equal(got, want["rgba"]), first_mismatch(got, want["rgba"])
            assert ctx.shadow_map_texel_bytes() == 0
            m = _map(ctx, w, h)
            assert bits_equal(m, want["shadow"]) and bool(np.isposinf(m).all())
        # a frame with a shadow pass afterwards: its coded map again
        w, h, k = 480, 270, 64
        s = scenes.scene_a_bench(100)
        out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        ctx.render_async(s, scenes.eye_camera(), sh, w, h, k, 0, out.data_ptr())
        ctx.synchronize()
        want = oracle.render(s, scenes.eye_camera(), sh, w, h, k, 0, nthreads=NT, want_shadow=True)
        assert bits_equal(out.cpu().numpy(), want["rgba"])
        assert ctx.shadow_map_texel_bytes() == 1
        assert bits_equal(_map(ctx, w, h), want["shadow"])
    finally:
        ctx.close()


@pytest.mark.parametrize("lanes", [1, 4])
def test_batched_sequence_of_main_scene(rtm, oracle, scenes, lanes):
    """config 7's sequence (64 frames per launch at 512x512 by the auto rule) with
    the scene's planes toggled: every frame == the oracle, the last map all +INF."""
    import torch
    fl = scenes.RAYTRACING_FLAGS
    eye, sh = scenes.perspective_eye_camera(), scenes.shadow_camera()
    w, h = 512, 512
    frames = [scenes.raytracing_plane0(i % 3 == 0) for i in range(96)]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    ctx = rtm.Context(0)
    try:
        ctx.set_lanes(lanes)
        torch.cuda.synchronize()
        ctx.render_frames_async(frames, eye, sh, w, h, 0, fl, [o.data_ptr() for o in outs])
        ctx.synchronize()
        wants = {b: oracle.render(scenes.raytracing_plane0(b), eye, sh, w, h, 0, fl, nthreads=NT)["rgba"]
                 for b in (False, True)}
        for i, o in enumerate(outs):
            assert bits_equal(o.cpu().numpy(), wants[i % 3 == 0]), i
        assert ctx.shadow_map_texel_bytes() == 0
        assert bool(np.isposinf(_map(ctx, w, h)).all())
    finally:
        ctx.close()
