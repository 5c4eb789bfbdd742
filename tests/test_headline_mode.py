"""The bench's exact execution modes pinned directly to the CPU oracle.

bench.py's headline renders Scene A-bench animation frames 100+i at 3840x2160,
K = 64 (BASELINE config 3; the reference's frame loop main.rs:1469-1633) through
ONE rtm_render_frames_async call with the library's auto rules: 4 lanes (streams
with their own shadow maps) x 8 frames per launch (batched kernels, one pulled
frame table per launch) and the 1-byte coded shadow map.  These tests run that
same call shape and compare every frame, and the last frame's shadow map,
with oracle.render bit for bit -- not with the library's own single-frame path.
The 8K configs (4, 5) run on 3 lanes x 2 frames per launch.
"""
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _smap(ctx, w, h):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    m = np.empty((h, w), np.float64)
    p = ctx.shadow_map_ptr()
    assert p, "no shadow map"
    assert hip.hipMemcpy(m.ctypes.data, p, w * h * 8, 2) == 0
    return m


def _sequence_vs_oracle(rtm, oracle, scenes, frames, w, h, k, lanes, batch, map_bytes):
    """Render `frames` in one auto-ruled sequence call on a fresh context and
    compare every frame and the last shadow map with the oracle."""
    import torch
    ctx = rtm.Context(0)
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    try:
        torch.cuda.synchronize()
        ctx.render_frames_async(frames, eye, sh, w, h, k, 0, [o.data_ptr() for o in outs])
        ctx.synchronize()
        assert ctx.last_lanes() == lanes, ctx.last_lanes()
        assert ctx.last_batch() == batch, ctx.last_batch()
        assert ctx.shadow_map_texel_bytes() == map_bytes
        for i, (s, o) in enumerate(zip(frames, outs)):
            want = oracle.render(s, eye, sh, w, h, k, 0, nthreads=NT,
                                 want_shadow=(i == len(frames) - 1))
            got = o.cpu().numpy()
            assert bits_equal(got, want["rgba"]), (i, first_mismatch(got, want["rgba"]))
        got_map = _smap(ctx, w, h)
        assert bits_equal(got_map, want["shadow"]), first_mismatch(got_map, want["shadow"])
    finally:
        del outs
        ctx.close()
        torch.cuda.empty_cache()


def test_headline_sequence_4k_four_lanes_eight_per_launch(rtm, oracle, scenes):
    """bench.py config 3 as timed: 32 frames (one bench step), auto 4 lanes x 8
    frames per launch; batch b of 4 runs on lane 3 - b, so every lane's shadow
    maps and table ring are exercised; the coded 1-B map."""
    frames = [scenes.scene_a_bench(100 + i) for i in range(32)]
    _sequence_vs_oracle(rtm, oracle, scenes, frames, 3840, 2160, 64, lanes=4, batch=8, map_bytes=1)


@pytest.mark.parametrize("cfg", [4, 5])
def test_8k_sequence_three_lanes_batched(rtm, oracle, scenes, cfg):
    """Configs 4 / 5 under the auto rule from 16 Mpixel: 3 lanes x 2 frames per
    launch (6 frames: three batches, one per lane)."""
    c = scenes.CONFIGS[cfg]
    if cfg == 4:
        frames = [scenes.scene_a_bench(100 + 3 * i) for i in range(6)]
    else:
        frames = [c["scene"]() for _ in range(6)]
    _sequence_vs_oracle(rtm, oracle, scenes, frames, c["width"], c["height"], c["steps"], lanes=3, batch=2,
                        map_bytes=1)


def test_batched_mixed_sphere_counts_pick_the_widest_code(rtm, oracle, scenes):
    """A launch's coded-map width must hold every frame's codes:
    K = 240 with a 0-sphere frame first (240 codes: fits a byte) and 16-sphere
    frames after it (256 codes: needs 2 bytes).  Same patches, so the frames
    share one launch; every frame and the last map == the oracle."""
    import torch
    sb = scenes.scene_b()
    bare = scenes.Scene([], list(sb.patches))
    frames = [bare, sb, bare, sb]
    w, h, k = 384, 232, 240
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    ctx = rtm.Context(0)
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    try:
        ctx.set_batch(4)
        ctx.set_lanes(1)
        torch.cuda.synchronize()
        ctx.render_frames_async(frames, eye, sh, w, h, k, 0, [o.data_ptr() for o in outs])
        ctx.synchronize()
        assert ctx.last_batch() == 4
        assert ctx.shadow_map_texel_bytes() == 2
        for i, (s, o) in enumerate(zip(frames, outs)):
            want = oracle.render(s, eye, sh, w, h, k, 0, nthreads=NT, want_shadow=True)
            got = o.cpu().numpy()
            assert bits_equal(got, want["rgba"]), (i, first_mismatch(got, want["rgba"]))
        assert bits_equal(_smap(ctx, w, h), want["shadow"])
        # the 16-sphere frame first, the bare one last: the decoded last map is the bare frame's
        ctx.render_frames_async(frames[::-1], eye, sh, w, h, k, 0, [o.data_ptr() for o in outs])
        ctx.synchronize()
        want = oracle.render(bare, eye, sh, w, h, k, 0, nthreads=NT, want_shadow=True)
        assert bits_equal(_smap(ctx, w, h), want["shadow"])
        for s, o in zip(frames[::-1], outs):
            assert bits_equal(o.cpu().numpy(), oracle.render(s, eye, sh, w, h, k, 0, nthreads=NT)["rgba"])
    finally:
        ctx.close()
