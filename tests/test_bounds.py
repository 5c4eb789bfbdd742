"""Pinning the round-3 GPU fault: the RT 3 eye tile (PERSPECTIVE eye
with ray-traced primitives) read its wave's primitive-mask word for tile rows past
the launch's part, i.e. up to 3 rows of words past the mask scratch when
rows % 4 != 0 (main.rs:569-642 is the pass; the masks are this port's cull).  Such
a read faults only when the scratch happens to end at an unmapped page, so a green
suite said nothing about it.

The library now checks every read of its host-built side tables (the per-wave
primitive masks, the coded shadow tile's row records) against the table's exact
length and counts, instead of performing, an out-of-range one
(rtm_ctx_oob_reads).  These tests drive the patterns that over-read -- a PERSPECTIVE
eye with primitives through the single-frame (rtm_render_rows_async, row parts with
rows % 4 in {1, 2, 3}), batched (rtm_render_frames_async) and striped paths, on both
the materialised-map and the all-+INF (trivial) shadow viewports, and row counts
that are no multiple of 64 for the row records -- and require the count to stay 0
and the image to equal the oracle's.  Built with the round-3 guard reverted
(tools/bounds_demo.sh: -DRTM_TEST_REVERT_MASK_GUARD), the same tests fail with a
nonzero count: the check sees exactly the old over-read, deterministically, without
the fault."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def oob(rtm, ctx):
    import ctypes as C
    lib = rtm.load_library()
    n = C.c_int64(-1)
    rtm.abi.check(lib, lib.rtm_ctx_oob_reads(ctx.handle, C.byref(n)), "rtm_ctx_oob_reads")
    return n.value


def _case(scenes, kind):
    if kind == "trivial":  # main()'s flags: no shadow raster, no march (the eye kernel without a lookup)
        return scenes.scene_r_bench(), scenes.perspective_eye_camera(), scenes.RAYTRACING_FLAGS, 0
    return scenes.scene_r_bench(), scenes.perspective_eye_camera(), 0, 16  # a materialised map (coded)


@pytest.mark.parametrize("kind", ["trivial", "map"])
@pytest.mark.parametrize("rows", [1025, 1026, 1027])
def test_rt_mask_rows_past_the_part_single_frame(rtm, oracle, scenes, gpu_ctx, kind, rows):
    """A row part of 2048 x rows (>= 1 Mpixel: the separate mask kernel and scratch),
    rows % 4 = 1, 2, 3: no out-of-range mask read, the oracle's rows."""
    import torch
    s, eye, flags, k = _case(scenes, kind)
    w, h, r0 = 2048, 1200, 101
    assert oob(rtm, gpu_ctx) >= 0  # clear
    out = torch.empty((rows, w, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.render_rows_async(s, eye, scenes.shadow_camera(), w, h, k, flags, 0, out.data_ptr(), r0, r0 + rows)
    gpu_ctx.synchronize()
    assert oob(rtm, gpu_ctx) == 0
    want = oracle.render(s, eye, scenes.shadow_camera(), w, h, k, flags, nthreads=NT)["rgba"][r0:r0 + rows]
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("kind", ["trivial", "map"])
def test_rt_mask_rows_past_the_part_batched(rtm, oracle, scenes, gpu_ctx, kind):
    """Frames of 640 x 483 rows (483 % 4 = 3, and 483 % 64 != 0 for the row records) in
    one batched launch per pass (every batched RT 3 frame carries masks)."""
    import torch
    s, eye, flags, k = _case(scenes, kind)
    w, h = 640, 483
    frames = [s] * 6
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    assert oob(rtm, gpu_ctx) >= 0
    try:
        gpu_ctx.set_batch(3)
        gpu_ctx.set_lanes(2)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, scenes.shadow_camera(), w, h, k, flags, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
        assert gpu_ctx.last_batch() == 3
    finally:
        gpu_ctx.set_batch(0)
        gpu_ctx.set_lanes(0)
    assert oob(rtm, gpu_ctx) == 0
    want = oracle.render(s, eye, scenes.shadow_camera(), w, h, k, flags, nthreads=NT)["rgba"]
    for o in outs:
        assert np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("n,S", [(3, 8), (5, 3)])
def test_rt_mask_rows_past_the_part_stripes(rtm, oracle, scenes, gpu_ctx, n, S):
    """Every part of a striped frame (the multi-GPU partition's rows, fused shadow):
    part row counts that are no multiple of 4."""
    import torch
    shard = __import__("importlib").import_module("2018rustraytracer_amd.shard")
    s, eye = scenes.scene_r_bench(), scenes.perspective_eye_camera()
    w, h, k = 2048, 1547, 16
    fl = rtm.abi.RTM_FLAG_FUSED_SHADOW
    want = oracle.render(s, eye, scenes.shadow_camera(), w, h, k, fl, nthreads=NT)["rgba"]
    assert oob(rtm, gpu_ctx) >= 0
    for r in range(n):
        rows = shard.stripe_rows_of(h, n, S, r)
        out = torch.empty((rows, w, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.render_stripes_async(s, eye, scenes.shadow_camera(), w, h, k, fl, 0, S, n, r, out.data_ptr())
        gpu_ctx.synchronize()
        assert oob(rtm, gpu_ctx) == 0, r
        assert np.array_equal(out.cpu().numpy().view(np.uint32),
                              want[shard.stripe_image_rows(h, n, S, r)].view(np.uint32)), r


@pytest.mark.parametrize("h", [97, 1027, 2161])
def test_coded_row_records_in_range(rtm, oracle, scenes, gpu_ctx, h):
    """The coded shadow tile's row records for heights that are no multiple of 64: the
    map (decoded) and the image equal the oracle's, no out-of-range record read."""
    import ctypes as C
    import torch
    w, k = 1000, 64
    s = scenes.scene_a_bench(100)
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    assert oob(rtm, gpu_ctx) >= 0
    torch.cuda.synchronize()
    gpu_ctx.render_async(s, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0, out.data_ptr())
    gpu_ctx.synchronize()
    assert gpu_ctx.shadow_map_texel_bytes() == 1
    assert oob(rtm, gpu_ctx) == 0
    want = oracle.render(s, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0, nthreads=NT, want_shadow=True)
    assert np.array_equal(out.cpu().numpy().view(np.uint32), want["rgba"].view(np.uint32))
    m = np.empty((h, w), np.float64)
    hip = C.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    assert hip.hipMemcpy(m.ctypes.data, gpu_ctx.shadow_map_ptr(), h * w * 8, 2) == 0
    assert np.array_equal(m.view(np.uint64), want["shadow"].view(np.uint64))
