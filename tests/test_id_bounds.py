"""The round-4 GPU fault study: frames shaped like
the one that faulted -- tests/golden f3_persp2_rt_640x360, perspectiveSimple2's
spheres under the PERSPECTIVE eye plus one circle plane and one capped cylinder,
flags 3 (no march, no shadow raster: the all-+INF viewport, no map decode) -- and
their neighbours, through every path that walks the per-wave primitive masks and
shades by a hit's scene id (processRaytracingRays, main.rs:569-642; renderColorImage
indexes the scene's primitives by id, main.rs:748, 773, 791):

  * single frames below 1 Mpixel (the in-kernel wave cull, rt_wave_mask) and above
    (the separate mask kernel, rt_cull_kernel);
  * batched frames (rt_cull_batch_kernel), 1-4 primitives of each kind;
  * the ORTHOGONAL eye (every existing slot, rt_slots) and the staged seam
    (vp_trace_kernel).

Every mask a producer builds must carry only the frame's existing slots, and every
id-indexed table read must stay in its table: the kernels check both and count a
violation in rtm_ctx_oob_reads (trace_pixel's slot check, wave_sphere_mask_ids,
checked_id, the staged shade's G-buffer id check).  Each test requires 0 and the
oracle's bits.  Built with the pre-dfafeba masks restored (every slot bit set:
tools/bounds_demo.sh slots, -DRTM_TEST_REVERT_SLOT_MASKS) the same tests fail with a
nonzero count -- the tree the round-4 fault ran on combined those masks with the
set-bit walk."""
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch
from test_bounds import oob

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _persp2_rt(scenes, n_pl=1, n_cy=1):
    """f3_persp2_rt's scene (tests/test_raytrace.py _case) with n_pl planes and n_cy
    cylinders (copies of the reference's, shifted, ids reversed)."""
    s = scenes.perspective_simple2()
    pl, cy = scenes.REFERENCE_CIRCLE_PLANE, scenes.REFERENCE_CAPPED_CYLINDER
    s.circlePlanePrimitives = [
        scenes.dataclasses.replace(pl, id=n_pl - 1 - i, pos=(pl.pos[0] + 0.3 * i, pl.pos[1] - 0.2 * i, pl.pos[2]))
        for i in range(n_pl)]
    s.cappedCylinderPrimitives = [
        scenes.dataclasses.replace(cy, id=n_cy - 1 - i, pA=(cy.pA[0] + 0.5 * i, cy.pA[1], cy.pA[2]),
                                   pB=(cy.pB[0] + 0.5 * i, cy.pB[1], cy.pB[2]))
        for i in range(n_cy)]
    return s


@pytest.mark.parametrize("flags", [3, 0])
@pytest.mark.parametrize("wh", [(640, 360), (2048, 600)], ids=["in-kernel-cull", "mask-kernel"])
@pytest.mark.parametrize("prims", [(1, 1), (0, 2), (3, 0), (4, 4)])
def test_persp2_rt_frames(rtm, oracle, scenes, gpu_ctx, flags, wh, prims):
    """rtm_render (the call that faulted: its D2H copy reported the fault) on
    f3_persp2_rt-shaped frames: no out-of-range read, the oracle's bits."""
    w, h = wh
    s = _persp2_rt(scenes, *prims)
    eye, sh = scenes.perspective_simple2_camera(), scenes.shadow_camera()
    k = 0 if flags == 3 else 16
    assert oob(rtm, gpu_ctx) >= 0  # clear
    got = rtm.render_frame(s, eye, sh, w, h, k, flags)
    assert oob(rtm, gpu_ctx) == 0
    want = oracle.render(s, eye, sh, w, h, k, flags, nthreads=NT)["rgba"]
    assert bits_equal(got, want), first_mismatch(got, want)


@pytest.mark.parametrize("flags", [3, 0])
def test_persp2_rt_batched(rtm, oracle, scenes, gpu_ctx, flags):
    """Batched launches (every batched PERSPECTIVE frame with primitives carries masks)."""
    import torch
    w, h = 640, 360
    eye, sh = scenes.perspective_simple2_camera(), scenes.shadow_camera()
    k = 0 if flags == 3 else 16
    frames = [_persp2_rt(scenes, 1 + i % 4, (i * 3) % 5) for i in range(8)]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    assert oob(rtm, gpu_ctx) >= 0
    try:
        gpu_ctx.set_batch(4)
        gpu_ctx.set_lanes(2)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, sh, w, h, k, flags, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
    finally:
        gpu_ctx.set_batch(0)
        gpu_ctx.set_lanes(0)
    assert oob(rtm, gpu_ctx) == 0
    for f, o in zip(frames, outs):
        want = oracle.render(f, eye, sh, w, h, k, flags, nthreads=NT)["rgba"]
        got = o.cpu().numpy()
        assert bits_equal(got, want), first_mismatch(got, want)


def test_orthographic_eye_and_staged_seam(rtm, oracle, scenes, gpu_ctx):
    """The ORTHOGONAL eye (masks of every existing slot) and the staged
    processRaytracingRays + renderColorImage (vp_trace_kernel / vp_shade_kernel)."""
    w, h = 320, 200
    s = scenes.mixed_rt(100)
    eye, shc = scenes.eye_camera(), scenes.shadow_camera()
    assert oob(rtm, gpu_ctx) >= 0
    got = rtm.render_frame(s, eye, shc, w, h, 16, 0)
    assert oob(rtm, gpu_ctx) == 0
    want = oracle.render(s, eye, shc, w, h, 16, 0, nthreads=NT)["rgba"]
    assert bits_equal(got, want), first_mismatch(got, want)
    vp1 = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.BACK, shc)
    vp1.rasterize(s)
    vp1.processRaymarchingRays(s.patches, 16)
    vp0 = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.FRONT, eye)
    vp0.rasterize(s)
    vp0.processRaytracingRays(s)
    img = rtm.renderColorImage(s, vp0, vp1)
    assert oob(rtm, gpu_ctx) == 0
    assert bits_equal(img, want), first_mismatch(img, want)
