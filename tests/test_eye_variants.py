"""Every eye-pass instantiation the library dispatches (rtm_kernels.hip
launch_eye_fmt), each against the oracle: scene kind (spheres only; ray-traced
primitives under an ORTHOGONAL eye; under a PERSPECTIVE eye, with its per-wave
primitive masks; PERSPECTIVE spheres; SDFs) x shadow viewport (materialised coded
map; fused on-demand texels; no march and no raster, i.e. no shadow lookup) x output format (RGBA f32,
writeColorImage's RGBA8 / RGB8 bytes) x one frame per launch / a batched launch.
Frames are small; the point is that no dispatched variant goes untested."""
import os

import numpy as np
import pytest

from test_formats_group import want_frame, to_host

pytestmark = pytest.mark.gpu

KINDS = ["spheres", "rt_ortho", "rt_persp", "persp_spheres", "sdf_ortho", "sdf_persp"]
SHADOWS = ["map", "fused", "trivial"]


def _kind(scenes, kind):
    if kind == "spheres":
        return scenes.scene_a_bench(100), scenes.eye_camera()
    if kind == "rt_ortho":
        return scenes.mixed_rt(100), scenes.eye_camera()
    if kind == "rt_persp":
        return scenes.scene_r_bench(), scenes.perspective_eye_camera()
    if kind == "persp_spheres":
        return scenes.perspective_simple1(), scenes.perspective_eye_camera()
    if kind == "sdf_ortho":
        return scenes.mixed_sdf(100), scenes.eye_camera()
    if kind == "sdf_persp":
        return scenes.sdf_bench_scene(), scenes.sdf_eye_camera()
    raise ValueError(kind)


def _flags(rtm, shadow):
    return {"map": 0, "fused": rtm.abi.RTM_FLAG_FUSED_SHADOW,
            "trivial": rtm.abi.RTM_FLAG_NO_MARCH | rtm.abi.RTM_FLAG_NO_SHADOW_RASTER}[shadow]


@pytest.mark.parametrize("fmt", [0, 1, 2], ids=["rgba32f", "rgba8", "rgb8"])
@pytest.mark.parametrize("shadow", SHADOWS)
@pytest.mark.parametrize("kind", KINDS)
def test_eye_variant_single_and_batched(rtm, oracle, scenes, gpu_ctx, kind, shadow, fmt):
    import torch
    s, eye = _kind(scenes, kind)
    flags = _flags(rtm, shadow)
    w, h, k = 192, 132, 16
    want = want_frame(oracle, s, eye, scenes.shadow_camera(), w, h, k, flags, fmt, rtm.abi)
    nb = rtm.abi.FORMAT_BYTES[fmt]
    # one frame per launch
    out = torch.empty(h * w * nb, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.render_rows_async(s, eye, scenes.shadow_camera(), w, h, k, flags, fmt, out.data_ptr(), 0, h)
    gpu_ctx.synchronize()
    got = out.cpu().numpy().reshape(h, w, nb if fmt else 16).view(np.uint8)
    assert np.array_equal(got.reshape(-1), want.view(np.uint8).reshape(-1)), "single"
    # three frames in one batched launch per pass (a one-member group renders in place
    # through the library's batched path, in any output format)
    g = rtm.Group(n_devices=1, loopback=True)
    try:
        outs = [torch.empty(h * w * nb, dtype=torch.uint8, device="cuda") for _ in range(3)]
        torch.cuda.synchronize()
        g.render_frames_async([s] * 3, eye, scenes.shadow_camera(), w, h, k, flags, fmt, 0, [o.data_ptr() for o in outs])
        g.synchronize(60000)
        wb = want.view(np.uint8).reshape(h, w, -1)
        for i, o in enumerate(outs):
            gb = o.cpu().numpy().reshape(h, w, -1)
            bad = np.argwhere(np.any(gb != wb, axis=-1))
            assert bad.size == 0, (f"batched frame {i}: {len(bad)} pixels differ, first (y, x) {tuple(bad[0])}, "
                                   f"rows {bad[:, 0].min()}..{bad[:, 0].max()}: got {gb[tuple(bad[0])]} "
                                   f"want {wb[tuple(bad[0])]}")
    finally:
        g.close()
