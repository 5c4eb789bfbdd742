"""The batched eye pass in 8 x 8 pixel blocks (rtm_kernels.hip `eye_block_mode`,
`eye_tile<BLK>`, `ray_cone_block`): small ray-traced frames without shadows and SDF
frames, at sizes that leave partial blocks and partial workgroups (W not a multiple of
32, rows not a multiple of 8 where the block count still fits the mask slot), frames
without primitives and with perspective spheres in the same batch, 4 block rows per
workgroup past the frame's last block row.  Every frame against the oracle, bit for
bit, with no out-of-range table read."""
import os

import numpy as np
import pytest

from conftest import bits_equal, device_smap, first_mismatch
from test_bounds import oob

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _thin_cylinders(scenes, seed):
    rng = np.random.default_rng(0x2018 + 500 + seed)
    S, C, P = scenes.Shading, scenes.PrimitiveCappedCylinder, scenes.PrimitiveCirclePlane
    cyls, planes = [], []
    for i in range(6):
        z = float(rng.uniform(2.0, 12.0))
        a = (float(rng.uniform(-1.0, 1.0) * z), float(rng.uniform(-1.0, 1.0) * z), z)
        d = rng.normal(size=3)
        d *= rng.uniform(1.0, 8.0) / np.linalg.norm(d)
        b = (a[0] + float(d[0]), a[1] + float(d[1]), a[2] + float(d[2]))
        cyls.append(C(i, S(*(float(v) for v in rng.uniform(0.05, 1.0, 3))), a, b,
                      float(rng.uniform(0.01, 0.2)), float(rng.uniform(0.01, 0.2))))
    for i in range(2):
        z = float(rng.uniform(3.0, 10.0))
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        planes.append(P(i, S(0.3, 0.6, 0.9), float(rng.uniform(0.2, 1.0)),
                        (float(rng.uniform(-0.8, 0.8) * z), float(rng.uniform(-0.8, 0.8) * z), z),
                        tuple(float(v) for v in n)))
    return scenes.Scene([], [], planes, cyls)


@pytest.mark.parametrize("w,h", [(200, 136), (517, 96), (640, 360), (72, 8)])
def test_block_mode_ray_traced_batches(rtm, oracle, scenes, gpu_ctx, w, h):
    import torch
    eye, sh = scenes.perspective_eye_camera(), scenes.shadow_camera()
    frames = [_thin_cylinders(scenes, 0), scenes.raytracing_plane0(), scenes.perspective_simple1(),
              _thin_cylinders(scenes, 1), scenes.raytracing_plane0(True), _thin_cylinders(scenes, 2)]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    assert oob(rtm, gpu_ctx) >= 0  # clear
    try:
        gpu_ctx.set_batch(len(frames))
        gpu_ctx.set_lanes(1)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, sh, w, h, 0, scenes.RAYTRACING_FLAGS, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
    finally:
        gpu_ctx.set_lanes(0)
        gpu_ctx.set_batch(0)
    # the batch really ran the 8 x 8 kernels (rtm_ctx_last_eye_blocks), not the 64 x 1 rows
    assert gpu_ctx.last_eye_blocks()
    assert oob(rtm, gpu_ctx) == 0
    for i, (s, o) in enumerate(zip(frames, outs)):
        want = oracle.render(s, eye, sh, w, h, 0, scenes.RAYTRACING_FLAGS, nthreads=NT)["rgba"]
        got = o.cpu().numpy()
        assert bits_equal(got, want), f"frame {i}: {first_mismatch(got, want)}"


@pytest.mark.parametrize("w,h", [(200, 136), (96, 72)])
def test_block_mode_sdf_batches(rtm, oracle, scenes, gpu_ctx, w, h):
    import torch
    eye, sh = scenes.sdf_eye_camera(), scenes.shadow_camera()
    frames = [scenes.sdf_preview_scene(), scenes.sdf_bench_scene(), scenes.sdf_preview_scene()]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    assert oob(rtm, gpu_ctx) >= 0
    try:
        gpu_ctx.set_batch(len(frames))
        gpu_ctx.set_lanes(1)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, sh, w, h, 0, scenes.RAYTRACING_FLAGS, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
    finally:
        gpu_ctx.set_lanes(0)
        gpu_ctx.set_batch(0)
    assert gpu_ctx.last_eye_blocks()
    assert oob(rtm, gpu_ctx) == 0
    for i, (s, o) in enumerate(zip(frames, outs)):
        want = oracle.render(s, eye, sh, w, h, 0, scenes.RAYTRACING_FLAGS, nthreads=NT)["rgba"]
        got = o.cpu().numpy()
        assert bits_equal(got, want), f"frame {i}: {first_mismatch(got, want)}"


@pytest.mark.parametrize("w,h", [(200, 136), (136, 200)])
def test_block_mode_shadowed_sdf_batches(rtm, oracle, scenes, gpu_ctx, w, h):
    """Shadowed, non-fused SDF batches (flags 0, march steps > 0: the materialised coded
    map, decoded by the SDF block kernel's lookups) at sizes with partial blocks and
    workgroups: the SDF beside Scene A-bench's spheres and patch, under the
    orthographic eye, with the sun's map; every frame and the last map == the oracle."""
    import torch
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    frames = [scenes.mixed_sdf(100 + 7 * i) for i in range(4)]
    k = 64
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    assert oob(rtm, gpu_ctx) >= 0
    try:
        gpu_ctx.set_batch(len(frames))
        gpu_ctx.set_lanes(1)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, sh, w, h, k, 0, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
    finally:
        gpu_ctx.set_lanes(0)
        gpu_ctx.set_batch(0)
    assert gpu_ctx.last_batch() == len(frames) and gpu_ctx.last_eye_blocks()
    assert gpu_ctx.shadow_map_texel_bytes() == 1
    assert oob(rtm, gpu_ctx) == 0
    for i, (s, o) in enumerate(zip(frames, outs)):
        want = oracle.render(s, eye, sh, w, h, k, 0, nthreads=NT, want_shadow=i == len(frames) - 1)
        got = o.cpu().numpy()
        assert bits_equal(got, want["rgba"]), f"frame {i}: {first_mismatch(got, want['rgba'])}"
    m = device_smap(gpu_ctx, w, h)
    assert bits_equal(m, want["shadow"]), first_mismatch(m, want["shadow"])


@pytest.mark.parametrize("w,h", [(200, 136), (1280, 832)])
def test_shared_primitive_masks(rtm, oracle, scenes, gpu_ctx, w, h):
    """A batch whose frames all hold frame 0's primitive table shares frame 0's masks (one
    frame's cull, rtm_api.cpp enqueue_batch), and a lane whose last shared cull had the same
    table, camera and sizes reuses its words without culling again; one differing frame
    anywhere in the batch makes every frame cull its own (and drops the lane's shared words).
    Blocks (200 x 136) and rows (1280 x 832, above 1 Mpixel) on one context: shared, shared
    again (reuse), unshared, another table shared twice, the first table again, then the
    first table under a moved camera (same table: must cull again).  Every frame against
    the oracle, no out-of-range read."""
    import torch
    eye, sh = scenes.perspective_eye_camera(), scenes.shadow_camera()
    eye2 = scenes.Camera(eye.type_, (0.3, -0.2, 0.5), eye.dirNormalized, eye.upNormalized, eye.sideNormalized)
    a, b = scenes.raytracing_plane0(True), _thin_cylinders(scenes, 3)
    seqs = [(eye, [a] * 6), (eye, [a] * 6), (eye, [a, a, a, b, a, a]), (eye, [b] * 6), (eye, [b] * 6),
            (eye, [a] * 6), (eye2, [a] * 6), (eye, [a] * 6)]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(6)]
    want = {}
    for e, frames in seqs:
        for s_ in frames:
            if (id(e), id(s_)) not in want:
                want[(id(e), id(s_))] = oracle.render(s_, e, sh, w, h, 0, scenes.RAYTRACING_FLAGS, nthreads=NT)["rgba"]
    assert oob(rtm, gpu_ctx) >= 0  # clear
    try:
        gpu_ctx.set_batch(6)
        gpu_ctx.set_lanes(1)
        for q, (e, frames) in enumerate(seqs):
            for o in outs:
                o.fill_(-1.0)
            torch.cuda.synchronize()
            gpu_ctx.render_frames_async(frames, e, sh, w, h, 0, scenes.RAYTRACING_FLAGS, [o.data_ptr() for o in outs])
            gpu_ctx.synchronize()
            assert gpu_ctx.last_eye_blocks() == (w * h < (1 << 20))
            for i, (s_, o) in enumerate(zip(frames, outs)):
                got, ref = o.cpu().numpy(), want[(id(e), id(s_))]
                assert bits_equal(got, ref), (q, i, first_mismatch(got, ref))
    finally:
        gpu_ctx.set_lanes(0)
        gpu_ctx.set_batch(0)
    assert oob(rtm, gpu_ctx) == 0
