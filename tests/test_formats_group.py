"""ABI v6 on the GPU: the eye pass's writeColorImage epilogue (RGBA8 / RGB8,
main.rs:660-704 as the output format, row f-2), the host-output entry points
(pageable and registered buffers), and the RCCL multi-GPU frame (SURVEY.md §8e:
row bands + one gather into the root's device buffer), all against the CPU
oracle (its f64 frame, then its writeColorImage encode) bit for bit.

The box has one GPU: the group runs with one rank (ncclCommInitAll over one
device, and the rank form ncclCommInitRank), with the root's band both in
place and staged through RCCL (send/recv to itself), so the transfer path runs.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def want_frame(oracle, scene, eye, shadow, w, h, k, flags, fmt, abi):
    rgba = oracle.render(scene, eye, shadow, w, h, k, flags, nthreads=NT)["rgba"]
    if fmt == abi.RTM_FORMAT_RGBA32F:
        return rgba
    rgb = oracle.encode_rgb8(rgba).astype(np.uint8)
    if fmt == abi.RTM_FORMAT_RGB8:
        return rgb
    return np.concatenate([rgb, np.full(rgb.shape[:-1] + (1,), 255, np.uint8)], -1)


def device_frame(torch, h, w, fmt, abi, pad=0):
    if fmt == abi.RTM_FORMAT_RGBA32F:
        t = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        return t, t
    nb = abi.FORMAT_BYTES[fmt]
    raw = torch.empty(h * w * nb + pad, dtype=torch.uint8, device="cuda")
    return raw, raw[pad:pad + h * w * nb]


def to_host(t, h, w, fmt, abi):
    a = t.cpu().numpy()
    return a.reshape(h, w, 4) if fmt == abi.RTM_FORMAT_RGBA32F else a.reshape(h, w, abi.FORMAT_BYTES[fmt])


CASES = [
    # (scene, eye, w, h, k, flags): W % 4 == 0 and != 0 (RGB8 dword vs byte stores), ragged waves
    ("a_bench", "eye", 640, 480, 64, 0),
    ("a_bench", "eye", 513, 77, 64, 0),
    ("a_bench", "eye", 516, 35, 32, 4),      # fused shadow
    ("orbit0", "eye", 512, 512, 500, 0),     # the reference's scene and march at 512^2
    ("mixed_rt", "eye", 300, 200, 64, 0),    # ray-traced primitives (row f-1)
    ("persp1", "persp", 260, 130, 0, 1),     # perspective spheres (row f-3), no march
    ("sdf", "sdf", 132, 100, 0, 1),          # SDF (row f-4)
]


def case_scene(scenes, name):
    if name == "a_bench":
        return scenes.scene_a_bench(100)
    if name == "orbit0":
        return scenes.closely_orbiting_sphere(0)
    if name == "mixed_rt":
        return scenes.mixed_rt(100)
    if name == "persp1":
        return scenes.perspective_simple1()
    return scenes.sdf_bench_scene()


def case_eye(scenes, name):
    return {"eye": scenes.eye_camera, "persp": scenes.perspective_eye_camera, "sdf": scenes.sdf_eye_camera}[name]()


@pytest.mark.parametrize("fmt", [1, 2])
@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[2]}x{c[3]}-k{c[4]}-f{c[5]}" for c in CASES])
def test_format_epilogue_matches_oracle(rtm, oracle, scenes, gpu_ctx, case, fmt):
    import torch
    abi = rtm.abi
    name, eyen, w, h, k, flags = case
    scene, eye, sh = case_scene(scenes, name), case_eye(scenes, eyen), scenes.shadow_camera()
    if flags == 1:
        flags = scenes.RAYTRACING_FLAGS
    want = want_frame(oracle, scene, eye, sh, w, h, k, flags, fmt, abi)
    for pad in (0, 1):  # aligned and 1-byte-offset output (RGB8: byte stores)
        raw, out = device_frame(torch, h, w, fmt, abi, pad)
        torch.cuda.synchronize()
        gpu_ctx.render_rows_async(scene, eye, sh, w, h, k, flags, fmt, out.data_ptr())
        gpu_ctx.synchronize()
        got = to_host(out, h, w, fmt, abi)
        assert np.array_equal(got, want), f"pad {pad}: {int((got != want).sum())} bytes differ"


def test_format_epilogue_row_bands(rtm, oracle, scenes, gpu_ctx):
    """Bands of a W % 4 != 0 frame in RGB8 concatenate to the full frame."""
    import torch
    abi = rtm.abi
    w, h, k = 333, 50, 64
    scene, eye, sh = scenes.scene_a_bench(3), scenes.eye_camera(), scenes.shadow_camera()
    want = want_frame(oracle, scene, eye, sh, w, h, k, 0, abi.RTM_FORMAT_RGB8, abi)
    parts = []
    for b0, b1 in ((0, 17), (17, 18), (18, 50)):
        out = torch.empty((b1 - b0) * w * 3, dtype=torch.uint8, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.render_rows_async(scene, eye, sh, w, h, k, 0, abi.RTM_FORMAT_RGB8, out.data_ptr(), b0, b1)
        gpu_ctx.synchronize()
        parts.append(out.cpu().numpy().reshape(b1 - b0, w, 3))
    assert np.array_equal(np.concatenate(parts, 0), want)


def test_format_epilogue_equals_encode_of_f32_frame_4k(rtm, scenes, gpu_ctx):
    """Config 3 at full size: the RGB8 epilogue equals rtm_encode_rgb8_async of the
    RGBA32F frame, and RGBA8 carries the same bytes (size-independent identity)."""
    import torch
    abi = rtm.abi
    w, h, k = 3840, 2160, 64
    scene, eye, sh = scenes.scene_a_bench(100), scenes.eye_camera(), scenes.shadow_camera()
    f32 = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    enc = torch.empty(h * w * 3, dtype=torch.uint8, device="cuda")
    rgb = torch.empty(h * w * 3, dtype=torch.uint8, device="cuda")
    rgba = torch.empty(h * w * 4, dtype=torch.uint8, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.render_async(scene, eye, sh, w, h, k, 0, f32.data_ptr())
    gpu_ctx.encode_rgb8_async(f32.data_ptr(), w * h, enc.data_ptr())
    gpu_ctx.render_rows_async(scene, eye, sh, w, h, k, 0, abi.RTM_FORMAT_RGB8, rgb.data_ptr())
    gpu_ctx.render_rows_async(scene, eye, sh, w, h, k, 0, abi.RTM_FORMAT_RGBA8, rgba.data_ptr())
    gpu_ctx.synchronize()
    assert torch.equal(rgb, enc)
    r4 = rgba.view(h * w, 4)
    assert torch.equal(r4[:, :3].reshape(-1), enc)
    assert bool((r4[:, 3] == 255).all())


@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_render_ex_host_pageable_and_registered(rtm, oracle, scenes, fmt):
    abi = rtm.abi
    w, h, k = 400, 300, 64
    scene, eye, sh = scenes.scene_a_bench(50), scenes.eye_camera(), scenes.shadow_camera()
    want = want_frame(oracle, scene, eye, sh, w, h, k, 0, fmt, abi)
    got = rtm.render_frame_ex(scene, eye, sh, w, h, k, 0, fmt)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    buf = np.zeros_like(want)
    with rtm.HostRegistration(buf):
        rtm.render_frame_ex(scene, eye, sh, w, h, k, 0, fmt, out=buf)
        assert np.array_equal(buf.view(np.uint8), want.view(np.uint8))
        buf[:] = 0
        rtm.render_frame_ex(scene, eye, sh, w, h, k, 0, fmt, n_gpus=1, out=buf)
        assert np.array_equal(buf.view(np.uint8), want.view(np.uint8))
    got = rtm.render_frame_ex(scene, eye, sh, w, h, k, 0, fmt, n_gpus=1)
    assert np.array_equal(got.view(np.uint8), want.view(np.uint8))


def test_render_ex_rejects_unknown_format(rtm, scenes):
    lib = rtm.load_library()
    assert [lib.rtm_format_bytes(f) for f in (0, 1, 2, 3, -1)] == [16, 4, 3, 0, 0]
    with pytest.raises(rtm.RtmError) as e:
        rtm.render_frame_ex(scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), 64, 64, 8, 0, 3,
                            out=np.empty((64, 64, 4), np.float32))
    assert e.value.code == rtm.abi.RTM_ERR_INVALID


# ---- the RCCL group on the box's one device ----

def group_frames(rtm, torch, g, frames, eye, sh, w, h, k, flags, fmt):
    outs = []
    for _ in frames:
        t = (torch.empty((h, w, 4), dtype=torch.float32, device="cuda") if fmt == 0 else
             torch.empty(h * w * rtm.abi.FORMAT_BYTES[fmt], dtype=torch.uint8, device="cuda"))
        outs.append(t)
    torch.cuda.synchronize()
    for s, t in zip(frames, outs):
        g.render_async(s, eye, sh, w, h, k, flags, fmt, 0, t.data_ptr())
    g.synchronize(60000)
    return [to_host(t, h, w, fmt, rtm.abi) for t in outs]


@pytest.mark.rccl
@pytest.mark.parametrize("staging", [False, True], ids=["in-place", "rccl-self-gather"])
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_group_comm_init_all_one_device(rtm, oracle, scenes, fmt, staging):
    """ncclCommInitAll over the one device; several frames back to back (the staging
    buffers alternate), each bit-equal to the oracle (and its encode)."""
    import torch
    g = rtm.Group(n_devices=1)
    assert g.info() == (1, 1, 0)
    g.set_root_staging(staging)
    w, h, k = 516, 301, 64
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    frames = [scenes.scene_a_bench(f) for f in (0, 40, 80)]
    got = group_frames(rtm, torch, g, frames, eye, sh, w, h, k, 0, fmt)
    for s, gi in zip(frames, got):
        want = want_frame(oracle, s, eye, sh, w, h, k, 0, fmt, rtm.abi)
        assert np.array_equal(gi.view(np.uint8), want.view(np.uint8))
    g.close()


@pytest.mark.rccl
def test_group_rank_form_one_rank(rtm, oracle, scenes):
    """ncclCommInitRank with a unique id (the one-process-per-GPU form bench.py uses)."""
    import torch
    uid = rtm.Group.unique_id()
    assert len(uid) == 128
    g = rtm.Group(device=0, n_ranks=1, rank=0, uid=uid)
    g.set_root_staging(True)
    w, h, k = 640, 360, 64
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    s = scenes.scene_a_bench(100)
    (got,) = group_frames(rtm, torch, g, [s], eye, sh, w, h, k, 0, 1)
    want = want_frame(oracle, s, eye, sh, w, h, k, 0, 1, rtm.abi)
    assert np.array_equal(got, want)
    g.close()


@pytest.mark.rccl
def test_group_full_size_config3(rtm, scenes, gpu_ctx):
    """Config 3 at full size through the group (RCCL self-gather, RGBA32F): equal to
    the single-context frame bit for bit."""
    import torch
    w, h, k = 3840, 2160, 64
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    s = scenes.scene_a_bench(100)
    ref = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.render_async(s, eye, sh, w, h, k, 0, ref.data_ptr())
    gpu_ctx.synchronize()
    g = rtm.Group(n_devices=1)
    g.set_root_staging(True)
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    g.render_async(s, eye, sh, w, h, k, 0, 0, 0, out.data_ptr())
    g.synchronize(60000)
    assert torch.equal(out.view(torch.int32), ref.view(torch.int32))
    g.close()


@pytest.mark.rccl
def test_group_rejects_bad_input_before_enqueue(rtm, scenes):
    import torch
    g = rtm.Group(n_devices=1)
    out = torch.empty((8, 8, 4), dtype=torch.float32, device="cuda")
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    with pytest.raises(rtm.RtmError):
        g.render_async(scenes.scene_a_bench(), eye, sh, 8, 8, 8, 0, 0, 1, out.data_ptr())  # root outside [0, 1)
    with pytest.raises(rtm.RtmError):
        g.render_async(scenes.scene_a_bench(), eye, sh, 8, 8, 8, 0, 9, 0, out.data_ptr())  # unknown format
    bad = scenes.scene_a_bench()
    bad.spherePrimitives[0].id = 7
    with pytest.raises(rtm.RtmError):
        g.render_async(bad, eye, sh, 8, 8, 8, 0, 0, 0, out.data_ptr())
    g.synchronize(10000)  # nothing was enqueued: returns at once
    g.close()


@pytest.mark.rccl
@pytest.mark.parametrize("staging", [False, True], ids=["in-place", "rccl-self-gather"])
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_group_render_host_output(rtm, oracle, scenes, fmt, staging):
    """rtm_group_render (ABI v8, the form a host without device memory calls): the
    gathered frame in host memory, pageable and registered, sizes that change from
    call to call (the group's root buffer grows), bit-equal to the oracle."""
    g = rtm.Group(n_devices=1)
    g.set_root_staging(staging)
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    for (w, h, f) in ((320, 180, 10), (517, 299, 60), (320, 180, 90)):
        s = scenes.scene_a_bench(f)
        want = want_frame(oracle, s, eye, sh, w, h, 64, 0, fmt, rtm.abi)
        got = g.render(s, eye, sh, w, h, 64, 0, fmt)
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
        buf = np.zeros_like(want)
        with rtm.HostRegistration(buf):
            g.render(s, eye, sh, w, h, 64, 0, fmt, out=buf)
        assert np.array_equal(buf.view(np.uint8), want.view(np.uint8))
    with pytest.raises(rtm.RtmError):
        g.render(scenes.scene_a_bench(), eye, sh, 8, 8, 8, 0, 9)  # unknown format
    g.close()


@pytest.mark.rccl
@pytest.mark.parametrize("staging", [False, True], ids=["in-place", "rccl-self-gather"])
@pytest.mark.parametrize("fmt", [0, 1])
def test_group_frame_sequence_batched(rtm, oracle, scenes, fmt, staging):
    """rtm_group_render_frames_async over 10 frames: the bands of a chunk render in
    one launch per pass (auto: 16 frames of 256x144 per launch), a repeated output
    pointer cuts the chunk so the later frame lands last; every output holds the
    oracle's frame (and encode) of the last frame written into it."""
    import torch
    g = rtm.Group(n_devices=1)
    g.set_root_staging(staging)
    w, h, k = 256, 144, 64
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    frames = [scenes.scene_a_bench(7 * i) for i in range(10)]
    bufs = [(torch.empty((h, w, 4), dtype=torch.float32, device="cuda") if fmt == 0 else
             torch.empty(h * w * rtm.abi.FORMAT_BYTES[fmt], dtype=torch.uint8, device="cuda")) for _ in range(4)]
    order = [0, 1, 2, 3, 0, 1, 2, 3, 1, 2]   # the last writers: buf0 <- 4, buf1 <- 8, buf2 <- 9, buf3 <- 7
    torch.cuda.synchronize()
    g.render_frames_async(frames, eye, sh, w, h, k, 0, fmt, 0, [bufs[o].data_ptr() for o in order])
    g.synchronize(60000)
    last = {o: i for i, o in enumerate(order)}
    for b, i in last.items():
        got = to_host(bufs[b], h, w, fmt, rtm.abi)
        want = want_frame(oracle, frames[i], eye, sh, w, h, k, 0, fmt, rtm.abi)
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8)), (b, i)
    g.close()


@pytest.mark.rccl
@pytest.mark.parametrize("fmt", [0, 2])
def test_group_frame_sequence_raytraced_perspective(rtm, scenes, gpu_ctx, fmt):
    """The group's batched bands with ray-traced primitives under a PERSPECTIVE eye
    (the batched per-wave primitive cull) and perspective spheres, in one chunk:
    every frame equals the single-device rtm_render_ex bytes."""
    import torch
    g = rtm.Group(n_devices=1)
    g.set_root_staging(True)
    w, h = 320, 240
    eye, sh = scenes.perspective_eye_camera(), scenes.shadow_camera()
    fl = scenes.RAYTRACING_FLAGS
    frames = [scenes.raytracing_plane0(), scenes.scene_r_bench(), scenes.perspective_simple1(),
              scenes.raytracing_plane0(True), scenes.scene_r_bench(), scenes.perspective_simple2()]
    bufs = [(torch.empty((h, w, 4), dtype=torch.float32, device="cuda") if fmt == 0 else
             torch.empty(h * w * rtm.abi.FORMAT_BYTES[fmt], dtype=torch.uint8, device="cuda")) for _ in frames]
    from test_bounds import oob
    assert oob(rtm, gpu_ctx) >= 0  # clear (the count is the device's, every context's)
    torch.cuda.synchronize()
    g.render_frames_async(frames, eye, sh, w, h, 0, fl, fmt, 0, [b.data_ptr() for b in bufs])
    g.synchronize(60000)
    assert oob(rtm, gpu_ctx) == 0  # (RGBA f32: the listed-block eye pass, its list in range)
    for s, b in zip(frames, bufs):
        want = rtm.render_frame_ex(s, eye, sh, w, h, 0, fl, fmt)
        got = to_host(b, h, w, fmt, rtm.abi)
        assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    g.close()
