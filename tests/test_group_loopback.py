"""The multi-rank frame of rtm_group run on the box's one GPU.

rtm_group_create_loopback builds an N-member group in one process whose gather
is a device copy per matched send/receive pair (same event ordering as the RCCL
pairs) instead of RCCL, so members may share a device.  Everything else is the
production path: the frame partitioned over N ranks (8-row cyclic stripes by
default, contiguous bands of ceil(H/N) rows, other stripe heights), each part
rendered with the fused shadow on its own context, double-buffered staging, the
root's receive loop over peers and its 2-D placement of striped parts, chunked
frame sequences.  Every frame is compared with the CPU oracle
(oracle.render, then its writeColorImage encode) bit for bit.

Also rtm_group_set_host_direct (ABI v9): rtm_group_render delivers the frame over
N host links, each band copied from its own device into its rows of the host
frame (the reference returns the owned image to the host, main.rs:710, 896-901).
"""
import os

import numpy as np
import pytest

from test_formats_group import to_host, want_frame

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)
_WANT = {}


def want_cached(oracle, rtm, scenes, cfg, frame, fmt):
    key = (cfg, frame, fmt)
    if key not in _WANT:
        c = scenes.CONFIGS[cfg]
        s = scenes.scene_a_bench(frame) if c["scene"] is scenes.scene_a_bench else c["scene"]()
        _WANT[key] = want_frame(oracle, s, scenes.eye_camera(), scenes.shadow_camera(), c["width"], c["height"],
                                c["steps"], c["flags"], fmt, rtm.abi)
    return _WANT[key]


def device_out(torch, rtm, h, w, fmt):
    if fmt == 0:
        return torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    return torch.empty(h * w * rtm.abi.FORMAT_BYTES[fmt], dtype=torch.uint8, device="cuda")


CASES = [
    # (config, members, format, root, root staged)
    (4, 2, 0, 0, False),
    (4, 3, 0, 0, False),
    (4, 4, 0, 2, False),
    (4, 8, 0, 0, False),
    (4, 8, 1, 5, True),
    (5, 2, 2, 0, True),
    (5, 8, 0, 7, False),
    (2, 3, 0, 1, True),
    (2, 8, 1, 0, False),
    (2, 8, 2, 3, True),
]


@pytest.mark.parametrize("case", CASES, ids=[f"cfg{c[0]}-n{c[1]}-fmt{c[2]}-root{c[3]}{'-staged' if c[4] else ''}"
                                             for c in CASES])
def test_loopback_group_frame_matches_oracle(rtm, oracle, scenes, case):
    """One frame over N members (the root's band in place or staged, any root): the
    assembled frame == the oracle's, bit for bit, at the BASELINE sizes."""
    import torch
    cfg, n, fmt, root, staged = case
    c = scenes.CONFIGS[cfg]
    w, h, k = c["width"], c["height"], c["steps"]
    s = scenes.scene_a_bench(100) if cfg != 5 else c["scene"]()
    g = rtm.Group(n_devices=n, loopback=True)
    try:
        assert g.info() == (n, n, 0)
        g.set_root_staging(staged)
        out = device_out(torch, rtm, h, w, fmt)
        out.fill_(0xAB if fmt else 7.0)
        torch.cuda.synchronize()
        g.render_async(s, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, c["flags"], fmt, root,
                       out.data_ptr())
        g.synchronize(120000)
        got = to_host(out, h, w, fmt, rtm.abi)
        want = want_cached(oracle, rtm, scenes, cfg, 100, fmt)
        bad = got.view(np.uint8) != want.view(np.uint8)
        assert not bad.any(), f"{int(bad.sum())} bytes differ, first rows {sorted(set(np.argwhere(bad)[:, 0]))[:5]}"
    finally:
        g.close()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("n,staged", [(4, False), (3, True), (8, False)])
def test_loopback_group_frame_sequence_reuses_staging(rtm, oracle, scenes, n, staged):
    """12 frames at 1920x1080 (auto frames per launch on a band), outputs reused so
    chunks are cut and both staging slots of every member are reused several
    times; each output holds the oracle's frame of its last writer."""
    import torch
    w, h, k = 1920, 1080, 32
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    frames = [scenes.scene_a_bench(11 * i) for i in range(12)]
    order = [0, 1, 2, 0, 3, 1, 2, 3, 0, 1, 2, 3]
    g = rtm.Group(n_devices=n, loopback=True)
    try:
        g.set_root_staging(staged)
        bufs = [device_out(torch, rtm, h, w, 0) for _ in range(4)]
        torch.cuda.synchronize()
        g.render_frames_async(frames, eye, sh, w, h, k, 0, 0, 0, [bufs[o].data_ptr() for o in order])
        g.synchronize(120000)
        last = {o: i for i, o in enumerate(order)}
        for b, i in last.items():
            want = oracle.render(frames[i], eye, sh, w, h, k, 0, nthreads=NT)["rgba"]
            got = to_host(bufs[b], h, w, 0, rtm.abi)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), (b, i)
    finally:
        g.close()


@pytest.mark.parametrize("n", [1, 3, 8])
@pytest.mark.parametrize("fmt", [0, 1, 2])
def test_group_render_host_direct(rtm, oracle, scenes, n, fmt):
    """rtm_group_render with direct host delivery: every band from its own member
    into its rows of the host frame (pageable, then registered), == the oracle;
    the gathered form of the same group gives the same bytes."""
    g = rtm.Group(n_devices=n, loopback=True)
    try:
        eye, sh = scenes.eye_camera(), scenes.shadow_camera()
        for (w, h, f) in ((1920, 1080, 100), (517, 299, 60)):
            s = scenes.scene_a_bench(f)
            want = want_frame(oracle, s, eye, sh, w, h, 64, 0, fmt, rtm.abi)
            g.set_host_direct(True)
            got = g.render(s, eye, sh, w, h, 64, 0, fmt)
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
            buf = np.zeros_like(want)
            with rtm.HostRegistration(buf):
                g.render(s, eye, sh, w, h, 64, 0, fmt, out=buf)
            assert np.array_equal(buf.view(np.uint8), want.view(np.uint8))
            g.set_host_direct(False)
            got = g.render(s, eye, sh, w, h, 64, 0, fmt)
            assert np.array_equal(got.view(np.uint8), want.view(np.uint8))
    finally:
        g.close()


@pytest.mark.rccl
def test_group_host_direct_rccl_one_device(rtm, oracle, scenes):
    """The RCCL group (ncclCommInitAll over the one device) in direct mode."""
    g = rtm.Group(n_devices=1)
    try:
        g.set_host_direct(True)
        eye, sh = scenes.eye_camera(), scenes.shadow_camera()
        s = scenes.scene_a_bench(100)
        want = want_frame(oracle, s, eye, sh, 3840, 2160, 64, 0, 2, rtm.abi)
        got = g.render(s, eye, sh, 3840, 2160, 64, 0, 2)
        assert np.array_equal(got, want)
    finally:
        g.close()


def test_loopback_rejects_bad_members(rtm):
    lib = rtm.load_library()
    import ctypes as C
    h = C.c_void_p()
    assert lib.rtm_group_create_loopback(0, None, C.byref(h)) == rtm.abi.RTM_ERR_INVALID
    devs = (C.c_int32 * 2)(0, 99)
    assert lib.rtm_group_create_loopback(2, devs, C.byref(h)) == rtm.abi.RTM_ERR_INVALID
    assert not h.value


PARTS = [
    # (config, members, format, root, staged, stripe rows): contiguous bands (0), odd stripes,
    # stripe periods that do not divide H, more ranks than stripes
    (4, 8, 0, 0, False, 0),
    (4, 4, 1, 3, True, 0),
    (2, 3, 0, 1, False, 7),
    (2, 8, 2, 0, True, 3),
    (5, 7, 0, 2, False, 8),
    (2, 8, 1, 5, False, 256),
]


@pytest.mark.parametrize("case", PARTS, ids=[f"cfg{c[0]}-n{c[1]}-fmt{c[2]}-root{c[3]}{'-staged' if c[4] else ''}-S{c[5]}"
                                             for c in PARTS])
def test_loopback_group_partitions(rtm, oracle, scenes, case):
    """Both partitions (contiguous bands, S-row cyclic stripes placed by the root's 2-D
    copies; the root's own stripes in place) give the oracle's frame."""
    import torch
    cfg, n, fmt, root, staged, S = case
    c = scenes.CONFIGS[cfg]
    w, h, k = c["width"], c["height"], c["steps"]
    s = scenes.scene_a_bench(100) if cfg != 5 else c["scene"]()
    g = rtm.Group(n_devices=n, loopback=True)
    try:
        assert g.partition == 8  # the default for N > 1
        g.set_partition(S)
        assert g.partition == S
        g.set_root_staging(staged)
        out = device_out(torch, rtm, h, w, fmt)
        out.fill_(0xAB if fmt else 7.0)
        torch.cuda.synchronize()
        g.render_async(s, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, c["flags"], fmt, root,
                       out.data_ptr())
        g.synchronize(120000)
        got = to_host(out, h, w, fmt, rtm.abi)
        want = want_cached(oracle, rtm, scenes, cfg, 100, fmt)
        bad = got.view(np.uint8) != want.view(np.uint8)
        assert not bad.any(), f"{int(bad.sum())} bytes differ, first rows {sorted(set(np.argwhere(bad)[:, 0]))[:5]}"
    finally:
        g.close()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("S,n", [(8, 8), (3, 5), (64, 3)])
def test_render_stripes_matches_oracle_rows(rtm, oracle, scenes, gpu_ctx, S, n):
    """rtm_render_stripes_async: every part's compact rows are the oracle's image rows
    of that part (RGBA f32 and RGB8), fused shadow as the group renders them."""
    import torch
    shard = __import__("importlib").import_module("2018rustraytracer_amd.shard")
    w, h, k = 1920, 1080, 32
    s, eye, sh = scenes.scene_a_bench(100), scenes.eye_camera(), scenes.shadow_camera()
    fl = rtm.abi.RTM_FLAG_FUSED_SHADOW
    want = {f: want_frame(oracle, s, eye, sh, w, h, k, fl, f, rtm.abi) for f in (0, 2)}
    for f in (0, 2):
        for r in range(n):
            rows = shard.stripe_rows_of(h, n, S, r)
            out = device_out(torch, rtm, rows, w, f)
            torch.cuda.synchronize()
            gpu_ctx.render_stripes_async(s, eye, sh, w, h, k, fl, f, S, n, r, out.data_ptr())
            gpu_ctx.synchronize()
            got = to_host(out, rows, w, f, rtm.abi)
            assert np.array_equal(got.view(np.uint8), want[f][shard.stripe_image_rows(h, n, S, r)].view(np.uint8)), (f, r)


def test_loopback_root_moves_between_calls(rtm, oracle, scenes):
    """The root changes from call to call on one group (8-row stripes: the parts land in
    the root's receive staging, the same buffer and placement code as over RCCL, which
    is reallocated when the root moves): every frame == the oracle's."""
    import torch
    c = scenes.CONFIGS[2]
    w, h, k = c["width"], c["height"], c["steps"]
    s = scenes.scene_a_bench(100)
    g = rtm.Group(n_devices=5, loopback=True)
    try:
        assert g.partition == 8
        want = want_cached(oracle, rtm, scenes, 2, 100, 0)
        for root in (0, 3, 4, 1, 0):
            out = device_out(torch, rtm, h, w, 0)
            out.fill_(7.0)
            torch.cuda.synchronize()
            g.render_async(s, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, c["flags"], 0, root,
                           out.data_ptr())
            g.synchronize(120000)
            got = to_host(out, h, w, 0, rtm.abi)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), root
    finally:
        g.close()


@pytest.mark.parametrize("n", [pytest.param(1, marks=pytest.mark.rccl), 3])
def test_group_sequence_spreads_chunks_over_lanes(rtm, oracle, scenes, n):
    """A long sequence: every member's chunks (frames per launch of its part) go to its
    context's lanes (4 below 16 Mpixel), as rtm_render_frames_async's batches do; frames
    sampled across the chunks == the oracle's (N = 1: the RCCL group, rendered in place)."""
    import torch
    w, h, k = 1920, 1080, 32
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    frames = [scenes.scene_a_bench(100 + i) for i in range(96)]
    g = rtm.Group(n_devices=1) if n == 1 else rtm.Group(n_devices=n, loopback=True)
    try:
        bufs = [device_out(torch, rtm, h, w, 0) for _ in frames]
        torch.cuda.synchronize()
        g.render_frames_async(frames, eye, sh, w, h, k, 0, 0, 0, [b.data_ptr() for b in bufs])
        g.synchronize(120000)
        # chunks of the library's auto frames per launch for member 0's part; lanes: 4 at most
        shard = __import__("importlib").import_module("2018rustraytracer_amd.shard")
        px = w * (shard.stripe_rows_of(h, n, 8, 0) if n > 1 else h)
        per = max(1, min(len(frames), 64 if px < (1 << 20) else 32, (64 << 20) // px))
        assert g.member_lanes(0) == min(4, -(-len(frames) // per))  # n = 1: 3 chunks of 32; n = 3: 2 of 64
        for i in (0, 31, 32, 63, 64, 95):
            fl = rtm.abi.RTM_FLAG_FUSED_SHADOW if n > 1 else 0
            want = oracle.render(frames[i], eye, sh, w, h, k, fl, nthreads=NT)["rgba"]
            got = to_host(bufs[i], h, w, 0, rtm.abi)
            assert np.array_equal(got.view(np.uint32), want.view(np.uint32)), i
    finally:
        g.close()
        torch.cuda.empty_cache()


@pytest.mark.parametrize("n", [pytest.param(1, marks=pytest.mark.rccl), 3])
def test_group_sequence_into_one_buffer_lands_in_order(rtm, oracle, scenes, n):
    """Every frame of a sequence into ONE root buffer: the repeated
    output starts a new chunk per frame, and chunks would go to different lanes; the
    member rendering the root's rows in place then keeps one lane, so the buffer holds
    the LAST frame (N = 1: the RCCL group in place; N = 3: loopback, the root's own
    stripes in place, the others' gathered)."""
    import torch
    w, h, k = 640, 360, 32
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    shard = __import__("importlib").import_module("2018rustraytracer_amd.shard")
    px = w * (shard.stripe_rows_of(h, n, 8, 0) if n > 1 else h)
    per = max(1, min(64 if px < (1 << 20) else 32, (64 << 20) // px))  # the auto frames per launch
    frames = [scenes.scene_a_bench(100 + 7 * i) for i in range(per + 1)]
    g = rtm.Group(n_devices=1) if n == 1 else rtm.Group(n_devices=n, loopback=True)
    try:
        buf = device_out(torch, rtm, h, w, 0)
        buf.fill_(float("nan"))
        torch.cuda.synchronize()
        g.render_frames_async(frames, eye, sh, w, h, k, 0, 0, 0, [buf.data_ptr()] * len(frames))
        g.synchronize(120000)
        assert g.member_lanes(0) == 1  # (member 0 holds the root, rendering in place)
        fl = rtm.abi.RTM_FLAG_FUSED_SHADOW if n > 1 else 0
        want = oracle.render(frames[-1], eye, sh, w, h, k, fl, nthreads=NT)["rgba"]
        got = to_host(buf, h, w, 0, rtm.abi)
        assert np.array_equal(got.view(np.uint32), want.view(np.uint32))
    finally:
        g.close()
        torch.cuda.empty_cache()


@pytest.mark.rccl
def test_group_distinct_outputs_keep_their_lanes(rtm, scenes):
    """The lane cap applies only where outputs overlap across chunks: distinct buffers
    keep the auto lanes (test_group_sequence_spreads_chunks_over_lanes checks the images)."""
    import torch
    w, h, k = 640, 360, 16
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    per = max(1, min(64, (64 << 20) // (w * h)))
    frames = [scenes.scene_a_bench(100)] * (3 * per)
    g = rtm.Group(n_devices=1)
    try:
        bufs = [device_out(torch, rtm, h, w, 0) for _ in frames]
        torch.cuda.synchronize()
        g.render_frames_async(frames, eye, sh, w, h, k, 0, 0, 0, [b.data_ptr() for b in bufs])
        g.synchronize(120000)
        assert g.member_lanes(0) == 3
    finally:
        g.close()
        torch.cuda.empty_cache()
