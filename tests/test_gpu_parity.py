"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bar: bit-exact RGBA f32 and f64 shadow maps (the north
star's 1e-5 per-channel tolerance is implied by bit equality, which is what we
assert).  Sizes cover every BASELINE config at full size plus ragged and edge
cases.  All calls go through librtm.so; nothing here falls back to the CPU.
"""
import math
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _oracle(oracle, scene, eye, shadow, w, h, k, flags=0, **kw):
    return oracle.render(scene, eye, shadow, w, h, k, flags, nthreads=NT, **kw)


def _check_frame(rtm, oracle, scene, eye, shadow, w, h, k, flags=0):
    got = rtm.render_frame(scene, eye, shadow, w, h, k, flags)
    want = _oracle(oracle, scene, eye, shadow, w, h, k, flags)["rgba"]
    assert bits_equal(got, want), first_mismatch(got, want)
    return got


@pytest.mark.parametrize("frame", [0, 37, 100, 250])
def test_reference_scene_512(rtm, oracle, scenes, frame):
    """testscene_closelyOrbitingSphere at the reference's own 512x512, 500 steps."""
    _check_frame(rtm, oracle, scenes.closely_orbiting_sphere(frame), scenes.eye_camera(),
                 scenes.shadow_camera(), 512, 512, 500)


def test_survey_kat_frame0_and_100(rtm, scenes):
    """SURVEY.md §8c-3 cross-check values, straight from the GPU."""
    import hashlib
    for frame, sha in ((0, "cf557d736f83a4f6"), (100, "cb7008f728da5208")):
        img = rtm.render_frame(scenes.closely_orbiting_sphere(frame), scenes.eye_camera(),
                               scenes.shadow_camera(), 512, 512, 500)
        rgb = np.ascontiguousarray(img[:, :, :3])
        assert hashlib.sha256(rgb.tobytes()).hexdigest()[:16] == sha
    img = rtm.render_frame(scenes.closely_orbiting_sphere(0), scenes.eye_camera(),
                           scenes.shadow_camera(), 512, 512, 500)
    assert img[256, 384, :3].tolist() == [9265101144064.0, 9265101144064.0, 463255038328832.0]
    assert img[300, 384, :3].tolist() == [3506.7421875, 3506.7421875, 175337.109375]


@pytest.mark.parametrize("cfg", [1, 2, 3])
def test_baseline_configs_full_size(rtm, oracle, scenes, cfg):
    c = scenes.CONFIGS[cfg]
    _check_frame(rtm, oracle, c["scene"](), scenes.eye_camera(), scenes.shadow_camera(),
                 c["width"], c["height"], c["steps"], c["flags"])


@pytest.mark.parametrize("cfg", [4, 5])
def test_baseline_configs_8k(rtm, oracle, scenes, cfg):
    c = scenes.CONFIGS[cfg]
    _check_frame(rtm, oracle, c["scene"](), scenes.eye_camera(), scenes.shadow_camera(),
                 c["width"], c["height"], c["steps"], c["flags"])


def test_overlapping_spheres(rtm, oracle, scenes):
    """testscene_overlappingSpheres: shadow pass commented out in the reference."""
    _check_frame(rtm, oracle, scenes.overlapping_spheres(), scenes.eye_camera(), scenes.shadow_camera(),
                 512, 512, 0, scenes.OVERLAPPING_FLAGS)


@pytest.mark.parametrize("wh", [(1, 1), (2, 3), (63, 65), (1000, 7), (7, 1000), (130, 66)])
def test_ragged_sizes(rtm, oracle, scenes, wh):
    w, h = wh
    _check_frame(rtm, oracle, scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), w, h, 64)


@pytest.mark.parametrize("k", [0, 1, 5, 33, 500])
def test_march_steps(rtm, oracle, scenes, k):
    _check_frame(rtm, oracle, scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), 256, 192, k)


def test_shadow_map_bits(rtm, oracle, scenes, gpu_ctx):
    """The shadow viewport's zBuffer (rasterize BACK + march) bit for bit."""
    import torch
    for scene, w, h, k in ((scenes.closely_orbiting_sphere(100), 512, 512, 500),
                           (scenes.scene_a_bench(), 1920, 1080, 32),
                           (scenes.scene_b(), 640, 360, 128)):
        out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.render_async(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0, out.data_ptr())
        gpu_ctx.synchronize()
        ptr = gpu_ctx.shadow_map_ptr()
        assert ptr
        got = _read_device_f64(ptr, h * w).reshape(h, w)
        want = _oracle(oracle, scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k,
                       want_shadow=True)
        assert bits_equal(got, want["shadow"]), first_mismatch(got, want["shadow"])
        assert bits_equal(out.cpu().numpy(), want["rgba"])


def _read_device_f64(ptr, n):
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    out = np.empty(n, np.float64)
    rc = hip.hipMemcpy(out.ctypes.data_as(ctypes.c_void_p), ctypes.c_void_p(ptr), ctypes.c_size_t(8 * n), 2)
    assert rc == 0
    return out


@pytest.mark.parametrize("seed", range(10))
def test_lean_shadow_path_fuzz(rtm, oracle, scenes, gpu_ctx, seed):
    """The default shadow kernel (shadow_lean2_kernel: separable camera, shared
    monotone z table, first-crossing search) under every table shape it takes:
    increasing and decreasing z (dir.z = +-1), camera offsets in x/y/z, march
    bounds around the register-fill (256) and LDS (2048) limits and past them,
    patches whose surface depth lands exactly on a march step (the guess's
    boundary case) or beyond K, partial tiles.  Shadow map and image bit for bit."""
    import torch
    rng = np.random.default_rng(0x2018 + 500 + seed)
    dz = 1.0 if seed % 2 == 0 else -1.0
    uy = 1.0 if seed % 3 else -1.0
    sx = 1.0 if seed % 4 < 2 else -1.0
    pos = (float(rng.uniform(-0.3, 0.3)), float(rng.uniform(-0.3, 0.3)), float(rng.choice([0.0, 0.25, -0.4])))
    shadow = scenes.Camera(scenes.ORTHOGONAL, pos, (0.0, 0.0, dz), (0.0, uy, 0.0), (sx, 0.0, 0.0))
    k = int([1, 63, 64, 65, 255, 256, 257, 1000, 2048, 2049][seed])
    scene = _random_scene(scenes, rng, int(rng.integers(0, 6)), 0)
    z0 = 0.0 if pos[2] == 0.0 else pos[2]
    step = dz * 0.03
    pats = []
    for _ in range(int(rng.integers(1, 4))):
        m = float(rng.integers(0, k + 3))  # a crossing on (or near) step m, maybe beyond K
        a0 = z0 + m * step
        pats.append(scenes.Bilinear(scenes.Linear(a0, a0 + float(rng.uniform(-0.5, 0.5))),
                                    scenes.Linear(a0 + float(rng.uniform(-0.5, 0.5)), float(rng.uniform(-1, 1)))))
    scene.patches = pats
    w, h = int(rng.integers(65, 331)), int(rng.integers(17, 201))
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.render_async(scene, scenes.eye_camera(), shadow, w, h, k, 0, out.data_ptr())
    gpu_ctx.synchronize()
    got = _read_device_f64(gpu_ctx.shadow_map_ptr(), h * w).reshape(h, w)
    want = _oracle(oracle, scene, scenes.eye_camera(), shadow, w, h, k, want_shadow=True)
    assert bits_equal(got, want["shadow"]), first_mismatch(got, want["shadow"])
    assert bits_equal(out.cpu().numpy(), want["rgba"]), first_mismatch(out.cpu().numpy(), want["rgba"])


def test_fused_shadow_identical(rtm, oracle, scenes):
    """RTM_FLAG_FUSED_SHADOW evaluates texels on demand: same image bits."""
    for scene, w, h, k in ((scenes.closely_orbiting_sphere(100), 512, 512, 500),
                           (scenes.scene_a_bench(), 1920, 1080, 32), (scenes.scene_b(), 800, 600, 128)):
        a = rtm.render_frame(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0)
        b = rtm.render_frame(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k,
                             rtm.abi.RTM_FLAG_FUSED_SHADOW)
        assert bits_equal(a, b), first_mismatch(b, a)


def test_row_bands_assemble(rtm, scenes, gpu_ctx):
    """rtm_render_async over row bands == the full frame (the multi-GPU shard unit)."""
    import torch
    w, h, k = 1000, 601, 64
    scene = scenes.scene_a_bench()
    full = rtm.render_frame(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k)
    for flags in (0, rtm.abi.RTM_FLAG_FUSED_SHADOW):
        parts = []
        bounds = [0, 1, 150, 333, 600, 601]
        for b0, b1 in zip(bounds[:-1], bounds[1:]):
            out = torch.empty((b1 - b0, w, 4), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            gpu_ctx.render_async(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, flags,
                                 out.data_ptr(), b0, b1)
            gpu_ctx.synchronize()
            parts.append(out.cpu().numpy())
        assert bits_equal(np.concatenate(parts, 0), full)


def test_staged_api_matches_oracle(rtm, oracle, scenes, gpu_ctx):
    """Viewport.rasterize / processRaymarchingRays / renderColorImage, one call
    per reference function, against the oracle's staged API."""
    for frame, w, h in ((100, 512, 512), (37, 300, 200)):
        scene = scenes.closely_orbiting_sphere(frame)
        vp1 = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.BACK, scenes.shadow_camera())
        vp1.rasterize(scene)
        vp1.processRaymarchingRays()
        vp0 = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.FRONT, scenes.eye_camera())
        vp0.rasterize(scene)
        img = rtm.renderColorImage(scene, vp0, vp1)
        o1 = oracle.Viewport(w, h, scenes.EnumFace.BACK, scenes.shadow_camera())
        o1.rasterize(scene)
        o1.processRaymarchingRays([scenes.REFERENCE_PATCH], 500)
        o0 = oracle.Viewport(w, h, scenes.EnumFace.FRONT, scenes.eye_camera())
        o0.rasterize(scene)
        want = oracle.render_color_image(scene, o0, o1)
        assert bits_equal(vp1.zBuffer(), o1.zbuffer())
        assert bits_equal(vp0.zBuffer(), o0.zbuffer())
        assert bits_equal(img, want), first_mismatch(img, want)
        # and the staged path equals the one-call frame path
        frame_img = rtm.render_frame(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, 500)
        assert bits_equal(img, frame_img)


def test_staged_perspective_march(rtm, oracle, scenes, gpu_ctx):
    """processRaymarchingRays with a PERSPECTIVE camera (normalised ray dirs,
    main.rs:1922-1939): the general (non-axis-aligned) march loop."""
    cam = scenes.Camera(scenes.PERSPECTIVE, (0.1, -0.2, -0.3), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0),
                        (1.0, 0.0, 0.0))
    patches = [scenes.BENCH_PATCH, scenes.SCENE_B_PATCH2]
    vp = rtm.Viewport(gpu_ctx, 200, 150, scenes.EnumFace.BACK, cam)
    vp.processRaymarchingRays(patches, 200)
    o = oracle.Viewport(200, 150, scenes.EnumFace.BACK, cam)
    o.processRaymarchingRays(patches, 200)
    got, want = vp.zBuffer(), o.zbuffer()
    assert np.isfinite(want).sum() > 1000
    assert bits_equal(got, want), first_mismatch(got, want)


def test_stats_match_oracle(rtm, oracle, scenes, gpu_ctx):
    for scene, w, h, k in ((scenes.closely_orbiting_sphere(100), 512, 512, 500),
                           (scenes.scene_a_bench(), 1920, 1080, 32), (scenes.scene_b(), 640, 480, 128)):
        got = gpu_ctx.stats(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k)
        want = _oracle(oracle, scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k,
                       want_stats=True)["stats"]
        assert got == want


def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    a, b, c, d = q
    return np.array([[a*a+b*b-c*c-d*d, 2*(b*c-a*d), 2*(b*d+a*c)],
                     [2*(b*c+a*d), a*a-b*b+c*c-d*d, 2*(c*d-a*b)],
                     [2*(b*d-a*c), 2*(c*d+a*b), a*a-b*b-c*c+d*d]])


def _random_scene(scenes, rng, ns, npch):
    sph = []
    for i in range(ns):
        sph.append(scenes.PrimitiveSphere(
            int(i), scenes.Shading(*[float(v) for v in rng.uniform(0, 1, 3)]),
            tuple(float(v) for v in rng.uniform(-0.8, 0.8, 3)), float(rng.uniform(0.02, 0.4))))
    # permute ids (the reference shades with spherePrimitives[id], main.rs:748)
    perm = rng.permutation(ns)
    for s, p in zip(sph, perm):
        s.id = int(p)
    pats = [scenes.Bilinear(scenes.Linear(*map(float, rng.uniform(-0.5, 1.5, 2))),
                            scenes.Linear(*map(float, rng.uniform(-0.5, 1.5, 2)))) for _ in range(npch)]
    return scenes.Scene(sph, pats)


def _random_camera(scenes, rng, axis_aligned):
    if axis_aligned:
        return scenes.shadow_camera()
    R = _rotation(rng)
    pos = tuple(float(v) for v in rng.uniform(-0.5, 0.5, 3))
    return scenes.Camera(scenes.ORTHOGONAL, pos, tuple(map(float, R[:, 2])), tuple(map(float, R[:, 1])),
                         tuple(map(float, R[:, 0])))


@pytest.mark.parametrize("seed", range(12))
def test_random_scenes(rtm, oracle, scenes, seed):
    """Seeded fuzz (splitmix-free numpy PCG64, seed 0x2018+i): random spheres,
    patches, permuted ids and rotated orthographic cameras (general march loop)."""
    rng = np.random.default_rng(0x2018 + seed)
    ns = int(rng.integers(0, 17))
    npch = int(rng.integers(0, 5))
    scene = _random_scene(scenes, rng, ns, npch)
    eye = _random_camera(scenes, rng, seed % 3 == 0)
    shadow = _random_camera(scenes, rng, seed % 2 == 0)
    w, h = int(rng.integers(1, 400)), int(rng.integers(1, 300))
    k = int(rng.integers(0, 200))
    _check_frame(rtm, oracle, scene, eye, shadow, w, h, k)


def test_degenerate_spheres(rtm, oracle, scenes):
    s = scenes.closely_orbiting_sphere(10)
    s.spherePrimitives.append(scenes.PrimitiveSphere(3, scenes.Shading(1, 1, 1), (0.0, 0.1, 0.2), 0.0))
    s.spherePrimitives.append(scenes.PrimitiveSphere(4, scenes.Shading(1, 1, 1), (0.0, 0.1, 0.2), -0.15))
    s.spherePrimitives.append(scenes.PrimitiveSphere(5, scenes.Shading(1, 0, 1), (5.0, 5.0, 5.0), 0.3))
    s.spherePrimitives.append(scenes.PrimitiveSphere(6, scenes.Shading(0, 1, 1), (0.0, 0.0, 0.0), 3.0))
    _check_frame(rtm, oracle, s, scenes.eye_camera(), scenes.shadow_camera(), 200, 200, 100)
    empty = scenes.Scene([], [])
    _check_frame(rtm, oracle, empty, scenes.eye_camera(), scenes.shadow_camera(), 64, 64, 10)


def test_error_codes(rtm, scenes):
    abi = rtm.abi
    persp = scenes.Camera(scenes.PERSPECTIVE, (0, 0, 0), (0, 0, 1), (0, 1, 0), (1, 0, 0))
    with pytest.raises(abi.RtmError) as e:  # Camera::project asserts ORTHOGONAL (main.rs:1949)
        rtm.render_frame(scenes.scene_a_bench(), scenes.eye_camera(), persp, 64, 64, 10)
    assert e.value.code == abi.RTM_ERR_UNSUPPORTED
    with pytest.raises(abi.RtmError) as e:
        rtm.render_frame(scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), 0, 64, 10)
    assert e.value.code == abi.RTM_ERR_INVALID
    bad = scenes.scene_a_bench()
    bad.spherePrimitives[0].id = 7
    with pytest.raises(abi.RtmError) as e:
        rtm.render_frame(bad, scenes.eye_camera(), scenes.shadow_camera(), 64, 64, 10)
    assert e.value.code == abi.RTM_ERR_INVALID
    many = scenes.scene_b()
    many.spherePrimitives.append(scenes.PrimitiveSphere(16, scenes.Shading(1, 1, 1), (0, 0, 0), 0.1))
    with pytest.raises(abi.RtmError) as e:
        rtm.render_frame(many, scenes.eye_camera(), scenes.shadow_camera(), 64, 64, 10)
    assert e.value.code == abi.RTM_ERR_INVALID


def _frames_vs_single(rtm, scenes, gpu_ctx, frames, eye, shadow, w, h, k, flags=0):
    import torch
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    torch.cuda.synchronize()
    gpu_ctx.render_frames_async(frames, eye, shadow, w, h, k, flags, [o.data_ptr() for o in outs])
    gpu_ctx.synchronize()
    for s, o in zip(frames, outs):
        want = rtm.render_frame(s, eye, shadow, w, h, k, flags)
        got = o.cpu().numpy()
        assert bits_equal(got, want), first_mismatch(got, want)


@pytest.mark.parametrize("n", [1, 2, 5])
def test_frame_sequence_matches_single_frames(rtm, scenes, gpu_ctx, n):
    """rtm_render_frames_async (batched launches over the context's lanes) ==
    frame-by-frame rtm_render."""
    frames = [scenes.scene_a_bench(100 + 7 * i) for i in range(n)]
    _frames_vs_single(rtm, scenes, gpu_ctx, frames, scenes.eye_camera(), scenes.shadow_camera(), 1920, 1080, 32)


def test_frame_sequence_reference_scene_and_oracle(rtm, oracle, scenes, gpu_ctx):
    import torch
    frames = [scenes.closely_orbiting_sphere(f) for f in (0, 1, 2, 100)]
    outs = [torch.empty((512, 512, 4), dtype=torch.float32, device="cuda") for _ in frames]
    torch.cuda.synchronize()
    gpu_ctx.render_frames_async(frames, scenes.eye_camera(), scenes.shadow_camera(), 512, 512, 500, 0,
                                [o.data_ptr() for o in outs])
    gpu_ctx.synchronize()
    for s, o in zip(frames, outs):
        want = oracle.render(s, scenes.eye_camera(), scenes.shadow_camera(), 512, 512, 500, 0)["rgba"]
        assert bits_equal(o.cpu().numpy(), want)


def test_frame_sequence_generic_shadow_tiles(rtm, scenes, gpu_ctx):
    """Rotated shadow camera: the sequence's batched launches use the generic shadow tile."""
    rng = np.random.default_rng(7)
    shadow = _random_camera(scenes, rng, False)
    frames = [_random_scene(scenes, np.random.default_rng(11), 6, 2) for _ in range(3)]
    _frames_vs_single(rtm, scenes, gpu_ctx, frames, scenes.eye_camera(), shadow, 333, 217, 80)


def test_frame_sequence_differing_patches(rtm, scenes, gpu_ctx):
    frames = [scenes.scene_a_bench(100), scenes.scene_b(), scenes.closely_orbiting_sphere(3)]
    _frames_vs_single(rtm, scenes, gpu_ctx, frames, scenes.eye_camera(), scenes.shadow_camera(), 640, 360, 64)


@pytest.mark.parametrize("lanes,batch", [(1, 1), (2, 1), (3, 1), (4, 1), (3, 2), (4, 2)])
def test_frame_lanes_in_subprocess(rtm, scenes, lanes, batch):
    """RTM_LANES=n (read once per process): the frame sequence spread over n
    streams, each with its own shadow map, == frame-by-frame rtm_render; the
    context's shadow map then holds the LAST frame's shadow pass; a sequence whose
    frames share one output falls back to one lane (the last frame's image wins).
    Lanes spread batches, so the batch is fixed (1 or 2 frames per launch: 8 or 4
    batches of the 8 frames) and the lane count the call used is asserted."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = r'''
import ctypes, importlib, sys
import numpy as np, torch
sys.path.insert(0, %r)
rtm = importlib.import_module("2018rustraytracer_amd")
sc = importlib.import_module("2018rustraytracer_amd.scenes")
eye, sh = sc.eye_camera(), sc.shadow_camera()
ctx = rtm.Context(0)
ctx.set_batch(BATCH)
w, h, k = 960, 540, 64
frames = [sc.scene_a_bench(100 + 5 * i) for i in range(7)] + [sc.scene_b()]
u32 = lambda a: a.view(np.uint32)
outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
torch.cuda.synchronize()
ctx.render_frames_async(frames, eye, sh, w, h, k, 0, [o.data_ptr() for o in outs])
ctx.synchronize()
assert ctx.last_lanes() == LANES, (ctx.last_lanes(), LANES)
assert ctx.last_batch() == BATCH, (ctx.last_batch(), BATCH)
last_map = torch.empty((h, w), dtype=torch.float64, device="cuda")
hip = ctypes.CDLL("libamdhip64.so")
hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
assert hip.hipMemcpy(last_map.data_ptr(), ctx.shadow_map_ptr(), h * w * 8, 3) == 0
for s, o in zip(frames, outs):
    assert np.array_equal(u32(o.cpu().numpy()), u32(rtm.render_frame(s, eye, sh, w, h, k, 0)))
one = rtm.Context(0)
one.render_async(frames[-1], eye, sh, w, h, k, 0, outs[0].data_ptr())
one.synchronize()
want_map = torch.empty_like(last_map)
assert hip.hipMemcpy(want_map.data_ptr(), one.shadow_map_ptr(), h * w * 8, 3) == 0
assert torch.equal(last_map.view(torch.int64), want_map.view(torch.int64))
shared = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
torch.cuda.synchronize()
ctx.render_frames_async(frames, eye, sh, w, h, k, 0, [shared.data_ptr()] * len(frames))
ctx.synchronize()
assert np.array_equal(u32(shared.cpu().numpy()), u32(rtm.render_frame(frames[-1], eye, sh, w, h, k, 0)))
assert ctx.last_lanes() == 1
print("lanes ok")
'''.replace("LANES", str(lanes)).replace("BATCH", str(batch)) % root
    env = dict(os.environ, RTM_LANES=str(lanes))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0 and "lanes ok" in r.stdout, r.stdout + r.stderr


def test_set_lanes_api(rtm, scenes, gpu_ctx):
    """rtm_ctx_set_lanes / rtm_ctx_last_lanes: range check, the requested count, the
    fallback to one lane for shared outputs, and frame-by-frame parity at 2 lanes."""
    import torch
    abi = rtm.abi
    for bad in (-1, 9):
        with pytest.raises(abi.RtmError) as e:
            gpu_ctx.set_lanes(bad)
        assert e.value.code == abi.RTM_ERR_INVALID
    w, h, k = 320, 200, 48
    frames = [scenes.scene_a_bench(100 + i) for i in range(3)]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    try:
        gpu_ctx.set_batch(1)  # lanes spread batches; one frame per batch here
        gpu_ctx.set_lanes(2)
        _frames_vs_single(rtm, scenes, gpu_ctx, frames, scenes.eye_camera(), scenes.shadow_camera(), w, h, k)
        assert gpu_ctx.last_lanes() == 2
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0,
                                    [outs[0].data_ptr()] * 3)
        gpu_ctx.synchronize()
        assert gpu_ctx.last_lanes() == 1
        gpu_ctx.set_lanes(8)  # more lanes than frames: one frame per lane
        gpu_ctx.render_frames_async(frames, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0,
                                    [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
        assert gpu_ctx.last_lanes() == 3
        gpu_ctx.set_batch(2)  # 3 frames in batches of 2: two batches, at most two lanes
        gpu_ctx.render_frames_async(frames, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0,
                                    [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
        assert gpu_ctx.last_lanes() == 2 and gpu_ctx.last_batch() == 2
    finally:
        gpu_ctx.set_lanes(0)
        gpu_ctx.set_batch(0)


def test_frame_sequence_scene_b_8k(rtm, oracle, scenes, gpu_ctx):
    """BASELINE config 5 geometry through a frame sequence, against the oracle."""
    import torch
    w, h, k = 7680, 4320, 128
    frames = [scenes.scene_b(), scenes.scene_b()]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    torch.cuda.synchronize()
    gpu_ctx.render_frames_async(frames, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0,
                                [o.data_ptr() for o in outs])
    gpu_ctx.synchronize()
    want = oracle.render(frames[0], scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0, nthreads=NT)["rgba"]
    for o in outs:
        assert bits_equal(o.cpu().numpy(), want)


def test_render_multi(rtm, oracle, scenes):
    """rtm_render_multi: row bands on devices 0..n-1 of this
    process, assembled in host memory == rtm_render == the oracle.  On a
    one-GPU box n = 1; n beyond the visible devices is rejected."""
    abi = rtm.abi
    n = rtm.device_count()
    args = (scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), 640, 361, 64)
    want = _oracle(oracle, *args)["rgba"]
    for k in range(1, n + 1):
        got = rtm.render_frame_multi(*args, n_gpus=k)
        assert bits_equal(got, want), (k, first_mismatch(got, want))
    with pytest.raises(abi.RtmError) as e:
        rtm.render_frame_multi(*args, n_gpus=n + 1)
    assert e.value.code == abi.RTM_ERR_INVALID
    with pytest.raises(abi.RtmError) as e:
        rtm.render_frame_multi(*args, n_gpus=0)
    assert e.value.code == abi.RTM_ERR_INVALID


@pytest.mark.parametrize("case", ["bench", "rbench", "thin"])
def test_maximum_size_frames(rtm, oracle, scenes, gpu_ctx, case):
    """RTM_MAX_DIM: a 32768 x 32768 frame (17 GB RGBA + 8.6 GB shadow map on
    the device; element indices past 2^32) against the row-window oracle
    (oracle.render_rows) on bands at the top, middle and bottom; the same rows
    through row-band launches, two-pass and fused.  'thin': 32768 x 1 and
    1 x 32768."""
    import torch
    abi = rtm.abi
    M = abi.RTM_MAX_DIM
    if case == "thin":
        for w, h in ((M, 1), (1, M)):
            args = (scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), w, h, 64, 0)
            got = rtm.render_frame(*args)
            want = _oracle(oracle, *args)["rgba"]
            assert bits_equal(got, want), (w, h, first_mismatch(got, want))
        return
    if case == "bench":
        args = (scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), M, M, 64, 0)
    else:
        args = (scenes.scene_r_bench(), scenes.perspective_eye_camera(), scenes.shadow_camera(), M, M, 0,
                scenes.RAYTRACING_FLAGS)
    scene, eye, shadow, W, H, K, flags = args
    out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
    torch.cuda.synchronize()
    gpu_ctx.render_async(scene, eye, shadow, W, H, K, flags, out.data_ptr())
    gpu_ctx.synchronize()
    bands = [(0, 2), (H // 2 - 3, H // 2 + 3), (H - 2, H)]
    if case == "bench":
        bands.append((H // 2 + 2500, H // 2 + 2504))  # through the spheres and their shadows
    for r0, r1 in bands:
        want, _ = oracle.render_rows(scene, eye, shadow, W, H, K, flags, r0, r1)
        got = out[r0:r1].cpu().numpy()
        assert bits_equal(got, want), (r0, r1, first_mismatch(got, want))
        for f in (flags, flags | abi.RTM_FLAG_FUSED_SHADOW):
            band = torch.empty((r1 - r0, W, 4), dtype=torch.float32, device="cuda")
            torch.cuda.synchronize()
            gpu_ctx.render_async(scene, eye, shadow, W, H, K, f, band.data_ptr(), r0, r1)
            gpu_ctx.synchronize()
            assert bits_equal(band.cpu().numpy(), want), (r0, r1, f)
    del out
    torch.cuda.empty_cache()


@pytest.mark.parametrize("batch,lanes", [(0, 1), (4, 1), (3, 2), (16, 1), (1, 3)])
def test_batched_frame_sequences(rtm, scenes, gpu_ctx, batch, lanes):
    """rtm_ctx_set_batch: runs of frames with the same patches share one launch per
    pass (frame index = grid z, constants from an uploaded table); a patch change
    splits a run; batches spread over lanes.  Every frame == rtm_render bit for bit,
    and the context's shadow map is the last frame's."""
    import torch
    w, h, k = 320, 200, 48
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    frames = ([scenes.scene_a_bench(100 + 3 * i) for i in range(6)] + [scenes.closely_orbiting_sphere(7)] +
              [scenes.scene_a_bench(1), scenes.scene_b(), scenes.scene_b(), scenes.mixed_rt(20), scenes.mixed_sdf(5)])
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    try:
        gpu_ctx.set_batch(batch)
        gpu_ctx.set_lanes(lanes)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, sh, w, h, k, 0, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
        assert gpu_ctx.last_batch() == min(batch or 16, len(frames))  # (auto at 320x200: 16, capped at n)
        for s, o in zip(frames, outs):
            assert bits_equal(o.cpu().numpy(), rtm.render_frame(s, eye, sh, w, h, k)), "frame differs"
        # the last frame's shadow map
        one = rtm.Context(0)
        ref = torch.empty((h, w, 4), dtype=torch.float32, device="cuda")
        one.render_async(frames[-1], eye, sh, w, h, k, 0, ref.data_ptr())
        one.synchronize()
        import ctypes
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        a = torch.empty((h, w), dtype=torch.float64, device="cuda")
        b = torch.empty_like(a)
        assert hip.hipMemcpy(a.data_ptr(), gpu_ctx.shadow_map_ptr(), h * w * 8, 3) == 0
        assert hip.hipMemcpy(b.data_ptr(), one.shadow_map_ptr(), h * w * 8, 3) == 0
        assert torch.equal(a.view(torch.int64), b.view(torch.int64))
        one.close()
        # perspective eye + ray-traced primitives, SDFs, fused shadow: the other kernel variants
        for eye2, fl, fr in ((scenes.perspective_eye_camera(), scenes.RAYTRACING_FLAGS,
                              [scenes.raytracing_plane0(True), scenes.perspective_simple2(), scenes.scene_r_bench(),
                               scenes.raytracing_plane0(), scenes.perspective_simple1()]),
                             (scenes.sdf_eye_camera(), scenes.RAYTRACING_FLAGS,
                              [scenes.sdf_bench_scene(), scenes.sdf_preview_scene(), scenes.sdf_bench_scene()]),
                             (eye, rtm.abi.RTM_FLAG_FUSED_SHADOW, [scenes.scene_a_bench(i) for i in range(5)])):
            o2 = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in fr]
            torch.cuda.synchronize()
            gpu_ctx.render_frames_async(fr, eye2, sh, w, h, k, fl, [o.data_ptr() for o in o2])
            gpu_ctx.synchronize()
            for s, o in zip(fr, o2):
                assert bits_equal(o.cpu().numpy(), rtm.render_frame(s, eye2, sh, w, h, k, fl)), "variant differs"
    finally:
        gpu_ctx.set_batch(0)
        gpu_ctx.set_lanes(0)


def test_batch_with_repeated_outputs(rtm, scenes, gpu_ctx):
    """Frames whose outputs repeat never share a launch: one shared output ends with
    the last frame's image, and a ring of 3 outputs holds the last 3 frames."""
    import torch
    w, h, k = 256, 160, 40
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    frames = [scenes.scene_a_bench(10 * i) for i in range(10)]
    ring = [torch.zeros((h, w, 4), dtype=torch.float32, device="cuda") for _ in range(3)]
    try:
        for b in (0, 16, 4):
            gpu_ctx.set_batch(b)
            for n_out in (1, 3):
                for r in ring:
                    r.zero_()
                torch.cuda.synchronize()
                gpu_ctx.render_frames_async(frames, eye, sh, w, h, k, 0, [ring[i % n_out].data_ptr()
                                                                         for i in range(len(frames))])
                gpu_ctx.synchronize()
                for j in range(n_out):
                    last = max(i for i in range(len(frames)) if i % n_out == j)
                    assert bits_equal(ring[j].cpu().numpy(), rtm.render_frame(frames[last], eye, sh, w, h, k))
    finally:
        gpu_ctx.set_batch(0)


def test_set_batch_api(rtm, gpu_ctx):
    for bad in (-1, 65):
        with pytest.raises(rtm.abi.RtmError) as e:
            gpu_ctx.set_batch(bad)
        assert e.value.code == rtm.abi.RTM_ERR_INVALID


@pytest.mark.parametrize("kind", ["spheres", "raytraced"])
def test_auto_batch_at_4k(rtm, scenes, gpu_ctx, kind):
    """The auto frames-per-launch rule at 3840x2160: 8 frames share a launch; 16
    frames make 2 batches, so 2 of the auto 4 lanes run (the full 4-lane headline
    is pinned to the oracle in test_headline_mode.py), spheres + patches or
    ray-traced primitives alike; every frame == rtm_render bit for bit."""
    import torch
    w, h, k = 3840, 2160, 64
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    if kind == "spheres":
        frames = [scenes.scene_a_bench(100 + i) for i in range(16)]
    else:
        frames = [scenes.mixed_rt(10 * i) for i in range(16)]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    try:
        gpu_ctx.set_batch(0)
        gpu_ctx.set_lanes(0)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, sh, w, h, k, 0, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
        assert gpu_ctx.last_batch() == 8
        assert gpu_ctx.last_lanes() == 2
        for s, o in zip(frames, outs):
            assert bits_equal(o.cpu().numpy(), rtm.render_frame(s, eye, sh, w, h, k)), "frame differs"
    finally:
        del outs
        torch.cuda.empty_cache()
