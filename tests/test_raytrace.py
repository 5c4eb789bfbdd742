"""Row f-1 on the GPU: ray-traced circle planes and capped cylinders
(processRaytracingRays, main.rs:569-642; iCappedCone, main.rs:2889-2959;
calcRayPlane, main.rs:2398-2408) with PERSPECTIVE eye rays (main.rs:1922-1939),
through the C ABI, against the CPU oracle and the golden fixtures of the
independent numpy restatement.  Bar: bit-exact RGBA f32 / f64 zBuffers.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _oracle(oracle, scene, eye, shadow, w, h, k, flags=0, **kw):
    return oracle.render(scene, eye, shadow, w, h, k, flags, nthreads=NT, **kw)


def _check(rtm, oracle, scene, eye, shadow, w, h, k, flags=0):
    got = rtm.render_frame(scene, eye, shadow, w, h, k, flags)
    want = _oracle(oracle, scene, eye, shadow, w, h, k, flags)["rgba"]
    assert bits_equal(got, want), first_mismatch(got, want)
    return got


def _case(scenes, name):
    if name.startswith("rt_plane0_withplane"):
        return scenes.raytracing_plane0(True), scenes.perspective_eye_camera()
    if name.startswith("rt_plane0"):
        return scenes.raytracing_plane0(), scenes.perspective_eye_camera()
    if name.startswith("rt_rbench"):
        return scenes.scene_r_bench(), scenes.perspective_eye_camera()
    if name.startswith("f3_persp1"):
        return scenes.perspective_simple1(), scenes.perspective_eye_camera()
    if name.startswith("f3_persp2_rt"):
        s = scenes.perspective_simple2()
        s.circlePlanePrimitives = [scenes.dataclasses.replace(scenes.REFERENCE_CIRCLE_PLANE)]
        s.cappedCylinderPrimitives = [scenes.dataclasses.replace(scenes.REFERENCE_CAPPED_CYLINDER)]
        return s, scenes.perspective_simple2_camera()
    if name.startswith("f3_persp2"):
        return scenes.perspective_simple2(), scenes.perspective_simple2_camera()
    if name.startswith("f4_preview"):
        return scenes.sdf_preview_scene(), scenes.sdf_eye_camera()
    if name.startswith("f4_bench"):
        return scenes.sdf_bench_scene(), scenes.sdf_eye_camera()
    if name.startswith("f4_mixed_orbit"):
        return scenes.mixed_sdf(100), scenes.eye_camera()
    return scenes.mixed_rt(100), scenes.eye_camera()


def _rt_golden():
    with open(os.path.join(GOLD, "golden.json")) as f:
        return {k: v for k, v in json.load(f)["cases"].items() if k.startswith(("rt_", "f3_", "f4_"))}


@pytest.mark.parametrize("name", sorted(_rt_golden().keys()))
def test_golden_cases(rtm, scenes, name):
    """Every f-1 golden case of tests/golden (sha256 of the full RGBA f32 frame)."""
    g = _rt_golden()[name]
    scene, eye = _case(scenes, name)
    img = rtm.render_frame(scene, eye, scenes.shadow_camera(), g["width"], g["height"], g["steps"], g["flags"])
    assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == g["rgba_sha256"]


def test_raytracing_plane0_reference_512(rtm, oracle, scenes, gpu_ctx):
    """testscene_raytracingPlane0 exactly as main() renders it: 512x512,
    perspective eye, one capped cylinder, empty shadow map."""
    img = _check(rtm, oracle, scenes.raytracing_plane0(), scenes.perspective_eye_camera(), scenes.shadow_camera(),
                 512, 512, 0, scenes.RAYTRACING_FLAGS)
    st = gpu_ctx.stats(scenes.raytracing_plane0(), scenes.perspective_eye_camera(), scenes.shadow_camera(),
                       512, 512, 0, scenes.RAYTRACING_FLAGS)
    assert st["eye_capped_cylinder_pixels"] == st["eye_hit_pixels"] == st["lit_pixels"] == 3257
    assert st["eye_circle_plane_pixels"] == 0
    assert np.all(img[:256, :, 1] == np.float32(0.2))  # nothing below the view axis


@pytest.mark.parametrize("wh", [(512, 512), (3840, 2160)])
def test_raytracing_plane0_with_plane(rtm, oracle, scenes, wh):
    """The circle plane testscene_raytracingPlane0 has commented out, enabled."""
    _check(rtm, oracle, scenes.raytracing_plane0(True), scenes.perspective_eye_camera(), scenes.shadow_camera(),
           *wh, 0, scenes.RAYTRACING_FLAGS)


def test_scene_r_bench_4k(rtm, oracle, scenes, gpu_ctx):
    """The f-1 bench workload at full size, image and per-kind pixel counts."""
    args = (scenes.scene_r_bench(), scenes.perspective_eye_camera(), scenes.shadow_camera(), 3840, 2160, 0,
            scenes.RAYTRACING_FLAGS)
    got = rtm.render_frame(*args)
    want = _oracle(oracle, *args, want_stats=True)
    assert bits_equal(got, want["rgba"]), first_mismatch(got, want["rgba"])
    st, ws = gpu_ctx.stats(*args), want["stats"]
    cull = ("eye_plane_tests", "eye_cylinder_tests")
    assert {k: v for k, v in st.items() if k not in cull} == {k: v for k, v in ws.items() if k not in cull}
    # the per-wave cull (rt_wave_mask) skips most (pixel, primitive) tests; the oracle runs them all
    assert ws["eye_plane_tests"] == 3840 * 2160 * 4 and ws["eye_cylinder_tests"] == 3840 * 2160 * 9
    assert 0 < st["eye_plane_tests"] < ws["eye_plane_tests"]
    assert 0 < st["eye_cylinder_tests"] < ws["eye_cylinder_tests"] // 2


@pytest.mark.parametrize("flags", [0, 4])
def test_mixed_scene_1080p(rtm, oracle, scenes, gpu_ctx, flags):
    """Spheres + patch shadow map + planes + cylinders under the orthographic
    eye: ray-traced hits against sphere depths, shadowed ray-traced pixels;
    two-pass and fused shadow."""
    args = (scenes.mixed_rt(100), scenes.eye_camera(), scenes.shadow_camera(), 1920, 1080, 64, flags)
    got = rtm.render_frame(*args)
    want = _oracle(oracle, *args, want_stats=True)
    assert bits_equal(got, want["rgba"]), first_mismatch(got, want["rgba"])
    st = gpu_ctx.stats(*args)
    for key in ("eye_hit_pixels", "lit_pixels", "eye_hits", "eye_circle_plane_pixels", "eye_capped_cylinder_pixels"):
        assert st[key] == want["stats"][key], key
    assert st["eye_circle_plane_pixels"] > 1000 and st["eye_capped_cylinder_pixels"] > 1000
    assert st["lit_pixels"] < st["eye_hit_pixels"]


def test_mixed_row_bands(rtm, scenes, gpu_ctx):
    import torch
    w, h, k = 700, 333, 64
    scene = scenes.mixed_rt(40)
    full = rtm.render_frame(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k)
    parts = []
    for b0, b1 in ((0, 100), (100, 101), (101, 333)):
        out = torch.empty((b1 - b0, w, 4), dtype=torch.float32, device="cuda")
        torch.cuda.synchronize()
        gpu_ctx.render_async(scene, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, 0, out.data_ptr(), b0, b1)
        gpu_ctx.synchronize()
        parts.append(out.cpu().numpy())
    assert bits_equal(np.concatenate(parts, 0), full)


@pytest.mark.parametrize("lanes", [1, 2, 3])
def test_frames_async_with_raytraced_scenes(rtm, scenes, gpu_ctx, lanes):
    """A frame sequence whose scenes differ in ray-traced primitives, SDFs and
    spheres, spread over 1-3 lanes: each lane uploads each frame's primitive,
    SDF and (perspective eye) sphere tables into its own buffers, stream-ordered,
    and every frame matches rtm_render bit for bit."""
    import torch
    w, h, k = 640, 480, 64
    cases = [
        (scenes.eye_camera(), 0,
         [scenes.mixed_rt(f) for f in (0, 50, 100)] + [scenes.scene_a_bench(7), scenes.mixed_rt(9),
                                                        scenes.mixed_sdf(30), scenes.mixed_sdf(60)]),
        (scenes.perspective_eye_camera(), scenes.RAYTRACING_FLAGS,
         [scenes.perspective_simple1(), scenes.raytracing_plane0(True), scenes.perspective_simple2(),
          scenes.scene_r_bench(), scenes.raytracing_plane0()]),
    ]
    cases[0][2][1].cappedCylinderPrimitives = cases[0][2][1].cappedCylinderPrimitives[:1]
    try:
        gpu_ctx.set_batch(1)  # one frame per launch: the lanes carry single frames
        gpu_ctx.set_lanes(lanes)
        for eye, flags, frames in cases:
            outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
            torch.cuda.synchronize()
            gpu_ctx.render_frames_async(frames, eye, scenes.shadow_camera(), w, h, k, flags,
                                        [o.data_ptr() for o in outs])
            gpu_ctx.synchronize()
            assert gpu_ctx.last_lanes() == lanes
            for s, o in zip(frames, outs):
                want = rtm.render_frame(s, eye, scenes.shadow_camera(), w, h, k, flags)
                assert bits_equal(o.cpu().numpy(), want)
    finally:
        gpu_ctx.set_lanes(0)
        gpu_ctx.set_batch(0)


def test_staged_seams_match_oracle(rtm, oracle, scenes, gpu_ctx):
    """Viewport.rasterize + processRaytracingRays + renderColorImage, one call per
    reference function (main.rs:1033-1042), vs the oracle's staged API and the
    one-call frame."""
    for scene, eye, w, h, k in ((scenes.raytracing_plane0(True), scenes.perspective_eye_camera(), 512, 512, 0),
                                (scenes.mixed_rt(100), scenes.eye_camera(), 300, 200, 64)):
        vp1 = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.BACK, scenes.shadow_camera())
        o1 = oracle.Viewport(w, h, scenes.EnumFace.BACK, scenes.shadow_camera())
        if k:
            vp1.rasterize(scene)
            vp1.processRaymarchingRays(scene.patches, k)
            o1.rasterize(scene)
            o1.processRaymarchingRays(scene.patches, k)
        vp0 = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.FRONT, eye)
        vp0.rasterize(scene)
        vp0.processRaytracingRays(scene)
        o0 = oracle.Viewport(w, h, scenes.EnumFace.FRONT, eye)
        o0.rasterize(scene)
        o0.processRaytracingRays(scene)
        assert bits_equal(vp0.zBuffer(), o0.zbuffer())
        img = rtm.renderColorImage(scene, vp0, vp1)
        want = oracle.render_color_image(scene, o0, o1)
        assert bits_equal(img, want), first_mismatch(img, want)
        flags = 0 if k else scenes.RAYTRACING_FLAGS
        assert bits_equal(img, rtm.render_frame(scene, eye, scenes.shadow_camera(), w, h, k, flags))


def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    a, b, c, d = q
    return np.array([[a*a+b*b-c*c-d*d, 2*(b*c-a*d), 2*(b*d+a*c)],
                     [2*(b*c+a*d), a*a-b*b+c*c-d*d, 2*(c*d-a*b)],
                     [2*(b*d-a*c), 2*(c*d+a*b), a*a-b*b-c*c+d*d]])


def _random_rt_scene(scenes, rng, with_spheres):
    def col():
        return scenes.Shading(*[float(v) for v in rng.uniform(0, 1, 3)])

    def v3(lo, hi):
        return tuple(float(v) for v in rng.uniform(lo, hi, 3))

    npl, ncy = int(rng.integers(0, 17)), int(rng.integers(0, 17))
    planes = [scenes.PrimitiveCirclePlane(i, col(), float(rng.uniform(0.05, 1.5)), v3(-1, 1),
                                          scenes.normalize(v3(-1, 1))) for i in range(npl)]
    cyls = []
    for i in range(ncy):
        ra = float(rng.uniform(0.02, 0.5))
        rb = ra if rng.uniform() < 0.2 else float(rng.uniform(0.02, 0.5))  # rr == 0 (a true cylinder) too
        cyls.append(scenes.PrimitiveCappedCylinder(i, col(), v3(-1, 1), v3(-1, 1), ra, rb))
    # permuted ids: shading uses the id-th primitive (main.rs:773, 791)
    for prims in (planes, cyls):
        for p, q in zip(prims, rng.permutation(len(prims))):
            p.id = int(q)
    sph = []
    if with_spheres:
        for i in range(int(rng.integers(0, 6))):
            sph.append(scenes.PrimitiveSphere(i, col(), v3(-0.8, 0.8), float(rng.uniform(0.05, 0.4))))
    pats = [scenes.BENCH_PATCH] if with_spheres else []
    return scenes.Scene(sph, pats, planes, cyls)


@pytest.mark.parametrize("seed", range(10))
def test_random_raytraced_scenes(rtm, oracle, scenes, seed):
    """Seeded fuzz (numpy PCG64, seed 0x2018+100+i): up to 16 planes and 16
    cylinders with permuted ids, perspective eyes at random poses (even seeds)
    or rotated orthographic eyes with spheres + a patch (odd seeds)."""
    rng = np.random.default_rng(0x2018 + 100 + seed)
    persp = seed % 2 == 0
    scene = _random_rt_scene(scenes, rng, not persp)
    R = _rotation(rng)
    if persp:
        pos = tuple(float(v) for v in rng.uniform(-0.3, 0.3, 3) - 2.5 * R[:, 2])
        eye = scenes.Camera(scenes.PERSPECTIVE, pos, tuple(map(float, R[:, 2])), tuple(map(float, R[:, 1])),
                            tuple(map(float, R[:, 0])))
    else:
        eye = scenes.Camera(scenes.ORTHOGONAL, tuple(float(v) for v in -1.5 * R[:, 2]), tuple(map(float, R[:, 2])),
                            tuple(map(float, R[:, 1])), tuple(map(float, R[:, 0])))
    w, h = int(rng.integers(1, 420)), int(rng.integers(1, 300))
    flags = scenes.RAYTRACING_FLAGS if persp else 0
    _check(rtm, oracle, scene, eye, scenes.shadow_camera(), w, h, 48, flags)


def test_degenerate_primitives(rtm, oracle, scenes):
    """Planes parallel to the rays (|denom| <= 1e-4 -> None), a zero-length
    cylinder (baba = 0: inversesqrt = inf), zero radii, primitives behind and
    enclosing the camera, exact ties between a plane and a cylinder cap."""
    S, P, C = scenes.Shading, scenes.PrimitiveCirclePlane, scenes.PrimitiveCappedCylinder
    planes = [P(0, S(1, 0, 0), 1.0, (0.0, 0.0, 3.0), (1.0, 0.0, 0.0)),            # parallel to the view axis
              P(1, S(0, 1, 0), 0.0, (0.0, 0.0, 2.0), (0.0, 0.0, 1.0)),            # zero radius
              P(2, S(0, 0, 1), 5.0, (0.0, 0.0, -1.0), (0.0, 0.0, 1.0)),           # behind the camera
              P(3, S(1, 1, 0), 0.3, (0.2, 0.2, 4.0), (0.0, 0.0, -1.0))]           # faces the camera
    cyls = [C(0, S(1, 0, 1), (0.1, 0.1, 2.0), (0.1, 0.1, 2.0), 0.2, 0.2),          # pA == pB
            C(1, S(0, 1, 1), (0.2, 0.2, 4.0), (0.2, 0.2, 5.0), 0.3, 0.3),          # cap A coincides with plane 3
            C(2, S(1, 1, 1), (0.0, 0.0, -5.0), (0.0, 0.0, 50.0), 4.0, 4.0),        # encloses the camera
            C(3, S(0.5, 0.5, 0.5), (-0.5, 0.0, 3.0), (-0.5, 0.0, 3.5), 0.0, 0.2)]  # cone tip
    scene = scenes.Scene([], [], planes, cyls)
    for eye in (scenes.perspective_eye_camera(),
                scenes.Camera(scenes.ORTHOGONAL, (0.0, 0.0, 0.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0), (1.0, 0.0, 0.0))):
        _check(rtm, oracle, scene, eye, scenes.shadow_camera(), 257, 193, 0, scenes.RAYTRACING_FLAGS)


@pytest.mark.parametrize("seed", range(6))
def test_wave_cull_stress(rtm, oracle, scenes, seed):
    """The per-wave primitive cull of the PERSPECTIVE eye pass (rt_wave_mask):
    many small primitives scattered over the frustum so that most waves cull
    most of them, primitives straddling the wave and frame edges, behind the
    camera, enclosing it, near-cylinders (|rb - ra| tiny or 0: never culled)
    and a frame width that leaves a partial last wave.  Bit-exact vs the
    oracle, which has no cull."""
    rng = np.random.default_rng(0x2018 + 300 + seed)
    S, P, C = scenes.Shading, scenes.PrimitiveCirclePlane, scenes.PrimitiveCappedCylinder

    def col():
        return S(*(float(v) for v in rng.uniform(0.05, 1.0, 3)))

    def front(zlo, zhi):
        z = float(rng.uniform(zlo, zhi))
        return (float(rng.uniform(-1.1, 1.1) * z), float(rng.uniform(-1.1, 1.1) * z), z)

    planes, cyls = [], []
    for i in range(16):
        c = front(0.5, 12.0) if i else (0.0, 0.0, -2.0)  # plane 0 behind the camera
        n = rng.normal(size=3)
        n /= np.linalg.norm(n)
        planes.append(P(i, col(), float(rng.uniform(0.01, 0.4)), c, tuple(float(v) for v in n)))
    for i in range(16):
        a = front(0.5, 12.0)
        d = rng.normal(size=3) * rng.uniform(0.05, 1.5)
        b = (a[0] + float(d[0]), a[1] + float(d[1]), a[2] + float(d[2]))
        ra = float(rng.uniform(0.01, 0.3))
        kind = i % 4
        rb = ra if kind == 0 else ra * (1.0 + 1e-5) if kind == 1 else float(rng.uniform(0.01, 0.3))
        if i == 15:  # encloses the camera origin
            a, b, ra, rb = (0.0, 0.0, -1.0), (0.0, 0.0, 1.0), 0.5, 0.4
        cyls.append(C(i, col(), a, b, ra, rb))
    ids = rng.permutation(16)
    for i, p in enumerate(planes):
        p.id = int(ids[i])
    scene = scenes.Scene([], [], planes, cyls)
    w, h = (961, 541) if seed % 2 == 0 else (1283, 97)
    _check(rtm, oracle, scene, scenes.perspective_eye_camera(), scenes.shadow_camera(), w, h, 0,
           scenes.RAYTRACING_FLAGS)


@pytest.mark.parametrize("seed", range(4))
def test_capsule_cull_stress(rtm, oracle, scenes, seed):
    """The cylinders' capsule cull (capsule_culls): long, thin capped cones in every
    orientation -- along the view direction, across it, through the frustum's edges,
    grazing wave rows, one passing next to the camera -- whose capsules the wave
    cones just miss or just meet.  Bit-exact vs the oracle, which has no cull."""
    rng = np.random.default_rng(0x2018 + 400 + seed)
    S, C = scenes.Shading, scenes.PrimitiveCappedCylinder
    cyls = []
    for i in range(16):
        z = float(rng.uniform(1.0, 14.0))
        a = (float(rng.uniform(-1.2, 1.2) * z), float(rng.uniform(-1.2, 1.2) * z), z)
        d = rng.normal(size=3)
        d *= rng.uniform(1.0, 12.0) / np.linalg.norm(d)
        if i % 4 == 0:  # along the view direction
            d = np.array([0.0, 0.0, float(rng.uniform(2.0, 10.0))])
        b = (a[0] + float(d[0]), a[1] + float(d[1]), a[2] + float(d[2]))
        ra = float(rng.uniform(0.002, 0.15))
        rb = float(rng.uniform(0.002, 0.15))
        if i == 15:  # passes 0.2 from the camera origin
            a, b, ra, rb = (-3.0, 0.2, 0.0), (3.0, 0.2, 0.5), 0.05, 0.12
        cyls.append(C(i, S(*(float(v) for v in rng.uniform(0.05, 1.0, 3))), a, b, ra, rb))
    scene = scenes.Scene([], [], [], cyls)
    w, h = (640, 480) if seed % 2 == 0 else (1283, 97)
    _check(rtm, oracle, scene, scenes.perspective_eye_camera(), scenes.shadow_camera(), w, h, 0,
           scenes.RAYTRACING_FLAGS)


def test_raytrace_error_codes(rtm, scenes, gpu_ctx):
    abi = rtm.abi
    # a perspective shadow camera: Camera::project asserts ORTHOGONAL (main.rs:1949)
    with pytest.raises(abi.RtmError) as e:
        rtm.render_frame(scenes.raytracing_plane0(), scenes.perspective_eye_camera(),
                         scenes.perspective_eye_camera(), 64, 64, 0)
    assert e.value.code == abi.RTM_ERR_UNSUPPORTED
    # id out of range (the reference would index past the array and panic)
    s = scenes.raytracing_plane0(True)
    s.circlePlanePrimitives[0].id = 1
    with pytest.raises(abi.RtmError) as e:
        rtm.render_frame(s, scenes.perspective_eye_camera(), scenes.shadow_camera(), 64, 64, 0)
    assert e.value.code == abi.RTM_ERR_INVALID
    # too many cylinders
    s = scenes.raytracing_plane0()
    s.cappedCylinderPrimitives = [scenes.PrimitiveCappedCylinder(i, scenes.Shading(1, 1, 1), (0, 0, 1), (0, 1, 1),
                                                                 0.1, 0.1) for i in range(17)]
    with pytest.raises(abi.RtmError) as e:
        rtm.render_frame(s, scenes.perspective_eye_camera(), scenes.shadow_camera(), 64, 64, 0)
    assert e.value.code == abi.RTM_ERR_INVALID
    # staged: shading with a scene that lacks the traced primitives
    vp0 = rtm.Viewport(gpu_ctx, 64, 64, scenes.EnumFace.FRONT, scenes.perspective_eye_camera())
    vp0.processRaytracingRays(scenes.raytracing_plane0(True))
    vp1 = rtm.Viewport(gpu_ctx, 64, 64, scenes.EnumFace.BACK, scenes.shadow_camera())
    with pytest.raises(abi.RtmError) as e:
        rtm.renderColorImage(scenes.raytracing_plane0(False), vp0, vp1)
    assert e.value.code == abi.RTM_ERR_INVALID


def test_viewport_outliving_its_context(rtm, scenes):
    """A viewport whose context is destroyed first: calls fail cleanly, destroy
    still frees it (no use-after-free of the context)."""
    abi = rtm.abi
    ctx = rtm.Context(0)
    vp = rtm.Viewport(ctx, 32, 32, scenes.EnumFace.FRONT, scenes.perspective_eye_camera())
    vp.processRaytracingRays(scenes.raytracing_plane0())
    ctx.close()
    with pytest.raises(abi.RtmError) as e:
        vp.processRaytracingRays(scenes.raytracing_plane0())
    assert e.value.code == abi.RTM_ERR_INVALID
    with pytest.raises(abi.RtmError):
        vp.zBuffer()
    vp.close()


@pytest.mark.parametrize("batch,lanes", [(3, 1), (4, 2), (16, 1)])
def test_batched_perspective_raytraced_frames(rtm, scenes, gpu_ctx, batch, lanes):
    """Batched launches of PERSPECTIVE-eye frames with ray-traced primitives: the
    per-wave primitive masks are computed per frame of the batch
    (rt_cull_batch_kernel) and every frame == rtm_render bit for bit, including
    frames without primitives and with spheres only inside the same batch."""
    import torch
    w, h, k = 512, 384, 64
    eye, sh = scenes.perspective_eye_camera(), scenes.shadow_camera()
    frames = [scenes.raytracing_plane0(), scenes.scene_r_bench(), scenes.raytracing_plane0(True),
              scenes.perspective_simple1(), scenes.scene_r_bench(), scenes.raytracing_plane0(),
              scenes.perspective_simple2(), scenes.raytracing_plane0(True)]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    try:
        gpu_ctx.set_batch(batch)
        gpu_ctx.set_lanes(lanes)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, sh, w, h, k, scenes.RAYTRACING_FLAGS, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
        assert gpu_ctx.last_batch() == min(batch, len(frames))
        for s, o in zip(frames, outs):
            want = rtm.render_frame(s, eye, sh, w, h, k, scenes.RAYTRACING_FLAGS)
            assert bits_equal(o.cpu().numpy(), want)
    finally:
        gpu_ctx.set_lanes(0)
        gpu_ctx.set_batch(0)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["rt", "sdf"])
def test_batched_repeated_frames_share_tables(rtm, scenes, gpu_ctx, kind):
    """A batch whose consecutive frames carry equal primitive tables uploads each
    run of equal tables once and points the frames at it (enqueue_batch); runs of
    repeats, changes back and forth and a lone last frame all == rtm_render bit for
    bit."""
    import torch
    w, h, k = 256, 192, 64
    if kind == "rt":
        eye, flags = scenes.perspective_eye_camera(), scenes.RAYTRACING_FLAGS
        a, b, c = scenes.raytracing_plane0(), scenes.scene_r_bench(), scenes.perspective_simple1()
    else:
        eye, flags = scenes.sdf_eye_camera(), 0
        a, b, c = scenes.sdf_preview_scene(), scenes.sdf_bench_scene(), scenes.mixed_sdf(101)
    sh = scenes.shadow_camera()
    frames = [a, a, a, b, b, a, c, c, b, a]
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    try:
        gpu_ctx.set_batch(len(frames))
        gpu_ctx.set_lanes(1)
        torch.cuda.synchronize()
        gpu_ctx.render_frames_async(frames, eye, sh, w, h, k, flags, [o.data_ptr() for o in outs])
        gpu_ctx.synchronize()
        assert gpu_ctx.last_batch() == len(frames)
        for i, (s, o) in enumerate(zip(frames, outs)):
            want = rtm.render_frame(s, eye, sh, w, h, k, flags)
            got = o.cpu().numpy()
            assert bits_equal(got, want), (i, first_mismatch(got, want))
    finally:
        gpu_ctx.set_lanes(0)
        gpu_ctx.set_batch(0)
