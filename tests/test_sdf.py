"""Row f-4 on the GPU: the GL preview's SDF implicit surface (distanceFn0,
entry.frag:416-442; the sphere-tracing leaf of bvhProcessLeafHit,
entry.frag:842-917) traced after the planes and cylinders of
processRaytracingRays, through the C ABI, against the CPU oracle.  The f64
semantics are the ones oracle/rtm_oracle.c fixes (GLSL leaves min/max/sign of
NaN and signed zero implementation-defined): parity is bit-exact RGBA f32 / f64
zBuffers and exact per-kind pixel and distance-evaluation counts.
"""
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _check(rtm, oracle, gpu_ctx, scenes, scene, eye, w, h, k=0, flags=None, stats=True):
    flags = scenes.RAYTRACING_FLAGS if flags is None else flags
    args = (scene, eye, scenes.shadow_camera(), w, h, k, flags)
    got = rtm.render_frame(*args)
    want = oracle.render(*args, nthreads=NT, want_stats=stats)
    assert bits_equal(got, want["rgba"]), first_mismatch(got, want["rgba"])
    if stats:
        st = gpu_ctx.stats(*args)
        # fused shadow: the shadow-pass counters cover only the texels the eye reads
        keys = [k for k in st if not (flags & scenes.abi.RTM_FLAG_FUSED_SHADOW and
                                      k in ("shadow_sphere_tests", "march_iterations", "march_hits", "march_in_range"))]
        assert {k: st[k] for k in keys} == {k: want["stats"][k] for k in keys}, \
            {k: (st[k], want["stats"][k]) for k in keys if st[k] != want["stats"][k]}
        return got, st
    return got, None


def test_preview_sdf_512(rtm, oracle, scenes, gpu_ctx):
    """The shader's one instance with its own constants (entry.frag:850-887)."""
    img, st = _check(rtm, oracle, gpu_ctx, scenes, scenes.sdf_preview_scene(), scenes.sdf_eye_camera(), 512, 512)
    assert st["eye_sdf_pixels"] > 1000 and st["eye_sdf_pixels"] == st["eye_hit_pixels"]
    assert st["sdf_distance_evals"] > 10 * st["eye_sdf_pixels"]


@pytest.mark.parametrize("wh", [(640, 360), (3840, 2160)])
def test_sdf_bench_scene(rtm, oracle, scenes, gpu_ctx, wh):
    """Scene S-bench (the row f-4 bench workload) incl. full size."""
    _, st = _check(rtm, oracle, gpu_ctx, scenes, scenes.sdf_bench_scene(), scenes.sdf_eye_camera(), *wh)
    assert st["eye_sdf_pixels"] > 0 and st["eye_circle_plane_pixels"] > 0


@pytest.mark.parametrize("flags", [0, 4])
def test_mixed_sdf_spheres_and_shadow(rtm, oracle, scenes, gpu_ctx, flags):
    """SDF hits against sphere depths under the orthographic eye, shadowed by the
    spheres + patch shadow map; two-pass and fused shadow."""
    _, st = _check(rtm, oracle, gpu_ctx, scenes, scenes.mixed_sdf(100), scenes.eye_camera(), 800, 600, 64, flags)
    assert st["eye_sdf_pixels"] > 100 and st["lit_pixels"] < st["eye_hit_pixels"]


def _random_sdf_scene(scenes, rng):
    def v3(lo, hi):
        return tuple(float(v) for v in rng.uniform(lo, hi, 3))

    n = int(rng.integers(1, scenes.abi.RTM_MAX_SDFS + 1))
    sdfs = []
    for i in range(n):
        c = v3(-1.0, 1.0)
        sdfs.append(scenes.PrimitiveSdf(i, scenes.Shading(*v3(0, 1)), c, tuple(np.add(c, v3(-1.2, 0.2))),
                                        tuple(np.add(c, v3(-0.3, 0.3))), v3(0.2, 1.5),
                                        int(rng.integers(0, 100))))
    for p, q in zip(sdfs, rng.permutation(n)):  # permuted ids: shading uses the id-th SDF
        p.id = int(q)
    cyl = scenes.PrimitiveCappedCylinder(0, scenes.Shading(0.3, 0.9, 0.3), v3(-1, 1), v3(-1, 1), 0.2, 0.3)
    return scenes.Scene([], [], [], [cyl] if rng.uniform() < 0.5 else [], sdfs)


@pytest.mark.parametrize("seed", range(6))
def test_random_sdf_scenes(rtm, oracle, scenes, gpu_ctx, seed):
    """Seeded fuzz (numpy PCG64, seed 0x2018+400+i): 1-8 SDFs with random
    anchors, AABBs (eye inside some), step caps 0-99 and permuted ids, maybe a
    cylinder, perspective eyes at random poses."""
    rng = np.random.default_rng(0x2018 + 400 + seed)
    scene = _random_sdf_scene(scenes, rng)
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    a, b, c, d = q
    R = np.array([[a*a+b*b-c*c-d*d, 2*(b*c-a*d), 2*(b*d+a*c)],
                  [2*(b*c+a*d), a*a-b*b+c*c-d*d, 2*(c*d-a*b)],
                  [2*(b*d-a*c), 2*(c*d+a*b), a*a-b*b-c*c+d*d]])
    pos = tuple(float(v) for v in rng.uniform(-0.3, 0.3, 3) - 3.0 * R[:, 2])
    eye = scenes.Camera(scenes.PERSPECTIVE, pos, tuple(map(float, R[:, 2])), tuple(map(float, R[:, 1])),
                        tuple(map(float, R[:, 0])))
    w, h = int(rng.integers(1, 300)), int(rng.integers(1, 240))
    _check(rtm, oracle, gpu_ctx, scenes, scene, eye, w, h)


def test_staged_sdf_matches_oracle(rtm, oracle, scenes, gpu_ctx):
    """Viewport.rasterize + processRaytracingRays + renderColorImage with SDFs
    (hit normals through the G-buffer) vs the oracle's staged API and the frame."""
    for scene, eye, w, h, k in ((scenes.sdf_bench_scene(), scenes.sdf_eye_camera(), 320, 200, 0),
                                (scenes.mixed_sdf(100), scenes.eye_camera(), 300, 200, 64)):
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


def test_sdf_step_cap_zero_and_eye_inside(rtm, oracle, scenes, gpu_ctx):
    """max_steps 0 (never hits), the eye inside the AABB (tIn < 0: no hit,
    entry.frag:858), an AABB behind the eye, and a degenerate zero extent."""
    S, F = scenes.Shading, scenes.PrimitiveSdf
    sdfs = [F(0, S(1, 0, 0), max_steps=0),
            F(1, S(0, 1, 0), (3.0, 0.3, 0.5), (3.5, 0.3, 1.5), (3.0, 0.3, 0.5), (1.0, 1.0, 1.0)),
            F(2, S(0, 0, 1), (3.0, 0.0, -4.0), (3.5, 0.0, -3.0), (3.0, 0.0, -4.0), (1.0, 1.0, 1.0)),
            F(3, S(1, 1, 0), (3.0, 0.0, 5.0), (3.5, 0.0, 6.0), (3.0, 0.0, 5.0), (0.0, 0.0, 0.0))]
    _check(rtm, oracle, gpu_ctx, scenes, scenes.Scene([], [], [], [], sdfs), scenes.sdf_eye_camera(), 200, 150)


def test_sdf_error_codes(rtm, scenes, gpu_ctx):
    abi = rtm.abi
    eye = scenes.sdf_eye_camera()
    for mutate in (lambda s: setattr(s.sdfPrimitives[0], "id", 1),
                   lambda s: setattr(s.sdfPrimitives[0], "max_steps", -1),
                   lambda s: setattr(s, "sdfPrimitives", [scenes.PrimitiveSdf(i, scenes.Shading(1, 1, 1))
                                                          for i in range(abi.RTM_MAX_SDFS + 1)])):
        s = scenes.sdf_preview_scene()
        mutate(s)
        with pytest.raises(abi.RtmError) as e:
            rtm.render_frame(s, eye, scenes.shadow_camera(), 32, 32, 0, scenes.RAYTRACING_FLAGS)
        assert e.value.code == abi.RTM_ERR_INVALID
    # staged: shading with a scene that lacks the traced SDF
    vp0 = rtm.Viewport(gpu_ctx, 32, 32, scenes.EnumFace.FRONT, eye)
    vp0.processRaytracingRays(scenes.sdf_preview_scene())
    vp1 = rtm.Viewport(gpu_ctx, 32, 32, scenes.EnumFace.BACK, scenes.shadow_camera())
    with pytest.raises(abi.RtmError) as e:
        rtm.renderColorImage(scenes.Scene([], []), vp0, vp1)
    assert e.value.code == abi.RTM_ERR_INVALID
