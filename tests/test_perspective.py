"""Row f-3 on the GPU: spheres under a PERSPECTIVE eye camera (Viewport::
rasterize's perspective branch, main.rs:473-530, with projectSphere,
main.rs:2796-2837, and nalgebra Perspective3 restated).  Parity is against the
CPU oracle and the independent numpy restatement's golden frames (the
reference itself cannot run here and has no output for this branch: parity
unpinned).  Bar: bit-exact.
"""
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _check(rtm, oracle, scene, eye, shadow, w, h, k, flags=0):
    got = rtm.render_frame(scene, eye, shadow, w, h, k, flags)
    want = oracle.render(scene, eye, shadow, w, h, k, flags, nthreads=NT)["rgba"]
    assert bits_equal(got, want), first_mismatch(got, want)
    return got


@pytest.mark.parametrize("which,wh", [(1, (512, 512)), (2, (512, 512)), (1, (3840, 2160)), (2, (333, 250))])
def test_perspective_simple_scenes(rtm, oracle, scenes, gpu_ctx, which, wh):
    """testscene_perspectiveSimple1/2 (main.rs:1059-1316), at the reference's
    512x512 and at other sizes (the aspect W/H enters Perspective3)."""
    scene = scenes.perspective_simple1() if which == 1 else scenes.perspective_simple2()
    eye = scenes.perspective_eye_camera() if which == 1 else scenes.perspective_simple2_camera()
    _check(rtm, oracle, scene, eye, scenes.shadow_camera(), *wh, 0, scenes.RAYTRACING_FLAGS)
    if wh == (512, 512):
        st = gpu_ctx.stats(scene, eye, scenes.shadow_camera(), 512, 512, 0, scenes.RAYTRACING_FLAGS)
        assert st["eye_hits"][:len(scene.spherePrimitives)] == ([8949] if which == 1 else [9607, 2185])


@pytest.mark.parametrize("flags", [0, 4])
def test_perspective_eye_with_shadows_and_primitives(rtm, oracle, scenes, flags):
    """Perspective spheres + ray-traced primitives + the orthographic shadow
    pass (spheres + patch), two-pass and fused."""
    s = scenes.perspective_simple2()
    s.patches = [scenes.BENCH_PATCH]
    s.circlePlanePrimitives = [scenes.dataclasses.replace(scenes.REFERENCE_CIRCLE_PLANE)]
    s.cappedCylinderPrimitives = [scenes.dataclasses.replace(scenes.REFERENCE_CAPPED_CYLINDER)]
    _check(rtm, oracle, s, scenes.perspective_simple2_camera(), scenes.shadow_camera(), 960, 540, 64, flags)


def test_perspective_staged_seams(rtm, oracle, scenes, gpu_ctx):
    """Viewport.rasterize with a PERSPECTIVE camera (staged API) == the oracle's
    staged viewport (zBuffer and image)."""
    scene = scenes.perspective_simple2()
    cam = scenes.perspective_simple2_camera()
    for w, h in ((512, 512), (300, 180)):
        vp0 = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.FRONT, cam)
        vp0.rasterize(scene)
        vp1 = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.BACK, scenes.shadow_camera())
        o0 = oracle.Viewport(w, h, scenes.EnumFace.FRONT, cam)
        o0.rasterize(scene)
        o1 = oracle.Viewport(w, h, scenes.EnumFace.BACK, scenes.shadow_camera())
        assert bits_equal(vp0.zBuffer(), o0.zbuffer())
        img = rtm.renderColorImage(scene, vp0, vp1)
        want = oracle.render_color_image(scene, o0, o1)
        assert bits_equal(img, want), first_mismatch(img, want)
        # face BACK under a perspective camera (a shadow-style viewport)
        vb = rtm.Viewport(gpu_ctx, w, h, scenes.EnumFace.BACK, cam)
        vb.rasterize(scene)
        ob = oracle.Viewport(w, h, scenes.EnumFace.BACK, cam)
        ob.rasterize(scene)
        assert bits_equal(vb.zBuffer(), ob.zbuffer())


def _rotation(rng):
    q = rng.normal(size=4)
    q /= np.linalg.norm(q)
    a, b, c, d = q
    return np.array([[a*a+b*b-c*c-d*d, 2*(b*c-a*d), 2*(b*d+a*c)],
                     [2*(b*c+a*d), a*a-b*b+c*c-d*d, 2*(c*d-a*b)],
                     [2*(b*d-a*c), 2*(c*d+a*b), a*a-b*b-c*c+d*d]])


@pytest.mark.parametrize("seed", range(10))
def test_random_perspective_scenes(rtm, oracle, scenes, seed):
    """Seeded fuzz (numpy PCG64, seed 0x2018+200+i): up to 16 spheres with
    permuted ids in front of, behind, around and enclosing a rotated
    PERSPECTIVE eye; ragged sizes (aspect != 1); the shadow pass on."""
    rng = np.random.default_rng(0x2018 + 200 + seed)
    R = _rotation(rng)
    pos = rng.uniform(-1, 1, 3)
    eye = scenes.Camera(scenes.PERSPECTIVE, tuple(map(float, pos)), tuple(map(float, R[:, 2])),
                        tuple(map(float, R[:, 1])), tuple(map(float, R[:, 0])))
    ns = int(rng.integers(1, 17))
    sph = []
    for i in range(ns):
        depth = float(rng.uniform(-2, 8))
        off = rng.uniform(-2, 2, 2)
        c = pos + R[:, 2] * depth + R[:, 0] * off[0] + R[:, 1] * off[1]
        sph.append(scenes.PrimitiveSphere(i, scenes.Shading(*map(float, rng.uniform(0, 1, 3))),
                                          tuple(map(float, c)), float(rng.uniform(0.05, 1.5))))
    for s_, p in zip(sph, rng.permutation(ns)):
        s_.id = int(p)
    scene = scenes.Scene(sph, [scenes.BENCH_PATCH])
    w, h = int(rng.integers(1, 420)), int(rng.integers(1, 300))
    _check(rtm, oracle, scene, eye, scenes.shadow_camera(), w, h, 40)
