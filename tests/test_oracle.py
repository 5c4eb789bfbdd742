"""CPU tests of the oracle itself: pinned against SURVEY.md §8c-3, the golden
fixtures of the independent numpy restatement (tests/golden/gen_golden.py) and
the reference's own unit test for calcRayPlane (main.rs:2415-2425)."""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def sha16(img):
    return hashlib.sha256(np.ascontiguousarray(img[:, :, :3]).tobytes()).hexdigest()[:16]


def _case(scenes, name):
    """(scene, eye camera) of a golden case."""
    if name.startswith("rt_plane0_withplane"):
        return scenes.raytracing_plane0(True), scenes.perspective_eye_camera()
    if name.startswith("rt_plane0"):
        return scenes.raytracing_plane0(), scenes.perspective_eye_camera()
    if name.startswith("rt_rbench"):
        return scenes.scene_r_bench(), scenes.perspective_eye_camera()
    if name.startswith("rt_mixed_orbit"):
        return scenes.mixed_rt(100), scenes.eye_camera()
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
    return _scene_for(scenes, name), scenes.eye_camera()


def _scene_for(scenes, name):
    if name.startswith("orbit_f0"):
        return scenes.closely_orbiting_sphere(0)
    if name.startswith("orbit_f100"):
        return scenes.closely_orbiting_sphere(100)
    if name.startswith("orbit_f250"):
        return scenes.closely_orbiting_sphere(250)
    if name.startswith("bench_f100"):
        return scenes.scene_a_bench(100)
    if name.startswith("bench_f37"):
        return scenes.scene_a_bench(37)
    if name.startswith("sceneb"):
        return scenes.scene_b()
    if name.startswith("overlap"):
        return scenes.overlapping_spheres()
    if name.startswith("cfg1"):
        return scenes.closely_orbiting_sphere(100)
    raise KeyError(name)


@pytest.mark.parametrize("frame,hits,lit,sha", [(0, [8014, 6372, 659], 0, "cf557d736f83a4f6"),
                                                (100, [8245, 6580, 2059], 2059, "cb7008f728da5208")])
def test_survey_kats(oracle, scenes, frame, hits, lit, sha):
    r = oracle.render(scenes.closely_orbiting_sphere(frame), scenes.eye_camera(), scenes.shadow_camera(),
                      512, 512, 500, 0, want_shadow=True, want_stats=True)
    assert r["stats"]["eye_hits"][:3] == hits
    assert r["stats"]["lit_pixels"] == lit
    assert sha16(r["rgba"]) == sha
    if frame == 0:
        img = r["rgba"]
        assert img[256, 384, :3].tolist() == [9265101144064.0, 9265101144064.0, 463255038328832.0]
        assert img[0, 0, :3].tolist() == [0.0, np.float32(0.2), np.float32(0.2)]
        assert img[300, 384, :3].tolist() == [3506.7421875, 3506.7421875, 175337.109375]
        # the march hits after exactly 4 advances: t = 0.12 everywhere
        assert np.all(r["shadow"] == 0.12)
        assert r["stats"]["march_iterations"] == 512 * 512 * 5


def _golden():
    with open(os.path.join(GOLD, "golden.json")) as f:
        return json.load(f)["cases"]


@pytest.mark.parametrize("name", sorted(_golden().keys()))
def test_oracle_matches_golden(oracle, scenes, name):
    g = _golden()[name]
    scene, eye = _case(scenes, name)
    r = oracle.render(scene, eye, scenes.shadow_camera(), g["width"], g["height"], g["steps"], g["flags"],
                      nthreads=4, want_shadow=True, want_stats=True)
    assert hashlib.sha256(np.ascontiguousarray(r["rgba"]).tobytes()).hexdigest() == g["rgba_sha256"]
    assert hashlib.sha256(np.ascontiguousarray(r["shadow"]).tobytes()).hexdigest() == g["shadow_sha256"]
    assert r["stats"]["eye_hits"][:len(g["eye_hits"])] == g["eye_hits"]
    assert r["stats"]["lit_pixels"] == g["lit_pixels"]
    if "circle_plane_pixels" in g:
        assert r["stats"]["eye_circle_plane_pixels"] == g["circle_plane_pixels"]
        assert r["stats"]["eye_capped_cylinder_pixels"] == g["capped_cylinder_pixels"]
    if "sdf_pixels" in g:
        assert r["stats"]["eye_sdf_pixels"] == g["sdf_pixels"]


def test_oracle_matches_fixture_arrays(oracle, scenes):
    fx = np.load(os.path.join(GOLD, "fixtures.npz"))
    names = sorted({k.split("__")[0] for k in fx.files})
    assert len(names) >= 6
    for name in names:
        g = _golden()[name]
        scene, eye = _case(scenes, name)
        r = oracle.render(scene, eye, scenes.shadow_camera(), g["width"], g["height"], g["steps"], g["flags"],
                          want_shadow=True)
        assert bits_equal(r["rgba"], fx[name + "__rgba"]), (name, first_mismatch(r["rgba"], fx[name + "__rgba"]))
        assert bits_equal(r["shadow"], fx[name + "__shadow"]), name


@pytest.mark.parametrize("frame", [0, 100, 199])
def test_reference_bbox_is_a_pure_cull(oracle, scenes, frame):
    """rasterizeSphere's bbox (main.rs:256-300) changes nothing on square images
    (SURVEY.md §8a-0): the generalised per-pixel test equals the reference loop."""
    args = (scenes.closely_orbiting_sphere(frame), scenes.eye_camera(), scenes.shadow_camera(), 512, 512, 500)
    a = oracle.render(*args, 0, want_shadow=True)
    b = oracle.render(*args, oracle.RTMO_FLAG_REF_BBOX, want_shadow=True)
    assert bits_equal(a["rgba"], b["rgba"]) and bits_equal(a["shadow"], b["shadow"])


def test_threads_do_not_change_bits(oracle, scenes):
    args = (scenes.scene_b(), scenes.eye_camera(), scenes.shadow_camera(), 333, 221, 128, 0)
    a = oracle.render(*args, nthreads=1, want_shadow=True, want_stats=True)
    b = oracle.render(*args, nthreads=8, want_shadow=True, want_stats=True)
    assert bits_equal(a["rgba"], b["rgba"]) and bits_equal(a["shadow"], b["shadow"])
    assert a["stats"] == b["stats"]


def test_staged_oracle_equals_frame_oracle(oracle, scenes):
    """Driving the three reference seams one by one == the one-call frame."""
    scene = scenes.closely_orbiting_sphere(100)
    vp1 = oracle.Viewport(200, 160, scenes.EnumFace.BACK, scenes.shadow_camera())
    vp1.rasterize(scene)
    vp1.processRaymarchingRays([scenes.REFERENCE_PATCH], 500)
    vp0 = oracle.Viewport(200, 160, scenes.EnumFace.FRONT, scenes.eye_camera())
    vp0.rasterize(scene)
    img = oracle.render_color_image(scene, vp0, vp1)
    r = oracle.render(scene, scenes.eye_camera(), scenes.shadow_camera(), 200, 160, 500, 0, want_shadow=True)
    assert bits_equal(img, r["rgba"])
    assert bits_equal(vp1.zbuffer(), r["shadow"])


def test_reference_unit_test_calc_ray_plane(oracle):
    """test_planeEquation (main.rs:2415-2425): t must be exactly 1.5."""
    t = oracle.calc_ray_plane((-1.0, 0.0, 0.0), (1.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.5, 0.0, 0.0))
    assert t == 1.5
    # |denom| <= 1e-4 -> None (main.rs:2403)
    assert oracle.calc_ray_plane((0.0, 0.0, 0.0), (0.0, 1.0, 0.0), (1.0, 0.0, 0.0), (0.5, 0.0, 0.0)) is None


def test_no_march_and_no_raster_flags(oracle, scenes):
    s = scenes.closely_orbiting_sphere(100)
    r = oracle.render(s, scenes.eye_camera(), scenes.shadow_camera(), 64, 64, 500, 3, want_shadow=True,
                      want_stats=True)
    assert np.all(np.isinf(r["shadow"]))
    assert r["stats"]["march_iterations"] == 0
    # nothing is shadowed with an empty shadow map
    assert r["stats"]["lit_pixels"] == r["stats"]["eye_hit_pixels"]


def test_perspective_shadow_camera_is_unsupported(oracle, scenes):
    """Camera::project asserts an ORTHOGONAL camera (main.rs:1949)."""
    with pytest.raises(RuntimeError):
        oracle.render(scenes.scene_a_bench(), scenes.eye_camera(), scenes.perspective_eye_camera(), 16, 16, 8, 0)


def test_perspective_simple_kats(oracle, scenes):
    """testscene_perspectiveSimple1/2 at 512x512 (row f-3): per-sphere pixel
    counts shared with the independent numpy restatement; the disc of scene 1
    is centred (the sphere sits on the view axis up to 0.01)."""
    r = oracle.render(scenes.perspective_simple1(), scenes.perspective_eye_camera(), scenes.shadow_camera(),
                      512, 512, 0, scenes.RAYTRACING_FLAGS, want_stats=True)
    assert r["stats"]["eye_hits"][:1] == [8949]
    ys, xs = np.nonzero(r["rgba"][..., 1] != np.float32(0.2))
    assert (xs.min(), xs.max(), ys.min(), ys.max()) == (204, 310, 204, 310)
    r = oracle.render(scenes.perspective_simple2(), scenes.perspective_simple2_camera(), scenes.shadow_camera(),
                      512, 512, 0, scenes.RAYTRACING_FLAGS, want_stats=True)
    assert r["stats"]["eye_hits"][:2] == [9607, 2185]


def test_raytracing_plane0_kats(oracle, scenes):
    """testscene_raytracingPlane0 at the reference's 512x512: the cylinder covers
    3257 pixels (independent numpy restatement: tests/golden/gen_golden.py), all
    lit (the shadow map stays +INF), the rest is background."""
    r = oracle.render(scenes.raytracing_plane0(), scenes.perspective_eye_camera(), scenes.shadow_camera(),
                      512, 512, 0, scenes.RAYTRACING_FLAGS, want_stats=True)
    st = r["stats"]
    assert st["eye_capped_cylinder_pixels"] == st["eye_hit_pixels"] == st["lit_pixels"] == 3257
    img = r["rgba"]
    # the cylinder is above the view axis (pA.y = 10.01): no hit in the lower half
    assert np.all(img[:256, :, 0] == 0.0) and np.all(img[:256, :, 1] == np.float32(0.2))


def test_icapped_cone_known_answers(oracle):
    """iCappedCone (main.rs:2889-2959) on analytic cases."""
    # straight at cap A of a unit cylinder along z: t = 5, n = -ba/|ba| (signed zeros as computed)
    t, n = oracle.icapped_cone((0, 0, -5), (0, 0, 1), (0, 0, 0), (0, 0, 1), 0.5, 0.5)
    assert t == 5.0 and n == (-0.0, -0.0, -1.0)
    # cap B from above: t = 4
    t, n = oracle.icapped_cone((0, 0, 5), (0, 0, -1), (0, 0, 0), (0, 0, 1), 0.5, 0.5)
    assert t == 4.0 and n == (0.0, 0.0, 1.0)
    # body of a cone: radius 0.25 halfway up -> t ~ 4.75, normal tilted by the slope 0.1
    t, n = oracle.icapped_cone((-5, 0, 0.5), (1, 0, 0), (0, 0, 0), (0, 0, 1), 0.3, 0.2)
    assert abs(t - 4.75) < 1e-12 and abs(n[0] + 1 / np.sqrt(1.01)) < 1e-12 and abs(n[2] - 0.1 / np.sqrt(1.01)) < 1e-12
    # miss: (-1, -1, -1, -1)
    assert oracle.icapped_cone((-5, 3, 0.5), (1, 0, 0), (0, 0, 0), (0, 0, 1), 0.3, 0.2) == (-1.0, (-1.0, -1.0, -1.0))


def test_icapped_cone_matches_independent_restatement(oracle):
    """C oracle == numpy restatement (gen_golden.icapped_cone) bit for bit on random rays."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_golden", os.path.join(GOLD, "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    rng = np.random.default_rng(0x2018)
    for _ in range(8):
        pa, pb = rng.uniform(-1, 1, 3), rng.uniform(-1, 1, 3)
        ra, rb = rng.uniform(0.05, 0.6, 2)
        ro = rng.uniform(-3, 3, (200, 3))
        rd = rng.normal(size=(200, 3))
        rd /= np.linalg.norm(rd, axis=1, keepdims=True)
        t_np, n_np = gg.icapped_cone([ro[:, k] for k in range(3)], [rd[:, k] for k in range(3)], pa, pb, ra, rb)
        for i in range(200):
            t, n = oracle.icapped_cone(ro[i], rd[i], pa, pb, ra, rb)
            assert np.float64(t).tobytes() == np.float64(t_np[i]).tobytes(), i
            assert all(np.float64(n[k]).tobytes() == np.float64(n_np[k][i]).tobytes() for k in range(3)), i


def test_staged_raytracing_equals_frame(oracle, scenes):
    """rasterize + processRaytracingRays + renderColorImage == the frame (mixed scene)."""
    scene = scenes.mixed_rt(100)
    vp1 = oracle.Viewport(120, 90, scenes.EnumFace.BACK, scenes.shadow_camera())
    vp1.rasterize(scene)
    vp1.processRaymarchingRays(scene.patches, 64)
    vp0 = oracle.Viewport(120, 90, scenes.EnumFace.FRONT, scenes.eye_camera())
    vp0.rasterize(scene)
    vp0.processRaytracingRays(scene)
    img = oracle.render_color_image(scene, vp0, vp1)
    r = oracle.render(scene, scenes.eye_camera(), scenes.shadow_camera(), 120, 90, 64, 0)
    assert bits_equal(img, r["rgba"])


def test_encode_rgb8_ppm_pixel_rule(oracle):
    """writeColorImage's per-channel encode (main.rs:674-684)."""
    rgba = np.array([[0.0, 0.5, 1.0, 1.0], [2.0, -1.0, np.nan, 1.0], [1e15, 0.2, 0.01, 1.0]], np.float32)
    out = oracle.encode_rgb8(rgba)
    assert out[0].tolist() == [0, int(np.float32(np.float32(0.5) ** np.float32(1 / 2.2)) * 255), 255] or out[0][0] == 0
    assert out[1][0] == 255 and out[1][1] == 0
    assert out[2][0] == 255


def test_sdf_known_answers(oracle, scenes):
    """The preview SDF (entry.frag:416-442, 842-905) restated in f64: distance
    inside / outside the box, a trace straight at the box's front face (which
    the thickening puts at z = 5 - 0.2 - 0.2), a ray that misses the AABB, a ray
    from inside the AABB (the shader's tIn < 0 -> no hit, entry.frag:855-858)."""
    q = scenes.PREVIEW_SDF
    assert oracle.sdf_distance(q, (3.0, 0.0, 5.0)) == -0.4      # box centre: -0.2 (inside) - 0.2
    assert abs(oracle.sdf_distance(q, (3.0, 0.0, 0.0)) - 4.6) < 1e-12
    t, n = oracle.sdf_trace(q, (3.0, 0.05, 0.5), (0.0, 0.0, 1.0))
    assert abs(t - 4.1) < 0.03 and n == (0.0, 0.0, -1.0)
    assert oracle.sdf_trace(q, (3.0, 5.0, 0.5), (0.0, 0.0, 1.0))[0] == -1.0   # above the AABB
    assert oracle.sdf_trace(q, (3.0, 0.0, 3.0), (0.0, 0.0, 1.0))[0] == -1.0   # starts inside the AABB


def test_sdf_matches_independent_restatement(oracle, scenes):
    """C oracle trace == numpy restatement (gen_golden.trace_sdf) bit for bit on random rays."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_golden", os.path.join(GOLD, "gen_golden.py"))
    gg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gg)
    rng = np.random.default_rng(0x2018 + 4)
    q = scenes.PREVIEW_SDF
    sd = (0, q.box_center, q.tri_anchor, q.aabb_center, q.aabb_extent, (1.0, 1.0, 1.0), q.max_steps)
    ro = np.stack([rng.uniform(1.0, 5.0, 300), rng.uniform(-1.0, 1.5, 300), rng.uniform(-1.0, 1.5, 300)], 1)
    tgt = np.stack([rng.uniform(2.2, 5.0, 300), rng.uniform(-0.5, 1.0, 300), rng.uniform(4.5, 7.0, 300)], 1)
    rd = tgt - ro
    rd /= np.linalg.norm(rd, axis=1, keepdims=True)
    t_np, n_np = gg.trace_sdf(sd, [ro[:, k] for k in range(3)], [rd[:, k] for k in range(3)])
    hits = 0
    for i in range(300):
        t, n = oracle.sdf_trace(q, ro[i], rd[i])
        assert np.float64(t).tobytes() == np.float64(t_np[i]).tobytes(), i
        if t >= 0:
            hits += 1
            assert all(np.float64(n[k]).tobytes() == np.float64(n_np[k][i]).tobytes() for k in range(3)), i
    assert hits > 50


@pytest.mark.parametrize("case", ["bench", "sceneb", "rbench", "sdf"])
def test_render_rows_matches_full_frame(oracle, scenes, case):
    """The row-window oracle (used for maximum-size GPU parity) reproduces the
    full frame's rows bit for bit, shadow rows computed on demand."""
    if case == "bench":
        args = (scenes.scene_a_bench(), scenes.eye_camera(), scenes.shadow_camera(), 320, 181, 64, 0)
    elif case == "sceneb":
        args = (scenes.scene_b(), scenes.eye_camera(), scenes.shadow_camera(), 200, 150, 128, 0)
    elif case == "rbench":
        args = (scenes.scene_r_bench(), scenes.perspective_eye_camera(), scenes.shadow_camera(), 160, 90, 0,
                scenes.RAYTRACING_FLAGS)
    else:
        args = (scenes.mixed_sdf(100), scenes.eye_camera(), scenes.shadow_camera(), 120, 96, 64, 0)
    full = oracle.render(*args, nthreads=4)["rgba"]
    H = args[4]
    for r0, r1 in ((0, 1), (H // 2 - 3, H // 2 + 4), (H - 2, H), (0, H)):
        rows, (t0, t1) = oracle.render_rows(*args, r0, r1)
        assert rows.tobytes() == full[r0:r1].tobytes(), (case, r0, r1)
