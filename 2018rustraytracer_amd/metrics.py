"""Algorithmic work per frame and the MI355X roofs it is priced against.

Units of work are the f64 operations the algorithm needs once per-(camera,
sphere) constants, per-column/row NDC values and loop invariants are hoisted
(add/sub/mul/div/sqrt/compare/class-test = 1 op each; no FMA — contraction is
off for bit parity).  Per-unit figures:

  shadow texel   4 per sphere (cull)      + 19 per covering sphere
                 32 per patch (ray origin, domain map, surface depth, entry sign,
                    in-range test, step vector, strict-min update)
                 3 per march iteration    (z - D, class test, z += step.z) for a ray
                                          without x/y motion (march_axis)
                 16 per march iteration   for a ray that moves in x/y (the general
                                          loop, e.g. a tilted sun): p += step (3),
                                          bilinear (7), z - h, class test, two
                                          in-range tests (2 each)
    separable axis-aligned shadow camera with a shared z sequence (every
    BASELINE scene): the per-wave cull is scalar, D = d0[x] + dd[x]*py[y],
    z_k is one host table for all texels, so per texel:
                 19 per covering sphere, 4 per patch (D: mul+add, entry compare,
                 min), 1 per march iteration (the compare z_k < D)
    ... and when the host proved that table monotone (every BASELINE scene) the
    implemented march is a first-crossing search, constant work per texel and
    patch, no per-iteration term:
                 10 per patch (D: 2, entry compare, index guess (D - z0)/sz with
                 clamp + ceil: 5, two verifying compares) — also the work of a
                 fused (on-demand) shadow texel
  eye pixel      4 per sphere (cull)      + 21 per covering sphere (incl. z-test)
                 84 per hit pixel         (ray, world pos, normal, Lambert,
                                           reflect, powi(32), shadow projection)

  ray-traced primitives (row f-1), per eye pixel, common path:
                 12 ray origin (ORTHOGONAL) / 24 normalised ray dir (PERSPECTIVE)
                 33 per circle plane      (calcRayPlane 15, hit point + radius test 18)
                 88 per capped cylinder   (iCappedCone: projections 22, cap test ~16,
                                           body quadratic 50)
                 -- per (pixel, primitive) test run: stats eye_plane_tests /
                 eye_cylinder_tests, after the PERSPECTIVE eye's per-wave cull
    PERSPECTIVE eye without SDFs (the RT 3 kernel): every ray starts at the
    camera, so the host evaluates calcRayPlane's numerator and iCappedCone's
    origin-only terms once per (camera, primitive) (RtK::persp); per test:
                 24 per circle plane      (denominator 5, its test, t, t tests 4,
                                           hit point + radius test 15)
                 48 per capped cylinder   (rd.ba 5, cap branch ~16, body quadratic 27)

HBM bytes the two-kernel design must move:
  shadow pass    8 B per texel            (f64 shadow-map store)
  eye pass       16 B per pixel           (RGBA f32 store)
               + 8 B per hit pixel        (f64 shadow-map lookup)

Peaks (/opt/skills/guides/MI355X_MICROARCH.md + datasheet): HBM 8.0 TB/s;
FP64 vector 78.6 TFLOP/s counts an FMA as 2 flops, i.e. 256 CU x 64 f64
lanes/clk x 2.4 GHz = 39.3 T f64 instructions-lanes/s — the ceiling for
non-FMA f64 ops, which is what this path issues.
"""
from __future__ import annotations

PEAK_HBM_GBS = 8000.0
PEAK_FP64_FMA_TFLOPS = 78.6
PEAK_FP64_OPS_T = 39.3  # non-FMA f64 ops per second (x1e12)

SHADOW_PER_SPHERE = 4
SHADOW_PER_COVER = 19
SHADOW_PER_PATCH = 32
SHADOW_PER_ITER = 3
SHADOW_PER_ITER_MOVING = 16
SEP_PER_PATCH = 4
SEP_PER_ITER = 1
SEARCH_PER_PATCH = 10
EYE_PER_SPHERE = 4
EYE_PER_COVER = 21
EYE_PER_HIT = 84
RT_RAY_ORTHO = 12
RT_RAY_PERSP = 24
RT_PER_PLANE = 33
RT_PER_CYL = 88
RT_PER_PLANE_PERSP = 24
RT_PER_CYL_PERSP = 48
# row f-4 (entry.frag distanceFn0 + the sphere-tracing leaf, restated in f64):
# per (pixel, SDF): two sBox slab tests + the loop set-up; per distanceFn0
# evaluation: sdBox 19 + udTriangleSingle's sign test 30 + its edge branch 59
# (the usual one) + union/offset 2 + the march step's p = ro + rd*t, compare and
# advance 8; per SDF hit: the 4-tap normal's offsets/combination/normalize.
SDF_PER_TRACE = 48
SDF_PER_EVAL = 118
SDF_PER_HIT = 31


def shared_z_separable(shadow_cam) -> bool:
    """The host-side rule (rtm_api.cpp shared_z0 + separable) for the shadow camera."""
    import math
    d, u, s, p = shadow_cam.dirNormalized, shadow_cam.upNormalized, shadow_cam.sideNormalized, shadow_cam.position
    return (shadow_cam.type_ == 0 and d[0] * 0.03 == 0.0 and d[1] * 0.03 == 0.0 and s[2] == 0.0 and u[2] == 0.0
            and not (p[2] == 0.0 and math.copysign(1.0, p[2]) < 0) and u[0] == 0.0 and s[1] == 0.0
            and not (p[1] == 0.0 and math.copysign(1.0, p[1]) < 0))


def frame_work(stats: dict, width: int, height: int, n_spheres: int, n_patches: int, flags: int = 0,
               fused: bool = False, sep: bool = False, n_planes: int = 0, n_cyls: int = 0,
               perspective: bool = False, search: bool = False, n_sdfs: int = 0, map_texel_bytes: int = 8,
               moving: bool = False, map_stored_bytes: int | None = None, span_records: bool = False) -> dict:
    """search: the march is the first-crossing search (monotone shared z table).
    map_texel_bytes: the shadow map's storage per texel (8: f64; 2 or 1: the coded
    map, rtm_ctx_shadow_map_texel_bytes) -- stored once per texel by the shadow
    pass, gathered once per hit pixel by the eye pass.
    map_stored_bytes: what the shadow pass stored per frame when measured
    (rtm_ctx_shadow_map_stored_bytes: with span records, the records plus the spans
    stored texel by texel); span_records: an eye lookup reads the 4-byte record beside
    the texel's byte.
    moving: the shadow rays move in x/y (the general march loop)."""
    px = width * height
    no_march = bool(flags & 0x1)
    no_sraster = bool(flags & 0x2)
    texels = px if not fused else stats["eye_hit_pixels"]
    sh_ops = 0
    if not no_sraster:
        sh_ops += (0 if sep else texels * SHADOW_PER_SPHERE * n_spheres) + SHADOW_PER_COVER * stats["shadow_sphere_tests"]
    if not no_march:
        if search:
            sh_ops += texels * n_patches * SEARCH_PER_PATCH
        elif sep and not fused:
            sh_ops += texels * n_patches * SEP_PER_PATCH + SEP_PER_ITER * stats["march_iterations"]
        else:
            sh_ops += texels * n_patches * SHADOW_PER_PATCH + (
                SHADOW_PER_ITER_MOVING if moving else SHADOW_PER_ITER) * stats["march_iterations"]
    eye_ops = (px * EYE_PER_SPHERE * n_spheres + EYE_PER_COVER * stats["eye_sphere_tests"]
               + EYE_PER_HIT * stats["eye_hit_pixels"])
    if n_planes or n_cyls or n_sdfs:
        # (pixel, primitive) tests actually run: the GPU's per-wave cull skips
        # primitives no ray of a wave can reach (stats, ABI v4)
        pl_tests = stats.get("eye_plane_tests", px * n_planes)
        cy_tests = stats.get("eye_cylinder_tests", px * n_cyls)
        hoisted = perspective and not n_sdfs  # the RT 3 kernel (host-hoisted origin terms)
        eye_ops += (px * ((RT_RAY_PERSP if perspective else RT_RAY_ORTHO) + SDF_PER_TRACE * n_sdfs)
                    + (RT_PER_PLANE_PERSP if hoisted else RT_PER_PLANE) * pl_tests
                    + (RT_PER_CYL_PERSP if hoisted else RT_PER_CYL) * cy_tests)
        eye_ops += SDF_PER_EVAL * stats.get("sdf_distance_evals", 0) + SDF_PER_HIT * stats.get("eye_sdf_pixels", 0)
    sh_bytes = 0 if fused else (map_stored_bytes if map_stored_bytes is not None else map_texel_bytes * px)
    lookup = map_texel_bytes + (4 if span_records else 0)
    eye_bytes = 16 * px + (0 if fused else lookup * stats["eye_hit_pixels"])
    return dict(shadow_pass=dict(ops=sh_ops, bytes=sh_bytes),
                eye_pass=dict(ops=eye_ops + (sh_ops if fused else 0), bytes=eye_bytes))


def roofline(kernel: str, work: dict, ms: float, traffic_bytes=None) -> dict:
    """Both roofs for one kernel; `bound` is the one it sits closer to."""
    w = work[kernel]
    s = ms * 1e-3
    gbs = w["bytes"] / s / 1e9 if s > 0 else 0.0
    tops = w["ops"] / s / 1e12 if s > 0 else 0.0
    hbm = dict(bound="hbm", achieved=round(gbs, 2), peak=PEAK_HBM_GBS, unit="GB/s",
               frac=round(gbs / PEAK_HBM_GBS, 4))
    alu = dict(bound="valu_fp64", achieved=round(tops, 3), peak=PEAK_FP64_OPS_T,
               unit="T f64-ops/s (non-FMA; = 78.6 TFLOP/s FMA-counted datasheet peak / 2)",
               frac=round(tops / PEAK_FP64_OPS_T, 4))
    main, other = (hbm, alu) if hbm["frac"] >= alu["frac"] else (alu, hbm)
    main = dict(main)
    main["kernel"] = kernel
    main["traffic"] = traffic_bytes
    main["other_roof"] = other
    main["algorithmic_bytes_per_launch"] = w["bytes"]
    main["algorithmic_f64_ops_per_launch"] = w["ops"]
    main["ops_basis"] = ("reference-equivalent: every f64 add/sub/mul/div/sqrt/compare/class test/abs of the "
                         "restated algorithm (module docstring) counts 1, priced at the non-FMA f64 peak; "
                         "compares and abs are not FMA-pipe flops, so `pmc` beside it gives the issued view")
    main["avg_launch_ms"] = round(ms, 5)
    return main
