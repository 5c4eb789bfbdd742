"""Scene description (reference main.rs:334-422) and the reference's test scenes.

Plain-Python mirror of the reference's scene types so host code reads like the
reference's scene scripts (testscene_*, main.rs:910-1633).  Trigonometry for
animated spheres is evaluated here on the host (libm, as Rust's f64::sin/cos
are on Linux) and passed to the device as data.
"""
from __future__ import annotations

import ctypes as C
import dataclasses
import math
from dataclasses import dataclass, field
from typing import List

from . import abi


@dataclass
class Shading:  # main.rs:336-340
    colorR: float
    colorG: float
    colorB: float


@dataclass
class PrimitiveSphere:  # main.rs:343-349
    id: int
    shading: Shading
    pos: tuple
    r: float


@dataclass
class PrimitiveCirclePlane:  # main.rs:370-380
    id: int
    shading: Shading
    radius: float
    pos: tuple
    n: tuple


@dataclass
class PrimitiveCappedCylinder:  # main.rs:382-391
    id: int
    shading: Shading
    pA: tuple
    pB: tuple
    radiusA: float
    radiusB: float


@dataclass
class PrimitiveSdf:  # the GL preview's implicit surface (entry.frag:842-947), row f-4
    id: int
    shading: Shading
    box_center: tuple = (3.0, 0.0, 5.0)    # descriptor vecs[0] (entry.frag:878)
    tri_anchor: tuple = (3.5, 0.0, 6.0)    # descriptor vecs[2] (entry.frag:880)
    aabb_center: tuple = (3.0, 0.0, 5.0)   # entry.frag:850
    aabb_extent: tuple = (3.0, 3.0, 3.0)   # entry.frag:851
    max_steps: int = 180                   # entry.frag:887


@dataclass
class Linear:  # main.rs:2134-2137
    a: float
    b: float


@dataclass
class Bilinear:  # main.rs:2139-2142
    _0: Linear
    _1: Linear


# rayEntry_ShadowRay_testing's hard-coded patch and step count (main.rs:2024-2031)
REFERENCE_PATCH = Bilinear(Linear(0.1, 0.1), Linear(0.1, 0.1))
REFERENCE_MARCH_STEPS = 500

ORTHOGONAL = abi.RTM_CAMERA_ORTHOGONAL
PERSPECTIVE = abi.RTM_CAMERA_PERSPECTIVE


class EnumFace:  # main.rs:225-228
    FRONT = abi.RTM_FACE_FRONT
    BACK = abi.RTM_FACE_BACK


@dataclass
class Camera:  # main.rs:1887-1898 (resolution comes from the viewport)
    type_: int
    position: tuple
    dirNormalized: tuple
    upNormalized: tuple
    sideNormalized: tuple

    def to_c(self) -> abi.rtm_camera:
        c = abi.rtm_camera()
        c.type = self.type_
        c.pos[:] = [float(v) for v in self.position]
        c.dir[:] = [float(v) for v in self.dirNormalized]
        c.up[:] = [float(v) for v in self.upNormalized]
        c.side[:] = [float(v) for v in self.sideNormalized]
        return c


@dataclass
class Scene:  # main.rs:404-410 (+ the implicit patches the march path takes as data)
    spherePrimitives: List[PrimitiveSphere] = field(default_factory=list)
    patches: List[Bilinear] = field(default_factory=list)
    circlePlanePrimitives: List[PrimitiveCirclePlane] = field(default_factory=list)
    cappedCylinderPrimitives: List[PrimitiveCappedCylinder] = field(default_factory=list)
    sdfPrimitives: List[PrimitiveSdf] = field(default_factory=list)

    def to_c(self):
        """Returns (rtm_scene, keepalive) — keep the second value alive while
        the first is in use."""
        ns, npch = len(self.spherePrimitives), len(self.patches)
        sph = (abi.rtm_sphere * max(ns, 1))()
        for i, s in enumerate(self.spherePrimitives):
            sph[i].id = int(s.id)
            sph[i].pos[:] = [float(v) for v in s.pos]
            sph[i].r = float(s.r)
            sph[i].color[:] = [float(s.shading.colorR), float(s.shading.colorG), float(s.shading.colorB)]
        pat = (abi.rtm_patch * max(npch, 1))()
        for i, p in enumerate(self.patches):
            pat[i].a0, pat[i].b0 = float(p._0.a), float(p._0.b)
            pat[i].a1, pat[i].b1 = float(p._1.a), float(p._1.b)
        npl, ncy = len(self.circlePlanePrimitives), len(self.cappedCylinderPrimitives)
        pl = (abi.rtm_circle_plane * max(npl, 1))()
        for i, q in enumerate(self.circlePlanePrimitives):
            pl[i].id = int(q.id)
            pl[i].pos[:] = [float(v) for v in q.pos]
            pl[i].n[:] = [float(v) for v in q.n]
            pl[i].radius = float(q.radius)
            pl[i].color[:] = [float(q.shading.colorR), float(q.shading.colorG), float(q.shading.colorB)]
        cy = (abi.rtm_capped_cylinder * max(ncy, 1))()
        for i, q in enumerate(self.cappedCylinderPrimitives):
            cy[i].id = int(q.id)
            cy[i].pa[:] = [float(v) for v in q.pA]
            cy[i].pb[:] = [float(v) for v in q.pB]
            cy[i].ra, cy[i].rb = float(q.radiusA), float(q.radiusB)
            cy[i].color[:] = [float(q.shading.colorR), float(q.shading.colorG), float(q.shading.colorB)]
        sc = abi.rtm_scene()
        sc.spheres = C.cast(sph, C.POINTER(abi.rtm_sphere))
        sc.patches = C.cast(pat, C.POINTER(abi.rtm_patch))
        sc.n_spheres = ns
        sc.n_patches = npch
        sc.circle_planes = C.cast(pl, C.POINTER(abi.rtm_circle_plane))
        sc.capped_cylinders = C.cast(cy, C.POINTER(abi.rtm_capped_cylinder))
        sc.n_circle_planes = npl
        sc.n_capped_cylinders = ncy
        nsd = len(self.sdfPrimitives)
        sd = (abi.rtm_sdf * max(nsd, 1))()
        for i, q in enumerate(self.sdfPrimitives):
            sd[i].id = int(q.id)
            sd[i].box_center[:] = [float(v) for v in q.box_center]
            sd[i].tri_anchor[:] = [float(v) for v in q.tri_anchor]
            sd[i].aabb_center[:] = [float(v) for v in q.aabb_center]
            sd[i].aabb_extent[:] = [float(v) for v in q.aabb_extent]
            sd[i].color[:] = [float(q.shading.colorR), float(q.shading.colorG), float(q.shading.colorB)]
            sd[i].max_steps = int(q.max_steps)
        sc.sdfs = C.cast(sd, C.POINTER(abi.rtm_sdf))
        sc.n_sdfs = nsd
        return sc, (sph, pat, pl, cy, sd)


# ---- cameras of the orthographic test scenes ----
def shadow_camera() -> Camera:
    """Shadow-map camera: the sun shines along +z (main.rs:1552-1563)."""
    return Camera(ORTHOGONAL, (0.0, 0.0, 0.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0), (1.0, 0.0, 0.0))


def eye_camera() -> Camera:
    """Eye camera at (-1,0,0) looking along +x (main.rs:1598-1609)."""
    return Camera(ORTHOGONAL, (-1.0, 0.0, 0.0), (1.0, 0.0, 0.0), (0.0, 1.0, 0.0), (0.0, 0.0, 1.0))


def tilted_shadow_camera() -> Camera:
    """An orthographic sun that does not shine along an axis (synthetic, bench
    config 9): its shadow rays move in x and y as they march, so the march takes
    the general per-step loop (in-range test and surface depth re-evaluated every
    step, main.rs:2247-2274) instead of the axis-aligned first-crossing search.
    dir = normalize(0.25, -0.15, 1), side = normalize(up0 x dir) with up0 = +y,
    up = dir x side, all f64 on the host (Camera::project only needs an
    ORTHOGONAL camera, main.rs:1949)."""
    def cross(a, b):
        return (a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0])
    d = normalize((0.25, -0.15, 1.0))
    s = normalize(cross((0.0, 1.0, 0.0), d))
    u = cross(d, s)
    return Camera(ORTHOGONAL, (0.0, 0.0, 0.0), d, u, s)


# ---- scenes ----
def closely_orbiting_sphere(frame: int, patches=None) -> Scene:
    """testscene_closelyOrbitingSphere frame `frame` (main.rs:1468-1522).
    Default patches: the reference's hard-coded one (Scene A-ref)."""
    f = float(frame)
    spheres = [
        PrimitiveSphere(0, Shading(0.02, 0.02, 1.0), (0.0, 0.0, 0.5), 0.2),
        PrimitiveSphere(1, Shading(0.02, 0.02, 1.0), (0.0, 0.0, 0.5 + 0.2 * 2.0), 0.2),
        PrimitiveSphere(2, Shading(0.9, 0.2, 0.2),
                        (-0.0, math.sin(f * 0.025) * 0.7, math.cos(f * 0.025) * 0.7), 0.1),
    ]
    return Scene(spheres, list(patches) if patches is not None else [REFERENCE_PATCH])


BENCH_PATCH = Bilinear(Linear(0.3, 2.1), Linear(0.9, 2.7))  # SURVEY.md §8d-2 Scene A-bench
SCENE_B_PATCH2 = Bilinear(Linear(0.5, 1.5), Linear(1.2, 3.3))


def scene_a_bench(frame: int = 100) -> Scene:
    """Scene A-bench: frame 100 with a tilted patch so texels cross at 10..90
    steps and the march bound K actually limits work."""
    return closely_orbiting_sphere(frame, [BENCH_PATCH])


_COLORS_B = [(0.02, 0.02, 1.0), (0.9, 0.2, 0.2), (0.2, 0.9, 0.2), (0.9, 0.9, 0.2)]


def scene_b() -> Scene:
    """Scene B: 16 spheres + 2 implicit patches (BASELINE config 5)."""
    spheres = []
    for i in range(16):
        a = 2.0 * math.pi * i / 16.0
        spheres.append(PrimitiveSphere(
            i, Shading(*_COLORS_B[i % 4]),
            (-0.5 + 0.0625 * i, 0.6 * math.sin(a), 0.6 + 0.6 * math.cos(a)),
            0.08 + 0.01 * (i % 4)))
    return Scene(spheres, [BENCH_PATCH, SCENE_B_PATCH2])


def overlapping_spheres() -> Scene:
    """testscene_overlappingSpheres (main.rs:1322-1458): two spheres, shadow pass
    commented out (render with RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER)."""
    return Scene([
        PrimitiveSphere(0, Shading(0.02, 0.02, 1.0), (0.0, 0.0, 0.0), 0.5),
        PrimitiveSphere(1, Shading(1.0, 1.0, 1.0), (0.0, 0.0, 0.5), 0.5),
    ], [])


OVERLAPPING_FLAGS = abi.RTM_FLAG_NO_MARCH | abi.RTM_FLAG_NO_SHADOW_RASTER



# ---- testscene_raytracingPlane0 (main.rs:910-1046): main()'s default scene ----
def normalize(v) -> tuple:
    """normalize (main.rs:105-108): v.scale(1.0 / |v|), |v| = sqrt((x*x + y*y) + z*z)."""
    m = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    inv = 1.0 / m
    return (v[0] * inv, v[1] * inv, v[2] * inv)


def perspective_eye_camera() -> Camera:
    """viewport0's PERSPECTIVE camera at the origin looking along +z (main.rs:1016-1027)."""
    return Camera(PERSPECTIVE, (0.0, 0.0, 0.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0), (1.0, 0.0, 0.0))


# the circle plane testscene_raytracingPlane0 has commented out (main.rs:916-929)
REFERENCE_CIRCLE_PLANE = PrimitiveCirclePlane(0, Shading(0.02, 0.02, 1.0), 0.5, (0.01, 0.01, 2.0),
                                              normalize((-1.0, 0.0, 1.0)))
# its one capped cylinder (main.rs:931-943)
REFERENCE_CAPPED_CYLINDER = PrimitiveCappedCylinder(0, Shading(1.0, 0.02, 0.02), (0.01, 10.01, 10.01),
                                                    (0.01, 0.01, 10.01), 0.3, 0.2)
# both shadow passes are commented out (main.rs:998-1003): the shadow map stays +INF
RAYTRACING_FLAGS = abi.RTM_FLAG_NO_MARCH | abi.RTM_FLAG_NO_SHADOW_RASTER


def raytracing_plane0(with_plane: bool = False) -> Scene:
    """testscene_raytracingPlane0's scene: one capped cylinder (and, with
    with_plane, the circle plane the reference has commented out).  Render with
    perspective_eye_camera(), shadow_camera() and RAYTRACING_FLAGS."""
    return Scene([], [], [dataclasses.replace(REFERENCE_CIRCLE_PLANE)] if with_plane else [],
                 [dataclasses.replace(REFERENCE_CAPPED_CYLINDER)])


_COLORS_R = [(1.0, 0.02, 0.02), (0.02, 0.02, 1.0), (0.2, 0.9, 0.2), (0.9, 0.9, 0.2), (0.9, 0.2, 0.9)]


def scene_r_bench() -> Scene:
    """Scene R-bench (row f-1 measurement, synthetic): the
    reference's cylinder and circle plane plus a ring of 8 capped cylinders
    around the view axis and 3 more discs, one a backdrop covering most of the
    frame, so most eye rays test and hit several primitives."""
    cyl = [dataclasses.replace(REFERENCE_CAPPED_CYLINDER)]
    for i in range(8):
        a = 2.0 * math.pi * i / 8.0
        c = (1.5 * math.cos(a), 1.5 * math.sin(a), 5.0)
        h = (0.4 * math.cos(a + 1.0), 0.4 * math.sin(a + 1.0), -0.8)
        cyl.append(PrimitiveCappedCylinder(
            i + 1, Shading(*_COLORS_R[i % 5]), (c[0] + h[0], c[1] + h[1], c[2] + h[2]),
            (c[0] - h[0], c[1] - h[1], c[2] - h[2]), 0.25 + 0.05 * (i % 3), 0.15 + 0.05 * (i % 2)))
    planes = [
        dataclasses.replace(REFERENCE_CIRCLE_PLANE),
        PrimitiveCirclePlane(1, Shading(0.9, 0.9, 0.2), 16.0, (0.0, 0.0, 12.0), normalize((0.2, 0.1, -1.0))),
        PrimitiveCirclePlane(2, Shading(0.2, 0.9, 0.2), 1.2, (-1.5, -1.0, 7.0), normalize((0.5, 0.3, -1.0))),
        PrimitiveCirclePlane(3, Shading(0.9, 0.2, 0.9), 0.9, (1.2, 1.4, 6.0), normalize((-0.4, -0.6, -1.0))),
    ]
    return Scene([], [], planes, cyl)


def mixed_rt(frame: int = 100) -> Scene:
    """Scene A-bench frame `frame` plus two circle planes and two capped cylinders
    in front of the orthographic eye camera: ray-traced hits compete with
    rasterized spheres in the eye zBuffer (main.rs:592, 633) and are shadowed by
    the spheres + patch shadow map (tests only; parity of the mixed frame)."""
    s = scene_a_bench(frame)
    s.circlePlanePrimitives = [
        PrimitiveCirclePlane(0, Shading(0.2, 0.9, 0.2), 0.4, (0.3, -0.3, 0.3), normalize((-1.0, 0.2, 0.1))),
        PrimitiveCirclePlane(1, Shading(0.9, 0.9, 0.2), 0.25, (0.05, 0.35, -0.45), normalize((-1.0, -0.5, 0.3))),
    ]
    s.cappedCylinderPrimitives = [
        PrimitiveCappedCylinder(0, Shading(0.9, 0.2, 0.9), (0.0, -0.6, -0.5), (0.2, 0.5, -0.3), 0.1, 0.15),
        PrimitiveCappedCylinder(1, Shading(1.0, 0.02, 0.02), (-0.1, 0.1, 0.3), (0.5, 0.1, 0.9), 0.12, 0.12),
    ]
    return s


# BASELINE.json configs 1-5 (+ row f-1 workloads 6-7):
# width, height, march_steps, scene factory, flags, eye camera factory (default eye_camera)
CONFIGS = {
    1: dict(width=256, height=256, steps=0, scene=lambda: closely_orbiting_sphere(100),
            flags=abi.RTM_FLAG_NO_MARCH, desc="256x256, 3 spheres, no ray-march (CPU plumbing)"),
    2: dict(width=1920, height=1080, steps=32, scene=scene_a_bench, flags=0,
            desc="1920x1080, 3 spheres + 1 implicit, 32 march steps"),
    3: dict(width=3840, height=2160, steps=64, scene=scene_a_bench, flags=0,
            desc="3840x2160, 3 spheres + 1 implicit, 64 march steps"),
    4: dict(width=7680, height=4320, steps=64, scene=scene_a_bench, flags=0,
            desc="7680x4320, 3 spheres + 1 implicit, 64 march steps"),
    5: dict(width=7680, height=4320, steps=128, scene=scene_b, flags=0,
            desc="7680x4320, 16 spheres + 2 implicits, 128 march steps"),
    # row f-1 measurement workloads, PERSPECTIVE eye camera
    6: dict(width=3840, height=2160, steps=0, scene=scene_r_bench, flags=RAYTRACING_FLAGS,
            eye=perspective_eye_camera,
            desc="3840x2160, Scene R-bench: 9 capped cylinders + 4 circle planes, perspective (row f-1)"),
    7: dict(width=512, height=512, steps=0, scene=raytracing_plane0, flags=RAYTRACING_FLAGS,
            eye=perspective_eye_camera,
            desc="512x512, testscene_raytracingPlane0 as main() renders it (row f-1)"),
    # row f-4: Scene S-bench (8 preview SDFs + a backdrop circle plane); the
    # factories are defined below, hence the lambdas
    8: dict(width=3840, height=2160, steps=0, scene=lambda: sdf_bench_scene(), flags=RAYTRACING_FLAGS,
            eye=lambda: sdf_eye_camera(),
            desc="3840x2160, Scene S-bench: 8 GL-preview SDFs + 1 circle plane, perspective (row f-4)"),
    # the general march: Scene A-bench under a tilted orthographic sun, so every
    # shadow ray moves in x/y and the march is the per-step loop (raymarchPatch as
    # written) rather than the axis-aligned first-crossing search
    9: dict(width=3840, height=2160, steps=64, scene=scene_a_bench, flags=0, shadow=lambda: tilted_shadow_camera(),
            desc="3840x2160, 3 spheres + 1 implicit, 64 march steps, tilted orthographic sun (general march)",
            metric="Mpixels/s at 3840x2160, 64 march steps, general (x/y-moving) shadow rays"),
}


# ---- row f-3: testscene_perspectiveSimple1/2 (main.rs:1059-1316) ----
def perspective_simple1() -> Scene:
    """testscene_perspectiveSimple1 (main.rs:1059-1182): one sphere in front of
    the PERSPECTIVE eye camera at the origin; no shadow pass (main.rs:1115-1120).
    Render with perspective_eye_camera(), shadow_camera(), RAYTRACING_FLAGS."""
    return Scene([PrimitiveSphere(0, Shading(0.02, 0.02, 1.0), (0.01, 0.01, 4.0), 0.5)], [])


def perspective_simple2() -> Scene:
    """testscene_perspectiveSimple2 (main.rs:1184-1316): two spheres; render with
    perspective_simple2_camera()."""
    return Scene([PrimitiveSphere(0, Shading(0.02, 0.02, 1.0), (0.01, 0.01, 4.0), 0.5),
                  PrimitiveSphere(1, Shading(0.02, 1.0, 0.02), (0.01, 0.01, 6.0), 0.5)], [])


def perspective_simple2_camera() -> Camera:
    """viewport0's camera of testscene_perspectiveSimple2 (main.rs:1283-1295)."""
    return Camera(PERSPECTIVE, (0.0, 1.5, 0.0), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0), (1.0, 0.0, 0.0))


# ---- row f-4: the GL preview's SDF implicit surface (entry.frag:842-947) ----
PREVIEW_SDF = PrimitiveSdf(0, Shading(0.9, 0.6, 0.2))  # the shader's one instance, its own constants


def sdf_eye_camera() -> Camera:
    """PERSPECTIVE eye outside the preview SDF's AABB (x 0..6, y -3..3, z 2..8), looking along +z."""
    return Camera(PERSPECTIVE, (3.0, 0.3, 0.5), (0.0, 0.0, 1.0), (0.0, 1.0, 0.0), (1.0, 0.0, 0.0))


def sdf_preview_scene() -> Scene:
    """The preview shader's implicit surface alone (tests; render with
    sdf_eye_camera(), shadow_camera(), RAYTRACING_FLAGS)."""
    return Scene([], [], [], [], [dataclasses.replace(PREVIEW_SDF)])


def sdf_bench_scene() -> Scene:
    """Scene S-bench (row f-4 measurement, synthetic): 8 copies of the preview
    SDF, each with its own AABB, in a 4 x 2 grid in front of sdf_eye_camera(),
    plus the reference's circle plane as a backdrop."""
    sdfs = []
    for i in range(8):
        dx, dy = -2.25 + 1.5 * (i % 4), -0.9 + 1.8 * (i // 4)
        base = (3.0 + dx, dy, 5.0 + 0.25 * i)
        sdfs.append(PrimitiveSdf(i, Shading(*_COLORS_R[i % 5]), base, (base[0] + 0.5, base[1], base[2] + 1.0),
                                 base, (1.6, 1.4, 2.0)))
    back = PrimitiveCirclePlane(0, Shading(0.2, 0.2, 0.25), 30.0, (3.0, 0.0, 12.0), (0.0, 0.0, -1.0))
    return Scene([], [], [back], [], sdfs)


def mixed_sdf(frame: int = 100) -> Scene:
    """Scene A-bench plus one preview SDF beside the spheres, in front of the
    orthographic eye camera (tests: SDF hits against sphere depths and under
    the spheres + patch shadow map)."""
    s = scene_a_bench(frame)
    s.sdfPrimitives = [PrimitiveSdf(0, Shading(0.9, 0.6, 0.2), (0.4, -0.3, 0.0), (-1.0, -1.2, -1.2),
                                    (0.4, -0.3, 0.0), (1.0, 1.0, 1.0), 120)]
    return s
