"""The per-wave primitive cull's geometry (rtm_kernels.hip `cull_prepare` / `cull_test`,
`ray_cone`), restated in numpy: the bounds it culls by must hold every point a hit can
report, so a culled primitive is one no ray of the wave can hit.  The GPU tests
(`test_raytrace.py::test_capsule_cull_stress`, `test_wave_cull_stress`) check the
device code against the oracle image; this checks the bound itself against the exact
angular distance from the wave's cone axis to the capsule (a dense scan of the
segment), on random cones and capsules, CPU only."""
import math

import numpy as np


def capsule_terms(pos, pa, pb, R):
    """cull_prepare's capsule terms (None: the slot is kept)."""
    Rc = R * 1.001 + 1e-7
    p0 = pa - pos
    e = pb - pa
    ee = float(e @ e)
    t = min(max(-float(p0 @ e) / ee, 0.0), 1.0) if ee > 0.0 else 0.0
    q = p0 + e * t
    dmin = math.sqrt(float(q @ q))
    p1 = p0 + e
    l0, l1 = math.sqrt(float(p0 @ p0)), math.sqrt(float(p1 @ p1))
    if not (dmin > Rc and math.isfinite(dmin) and math.isfinite(l0) and math.isfinite(l1)):
        return None
    csb = Rc / dmin
    ccb = math.sqrt(max(1.0 - csb * csb, 0.0))
    u0, u1 = p0 / l0, p1 / l1
    n = np.cross(u0, u1)
    nn = math.sqrt(float(n @ n))
    nh = n / nn if nn > 1e-12 else None
    return u0, u1, nh, csb, ccb


def capsule_test(ax, ct, st, terms):
    """cull_test's capsule half: True = culled."""
    u0, u1, nh, csb, ccb = terms
    thr = ct * ccb - st * csb - 1e-7
    cg = max(float(ax @ u0), float(ax @ u1))
    if nh is not None:
        an = float(ax @ nh)
        ap = ax - an * nh
        w0 = float(np.cross(u0, ap) @ nh)
        w1 = float(np.cross(ap, u1) @ nh)
        if not (w0 < -1e-6) and not (w1 < -1e-6):
            cg = max(cg, math.sqrt(max(1.0 - an * an, 0.0)))
    return cg < thr


def exact_clear(pos, ax, theta, pa, pb, R, n=4001):
    """True when the capsule lies outside the cone by the exact angular distance."""
    s = np.linspace(0.0, 1.0, n)
    P = pa[None, :] + s[:, None] * (pb - pa)[None, :] - pos[None, :]
    L = np.linalg.norm(P, axis=1)
    if (L <= R).any():
        return False
    ang = np.arccos(np.clip((P @ ax) / L, -1.0, 1.0)) - np.arcsin(R / L)
    return bool(ang.min() > theta)


def test_capsule_cull_is_conservative_and_tight():
    rng = np.random.default_rng(0x2018)
    culled = clear = 0
    for _ in range(3000):
        pos = rng.normal(size=3)
        ax = rng.normal(size=3)
        ax /= np.linalg.norm(ax)
        theta = float(rng.uniform(0.001, 0.5))
        pa = pos + ax * rng.uniform(1.0, 5.0) + rng.normal(size=3) * rng.uniform(0.1, 2.0)
        pb = pa + rng.normal(size=3) * rng.uniform(0.01, 5.0)
        R = float(rng.uniform(0.01, 0.5))
        terms = capsule_terms(pos, pa, pb, R)
        c = terms is not None and capsule_test(ax, math.cos(theta), math.sin(theta), terms)
        e = exact_clear(pos, ax, theta, pa, pb, R)
        assert not (c and not e), "culled a capsule the cone meets"
        culled += c
        clear += e
    # and it is tight: it culls nearly every capsule the exact distance allows
    assert clear > 500 and culled >= 0.9 * clear


def test_capsule_cull_keeps_degenerate_and_non_finite():
    pos = np.zeros(3)
    ax = np.array([0.0, 0.0, 1.0])
    # the apex inside the capsule
    assert capsule_terms(pos, np.array([0.0, 0.0, -1.0]), np.array([0.0, 0.0, 1.0]), 0.3) is None
    # non-finite ends (inf - inf is NaN, as on the device)
    with np.errstate(invalid="ignore"):
        assert capsule_terms(pos, np.array([np.inf, 0.0, 5.0]), np.array([0.0, 0.0, 5.0]), 0.3) is None
        assert capsule_terms(pos, np.array([np.nan, 0.0, 5.0]), np.array([0.0, 0.0, 5.0]), 0.3) is None
    # a segment pointing at the apex (its directions one point): the endpoints decide
    t = capsule_terms(pos, np.array([1.0, 0.0, 5.0]), np.array([2.0, 0.0, 10.0]), 0.1)
    assert t is not None and t[2] is None
    assert not capsule_test(np.array([0.19611614, 0.0, 0.98058068]), math.cos(0.01), math.sin(0.01), t)
    # main()'s cylinder (main.rs:931-943) from the origin: a wave looking straight at its
    # middle keeps it, one looking 10 degrees to the side culls it
    pa, pb = np.array([0.01, 10.01, 10.01]), np.array([0.01, 0.01, 10.01])
    t = capsule_terms(pos, pa, pb, 0.3)
    mid = (pa + pb) / 2
    assert not capsule_test(mid / np.linalg.norm(mid), math.cos(0.05), math.sin(0.05), t)
    side = np.array([math.sin(math.radians(10)), 0.0, math.cos(math.radians(10))])
    assert capsule_test(side, math.cos(0.05), math.sin(0.05), t)


def _strip_rasters_disc(nx, ny, xb, xe, s0, ye, cx, cy, r):
    """rtm_kernels.hip strip_rasters' disc test (its pixel-range test aside): False = no
    texel of the strip's NDC rectangle can be covered."""
    X0, X1, Y0, Y1 = nx[xb], nx[xe], ny[s0], ny[ye]
    dx = cx - np.fmin(np.fmax(cx, X0), X1)
    dy = cy - np.fmin(np.fmax(cy, Y0), Y1)
    return not (dx * dx + dy * dy > (r * r) * (1.0 + 1e-6))


def test_strip_split_disc_test_is_conservative():
    """The split shadow launch gives a 128 x 16 strip to the raster-free part only when
    strip_rasters says no sphere covers a texel of it (round 6: per sphere disc, not the
    union box).  Against the kernels' own coverage -- pa = ((x - cx) * n) / m with n =
    r * (1/m), m = sqrt(r*r + 0*0), covered iff sqrt(pa^2 + pb^2) < 1 -- on random spheres
    (both signs of r, tiny and large, centres off the map) and map sizes: no rejected strip
    holds a covered texel, and the test rejects most strips the spheres do not reach."""
    rng = np.random.default_rng(0x5EED)
    rejected = reachable_rejects = 0
    for _ in range(60):
        W, H = int(rng.integers(130, 900)), int(rng.integers(17, 700))
        nx = (np.arange(W, dtype=np.float64) / np.float64(W)) * 2.0 - 1.0
        ny = (np.arange(H, dtype=np.float64) / np.float64(H)) * 2.0 - 1.0
        cx, cy = float(rng.uniform(-1.3, 1.3)), float(rng.uniform(-1.3, 1.3))
        r = float(rng.choice([-1.0, 1.0]) * 10.0 ** rng.uniform(-3.5, -0.3))
        m = math.sqrt(r * r + 0.0 * 0.0)
        n = r * (1.0 / m)
        pa = ((nx - cx) * n) / m
        pb = ((ny - cy) * n) / m
        cov = np.sqrt(pa[None, :] * pa[None, :] + pb[:, None] * pb[:, None]) < 1.0  # [y, x]
        for xb in range(0, W, 128):
            xe = min(xb + 127, W - 1)
            for s0 in range(0, H, 16):
                ye = min(s0 + 15, H - 1)
                hit = bool(cov[s0:ye + 1, xb:xe + 1].any())
                if not _strip_rasters_disc(nx, ny, xb, xe, s0, ye, cx, cy, r):
                    rejected += 1
                    assert not hit, (W, H, cx, cy, r, xb, s0)
                elif not hit:
                    reachable_rejects += 1
    # (the bound is tight: strips it keeps without a covered texel graze the disc)
    assert rejected > 10 * max(reachable_rejects, 1)
