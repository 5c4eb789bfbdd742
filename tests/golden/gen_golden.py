#!/usr/bin/env python3
"""Golden-vector generator: an INDEPENDENT numpy restatement of the reference
hot path (PtrMan/2018RustRayTracer src/main.rs), written separately from the C
oracle so the two cross-check each other.

Why numpy: every ufunc (add, multiply, divide, sqrt) is an elementwise IEEE
f64 operation with no FMA contraction, so a vectorised restatement that keeps
the reference's operation order is bit-exact and fast enough for 1080p.

The reference itself cannot be built here (no Rust toolchain)
and ships no golden vectors for this path, so these fixtures are generated,
not copied.  SURVEY.md §8c-3's cross-check values (computed by a third
restatement during the survey) are re-asserted below before anything is
written.

Outputs (tests/golden/):
  fixtures.npz   small frames (rgba f32 + shadow-map f64) for exact comparison
  golden.json    sha256 of larger frames + hit statistics

Run:  python tests/golden/gen_golden.py
"""
from __future__ import annotations

import hashlib
import json
import math
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))

# ---------------- scenes (same definitions as 2018rustraytracer_amd/scenes.py) ---------------
SHADOW_CAM = dict(type=0, pos=(0.0, 0.0, 0.0), dir=(0.0, 0.0, 1.0), up=(0.0, 1.0, 0.0), side=(1.0, 0.0, 0.0))
EYE_CAM = dict(type=0, pos=(-1.0, 0.0, 0.0), dir=(1.0, 0.0, 0.0), up=(0.0, 1.0, 0.0), side=(0.0, 0.0, 1.0))
REF_PATCH = (0.1, 0.1, 0.1, 0.1)
BENCH_PATCH = (0.3, 2.1, 0.9, 2.7)
PATCH_B2 = (0.5, 1.5, 1.2, 3.3)


def orbit_scene(frame, patches):
    f = float(frame)
    sph = [
        (0, (0.0, 0.0, 0.5), 0.2, (0.02, 0.02, 1.0)),
        (1, (0.0, 0.0, 0.5 + 0.2 * 2.0), 0.2, (0.02, 0.02, 1.0)),
        (2, (-0.0, math.sin(f * 0.025) * 0.7, math.cos(f * 0.025) * 0.7), 0.1, (0.9, 0.2, 0.2)),
    ]
    return sph, list(patches)


def scene_b():
    cols = [(0.02, 0.02, 1.0), (0.9, 0.2, 0.2), (0.2, 0.9, 0.2), (0.9, 0.9, 0.2)]
    sph = []
    for i in range(16):
        a = 2.0 * math.pi * i / 16.0
        sph.append((i, (-0.5 + 0.0625 * i, 0.6 * math.sin(a), 0.6 + 0.6 * math.cos(a)), 0.08 + 0.01 * (i % 4),
                    cols[i % 4]))
    return sph, [BENCH_PATCH, PATCH_B2]


def overlapping():
    return [(0, (0.0, 0.0, 0.0), 0.5, (0.02, 0.02, 1.0)), (1, (0.0, 0.0, 0.5), 0.5, (1.0, 1.0, 1.0))], []


# ---- row f-1: testscene_raytracingPlane0 (main.rs:910-1046) ----
PERSP_CAM = dict(type=1, pos=(0.0, 0.0, 0.0), dir=(0.0, 0.0, 1.0), up=(0.0, 1.0, 0.0), side=(1.0, 0.0, 0.0))


def _normalize(v):
    m = math.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
    inv = 1.0 / m
    return (v[0] * inv, v[1] * inv, v[2] * inv)


# (id, pos, n, radius, color) / (id, pA, pB, ra, rb, color)
REF_PLANE = (0, (0.01, 0.01, 2.0), _normalize((-1.0, 0.0, 1.0)), 0.5, (0.02, 0.02, 1.0))
REF_CYL = (0, (0.01, 10.01, 10.01), (0.01, 0.01, 10.01), 0.3, 0.2, (1.0, 0.02, 0.02))


def rbench():
    cols = [(1.0, 0.02, 0.02), (0.02, 0.02, 1.0), (0.2, 0.9, 0.2), (0.9, 0.9, 0.2), (0.9, 0.2, 0.9)]
    cyl = [REF_CYL]
    for i in range(8):
        a = 2.0 * math.pi * i / 8.0
        c = (1.5 * math.cos(a), 1.5 * math.sin(a), 5.0)
        h = (0.4 * math.cos(a + 1.0), 0.4 * math.sin(a + 1.0), -0.8)
        cyl.append((i + 1, (c[0] + h[0], c[1] + h[1], c[2] + h[2]), (c[0] - h[0], c[1] - h[1], c[2] - h[2]),
                    0.25 + 0.05 * (i % 3), 0.15 + 0.05 * (i % 2), cols[i % 5]))
    planes = [REF_PLANE,
              (1, (0.0, 0.0, 12.0), _normalize((0.2, 0.1, -1.0)), 16.0, (0.9, 0.9, 0.2)),
              (2, (-1.5, -1.0, 7.0), _normalize((0.5, 0.3, -1.0)), 1.2, (0.2, 0.9, 0.2)),
              (3, (1.2, 1.4, 6.0), _normalize((-0.4, -0.6, -1.0)), 0.9, (0.9, 0.2, 0.9))]
    return planes, cyl


# ray-traced primitives seen by the orthographic eye camera of the orbit scene
# (a disc and a cone crossing the spheres' depth range; same as tests' scenes.mixed_rt)
MIXED_PLANES = [(0, (0.3, -0.3, 0.3), _normalize((-1.0, 0.2, 0.1)), 0.4, (0.2, 0.9, 0.2)),
                (1, (0.05, 0.35, -0.45), _normalize((-1.0, -0.5, 0.3)), 0.25, (0.9, 0.9, 0.2))]
MIXED_CYLS = [(0, (0.0, -0.6, -0.5), (0.2, 0.5, -0.3), 0.1, 0.15, (0.9, 0.2, 0.9)),
              (1, (-0.1, 0.1, 0.3), (0.5, 0.1, 0.9), 0.12, 0.12, (1.0, 0.02, 0.02))]


# ---------------- restatement ----------------
def signum(v):  # Rust f64::signum
    return np.where(np.isnan(v), v, np.copysign(1.0, v))


def grid(W, H):
    xi = np.arange(W, dtype=np.float64)[None, :].repeat(H, 0)
    yi = np.arange(H, dtype=np.float64)[:, None].repeat(W, 1)
    # (i as f64 / res as f64) * 2.0 - 1.0   (main.rs:306-307, 1903-1907)
    return (xi / float(W)) * 2.0 - 1.0, (yi / float(H)) * 2.0 - 1.0


def dot(a, b):
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]


def rays(cam, W, H):
    """Camera::calcRayOriginAndDirection (main.rs:1902-1942) for every pixel."""
    s, u = grid(W, H)
    if cam["type"] == 0:
        o = [(cam["pos"][k] + cam["side"][k] * s) + cam["up"][k] * u for k in range(3)]
        d = [np.full(s.shape, cam["dir"][k]) for k in range(3)]
    else:
        v = [(cam["dir"][k] + cam["side"][k] * (s * 1.0)) + cam["up"][k] * (u * 1.0) for k in range(3)]
        m = np.sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2])
        inv = 1.0 / m
        o = [np.full(s.shape, cam["pos"][k]) for k in range(3)]
        d = [v[k] * inv for k in range(3)]
    return o, d


def icapped_cone(ro, rd, pa, pb, ra, rb):
    """iCappedCone (main.rs:2889-2959) vectorised; branches become masks."""
    with np.errstate(all="ignore"):
        ba = [pb[k] - pa[k] for k in range(3)]
        oa = [ro[k] - pa[k] for k in range(3)]
        ob = [ro[k] - pb[k] for k in range(3)]
        baba = dot(ba, ba)
        rdba = dot(rd, ba)
        oaba = dot(oa, ba)
        obba = dot(ob, ba)
        isq = 1.0 / math.sqrt(baba)
        w = [oa[k] * rdba - rd[k] * oaba for k in range(3)]
        capA = (oaba < 0.0) & (dot(w, w) < ra * ra * rdba * rdba)
        tA = -oaba / rdba
        tB = -obba / rdba
        w = [ob[k] + rd[k] * tB for k in range(3)]
        capB = ~(oaba < 0.0) & (obba > 0.0) & (dot(w, w) < rb * rb)
        rr = rb - ra
        hy = baba + rr * rr
        oc = [oa[k] * rb - ob[k] * ra for k in range(3)]
        ocba, ocrd, ococ = dot(oc, ba), dot(oc, rd), dot(oc, oc)
        k2 = baba * baba - hy * rdba * rdba
        k1 = baba * baba * ocrd - hy * rdba * ocba
        k0 = baba * baba * ococ - hy * ocba * ocba
        h = k1 * k1 - k2 * k0
        sg = 1.0 if rr >= 0.0 else -1.0
        tb = (-k1 - sg * np.sqrt(np.where(h < 0.0, 0.0, h))) / (k2 * rr)
        y = oaba + rdba * tb
        body = ~capA & ~capB & ~(h < 0.0) & (y > 0.0) & (y < baba)
        inside = [((oa[k] + rd[k] * tb) * baba - ba[k] * (rr * ra)) * baba - ba[k] * (hy * y) for k in range(3)]
        m = np.sqrt(inside[0] * inside[0] + inside[1] * inside[1] + inside[2] * inside[2])
        inv = 1.0 / m
        nb = [inside[k] * inv for k in range(3)]
        t = np.where(capA, tA, np.where(capB, tB, np.where(body, tb, -1.0)))
        n = [np.where(capA, ba[k] * -isq, np.where(capB, ba[k] * isq, np.where(body, nb[k], -1.0)))
             for k in range(3)]
    return t, n


# ---- row f-4: the GL preview's SDF (entry.frag), f64 restatement, vectorised ----
def _fmax(a, b):
    a, b = np.broadcast_arrays(np.asarray(a, np.float64), np.asarray(b, np.float64))
    return np.where(np.isnan(a), b, np.where(np.isnan(b), a, np.where(a > b, a, np.where(b > a, b,
                    np.where(np.signbit(a), b, a)))))


def _fmin(a, b):
    a, b = np.broadcast_arrays(np.asarray(a, np.float64), np.asarray(b, np.float64))
    return np.where(np.isnan(a), b, np.where(np.isnan(b), a, np.where(a < b, a, np.where(b < a, b,
                    np.where(np.signbit(a), a, b)))))


def _gsign(x):
    return np.where(x > 0.0, 1.0, np.where(x < 0.0, -1.0, 0.0))


def _cross(x, y):
    return (x[1] * y[2] - y[1] * x[2], x[2] * y[0] - y[2] * x[0], x[0] * y[1] - y[0] * x[1])


def _sub3(a, b):
    return tuple(a[k] - b[k] for k in range(3))


def _sdf_geom(sd):
    _id, box, tri, _c, _e, _col, _steps = sd
    v1 = tuple(tri[k] + (0.8, 0.8, 0.8)[k] for k in range(3))
    v2 = tuple(tri[k] + (1.3, 0.8, 0.8)[k] for k in range(3))
    v3 = tuple(tri[k] + (1.0, 0.7, 0.2)[k] for k in range(3))
    v21, v32, v13 = _sub3(v2, v1), _sub3(v3, v2), _sub3(v1, v3)
    nor = _cross(v21, v13)
    return dict(box=box, v=(v1, v2, v3), e=(v21, v32, v13), nor=nor,
                c=(_cross(v21, nor), _cross(v32, nor), _cross(v13, nor)),
                d=(dot(v21, v21), dot(v32, v32), dot(v13, v13)), dnor=dot(nor, nor))


def _dist(g, p):
    """distanceFn0 (entry.frag:416-442) at points p (3 arrays)."""
    with np.errstate(all="ignore"):
        q = _sub3(p, g["box"])
        dd = [np.abs(q[k]) - (0.4, 0.2, 0.2)[k] for k in range(3)]
        m = [_fmax(dd[k], 0.0) for k in range(3)]
        d0 = _fmin(_fmax(dd[0], _fmax(dd[1], dd[2])), 0.0) + np.sqrt(dot(m, m))
        ps = [_sub3(p, g["v"][i]) for i in range(3)]
        inside = (_gsign(dot(g["c"][0], ps[0])) + _gsign(dot(g["c"][1], ps[1])) + _gsign(dot(g["c"][2], ps[2]))) < 2.0
        es = []
        for i in range(3):
            cl = _fmin(_fmax(dot(g["e"][i], ps[i]) / g["d"][i], 0.0), 1.0)
            e = [g["e"][i][k] * cl - ps[i][k] for k in range(3)]
            es.append(dot(e, e))
        edges = _fmin(_fmin(es[0], es[1]), es[2])
        dn = dot(g["nor"], ps[0])
        face = dn * dn / g["dnor"]
        d1 = np.where(inside, edges, face)
        return _fmin(d0, d1) - 0.2


def _sbox(ro, rd, c, e, check):
    with np.errstate(all="ignore"):
        roo = _sub3(ro, c)
        m = [1.0 / rd[k] for k in range(3)]
        n = [m[k] * roo[k] for k in range(3)]
        kk = [np.abs(m[k]) * e[k] for k in range(3)]
        t1 = [-n[k] - kk[k] for k in range(3)]
        t2 = [-n[k] + kk[k] for k in range(3)]
        tN = _fmax(_fmax(t1[0], t1[1]), t1[2])
        tF = _fmin(_fmin(t2[0], t2[1]), t2[2])
        if check:
            tN = np.where((tN > tF) | (tF < 0.0), -1.0, tN)
        return tN


def trace_sdf(sd, ro, rd):
    """entry.frag:842-905 per pixel: (t or -1, normal)."""
    g = _sdf_geom(sd)
    c, e, steps = sd[3], sd[4], sd[6]
    tIn = _sbox(ro, rd, c, e, True)
    ok = tIn >= 0.0
    tOut = -_sbox(ro, tuple(-rd[k] for k in range(3)), c, e, False)
    t = np.where(ok, tIn, 0.0)
    active = ok.copy()
    hit = np.zeros(ok.shape, bool)
    for _ in range(steps):
        if not active.any():
            break
        p = tuple(ro[k] + rd[k] * t for k in range(3))
        dist = _dist(g, p)
        newhit = active & (dist < 0.03)
        hit |= newhit
        active &= ~newhit
        active &= ~(t > tOut)
        t = np.where(active, t + dist, t)
    p = tuple(ro[k] + rd[k] * t for k in range(3))
    h = 0.001
    ks = ((1.0, -1.0, -1.0), (-1.0, -1.0, 1.0), (-1.0, 1.0, -1.0), (1.0, 1.0, 1.0))
    taps = [_dist(g, tuple(p[k] + (s[k] * h) for k in range(3))) for s in ks]
    v = [((ks[0][k] * taps[0] + ks[1][k] * taps[1]) + ks[2][k] * taps[2]) + ks[3][k] * taps[3] for k in range(3)]
    with np.errstate(all="ignore"):
        inv = 1.0 / np.sqrt(dot(v, v))
    n = [v[k] * inv for k in range(3)]
    return np.where(hit, t, -1.0), n


def raytrace(cam, planes, cyls, W, H, zbuf, g, sdfs=()):
    """processRaytracingRays (main.rs:569-642): planes then cylinders, in order
    (then the row f-4 SDFs, accepted for 0 < t < depth)."""
    o, d = rays(cam, W, H)
    with np.errstate(all="ignore"):
        for (pid, c, n, radius, _col) in planes:
            denom = dot(n, d)
            t = dot([c[k] - o[k] for k in range(3)], n) / denom
            P = [o[k] + d[k] * t for k in range(3)]
            q = [P[k] - c[k] for k in range(3)]
            dist = np.sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2])
            win = (np.abs(denom) > 0.0001) & ~(t < 0.0) & ~(t > zbuf) & ~(dist > radius)
            zbuf[win] = t[win]
            g["kind"][win] = 2
            g["id"][win] = pid
            g["t"][win] = t[win]
        for (cid, pa, pb, ra, rb, _col) in cyls:
            t, n = icapped_cone(o, d, pa, pb, ra, rb)
            win = ~(t < 0.0) & ~(t > zbuf)
            zbuf[win] = t[win]
            g["kind"][win] = 3
            g["id"][win] = cid
            g["t"][win] = t[win]
            for k in range(3):
                g["n%d" % k][win] = n[k][win]
        for sd in sdfs:
            t, n = trace_sdf(sd, o, d)
            win = (t > 0.0) & (t < zbuf)
            zbuf[win] = t[win]
            g["kind"][win] = 4
            g["id"][win] = sd[0]
            g["t"][win] = t[win]
            for k in range(3):
                g["n%d" % k][win] = n[k][win]


# ---- row f-3: perspective projection (main.rs:473-530, 2796-2837; nalgebra 0.16) ----
def _gemv(a, x):
    """nalgebra fixed 4x4 gemv: y_i = v0*m_i0, then y_i = v_j*m_ij + 1*y_i."""
    y = [x[0] * a[i][0] for i in range(4)]
    for j in range(1, 4):
        y = [x[j] * a[i][j] + 1.0 * y[i] for i in range(4)]
    return y


def _mm(a, b):
    cols = [_gemv(a, [b[0][j], b[1][j], b[2][j], b[3][j]]) for j in range(4)]
    return [[cols[j][i] for j in range(4)] for i in range(4)]


def _perspective3(aspect, fovy, znear, zfar):
    p = [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)]
    old = p[1][1]
    p[1][1] = 1.0 / math.tan(fovy / 2.0)            # set_fovy
    p[0][0] = p[0][0] * (p[1][1] / old)
    p[0][0] = p[1][1] / aspect                       # set_aspect
    p[2][2] = (zfar + znear) / (znear - zfar)        # set_znear_and_zfar
    p[2][3] = zfar * znear * 2.0 / (znear - zfar)
    p[3][3] = 0.0
    p[3][2] = -1.0
    return p


def project_perspective(cam, W, H, pos, r):
    """(center, axisA, axisB) of a sphere seen by a PERSPECTIVE camera."""
    rel = [[cam["side"][0], cam["side"][1], cam["side"][2], 0.0], [cam["up"][0], cam["up"][1], cam["up"][2], 0.0],
           [cam["dir"][0], cam["dir"][1], cam["dir"][2], 0.0], [0.0, 0.0, 0.0, 1.0]]
    diff = [pos[k] - cam["pos"][k] for k in range(3)]
    local = _gemv(rel, diff + [1.0])[:3]
    fov = 3.14 / 2.0
    refl = [[1.0 if i == j else 0.0 for j in range(4)] for i in range(4)]
    refl[2][2] = -1.0
    cm = _mm(_perspective3(float(W) / float(H), fov, 0.1, 1000.0), refl)
    o = _gemv(cm, local + [1.0])[:3]
    r2 = r * r
    z2 = o[2] * o[2]
    l2 = (o[0] * o[0] + o[1] * o[1]) + o[2] * o[2]

    def safe_sqrt(v):
        return math.sqrt(v) if v >= 0.0 else float("nan")

    with np.errstate(all="ignore"):
        sa = fle_sqrt = fov * safe_sqrt(-r2 * (r2 - l2) / ((l2 - z2) * (r2 - z2) * (r2 - z2)))
        sb = fov * safe_sqrt(-r2 * (r2 - l2) / ((l2 - z2) * (r2 - z2) * (r2 - l2)))
    del fle_sqrt
    axa = (o[0] * sa, o[1] * sa)
    axb = (-o[1] * sb, o[0] * sb)
    sc = fov * o[2] / (z2 - r2)
    return (o[0] * sc, o[1] * sc), axa, axb


def rasterize(cam, spheres, W, H, face, zbuf, gbuf):
    """Viewport::rasterize (main.rs:445-547), orthographic or perspective, no bbox."""
    x, y = grid(W, H)
    for (sid, pos, r, _col) in spheres:
        diff = tuple(pos[k] - cam["pos"][k] for k in range(3))
        z = dot(cam["dir"], diff)
        if cam["type"] == 0:
            cx, cy = dot(diff, cam["side"]), dot(diff, cam["up"])
            axA, axB = (r, 0.0), (0.0, r)
        else:
            (cx, cy), axA, axB = project_perspective(cam, W, H, pos, r)
        # calcEllipseDistToCenter: Vec2::normalized = v.scale(1/|v|), |v| = sqrt(x*x + y*y)
        mA = math.sqrt(axA[0] * axA[0] + axA[1] * axA[1]) if not any(map(math.isnan, axA)) else float("nan")
        mB = math.sqrt(axB[0] * axB[0] + axB[1] * axB[1]) if not any(map(math.isnan, axB)) else float("nan")
        with np.errstate(all="ignore"):
            iA = np.float64(1.0) / np.float64(mA)
            iB = np.float64(1.0) / np.float64(mB)
        nA = (axA[0] * iA, axA[1] * iA)
        nB = (axB[0] * iB, axB[1] * iB)
        relx, rely = x - cx, y - cy
        with np.errstate(all="ignore"):
            pa = (relx * nA[0] + rely * nA[1]) / mA
            pb = (relx * nB[0] + rely * nB[1]) / mB
            d = np.sqrt(pa * pa + pb * pb)
            cov = d < 1.0
            h = np.sqrt(np.where(cov, 1.0 - d * d, 0.0))
        depth = z - h * r if face == 0 else z + h * r
        win = cov & (depth < zbuf)
        zbuf[win] = depth[win]
        if gbuf is not None:
            gbuf["kind"][win] = 1
            gbuf["id"][win] = sid
            gbuf["h"][win] = h[win]
            gbuf["z"][win] = z


def march(cam, patches, W, H, steps, zbuf):
    """processRaymarchingRays + raymarchPatch (main.rs:551-565, 2179-2278), orthographic."""
    s, u = grid(W, H)
    o = [(cam["pos"][k] + cam["side"][k] * s) + cam["up"][k] * u for k in range(3)]
    for (a0, b0, a1, b1) in patches:
        def bil(px, py):
            d0 = a0 + (b0 - a0) * px
            d1 = a1 + (b1 - a1) * px
            return d0 + (d1 - d0) * py
        px = (o[0] + 1.0) * 0.5
        py = (o[1] + 1.0) * 0.5
        pz = o[2].copy()
        st = (cam["dir"][0] * 0.03, cam["dir"][1] * 0.03, cam["dir"][2] * 0.03)
        t = np.zeros_like(pz)
        entry = signum(pz - bil(px, py))
        done = np.zeros(pz.shape, bool)
        hit_t = np.full(pz.shape, np.nan)
        for _ in range(steps):
            inr = (np.abs(px - 0.5) <= 0.5) & (np.abs(py - 0.5) <= 0.5)
            sg = signum(pz - bil(px, py))
            newhit = (~done) & inr & (sg != entry)
            hit_t[newhit] = t[newhit]
            done |= newhit
            px = px + st[0]
            py = py + st[1]
            pz = pz + st[2]
            t = t + 0.03
            if done.all():
                break
        upd = done & (hit_t < zbuf)
        zbuf[upd] = hit_t[upd]


def render(spheres, patches, W, H, steps, no_march=False, no_sraster=False, planes=(), cyls=(), eye=EYE_CAM,
           sdfs=()):
    zs = np.full((H, W), np.inf)
    if not no_sraster:
        rasterize(SHADOW_CAM, spheres, W, H, 1, zs, None)
    if not no_march:
        march(SHADOW_CAM, patches, W, H, steps, zs)
    ze = np.full((H, W), np.inf)
    g = dict(kind=np.zeros((H, W), np.int64), id=np.full((H, W), -1, np.int64), h=np.zeros((H, W)),
             z=np.zeros((H, W)), t=np.zeros((H, W)), n0=np.zeros((H, W)), n1=np.zeros((H, W)),
             n2=np.zeros((H, W)))
    if spheres:
        rasterize(eye, spheres, W, H, 0, ze, g)
    raytrace(eye, planes, cyls, W, H, ze, g, sdfs)
    # renderColorImage (main.rs:710-902)
    img = np.zeros((H, W, 4), np.float32)
    img[..., 1] = np.float32(0.2)
    img[..., 2] = np.float32(0.2)
    img[..., 3] = 1.0
    hit = g["kind"] > 0
    if hit.any():
        kind = g["kind"][hit]
        ids = g["id"][hit]
        o, d = rays(eye, W, H)
        o, d = [a[hit] for a in o], [a[hit] for a in d]
        sprm = {sid: (pos, r, col) for (sid, pos, r, col) in spheres}
        pprm = {pid: (n, col) for (pid, _c, n, _r, col) in planes}
        cprm = {cid: col for (cid, _a, _b, _ra, _rb, col) in cyls}
        sdprm = {sd[0]: sd[5] for sd in sdfs}
        sph = kind == 1
        R = np.array([sprm[i][1] if k == 1 else 1.0 for i, k in zip(ids, kind)])
        P = np.array([sprm[i][0] if k == 1 else (0.0, 0.0, 0.0) for i, k in zip(ids, kind)]).reshape(-1, 3)
        COL = np.array([sprm[i][2] if k == 1 else pprm[i][1] if k == 2 else cprm[i] if k == 3 else sdprm[i]
                        for i, k in zip(ids, kind)]).reshape(-1, 3)
        # calcDepth (main.rs:155-173)
        depth = np.where(sph, g["z"][hit] - g["h"][hit] * R, g["t"][hit])
        wp = [o[k] + d[k] * depth for k in range(3)]
        PN = np.array([pprm[i][0] if k == 2 else (0.0, 0.0, 0.0) for i, k in zip(ids, kind)]).reshape(-1, 3)
        n = [np.where(sph, (wp[k] - P[:, k]) * (1.0 / R), np.where(kind == 2, PN[:, k], g["n%d" % k][hit]))
             for k in range(3)]
        cam = eye
        L = (1.0 * -1.0, 0.0 * -1.0, 0.0 * -1.0)
        diffuse = np.fmax(n[0] * L[0] + n[1] * L[1] + n[2] * L[2], 0.0)
        k2 = -2.0 * (L[0] * n[0] + L[1] * n[1] + L[2] * n[2])
        Rv = [L[k] - n[k] * k2 for k in range(3)]
        # retViewDirOfPixel (main.rs:1981-2013)
        view = [cam["dir"][k] * -1.0 for k in range(3)] if cam["type"] == 0 else [d[k] * -1.0 for k in range(3)]
        sp = np.fmax(view[0] * Rv[0] + view[1] * Rv[1] + view[2] * Rv[2], 0.0)
        with np.errstate(over="ignore"):
            for _ in range(5):
                sp = sp * sp
        sc = SHADOW_CAM
        df = [wp[k] - sc["pos"][k] for k in range(3)]
        qx, qy, qz = dot(df, sc["side"]), dot(df, sc["up"]), dot(df, sc["dir"])
        half_w, half_h = W // 2, H // 2

        def trunc_i64(v):
            v = np.where(np.isnan(v), 0.0, v)
            v = np.clip(v, -4e18, 4e18)
            return np.trunc(v).astype(np.int64)

        tx = half_w + trunc_i64(qx * float(half_w))
        ty = half_h + trunc_i64(qy * float(half_h))
        inb = (tx >= 0) & (tx < W) & (ty >= 0) & (ty < H)
        dsm = np.full(tx.shape, np.inf)
        dsm[inb] = zs[ty[inb], tx[inb]]
        lit = dsm > qz - 0.0
        lm = np.where(lit, 1.0, 0.25)
        base = diffuse + sp
        with np.errstate(over="ignore"):
            img[hit, 0] = ((base * lm) * COL[:, 0]).astype(np.float32)
            img[hit, 1] = ((base * lm) * COL[:, 1]).astype(np.float32)
            img[hit, 2] = ((base * lm) * COL[:, 2]).astype(np.float32)
        stats = dict(eye_hits=[int(((ids == i) & sph).sum()) for i in range(len(spheres))], lit=int(lit.sum()))
        stats["plane_px"] = int((kind == 2).sum())
        stats["cyl_px"] = int((kind == 3).sum())
        stats["sdf_px"] = int((kind == 4).sum())
    else:
        stats = dict(eye_hits=[0] * len(spheres), lit=0, plane_px=0, cyl_px=0, sdf_px=0)
    return img, zs, stats


def sha16(img):
    return hashlib.sha256(np.ascontiguousarray(img[:, :, :3]).tobytes()).hexdigest()[:16]


def sha_full(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# (name, scene factory, W, H, steps, flags) — small ones go to fixtures.npz, all to golden.json
CASES = [
    ("orbit_f0_64", lambda: orbit_scene(0, [REF_PATCH]), 64, 64, 500, 0, True),
    ("orbit_f100_96x80", lambda: orbit_scene(100, [REF_PATCH]), 96, 80, 500, 0, True),
    ("bench_f100_128x72_k64", lambda: orbit_scene(100, [BENCH_PATCH]), 128, 72, 64, 0, True),
    ("bench_f37_33x65_k32", lambda: orbit_scene(37, [BENCH_PATCH]), 33, 65, 32, 0, True),
    ("sceneb_120x90_k128", scene_b, 120, 90, 128, 0, True),
    ("overlap_64", overlapping, 64, 64, 0, 3, True),
    ("cfg1_256_nomarch", lambda: orbit_scene(100, [REF_PATCH]), 256, 256, 0, 1, False),
    ("orbit_f0_512", lambda: orbit_scene(0, [REF_PATCH]), 512, 512, 500, 0, False),
    ("orbit_f100_512", lambda: orbit_scene(100, [REF_PATCH]), 512, 512, 500, 0, False),
    ("orbit_f250_512", lambda: orbit_scene(250, [REF_PATCH]), 512, 512, 500, 0, False),
    ("bench_f100_1920x1080_k32", lambda: orbit_scene(100, [BENCH_PATCH]), 1920, 1080, 32, 0, False),
    ("sceneb_640x360_k128", scene_b, 640, 360, 128, 0, False),
]

# row f-1 cases: (name, spheres, patches, planes, cyls, eye, W, H, steps, flags, small)
# (id, box_center, tri_anchor, aabb_center, aabb_extent, color, max_steps): scenes.PREVIEW_SDF etc.
SDF_PREVIEW = (0, (3.0, 0.0, 5.0), (3.5, 0.0, 6.0), (3.0, 0.0, 5.0), (3.0, 3.0, 3.0), (0.9, 0.6, 0.2), 180)
SDF_CAM = dict(type=1, pos=(3.0, 0.3, 0.5), dir=(0.0, 0.0, 1.0), up=(0.0, 1.0, 0.0), side=(1.0, 0.0, 0.0))


def sdf_bench():
    cols = [(1.0, 0.02, 0.02), (0.02, 0.02, 1.0), (0.2, 0.9, 0.2), (0.9, 0.9, 0.2), (0.9, 0.2, 0.9)]
    sdfs = []
    for i in range(8):
        dx, dy = -2.25 + 1.5 * (i % 4), -0.9 + 1.8 * (i // 4)
        base = (3.0 + dx, dy, 5.0 + 0.25 * i)
        sdfs.append((i, base, (base[0] + 0.5, base[1], base[2] + 1.0), base, (1.6, 1.4, 2.0), cols[i % 5], 180))
    back = (0, (3.0, 0.0, 12.0), (0.0, 0.0, -1.0), 30.0, (0.2, 0.2, 0.25))
    return [back], sdfs


# an SDF beside the orbit scene's spheres, seen by its orthographic eye (scenes.mixed_sdf)
SDF_MIXED = (0, (0.4, -0.3, 0.0), (-1.0, -1.2, -1.2), (0.4, -0.3, 0.0), (1.0, 1.0, 1.0), (0.9, 0.6, 0.2), 120)

P1 = [(0, (0.01, 0.01, 4.0), 0.5, (0.02, 0.02, 1.0))]
P2 = P1 + [(1, (0.01, 0.01, 6.0), 0.5, (0.02, 1.0, 0.02))]
PERSP2_CAM = dict(PERSP_CAM, pos=(0.0, 1.5, 0.0))

RT_CASES = [
    ("f3_persp1_96", P1, [], [], [], PERSP_CAM, 96, 96, 0, 3, True),
    ("f3_persp2_80x64", P2, [], [], [], PERSP2_CAM, 80, 64, 0, 3, True),
    ("f3_persp1_512", P1, [], [], [], PERSP_CAM, 512, 512, 0, 3, False),
    ("f3_persp2_512", P2, [], [], [], PERSP2_CAM, 512, 512, 0, 3, False),
    ("f3_persp2_rt_640x360", P2, [], [REF_PLANE], [REF_CYL], PERSP2_CAM, 640, 360, 0, 3, False),
    ("f4_preview_96", [], [], [], [], SDF_CAM, 96, 96, 0, 3, True, [SDF_PREVIEW]),
    ("f4_bench_128x72", [], [], sdf_bench()[0], [], SDF_CAM, 128, 72, 0, 3, True, sdf_bench()[1]),
    ("f4_mixed_orbit_96", *orbit_scene(100, [BENCH_PATCH]), [], [], EYE_CAM, 96, 96, 64, 0, True, [SDF_MIXED]),
    ("f4_preview_512", [], [], [], [], SDF_CAM, 512, 512, 0, 3, False, [SDF_PREVIEW]),
    ("f4_bench_640x360", [], [], sdf_bench()[0], [], SDF_CAM, 640, 360, 0, 3, False, sdf_bench()[1]),
    ("rt_plane0_64", [], [], [], [REF_CYL], PERSP_CAM, 64, 64, 0, 3, True),
    ("rt_plane0_withplane_96x80", [], [], [REF_PLANE], [REF_CYL], PERSP_CAM, 96, 80, 0, 3, True),
    ("rt_rbench_128x72", [], [], *rbench(), PERSP_CAM, 128, 72, 0, 3, True),
    ("rt_mixed_orbit_96", *orbit_scene(100, [BENCH_PATCH]), MIXED_PLANES, MIXED_CYLS, EYE_CAM, 96, 96, 64, 0, True),
    ("rt_plane0_512", [], [], [], [REF_CYL], PERSP_CAM, 512, 512, 0, 3, False),
    ("rt_plane0_withplane_512", [], [], [REF_PLANE], [REF_CYL], PERSP_CAM, 512, 512, 0, 3, False),
    ("rt_rbench_640x360", [], [], *rbench(), PERSP_CAM, 640, 360, 0, 3, False),
    ("rt_mixed_orbit_320x180", *orbit_scene(100, [BENCH_PATCH]), MIXED_PLANES, MIXED_CYLS, EYE_CAM, 320, 180, 64,
     0, False),
]


def main():
    # pin against SURVEY.md §8c-3 before writing anything
    img0, _, st0 = render(*orbit_scene(0, [REF_PATCH]), 512, 512, 500)
    assert (st0["eye_hits"], st0["lit"]) == ([8014, 6372, 659], 0), st0
    assert sha16(img0) == "cf557d736f83a4f6"
    assert img0[256, 384, :3].tolist() == [9265101144064.0, 9265101144064.0, 463255038328832.0]
    assert img0[300, 384, :3].tolist() == [3506.7421875, 3506.7421875, 175337.109375]
    img100, _, st100 = render(*orbit_scene(100, [REF_PATCH]), 512, 512, 500)
    assert (st100["eye_hits"], st100["lit"]) == ([8245, 6580, 2059], 2059), st100
    assert sha16(img100) == "cb7008f728da5208"

    fixtures, golden = {}, {}
    for name, fac, W, H, K, flags, small in CASES:
        sph, pat = fac()
        img, zs, st = render(sph, pat, W, H, K, no_march=bool(flags & 1), no_sraster=bool(flags & 2))
        golden[name] = dict(width=W, height=H, steps=K, flags=flags, rgba_sha256=sha_full(img),
                            shadow_sha256=sha_full(zs), eye_hits=st["eye_hits"], lit_pixels=st["lit"])
        if small:
            fixtures[name + "__rgba"] = img
            fixtures[name + "__shadow"] = zs
        print(name, golden[name]["rgba_sha256"][:16], st)
    for case in RT_CASES:
        name, sph, pat, planes, cyls, eye, W, H, K, flags, small = case[:11]
        sdfs = case[11] if len(case) > 11 else []
        img, zs, st = render(sph, pat, W, H, K, no_march=bool(flags & 1), no_sraster=bool(flags & 2),
                             planes=planes, cyls=cyls, eye=eye, sdfs=sdfs)
        golden[name] = dict(width=W, height=H, steps=K, flags=flags, rgba_sha256=sha_full(img),
                            shadow_sha256=sha_full(zs), eye_hits=st["eye_hits"], lit_pixels=st["lit"],
                            circle_plane_pixels=st.get("plane_px", 0), capped_cylinder_pixels=st.get("cyl_px", 0),
                            sdf_pixels=st.get("sdf_px", 0))
        if small:
            fixtures[name + "__rgba"] = img
            fixtures[name + "__shadow"] = zs
        print(name, golden[name]["rgba_sha256"][:16], st)
    np.savez_compressed(os.path.join(HERE, "fixtures.npz"), **fixtures)
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_golden.py (independent numpy restatement of main.rs)",
                       survey_kat_checked=True, cases=golden), f, indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
