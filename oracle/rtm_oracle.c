/*
 * rtm_oracle.c — CPU ORACLE (test infrastructure only; never shipped, never on
 * the product path).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it, and only as the checker / CPU baseline.
 *
 * A plain-C f64 restatement of the per-pixel hot path of
 * PtrMan/2018RustRayTracer src/main.rs, written function by function in the
 * reference's structure and floating-point operation order (no hoisting, no
 * FMA contraction: build with -ffp-contract=off -fno-fast-math).  Each
 * function cites the reference lines it restates.
 *
 * Parity status: the reference cannot be built here (Rust toolchain absent;
 * SURVEY.md §8c-1) and holds no golden vectors for this path (its only tests,
 * main.rs:2415-2457, cover calcRayPlane / calcRayQuadPlane).  This oracle is
 * therefore pinned by (a) the independent f64 cross-check values of SURVEY.md
 * §8c-3 (hit counts, pixel values, sha256 of the 512x512 frames 0 and 100),
 * (b) an independent pure-Python restatement (tests/golden/gen_golden.py) and
 * (c) the reference's own calcRayPlane test (main.rs:2415-2425) for the
 * ray-plane intersector.  See DESIGN.md §Parity.
 *
 * Generalisation: the reference's 512 constants become the
 * viewport width/height; with RTMO_FLAG_REF_BBOX the sphere bounding box of
 * main.rs:256-300 is applied exactly as written (a pure cull on square images).
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../include/rtm.h"

#ifdef _OPENMP
#include <omp.h>
#endif

#define RTMO_FLAG_REF_BBOX 0x100 /* oracle-only: reference sphere bbox, main.rs:256-300 */

/* ------------------------------------------------------------------ */
/* L0 math — Vec3 / Vec2 (main.rs:58-115, 2083-2130)                   */
/* ------------------------------------------------------------------ */
typedef struct { double x, y, z; } Vec3;
typedef struct { double x, y; } Vec2;

static Vec3 v3(double x, double y, double z) { Vec3 r = {x, y, z}; return r; }
/* Add / Sub (main.rs:85-99) */
static Vec3 v3_add(Vec3 a, Vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
static Vec3 v3_sub(Vec3 a, Vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
/* Vec3::scale (main.rs:76-78) */
static Vec3 v3_scale(Vec3 a, double s) { return v3(a.x * s, a.y * s, a.z * s); }
/* dot (main.rs:101-103): (a.x*b.x + a.y*b.y) + a.z*b.z */
static double dot(Vec3 a, Vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
/* Vec3::magnitude (main.rs:71-73) */
static double v3_magnitude(Vec3 a) { return sqrt(dot(a, a)); }
/* normalize (main.rs:105-108) */
static Vec3 normalize(Vec3 v) { double m = v3_magnitude(v); return v3_scale(v, 1.0 / m); }

static Vec2 v2(double x, double y) { Vec2 r = {x, y}; return r; }
static Vec2 v2_sub(Vec2 a, Vec2 b) { return v2(a.x - b.x, a.y - b.y); }
static Vec2 v2_scale(Vec2 a, double s) { return v2(a.x * s, a.y * s); }
/* Vec2::magnitudeSquared / magnitude / normalized (main.rs:2098-2109) */
static double v2_magnitude(Vec2 a) { return sqrt(a.x * a.x + a.y * a.y); }
static Vec2 v2_normalized(Vec2 a) { double m = v2_magnitude(a); return v2_scale(a, 1.0 / m); }
/* dot2d (main.rs:2128-2130) */
static double dot2d(Vec2 a, Vec2 b) { return a.x * b.x + a.y * b.y; }

/* Rust f64::signum: +1 for +0/+x/+inf, -1 for -0/-x/-inf, NaN for NaN */
static double rust_signum(double v) { return isnan(v) ? v : copysign(1.0, v); }
/* Rust f64::max: a NaN operand (quiet or signaling) yields the other one.
 * (glibc fmax returns NaN for a signaling NaN, per IEEE 754-2008 maxNum.) */
static double rust_max(double a, double b) { return isnan(a) ? b : (isnan(b) ? a : fmax(a, b)); }
/* Rust f32::max / f32::min, same NaN rule */
static float rust_maxf(float a, float b) { return isnan(a) ? b : (isnan(b) ? a : fmaxf(a, b)); }
static float rust_minf(float a, float b) { return isnan(a) ? b : (isnan(b) ? a : fminf(a, b)); }
/* Rust `as i64` from f64: truncate toward zero, saturate, NaN -> 0 */
static int64_t rust_as_i64(double v) {
    if (isnan(v)) return 0;
    if (v >= 9223372036854775807.0) return INT64_MAX;
    if (v <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)v;
}
/* Rust i64 `+` in a release build wraps */
static int64_t wrap_add_i64(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
/* f64::powi(32) = compiler-rt __powidf2: repeated squaring (exact op sequence) */
static double powi(double a, int b) {
    int recip = b < 0;
    double r = 1.0;
    for (;;) {
        if (b & 1) r *= a;
        b /= 2;
        if (b == 0) break;
        a *= a;
    }
    return recip ? 1.0 / r : r;
}

/* ------------------------------------------------------------------ */
/* L1 camera (main.rs:1880-2014)                                       */
/* ------------------------------------------------------------------ */
typedef struct {
    int32_t type;
    Vec3 pos, dir, up, side;
    int64_t resX, resY;
} Camera;

static Camera camera_from(const rtm_camera* c, int64_t resX, int64_t resY) {
    Camera k;
    k.type = c->type;
    k.pos = v3(c->pos[0], c->pos[1], c->pos[2]);
    k.dir = v3(c->dir[0], c->dir[1], c->dir[2]);
    k.up = v3(c->up[0], c->up[1], c->up[2]);
    k.side = v3(c->side[0], c->side[1], c->side[2]);
    k.resX = resX;
    k.resY = resY;
    return k;
}

/* Camera::calcRayOriginAndDirection (main.rs:1902-1942) */
static void calcRayOriginAndDirection(const Camera* c, int64_t pixelX, int64_t pixelY, Vec3* origin,
                                      Vec3* dir) {
    double sideScale01 = (double)pixelX / (double)c->resX;
    double upScale01 = (double)pixelY / (double)c->resY;
    double sideScalem11 = sideScale01 * 2.0 - 1.0;
    double upScalem11 = upScale01 * 2.0 - 1.0;
    if (c->type == RTM_CAMERA_ORTHOGONAL) {
        Vec3 positionP = c->pos;
        positionP = v3_add(positionP, v3_scale(c->side, sideScalem11));
        positionP = v3_add(positionP, v3_scale(c->up, upScalem11));
        *origin = positionP;
        *dir = c->dir;
    } else {
        double scaleSide = 1.0, scaleUp = 1.0;
        Vec3 rayDirection = c->dir;
        rayDirection = v3_add(rayDirection, v3_scale(c->side, sideScalem11 * scaleSide));
        rayDirection = v3_add(rayDirection, v3_scale(c->up, upScalem11 * scaleUp));
        *origin = c->pos;
        *dir = normalize(rayDirection);
    }
}

/* Camera::project, orthogonal only (main.rs:1947-1958) */
static Vec3 camera_project(const Camera* c, Vec3 position) {
    Vec3 diff = v3(position.x - c->pos.x, position.y - c->pos.y, position.z - c->pos.z);
    return v3(dot(diff, c->side), dot(diff, c->up), dot(diff, c->dir));
}

/* Camera::calcDepthOfProjectedPoint (main.rs:1962-1978); both branches are the same dot */
static double calcDepthOfProjectedPoint(const Camera* c, Vec3 p) {
    Vec3 positionDiff = v3_sub(p, c->pos);
    return dot(c->dir, positionDiff);
}

/* Camera::retViewDirOfPixel (main.rs:1981-2013) */
static Vec3 retViewDirOfPixel(const Camera* c, int64_t pixelX, int64_t pixelY) {
    if (c->type == RTM_CAMERA_ORTHOGONAL) return v3_scale(c->dir, -1.0);
    double sideScale01 = (double)pixelX / (double)c->resX;
    double upScale01 = (double)pixelY / (double)c->resY;
    double sideScalem11 = sideScale01 * 2.0 - 1.0;
    double upScalem11 = upScale01 * 2.0 - 1.0;
    Vec3 rayDirection = c->dir;
    rayDirection = v3_add(rayDirection, v3_scale(c->side, sideScalem11 * 1.0));
    rayDirection = v3_add(rayDirection, v3_scale(c->up, upScalem11 * 1.0));
    Vec3 dirNormalized = normalize(rayDirection);
    return v3_scale(dirNormalized, -1.0);
}

/* ------------------------------------------------------------------ */
/* L2 sphere coverage (main.rs:122-331, 2844-2857)                     */
/* ------------------------------------------------------------------ */
typedef struct {
    int64_t id;
    double z;
    Vec2 center;
    double r;
    Vec2 axisA, axisB;
} ProjectedSphere; /* main.rs:199-208 */

/* calcHeightOfSphereOnUnit (main.rs:123-133); returns 1 and *h if Some */
static int calcHeightOfSphereOnUnit(double distUnit, double* h) {
    if (distUnit < 1.0) {
        *h = sqrt(1.0 - distUnit * distUnit);
        return 1;
    }
    return 0;
}

/* calcZValueOfProjectedSphere (main.rs:236-246) */
static double calcZValueOfProjectedSphere(double z, double absoluteProjectedRadius, int face) {
    return face == RTM_FACE_FRONT ? z - absoluteProjectedRadius : z + absoluteProjectedRadius;
}

/* calcEllipseDistToCenter + calcDistToCenter (main.rs:2848-2857) */
static double calcEllipseDistToCenter(Vec2 rel, Vec2 axisA, Vec2 axisB) {
    double projectedA = dot2d(rel, v2_normalized(axisA)) / v2_magnitude(axisA);
    double projectedB = dot2d(rel, v2_normalized(axisB)) / v2_magnitude(axisB);
    return v2_magnitude(v2(projectedA, projectedB));
}

/* ProjectedSphere::calcOthoDistanceByAbsPosition (main.rs:214-217) */
static double calcOthoDistanceByAbsPosition(const ProjectedSphere* s, Vec2 p) {
    Vec2 rel = v2_sub(p, s->center);
    return calcEllipseDistToCenter(rel, s->axisA, s->axisB);
}

/* G-buffer entry: Option<PixelSurfaceInfo> (main.rs:136-150):
 *   RasterizedSphere{relativeHeight, id, z}            kind GK_SPHERE
 *   RaytracedCirlcePlaneIntersection{id, rayT}          kind GK_PLANE
 *   RaytracedCappedCylinderIntersection{id, rayT, n}    kind GK_CYLINDER */
enum { GK_SPHERE = 1, GK_PLANE = 2, GK_CYLINDER = 3, GK_SDF = 4 };
typedef struct {
    int32_t some; /* kind, 0 = None */
    int64_t id;
    double relativeHeight;
    double z;
    double rayT;
    Vec3 n;
} GEntry;

typedef struct {
    int64_t W, H;
    int face;
    Camera camera;
    double* zBuffer; /* Map2d<f64> row-major y*W+x (main.rs:2351-2373) */
    GEntry* rasterized;
    /* rows held: [y0, y0 + rows) (the whole viewport unless a row window was
     * asked for, rtmo_render_rows); element (y, x) is at (y - y0) * W + x */
    int64_t y0, rows;
} Viewport;

typedef struct {
    int64_t eye_hits[RTM_MAX_SPHERES];
    int64_t eye_hit_pixels, lit_pixels, eye_sphere_tests, shadow_sphere_tests;
    int64_t march_iterations, march_hits, march_in_range;
    int64_t eye_circle_plane_pixels, eye_capped_cylinder_pixels, eye_sdf_pixels;
    int64_t sdf_distance_evals;
    int64_t eye_plane_tests, eye_cylinder_tests;
} Counts; /* layout == rtm_stats */

/* rasterizeSphere (main.rs:249-331).  Pixel loop over rows [y0,y1).  The
 * bbox (main.rs:256-300) is applied only with RTMO_FLAG_REF_BBOX. */
static void rasterizeSphere(const ProjectedSphere* ps, double r, Viewport* vp, int flags, int64_t y0,
                            int64_t y1, int64_t* tests) {
    int64_t minX = 0, maxX = vp->W, minY = 0, maxY = vp->H;
    if (flags & RTMO_FLAG_REF_BBOX) {
        double maxAxisLength = v2_magnitude(ps->axisA);
        maxAxisLength = rust_max(maxAxisLength, v2_magnitude(ps->axisB));
        double resW = (double)vp->W, resH = (double)vp->H;
        double aspectY = (double)vp->H / (double)vp->W;
#define CONV(rel, res, asp) rust_as_i64((((rel) + 1.0) * 0.5) * (asp) * (res))
        int64_t boundXMin = CONV(ps->center.x - maxAxisLength, resW, 1.0) + 1;
        boundXMin -= 1;
        int64_t boundXMax = CONV(ps->center.x + maxAxisLength, resW, 1.0) + 1;
        boundXMax += 1;
        if (boundXMin > minX) minX = boundXMin;
        if (boundXMax < maxX) maxX = boundXMax;
        int64_t boundYMin = CONV(ps->center.y - maxAxisLength, resH, aspectY) + 1;
        boundYMin -= 1;
        int64_t boundYMax = CONV(ps->center.y + maxAxisLength, resH, aspectY) + 1;
        boundYMax += 1;
#undef CONV
        if (boundYMin > minY) minY = boundYMin;
        if (boundYMax < maxY) maxY = boundYMax;
    }
    if (minY < y0) minY = y0;
    if (maxY > y1) maxY = y1;
    for (int64_t yi = minY; yi < maxY; yi++) {
        for (int64_t xi = minX; xi < maxX; xi++) {
            /* main.rs:306-307 with 512 -> W/H */
            double x = ((double)xi / (double)vp->W) * 2.0 - 1.0;
            double y = ((double)yi / (double)vp->H) * 2.0 - 1.0;
            Vec2 p = v2(x, y);
            /* projectSphereAtZBuffer (main.rs:176-195) */
            double distanceToCenterUnit = calcOthoDistanceByAbsPosition(ps, p);
            double relativeHeight;
            if (!calcHeightOfSphereOnUnit(distanceToCenterUnit, &relativeHeight)) continue;
            if (tests) (*tests)++;
            double depth = calcZValueOfProjectedSphere(ps->z, relativeHeight * r, vp->face);
            int64_t idx = (yi - vp->y0) * vp->W + xi;
            if (depth < vp->zBuffer[idx]) {
                vp->rasterized[idx].some = GK_SPHERE;
                vp->rasterized[idx].id = ps->id;
                vp->rasterized[idx].relativeHeight = relativeHeight;
                vp->rasterized[idx].z = ps->z;
                vp->zBuffer[idx] = depth;
            }
        }
    }
}

/* ---- PERSPECTIVE sphere projection (row f-3, main.rs:473-530, 2796-2837) ----
 * nalgebra (Cargo.toml: nalgebra = "^0.16.12"; not in /root/reference, no
 * Cargo.lock) is restated from its published 0.16 source:
 *   Matrix4::new(m11, m12, …) takes its 16 elements row by row;
 *   Matrix * Matrix / Vector (fixed 4x4) = gemm → per output column one gemv,
 *     y_i = v_0*m_i0, then y_i = v_j*m_ij + 1*y_i for j = 1..3 (axpy), i.e.
 *     ((m_i0 v_0 + m_i1 v_1) + m_i2 v_2) + m_i3 v_3, zero terms included;
 *   Perspective3::new(aspect, fovy, znear, zfar): identity, then set_fovy
 *     (m11 = 1 / tan(fovy / 2); m00 = m00 * (m11 / old m11)), set_aspect
 *     (m00 = m11 / aspect), set_znear_and_zfar (m22 = (zfar + znear) /
 *     (znear - zfar); m23 = zfar * znear * 2 / (znear - zfar)), m33 = 0, m32 = -1;
 *   Matrix4::new_nonuniform_scaling(v) = identity with the diagonal v.
 * tan is the platform libm's, as Rust's f64::tan.  No reference output exists
 * for this branch: parity unpinned, cross-checked against the
 * independent restatement in tests/golden/gen_golden.py. */
typedef struct { double m[4][4]; } M44;

static M44 m44_identity(void) {
    M44 r;
    memset(&r, 0, sizeof r);
    for (int i = 0; i < 4; i++) r.m[i][i] = 1.0;
    return r;
}

/* nalgebra gemv: y = a * x (fixed 4x4, column-by-column axpy) */
static void m44_gemv(const M44* a, const double x[4], double y[4]) {
    for (int i = 0; i < 4; i++) y[i] = x[0] * a->m[i][0];
    for (int j = 1; j < 4; j++)
        for (int i = 0; i < 4; i++) y[i] = x[j] * a->m[i][j] + 1.0 * y[i];
}

/* nalgebra gemm: r = a * b, one gemv per column of b */
static M44 m44_mul(const M44* a, const M44* b) {
    M44 r;
    for (int j = 0; j < 4; j++) {
        double x[4] = {b->m[0][j], b->m[1][j], b->m[2][j], b->m[3][j]}, y[4];
        m44_gemv(a, x, y);
        for (int i = 0; i < 4; i++) r.m[i][j] = y[i];
    }
    return r;
}

/* mul (main.rs:2321-2326): (m * (v, 1.0)).xyz */
static Vec3 m44_mul_point(const M44* m, Vec3 v) {
    double x[4] = {v.x, v.y, v.z, 1.0}, y[4];
    m44_gemv(m, x, y);
    return v3(y[0], y[1], y[2]);
}

/* Perspective3::new(aspect, fovy, znear, zfar).to_homogeneous() */
static M44 perspective3(double aspect, double fovy, double znear, double zfar) {
    M44 p = m44_identity();
    double old_m22 = p.m[1][1];
    p.m[1][1] = 1.0 / tan(fovy / 2.0);
    p.m[0][0] = p.m[0][0] * (p.m[1][1] / old_m22);
    p.m[0][0] = p.m[1][1] / aspect;
    p.m[2][2] = (zfar + znear) / (znear - zfar);
    p.m[2][3] = zfar * znear * 2.0 / (znear - zfar);
    p.m[3][3] = 0.0;
    p.m[3][2] = -1.0;
    return p;
}

/* projectSphere (main.rs:2796-2837): center and the two ellipse axes */
static void projectSphere(const double sphere[4], const M44* cameraMat, double fle, Vec2* center, Vec2* axa,
                          Vec2* axb) {
    Vec3 o = m44_mul_point(cameraMat, v3(sphere[0], sphere[1], sphere[2]));
    double r2 = sphere[3] * sphere[3];
    double z2 = o.z * o.z;
    double l2 = dot(o, o);
    *axa = v2_scale(v2(o.x, o.y), fle * sqrt(-r2 * (r2 - l2) / ((l2 - z2) * (r2 - z2) * (r2 - z2))));
    *axb = v2_scale(v2(-o.y, o.x), fle * sqrt(-r2 * (r2 - l2) / ((l2 - z2) * (r2 - z2) * (r2 - l2))));
    *center = v2_scale(v2(o.x, o.y), fle * o.z / (z2 - r2));
}

/* Viewport::rasterize's per-sphere projection, PERSPECTIVE branch (main.rs:473-524).
 * The image aspect generalises (512 as f64) / (512 as f64) (main.rs:496) to W / H. */
void rtmo_project_sphere_perspective(const rtm_camera* cam, int32_t W, int32_t H, const double pos[3], double r,
                                     double out[6]) {
    Camera c = camera_from(cam, W, H);
    M44 rel;
    memset(&rel, 0, sizeof rel);
    rel.m[0][0] = c.side.x; rel.m[0][1] = c.side.y; rel.m[0][2] = c.side.z;
    rel.m[1][0] = c.up.x;   rel.m[1][1] = c.up.y;   rel.m[1][2] = c.up.z;
    rel.m[2][0] = c.dir.x;  rel.m[2][1] = c.dir.y;  rel.m[2][2] = c.dir.z;
    rel.m[3][3] = 1.0;
    Vec3 local = m44_mul_point(&rel, v3_sub(v3(pos[0], pos[1], pos[2]), c.pos));
    double fov = 3.14 / 2.0;
    M44 persp = perspective3((double)W / (double)H, fov, 0.1, 1000.0);
    M44 refl = m44_identity();
    refl.m[2][2] = -1.0;  /* new_nonuniform_scaling(&Vector3::new(1.0, 1.0, -1.0)) */
    M44 cameraMat = m44_mul(&persp, &refl);
    double sphere4[4] = {local.x, local.y, local.z, r};
    Vec2 center, axa, axb;
    projectSphere(sphere4, &cameraMat, fov, &center, &axa, &axb);
    out[0] = center.x;
    out[1] = center.y;
    out[2] = axa.x;
    out[3] = axa.y;
    out[4] = axb.x;
    out[5] = axb.y;
}

/* Viewport::rasterize (main.rs:445-547) over rows [y0,y1): ORTHOGONAL
 * (main.rs:452-471) or PERSPECTIVE (main.rs:473-524, row f-3) projection,
 * then rasterizeSphere (main.rs:540-542). */
static int viewport_rasterize(Viewport* vp, const rtm_scene* scene, int flags, int64_t y0, int64_t y1,
                              int64_t* tests) {
    if (scene->n_spheres == 0) return RTM_OK;
    if (vp->camera.type != RTM_CAMERA_ORTHOGONAL) {
        rtm_camera cc;
        memset(&cc, 0, sizeof cc);
        cc.type = vp->camera.type;
        cc.pos[0] = vp->camera.pos.x; cc.pos[1] = vp->camera.pos.y; cc.pos[2] = vp->camera.pos.z;
        cc.dir[0] = vp->camera.dir.x; cc.dir[1] = vp->camera.dir.y; cc.dir[2] = vp->camera.dir.z;
        cc.up[0] = vp->camera.up.x;   cc.up[1] = vp->camera.up.y;   cc.up[2] = vp->camera.up.z;
        cc.side[0] = vp->camera.side.x; cc.side[1] = vp->camera.side.y; cc.side[2] = vp->camera.side.z;
        for (int32_t i = 0; i < scene->n_spheres; i++) {
            const rtm_sphere* s = &scene->spheres[i];
            Vec3 pos = v3(s->pos[0], s->pos[1], s->pos[2]);
            double pr[6];
            rtmo_project_sphere_perspective(&cc, (int32_t)vp->W, (int32_t)vp->H, s->pos, s->r, pr);
            ProjectedSphere ps;
            ps.id = s->id;
            ps.z = calcDepthOfProjectedPoint(&vp->camera, pos);
            ps.center = v2(pr[0], pr[1]);
            ps.r = s->r;
            ps.axisA = v2(pr[2], pr[3]);
            ps.axisB = v2(pr[4], pr[5]);
            rasterizeSphere(&ps, ps.r, vp, flags, y0, y1, tests);
        }
        return RTM_OK;
    }
    for (int32_t i = 0; i < scene->n_spheres; i++) {
        const rtm_sphere* s = &scene->spheres[i];
        Vec3 pos = v3(s->pos[0], s->pos[1], s->pos[2]);
        double z = calcDepthOfProjectedPoint(&vp->camera, pos);
        Vec3 projectedPosition = camera_project(&vp->camera, pos);
        ProjectedSphere ps;
        ps.id = s->id;
        ps.z = z;
        ps.center = v2(projectedPosition.x, projectedPosition.y);
        ps.r = s->r;
        ps.axisA = v2(s->r, 0.0);
        ps.axisB = v2(0.0, s->r);
        rasterizeSphere(&ps, ps.r, vp, flags, y0, y1, tests);
    }
    return RTM_OK;
}

/* ------------------------------------------------------------------ */
/* L2 implicit-surface march (main.rs:2016-2051, 2066-2080, 2133-2284) */
/* ------------------------------------------------------------------ */
/* linear (main.rs:2066-2069) */
static double linear(double t, double a, double b) {
    double diff = b - a;
    return a + diff * t;
}
/* bilinear (main.rs:2073-2080) */
static double bilinear(Vec2 t, double d00, double d01, double d10, double d11) {
    double d0 = linear(t.x, d00, d01);
    double d1 = linear(t.x, d10, d11);
    return linear(t.y, d0, d1);
}
/* calcDepthBilinear (main.rs:2146-2148) */
static double calcDepthBilinear(Vec3 p, const rtm_patch* b) {
    return bilinear(v2(p.x, p.y), b->a0, b->b0, b->a1, b->b1);
}
/* inRange01 (main.rs:2282-2284) */
static int inRange01(double v) { return fabs(v - 0.5) <= 0.5; }

/* raymarchPatch (main.rs:2219-2278).  The normal (calcNormalBilinear,
 * main.rs:2151-2174) is computed by the reference but discarded by its only
 * caller (main.rs:2047), so it is not restated. */
static int raymarchPatch(Vec3 pStart, Vec3 dir, int64_t steps, const rtm_patch* patch, double* tOut,
                         int64_t* iters) {
    const int checkBoundsIteration = 1;
    double magnitudeOfStepsize = 0.03;
    Vec3 step = v3_scale(dir, magnitudeOfStepsize);
    Vec3 p = pStart;
    double t = 0.0;
    double signEntry;
    {
        double depthOfSurface = calcDepthBilinear(p, patch);
        signEntry = rust_signum(p.z - depthOfSurface);
    }
    for (int64_t s = 0; s < steps; s++) {
        if (iters) (*iters)++;
        if (checkBoundsIteration) {
            if (!inRange01(p.x) || !inRange01(p.y)) {
                p = v3_add(p, step);
                t += magnitudeOfStepsize;
                continue;
            }
        }
        double depthOfSurface = calcDepthBilinear(p, patch);
        double sign = rust_signum(p.z - depthOfSurface);
        if (sign != signEntry) {
            *tOut = t;
            return 1;
        }
        p = v3_add(p, step);
        t += magnitudeOfStepsize;
    }
    return 0;
}

/* raymarchPatchDomainM11 (main.rs:2179-2197) */
static int raymarchPatchDomainM11(Vec3 pStart, Vec3 dir, int64_t steps, const rtm_patch* patch,
                                  double* tOut, int64_t* iters) {
    double x = (pStart.x + 1.0) * 0.5;
    double y = (pStart.y + 1.0) * 0.5;
    return raymarchPatch(v3(x, y, pStart.z), dir, steps, patch, tOut, iters);
}

/* Viewport::processRaymarchingRays + rayEntry_ShadowRay_testing (main.rs:551-565,
 * 2022-2051), with the patch list and step count as arguments. */
static void viewport_process_raymarching_rays(Viewport* vp, const rtm_patch* patches, int32_t n_patches,
                                              int64_t steps, int64_t y0, int64_t y1, Counts* cnt) {
    for (int64_t yi = y0; yi < y1; yi++) {
        for (int64_t xi = 0; xi < vp->W; xi++) {
            for (int32_t k = 0; k < n_patches; k++) {
                Vec3 pStart, dirN;
                calcRayOriginAndDirection(&vp->camera, xi, yi, &pStart, &dirN);
                if (cnt) {
                    double mx = (pStart.x + 1.0) * 0.5, my = (pStart.y + 1.0) * 0.5;
                    if (inRange01(mx) && inRange01(my)) cnt->march_in_range++;
                }
                double rayDepth;
                if (raymarchPatchDomainM11(pStart, dirN, steps, &patches[k], &rayDepth,
                                           cnt ? &cnt->march_iterations : NULL)) {
                    if (cnt) cnt->march_hits++;
                    int64_t idx = (yi - vp->y0) * vp->W + xi;
                    if (rayDepth < vp->zBuffer[idx]) vp->zBuffer[idx] = rayDepth;
                }
            }
        }
    }
}

/* ------------------------------------------------------------------ */
/* L2 ray-traced primitives (row f-1: main.rs:569-642, 2390-2408, 2884-2974) */
/* ------------------------------------------------------------------ */
/* calcRayPlane (main.rs:2398-2408); returns 1 and *t on Some */
static int calcRayPlane(Vec3 rayOrigin, Vec3 rayDir, Vec3 planeN, Vec3 planeCenter, double* t) {
    double denom = dot(planeN, rayDir);
    if (fabs(denom) > 0.0001) {
        *t = dot(v3_sub(planeCenter, rayOrigin), planeN) / denom;
        return 1;
    }
    return 0;
}

/* dot2 (main.rs:2884-2886), inversesqrt (main.rs:2963-2965), sign (main.rs:2967-2974) */
static double dot2(Vec3 v) { return dot(v, v); }
static double inversesqrt(double v) { return 1.0 / sqrt(v); }
static double sign_of(double v) { return v >= 0.0 ? 1.0 : -1.0; }

/* iCappedCone (main.rs:2889-2959; Inigo Quilez's capped-cone intersector
 * restated in the reference's f64 operation order).  Returns (t, normal);
 * t = -1 and normal = (-1,-1,-1) on a miss. */
static double iCappedCone(Vec3 ro, Vec3 rd, Vec3 pa, Vec3 pb, double ra, double rb, Vec3* nOut) {
    Vec3 ba = v3_sub(pb, pa);
    Vec3 oa = v3_sub(ro, pa);
    Vec3 ob = v3_sub(ro, pb);
    double baba = dot(ba, ba);
    double rdba = dot(rd, ba);
    double oaba = dot(oa, ba);
    double obba = dot(ob, ba);
    /* caps */
    if (oaba < 0.0) {
        if (dot2(v3_sub(v3_scale(oa, rdba), v3_scale(rd, oaba))) < ra * ra * rdba * rdba) {
            *nOut = v3_scale(ba, -inversesqrt(baba));
            return -oaba / rdba;
        }
    } else if (obba > 0.0) {
        double t = -obba / rdba;
        if (dot2(v3_add(ob, v3_scale(rd, t))) < rb * rb) {
            *nOut = v3_scale(ba, inversesqrt(baba));
            return t;
        }
    }
    /* body */
    double rr = rb - ra;
    double hy = baba + rr * rr;
    Vec3 oc = v3_sub(v3_scale(oa, rb), v3_scale(ob, ra));
    double ocba = dot(oc, ba);
    double ocrd = dot(oc, rd);
    double ococ = dot(oc, oc);
    double k2 = baba * baba - hy * rdba * rdba;
    double k1 = baba * baba * ocrd - hy * rdba * ocba;
    double k0 = baba * baba * ococ - hy * ocba * ocba;
    double h = k1 * k1 - k2 * k0;
    if (h < 0.0) {
        *nOut = v3(-1.0, -1.0, -1.0);
        return -1.0;
    }
    double t = (-k1 - sign_of(rr) * sqrt(h)) / (k2 * rr);
    double y = oaba + rdba * t;
    if (y > 0.0 && y < baba) {
        Vec3 insideNormalize = v3_sub(v3_scale(v3_sub(v3_scale(v3_add(oa, v3_scale(rd, t)), baba), v3_scale(ba, rr * ra)), baba),
                                      v3_scale(ba, hy * y));
        *nOut = normalize(insideNormalize);
        return t;
    }
    *nOut = v3(-1.0, -1.0, -1.0);
    return -1.0;
}

/* ---- row f-4: the GL preview's SDF implicit surface, restated in f64 ----
 * entry.frag is GLSL (f32, implementation-defined min/max/normalize); this
 * restatement fixes the f64 semantics the GPU kernels share:
 *   min/max: NaN-ignoring, +0 > -0;  sign: GLSL (0 for 0 and NaN);
 *   cross(x, y) = (x.y y.z - y.y x.z, x.z y.x - y.z x.x, x.x y.y - y.x x.y) (GLSL spec);
 *   normalize(v) = v * (1 / sqrt(dot(v, v)));  dot = (x + y) + z;
 *   sBox's translate(-c) applied as ro - c, rd unchanged. */
static double fmax_d(double a, double b) {
    if (isnan(a)) return b;
    if (isnan(b)) return a;
    if (a > b) return a;
    if (b > a) return b;
    return signbit(a) ? b : a;
}
static double fmin_d(double a, double b) {
    if (isnan(a)) return b;
    if (isnan(b)) return a;
    if (a < b) return a;
    if (b < a) return b;
    return signbit(a) ? a : b;
}
static double glsl_sign(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : 0.0); }
static Vec3 cross3(Vec3 x, Vec3 y) {
    return v3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y);
}

typedef struct {
    Vec3 box;                  /* descriptor vecs[0] */
    Vec3 v1, v2, v3;           /* triangle (entry.frag:436) */
    Vec3 v21, v32, v13, nor;   /* udTriangleSingle's point-independent terms (entry.frag:318-321) */
    Vec3 c1, c2, c3;           /* cross(v21,nor), cross(v32,nor), cross(v13,nor) */
    double d21, d32, d13, dnor;
} SdfGeom;

static void sdf_geom(const rtm_sdf* s, SdfGeom* g) {
    Vec3 a = v3(s->tri_anchor[0], s->tri_anchor[1], s->tri_anchor[2]);
    g->box = v3(s->box_center[0], s->box_center[1], s->box_center[2]);
    g->v1 = v3_add(a, v3(0.8, 0.8, 0.8));
    g->v2 = v3_add(a, v3(1.3, 0.8, 0.8));
    g->v3 = v3_add(a, v3(1.0, 0.7, 0.2));
    g->v21 = v3_sub(g->v2, g->v1);
    g->v32 = v3_sub(g->v3, g->v2);
    g->v13 = v3_sub(g->v1, g->v3);
    g->nor = cross3(g->v21, g->v13);
    g->c1 = cross3(g->v21, g->nor);
    g->c2 = cross3(g->v32, g->nor);
    g->c3 = cross3(g->v13, g->nor);
    g->d21 = dot(g->v21, g->v21);
    g->d32 = dot(g->v32, g->v32);
    g->d13 = dot(g->v13, g->v13);
    g->dnor = dot(g->nor, g->nor);
}

/* sdBox (entry.frag:290-298) */
static double sdBox(Vec3 p, Vec3 b) {
    Vec3 d = v3(fabs(p.x) - b.x, fabs(p.y) - b.y, fabs(p.z) - b.z);
    Vec3 m = v3(fmax_d(d.x, 0.0), fmax_d(d.y, 0.0), fmax_d(d.z, 0.0));
    return fmin_d(fmax_d(d.x, fmax_d(d.y, d.z)), 0.0) + sqrt(dot(m, m));
}

/* udTriangleSingle (entry.frag:312-340): the SQUARED distance */
static double udTriangleSingle(const SdfGeom* g, Vec3 p) {
    Vec3 p1 = v3_sub(p, g->v1), p2 = v3_sub(p, g->v2), p3 = v3_sub(p, g->v3);
    if (glsl_sign(dot(g->c1, p1)) + glsl_sign(dot(g->c2, p2)) + glsl_sign(dot(g->c3, p3)) < 2.0) {
        Vec3 e1 = v3_sub(v3_scale(g->v21, fmin_d(fmax_d(dot(g->v21, p1) / g->d21, 0.0), 1.0)), p1);
        Vec3 e2 = v3_sub(v3_scale(g->v32, fmin_d(fmax_d(dot(g->v32, p2) / g->d32, 0.0), 1.0)), p2);
        Vec3 e3 = v3_sub(v3_scale(g->v13, fmin_d(fmax_d(dot(g->v13, p3) / g->d13, 0.0), 1.0)), p3);
        return fmin_d(fmin_d(dot(e1, e1), dot(e2, e2)), dot(e3, e3));
    }
    double dn = dot(g->nor, p1);
    return dn * dn / g->dnor;
}

/* distanceFn0 (entry.frag:416-442) */
static double distanceFn0(const SdfGeom* g, Vec3 p) {
    double d0 = sdBox(v3_sub(p, g->box), v3(0.4, 0.2, 0.2));
    double d1 = udTriangleSingle(g, p);
    double d2 = fmin_d(d0, d1);
    d2 -= 0.2;
    return d2;
}

/* sBox (entry.frag:85-110) with txx = translate(-center) */
static double sBox(Vec3 ro, Vec3 rd, Vec3 center, Vec3 rad, int checkFirstIntersection) {
    Vec3 roo = v3_sub(ro, center);
    Vec3 m = v3(1.0 / rd.x, 1.0 / rd.y, 1.0 / rd.z);
    Vec3 n = v3(m.x * roo.x, m.y * roo.y, m.z * roo.z);
    Vec3 k = v3(fabs(m.x) * rad.x, fabs(m.y) * rad.y, fabs(m.z) * rad.z);
    Vec3 t1 = v3(-n.x - k.x, -n.y - k.y, -n.z - k.z);
    Vec3 t2 = v3(-n.x + k.x, -n.y + k.y, -n.z + k.z);
    double tN = fmax_d(fmax_d(t1.x, t1.y), t1.z);
    double tF = fmin_d(fmin_d(t2.x, t2.y), t2.z);
    if (checkFirstIntersection && (tN > tF || tF < 0.0)) return -1.0;
    return tN;
}

/* The implicit-surface branch of bvhProcessLeafHit (entry.frag:842-917): t of
 * the hit or -1, and the sdNormalFast normal (entry.frag:356-364, 893-905). */
static double traceSdf(const rtm_sdf* s, const SdfGeom* g, Vec3 ro, Vec3 rd, Vec3* nOut, int64_t* evals) {
    Vec3 c = v3(s->aabb_center[0], s->aabb_center[1], s->aabb_center[2]);
    Vec3 e = v3(s->aabb_extent[0], s->aabb_extent[1], s->aabb_extent[2]);
    double tIn = sBox(ro, rd, c, e, 1);
    if (!(tIn >= 0.0)) return -1.0;
    double tOut = -sBox(ro, v3(-rd.x, -rd.y, -rd.z), c, e, 0);
    double t = tIn;
    int hit = 0;
    for (int32_t stepI = 0; stepI < s->max_steps; stepI++) {
        Vec3 p = v3_add(ro, v3_scale(rd, t));
        double distance = distanceFn0(g, p);
        if (evals) ++*evals;
        if (distance < 0.03) {
            hit = 1;
            break;
        }
        if (t > tOut) break;
        t += distance;
    }
    if (!hit) return -1.0;
    if (evals) *evals += 4;
    Vec3 p = v3_add(ro, v3_scale(rd, t));
    const double h = 0.001;
    double pnn = distanceFn0(g, v3_add(p, v3(1.0 * h, -1.0 * h, -1.0 * h)));
    double nnp = distanceFn0(g, v3_add(p, v3(-1.0 * h, -1.0 * h, 1.0 * h)));
    double npn = distanceFn0(g, v3_add(p, v3(-1.0 * h, 1.0 * h, -1.0 * h)));
    double ppp = distanceFn0(g, v3_add(p, v3(1.0 * h, 1.0 * h, 1.0 * h)));
    Vec3 v = v3(((1.0 * pnn + -1.0 * nnp) + -1.0 * npn) + 1.0 * ppp,
                ((-1.0 * pnn + -1.0 * nnp) + 1.0 * npn) + 1.0 * ppp,
                ((-1.0 * pnn + 1.0 * nnp) + -1.0 * npn) + 1.0 * ppp);
    *nOut = normalize(v);
    return t;
}

/* test hooks */
double rtmo_sdf_distance(const rtm_sdf* s, const double p[3]) {
    SdfGeom g;
    sdf_geom(s, &g);
    return distanceFn0(&g, v3(p[0], p[1], p[2]));
}
double rtmo_sdf_trace(const rtm_sdf* s, const double ro[3], const double rd[3], double n[3], int64_t* evals) {
    SdfGeom g;
    sdf_geom(s, &g);
    Vec3 nn = v3(0.0, 0.0, 0.0);
    double t = traceSdf(s, &g, v3(ro[0], ro[1], ro[2]), v3(rd[0], rd[1], rd[2]), &nn, evals);
    n[0] = nn.x;
    n[1] = nn.y;
    n[2] = nn.z;
    return t;
}

/* Viewport::processRaytracingRays (main.rs:569-642) over rows [y0,y1) */
static void viewport_process_raytracing_rays(Viewport* vp, const rtm_scene* scene, int64_t y0, int64_t y1,
                                             int64_t* evals) {
    SdfGeom geoms[RTM_MAX_SDFS];
    for (int32_t i = 0; i < scene->n_sdfs && i < RTM_MAX_SDFS; i++) sdf_geom(&scene->sdfs[i], &geoms[i]);
    for (int64_t yi = y0; yi < y1; yi++) {
        for (int64_t xi = 0; xi < vp->W; xi++) {
            Vec3 o, d;
            calcRayOriginAndDirection(&vp->camera, xi, yi, &o, &d);
            int64_t idx = (yi - vp->y0) * vp->W + xi;
            for (int32_t i = 0; i < scene->n_circle_planes; i++) {
                const rtm_circle_plane* pl = &scene->circle_planes[i];
                Vec3 n = v3(pl->n[0], pl->n[1], pl->n[2]);
                Vec3 c = v3(pl->pos[0], pl->pos[1], pl->pos[2]);
                double t;
                if (!calcRayPlane(o, d, n, c, &t)) continue;
                if (t < 0.0) continue;                   /* behind the camera */
                if (t > vp->zBuffer[idx]) continue;      /* behind a known intersection */
                Vec3 p = v3_add(o, v3_scale(d, t));
                double distance = v3_magnitude(v3_sub(p, c));
                if (distance > pl->radius) continue;
                GEntry* g = &vp->rasterized[idx];
                g->some = GK_PLANE;
                g->id = pl->id;
                g->rayT = t;
                vp->zBuffer[idx] = t;
            }
            for (int32_t i = 0; i < scene->n_capped_cylinders; i++) {
                const rtm_capped_cylinder* cy = &scene->capped_cylinders[i];
                Vec3 n;
                double t = iCappedCone(o, d, v3(cy->pa[0], cy->pa[1], cy->pa[2]), v3(cy->pb[0], cy->pb[1], cy->pb[2]),
                                       cy->ra, cy->rb, &n);
                if (t < 0.0) continue;
                if (t > vp->zBuffer[idx]) continue;
                GEntry* g = &vp->rasterized[idx];
                g->some = GK_CYLINDER;
                g->id = cy->id;
                g->rayT = t;
                g->n = n;
                vp->zBuffer[idx] = t;
            }
            for (int32_t i = 0; i < scene->n_sdfs; i++) {
                /* row f-4, after the cylinders; the shader's acceptance: 0 < t < depth (entry.frag:908-917) */
                Vec3 n;
                double t = traceSdf(&scene->sdfs[i], &geoms[i], o, d, &n, evals);
                if (!(t > 0.0) || !(t < vp->zBuffer[idx])) continue;
                GEntry* g = &vp->rasterized[idx];
                g->some = GK_SDF;
                g->id = scene->sdfs[i].id;
                g->rayT = t;
                g->n = n;
                vp->zBuffer[idx] = t;
            }
        }
    }
}

/* ------------------------------------------------------------------ */
/* L3 shading (main.rs:155-173, 709-902, 2872-2875)                    */
/* ------------------------------------------------------------------ */
/* reflect (main.rs:2872-2875) — sign-flipped as written */
static Vec3 reflect(Vec3 d, Vec3 n) { return v3_sub(d, v3_scale(n, -2.0 * dot(d, n))); }

/* renderColorImage (main.rs:710-902) over rows [y0,y1).  out holds the eye
 * viewport's rows from vp->y0.  texrows (nullable): instead of shading, record
 * the range of shadow-map rows the hit pixels look up (rtmo_render_rows). */
static void renderColorImage(const rtm_scene* scene, const Viewport* vp, const Viewport* vps, float* out,
                             int64_t y0, int64_t y1, Counts* cnt, int64_t* texrows) {
    for (int64_t iy = y0; iy < y1; iy++) {
        for (int64_t ix = 0; ix < vp->W; ix++) {
            const GEntry* iPixel = &vp->rasterized[(iy - vp->y0) * vp->W + ix];
            double r = 0.0, g = 0.2, b = 0.2;
            if (iPixel->some) {
                Vec3 viewDir = retViewDirOfPixel(&vp->camera, ix, iy);
                Vec3 worldPosition, normal;
                const double* color;
                Vec3 o, d;
                calcRayOriginAndDirection(&vp->camera, ix, iy, &o, &d);
                if (iPixel->some == GK_SPHERE) { /* main.rs:731-755 */
                    const rtm_sphere* prim = &scene->spheres[iPixel->id];
                    /* calcDepth (main.rs:155-165) */
                    double rMulHeight = iPixel->relativeHeight * prim->r;
                    double depth = calcZValueOfProjectedSphere(iPixel->z, rMulHeight, RTM_FACE_FRONT);
                    worldPosition = v3_add(o, v3_scale(d, depth));
                    Vec3 diffOfPositionToCenter = v3_sub(worldPosition, v3(prim->pos[0], prim->pos[1], prim->pos[2]));
                    normal = v3_scale(diffOfPositionToCenter, 1.0 / prim->r);
                    color = prim->color;
                } else if (iPixel->some == GK_PLANE) { /* main.rs:761-777; calcDepth = rayT (main.rs:166-168) */
                    worldPosition = v3_add(o, v3_scale(d, iPixel->rayT));
                    const rtm_circle_plane* pl = &scene->circle_planes[iPixel->id];
                    color = pl->color;
                    normal = v3(pl->n[0], pl->n[1], pl->n[2]);
                } else if (iPixel->some == GK_CYLINDER) { /* main.rs:779-795; calcDepth = rayT (main.rs:169-171) */
                    worldPosition = v3_add(o, v3_scale(d, iPixel->rayT));
                    color = scene->capped_cylinders[iPixel->id].color;
                    normal = iPixel->n;
                } else { /* row f-4: shaded like the cylinder kind, with the sdNormalFast normal */
                    worldPosition = v3_add(o, v3_scale(d, iPixel->rayT));
                    color = scene->sdfs[iPixel->id].color;
                    normal = iPixel->n;
                }

                Vec3 incommingLightDir = v3(1.0, 0.0, 0.0);
                Vec3 invertedIncommingLightDir = v3_scale(incommingLightDir, -1.0);
                double diffuse = dot(normal, invertedIncommingLightDir);
                diffuse = rust_max(diffuse, 0.0);
                Vec3 reflectionDir = reflect(invertedIncommingLightDir, normal);
                double specularMagnitude = powi(rust_max(dot(viewDir, reflectionDir), 0.0), 32);
                double lightMagnitude = 1.0;

                /* shadow mapping (main.rs:834-857) */
                Vec3 projectedPosition = camera_project(&vps->camera, worldPosition);
                int64_t halfW = vps->W / 2, halfH = vps->H / 2;
                int64_t texX = wrap_add_i64(halfW, rust_as_i64(projectedPosition.x * (double)halfW));
                int64_t texY = wrap_add_i64(halfH, rust_as_i64(projectedPosition.y * (double)halfH));
                double depthFromShadowMap = INFINITY;
                if (texrows) {
                    if (texY >= 0 && texY < vps->H && texX >= 0 && texX < vps->W) {
                        if (texY < texrows[0]) texrows[0] = texY;
                        if (texY > texrows[1]) texrows[1] = texY;
                    }
                    continue;
                }
                if (texY >= 0 && texY < vps->H && texX >= 0 && texX < vps->W) {
                    if (texY < vps->y0 || texY >= vps->y0 + vps->rows) abort(); /* outside the row window */
                    depthFromShadowMap = vps->zBuffer[(texY - vps->y0) * vps->W + texX];
                }
                double bias = 0.0;
                int inLight = depthFromShadowMap > projectedPosition.z - bias;
                if (!inLight) lightMagnitude = 0.25;

                r = (diffuse + specularMagnitude) * lightMagnitude * color[0];
                g = (diffuse + specularMagnitude) * lightMagnitude * color[1];
                b = (diffuse + specularMagnitude) * lightMagnitude * color[2];
                if (cnt) {
                    cnt->eye_hit_pixels++;
                    if (iPixel->some == GK_SPHERE && iPixel->id >= 0 && iPixel->id < RTM_MAX_SPHERES)
                        cnt->eye_hits[iPixel->id]++;
                    if (iPixel->some == GK_PLANE) cnt->eye_circle_plane_pixels++;
                    if (iPixel->some == GK_CYLINDER) cnt->eye_capped_cylinder_pixels++;
                    if (iPixel->some == GK_SDF) cnt->eye_sdf_pixels++;
                    if (inLight) cnt->lit_pixels++;
                }
            }
            if (texrows) continue;
            float* px = out + 4 * ((iy - vp->y0) * vp->W + ix);
            px[0] = (float)r;
            px[1] = (float)g;
            px[2] = (float)b;
            px[3] = 1.0f;
        }
    }
}

/* ------------------------------------------------------------------ */
/* Exported oracle API (prefix rtmo_)                                   */
/* ------------------------------------------------------------------ */
static int validate_scene(const rtm_scene* scene) {
    if (!scene || scene->n_spheres < 0 || scene->n_patches < 0) return RTM_ERR_INVALID;
    if (scene->n_spheres > 0 && !scene->spheres) return RTM_ERR_INVALID;
    if (scene->n_patches > 0 && !scene->patches) return RTM_ERR_INVALID;
    for (int32_t i = 0; i < scene->n_spheres; i++)
        if (scene->spheres[i].id < 0 || scene->spheres[i].id >= scene->n_spheres) return RTM_ERR_INVALID;
    if (scene->n_circle_planes < 0 || scene->n_capped_cylinders < 0) return RTM_ERR_INVALID;
    if (scene->n_circle_planes > 0 && !scene->circle_planes) return RTM_ERR_INVALID;
    if (scene->n_capped_cylinders > 0 && !scene->capped_cylinders) return RTM_ERR_INVALID;
    for (int32_t i = 0; i < scene->n_circle_planes; i++)
        if (scene->circle_planes[i].id < 0 || scene->circle_planes[i].id >= scene->n_circle_planes)
            return RTM_ERR_INVALID;
    for (int32_t i = 0; i < scene->n_capped_cylinders; i++)
        if (scene->capped_cylinders[i].id < 0 || scene->capped_cylinders[i].id >= scene->n_capped_cylinders)
            return RTM_ERR_INVALID;
    if (scene->n_sdfs < 0 || scene->n_sdfs > RTM_MAX_SDFS || (scene->n_sdfs > 0 && !scene->sdfs)) return RTM_ERR_INVALID;
    for (int32_t i = 0; i < scene->n_sdfs; i++)
        if (scene->sdfs[i].id < 0 || scene->sdfs[i].id >= scene->n_sdfs || scene->sdfs[i].max_steps < 0)
            return RTM_ERR_INVALID;
    return RTM_OK;
}

static void viewport_init_rows(Viewport* vp, int64_t W, int64_t H, int face, const rtm_camera* cam, int64_t y0,
                               int64_t rows) {
    vp->W = W;
    vp->H = H;
    vp->face = face;
    vp->camera = camera_from(cam, W, H);
    vp->y0 = y0;
    vp->rows = rows;
    vp->zBuffer = (double*)malloc(sizeof(double) * (size_t)(W * rows));
    vp->rasterized = (GEntry*)calloc((size_t)(W * rows), sizeof(GEntry));
    for (int64_t i = 0; i < W * rows; i++) vp->zBuffer[i] = INFINITY;
}

static void viewport_init(Viewport* vp, int64_t W, int64_t H, int face, const rtm_camera* cam) {
    viewport_init_rows(vp, W, H, face, cam, 0, H);
}

static void viewport_free(Viewport* vp) {
    free(vp->zBuffer);
    free(vp->rasterized);
}

int32_t rtmo_abi_version(void) { return RTM_ABI_VERSION; }

/* Whole two-viewport frame (testscene_closelyOrbitingSphere body, main.rs:1533-1628).
 * nthreads<=1: single thread, the reference's sequential loops; otherwise
 * OpenMP over row bands (pixels are independent; per-pixel sphere order kept).
 * out_shadow (nullable): the shadow viewport's zBuffer.  stats (nullable). */
int rtmo_render(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t W,
                int32_t H, int32_t steps, int32_t flags, int32_t nthreads, float* out_rgba,
                double* out_shadow, rtm_stats* stats) {
    int rc = validate_scene(scene);
    if (rc) return rc;
    if (!eye || !shadow || !out_rgba || W <= 0 || H <= 0 || steps < 0) return RTM_ERR_INVALID;
    if (shadow->type != RTM_CAMERA_ORTHOGONAL) return RTM_ERR_UNSUPPORTED;
    Viewport vs, ve;
    viewport_init(&vs, W, H, RTM_FACE_BACK, shadow);
    viewport_init(&ve, W, H, RTM_FACE_FRONT, eye);
    Counts total;
    memset(&total, 0, sizeof total);
    int nt = nthreads < 1 ? 1 : nthreads;
    int64_t band = 8;
    int64_t nb = (H + band - 1) / band;

    /* pass 1: shadow viewport rasterize + march; pass 2: eye rasterize; pass 3: shade.
     * Rows are independent within a pass, so bands may run in any order. */
    for (int pass = 0; pass < 3; pass++) {
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nt)
#endif
        for (int64_t bi = 0; bi < nb; bi++) {
            int64_t y0 = bi * band, y1 = y0 + band < H ? y0 + band : H;
            Counts c;
            memset(&c, 0, sizeof c);
            if (pass == 0) {
                if (!(flags & RTM_FLAG_NO_SHADOW_RASTER))
                    viewport_rasterize(&vs, scene, flags, y0, y1, &c.shadow_sphere_tests);
                if (!(flags & RTM_FLAG_NO_MARCH))
                    viewport_process_raymarching_rays(&vs, scene->patches, scene->n_patches, steps, y0, y1, &c);
            } else if (pass == 1) {
                viewport_rasterize(&ve, scene, flags, y0, y1, &c.eye_sphere_tests);
                viewport_process_raytracing_rays(&ve, scene, y0, y1, &c.sdf_distance_evals);
                c.eye_plane_tests = (y1 - y0) * W * scene->n_circle_planes;  /* every pixel, every primitive */
                c.eye_cylinder_tests = (y1 - y0) * W * scene->n_capped_cylinders;
            } else {
                renderColorImage(scene, &ve, &vs, out_rgba, y0, y1, &c, NULL);
            }
#ifdef _OPENMP
#pragma omp critical
#endif
            {
                int64_t* dst = (int64_t*)&total;
                const int64_t* src = (const int64_t*)&c;
                for (size_t k = 0; k < sizeof(Counts) / sizeof(int64_t); k++) dst[k] += src[k];
            }
        }
    }
    if (out_shadow) memcpy(out_shadow, vs.zBuffer, sizeof(double) * (size_t)W * (size_t)H);
    if (stats) memcpy(stats, &total, sizeof total);
    viewport_free(&vs);
    viewport_free(&ve);
    return RTM_OK;
}

/* Eye rows [r0, r1) of the W x H frame, without holding the whole frame: the
 * eye viewport holds only those rows, and the shadow viewport only the rows
 * [t0, t1] the band's hit pixels look up (found by a first shading pass that
 * records texY instead of shading).  Same functions, same order: the rows are
 * bit-identical to rtmo_render's.  For maximum-size parity checks (RTM_MAX_DIM),
 * where the full frame would not fit the host.  out_rgba: (r1 - r0) * W * 4
 * floats; t0_out, t1_out (nullable): the shadow rows computed (t1 < t0 when the
 * band looks nothing up). */
int rtmo_render_rows(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t W,
                     int32_t H, int32_t steps, int32_t flags, int32_t r0, int32_t r1, float* out_rgba,
                     int64_t* t0_out, int64_t* t1_out) {
    int rc = validate_scene(scene);
    if (rc) return rc;
    if (!eye || !shadow || !out_rgba || W <= 0 || H <= 0 || steps < 0 || r0 < 0 || r1 > H || r0 >= r1)
        return RTM_ERR_INVALID;
    if (shadow->type != RTM_CAMERA_ORTHOGONAL) return RTM_ERR_UNSUPPORTED;
    Viewport ve, vs;
    viewport_init_rows(&ve, W, H, RTM_FACE_FRONT, eye, r0, r1 - r0);
    viewport_rasterize(&ve, scene, flags, r0, r1, NULL);
    viewport_process_raytracing_rays(&ve, scene, r0, r1, NULL);
    int64_t tr[2] = {H, -1};
    viewport_init_rows(&vs, W, H, RTM_FACE_BACK, shadow, 0, 0);  /* camera only, for the texel rows */
    renderColorImage(scene, &ve, &vs, out_rgba, r0, r1, NULL, tr);
    viewport_free(&vs);
    const int64_t t0 = tr[1] >= tr[0] ? tr[0] : 0, t1 = tr[1] >= tr[0] ? tr[1] : -1;
    viewport_init_rows(&vs, W, H, RTM_FACE_BACK, shadow, t0, t1 - t0 + 1);
    if (t1 >= t0) {
        if (!(flags & RTM_FLAG_NO_SHADOW_RASTER)) viewport_rasterize(&vs, scene, flags, t0, t1 + 1, NULL);
        if (!(flags & RTM_FLAG_NO_MARCH))
            viewport_process_raymarching_rays(&vs, scene->patches, scene->n_patches, steps, t0, t1 + 1, NULL);
    }
    renderColorImage(scene, &ve, &vs, out_rgba, r0, r1, NULL, NULL);
    if (t0_out) *t0_out = t0;
    if (t1_out) *t1_out = t1;
    viewport_free(&vs);
    viewport_free(&ve);
    return RTM_OK;
}

/* ---- staged (reference-seam) oracle API, host buffers ---- */
typedef struct rtmo_viewport {
    Viewport vp;
} rtmo_viewport;

int rtmo_viewport_create(int32_t W, int32_t H, int32_t face, const rtm_camera* cam, rtmo_viewport** out) {
    if (!cam || !out || W <= 0 || H <= 0 || (face != RTM_FACE_FRONT && face != RTM_FACE_BACK)) return RTM_ERR_INVALID;
    rtmo_viewport* v = (rtmo_viewport*)calloc(1, sizeof *v);
    viewport_init(&v->vp, W, H, face, cam);
    *out = v;
    return RTM_OK;
}

void rtmo_viewport_destroy(rtmo_viewport* v) {
    if (!v) return;
    viewport_free(&v->vp);
    free(v);
}

int rtmo_viewport_rasterize(rtmo_viewport* v, const rtm_scene* scene, int32_t flags) {
    int rc = validate_scene(scene);
    if (rc) return rc;
    return viewport_rasterize(&v->vp, scene, flags, 0, v->vp.H, NULL);
}

int rtmo_viewport_process_raytracing_rays(rtmo_viewport* v, const rtm_scene* scene) {
    int rc = validate_scene(scene);
    if (rc) return rc;
    viewport_process_raytracing_rays(&v->vp, scene, 0, v->vp.H, NULL);
    return RTM_OK;
}

int rtmo_viewport_process_raymarching_rays(rtmo_viewport* v, const rtm_patch* patches, int32_t n, int32_t steps) {
    if (n < 0 || (n > 0 && !patches) || steps < 0) return RTM_ERR_INVALID;
    viewport_process_raymarching_rays(&v->vp, patches, n, steps, 0, v->vp.H, NULL);
    return RTM_OK;
}

int rtmo_render_color_image(const rtm_scene* scene, const rtmo_viewport* v, const rtmo_viewport* vs, float* out) {
    int rc = validate_scene(scene);
    if (rc) return rc;
    if (!v || !vs || !out) return RTM_ERR_INVALID;
    if (vs->vp.camera.type != RTM_CAMERA_ORTHOGONAL) return RTM_ERR_UNSUPPORTED;
    renderColorImage(scene, &v->vp, &vs->vp, out, 0, v->vp.H, NULL, NULL);
    return RTM_OK;
}

int rtmo_viewport_read_zbuffer(const rtmo_viewport* v, double* out) {
    if (!v || !out) return RTM_ERR_INVALID;
    memcpy(out, v->vp.zBuffer, sizeof(double) * (size_t)(v->vp.W * v->vp.H));
    return RTM_OK;
}

/* ---- row f-1 helpers (calcRayPlane is pinned by the reference's own unit test) ---- */
/* calcRayPlane (main.rs:2398-2408); returns 1 and *t on Some */
int rtmo_calc_ray_plane(const double origin[3], const double dir[3], const double plane_n[3],
                        const double plane_center[3], double* t) {
    return calcRayPlane(v3(origin[0], origin[1], origin[2]), v3(dir[0], dir[1], dir[2]),
                        v3(plane_n[0], plane_n[1], plane_n[2]), v3(plane_center[0], plane_center[1], plane_center[2]), t);
}

/* iCappedCone (main.rs:2889-2959): out4 = (t, n.x, n.y, n.z) */
void rtmo_icapped_cone(const double ro[3], const double rd[3], const double pa[3], const double pb[3], double ra,
                       double rb, double out4[4]) {
    Vec3 n;
    double t = iCappedCone(v3(ro[0], ro[1], ro[2]), v3(rd[0], rd[1], rd[2]), v3(pa[0], pa[1], pa[2]),
                           v3(pb[0], pb[1], pb[2]), ra, rb, &n);
    out4[0] = t;
    out4[1] = n.x;
    out4[2] = n.y;
    out4[3] = n.z;
}


/* writeColorImage per-channel byte (main.rs:674-684), f32 arithmetic, libm powf */
static int64_t enc_byte(float c) {
    float v = rust_minf(rust_maxf(c, 0.0f), 1.0f); /* c.max(0.0).min(1.0): any NaN -> 0.0 */
    float gamma = 2.2f;
    v = powf(v, 1.0f / gamma);
    return rust_as_i64((double)(v * 255.0f));
}

/* Exhaustive scan of every f32 in [+0, 1.0]: is the byte map monotone, and its
 * thresholds T[k] = first v with byte >= k.  Returns the number of monotonicity
 * violations (0 expected). */
int64_t rtmo_encode_scan(float thresholds[256], int32_t nthreads) {
    const uint32_t top = 0x3F800000u; /* bits of 1.0f */
    enum { NCH = 64 };
    static uint32_t first[NCH][256];
    static int64_t lo_b[NCH], hi_b[NCH], viol[NCH];
    const uint32_t per = (top + NCH) / NCH;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads < 1 ? 1 : nthreads)
#endif
    for (int ch = 0; ch < NCH; ch++) {
        uint32_t b0 = (uint32_t)ch * per, b1 = b0 + per - 1;
        if (b1 > top) b1 = top;
        for (int k = 0; k < 256; k++) first[ch][k] = 0xFFFFFFFFu;
        viol[ch] = 0;
        int64_t prev = -1;
        for (uint32_t b = b0;; b++) {
            float v;
            memcpy(&v, &b, sizeof v);
            int64_t k = enc_byte(v);
            if (k < prev) viol[ch]++;
            if (b == b0) lo_b[ch] = k;
            if (k != prev)
                for (int64_t j = prev + 1; j <= k && j < 256; j++)
                    if (j >= 0 && first[ch][j] == 0xFFFFFFFFu) first[ch][j] = b;
            prev = k;
            if (b == b1) break;
        }
        hi_b[ch] = prev;
    }
    int64_t total = 0;
    for (int ch = 0; ch < NCH; ch++) {
        total += viol[ch];
        if (ch > 0 && lo_b[ch] < hi_b[ch - 1]) total++;
    }
    for (int k = 0; k < 256; k++) {
        uint32_t best = 0xFFFFFFFFu;
        for (int ch = 0; ch < NCH; ch++)
            if (first[ch][k] < best) best = first[ch][k];
        float t = INFINITY;
        if (best != 0xFFFFFFFFu) memcpy(&t, &best, sizeof t);
        thresholds[k] = k == 0 ? 0.0f : t;
    }
    return total;
}

/* writeColorImage (main.rs:660-704) text: "P3\n{W} {H}\n255\n", then per pixel
 * format!("{} {} {}  ", r, g, b), '\n' after each row.  Returns the length, or
 * -1 if it does not fit `cap`. */
int64_t rtmo_write_ppm(const float* rgba, int32_t W, int32_t H, char* out, int64_t cap) {
    int64_t n = 0;
    char buf[64];
    int l = snprintf(buf, sizeof buf, "P3\n%d %d\n255\n", W, H);
    if (n + l > cap) return -1;
    memcpy(out + n, buf, (size_t)l);
    n += l;
    for (int64_t iy = 0; iy < H; iy++) {
        for (int64_t ix = 0; ix < W; ix++) {
            const float* c = rgba + 4 * (iy * W + ix);
            l = snprintf(buf, sizeof buf, "%lld %lld %lld  ", (long long)enc_byte(c[0]), (long long)enc_byte(c[1]),
                         (long long)enc_byte(c[2]));
            if (n + l > cap) return -1;
            memcpy(out + n, buf, (size_t)l);
            n += l;
        }
        if (n + 1 > cap) return -1;
        out[n++] = '\n';
    }
    return n;
}

/* writeColorImage pixel encode (main.rs:674-684): clamp, f32 powf(1/2.2), (v*255) as i64 */
void rtmo_encode_rgb8(const float* rgba, int64_t n_pixels, int64_t* out_rgb) {
    for (int64_t i = 0; i < n_pixels; i++)
        for (int c = 0; c < 3; c++) out_rgb[3 * i + c] = enc_byte(rgba[4 * i + c]);
}
