// rtm_api.cpp — the C ABI (include/rtm.h) over the HIP kernels.
//
// Host responsibilities: validate the reference-shaped inputs, precompute the
// per-(camera, sphere) constants in the reference's f64 operation order
// (compiled with -ffp-contract=off), own device buffers / stream / events per
// context, and return status codes instead of panicking (main.rs:700, 1949).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <memory>
#include <string>
#include <thread>
#include <limits>
#include <vector>

#include "rtm_encode.h"
#include "rtm_internal.h"
#include "rtm_kernels.h"

#pragma clang fp contract(off)

using namespace rtm;

namespace rtm {
// What a frame needs beyond FrameArgs, in device memory: its ray-traced
// primitives (row f-1) and the eye's PERSPECTIVE sphere projections (row f-3).
struct FrameExtra {
    RtK rt;
    PerspK psp;
    SdfTabK sdf;
    bool has_rt = false, has_psp = false, has_sdf = false;
};
namespace internal {
struct PreparedFrame {  // rtm_internal.h
    FrameArgs a;
    FrameExtra x;
};
}  // namespace internal
}  // namespace rtm

namespace {

thread_local std::string g_last_error;

int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define HIP_TRY(expr)                                                                    \
    do {                                                                                 \
        hipError_t e_ = (expr);                                                          \
        if (e_ != hipSuccess) return fail(RTM_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
    int device = 0;
    ~DevBuf() {
        if (p) {
            int cur = 0;
            (void)hipGetDevice(&cur);
            (void)hipSetDevice(device);
            (void)hipFree(p);
            (void)hipSetDevice(cur);
        }
    }
    int ensure(size_t need, int dev) {
        if (need <= bytes) return RTM_OK;
        if (p) {
            (void)hipFree(p);
            p = nullptr;
            bytes = 0;
        }
        device = dev;
        if (hipMalloc(&p, need) != hipSuccess) return fail(RTM_ERR_OOM, "hipMalloc(%zu) failed", need);
        bytes = need;
        return RTM_OK;
    }
};

// ---- host-side precompute, reference op order ----
inline double dot3(const double a[3], const double b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }

// ((i as f64) / (n as f64)) * 2.0 - 1.0 (main.rs:306-307, 1903-1906)
inline double ndc(int32_t i, int32_t n) { return ((double)i / (double)n) * 2.0 - 1.0; }

// {i in [0,n) : |ndc(i) - c| <= R} is an interval because ndc(i) - c is
// monotone in i; found by binary search on exactly the values the kernel sees.
void pixel_range(double c, double R, int32_t n, int32_t* lo, int32_t* hi) {
    *lo = 1;
    *hi = 0;
    if (!(R >= 0.0) || !std::isfinite(c)) return;
    int32_t a = 0, b = n;  // first i with ndc(i) - c >= -R
    while (a < b) {
        int32_t m = a + (b - a) / 2;
        if (ndc(m, n) - c >= -R) b = m;
        else a = m + 1;
    }
    int32_t first = a;
    a = 0;
    b = n;  // first i with ndc(i) - c > R
    while (a < b) {
        int32_t m = a + (b - a) / 2;
        if (ndc(m, n) - c > R) b = m;
        else a = m + 1;
    }
    int32_t last = a - 1;
    if (first <= last) {
        *lo = first;
        *hi = last;
    }
}

// Viewport::rasterize ORTHOGONAL projection of one sphere (main.rs:449-470) and the
// axis normalisation of calcEllipseDistToCenter (main.rs:2849-2850), for a W x H viewport.
RasterSphereK project_sphere(const rtm_camera& c, const rtm_sphere& s, int32_t W, int32_t H) {
    RasterSphereK k{};
    double diff[3] = {s.pos[0] - c.pos[0], s.pos[1] - c.pos[1], s.pos[2] - c.pos[2]};
    k.z = dot3(c.dir, diff);    // calcDepthOfProjectedPoint: dot(dir, p - pos)
    k.cx = dot3(diff, c.side);  // Camera::project: dot(diff, side)
    k.cy = dot3(diff, c.up);
    k.r = s.r;
    const double m = std::sqrt(s.r * s.r + 0.0 * 0.0);  // Vec2::magnitude of (r, 0)
    const double inv = 1.0 / m;                          // Vec2::normalized: scale(1.0/m)
    k.n = s.r * inv;
    k.m = m;
    k.id = (int32_t)s.id;
    // A covered pixel has d < 1, hence |rel.x|, |rel.y| < m*(1 + 8 ulp); R adds a
    // 1e-9 relative margin.  Non-finite / zero m can never cover a pixel.
    k.ix0 = k.iy0 = 1;
    k.ix1 = k.iy1 = 0;
    if (std::isfinite(m) && m > 0.0 && std::isfinite(k.n)) {
        const double R = m * (1.0 + 1e-9);
        pixel_range(k.cx, R, W, &k.ix0, &k.ix1);
        pixel_range(k.cy, R, H, &k.iy0, &k.iy1);
        if (k.ix0 > k.ix1 || k.iy0 > k.iy1) {
            k.ix0 = k.iy0 = 1;
            k.ix1 = k.iy1 = 0;
        }
    }
    return k;
}

// ---- PERSPECTIVE sphere projection (row f-3) ----
// nalgebra 0.16 semantics (Cargo.toml nalgebra = "^0.16.12"): Matrix4::new is
// row-major; a fixed 4x4 product is one gemv per output column, y_i = v0*m_i0
// then y_i = v_j*m_ij + 1*y_i (axpy), zero terms included; Perspective3::new =
// identity, set_fovy, set_aspect, set_znear_and_zfar, m33 = 0, m32 = -1.
struct M44 {
    double m[4][4];
};

M44 m44_identity() {
    M44 r{};
    for (int i = 0; i < 4; ++i) r.m[i][i] = 1.0;
    return r;
}

void m44_gemv(const M44& a, const double x[4], double y[4]) {
    for (int i = 0; i < 4; ++i) y[i] = x[0] * a.m[i][0];
    for (int j = 1; j < 4; ++j)
        for (int i = 0; i < 4; ++i) y[i] = x[j] * a.m[i][j] + 1.0 * y[i];
}

M44 m44_mul(const M44& a, const M44& b) {
    M44 r{};
    for (int j = 0; j < 4; ++j) {
        const double x[4] = {b.m[0][j], b.m[1][j], b.m[2][j], b.m[3][j]};
        double y[4];
        m44_gemv(a, x, y);
        for (int i = 0; i < 4; ++i) r.m[i][j] = y[i];
    }
    return r;
}

// Viewport::rasterize, PERSPECTIVE branch (main.rs:473-524) for one sphere, and
// projectSphere (main.rs:2796-2837).  The aspect (512 as f64)/(512 as f64)
// (main.rs:496) generalises to W/H.  tan is the platform libm's (Rust f64::tan).
RasterSphereK project_sphere_persp(const rtm_camera& c, const rtm_sphere& s, int32_t W, int32_t H, PerspSphK& q) {
    RasterSphereK k{};
    const double diff[3] = {s.pos[0] - c.pos[0], s.pos[1] - c.pos[1], s.pos[2] - c.pos[2]};
    k.z = dot3(c.dir, diff);  // calcDepthOfProjectedPoint (main.rs:1962-1978)
    k.r = s.r;
    k.id = (int32_t)s.id;
    M44 rel{};  // relativeGlobalToCamera (main.rs:484-489)
    for (int i = 0; i < 3; ++i) {
        rel.m[0][i] = c.side[i];
        rel.m[1][i] = c.up[i];
        rel.m[2][i] = c.dir[i];
    }
    rel.m[3][3] = 1.0;
    const double d4[4] = {diff[0], diff[1], diff[2], 1.0};
    double local[4];
    m44_gemv(rel, d4, local);  // mul(&relativeGlobalToCamera, &(pos - camera.position)) (main.rs:492)
    const double fov = 3.14 / 2.0;
    M44 p = m44_identity();  // Perspective3::new(W/H, fov, 0.1, 1000.0).to_homogeneous() (main.rs:496-499)
    const double old_m22 = p.m[1][1];
    p.m[1][1] = 1.0 / std::tan(fov / 2.0);
    p.m[0][0] = p.m[0][0] * (p.m[1][1] / old_m22);
    p.m[0][0] = p.m[1][1] / ((double)W / (double)H);
    p.m[2][2] = (1000.0 + 0.1) / (0.1 - 1000.0);
    p.m[2][3] = 1000.0 * 0.1 * 2.0 / (0.1 - 1000.0);
    p.m[3][3] = 0.0;
    p.m[3][2] = -1.0;
    M44 refl = m44_identity();  // new_nonuniform_scaling(&Vector3::new(1.0, 1.0, -1.0)) (main.rs:503)
    refl.m[2][2] = -1.0;
    const M44 cam = m44_mul(p, refl);  // perspectiveMat * reflectionZMat (main.rs:506)
    // projectSphere(&Vec4(local, r), &cameraMat, fov)
    const double l4[4] = {local[0], local[1], local[2], 1.0};
    double o[4];
    m44_gemv(cam, l4, o);
    const double r2 = s.r * s.r;
    const double z2 = o[2] * o[2];
    const double l2 = o[0] * o[0] + o[1] * o[1] + o[2] * o[2];
    const double sa = fov * std::sqrt(-r2 * (r2 - l2) / ((l2 - z2) * (r2 - z2) * (r2 - z2)));
    const double sb = fov * std::sqrt(-r2 * (r2 - l2) / ((l2 - z2) * (r2 - z2) * (r2 - l2)));
    const double axa[2] = {o[0] * sa, o[1] * sa};
    const double axb[2] = {-o[1] * sb, o[0] * sb};
    const double sc = fov * o[2] / (z2 - r2);
    q.cx = o[0] * sc;
    q.cy = o[1] * sc;
    // calcEllipseDistToCenter's normalized() / magnitude() (main.rs:2849-2850, 2098-2109)
    q.mA = std::sqrt(axa[0] * axa[0] + axa[1] * axa[1]);
    q.mB = std::sqrt(axb[0] * axb[0] + axb[1] * axb[1]);
    const double iA = 1.0 / q.mA, iB = 1.0 / q.mB;
    q.nAx = axa[0] * iA;
    q.nAy = axa[1] * iA;
    q.nBx = axb[0] * iB;
    q.nBy = axb[1] * iB;
    k.cx = q.cx;
    k.cy = q.cy;
    k.n = 0.0;
    k.m = q.mA;
    // The axes are perpendicular, so d < 1 implies |rel| < max(mA, mB): each
    // coordinate is within R of the centre (1e-6 relative margin for the
    // rounding of the unit axes).  Non-finite or zero axes cover nothing.
    k.ix0 = k.iy0 = 1;
    k.ix1 = k.iy1 = 0;
    const bool ok = std::isfinite(q.mA) && std::isfinite(q.mB) && q.mA > 0.0 && q.mB > 0.0 && std::isfinite(q.cx) &&
                    std::isfinite(q.cy) && std::isfinite(q.nAx) && std::isfinite(q.nAy) && std::isfinite(q.nBx) &&
                    std::isfinite(q.nBy);
    if (ok) {
        const double R = std::max(q.mA, q.mB) * (1.0 + 1e-6);
        pixel_range(q.cx, R, W, &k.ix0, &k.ix1);
        pixel_range(q.cy, R, H, &k.iy0, &k.iy1);
        if (k.ix0 > k.ix1 || k.iy0 > k.iy1) {
            k.ix0 = k.iy0 = 1;
            k.ix1 = k.iy1 = 0;
        }
    }
    return k;
}

ShadeSphereK shade_sphere(const rtm_sphere& s) {
    ShadeSphereK k{};
    k.px = s.pos[0];
    k.py = s.pos[1];
    k.pz = s.pos[2];
    k.r = s.r;
    k.inv_r = 1.0 / s.r;
    k.cr = s.color[0];
    k.cg = s.color[1];
    k.cb = s.color[2];
    return k;
}

CamK cam_k(const rtm_camera& c) {
    CamK k{};
    for (int i = 0; i < 3; ++i) {
        k.pos[i] = c.pos[i];
        k.dir[i] = c.dir[i];
        k.up[i] = c.up[i];
        k.side[i] = c.side[i];
    }
    k.type = c.type;
    return k;
}

PatchK patch_k(const rtm_patch& p) {
    PatchK k{};
    k.a0 = p.a0;
    k.d0 = p.b0 - p.a0;  // linear(): diff = b - a (main.rs:2067)
    k.a1 = p.a1;
    k.d1 = p.b1 - p.a1;
    return k;
}

int validate_scene(const rtm_scene* scene) {
    if (!scene) return fail(RTM_ERR_INVALID, "scene is NULL");
    if (scene->n_spheres < 0 || scene->n_spheres > RTM_MAX_SPHERES)
        return fail(RTM_ERR_INVALID, "n_spheres=%d outside [0,%d]", scene->n_spheres, RTM_MAX_SPHERES);
    if (scene->n_patches < 0 || scene->n_patches > RTM_MAX_PATCHES)
        return fail(RTM_ERR_INVALID, "n_patches=%d outside [0,%d]", scene->n_patches, RTM_MAX_PATCHES);
    if (scene->n_spheres > 0 && !scene->spheres) return fail(RTM_ERR_INVALID, "spheres is NULL");
    if (scene->n_patches > 0 && !scene->patches) return fail(RTM_ERR_INVALID, "patches is NULL");
    for (int i = 0; i < scene->n_spheres; ++i) {
        int64_t id = scene->spheres[i].id;
        // the reference indexes scene.spherePrimitives[id] (main.rs:158, 748): out of range panics there
        if (id < 0 || id >= scene->n_spheres)
            return fail(RTM_ERR_INVALID, "sphere %d has id %lld outside [0,%d)", i, (long long)id, scene->n_spheres);
    }
    const int np = scene->n_circle_planes, nc = scene->n_capped_cylinders;
    if (np < 0 || np > RTM_MAX_CIRCLE_PLANES)
        return fail(RTM_ERR_INVALID, "n_circle_planes=%d outside [0,%d]", np, RTM_MAX_CIRCLE_PLANES);
    if (nc < 0 || nc > RTM_MAX_CAPPED_CYLINDERS)
        return fail(RTM_ERR_INVALID, "n_capped_cylinders=%d outside [0,%d]", nc, RTM_MAX_CAPPED_CYLINDERS);
    if (np > 0 && !scene->circle_planes) return fail(RTM_ERR_INVALID, "circle_planes is NULL");
    if (nc > 0 && !scene->capped_cylinders) return fail(RTM_ERR_INVALID, "capped_cylinders is NULL");
    // renderColorImage indexes circlePlanePrimitives[id] / cappedCylinderPrimitives[id] (main.rs:773, 791)
    for (int i = 0; i < np; ++i)
        if (scene->circle_planes[i].id < 0 || scene->circle_planes[i].id >= np)
            return fail(RTM_ERR_INVALID, "circle plane %d has id %lld outside [0,%d)", i,
                        (long long)scene->circle_planes[i].id, np);
    for (int i = 0; i < nc; ++i)
        if (scene->capped_cylinders[i].id < 0 || scene->capped_cylinders[i].id >= nc)
            return fail(RTM_ERR_INVALID, "capped cylinder %d has id %lld outside [0,%d)", i,
                        (long long)scene->capped_cylinders[i].id, nc);
    const int ns = scene->n_sdfs;
    if (ns < 0 || ns > RTM_MAX_SDFS) return fail(RTM_ERR_INVALID, "n_sdfs=%d outside [0,%d]", ns, RTM_MAX_SDFS);
    if (ns > 0 && !scene->sdfs) return fail(RTM_ERR_INVALID, "sdfs is NULL");
    for (int i = 0; i < ns; ++i) {
        if (scene->sdfs[i].id < 0 || scene->sdfs[i].id >= ns)
            return fail(RTM_ERR_INVALID, "sdf %d has id %lld outside [0,%d)", i, (long long)scene->sdfs[i].id, ns);
        if (scene->sdfs[i].max_steps < 0)
            return fail(RTM_ERR_INVALID, "sdf %d has max_steps=%d", i, scene->sdfs[i].max_steps);
    }
    return RTM_OK;
}


bool build_rt(const rtm_scene* scene, const rtm_camera* eye, RtK& k);
bool build_sdf(const rtm_scene* scene, SdfTabK& k);

void build_extra(const rtm_scene* scene, const rtm_camera* eye, int32_t W, int32_t H, FrameExtra& x) {
    x.has_rt = build_rt(scene, eye, x.rt);
    x.has_sdf = build_sdf(scene, x.sdf);
    std::memset(&x.psp, 0, sizeof x.psp);
    x.has_psp = eye->type != RTM_CAMERA_ORTHOGONAL && scene->n_spheres > 0;
    if (x.has_psp)
        for (int i = 0; i < scene->n_spheres; ++i) (void)project_sphere_persp(*eye, scene->spheres[i], W, H, x.psp.s[i]);
}

// The largest double s >= +0 with sqrt(s) <= r (sqrt correctly rounded, monotone), so
// that !(sqrt(s) > r) == !(s > T) for every s the radius test sees (s = q.q is +0,
// positive, +inf or NaN): r NaN -> NaN (both tests always pass), r < 0 -> -1 (both
// always fail for non-NaN s), r = +inf -> +inf; otherwise a search over the ordered
// bit patterns of [+0, +inf).
// The boundary is searched first next to r*r (sqrt(fl(r*r)) is within an ulp or
// so of r: a few steps), which the per-frame host build of a ray-traced frame pays
// per circle plane; any start gives the same boundary (the set {s : sqrt(s) <= r}
// is a prefix of the ordered bit patterns), and a start that needs more than 64
// steps falls back to the full bisection.
double sqrt_le_threshold(double r) {
    if (r != r) return r;
    if (r < 0.0) return -1.0;
    if (std::sqrt(INFINITY) <= r) return INFINITY;
    {
        double g = r * r;
        uint64_t b;
        if (!(g < INFINITY)) g = std::numeric_limits<double>::max();
        std::memcpy(&b, &g, sizeof b);
        auto ok = [r](uint64_t bits) {
            double v;
            std::memcpy(&v, &bits, sizeof v);
            return std::sqrt(v) <= r;
        };
        int n = 0;
        while (n < 64 && !ok(b)) --b, ++n;                                // b = +0 is always ok
        while (n < 64 && b + 1u < 0x7FF0000000000000ull && ok(b + 1u)) ++b, ++n;
        if (n < 64) {
            double t;
            std::memcpy(&t, &b, sizeof t);
            return t;
        }
    }
    uint64_t lo = 0u, hi = 0x7FF0000000000000ull;  // sqrt(+0) <= r (r >= +-0), sqrt(+inf) > r
    while (hi - lo > 1u) {
        const uint64_t mid = lo + (hi - lo) / 2u;
        double v;
        std::memcpy(&v, &mid, sizeof v);
        if (std::sqrt(v) <= r) lo = mid;
        else hi = mid;
    }
    double t;
    std::memcpy(&t, &lo, sizeof t);
    return t;
}

// Ray-traced primitives of a (validated) scene, with iCappedCone's
// ray-independent terms in the reference's operation order (main.rs:2906-2934).
// With a PERSPECTIVE `eye` every ray starts at eye->pos (main.rs:1922-1939), so
// the origin-only terms of calcRayPlane and iCappedCone are constants too
// (k.persp; the kernel's plane_hit_persp / icapped_persp): computed here with the
// kernel's operations in its order, hence the same bits.  Returns true when the
// scene has any primitive.
bool build_rt(const rtm_scene* scene, const rtm_camera* eye, RtK& k) {
    std::memset(&k, 0, sizeof k);
    k.n_pl = scene->n_circle_planes;
    k.n_cy = scene->n_capped_cylinders;
    k.persp = eye && eye->type == RTM_CAMERA_PERSPECTIVE;
    const double* ro = eye ? eye->pos : nullptr;
    for (int i = 0; i < k.n_pl; ++i) {
        const rtm_circle_plane& q = scene->circle_planes[i];
        PlaneK& p = k.pl[i];
        p.cx = q.pos[0];
        p.cy = q.pos[1];
        p.cz = q.pos[2];
        p.nx = q.n[0];
        p.ny = q.n[1];
        p.nz = q.n[2];
        p.radius = q.radius;
        p.r2max = sqrt_le_threshold(q.radius);
        p.cr = q.color[0];
        p.cg = q.color[1];
        p.cb = q.color[2];
        p.id = (int32_t)q.id;
        if (k.persp)  // calcRayPlane: dot(planeCenter - rayOrigin, planeN) (main.rs:2402)
            p.num = (p.cx - ro[0]) * p.nx + (p.cy - ro[1]) * p.ny + (p.cz - ro[2]) * p.nz;
    }
    for (int i = 0; i < k.n_cy; ++i) {
        const rtm_capped_cylinder& q = scene->capped_cylinders[i];
        CylK& c = k.cy[i];
        for (int j = 0; j < 3; ++j) {
            c.pa[j] = q.pa[j];
            c.pb[j] = q.pb[j];
            c.ba[j] = q.pb[j] - q.pa[j];
        }
        c.ra = q.ra;
        c.rb = q.rb;
        c.baba = c.ba[0] * c.ba[0] + c.ba[1] * c.ba[1] + c.ba[2] * c.ba[2];
        c.rr = q.rb - q.ra;
        c.hy = c.baba + c.rr * c.rr;
        c.isq = 1.0 / std::sqrt(c.baba);
        c.cr = q.color[0];
        c.cg = q.color[1];
        c.cb = q.color[2];
        c.id = (int32_t)q.id;
        if (k.persp) {  // iCappedCone's origin-only terms (main.rs:2907-2936), the kernel's order
            for (int j = 0; j < 3; ++j) {
                c.oa[j] = ro[j] - c.pa[j];
                c.ob[j] = ro[j] - c.pb[j];
            }
            c.oaba = c.oa[0] * c.ba[0] + c.oa[1] * c.ba[1] + c.oa[2] * c.ba[2];
            c.obba = c.ob[0] * c.ba[0] + c.ob[1] * c.ba[1] + c.ob[2] * c.ba[2];
            for (int j = 0; j < 3; ++j) c.oc[j] = c.oa[j] * c.rb - c.ob[j] * c.ra;
            c.ocba = c.oc[0] * c.ba[0] + c.oc[1] * c.ba[1] + c.oc[2] * c.ba[2];
            const double ococ = c.oc[0] * c.oc[0] + c.oc[1] * c.oc[1] + c.oc[2] * c.oc[2];
            c.bb = c.baba * c.baba;
            c.k0 = c.bb * ococ - c.hy * c.ocba * c.ocba;
        }
    }
    return k.n_pl + k.n_cy > 0;
}

// SDF primitives (row f-4) with udTriangleSingle's point-independent terms
// (entry.frag:318-321, 436), computed as oracle/rtm_oracle.c's sdf_geom does.
bool build_sdf(const rtm_scene* scene, SdfTabK& k) {
    std::memset(&k, 0, sizeof k);
    k.n = scene->n_sdfs;
    auto cross = [](const double x[3], const double y[3], double r[3]) {  // GLSL cross
        r[0] = x[1] * y[2] - y[1] * x[2];
        r[1] = x[2] * y[0] - y[2] * x[0];
        r[2] = x[0] * y[1] - y[0] * x[1];
    };
    auto dot = [](const double x[3], const double y[3]) { return x[0] * y[0] + x[1] * y[1] + x[2] * y[2]; };
    static const double o1[3] = {0.8, 0.8, 0.8}, o2[3] = {1.3, 0.8, 0.8}, o3[3] = {1.0, 0.7, 0.2};
    for (int i = 0; i < k.n; ++i) {
        const rtm_sdf& q = scene->sdfs[i];
        SdfK& g = k.s[i];
        for (int j = 0; j < 3; ++j) {
            g.box[j] = q.box_center[j];
            g.v1[j] = q.tri_anchor[j] + o1[j];
            g.v2[j] = q.tri_anchor[j] + o2[j];
            g.v3[j] = q.tri_anchor[j] + o3[j];
            g.ac[j] = q.aabb_center[j];
            g.ae[j] = q.aabb_extent[j];
        }
        for (int j = 0; j < 3; ++j) {
            g.e21[j] = g.v2[j] - g.v1[j];
            g.e32[j] = g.v3[j] - g.v2[j];
            g.e13[j] = g.v1[j] - g.v3[j];
        }
        cross(g.e21, g.e13, g.nor);
        cross(g.e21, g.nor, g.c1);
        cross(g.e32, g.nor, g.c2);
        cross(g.e13, g.nor, g.c3);
        g.d21 = dot(g.e21, g.e21);
        g.d32 = dot(g.e32, g.e32);
        g.d13 = dot(g.e13, g.e13);
        g.dnor = dot(g.nor, g.nor);
        g.cr = q.color[0];
        g.cg = q.color[1];
        g.cb = q.color[2];
        g.id = (int32_t)q.id;
        g.steps = q.max_steps;
    }
    return k.n > 0;
}

int validate_camera(const rtm_camera* c, const char* what) {
    if (!c) return fail(RTM_ERR_INVALID, "%s camera is NULL", what);
    if (c->type != RTM_CAMERA_ORTHOGONAL && c->type != RTM_CAMERA_PERSPECTIVE)
        return fail(RTM_ERR_INVALID, "%s camera type %d", what, c->type);
    return RTM_OK;
}

int validate_dims(int32_t w, int32_t h) {
    if (w <= 0 || h <= 0 || w > RTM_MAX_DIM || h > RTM_MAX_DIM)
        return fail(RTM_ERR_INVALID, "image size %dx%d outside [1,%d]", w, h, RTM_MAX_DIM);
    return RTM_OK;
}

// Everything build_frame can reject, without building anything (the group's up-front
// check of a whole call's frames: a full build per frame there cost the group path a
// second build of every frame before its first launch).
int validate_frame(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t W, int32_t H,
                   int32_t steps, int32_t flags) {
    int rc;
    if ((rc = validate_scene(scene)) || (rc = validate_camera(eye, "eye")) || (rc = validate_camera(shadow, "shadow")) ||
        (rc = validate_dims(W, H)))
        return rc;
    if (steps < 0) return fail(RTM_ERR_INVALID, "march_steps=%d < 0", steps);
    if (flags & ~(RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER | RTM_FLAG_FUSED_SHADOW))
        return fail(RTM_ERR_INVALID, "unknown flags 0x%x", flags);
    // Camera::project asserts ORTHO (main.rs:1949) for the shadow viewport and the
    // shadow lookup; the eye may be PERSPECTIVE (spheres via project_sphere_persp, row f-3).
    if (shadow->type != RTM_CAMERA_ORTHOGONAL)
        return fail(RTM_ERR_UNSUPPORTED, "frame path needs an ORTHOGONAL shadow camera");
    return RTM_OK;
}

int build_frame(FrameArgs& a, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t W,
                int32_t H, int32_t steps, int32_t flags) {
    int rc;
    if ((rc = validate_frame(scene, eye, shadow, W, H, steps, flags))) return rc;
    std::memset(&a, 0, sizeof a);
    ShadowPart& sh = a.sh;
    EyePart& ey = a.ey;
    PerspSphK unused;
    for (int i = 0; i < scene->n_spheres; ++i) {
        ey.sph[i] = eye->type == RTM_CAMERA_ORTHOGONAL ? project_sphere(*eye, scene->spheres[i], W, H)
                                                       : project_sphere_persp(*eye, scene->spheres[i], W, H, unused);
        sh.sph[i] = project_sphere(*shadow, scene->spheres[i], W, H);
        ey.shade[i] = shade_sphere(scene->spheres[i]);
    }
    for (int i = 0; i < scene->n_patches; ++i) sh.patch[i] = patch_k(scene->patches[i]);
    sh.cam = cam_k(*shadow);
    sh.W = W;  // the shadow map has the eye image's size
    sh.H = H;
    sh.n_spheres = scene->n_spheres;
    sh.n_patches = scene->n_patches;
    sh.steps = steps;
    sh.flags = flags;
    ey.eye = cam_k(*eye);
    ey.shadow = sh.cam;
    ey.W = W;
    ey.H = H;
    ey.Ws = W;
    ey.Hs = H;
    ey.n_spheres = scene->n_spheres;
    // union of the spheres' pixel ranges per viewport (empty: x0 > x1); a wave
    // outside it skips the per-sphere culls
    auto cull_union = [&](const RasterSphereK* sph, int32_t* x0, int32_t* x1, int32_t* y0, int32_t* y1) {
        *x0 = *y0 = 1;
        *x1 = *y1 = 0;
        for (int i = 0; i < scene->n_spheres; ++i) {
            const RasterSphereK& k = sph[i];
            if (k.ix0 > k.ix1 || k.iy0 > k.iy1) continue;  // covers nothing
            const bool first = *x0 > *x1;
            *x0 = first ? k.ix0 : std::min(*x0, k.ix0);
            *x1 = first ? k.ix1 : std::max(*x1, k.ix1);
            *y0 = first ? k.iy0 : std::min(*y0, k.iy0);
            *y1 = first ? k.iy1 : std::max(*y1, k.iy1);
        }
    };
    cull_union(ey.sph, &ey.cull_x0, &ey.cull_x1, &ey.cull_y0, &ey.cull_y1);
    cull_union(sh.sph, &sh.cull_x0, &sh.cull_x1, &sh.cull_y0, &sh.cull_y1);
    ey.flags = flags;
    ey.row_begin = 0;
    ey.row_end = H;
    return RTM_OK;
}

// writeColorImage's per-channel byte (main.rs:674-684), f32 arithmetic with the
// platform powf — the same libm call the Rust binary makes.
inline int64_t enc_byte(float v) {
    const float gamma = 2.2f;
    const float p = powf(v, 1.0f / gamma);
    return (int64_t)(p * 255.0f);
}

inline float f32_from_bits(uint32_t b) {
    float f;
    std::memcpy(&f, &b, sizeof f);
    return f;
}

// T[k] = smallest f32 in [0,1] with enc_byte >= k, by binary search over the
// ordered bit patterns of [+0, 1.0]; bucket[i] = number of thresholds <= the
// first value of bucket i (its byte), see rtm_encode.h.
const EncodeTable& encode_table() {
    static const EncodeTable tab = [] {
        EncodeTable t{};
        uint32_t tb[256];
        t.t[0] = 0.0f;
        tb[0] = 0u;
        for (int k = 1; k < 256; ++k) {
            uint32_t lo = 0u, hi = 0x3F800000u + 1u;  // [lo, hi)
            while (lo < hi) {
                const uint32_t mid = lo + (hi - lo) / 2u;
                if (enc_byte(f32_from_bits(mid)) >= k) hi = mid;
                else lo = mid + 1u;
            }
            tb[k] = lo;
            t.t[k] = lo <= 0x3F800000u ? f32_from_bits(lo) : INFINITY;
        }
        int k = 0;
        t.max_crossings = 0;
        for (int i = 0; i < ENC_BUCKETS; ++i) {
            const uint32_t first = (uint32_t)i << ENC_BUCKET_SHIFT;
            const uint32_t last = std::min(first + ((1u << ENC_BUCKET_SHIFT) - 1u), 0x3F800000u);
            while (k < 255 && tb[k + 1] <= first) ++k;
            t.bucket[i] = (uint8_t)k;
            int c = 0;
            while (k + c < 255 && tb[k + c + 1] <= last) ++c;
            t.max_crossings = std::max(t.max_crossings, c);
        }
        return t;
    }();
    return tab;
}

}  // namespace

struct TimingSlot {
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // shadow start/stop, eye (or pipe) start/stop
    bool shadow = false;
};

// Batched frame uploads of one lane: a ring of R slots, each a pinned host
// staging area and a device copy of a batch's BatchFrame table (+ the frames'
// ray-traced / perspective / SDF tables).  A slot's host side is refilled once
// its previous upload has completed (copied[j]), its device side once the
// kernels that read it have run (used[j]); the upload runs on its own stream, so
// batch i+1's table crosses PCIe while batch i renders.
// A batch's frame table reaches the device by a pull kernel on the lane's stream
// reading the pinned slot.  (An async copy, on a copy stream or on the lane's stream,
// went to a copy engine past a few tens of KB: 8 frames per launch at 3840x2160
// (32 KB) ran at 91 instead of 248 Gpix/s with kernels of the same duration,
// profiles/r02_ab_batch_pull.txt.)

struct BatchRing {
    static constexpr int R = 4;
    void* host[R] = {};
    void* host_dev[R] = {};  // the pinned host slot's device address (the pull kernel reads it)
    size_t host_bytes[R] = {};
    DevBuf dev[R];
    hipEvent_t copied[R] = {}, used[R] = {};
    int next = 0;
    DevBuf smaps;  // the batch's shadow maps, B x W x H f64
    DevBuf rtmask; // per-wave primitive masks of the batch's PERSPECTIVE eye passes (row f-1)
    // what the shared masks in rtmask were culled for (enqueue_batch's mask key), valid while
    // no unshared batch has written the buffer since
    std::vector<char> mask_key;
    const void* mask_buf = nullptr;
    int device = 0;
    ~BatchRing() {
        int cur = 0;
        (void)hipGetDevice(&cur);
        (void)hipSetDevice(device);
        for (int j = 0; j < R; ++j) {
            if (used[j]) (void)hipEventSynchronize(used[j]);
            if (host[j]) (void)hipHostFree(host[j]);
            if (copied[j]) (void)hipEventDestroy(copied[j]);
            if (used[j]) (void)hipEventDestroy(used[j]);
        }
        (void)hipSetDevice(cur);
    }
};

// An extra stream of a context with its own per-frame buffers: the frame
// sequence call spreads independent frames over lanes so one frame's kernels
// fill the ramp and tail of another's (see frame_lanes).
struct Lane {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;  // join: the context stream waits on it
    DevBuf smap, rtk, pspk, sdfk, rtmask;
    std::unique_ptr<BatchRing> batch;
};

struct rtm_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::vector<std::unique_ptr<Lane>> lanes;  // extra lanes 1..n (lane 0 is the context itself)
    hipEvent_t fork = nullptr;                 // lanes wait on the context stream's earlier work
    int32_t lanes_req = 0;                     // rtm_ctx_set_lanes (0 = auto)
    int32_t lanes_last = 0;                    // lanes of the last frame-sequence call
    int32_t batch_req = 0;                     // rtm_ctx_set_batch (0 = auto)
    int32_t batch_last = 1;                    // frames per launch of the last frame-sequence call
    int32_t eye_blocks_last = 0;               // the last eye launch ran 8 x 8-pixel blocks (rtm_ctx_last_eye_blocks)
    std::unique_ptr<BatchRing> batch;          // lane 0's batch uploads
    std::vector<TimingSlot> ring;  // per-render kernel events (capacity = ring.size())
    int64_t renders = 0;           // renders recorded into the ring
    int64_t calls = 0;             // renders enqueued (for the stride)
    int32_t stride = 1;
    bool have_shadow_pass = false;
    DevBuf smap;    // shadow map (coded or f64, ShadowPart::smap_fmt)
    const double* last_smap = nullptr;
    bool last_trivial = false;  // the last frame's shadow viewport was all +INF and not materialised
    ShadowPart last_sh{};  // the last shadow pass's arguments (smap_fmt: how last_smap is stored)
    DevBuf smap_dec;       // rtm_ctx_shadow_map's f64 view of a coded map
    DevBuf out;     // staging for rtm_render's host output
    DevBuf stats;
    int32_t smap_w = 0, smap_h = 0;
    DevBuf tabs;  // [t (steps) | nx (W) | ny (H)] f64, see Tables
    DevBuf enc_rgb, enc_rows, enc_text;  // writeColorImage scratch
    DevBuf enc_tab;                      // EncodeTable on the device (t | bucket)
    DevBuf rtk;                          // RtK of the frame being enqueued (row f-1)
    DevBuf pspk;                         // PerspK of the frame being enqueued (row f-3)
    DevBuf sdfk;                         // SdfTabK of the frame being enqueued (row f-4)
    DevBuf rtmask;                       // per-wave primitive masks of a PERSPECTIVE eye pass (row f-1)
    std::vector<rtm_viewport*> viewports;  // live viewports (orphaned when the context goes first)
    bool enc_tab_ready = false;
    uint64_t tab_key = 0;
    int64_t tab_nt = 0, tab_nz = 0, tab_nd = 0;
    int32_t tab_w = 0, tab_h = 0, tab_np = 0, tab_zmono = 0;
    double tab_z0 = 0.0;
    double tab_inv_sz = 0.0;
    double tab_sz = 0.0;
    int64_t tab_rec = -1;  // offset (doubles) of the coded tile's records, -1: none
    bool tab_hast = false, tab_sep = false;
};

struct rtm_viewport {
    rtm_ctx* ctx = nullptr;
    int32_t W = 0, H = 0, face = 0;
    rtm_camera cam{};
    DevBuf zbuf, gh, gz, gid;
    DevBuf gn;  // capped-cylinder / SDF hit normals (3 f64 per pixel), allocated by the first trace
    int32_t traced_pl = 0, traced_cy = 0, traced_sdf = 0;  // max primitive counts traced into the G-buffer
    int32_t raster_sp = 0;                 // ... and rasterized
};

namespace {

// Shared march depth sequence: an ORTHOGONAL camera with no x/y ray motion and
// side.z == up.z == 0 starts every texel at the same z (origin z =
// (pos.z + side.z*s) + up.z*u == pos.z bit for bit, or +0.0 when pos.z == +0.0;
// a -0.0 pos.z would make the sign of zero depend on s, u: not shared).
bool shared_z0(const rtm_camera* c, double* z0, double* sz) {
    if (!c || c->type != RTM_CAMERA_ORTHOGONAL) return false;
    if (!(c->dir[0] * 0.03 == 0.0 && c->dir[1] * 0.03 == 0.0)) return false;
    if (!(c->side[2] == 0.0 && c->up[2] == 0.0)) return false;
    if (c->pos[2] == 0.0 && std::signbit(c->pos[2])) return false;
    *z0 = c->pos[2] == 0.0 ? 0.0 : c->pos[2];
    *sz = c->dir[2] * 0.03;  // dir.scale(magnitudeOfStepsize) (main.rs:2233)
    return std::isfinite(*z0) && std::isfinite(*sz);
}

uint64_t bits_of(double v) {
    uint64_t b;
    std::memcpy(&b, &v, sizeof b);
    return b;
}

uint64_t fnv(uint64_t h, const void* p, size_t n) {
    const unsigned char* b = (const unsigned char*)p;
    for (size_t i = 0; i < n; ++i) h = (h ^ b[i]) * 1099511628211ull;
    return h;
}

// Separable axis-aligned march camera: the domain-mapped ray start
// ((o.x+1)*0.5, (o.y+1)*0.5) (main.rs:2187-2188) depends only on the column (x) and
// only on the row (y), bit for bit.  o.x = (pos.x + side.x*s) + up.x*u: with
// up.x == 0 the second term is +-0, which leaves a non-(-0) first term unchanged;
// o.y = (pos.y + side.y*s) + up.y*u: with side.y == 0 and pos.y != -0 the first
// term is the same for every column.
bool separable(const rtm_camera* c, int32_t W, std::vector<double>& colx, double* cy) {
    if (!(c->up[0] == 0.0 && c->side[1] == 0.0)) return false;
    if (c->pos[1] == 0.0 && std::signbit(c->pos[1])) return false;
    colx.resize((size_t)W);
    for (int32_t i = 0; i < W; ++i) {
        colx[(size_t)i] = c->pos[0] + c->side[0] * ndc(i, W);
        if (colx[(size_t)i] == 0.0 && std::signbit(colx[(size_t)i])) return false;
    }
    *cy = c->pos[1] == 0.0 ? 0.0 : c->pos[1];
    return true;
}

inline bool in01(double v) { return std::fabs(v - 0.5) <= 0.5; }

// An f32 index-guess term of the coded shadow tile, clamped to +-2^24 (NaN -> 0).
inline double guess_term(double v) { return v != v ? 0.0 : std::min(std::max(v, -16777216.0), 16777216.0); }

// Build (or reuse) the context's lookup tables for (steps, W, H, march camera, patches).
int ensure_tables(rtm_ctx* ctx, int32_t steps, int32_t W, int32_t H, const rtm_camera* march_cam,
                  const PatchK* patches, int32_t n_patches, Tables* out) {
    const bool with_t = steps <= RTM_T_TABLE_MAX;
    const int64_t nt = with_t ? steps : 0;
    uint64_t key = 1469598103934665603ull;
    key = fnv(key, &steps, sizeof steps);
    key = fnv(key, &W, sizeof W);
    key = fnv(key, &H, sizeof H);
    if (march_cam) key = fnv(key, march_cam, sizeof *march_cam);
    key = fnv(key, &n_patches, sizeof n_patches);
    if (n_patches > 0) key = fnv(key, patches, sizeof(PatchK) * (size_t)n_patches);
    if (!(ctx->tabs.p && ctx->tab_key == key)) {
        double z0 = 0.0, sz = 0.0;
        bool with_z = with_t && shared_z0(march_cam, &z0, &sz);
        std::vector<double> zt;
        if (with_z) {
            // 8 entries of padding past `steps`: the kernels prefetch one 8-step chunk ahead
            zt.resize((size_t)nt + 8);
            double z = z0;  // p.z after k advances: p = &p + &step (main.rs:2272)
            for (int64_t k = 0; k < nt + 8; ++k) {
                zt[(size_t)k] = z;
                z = z + sz;
                if (k < nt && !std::isfinite(zt[(size_t)k])) with_z = false;
            }
            if (nt == 0) with_z = false;
        }
        int32_t zmono = 0;  // the search march needs a monotone table (re-checked, not assumed)
        if (with_z) {
            bool up = true, down = true;
            for (int64_t k = 0; k + 1 < nt; ++k) {
                up = up && zt[(size_t)k + 1] >= zt[(size_t)k];
                down = down && zt[(size_t)k + 1] <= zt[(size_t)k];
            }
            zmono = up ? 1 : (down ? -1 : 0);
        }
        std::vector<double> colx;
        double cy = 0.0;
        const bool with_sep = with_z && n_patches > 0 && separable(march_cam, W, colx, &cy);
        const int64_t nz = with_z ? nt + 8 : 0;
        const int64_t nsep = with_sep ? (int64_t)H + 2 * (int64_t)n_patches * W : 0;
        const int64_t nd = nt + W + H + nz + nsep;
        const int64_t nok = with_sep ? (int64_t)W + H : 0;
        // the coded shadow tile's records (rtm_kernels.h ZRecK / ColRecK / RowRecK), 32-byte aligned
        // (and t strictly rising in k, so the coded tile may compare march codes for t)
        bool t_rising = true;
        {
            double tk = 0.0;  // the t table below: sequential sums of 0.03
            for (int64_t k = 0; k + 1 < nt && t_rising; ++k) {
                const double tn = tk + 0.03;
                t_rising = tn > tk;
                tk = tn;
            }
        }
        const bool with_rec = with_sep && zmono != 0 && nt >= 1 && t_rising;
        const int64_t rec_at = ((nd + (nok + 1) / 2) + 3) / 4 * 4;
        const int64_t h_pad = ((int64_t)H + 63) / 64 * 64;  // row records padded (RowRecK)
        const int64_t nrec = with_rec ? 4 * (nt + 1) + 4 * (int64_t)n_patches * W + 2 * h_pad : 0;
        std::vector<double> h((size_t)(with_rec ? rec_at + nrec : nd + (nok + 1) / 2));
        double t = 0.0;  // raymarchPatch: t = 0.0; ... t += magnitudeOfStepsize (main.rs:2237, 2273)
        for (int64_t k = 0; k < nt; ++k) {
            h[(size_t)k] = t;
            t = t + 0.03;
        }
        for (int32_t i = 0; i < W; ++i) h[(size_t)(nt + i)] = ndc(i, W);
        for (int32_t i = 0; i < H; ++i) h[(size_t)(nt + W + i)] = ndc(i, H);
        for (int64_t k = 0; k < nz; ++k) h[(size_t)(nt + W + H + k)] = zt[(size_t)k];
        if (with_sep) {
            double* py = &h[(size_t)(nt + W + H + nz)];
            double* d0 = py + H;
            double* dd = d0 + (int64_t)n_patches * W;
            int32_t* ok = (int32_t*)&h[(size_t)nd];
            for (int32_t j = 0; j < H; ++j) {
                const double oy = cy + march_cam->up[1] * ndc(j, H);
                py[j] = (oy + 1.0) * 0.5;  // raymarchPatchDomainM11 (main.rs:2188)
                ok[W + j] = in01(py[j]);
            }
            for (int32_t i = 0; i < W; ++i) {
                const double px = (colx[(size_t)i] + 1.0) * 0.5;  // main.rs:2187
                ok[i] = in01(px);
                for (int32_t k = 0; k < n_patches; ++k) {
                    const PatchK& p = patches[k];
                    const double a = p.a0 + p.d0 * px;  // linear(t.x, d00, d01): d00 + (d01-d00)*x
                    const double b = p.a1 + p.d1 * px;  // linear(t.x, d10, d11)
                    d0[(int64_t)k * W + i] = a;
                    dd[(int64_t)k * W + i] = b - a;  // linear(t.y, d0, d1): diff = d1 - d0
                }
            }
        }
        if (with_rec) {
            const double* py = &h[(size_t)(nt + W + H + nz)];
            const double* d0 = py + H;
            const double* dd = d0 + (int64_t)n_patches * W;
            const int32_t* ok = (const int32_t*)&h[(size_t)nd];
            ZRecK* zr = reinterpret_cast<ZRecK*>(&h[(size_t)rec_at]);
            ColRecK* cr = reinterpret_cast<ColRecK*>(zr + nt + 1);
            RowRecK* rr = reinterpret_cast<RowRecK*>(cr + (int64_t)n_patches * W);
            const double past = zmono > 0 ? INFINITY : -INFINITY;  // compares as "past the surface"
            for (int64_t k = 0; k <= nt; ++k) {
                zr[k].zprev = zt[(size_t)(k > 0 ? k - 1 : 0)];
                zr[k].z = k < nt ? zt[(size_t)k] : past;
                zr[k].t = k < nt ? h[(size_t)k] : INFINITY;
                zr[k].pad = 0.0;
            }
            const double inv_sz = 1.0 / sz;
            for (int32_t k = 0; k < n_patches; ++k)
                for (int32_t i = 0; i < W; ++i) {
                    ColRecK& c = cr[(int64_t)k * W + i];
                    c.d0 = d0[(int64_t)k * W + i];
                    c.dd = dd[(int64_t)k * W + i];
                    if (!ok[i]) {
                        // a column outside inRange01 never hits (main.rs:2249): a finite
                        // surface depth "before the start" for the table's direction makes
                        // the tile's check neither hit nor go slow there (see the kernel)
                        c.d0 = zmono > 0 ? -1.0e300 : 1.0e300;
                        c.dd = 0.0;
                    }
                    // bounded and finite, so the kernel's f32 -> int conversion of
                    // g0 + g1*pyf is always defined (|pyf| <= 4 below)
                    c.g0 = (float)guess_term((c.d0 - z0) * inv_sz);
                    c.g1 = (float)guess_term(c.dd * inv_sz);
                    c.ok = ok[i];
                    c.pad = 0;
                }
            for (int64_t j = 0; j < h_pad; ++j) {
                const int32_t jj = (int32_t)std::min<int64_t>(j, H - 1);  // padding: row H-1's terms, no march
                rr[j].py = py[jj];
                rr[j].pyf = py[jj] != py[jj] ? 0.0f : (float)std::min(std::max(py[jj], -4.0), 4.0);  // a guess term
                rr[j].ok = j < H ? ok[W + jj] : 0;
            }
        }
        HIP_TRY(hipStreamSynchronize(ctx->stream));  // earlier launches may still read the old tables
        for (auto& l : ctx->lanes) HIP_TRY(hipStreamSynchronize(l->stream));
        int rc = ctx->tabs.ensure(h.size() * sizeof(double), ctx->device);
        if (rc) return rc;
        HIP_TRY(hipMemcpy(ctx->tabs.p, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice));
        ctx->tab_key = key;
        ctx->tab_nt = nt;
        ctx->tab_hast = with_t;
        ctx->tab_nz = nz;
        ctx->tab_sep = with_sep;
        ctx->tab_nd = nd;
        ctx->tab_w = W;
        ctx->tab_h = H;
        ctx->tab_np = n_patches;
        ctx->tab_zmono = zmono;
        ctx->tab_z0 = nz ? zt[0] : 0.0;
        ctx->tab_rec = with_rec ? rec_at : -1;
        ctx->tab_inv_sz = nz ? 1.0 / sz : 0.0;
        ctx->tab_sz = nz ? sz : 0.0;
    }
    const double* base = (const double*)ctx->tabs.p;
    const int64_t nt2 = ctx->tab_nt, nz2 = ctx->tab_nz;
    out->t = ctx->tab_hast ? base : nullptr;
    out->nx = base + nt2;
    out->ny = base + nt2 + W;
    out->z = nz2 ? base + nt2 + W + H : nullptr;
    out->zmono = nz2 ? ctx->tab_zmono : 0;
    out->z0 = nz2 ? ctx->tab_z0 : 0.0;
    out->inv_sz = nz2 ? ctx->tab_inv_sz : 0.0;
    out->sz = nz2 ? ctx->tab_sz : 0.0;
    if (ctx->tab_sep) {
        out->py = base + nt2 + W + H + nz2;
        out->d0 = out->py + H;
        out->dd = out->d0 + (int64_t)ctx->tab_np * W;
        out->ok = (const int32_t*)(base + ctx->tab_nd);
    } else {
        out->py = out->d0 = out->dd = nullptr;
        out->ok = nullptr;
    }
    out->row_recs = ctx->tab_rec >= 0 ? (int32_t)(((int64_t)H + 63) / 64 * 64) : 0;
    if (ctx->tab_rec >= 0) {
        out->zrec = reinterpret_cast<const ZRecK*>(base + ctx->tab_rec);
        out->col = reinterpret_cast<const ColRecK*>(out->zrec + nt2 + 1);
        out->row = reinterpret_cast<const RowRecK*>(out->col + (int64_t)ctx->tab_np * W);
    } else {
        out->zrec = nullptr;
        out->col = nullptr;
        out->row = nullptr;
    }
    return RTM_OK;
}

struct DeviceGuard {
    int prev = 0;
    explicit DeviceGuard(int dev) {
        (void)hipGetDevice(&prev);
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = 0;
        (void)hipGetDevice(&cur);
        if (cur != prev) (void)hipSetDevice(prev);
    }
};

rtm_camera to_camera(const CamK& k) {
    rtm_camera c{};
    c.type = k.type;
    for (int i = 0; i < 3; ++i) {
        c.pos[i] = k.pos[i];
        c.dir[i] = k.dir[i];
        c.up[i] = k.up[i];
        c.side[i] = k.side[i];
    }
    return c;
}

int frame_tables(rtm_ctx* ctx, FrameArgs& a) {
    rtm_camera sc = to_camera(a.sh.cam);
    int rc = ensure_tables(ctx, a.sh.steps, a.sh.W, a.sh.H, &sc, a.sh.patch, a.sh.n_patches, &a.sh.tab);
    if (rc) return rc;
    a.ey.nx = a.sh.tab.nx;  // eye and shadow viewports share dims
    a.ey.ny = a.sh.tab.ny;
    return RTM_OK;
}

TimingSlot* next_slot(rtm_ctx* ctx) {
    const bool timed = !ctx->ring.empty() && (ctx->calls++ % ctx->stride) == 0;
    return timed ? &ctx->ring[(size_t)(ctx->renders % (int64_t)ctx->ring.size())] : nullptr;
}

int enc_tab_dev(rtm_ctx* ctx, const void** out);

int32_t format_bytes(int32_t fmt) {
    return fmt == RTM_FORMAT_RGBA32F ? 16 : fmt == RTM_FORMAT_RGBA8 ? 4 : fmt == RTM_FORMAT_RGB8 ? 3 : 0;
}

int validate_format(int32_t fmt, const void* out) {
    if (!format_bytes(fmt)) return fail(RTM_ERR_INVALID, "unknown output format %d", fmt);
    if (fmt == RTM_FORMAT_RGBA32F && ((uintptr_t)out & 15))
        return fail(RTM_ERR_INVALID, "RGBA32F output must be 16-byte aligned");
    return RTM_OK;
}

// The background pixel (0.0, 0.2, 0.2) (main.rs:718-720) through writeColorImage's
// encode (main.rs:674-684), R | G<<8 | B<<16: the eye epilogue stores it without a lookup.
uint32_t background_bytes() {
    static const uint32_t v = (uint32_t)enc_byte(0.0f) | ((uint32_t)enc_byte(0.2f) << 8) |
                              ((uint32_t)enc_byte(0.2f) << 16);
    return v;
}

// The eye pass's output format: the encode table and background for RGBA8/RGB8,
// and whether RGB8 rows start 4-byte aligned (W % 4 == 0, aligned base: dword stores).
int format_tabs(rtm_ctx* ctx, int32_t fmt, int32_t W, const void* out, DevTabs& t) {
    t.fmt = fmt;
    t.enc = nullptr;
    t.bg = 0u;
    if (fmt == RTM_FORMAT_RGBA32F) return RTM_OK;
    int rc = enc_tab_dev(ctx, &t.enc);
    if (rc) return rc;
    t.bg = background_bytes();
    if (fmt == RTM_FORMAT_RGB8 && W % 4 == 0 && ((uintptr_t)out & 3) == 0) t.fmt |= FMT_RGB8_DWORDS;
    return RTM_OK;
}

// The frame's ray-traced primitives into the lane's rtk (stream-ordered; the
// lane's previous frame has consumed the old contents by the time the upload runs).
int upload_rt(rtm_ctx* ctx, DevBuf& buf, hipStream_t s, const RtK& rt, const RtK** dev) {
    int rc = buf.ensure(sizeof(RtK), ctx->device);
    if (rc) return rc;
    if ((rc = launch_upload(&rt, sizeof rt, buf.p, s))) return fail(rc, "rt upload launch failed");
    *dev = (const RtK*)buf.p;
    return RTM_OK;
}

int upload_persp(rtm_ctx* ctx, DevBuf& buf, hipStream_t s, const PerspK& k, const PerspK** dev) {
    int rc = buf.ensure(sizeof(PerspK), ctx->device);
    if (rc) return rc;
    if ((rc = launch_upload(&k, sizeof k, buf.p, s))) return fail(rc, "upload launch failed");
    *dev = (const PerspK*)buf.p;
    return RTM_OK;
}

int upload_sdf(rtm_ctx* ctx, DevBuf& buf, hipStream_t s, const SdfTabK& k, const SdfTabK** dev) {
    int rc = buf.ensure(sizeof(SdfTabK), ctx->device);
    if (rc) return rc;
    if ((rc = launch_upload(&k, sizeof k, buf.p, s))) return fail(rc, "sdf upload launch failed");
    *dev = (const SdfTabK*)buf.p;
    return RTM_OK;
}

// A frame with RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER (main()'s own scene,
// main.rs:910-1046) has an all-+INF shadow viewport: it skips the shadow pass and its
// eye pass takes the fused path, whose on-demand texel is +INF at once -- the same
// bits, one kernel instead of two.  rtm_ctx_shadow_map then materialises the +INF
// map on request.
bool trivial_shadow(int32_t flags) {
    const int32_t both = RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER;
    return (flags & both) == both && !(flags & RTM_FLAG_FUSED_SHADOW);
}

void note_trivial(rtm_ctx* ctx, const ShadowPart& sh) {
    ctx->have_shadow_pass = true;
    ctx->last_trivial = true;
    ctx->last_smap = nullptr;
    ctx->last_sh = sh;
    ctx->smap_w = sh.W;
    ctx->smap_h = sh.H;
}

// lane 0: the context's own stream and buffers; lane k > 0: ctx->lanes[k-1]
int enqueue_frame(rtm_ctx* ctx, FrameArgs& a, const FrameExtra* x, void* out_dev, StatsK* stats, int lane = 0,
                  int32_t fmt = RTM_FORMAT_RGBA32F) {
    int rc;
    if ((rc = frame_tables(ctx, a))) return rc;
    Lane* l = lane > 0 ? ctx->lanes[(size_t)lane - 1].get() : nullptr;
    hipStream_t s = l ? l->stream : ctx->stream;
    DevTabs tabs{};
    if ((rc = format_tabs(ctx, fmt, a.ey.W, out_dev, tabs))) return rc;
    if (x && x->has_rt && (rc = upload_rt(ctx, l ? l->rtk : ctx->rtk, s, x->rt, &tabs.rt))) return rc;
    if (x && x->has_psp && (rc = upload_persp(ctx, l ? l->pspk : ctx->pspk, s, x->psp, &tabs.psp))) return rc;
    if (x && x->has_sdf && (rc = upload_sdf(ctx, l ? l->sdfk : ctx->sdfk, s, x->sdf, &tabs.sdf))) return rc;
    if (x && x->has_rt && x->rt.persp && !stats) {
        // RT 3 (the host's origin-only primitive constants); from 1 Mpixel on, the
        // per-wave primitive masks come from a separate one-thread-per-wave kernel
        // (config 6 eye pass 160 -> 90 us); below, its launch costs more than it saves
        tabs.rt_persp = 1;
    }
    if (x && x->has_rt && x->rt.persp && !stats && (int64_t)a.ey.W * (a.ey.row_end - a.ey.row_begin) >= (1 << 20)) {
        DevBuf& mb = l ? l->rtmask : ctx->rtmask;
        const size_t words = (size_t)((a.ey.W + 63) / 64) * (size_t)(a.ey.row_end - a.ey.row_begin);
        if ((rc = mb.ensure(words * sizeof(uint32_t), ctx->device))) return rc;
        tabs.rtmask = (uint32_t*)mb.p;
        tabs.rtmask_words = (int32_t)words;
    }
    const bool trivial = !stats && trivial_shadow(a.ey.flags);
    if (trivial) a.ey.flags |= RTM_FLAG_FUSED_SHADOW;
    const bool fused = (a.ey.flags & RTM_FLAG_FUSED_SHADOW) != 0;
    double* smap = nullptr;
    TimingSlot* slot = next_slot(ctx);
    if (!fused) {
        // the map's storage: coded (1-2 B per texel) unless counting (f64)
        a.sh.smap_fmt = stats ? SMAP_F64 : shadow_map_format(a.sh);
        a.sh.smap_bw = (int16_t)((a.sh.W + 127) / 128);
        a.sh.smap_spans = (int16_t)(stats ? 0 : shadow_map_spans(a.sh));
        DevBuf& sb = l ? l->smap : ctx->smap;
        if ((rc = sb.ensure((size_t)smap_bytes(a.sh.smap_fmt, a.sh.W, a.sh.H, a.sh.smap_spans), ctx->device)))
            return rc;
        smap = (double*)sb.p;
        ctx->smap_w = a.sh.W;
        ctx->smap_h = a.sh.H;
        if (slot) HIP_TRY(hipEventRecord(slot->ev[0], s));
        if ((rc = launch_shadow_pass(a, smap, s, stats))) return fail(rc, "shadow pass launch failed");
        if (slot) HIP_TRY(hipEventRecord(slot->ev[1], s));
        ctx->have_shadow_pass = true;
        ctx->last_trivial = false;
        ctx->last_smap = smap;
        ctx->last_sh = a.sh;
    } else if (trivial) {
        note_trivial(ctx, a.sh);
    } else {
        ctx->have_shadow_pass = false;
    }
    if (slot) HIP_TRY(hipEventRecord(slot->ev[2], s));
    if ((rc = launch_eye_pass(a, smap, out_dev, s, stats, tabs))) return fail(rc, "eye pass launch failed");
    ctx->eye_blocks_last = 0;  // (single frames render 64 x 1 rows)
    if (slot) {
        HIP_TRY(hipEventRecord(slot->ev[3], s));
        slot->shadow = !fused;
        ctx->renders++;
    }
    return RTM_OK;
}

// How many lanes a frame sequence spreads over.  Frames are independent (own
// scene, own shadow map, own output), so frame i can run beside frame i+1: at
// 3840x2160 one frame's two kernels leave the chip part-empty in their ramp and
// tail (the shadow pass is latency-bound): with the coded shadow map, 2 lanes take
// config 3 from 40.1 to 33.3 us per frame (3 lanes 33.9), config 2 from 13.7 to
// 9.5 (3 lanes 10.7) and 7680x4320 from 134 to 128 (with the 8-byte map a second
// lane only added cache pressure there: 133 -> 157 us) (profiles/r02_ab_lanes.txt);
// at 512x512 with 64 frames per launch 60 -> 80 Gpix/s (one frame per launch,
// round 1, lanes had lost there: the host's launch rate was the limit).  RTM_LANES=n
// overrides.
// Frame i goes to lane (n-1-i) % L, so the last frame runs on lane 0 and the
// context's shadow map holds its shadow pass, as on one lane.  Lanes stay at 1
// when two frames of different lanes write overlapping output.
int frame_lanes(int32_t req, int32_t n, int32_t W, int32_t H, float* const* out, int32_t B = 1) {
    static const int env = [] {
        const char* e = getenv("RTM_LANES");
        return e ? atoi(e) : 0;
    }();
    // auto: 4 lanes below 16 Mpixel, 3 from 16 Mpixel up.  With the batch tables pulled
    // by the lanes (r02_v10), more lanes pay: 3840x2160 263 -> 276 Gpix/s at 4 (274-276
    // at 3, 268-273 at 6), 1920x1080 259 -> 267 (3 and 4), 512x512 119 -> 141,
    // 7680x4320 best at 3 (profiles/r02_ab_lanes_v12.txt)
    int L = req > 0 ? req : env > 0 ? env : ((int64_t)W * H >= (16LL << 20) ? 3 : 4);
    const int32_t nb = (n + B - 1) / B;  // batches of B frames; batch b runs on lane (nb-1-b) % L
    if (L > 8) L = 8;
    if (L > nb) L = nb;
    if (L <= 1) return 1;
    const uintptr_t bytes = (uintptr_t)W * (uintptr_t)H * 4u * sizeof(float);
    std::vector<std::pair<uintptr_t, int>> r((size_t)n);
    for (int32_t i = 0; i < n; ++i) r[(size_t)i] = {(uintptr_t)out[i], (nb - 1 - i / B) % L};
    std::sort(r.begin(), r.end());
    // equal-length ranges: any two overlapping ranges are joined by a chain of
    // overlapping sorted neighbours, so checking neighbours checks every pair
    for (size_t i = 1; i < r.size(); ++i)
        if (r[i].first < r[i - 1].first + bytes && r[i].second != r[i - 1].second) return 1;
    return L;
}

int ensure_lanes(rtm_ctx* ctx, int L) {
    if (!ctx->fork) HIP_TRY(hipEventCreateWithFlags(&ctx->fork, hipEventDisableTiming));
    while ((int)ctx->lanes.size() < L - 1) {
        std::unique_ptr<Lane> l(new Lane);
        HIP_TRY(hipStreamCreateWithFlags(&l->stream, hipStreamNonBlocking));
        if (hipEventCreateWithFlags(&l->done, hipEventDisableTiming) != hipSuccess) {
            (void)hipStreamDestroy(l->stream);
            return fail(RTM_ERR_HIP, "hipEventCreateWithFlags failed");
        }
        ctx->lanes.push_back(std::move(l));
    }
    return RTM_OK;
}

// Frames per launch of a frame sequence (profiles/r02_ab_batch.txt,
// r02_ab_batch_pull.txt).  One frame per launch leaves small frames bound by the
// host's per-frame launches (512x512: 12 Gpix/s at one frame per launch, 43 at 16;
// 1920x1080: 123 at 1, 181 at 4, tools/probes/batch_probe.py), and a big frame's two
// kernels pay a ramp and a tail each (3840x2160 at 4 frames: each frame's shadow pass
// 13.4 instead of 16.2 us, its eye pass 21.7 instead of 25.1).  Until r02_v10 the rule
// was 8 Mpixel worth from 1 to 4 Mpixel and 32 Mpixel worth from 4 to 16: bigger
// tables went through a copy engine.  rtm_ctx_set_batch overrides (1 = one frame per
// launch).
int frame_batch(int32_t req, int32_t W, int32_t H) {
    const int64_t px = (int64_t)W * H;
    // 64 Mpixel worth of frames, at most 64 below 1 Mpixel (512x512: 64 frames per
    // launch) and 32 above (1920x1080: 32, 3840x2160: 8, 7680x4320: 2; the cap was 16
    // until r03: 1920x1080 298 -> 304-305 Gpix/s at 32, profiles/r03_ab_batch_split.txt).  With the
    // batch table pulled by the lane's stream (r02_v10) bigger batches pay: 3840x2160
    // 250 -> 262 Gpix/s at 8 frames, 1920x1080 218 -> 248 at 16; with the async copy
    // the larger table went to a copy engine and 8 frames ran at 91-150 Gpix/s
    // (profiles/r02_ab_batch_pull.txt).
    const int64_t target = 64LL << 20;
    const int64_t cap = px < (1LL << 20) ? 64 : 32;
    int B = req > 0 ? req : (int)std::max<int64_t>(1, std::min<int64_t>(cap, target / px));
    return std::max(1, std::min(B, 64));
}

// Enqueue frames [0, n) of `fa` (same tables, flags and sizes) as ONE batched
// launch per pass on `lane`; a frame's output is outs[k] (RGBA f32).
// alone: no other lane of the call runs beside this one (the shadow pass's split launch
// then runs as one launch, launch_shadow_batch).
int enqueue_batch(rtm_ctx* ctx, int lane, FrameArgs* fa, const FrameExtra* const* exs, void* const* outs, int n,
                  int32_t fmt = RTM_FORMAT_RGBA32F, bool alone = false) {
    int rc;
    if ((rc = frame_tables(ctx, fa[0]))) return rc;
    for (int k = 1; k < n; ++k) {
        fa[k].sh.tab = fa[0].sh.tab;
        fa[k].ey.nx = fa[0].ey.nx;
        fa[k].ey.ny = fa[0].ey.ny;
    }
    Lane* l = lane > 0 ? ctx->lanes[(size_t)lane - 1].get() : nullptr;
    hipStream_t s = l ? l->stream : ctx->stream;
    std::unique_ptr<BatchRing>& brp = l ? l->batch : ctx->batch;
    if (!brp) {
        std::unique_ptr<BatchRing> b(new BatchRing);
        b->device = ctx->device;
        for (int j = 0; j < BatchRing::R; ++j) {
            HIP_TRY(hipEventCreateWithFlags(&b->copied[j], hipEventDisableTiming));
            HIP_TRY(hipEventCreateWithFlags(&b->used[j], hipEventDisableTiming));
        }
        brp = std::move(b);
    }
    BatchRing& br = *brp;
    const bool trivial = trivial_shadow(fa[0].ey.flags);  // (a batch shares its flags)
    if (trivial)
        for (int k = 0; k < n; ++k) fa[k].ey.flags |= RTM_FLAG_FUSED_SHADOW;
    const bool fused = (fa[0].ey.flags & RTM_FLAG_FUSED_SHADOW) != 0;
    // One storage for the whole launch (the batched shadow kernel is instantiated per
    // storage), so it must hold every frame's codes: steps + the most spheres of any
    // frame (frames of a batch may differ in sphere count; a byte map chosen for
    // frame 0 alone would truncate a later frame's sphere codes).
    ShadowPart widest = fa[0].sh;
    for (int k = 1; k < n; ++k) widest.n_spheres = std::max(widest.n_spheres, fa[k].sh.n_spheres);
    const int32_t sfmt = fused ? SMAP_F64 : shadow_map_format(widest);
    // (the batch's shadow launch is frame 0's kernel: its span rule holds for every frame)
    fa[0].sh.smap_fmt = sfmt;
    const int32_t spans = fused ? 0 : shadow_map_spans(fa[0].sh);
    for (int k = 0; k < n; ++k) {
        fa[k].sh.smap_fmt = sfmt;
        fa[k].sh.smap_bw = (int16_t)((fa[k].sh.W + 127) / 128);
        fa[k].sh.smap_spans = (int16_t)spans;
    }
    const size_t map_bytes = ((size_t)smap_bytes(sfmt, fa[0].sh.W, fa[0].sh.H, spans) + 255) & ~(size_t)255;
    if (!fused && (rc = br.smaps.ensure(map_bytes * (size_t)n, ctx->device))) return rc;
    // layout of the upload: the BatchFrame table, then each frame's device tables
    auto up = [](size_t v) { return (v + 255) & ~(size_t)255; };
    size_t off = up(sizeof(BatchFrame) * (size_t)n);
    std::vector<size_t> o_rt((size_t)n, 0), o_psp((size_t)n, 0), o_sdf((size_t)n, 0);
    // a table equal to the previous frame's (a static scene, or primitives that did not
    // move) is uploaded once and shared: same bytes, so the same bits
    std::vector<char> fresh_rt((size_t)n, 1), fresh_psp((size_t)n, 1), fresh_sdf((size_t)n, 1);
    for (int k = 0; k < n; ++k) {
        const FrameExtra* pv = k > 0 ? exs[k - 1] : nullptr;
        if (exs[k]->has_rt) {
            if (pv && pv->has_rt && std::memcmp(&pv->rt, &exs[k]->rt, sizeof(RtK)) == 0) {
                o_rt[(size_t)k] = o_rt[(size_t)k - 1];
                fresh_rt[(size_t)k] = 0;
            } else { o_rt[(size_t)k] = off; off = up(off + sizeof(RtK)); }
        }
        if (exs[k]->has_psp) {
            if (pv && pv->has_psp && std::memcmp(&pv->psp, &exs[k]->psp, sizeof(PerspK)) == 0) {
                o_psp[(size_t)k] = o_psp[(size_t)k - 1];
                fresh_psp[(size_t)k] = 0;
            } else { o_psp[(size_t)k] = off; off = up(off + sizeof(PerspK)); }
        }
        if (exs[k]->has_sdf) {
            if (pv && pv->has_sdf && std::memcmp(&pv->sdf, &exs[k]->sdf, sizeof(SdfTabK)) == 0) {
                o_sdf[(size_t)k] = o_sdf[(size_t)k - 1];
                fresh_sdf[(size_t)k] = 0;
            } else { o_sdf[(size_t)k] = off; off = up(off + sizeof(SdfTabK)); }
        }
    }
    const size_t bytes = off;
    const int j = br.next;
    br.next = (br.next + 1) % BatchRing::R;
    HIP_TRY(hipEventSynchronize(br.copied[j]));  // the slot's previous upload has left the host buffer
    if (br.host_bytes[j] < bytes) {
        if (br.host[j]) HIP_TRY(hipHostFree(br.host[j]));
        br.host[j] = nullptr;
        br.host_bytes[j] = 0;
        // (coarse-grained pinned memory: coherent at the pull kernel's dispatch, after the
        // host filled the slot; copied[j] keeps the host from refilling it earlier.  A
        // fine-grained ring measured the same, profiles/r04_ab_eye_prologue.txt)
        HIP_TRY(hipHostMalloc(&br.host[j], bytes, hipHostMallocDefault));
        br.host_bytes[j] = bytes;
        HIP_TRY(hipHostGetDevicePointer(&br.host_dev[j], br.host[j], 0));
    }
    if (br.dev[j].bytes < bytes) {
        HIP_TRY(hipEventSynchronize(br.used[j]));  // no kernel still reads the old device slot
        if ((rc = br.dev[j].ensure(bytes, ctx->device))) return rc;
    }
    char* hb = (char*)br.host[j];
    char* db = (char*)br.dev[j].p;
    DevTabs t0{};
    for (int k = 0; k < n; ++k) {
        BatchFrame& bf = *(BatchFrame*)(hb + sizeof(BatchFrame) * (size_t)k);
        bf.a = fa[k];
        bf.smap = fused ? nullptr : (double*)((char*)br.smaps.p + map_bytes * (size_t)k);
        bf.out = outs[k];
        if ((rc = format_tabs(ctx, fmt, fa[k].ey.W, outs[k], bf.tabs))) return rc;
        bf.tabs.rt = nullptr;
        bf.tabs.psp = nullptr;
        bf.tabs.sdf = nullptr;
        bf.tabs.rtmask = nullptr;
        bf.tabs.rtmask_words = 0;
        bf.tabs.rt_persp = 0;
        if (exs[k]->has_rt) {
            if (fresh_rt[(size_t)k]) std::memcpy(hb + o_rt[(size_t)k], &exs[k]->rt, sizeof(RtK));
            bf.tabs.rt = (const RtK*)(db + o_rt[(size_t)k]);
            bf.tabs.rt_persp = exs[k]->rt.persp;
            t0.rt = bf.tabs.rt;
            t0.rt_persp = exs[k]->rt.persp;
        }
        if (exs[k]->has_psp) {
            if (fresh_psp[(size_t)k]) std::memcpy(hb + o_psp[(size_t)k], &exs[k]->psp, sizeof(PerspK));
            bf.tabs.psp = (const PerspK*)(db + o_psp[(size_t)k]);
            t0.psp = bf.tabs.psp;
        }
        if (exs[k]->has_sdf) {
            if (fresh_sdf[(size_t)k]) std::memcpy(hb + o_sdf[(size_t)k], &exs[k]->sdf, sizeof(SdfTabK));
            bf.tabs.sdf = (const SdfTabK*)(db + o_sdf[(size_t)k]);
            t0.sdf = bf.tabs.sdf;
        }
    }
    // a frame without ray-traced primitives in a RT 3 batch: every frame shares the eye camera
    t0.rt_persp = t0.rt ? t0.rt_persp : 0;
    bool mask_shared = false, cull = true;
    const void* new_buf = nullptr;  // the shared masks' buffer once this batch's eye launch is in
    if (t0.rt && t0.rt_persp && !t0.sdf) {
        // per-wave primitive masks (rt_cull_batch_kernel) for every frame with primitives,
        // ceil(W/64) * rows words each; stream-ordered reuse on this lane.  A mask depends on
        // the eye camera, the rows and the primitive table only; a batch's frames share the
        // camera and rows, so when every frame has frame 0's table (stored once, fresh_rt)
        // they share frame 0's masks: one frame's cull per launch (main()'s scene: the same
        // cylinder every frame; config 7's cull 16 -> 0.3 us per 64-frame launch)
        mask_shared = n > 1;
        for (int k = 0; k < n && mask_shared; ++k) mask_shared = exs[k]->has_rt && (k == 0 || !fresh_rt[(size_t)k]);
        const size_t nw = (size_t)((fa[0].ey.W + 63) / 64) * (size_t)(fa[0].ey.row_end - fa[0].ey.row_begin);
        if ((rc = br.rtmask.ensure(sizeof(uint32_t) * nw * (size_t)(mask_shared ? 1 : n), ctx->device))) return rc;
        // Shared masks are a pure function of (primitive table, eye camera, sizes, rows,
        // stripes, format, flags): the same key as the lane's last shared cull, with the
        // buffer untouched since, finds the words already there (stream order: that cull ran
        // before this batch's eye pass).  main()'s scene, a static camera and cylinder, is
        // culled once per lane instead of once per launch.
        std::vector<char> key;
        if (mask_shared) {
            const EyePart& e = fa[0].ey;
            const int32_t sz[9] = {e.W, e.H, e.row_begin, e.row_end, e.stripe_rows, e.stripe_stride, e.stripe_phase,
                                   fmt, e.flags};
            key.resize(sizeof(RtK) + sizeof(CamK) + sizeof(sz));
            std::memcpy(key.data(), &exs[0]->rt, sizeof(RtK));
            std::memcpy(key.data() + sizeof(RtK), &e.eye, sizeof(CamK));
            std::memcpy(key.data() + sizeof(RtK) + sizeof(CamK), sz, sizeof(sz));
        }
        cull = !(mask_shared && br.mask_buf == br.rtmask.p && br.mask_key == key);
        // (the buffer's words count as this key's only once the batch's launches are in:
        // until then, and after any failure on the way, they count as nobody's)
        if (mask_shared) new_buf = br.rtmask.p;
        br.mask_key = std::move(key);
        br.mask_buf = nullptr;
        for (int k = 0; k < n; ++k)
            if (exs[k]->has_rt) {
                BatchFrame& bf = *(BatchFrame*)(hb + sizeof(BatchFrame) * (size_t)k);
                bf.tabs.rtmask = (uint32_t*)br.rtmask.p + nw * (size_t)(mask_shared ? 0 : k);
                bf.tabs.rtmask_words = (int32_t)nw;
            }
        t0.rtmask = (uint32_t*)br.rtmask.p;
        t0.rtmask_words = (int32_t)nw;
    }
    t0.fmt = fmt;
    // the lane's stream pulls the table from the pinned slot: in stream order after the
    // lane's earlier batches (the previous readers of this device slot), and copied[j]
    // tells the host when the slot may be refilled
    if ((rc = launch_pull(br.host_dev[j], bytes, db, s))) return fail(rc, "batch table pull failed");
    HIP_TRY(hipEventRecord(br.copied[j], s));
    TimingSlot* slot = next_slot(ctx);
    if (!fused) {
        if (slot) HIP_TRY(hipEventRecord(slot->ev[0], s));
        // the union of the frames' sphere boxes (the split coded launch)
        int32_t box[4] = {INT32_MAX, INT32_MIN, INT32_MAX, INT32_MIN};
        for (int k = 0; k < n; ++k) {
            const ShadowPart& q = fa[k].sh;
            if (q.cull_x0 > q.cull_x1 || q.cull_y0 > q.cull_y1) continue;
            box[0] = std::min(box[0], q.cull_x0);
            box[1] = std::max(box[1], q.cull_x1);
            box[2] = std::min(box[2], q.cull_y0);
            box[3] = std::max(box[3], q.cull_y1);
        }
        if ((rc = launch_shadow_batch((const BatchFrame*)db, n, fa[0], s, box, alone)))
            return fail(rc, "batched shadow pass failed");
        if (slot) HIP_TRY(hipEventRecord(slot->ev[1], s));
        ctx->have_shadow_pass = true;
        ctx->last_trivial = false;
        ctx->last_smap = (const double*)((const char*)br.smaps.p + map_bytes * (size_t)(n - 1));
        ctx->last_sh = fa[n - 1].sh;
        ctx->smap_w = fa[0].sh.W;
        ctx->smap_h = fa[0].sh.H;
    } else if (trivial) {
        note_trivial(ctx, fa[n - 1].sh);
    } else {
        ctx->have_shadow_pass = false;
    }
    if (slot) HIP_TRY(hipEventRecord(slot->ev[2], s));
    int blocks = 0;
    if ((rc = launch_eye_batch((const BatchFrame*)db, n, fa[0], t0, s, &blocks, mask_shared, cull)))
        return fail(rc, "batched eye pass failed");
    if (t0.rtmask) br.mask_buf = new_buf;  // (a batch without masks leaves the lane's words as they were)
    ctx->eye_blocks_last = blocks;
    if (slot) {
        HIP_TRY(hipEventRecord(slot->ev[3], s));
        slot->shadow = !fused;
        ctx->renders++;
    }
    HIP_TRY(hipEventRecord(br.used[j], s));
    return RTM_OK;
}

// Per-thread default contexts, one per device (rtm_render: device 0; rtm_render_multi: 0..n-1).
rtm_ctx* default_ctx(int* rc, int device = 0) {
    using Ctx = std::unique_ptr<rtm_ctx, void (*)(rtm_ctx*)>;
    thread_local std::vector<Ctx> cs;
    while ((int)cs.size() <= device) cs.emplace_back(nullptr, rtm_ctx_destroy);
    Ctx& c = cs[(size_t)device];
    if (!c) {
        rtm_ctx* p = nullptr;
        *rc = rtm_ctx_create(device, &p);
        if (*rc) return nullptr;
        c.reset(p);
    }
    *rc = RTM_OK;
    return c.get();
}



}  // namespace

extern "C" {

int32_t rtm_abi_version(void) { return RTM_ABI_VERSION; }

const char* rtm_last_error(void) { return g_last_error.c_str(); }

int32_t rtm_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int rtm_ctx_create(int32_t device, rtm_ctx** out) {
    if (!out) return fail(RTM_ERR_INVALID, "out is NULL");
    *out = nullptr;
    int n = rtm_device_count();
    if (n <= 0) return fail(RTM_ERR_NO_DEVICE, "no HIP device visible");
    if (device < 0 || device >= n) return fail(RTM_ERR_INVALID, "device %d outside [0,%d)", device, n);
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, device));
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(RTM_ERR_NO_DEVICE, "device %d is %s, this library is built for gfx950", device, prop.gcnArchName);
    std::unique_ptr<rtm_ctx> c(new rtm_ctx);
    c->device = device;
    DeviceGuard g(device);
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    *out = c.release();
    int rc = rtm_ctx_set_timing_capacity(*out, 1);
    if (rc) {
        rtm_ctx_destroy(*out);
        *out = nullptr;
        return rc;
    }
    return RTM_OK;
}

void rtm_ctx_destroy(rtm_ctx* ctx) {
    if (!ctx) return;
    for (rtm_viewport* vp : ctx->viewports) vp->ctx = nullptr;  // calls on them now fail; destroy still frees
    {
        DeviceGuard g(ctx->device);
        if (ctx->stream) (void)hipStreamSynchronize(ctx->stream);
        for (auto& l : ctx->lanes) {
            (void)hipStreamSynchronize(l->stream);
            l->batch.reset();
            if (l->done) (void)hipEventDestroy(l->done);
            (void)hipStreamDestroy(l->stream);
        }
        ctx->lanes.clear();
        ctx->batch.reset();
        if (ctx->fork) (void)hipEventDestroy(ctx->fork);
        for (auto& sl : ctx->ring)
            for (auto& e : sl.ev)
                if (e) (void)hipEventDestroy(e);
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
    }
    delete ctx;
}

void* rtm_ctx_stream(rtm_ctx* ctx) { return ctx ? (void*)ctx->stream : nullptr; }

int rtm_ctx_synchronize(rtm_ctx* ctx) {
    if (!ctx) return fail(RTM_ERR_INVALID, "ctx is NULL");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return RTM_OK;
}

int rtm_ctx_alloc(rtm_ctx* ctx, int64_t bytes, void** out_dev) {
    if (!ctx || !out_dev || bytes <= 0) return fail(RTM_ERR_INVALID, "ctx/out NULL or bytes %lld", (long long)bytes);
    *out_dev = nullptr;
    DeviceGuard g(ctx->device);
    if (hipMalloc(out_dev, (size_t)bytes) != hipSuccess) {
        *out_dev = nullptr;
        return fail(RTM_ERR_OOM, "hipMalloc(%lld) failed", (long long)bytes);
    }
    return RTM_OK;
}

int rtm_ctx_free(rtm_ctx* ctx, void* dev) {
    if (!ctx) return fail(RTM_ERR_INVALID, "ctx is NULL");
    if (!dev) return RTM_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));  // no enqueued frame still writes it
    HIP_TRY(hipFree(dev));
    return RTM_OK;
}

int rtm_ctx_copy_to_host(rtm_ctx* ctx, const void* dev, void* host, int64_t bytes) {
    if (!ctx || !dev || !host || bytes < 0) return fail(RTM_ERR_INVALID, "bad arguments");
    if (bytes == 0) return RTM_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipMemcpyAsync(host, dev, (size_t)bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return RTM_OK;
}

int rtm_ctx_oob_reads(rtm_ctx* ctx, int64_t* count) {
    if (!ctx || !count) return fail(RTM_ERR_INVALID, "ctx/count is NULL");
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (auto& l : ctx->lanes) HIP_TRY(hipStreamSynchronize(l->stream));
    unsigned long long c = 0;
    if (read_oob_reads(&c, ctx->stream)) return fail(RTM_ERR_HIP, "reading the out-of-range count failed");
    *count = (int64_t)c;
    return RTM_OK;
}

int rtm_ctx_set_timing_capacity(rtm_ctx* ctx, int32_t capacity) {
    if (!ctx || capacity < 0 || capacity > (1 << 20)) return fail(RTM_ERR_INVALID, "ctx NULL or capacity %d", capacity);
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    for (auto& sl : ctx->ring)
        for (auto& e : sl.ev)
            if (e) (void)hipEventDestroy(e);
    ctx->ring.assign((size_t)capacity, TimingSlot{});
    ctx->renders = 0;
    // Timing-only events: no system-scope release fence when recorded (it would
    // write back and invalidate the caches between the frame's kernels, adding
    // ~2-3 us to each timed kernel and slowing the work after it).  They are read
    // only after the stream has been synchronised.
    for (auto& sl : ctx->ring)
        for (auto& e : sl.ev) HIP_TRY(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    return RTM_OK;
}

int rtm_ctx_set_timing_stride(rtm_ctx* ctx, int32_t stride) {
    if (!ctx || stride < 1) return fail(RTM_ERR_INVALID, "ctx NULL or stride %d < 1", stride);
    ctx->stride = stride;
    ctx->calls = 0;
    return RTM_OK;
}

int rtm_ctx_set_lanes(rtm_ctx* ctx, int32_t lanes) {
    if (!ctx || lanes < 0 || lanes > 8) return fail(RTM_ERR_INVALID, "ctx NULL or lanes %d outside [0,8]", lanes);
    ctx->lanes_req = lanes;
    return RTM_OK;
}

int rtm_ctx_set_batch(rtm_ctx* ctx, int32_t frames) {
    if (!ctx || frames < 0 || frames > 64) return fail(RTM_ERR_INVALID, "ctx NULL or batch %d outside [0,64]", frames);
    ctx->batch_req = frames;
    return RTM_OK;
}

int rtm_ctx_last_batch(rtm_ctx* ctx, int32_t* frames) {
    if (!ctx || !frames) return fail(RTM_ERR_INVALID, "bad arguments");
    *frames = ctx->batch_last;
    return RTM_OK;
}

int rtm_ctx_last_eye_blocks(rtm_ctx* ctx, int32_t* blocks) {
    if (!ctx || !blocks) return fail(RTM_ERR_INVALID, "bad arguments");
    *blocks = ctx->eye_blocks_last;
    return RTM_OK;
}

int rtm_ctx_frames_plan(rtm_ctx* ctx, int32_t width, int32_t rows, int32_t n_frames, int32_t* lanes,
                        int32_t* frames_per_launch) {
    if (!ctx || !lanes || !frames_per_launch || width < 1 || rows < 1 || n_frames < 1)
        return fail(RTM_ERR_INVALID, "bad arguments");
    // rtm_render_frames_async's own rules (frame_batch, frame_lanes) for distinct outputs
    const int32_t B = std::min<int32_t>(frame_batch(ctx->batch_req, width, rows), n_frames);
    std::vector<float*> outs((size_t)n_frames);
    for (int32_t i = 0; i < n_frames; ++i) outs[(size_t)i] = (float*)(uintptr_t)(((uintptr_t)i + 1) << 40);
    *frames_per_launch = B;
    *lanes = frame_lanes(ctx->lanes_req, n_frames, width, rows, outs.data(), B);
    return RTM_OK;
}

int rtm_ctx_shadow_map_stored_bytes(rtm_ctx* ctx, int64_t* bytes, int32_t* span_records) {
    if (!ctx || !bytes) return fail(RTM_ERR_INVALID, "bad arguments");
    *bytes = 0;
    if (span_records) *span_records = 0;
    const int32_t tb = rtm_ctx_shadow_map_texel_bytes(ctx);
    if (tb == 0) return RTM_OK;
    const ShadowPart& sh = ctx->last_sh;
    if (!sh.smap_spans) {
        *bytes = tb == 8 ? (int64_t)sh.W * sh.H * 8 : smap_bytes(sh.smap_fmt, sh.W, sh.H);
        return RTM_OK;
    }
    if (span_records) *span_records = 1;
    // the span records, then the block bytes of every span stored texel by texel (its
    // rows of whole 4-row blocks, 128-column blocks wide as the tile stores them)
    DeviceGuard g(ctx->device);
    const int64_t pitch = (int64_t)sh.smap_bw * 128, nspan = (sh.H + SPAN_ROWS - 1) / SPAN_ROWS;
    std::vector<uint32_t> rec((size_t)(pitch * nspan));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    HIP_TRY(hipMemcpy(rec.data(), (const char*)ctx->last_smap + smap_span_offset(sh.W, sh.H),
                      rec.size() * sizeof(uint32_t), hipMemcpyDeviceToHost));
    const int32_t H4 = (sh.H + 3) & ~3;
    int64_t n = (int64_t)rec.size() * 4;
    for (int64_t sp = 0; sp < nspan; ++sp) {
        const int64_t rows = std::min<int64_t>(SPAN_ROWS, H4 - sp * SPAN_ROWS);
        for (int64_t x = 0; x < pitch; ++x) n += rec[(size_t)(sp * pitch + x)] == SPAN_DENSE ? rows : 0;
    }
    *bytes = n;
    return RTM_OK;
}

int rtm_ctx_last_lanes(rtm_ctx* ctx, int32_t* lanes) {
    if (!ctx || !lanes) return fail(RTM_ERR_INVALID, "bad arguments");
    *lanes = ctx->lanes_last;
    return RTM_OK;
}

int rtm_ctx_kernel_ms_history(rtm_ctx* ctx, float* shadow_ms, float* eye_ms, int32_t max, int32_t* count) {
    if (!ctx || max < 0 || !count) return fail(RTM_ERR_INVALID, "bad arguments");
    DeviceGuard g(ctx->device);
    const int64_t cap = (int64_t)ctx->ring.size();
    int64_t n = ctx->renders < cap ? ctx->renders : cap;
    if (n > max) n = max;
    for (int64_t i = 0; i < n; ++i) {
        const TimingSlot& sl = ctx->ring[(size_t)((ctx->renders - n + i) % cap)];
        float sm = 0.0f, em = 0.0f;
        if (sl.shadow) HIP_TRY(hipEventElapsedTime(&sm, sl.ev[0], sl.ev[1]));
        HIP_TRY(hipEventElapsedTime(&em, sl.ev[2], sl.ev[3]));
        if (shadow_ms) shadow_ms[i] = sm;
        if (eye_ms) eye_ms[i] = em;
    }
    *count = (int32_t)n;
    return RTM_OK;
}

int rtm_ctx_last_kernel_ms(rtm_ctx* ctx, float* shadow_ms, float* eye_ms) {
    if (!ctx) return fail(RTM_ERR_INVALID, "ctx is NULL");
    if (ctx->renders == 0 || ctx->ring.empty()) return fail(RTM_ERR_INVALID, "no timed render yet");
    int32_t n = 0;
    float sm = 0.0f, em = 0.0f;
    int rc = rtm_ctx_kernel_ms_history(ctx, &sm, &em, 1, &n);
    if (rc) return rc;
    if (shadow_ms) *shadow_ms = sm;
    if (eye_ms) *eye_ms = em;
    return RTM_OK;
}

int rtm_render_async(rtm_ctx* ctx, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                     int32_t width, int32_t height, int32_t march_steps, int32_t flags, int32_t row_begin,
                     int32_t row_end, float* out_rgba_dev) {
    return rtm_render_rows_async(ctx, scene, eye, shadow, width, height, march_steps, flags, RTM_FORMAT_RGBA32F,
                                 row_begin, row_end, out_rgba_dev);
}

int32_t rtm_ctx_shadow_map_texel_bytes(rtm_ctx* ctx) {
    if (!ctx || !ctx->have_shadow_pass || ctx->last_trivial) return 0;
    const int32_t f = ctx->last_sh.smap_fmt;
    return f == SMAP_U8 ? 1 : f == SMAP_U16 ? 2 : 8;
}

const double* rtm_ctx_shadow_map(rtm_ctx* ctx) {
    if (!ctx || !ctx->have_shadow_pass) return nullptr;
    if (ctx->last_trivial) {
        // the all-+INF viewport of a frame without shadow raster and march, materialised now
        DeviceGuard g(ctx->device);
        const int64_t n = (int64_t)ctx->last_sh.W * ctx->last_sh.H;
        if (ctx->smap_dec.ensure(sizeof(double) * (size_t)n, ctx->device)) return nullptr;
        if (launch_fill((double*)ctx->smap_dec.p, n, INFINITY, nullptr, 0, ctx->stream)) return nullptr;
        if (hipStreamSynchronize(ctx->stream) != hipSuccess) return nullptr;
        return (const double*)ctx->smap_dec.p;
    }
    if (ctx->last_sh.smap_fmt == SMAP_F64) return ctx->last_smap;
    // a coded map (rtm_kernels.h): its f64 values, decoded after the frame on the
    // context stream, then waited for
    DeviceGuard g(ctx->device);
    const ShadowPart& sh = ctx->last_sh;
    if (ctx->smap_dec.ensure(sizeof(double) * (size_t)sh.W * (size_t)sh.H, ctx->device)) return nullptr;
    if (launch_smap_decode(sh, ctx->last_smap, (double*)ctx->smap_dec.p, ctx->stream)) return nullptr;
    if (hipStreamSynchronize(ctx->stream) != hipSuccess) return nullptr;
    return (const double*)ctx->smap_dec.p;
}

int rtm_render_frames_async(rtm_ctx* ctx, int32_t n_frames, const rtm_scene* scenes, const rtm_camera* eye,
                            const rtm_camera* shadow, int32_t width, int32_t height, int32_t march_steps,
                            int32_t flags, float* const* out_rgba_dev) {
    if (!ctx || !scenes || !out_rgba_dev || n_frames < 1) return fail(RTM_ERR_INVALID, "bad arguments");
    for (int32_t i = 0; i < n_frames; ++i)
        if (!out_rgba_dev[i]) return fail(RTM_ERR_INVALID, "out_rgba_dev[%d] is NULL", i);
    // two kernels per frame (or per batch of frames): build each batch's arguments just
    // before its launches, so the GPU starts on batch 0 while the host prepares batch 1
    // (building all frames first left the GPU idle for the whole build).  (A software-
    // pipelined launch -- the shadow pass of frame i with the eye pass of frame i-1 in
    // one grid -- measured slower than two back-to-back kernels per frame, config 3 99.5
    // vs 79.1 us/frame, profiles/r01_ab_pipe.txt; a lane stagger lost at 3840x2160 and
    // 512x512, profiles/r02_ab_batch.txt.  Both are gone.)
    DeviceGuard g(ctx->device);
    int B = std::min<int32_t>(frame_batch(ctx->batch_req, width, height), n_frames);
    int L = frame_lanes(ctx->lanes_req, n_frames, width, height, out_rgba_dev, B);
    int rc = RTM_OK;
    if (L > 1) {  // fork: the lanes start after the context stream's earlier work
        if ((rc = ensure_lanes(ctx, L))) return rc;
        HIP_TRY(hipEventRecord(ctx->fork, ctx->stream));
        for (int k = 1; k < L; ++k) HIP_TRY(hipStreamWaitEvent(ctx->lanes[(size_t)k - 1]->stream, ctx->fork, 0));
    }
    ctx->lanes_last = L;
    ctx->batch_last = B;
    const int32_t nb = (n_frames + B - 1) / B;
    std::vector<FrameArgs> fa((size_t)B);
    std::vector<FrameExtra> fx((size_t)B);
    for (int32_t b = 0; b < nb && !rc; ++b) {
        const int32_t i0 = b * B, nf = std::min(B, n_frames - i0);
        const int lane = (nb - 1 - b) % L;
        for (int32_t k = 0; k < nf && !rc; ++k) {
            rc = build_frame(fa[(size_t)k], &scenes[i0 + k], eye, shadow, width, height, march_steps, flags);
            if (!rc) build_extra(&scenes[i0 + k], eye, width, height, fx[(size_t)k]);
        }
        if (rc) break;
        // runs of frames with the same march tables (patches) and disjoint outputs share
        // one launch per pass (frames of one launch run concurrently, so a repeated
        // output pointer starts a new run: the later frame still lands last); single
        // frames take the per-frame kernels
        const uintptr_t frame_bytes = (uintptr_t)width * (uintptr_t)height * 4u * sizeof(float);
        for (int32_t k = 0; k < nf && !rc;) {
            int32_t e = k + 1;
            auto disjoint = [&](int32_t q) {
                const uintptr_t o = (uintptr_t)out_rgba_dev[i0 + q];
                for (int32_t p = k; p < q; ++p) {
                    const uintptr_t op = (uintptr_t)out_rgba_dev[i0 + p];
                    if (o < op + frame_bytes && op < o + frame_bytes) return false;
                }
                return true;
            };
            while (e < nf && fa[(size_t)e].sh.n_patches == fa[(size_t)k].sh.n_patches &&
                   std::memcmp(fa[(size_t)e].sh.patch, fa[(size_t)k].sh.patch,
                               sizeof(PatchK) * (size_t)fa[(size_t)k].sh.n_patches) == 0 &&
                   disjoint(e))
                ++e;
            if (e - k >= 2) {
                std::vector<const FrameExtra*> xp((size_t)(e - k));
                for (int32_t q = k; q < e; ++q) xp[(size_t)(q - k)] = &fx[(size_t)q];
                rc = enqueue_batch(ctx, lane, &fa[(size_t)k], xp.data(),
                                   reinterpret_cast<void* const*>(out_rgba_dev + i0 + k), e - k, RTM_FORMAT_RGBA32F,
                                   L == 1);
            } else {
                rc = enqueue_frame(ctx, fa[(size_t)k], &fx[(size_t)k], out_rgba_dev[i0 + k], nullptr, lane);
            }
            k = e;
        }
    }
    // join every lane (also after an error, so the context stream still covers what
    // was enqueued); the first error, of the frames or of a join, is returned
    const std::string frame_err = rc ? g_last_error : std::string();
    int join_rc = RTM_OK;
    for (int k = 1; k < L; ++k) {
        Lane& l = *ctx->lanes[(size_t)k - 1];
        hipError_t e = hipEventRecord(l.done, l.stream);
        if (e == hipSuccess) e = hipStreamWaitEvent(ctx->stream, l.done, 0);
        if (e != hipSuccess && !join_rc) join_rc = fail(RTM_ERR_HIP, "lane %d join: %s", k, hipGetErrorString(e));
    }
    if (rc) {
        g_last_error = frame_err;
        return rc;
    }
    return join_rc;
}

int32_t rtm_format_bytes(int32_t format) { return format_bytes(format); }

int rtm_host_register(void* ptr, int64_t bytes) {
    if (!ptr || bytes <= 0) return fail(RTM_ERR_INVALID, "bad host buffer");
    if (rtm_device_count() <= 0) return fail(RTM_ERR_NO_DEVICE, "no HIP device visible");
    HIP_TRY(hipHostRegister(ptr, (size_t)bytes, hipHostRegisterPortable));
    return RTM_OK;
}

int rtm_host_unregister(void* ptr) {
    if (!ptr) return fail(RTM_ERR_INVALID, "ptr is NULL");
    HIP_TRY(hipHostUnregister(ptr));
    return RTM_OK;
}

int rtm_render_rows_async(rtm_ctx* ctx, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                          int32_t width, int32_t height, int32_t march_steps, int32_t flags, int32_t format,
                          int32_t row_begin, int32_t row_end, void* out_dev) {
    if (!ctx) return fail(RTM_ERR_INVALID, "ctx is NULL");
    if (!out_dev) return fail(RTM_ERR_INVALID, "out_dev is NULL");
    int rc = validate_format(format, out_dev);
    if (rc) return rc;
    FrameArgs a;
    if ((rc = build_frame(a, scene, eye, shadow, width, height, march_steps, flags))) return rc;
    if (row_begin < 0 || row_end > height || row_begin >= row_end)
        return fail(RTM_ERR_INVALID, "row range [%d,%d) outside [0,%d)", row_begin, row_end, height);
    a.ey.row_begin = row_begin;
    a.ey.row_end = row_end;
    FrameExtra x;
    build_extra(scene, eye, width, height, x);
    DeviceGuard g(ctx->device);
    return enqueue_frame(ctx, a, &x, out_dev, nullptr, 0, format);
}

int rtm_render_ex(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t width,
                  int32_t height, int32_t march_steps, int32_t flags, int32_t format, void* out_host) {
    if (!out_host) return fail(RTM_ERR_INVALID, "out is NULL");
    if (!format_bytes(format)) return fail(RTM_ERR_INVALID, "unknown output format %d", format);
    FrameArgs a;
    int rc = build_frame(a, scene, eye, shadow, width, height, march_steps, flags);
    if (rc) return rc;
    rtm_ctx* ctx = default_ctx(&rc);
    if (!ctx) return rc;
    FrameExtra x;
    build_extra(scene, eye, width, height, x);
    DeviceGuard g(ctx->device);
    const size_t bytes = (size_t)format_bytes(format) * (size_t)width * (size_t)height;
    if ((rc = ctx->out.ensure(bytes, ctx->device))) return rc;
    if ((rc = enqueue_frame(ctx, a, &x, ctx->out.p, nullptr, 0, format))) return rc;
    HIP_TRY(hipMemcpyAsync(out_host, ctx->out.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return RTM_OK;
}

int rtm_render(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t width,
               int32_t height, int32_t march_steps, int32_t flags, float* out_rgba) {
    return rtm_render_ex(scene, eye, shadow, width, height, march_steps, flags, RTM_FORMAT_RGBA32F, out_rgba);
}

int rtm_render_multi_ex(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t width,
                        int32_t height, int32_t march_steps, int32_t flags, int32_t format, void* out_host,
                        int32_t n_gpus) {
    if (!out_host) return fail(RTM_ERR_INVALID, "out is NULL");
    if (!format_bytes(format)) return fail(RTM_ERR_INVALID, "unknown output format %d", format);
    const int n_dev = rtm_device_count();
    if (n_dev <= 0) return fail(RTM_ERR_NO_DEVICE, "no HIP device visible");
    if (n_gpus < 1 || n_gpus > n_dev) return fail(RTM_ERR_INVALID, "n_gpus=%d outside [1,%d]", n_gpus, n_dev);
    // Row bands, one per device.  With more than one device every band evaluates
    // the shadow texels it reads (RTM_FLAG_FUSED_SHADOW: same image bits), so no
    // device needs another's shadow map and there is no device-to-device exchange:
    // each band goes straight from its device into its slice of the host frame.
    const int32_t f = flags | (n_gpus > 1 ? RTM_FLAG_FUSED_SHADOW : 0);
    FrameArgs a;
    int rc = build_frame(a, scene, eye, shadow, width, height, march_steps, f);
    if (rc) return rc;
    FrameExtra x;
    build_extra(scene, eye, width, height, x);
    const int32_t band = (height + n_gpus - 1) / n_gpus;
    const size_t bpp = (size_t)format_bytes(format);
    std::vector<rtm_ctx*> ctxs((size_t)n_gpus, nullptr);
    for (int d = 0; d < n_gpus; ++d) {
        const int32_t r0 = std::min(height, d * band), r1 = std::min(height, (d + 1) * band);
        if (r0 >= r1) continue;
        rtm_ctx* ctx = default_ctx(&rc, d);
        if (!ctx) return rc;
        ctxs[(size_t)d] = ctx;
        DeviceGuard g(ctx->device);
        FrameArgs ad = a;
        ad.ey.row_begin = r0;
        ad.ey.row_end = r1;
        const size_t bytes = bpp * (size_t)width * (size_t)(r1 - r0);
        if ((rc = ctx->out.ensure(bytes, ctx->device))) return rc;
        if ((rc = enqueue_frame(ctx, ad, &x, ctx->out.p, nullptr, 0, format))) return rc;
    }
    // The bands' D2H copies, one host thread per device: a pageable copy blocks its
    // calling thread, so issuing them from one thread would serialise the devices'
    // PCIe links; into a registered buffer the copies are DMA and return at once.
    std::vector<int> rcs((size_t)n_gpus, RTM_OK);
    std::vector<std::string> errs((size_t)n_gpus);
    auto copy_band = [&](int d) {
        rtm_ctx* ctx = ctxs[(size_t)d];
        const int32_t r0 = std::min(height, d * band), r1 = std::min(height, (d + 1) * band);
        DeviceGuard g(ctx->device);
        hipError_t e = hipMemcpyAsync((char*)out_host + bpp * (size_t)r0 * (size_t)width, ctx->out.p,
                                      bpp * (size_t)width * (size_t)(r1 - r0), hipMemcpyDeviceToHost, ctx->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(ctx->stream);
        if (e != hipSuccess) {
            rcs[(size_t)d] = RTM_ERR_HIP;
            errs[(size_t)d] = std::string("band copy from device ") + std::to_string(ctx->device) + ": " +
                              hipGetErrorString(e);
        }
    };
    int n_live = 0;
    for (rtm_ctx* c : ctxs) n_live += c != nullptr;
    if (n_live <= 1) {
        for (int d = 0; d < n_gpus; ++d)
            if (ctxs[(size_t)d]) copy_band(d);
    } else {
        std::vector<std::thread> th;
        for (int d = 0; d < n_gpus; ++d)
            if (ctxs[(size_t)d]) th.emplace_back(copy_band, d);
        for (auto& t : th) t.join();
    }
    for (int d = 0; d < n_gpus; ++d)
        if (rcs[(size_t)d]) return fail(rcs[(size_t)d], "%s", errs[(size_t)d].c_str());
    return RTM_OK;
}

int rtm_render_multi(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t width,
                     int32_t height, int32_t march_steps, int32_t flags, float* out_rgba, int32_t n_gpus) {
    return rtm_render_multi_ex(scene, eye, shadow, width, height, march_steps, flags, RTM_FORMAT_RGBA32F, out_rgba,
                               n_gpus);
}

int rtm_render_stats(rtm_ctx* ctx, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                     int32_t width, int32_t height, int32_t march_steps, int32_t flags, rtm_stats* out) {
    if (!ctx || !out) return fail(RTM_ERR_INVALID, "ctx/out is NULL");
    FrameArgs a;
    int rc = build_frame(a, scene, eye, shadow, width, height, march_steps, flags);
    if (rc) return rc;
    FrameExtra x;
    build_extra(scene, eye, width, height, x);
    DeviceGuard g(ctx->device);
    const size_t bytes = sizeof(float) * 4 * (size_t)width * (size_t)height;
    if ((rc = ctx->out.ensure(bytes, ctx->device))) return rc;
    if ((rc = ctx->stats.ensure(sizeof(StatsK), ctx->device))) return rc;
    HIP_TRY(hipMemsetAsync(ctx->stats.p, 0, sizeof(StatsK), ctx->stream));
    if ((rc = enqueue_frame(ctx, a, &x, (float*)ctx->out.p, (StatsK*)ctx->stats.p))) return rc;
    HIP_TRY(hipMemcpyAsync(out, ctx->stats.p, sizeof(StatsK), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return RTM_OK;
}

// ---- writeColorImage (row f-2) ----

int rtm_encode_thresholds(float out[256]) {
    if (!out) return fail(RTM_ERR_INVALID, "out is NULL");
    std::memcpy(out, encode_table().t, sizeof(float) * 256);
    return RTM_OK;
}

namespace {
// The encode tables on ctx's device (uploaded once per context, stream-ordered).
int enc_tab_dev(rtm_ctx* ctx, const void** out) {
    if (!ctx->enc_tab_ready) {
        const EncodeTable& t = encode_table();
        if (t.max_crossings > 1) return fail(RTM_ERR_UNSUPPORTED, "platform powf: bucket spans %d thresholds",
                                             t.max_crossings);
        int rc = ctx->enc_tab.ensure(ENC_DEV_BYTES, ctx->device);
        if (rc) return rc;
        // synchronous: the eye epilogue may read it from any of the context's streams
        HIP_TRY(hipMemcpy(ctx->enc_tab.p, t.t, 1024, hipMemcpyHostToDevice));
        HIP_TRY(hipMemcpy((char*)ctx->enc_tab.p + 1024, t.bucket, ENC_BUCKETS, hipMemcpyHostToDevice));
        ctx->enc_tab_ready = true;
    }
    *out = ctx->enc_tab.p;
    return RTM_OK;
}
}  // namespace

int rtm_encode_rgb8_async(rtm_ctx* ctx, const float* rgba_dev, int64_t n_pixels, uint8_t* rgb_dev) {
    if (!ctx || !rgba_dev || !rgb_dev || n_pixels < 0) return fail(RTM_ERR_INVALID, "bad arguments");
    if ((uintptr_t)rgba_dev & 15) return fail(RTM_ERR_INVALID, "rgba_dev must be 16-byte aligned");
    DeviceGuard g(ctx->device);
    const void* tab = nullptr;
    int rc = enc_tab_dev(ctx, &tab);
    if (rc) return rc;
    rc = launch_encode_rgb8(rgba_dev, n_pixels, rgb_dev, tab, ctx->stream);
    return rc ? fail(rc, "encode launch failed") : RTM_OK;
}

int64_t rtm_ppm_max_bytes(int32_t width, int32_t height) {
    if (width <= 0 || height <= 0) return 0;
    // header "P3\n" + "W H\n" + "255\n"; per pixel at most "255 255 255  " (13); '\n' per row
    return 3 + 24 + 4 + (int64_t)width * height * 13 + height;
}

int rtm_write_ppm(rtm_ctx* ctx, const float* rgba_dev, int32_t width, int32_t height, char* out, int64_t capacity,
                  int64_t* length) {
    if (!ctx || !rgba_dev || !length) return fail(RTM_ERR_INVALID, "bad arguments");
    if ((uintptr_t)rgba_dev & 15) return fail(RTM_ERR_INVALID, "rgba_dev must be 16-byte aligned");
    int rc;
    if ((rc = validate_dims(width, height))) return rc;
    char header[64];
    const int hl = snprintf(header, sizeof header, "P3\n%d %d\n255\n", width, height);  // main.rs:666-668
    const int64_t n = (int64_t)width * height;
    DeviceGuard g(ctx->device);
    if ((rc = ctx->enc_rgb.ensure((size_t)n * 3, ctx->device)) ||
        (rc = ctx->enc_rows.ensure(sizeof(int64_t) * (2 * (size_t)height + 1), ctx->device)) ||
        (rc = ctx->enc_text.ensure((size_t)rtm_ppm_max_bytes(width, height), ctx->device)))
        return rc;
    uint8_t* rgb = (uint8_t*)ctx->enc_rgb.p;
    int64_t* rowlen = (int64_t*)ctx->enc_rows.p;
    int64_t* rowoff = rowlen + height;
    int64_t* total = rowoff + height;
    char* text = (char*)ctx->enc_text.p;
    const void* tab = nullptr;
    if ((rc = enc_tab_dev(ctx, &tab))) return rc;
    if ((rc = launch_encode_rgb8(rgba_dev, n, rgb, tab, ctx->stream)))
        return fail(rc, "encode launch failed");
    if ((rc = launch_ppm_text(rgb, width, height, hl, rowlen, rowoff, total, text, ctx->stream)))
        return fail(rc, "ppm launch failed");
    int64_t tot = 0;
    HIP_TRY(hipMemcpyAsync(&tot, total, sizeof tot, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    *length = tot;
    if (!out || tot > capacity) return fail(RTM_ERR_INVALID, "ppm needs %lld bytes, capacity %lld", (long long)tot,
                                            (long long)capacity);
    std::memcpy(out, header, (size_t)hl);
    HIP_TRY(hipMemcpyAsync(out + hl, text + hl, (size_t)(tot - hl), hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return RTM_OK;
}

// ---- reference-seam API ----

int rtm_viewport_create(rtm_ctx* ctx, int32_t width, int32_t height, int32_t face, const rtm_camera* camera,
                        rtm_viewport** out) {
    if (!ctx || !out) return fail(RTM_ERR_INVALID, "ctx/out is NULL");
    *out = nullptr;
    int rc;
    if ((rc = validate_dims(width, height)) || (rc = validate_camera(camera, "viewport"))) return rc;
    if (face != RTM_FACE_FRONT && face != RTM_FACE_BACK) return fail(RTM_ERR_INVALID, "face %d", face);
    std::unique_ptr<rtm_viewport> v(new rtm_viewport);
    v->ctx = ctx;
    v->W = width;
    v->H = height;
    v->face = face;
    v->cam = *camera;
    DeviceGuard g(ctx->device);
    const size_t n = (size_t)width * (size_t)height;
    if ((rc = v->zbuf.ensure(n * sizeof(double), ctx->device)) || (rc = v->gh.ensure(n * sizeof(double), ctx->device)) ||
        (rc = v->gz.ensure(n * sizeof(double), ctx->device)) || (rc = v->gid.ensure(n * sizeof(int32_t), ctx->device)))
        return rc;
    // zBuffer: Map2d::new(.., INFINITY); rasterized: vec![None; ..] (main.rs:1534-1536)
    if ((rc = launch_fill((double*)v->zbuf.p, (int64_t)n, INFINITY, (int32_t*)v->gid.p, -1, ctx->stream)))
        return fail(rc, "viewport init launch failed");
    ctx->viewports.push_back(v.get());
    *out = v.release();
    return RTM_OK;
}

void rtm_viewport_destroy(rtm_viewport* vp) {
    if (!vp) return;
    if (vp->ctx) {  // (an orphaned viewport's context already drained its stream)
        DeviceGuard g(vp->ctx->device);
        (void)hipStreamSynchronize(vp->ctx->stream);
        auto& v = vp->ctx->viewports;
        v.erase(std::remove(v.begin(), v.end(), vp), v.end());
    }
    delete vp;
}

int rtm_viewport_rasterize(rtm_viewport* vp, const rtm_scene* scene) {
    if (!vp || !vp->ctx) return fail(RTM_ERR_INVALID, "viewport is NULL or its context was destroyed");
    int rc;
    if ((rc = validate_scene(scene))) return rc;
    if (scene->n_spheres == 0) return RTM_OK;  // main.rs:447: nothing to project
    RasterArgs a;
    std::memset(&a, 0, sizeof a);
    a.persp = vp->cam.type != RTM_CAMERA_ORTHOGONAL;
    for (int i = 0; i < scene->n_spheres; ++i)
        a.sph[i] = a.persp ? project_sphere_persp(vp->cam, scene->spheres[i], vp->W, vp->H, a.psp[i])
                           : project_sphere(vp->cam, scene->spheres[i], vp->W, vp->H);
    a.n_spheres = scene->n_spheres;
    a.face = vp->face;
    a.W = vp->W;
    a.H = vp->H;
    DeviceGuard g(vp->ctx->device);
    if ((rc = launch_vp_rasterize(a, (double*)vp->zbuf.p, (double*)vp->gh.p, (double*)vp->gz.p, (int32_t*)vp->gid.p,
                                  vp->ctx->stream)))
        return fail(rc, "rasterize launch failed");
    vp->raster_sp = std::max(vp->raster_sp, scene->n_spheres);
    return RTM_OK;
}

int rtm_viewport_process_raytracing_rays(rtm_viewport* vp, const rtm_scene* scene) {
    if (!vp || !vp->ctx) return fail(RTM_ERR_INVALID, "viewport is NULL or its context was destroyed");
    int rc;
    if ((rc = validate_scene(scene))) return rc;
    RtK k;
    SdfTabK sk;
    const bool has_rt = build_rt(scene, &vp->cam, k), has_sdf = build_sdf(scene, sk);
    if (!has_rt && !has_sdf) return RTM_OK;  // no circle planes, cylinders or SDFs: nothing to trace
    rtm_ctx* ctx = vp->ctx;
    DeviceGuard g(ctx->device);
    if ((rc = vp->gn.ensure(sizeof(double) * 3 * (size_t)vp->W * (size_t)vp->H, ctx->device))) return rc;
    TraceArgs a;
    std::memset(&a, 0, sizeof a);
    a.cam = cam_k(vp->cam);
    a.W = vp->W;
    a.H = vp->H;
    if (has_rt && (rc = upload_rt(ctx, ctx->rtk, ctx->stream, k, &a.rt))) return rc;
    if (has_sdf && (rc = upload_sdf(ctx, ctx->sdfk, ctx->stream, sk, &a.sdf))) return rc;
    if ((rc = launch_vp_trace(a, (double*)vp->zbuf.p, (double*)vp->gh.p, (int32_t*)vp->gid.p, (double*)vp->gn.p,
                              ctx->stream)))
        return fail(rc, "trace launch failed");
    vp->traced_pl = std::max(vp->traced_pl, k.n_pl);
    vp->traced_cy = std::max(vp->traced_cy, k.n_cy);
    vp->traced_sdf = std::max(vp->traced_sdf, sk.n);
    return RTM_OK;
}

int rtm_viewport_process_raymarching_rays(rtm_viewport* vp, const rtm_patch* patches, int32_t n_patches,
                                          int32_t steps) {
    if (!vp || !vp->ctx) return fail(RTM_ERR_INVALID, "viewport is NULL or its context was destroyed");
    if (n_patches < 0 || n_patches > RTM_MAX_PATCHES) return fail(RTM_ERR_INVALID, "n_patches=%d", n_patches);
    if (n_patches > 0 && !patches) return fail(RTM_ERR_INVALID, "patches is NULL");
    if (steps < 0) return fail(RTM_ERR_INVALID, "steps=%d", steps);
    MarchArgs a;
    std::memset(&a, 0, sizeof a);
    for (int i = 0; i < n_patches; ++i) a.patch[i] = patch_k(patches[i]);
    a.cam = cam_k(vp->cam);
    a.n_patches = n_patches;
    a.steps = steps;
    a.W = vp->W;
    a.H = vp->H;
    DeviceGuard g(vp->ctx->device);
    // (the staged march uses the per-ray path; no separable tables)
    int rc = ensure_tables(vp->ctx, steps, vp->W, vp->H, &vp->cam, nullptr, 0, &a.tab);
    if (rc) return rc;
    rc = launch_vp_march(a, (double*)vp->zbuf.p, vp->ctx->stream);
    if (rc) return fail(rc, "march launch failed");
    return RTM_OK;
}

int rtm_render_color_image(const rtm_scene* scene, const rtm_viewport* vp, const rtm_viewport* shadow_vp,
                           float* out_rgba) {
    if (!vp || !shadow_vp || !out_rgba) return fail(RTM_ERR_INVALID, "viewport/out is NULL");
    if (!vp->ctx || !shadow_vp->ctx) return fail(RTM_ERR_INVALID, "a viewport's context was destroyed");
    if (vp->ctx != shadow_vp->ctx) return fail(RTM_ERR_INVALID, "viewports belong to different contexts");
    int rc;
    if ((rc = validate_scene(scene))) return rc;
    if (shadow_vp->cam.type != RTM_CAMERA_ORTHOGONAL)
        return fail(RTM_ERR_UNSUPPORTED, "Camera::project is orthographic only (main.rs:1949)");
    // the G-buffer may hold ids of every primitive traced into it: the reference
    // indexes the scene's arrays with them and panics when out of range (main.rs:773, 791)
    if (vp->traced_pl > scene->n_circle_planes || vp->traced_cy > scene->n_capped_cylinders ||
        vp->traced_sdf > scene->n_sdfs || vp->raster_sp > scene->n_spheres)
        return fail(RTM_ERR_INVALID, "scene has fewer spheres/circle planes/cylinders/sdfs (%d/%d/%d/%d) than the "
                    "viewport holds (%d/%d/%d/%d)", scene->n_spheres, scene->n_circle_planes,
                    scene->n_capped_cylinders, scene->n_sdfs, vp->raster_sp, vp->traced_pl, vp->traced_cy,
                    vp->traced_sdf);
    ShadeArgs a;
    std::memset(&a, 0, sizeof a);
    for (int i = 0; i < scene->n_spheres; ++i) a.shade[i] = shade_sphere(scene->spheres[i]);
    a.eye = cam_k(vp->cam);
    a.shadow = cam_k(shadow_vp->cam);
    a.W = vp->W;
    a.H = vp->H;
    a.Ws = shadow_vp->W;
    a.Hs = shadow_vp->H;
    a.n_spheres = scene->n_spheres;
    rtm_ctx* ctx = vp->ctx;
    DeviceGuard g(ctx->device);
    const size_t bytes = sizeof(float) * 4 * (size_t)vp->W * (size_t)vp->H;
    if ((rc = ctx->out.ensure(bytes, ctx->device))) return rc;
    RtK k;
    SdfTabK sk;
    if (build_rt(scene, nullptr, k)) {  // shading lookups circlePlanePrimitives[id] / cappedCylinderPrimitives[id]
        if ((rc = upload_rt(ctx, ctx->rtk, ctx->stream, k, &a.rt))) return rc;
        a.gn = (const double*)vp->gn.p;
    }
    if (build_sdf(scene, sk)) {  // ... and the SDF colours (row f-4)
        if ((rc = upload_sdf(ctx, ctx->sdfk, ctx->stream, sk, &a.sdf))) return rc;
        a.gn = (const double*)vp->gn.p;
    }
    if ((rc = launch_vp_shade(a, (const double*)shadow_vp->zbuf.p, (const double*)vp->gh.p, (const double*)vp->gz.p,
                              (const int32_t*)vp->gid.p, (float*)ctx->out.p, ctx->stream)))
        return fail(rc, "shade launch failed");
    HIP_TRY(hipMemcpyAsync(out_rgba, ctx->out.p, bytes, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return RTM_OK;
}

int rtm_viewport_read_zbuffer(const rtm_viewport* vp, double* out) {
    if (!vp || !out || !vp->ctx) return fail(RTM_ERR_INVALID, "viewport/out is NULL or its context was destroyed");
    DeviceGuard g(vp->ctx->device);
    HIP_TRY(hipMemcpyAsync(out, vp->zbuf.p, sizeof(double) * (size_t)vp->W * (size_t)vp->H, hipMemcpyDeviceToHost,
                           vp->ctx->stream));
    HIP_TRY(hipStreamSynchronize(vp->ctx->stream));
    return RTM_OK;
}

}  // extern "C"

// ---- internal interface for rtm_group.cpp (rtm_internal.h) ----
namespace rtm {
namespace internal {

int check_frame(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t width,
                int32_t height, int32_t march_steps, int32_t flags) {
    return validate_frame(scene, eye, shadow, width, height, march_steps, flags);
}

PreparedFrame* new_prepared() { return new (std::nothrow) PreparedFrame; }

void delete_prepared(PreparedFrame* f) { delete f; }

int prepare_frame(PreparedFrame* f, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                  int32_t width, int32_t height, int32_t march_steps, int32_t flags) {
    int rc = build_frame(f->a, scene, eye, shadow, width, height, march_steps, flags);
    if (rc) return rc;
    build_extra(scene, eye, width, height, f->x);
    return RTM_OK;
}

int32_t stripe_rows_of(int32_t H, int32_t n, int32_t S, int32_t r) {
    const int32_t full = H / S, tail = H % S;  // stripes j = 0 .. ceil(H/S)-1, stripe j to rank j % n
    int32_t rows = (full / n + (r < full % n ? 1 : 0)) * S;
    if (tail && full % n == r) rows += tail;  // the last, short stripe is number `full`
    return rows;
}

void apply_rows(EyePart& ey, int32_t row_begin, int32_t row_end, const RowMap* m) {
    ey.row_begin = row_begin;
    ey.row_end = row_end;
    ey.stripe_rows = m ? m->stripe_rows : 0;
    ey.stripe_stride = m ? m->stride : 0;
    ey.stripe_phase = m ? m->phase : 0;
    ey.out_global = m ? m->out_global : 0;
}

int check_rows(const FrameArgs& a, int32_t row_begin, int32_t row_end, const RowMap* m) {
    if (row_begin < 0 || row_end > a.ey.H || row_begin >= row_end)
        return fail(RTM_ERR_INVALID, "row range [%d,%d) outside [0,%d)", row_begin, row_end, a.ey.H);
    if (m && m->stripe_rows > 0 && (row_begin != 0 || m->stride < m->stripe_rows || m->phase < 0 ||
                                    m->phase % m->stripe_rows != 0 || m->phase >= m->stride))
        return fail(RTM_ERR_INVALID, "bad row stripes");
    return RTM_OK;
}

int enqueue_prepared(rtm_ctx* ctx, const PreparedFrame* f, int32_t format, int32_t row_begin, int32_t row_end,
                     void* out_dev, const RowMap* map, int lane) {
    if (!ctx || !f || !out_dev) return fail(RTM_ERR_INVALID, "bad arguments");
    int rc = validate_format(format, out_dev);
    if (rc) return rc;
    if ((rc = check_rows(f->a, row_begin, row_end, map))) return rc;
    FrameArgs a = f->a;
    apply_rows(a.ey, row_begin, row_end, map);
    DeviceGuard g(ctx->device);
    return enqueue_frame(ctx, a, &f->x, out_dev, nullptr, lane, format);
}

int enqueue_prepared_batch(rtm_ctx* ctx, const PreparedFrame* const* fs, int n, int32_t format, int32_t row_begin,
                           int32_t row_end, void* const* outs, const RowMap* map, int lane) {
    if (!ctx || !fs || !outs || n < 1) return fail(RTM_ERR_INVALID, "bad arguments");
    if (lane < 0 || lane > (int)ctx->lanes.size()) return fail(RTM_ERR_INVALID, "lane %d of %zu", lane, ctx->lanes.size() + 1);
    if (n == 1) return enqueue_prepared(ctx, fs[0], format, row_begin, row_end, outs[0], map, lane);
    int rc;
    for (int k = 0; k < n; ++k) {
        if (!fs[k] || !outs[k]) return fail(RTM_ERR_INVALID, "bad arguments");
        if ((rc = validate_format(format, outs[k]))) return rc;
    }
    const FrameArgs& a0 = fs[0]->a;
    if ((rc = check_rows(a0, row_begin, row_end, map))) return rc;
    // one launch per pass needs the same march tables (patches) and sizes in every frame
    bool same = true;
    for (int k = 1; k < n && same; ++k) {
        const FrameArgs& b = fs[k]->a;
        same = b.sh.n_patches == a0.sh.n_patches && b.ey.W == a0.ey.W && b.ey.H == a0.ey.H &&
               b.sh.steps == a0.sh.steps && b.ey.flags == a0.ey.flags &&
               std::memcmp(&b.sh.cam, &a0.sh.cam, sizeof(CamK)) == 0 &&
               std::memcmp(&b.ey.eye, &a0.ey.eye, sizeof(CamK)) == 0 &&
               std::memcmp(b.sh.patch, a0.sh.patch, sizeof(PatchK) * (size_t)a0.sh.n_patches) == 0;
    }
    DeviceGuard g(ctx->device);
    if (!same) {
        for (int k = 0; k < n; ++k)
            if ((rc = enqueue_prepared(ctx, fs[k], format, row_begin, row_end, outs[k], map, lane))) return rc;
        return RTM_OK;
    }
    // the frames' arguments are copied (the rows and tables are set per launch); their
    // extras (13 KB of primitive tables each) are only read
    std::vector<FrameArgs> fa((size_t)n);
    std::vector<const FrameExtra*> xp((size_t)n);
    for (int k = 0; k < n; ++k) {
        fa[(size_t)k] = fs[k]->a;
        apply_rows(fa[(size_t)k].ey, row_begin, row_end, map);
        xp[(size_t)k] = &fs[k]->x;
    }
    return enqueue_batch(ctx, lane, fa.data(), xp.data(), outs, n, format);
}

int lanes_plan(const rtm_ctx* ctx, int32_t width, int32_t rows, int32_t n_batches) {
    // frame_lanes' rule for batches with disjoint outputs (the caller checks overlaps
    // and caps the count, lanes_begin's max_lanes)
    int L = ctx->lanes_req > 0 ? ctx->lanes_req : ((int64_t)width * rows >= (16LL << 20) ? 3 : 4);
    return std::max(1, std::min<int>(std::min(L, 8), n_batches));
}

int lanes_begin(rtm_ctx* ctx, int32_t width, int32_t rows, int32_t n_batches, int32_t max_lanes) {
    if (!ctx || n_batches < 1) return fail(RTM_ERR_INVALID, "bad arguments");
    int L = lanes_plan(ctx, width, rows, n_batches);
    if (max_lanes > 0) L = std::min<int>(L, max_lanes);
    ctx->lanes_last = std::max(L, 1);  // (rtm_ctx_last_lanes)
    if (L <= 1) return 1;
    DeviceGuard g(ctx->device);
    int rc = ensure_lanes(ctx, L);
    if (rc) return rc;
    HIP_TRY(hipEventRecord(ctx->fork, ctx->stream));
    for (int k = 1; k < L; ++k) HIP_TRY(hipStreamWaitEvent(ctx->lanes[(size_t)k - 1]->stream, ctx->fork, 0));
    return L;
}

int lanes_end(rtm_ctx* ctx, int L) {
    DeviceGuard g(ctx->device);
    for (int k = 1; k < L && k <= (int)ctx->lanes.size(); ++k) {
        Lane& l = *ctx->lanes[(size_t)k - 1];
        HIP_TRY(hipEventRecord(l.done, l.stream));
        HIP_TRY(hipStreamWaitEvent(ctx->stream, l.done, 0));
    }
    return RTM_OK;
}

hipStream_t lane_stream(const rtm_ctx* ctx, int lane) {
    return lane > 0 && lane <= (int)ctx->lanes.size() ? ctx->lanes[(size_t)lane - 1]->stream : ctx->stream;
}

int auto_frames_per_launch(int32_t width, int32_t rows) { return frame_batch(0, width, rows); }

int32_t bytes_per_pixel(int32_t format) { return format_bytes(format); }

int set_error(int code, const char* msg) { return fail(code, "%s", msg); }

int ctx_device(const rtm_ctx* ctx) { return ctx->device; }

hipStream_t ctx_stream(const rtm_ctx* ctx) { return ctx->stream; }

}  // namespace internal
}  // namespace rtm

extern "C" {

int rtm_render_stripes_async(rtm_ctx* ctx, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                             int32_t width, int32_t height, int32_t march_steps, int32_t flags, int32_t format,
                             int32_t stripe_rows, int32_t n_parts, int32_t part, void* out_dev) {
    if (!ctx) return fail(RTM_ERR_INVALID, "ctx is NULL");
    if (stripe_rows < 1 || n_parts < 1 || part < 0 || part >= n_parts)
        return fail(RTM_ERR_INVALID, "stripes: stripe_rows %d, part %d of %d", stripe_rows, part, n_parts);
    if ((int64_t)stripe_rows * n_parts > RTM_MAX_DIM * 8LL) return fail(RTM_ERR_INVALID, "stripe period too large");
    internal::PreparedFrame f;
    int rc = internal::prepare_frame(&f, scene, eye, shadow, width, height, march_steps, flags);
    if (rc) return rc;
    const int32_t rows = internal::stripe_rows_of(height, n_parts, stripe_rows, part);
    if (rows <= 0) return RTM_OK;  // a part with no rows (more parts than stripes)
    internal::RowMap m;
    m.stripe_rows = stripe_rows;
    m.stride = n_parts * stripe_rows;
    m.phase = part * stripe_rows;
    return internal::enqueue_prepared(ctx, &f, format, 0, rows, out_dev, &m);
}

int32_t rtm_stripe_rows(int32_t height, int32_t stripe_rows, int32_t n_parts, int32_t part) {
    if (height < 1 || stripe_rows < 1 || n_parts < 1 || part < 0 || part >= n_parts) return -1;
    return internal::stripe_rows_of(height, n_parts, stripe_rows, part);
}

}  // extern "C"
