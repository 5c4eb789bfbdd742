// rtm_kernels.hip — CDNA4 (gfx950) kernels for the per-pixel hot path of
// PtrMan/2018RustRayTracer src/main.rs.
//
// Numerics: IEEE f64 in the reference's operation order, FMA contraction off
// (file pragma + -ffp-contract=off), correctly-rounded f64 div/sqrt (the
// AMDGPU default lowering).  Every result is bit-identical to the reference
// semantics (tests/test_gpu_parity.py).
//
// Work mapping: one work-item per pixel; a 256-thread workgroup is a 64x4
// pixel tile, so each wave owns 64 consecutive pixels of one row: the RGBA f32
// store is one contiguous 1 KiB global_store_dwordx4 per wave and the f64
// shadow-map store 512 B.  Scene constants are kernel arguments (uniform:
// scalar cache -> SGPR operands); sphere culls are per-wave scalar compares.
// No MFMA: this is scalar per-pixel math, VALU-issue bound (profiles/).
#include <hip/hip_runtime.h>
#include <math.h>

#include <algorithm>
#include <type_traits>
#include <string>
#include <stdint.h>
#include <stdlib.h>

#include "rtm_kernels.h"

#pragma clang fp contract(off)

namespace rtm {

namespace {

constexpr int TILE_X = 64;  // one wave per tile row
constexpr int TILE_Y = 4;   // four waves per workgroup
constexpr int BLOCK = TILE_X * TILE_Y;

using cdouble = const __attribute__((address_space(4))) double;  // scalar-loaded table
using cint = const __attribute__((address_space(4))) int32_t;

// writeColorImage's per-channel byte (main.rs:674-684) by threshold lookup, as
// rtm_encode.hip's encode kernel computes it (the tables: rtm_encode.h): clamp as
// f32::max(0.0).min(1.0) (NaN -> 0), bucket byte, then at most one threshold.
__device__ __forceinline__ uint32_t enc_byte(float c, const float* __restrict__ T, const uint8_t* __restrict__ B) {
    float v = c > 0.0f ? c : 0.0f;
    v = v < 1.0f ? v : 1.0f;
    uint32_t k = B[__float_as_uint(v) >> 16];
    while (k < 255u && v >= T[k + 1]) ++k;
    return k;
}


// Out-of-range reads of the host-built side tables (the per-wave primitive masks,
// the coded tile's row records): every read of them is checked against the table's
// length; an index past it is counted here and not performed (the lanes that would
// make it are dead: rows past the launch's part).  rtm_ctx_oob_reads reads and
// clears the count; tests/test_bounds.py requires 0.
__device__ unsigned long long g_oob_reads;

__device__ __forceinline__ void note_oob() {
    if ((threadIdx.x & 63) == __builtin_ctzll(__ballot(1))) atomicAdd(&g_oob_reads, 1ull);
}


// main.rs:306-307 / 1903-1907: ((i as f64) / (res as f64)) * 2.0 - 1.0
__device__ __forceinline__ double ndc(int i, int res) { return ((double)i / (double)res) * 2.0 - 1.0; }

// inRange01 (main.rs:2282-2284)
__device__ __forceinline__ bool in01(double v) { return fabs(v - 0.5) <= 0.5; }

// calcDepthBilinear -> bilinear -> linear (main.rs:2146, 2073-2080, 2066-2069)
__device__ __forceinline__ double bil(const PatchK& p, double x, double y) {
    double d0 = p.a0 + p.d0 * x;
    double d1 = p.a1 + p.d1 * x;
    double dd = d1 - d0;
    return d0 + dd * y;
}

// Rust `as i64` followed by `(W/2) +`; only membership in [0,W) matters downstream,
// so magnitudes >= 4e18 map to an out-of-range sentinel (the reference's saturate+wrap
// is out of range as well).  NaN -> 0 exactly as Rust.
__device__ __forceinline__ int64_t tex_index(int64_t half, double v) {
    int64_t t;
    if (v != v) t = 0;
    else if (fabs(v) < 4.0e18) t = (int64_t)v;
    else t = v > 0.0 ? (int64_t)1 << 62 : -((int64_t)1 << 62);
    return half + t;
}

// Can any pixel of columns [xb, xe] in row y be covered by sphere s?  (exact
// pixel-index bbox, host-computed; wave-uniform when xb, xe, y are)
__device__ __forceinline__ bool may_cover(const RasterSphereK& s, int xb, int xe, int y) {
    return y >= s.iy0 && y <= s.iy1 && xe >= s.ix0 && xb <= s.ix1;
}

// The wave's sphere set: bit i set iff sphere i's pixel range can reach columns
// [xb, xe] of rows [ya, ye].  Lane i tests sphere i (one vector load of the range
// words) and a ballot gathers the bits, instead of a serial chain of per-sphere
// scalar loads and compares.  Call with every lane of the wave active.
__device__ __forceinline__ uint32_t wave_sphere_mask(const RasterSphereK* __restrict__ sph, int n, int xb, int xe,
                                                     int ya, int ye) {
    const int l = threadIdx.x & 63;
    bool m = false;
    if (l < n) {
        const RasterSphereK& s = sph[l];
        m = (ye >= s.iy0) & (ya <= s.iy1) & (xe >= s.ix0) & (xb <= s.ix1);
    }
    return (uint32_t)__ballot(m);
}

// Does the union of a viewport's sphere pixel ranges reach columns [xb, xe] of rows [ya, ye]?
// An empty union (no sphere covers anything: x0 > x1, the host's (1, 0, 1, 0)) reaches
// nothing -- without the emptiness test a range spanning row 0 and column 0 would
// "meet" it, and the split shadow launch would leave that strip to a part it never runs.
template <typename P>
__device__ __forceinline__ bool union_may_cover(const P& a, int xb, int xe, int ya, int ye) {
#if defined(RTM_TEST_REVERT_EMPTY_UNION)  // (tools/bounds_demo.sh only: the round-3 bug, no emptiness test)
    return (ye >= a.cull_y0) & (ya <= a.cull_y1) & (xe >= a.cull_x0) & (xb <= a.cull_x1);
#else
    return (a.cull_x0 <= a.cull_x1) & (a.cull_y0 <= a.cull_y1) & (ye >= a.cull_y0) & (ya <= a.cull_y1) &
           (xe >= a.cull_x0) & (xb <= a.cull_x1);
#endif
}

// Coverage under a PERSPECTIVE camera (row f-3): the same test with the general
// ellipse axes of projectSphere (main.rs:2848-2852, 2098-2109).
__device__ __forceinline__ bool cover_persp(const PerspSphK& s, double x, double y, double& h) {
    const double relx = x - s.cx;
    const double rely = y - s.cy;
    const double pa = (relx * s.nAx + rely * s.nAy) / s.mA;
    const double pb = (relx * s.nBx + rely * s.nBy) / s.mB;
    const double d = sqrt(pa * pa + pb * pb);
    if (d < 1.0) {
        h = sqrt(1.0 - d * d);
        return true;
    }
    return false;
}

// Sphere coverage of one pixel (projectSphereAtZBuffer, main.rs:176-195):
// calcOthoDistanceByAbsPosition -> calcEllipseDistToCenter -> calcHeightOfSphereOnUnit.
__device__ __forceinline__ bool cover(const RasterSphereK& s, double x, double y, double& h) {
    const double relx = x - s.cx;
    const double rely = y - s.cy;
    const double pa = (relx * s.n) / s.m;
    const double pb = (rely * s.n) / s.m;
    const double d = sqrt(pa * pa + pb * pb);
    if (d < 1.0) {
        h = sqrt(1.0 - d * d);
        return true;
    }
    return false;
}

struct MarchResult {
    bool hit;
    double t;
    int iters;  // loop iterations executed (stats only)
    int k;      // hit: the advances before it (t == t_after(tb, k), the coded map's march code)
};

// t after k advances (table built on the host by sequential summation; the
// fallback re-does the same sequential sum).
__device__ __forceinline__ double t_after(const Tables& tb, int k) {
    if (tb.t) return tb.t[k];
    double t = 0.0;
    for (int j = 0; j < k; ++j) t = t + 0.03;
    return t;
}

// v_cmp_class_f64 masks: bits 0-1 NaN, 2-5 negative (-inf,-norm,-denorm,-0),
// 6-9 positive (+0,+denorm,+norm,+inf).
constexpr int CLS_NAN = 0x003, CLS_NEG = 0x03C, CLS_POS = 0x3C0, CLS_ALL = 0x3FF;

// `signum(v) != signEntry` (main.rs:2244, 2261-2263) as one class test: with
// signEntry = signum(v0), the hit set is "the other sign, or NaN"; a NaN entry
// compares unequal to everything.
__device__ __forceinline__ int hit_class_mask(double v0) {
    if (v0 != v0) return CLS_ALL;
    return __builtin_signbit(v0) ? (CLS_POS | CLS_NAN) : (CLS_NEG | CLS_NAN);
}

// raymarchPatch's loop for a ray with no x/y motion (step.x == step.y == 0,
// main.rs:2247-2274): p.x, p.y, inRange01 and the surface depth D are loop
// invariants (p.x is never -0.0 here, so p.x + (+-0.0) == p.x bit for bit), so
// the loop carries only p.z.
//
// z_k = z_{k-1} + sz is monotone in k and so is fl(z_k - D); the class of
// (z_k - D) therefore leaves the entry class at most once (a NaN, from
// +inf - +inf, persists).  The first hit index is the number of steps that
// still "continue": counted with one compare and one add per step, no per-step
// control flow; every 8 steps the wave leaves the loop as soon as a ballot
// (__any) says no lane still continues — the per-ray `return` of the reference.
//
// With a shared z sequence (host table: every texel starts at the same z) and
// finite nonzero D, class(z - D) is POS iff z >= D (z - D is +0 when z == D)
// and NEG iff z < D, so each step is one compare against a scalar-loaded table
// entry.  Otherwise each step is fl(z - D) + a class test, exactly as written.
// First crossing of a texel's march in the monotone shared z table
// (MARCH_SEARCH).  With P(k) = [z_k < D] xor inc, P is false...false true...true
// over k (z non-decreasing: inc, P(k) = z_k >= D; non-increasing: P(k) = z_k < D),
// and P(0) false is exactly "z_0 on the entry side", so the reference's first
// hit step is the first k with P(k) (none if there is no such k < steps).
// The index is guessed from z_k ~ z_0 + k*sz and verified against the table
// (P(f-1) false, P(f) true); a failed guess falls back to a binary search, so
// the result never depends on the guess.  Returns steps for "no hit".
__device__ __forceinline__ int first_crossing(cdouble* zt, double D, double oz, double inv_sz, bool inc, int steps) {
    if ((oz < D) != inc) return steps;  // P(0): already past the surface, and z only moves away
    double g = (D - oz) * inv_sz;
    g = fmin(fmax(g, 0.0), (double)steps);  // NaN -> 0
    int f = (int)ceil(g);
    const bool ok = (f == 0 || ((zt[f - 1] < D) == inc)) && (f == steps || ((zt[f] < D) != inc));
    if (!ok) {
        int lo = 0, hi = steps;
        while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if ((zt[mid] < D) != inc) hi = mid;
            else lo = mid + 1;
        }
        f = lo;
    }
    return f;
}

template <bool COUNT>
__device__ __forceinline__ MarchResult march_axis(double D, bool inr0, double oz, double sz, int steps,
                                                  const Tables& tb) {
    MarchResult r{false, 0.0, 0, 0};
    int cnt = inr0 ? 0 : steps;
    const bool fast_ok = tb.z != nullptr && (!inr0 || (fabs(D) < INFINITY && D != 0.0));
    if (tb.zmono != 0 && __all(fast_ok)) {
        // monotone table (host-checked): locate the first crossing directly
        if (inr0) cnt = first_crossing((cdouble*)tb.z, D, oz, tb.inv_sz, tb.zmono > 0, steps);
    } else if (__any(inr0) && __all(fast_ok)) {
        cdouble* zt = (cdouble*)tb.z;
        const bool epos = !(oz < D);  // entry class POS <=> z0 >= D
        int lt = 0;                   // #steps with z_k < D
        int k = 0;
        bool all_stopped = false;
        for (; k + 8 <= steps; k += 8) {
            bool last_lt = false;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                last_lt = zt[k + u] < D;
                lt += last_lt ? 1 : 0;
            }
            const bool cont = inr0 && (epos ? !last_lt : last_lt);
            if (!__any(cont)) {
                k += 8;
                all_stopped = true;
                break;
            }
        }
        if (!all_stopped)
            for (; k < steps; ++k) lt += (zt[k] < D) ? 1 : 0;
        if (inr0) cnt = epos ? k - lt : lt;
    } else if (__any(inr0)) {
        const int keep = inr0 ? (~hit_class_mask(oz - D) & CLS_ALL) : 0;
        double z = oz;
        int k = 0;
        bool all_stopped = false;
        for (; k + 8 <= steps; k += 8) {
            bool cont = false;
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                cont = __builtin_amdgcn_class(z - D, keep);
                cnt += cont ? 1 : 0;
                z = z + sz;
            }
            if (!__any(cont)) {
                all_stopped = true;
                break;
            }
        }
        if (!all_stopped) {
            for (; k < steps; ++k) {
                const bool cont = __builtin_amdgcn_class(z - D, keep);
                cnt += cont ? 1 : 0;
                z = z + sz;
            }
        }
    }
    if (cnt < steps) {
        r.hit = true;
        r.t = t_after(tb, cnt);
        r.k = cnt;
    }
    if (COUNT) r.iters = cnt < steps ? cnt + 1 : steps;
    return r;
}

// raymarchPatchDomainM11 + raymarchPatch (main.rs:2179-2278) for one ray from
// origin o along d (any camera).
template <bool COUNT>
__device__ __forceinline__ MarchResult march(double ox, double oy, double oz, double dx, double dy,
                                             double dz, const PatchK& p, int steps, const Tables& tb) {
    const double px0 = (ox + 1.0) * 0.5;
    const double py0 = (oy + 1.0) * 0.5;
    const double mstep = 0.03;
    const double sx = dx * mstep, sy = dy * mstep, sz = dz * mstep;
    const bool inr0 = in01(px0) && in01(py0);
    if (sx == 0.0 && sy == 0.0) return march_axis<COUNT>(bil(p, px0, py0), inr0, oz, sz, steps, tb);
    // General ray (x/y motion): in-range and the surface depth change per step.
    // Per 4-step chunk the hits are collected as bits; the first set bit of the
    // first non-empty chunk is the reference's first hit.
    MarchResult r{false, 0.0, 0, 0};
    const int mask = hit_class_mask(oz - bil(p, px0, py0));
    int khit = -1;
    bool done = false;
    double x = px0, y = py0, z = oz;
    for (int k = 0; k < steps; k += 4) {
        if (__all(done)) break;
        unsigned bits = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const bool inr = in01(x) && in01(y);
            const bool h = (k + u < steps) && inr && __builtin_amdgcn_class(z - bil(p, x, y), mask);
            bits |= h ? (1u << u) : 0u;
            x = x + sx;
            y = y + sy;
            z = z + sz;
        }
        const bool first = !done && bits != 0u;
        khit = first ? k + __builtin_ctz(bits) : khit;
        done = done || first;
    }
    if (khit >= 0) {
        r.hit = true;
        r.t = t_after(tb, khit);
        r.k = khit;
    }
    if (COUNT) r.iters = khit >= 0 ? khit + 1 : steps;
    return r;
}

// Camera::calcRayOriginAndDirection (main.rs:1902-1942); s, u are the [-1,1] scales.
__device__ __forceinline__ void cam_ray(const CamK& c, double s, double u, double o[3], double d[3]) {
    if (c.type == RTM_CAMERA_ORTHOGONAL) {
        for (int k = 0; k < 3; ++k) {
            o[k] = (c.pos[k] + c.side[k] * s) + c.up[k] * u;
            d[k] = c.dir[k];
        }
    } else {
        double v[3];
        for (int k = 0; k < 3; ++k) v[k] = (c.dir[k] + c.side[k] * (s * 1.0)) + c.up[k] * (u * 1.0);
        double m = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
        double inv = 1.0 / m;
        for (int k = 0; k < 3; ++k) {
            o[k] = c.pos[k];
            d[k] = v[k] * inv;
        }
    }
}

// ---- ray-traced primitives (row f-1) ----

// One circle plane against one ray, as processRaytracingRays tests it
// (main.rs:575-604): calcRayPlane (main.rs:2398-2408), t >= 0, t <= the pixel's
// current depth zb, then |o + d*t - pos| <= radius.  NaN t passes both depth
// tests exactly as in the reference.
__device__ __forceinline__ bool plane_hit(const PlaneK& p, const double o[3], const double d[3], double zb,
                                          double& t) {
    const double denom = p.nx * d[0] + p.ny * d[1] + p.nz * d[2];  // dot(plane.n, rayDir)
    if (!(fabs(denom) > 0.0001)) return false;
    t = ((p.cx - o[0]) * p.nx + (p.cy - o[1]) * p.ny + (p.cz - o[2]) * p.nz) / denom;
    if (t < 0.0) return false;  // behind the camera
    if (t > zb) return false;   // behind a known intersection
    const double qx = (o[0] + d[0] * t) - p.cx;
    const double qy = (o[1] + d[1] * t) - p.cy;
    const double qz = (o[2] + d[2] * t) - p.cz;
    // !(sqrt(s) > radius) == !(s > r2max): sqrt is monotone and r2max is the largest s
    // whose (correctly rounded) root is <= radius, NaN and inf included (build_rt)
    return !(qx * qx + qy * qy + qz * qz > p.r2max);
}

// plane_hit for a ray from the PERSPECTIVE camera position o (RtK::persp): the
// numerator dot(pos - o, n) is the host's constant, the rest as plane_hit.
__device__ __forceinline__ bool plane_hit_persp(const PlaneK& p, const double o[3], const double d[3], double zb,
                                                double& t) {
    const double denom = p.nx * d[0] + p.ny * d[1] + p.nz * d[2];
    if (!(fabs(denom) > 0.0001)) return false;
    t = p.num / denom;
    if (t < 0.0) return false;
    if (t > zb) return false;
    const double qx = (o[0] + d[0] * t) - p.cx;
    const double qy = (o[1] + d[1] * t) - p.cy;
    const double qz = (o[2] + d[2] * t) - p.cz;
    return !(qx * qx + qy * qy + qz * qz > p.r2max);
}

// iCappedCone (main.rs:2889-2959) split in two: the t test per (ray, cylinder)
// and the hit normal, evaluated only for the cylinder that finally takes the pixel
// (trace_pixel): a cylinder hit behind a known intersection, or one a later
// primitive overrides, no longer pays the body normal's sqrt and division.  The
// normal is recomputed from the same inputs (ray, cylinder, t, part) with the same
// operations in the same order, so it has the same bits as if computed at the hit.
// part: 1 = cap at pa, 2 = cap at pb, 3 = body.
constexpr int CY_CAP_A = 1, CY_CAP_B = 2, CY_BODY = 3;

// The body normal of iCappedCone (main.rs:2950-2958): y = oaba + rdba*t, then
// normalize(baba*(baba*(oa + rd*t) - ba*rr*ra) - ba*hy*y).
__device__ __forceinline__ void icapped_body_normal(const CylK& c, const double oa[3], double oaba, double rdba,
                                                    const double rd[3], double t, double n[3]) {
    const double y = oaba + rdba * t;
    const double rra = c.rr * c.ra, hyy = c.hy * y;
    double v[3];
    for (int k = 0; k < 3; ++k) v[k] = ((oa[k] + rd[k] * t) * c.baba - c.ba[k] * rra) * c.baba - c.ba[k] * hyy;
    const double m = sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);  // normalize (main.rs:105-108)
    const double inv = 1.0 / m;
    for (int k = 0; k < 3; ++k) n[k] = v[k] * inv;
}

__device__ __forceinline__ void icapped_cap_normal(const CylK& c, int part, double n[3]) {
    const double sc = part == CY_CAP_A ? -c.isq : c.isq;
    for (int k = 0; k < 3; ++k) n[k] = c.ba[k] * sc;
}

// icapped for a ray from the PERSPECTIVE camera position (RtK::persp): oa, ob,
// oaba, obba, oc, ocba, baba*baba and k0 are the host's constants (the same
// operations in the same order), so the cap branches are uniform and only the
// terms with rd remain per pixel.  t (-1: miss) and the part hit.
__device__ __forceinline__ double icapped_persp_t(const CylK& c, const double rd[3], int& part) {
    const double rdba = rd[0] * c.ba[0] + rd[1] * c.ba[1] + rd[2] * c.ba[2];
    if (c.oaba < 0.0) {
        double w[3];
        for (int k = 0; k < 3; ++k) w[k] = c.oa[k] * rdba - rd[k] * c.oaba;
        if (w[0] * w[0] + w[1] * w[1] + w[2] * w[2] < c.ra * c.ra * rdba * rdba) {
            part = CY_CAP_A;
            return -c.oaba / rdba;
        }
    } else if (c.obba > 0.0) {
        const double t = -c.obba / rdba;
        double w[3];
        for (int k = 0; k < 3; ++k) w[k] = c.ob[k] + rd[k] * t;
        if (w[0] * w[0] + w[1] * w[1] + w[2] * w[2] < c.rb * c.rb) {
            part = CY_CAP_B;
            return t;
        }
    }
    const double ocrd = c.oc[0] * rd[0] + c.oc[1] * rd[1] + c.oc[2] * rd[2];
    const double k2 = c.bb - c.hy * rdba * rdba;
    const double k1 = c.bb * ocrd - c.hy * rdba * c.ocba;
    const double h = k1 * k1 - k2 * c.k0;
    if (h < 0.0) return -1.0;
    const double sg = c.rr >= 0.0 ? 1.0 : -1.0;
    const double t = (-k1 - sg * sqrt(h)) / (k2 * c.rr);
    const double y = c.oaba + rdba * t;
    if (y > 0.0 && y < c.baba) {
        part = CY_BODY;
        return t;
    }
    return -1.0;
}

__device__ __forceinline__ void icapped_persp_normal(const CylK& c, const double rd[3], double t, int part,
                                                     double n[3]) {
    if (part != CY_BODY) {
        icapped_cap_normal(c, part, n);
        return;
    }
    const double rdba = rd[0] * c.ba[0] + rd[1] * c.ba[1] + rd[2] * c.ba[2];
    icapped_body_normal(c, c.oa, c.oaba, rdba, rd, t, n);
}

// iCappedCone (main.rs:2889-2959) in the reference's operation order; the
// ray-independent terms (ba, baba, rr, hy, inversesqrt(baba)) come from the
// host.  t (-1: miss) and the part hit.
__device__ __forceinline__ double icapped_t(const CylK& c, const double ro[3], const double rd[3], int& part) {
    double oa[3], ob[3];
    for (int k = 0; k < 3; ++k) {
        oa[k] = ro[k] - c.pa[k];
        ob[k] = ro[k] - c.pb[k];
    }
    const double rdba = rd[0] * c.ba[0] + rd[1] * c.ba[1] + rd[2] * c.ba[2];
    const double oaba = oa[0] * c.ba[0] + oa[1] * c.ba[1] + oa[2] * c.ba[2];
    const double obba = ob[0] * c.ba[0] + ob[1] * c.ba[1] + ob[2] * c.ba[2];
    // caps
    if (oaba < 0.0) {
        double w[3];
        for (int k = 0; k < 3; ++k) w[k] = oa[k] * rdba - rd[k] * oaba;
        if (w[0] * w[0] + w[1] * w[1] + w[2] * w[2] < c.ra * c.ra * rdba * rdba) {
            part = CY_CAP_A;
            return -oaba / rdba;
        }
    } else if (obba > 0.0) {
        const double t = -obba / rdba;
        double w[3];
        for (int k = 0; k < 3; ++k) w[k] = ob[k] + rd[k] * t;
        if (w[0] * w[0] + w[1] * w[1] + w[2] * w[2] < c.rb * c.rb) {
            part = CY_CAP_B;
            return t;
        }
    }
    // body
    double oc[3];
    for (int k = 0; k < 3; ++k) oc[k] = oa[k] * c.rb - ob[k] * c.ra;
    const double ocba = oc[0] * c.ba[0] + oc[1] * c.ba[1] + oc[2] * c.ba[2];
    const double ocrd = oc[0] * rd[0] + oc[1] * rd[1] + oc[2] * rd[2];
    const double ococ = oc[0] * oc[0] + oc[1] * oc[1] + oc[2] * oc[2];
    const double bb = c.baba * c.baba;
    const double k2 = bb - c.hy * rdba * rdba;
    const double k1 = bb * ocrd - c.hy * rdba * ocba;
    const double k0 = bb * ococ - c.hy * ocba * ocba;
    const double h = k1 * k1 - k2 * k0;
    if (h < 0.0) return -1.0;
    const double sg = c.rr >= 0.0 ? 1.0 : -1.0;  // sign (main.rs:2967-2974)
    const double t = (-k1 - sg * sqrt(h)) / (k2 * c.rr);
    const double y = oaba + rdba * t;
    if (y > 0.0 && y < c.baba) {
        part = CY_BODY;
        return t;
    }
    return -1.0;
}

__device__ __forceinline__ void icapped_normal(const CylK& c, const double ro[3], const double rd[3], double t,
                                               int part, double n[3]) {
    if (part != CY_BODY) {
        icapped_cap_normal(c, part, n);
        return;
    }
    double oa[3];
    for (int k = 0; k < 3; ++k) oa[k] = ro[k] - c.pa[k];
    const double rdba = rd[0] * c.ba[0] + rd[1] * c.ba[1] + rd[2] * c.ba[2];
    const double oaba = oa[0] * c.ba[0] + oa[1] * c.ba[1] + oa[2] * c.ba[2];
    icapped_body_normal(c, oa, oaba, rdba, rd, t, n);
}

// ---- row f-4: the GL preview's SDF, the f64 restatement of oracle/rtm_oracle.c ----
// min/max: NaN-ignoring with +0 > -0 (a NaN a gives b, a NaN b gives a; a tie gives
// a unless the signs of zero decide): IEEE 754-2019 minimumNumber / maximumNumber,
// which v_min_f64 / v_max_f64 implement (one instruction each; the oracle's
// compare-and-select form gives the same value, NaN payloads aside, which never
// reach the output: a NaN distance never hits).  sign: GLSL (0 for 0 and NaN).
// (inline asm: the builtins' sNaN canonicalisation is not needed -- every operand is an
// arithmetic result -- and with them the allocator spilled 74 VGPRs in the SDF kernel)
__device__ __forceinline__ double fmax_d(double a, double b) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ __forceinline__ double fmin_d(double a, double b) {
    double r;
    asm("v_min_f64 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
// fmax_d(x, +0.0) and fmin_d(x, +0.0)
__device__ __forceinline__ double fmax0_d(double x) { return __builtin_fmaximum_num(x, 0.0); }
__device__ __forceinline__ double fmin0_d(double x) { return __builtin_fminimum_num(x, 0.0); }
// fmin_d(fmax_d(x, 0.0), 1.0)
__device__ __forceinline__ double clamp01_d(double x) {
    return __builtin_fminimum_num(__builtin_fmaximum_num(x, 0.0), 1.0);
}
// clamp01_d(x / d) for an edge parameter, d = |edge|^2 (>= 0, per-SDF constant):
// the IEEE division only where the quotient can land inside (0, 1).  x <= 0 or NaN
// gives 0 (x / d is <= 0, -0 or NaN for every d); x > 0 with x >= d, d finite and
// >= 0 gives a quotient >= 1 (+inf at d = 0), so 1.  Bit-identical to the plain
// form; a wave whose lanes all clamp skips the division sequence (the points of
// one wave's rays lie close together, so they usually clamp alike).
__device__ __forceinline__ double clamp_ratio01_d(double x, double d) {
    const bool one = (x >= d) & (d >= 0.0) & (d < __builtin_huge_val());
    if ((x > 0.0) & !one) return clamp01_d(x / d);
    return x > 0.0 ? 1.0 : 0.0;
}
__device__ __forceinline__ int gsign_i(double x) { return (int)(x > 0.0) - (int)(x < 0.0); }
__device__ __forceinline__ double dot3d(const double a[3], const double b[3]) {
    return a[0] * b[0] + a[1] * b[1] + a[2] * b[2];
}

// distanceFn0 (entry.frag:416-442): sdBox (290-298) union udTriangleSingle (312-340), - 0.2
__device__ __forceinline__ double sdf_dist(const SdfK& g, const double p[3]) {
    double dd[3], m[3];
    for (int k = 0; k < 3; ++k) {
        dd[k] = fabs(p[k] - g.box[k]) - (k == 0 ? 0.4 : 0.2);
        m[k] = fmax0_d(dd[k]);
    }
    const double d0 = fmin0_d(fmax_d(dd[0], fmax_d(dd[1], dd[2]))) + sqrt(dot3d(m, m));
    double p1[3], p2[3], p3[3];
    for (int k = 0; k < 3; ++k) {
        p1[k] = p[k] - g.v1[k];
        p2[k] = p[k] - g.v2[k];
        p3[k] = p[k] - g.v3[k];
    }
    double d1;
    // (the sum of three signs is a small integer: exact in f64 and in int)
    if (gsign_i(dot3d(g.c1, p1)) + gsign_i(dot3d(g.c2, p2)) + gsign_i(dot3d(g.c3, p3)) < 2) {
        const double s1 = clamp_ratio01_d(dot3d(g.e21, p1), g.d21);
        const double s2 = clamp_ratio01_d(dot3d(g.e32, p2), g.d32);
        const double s3 = clamp_ratio01_d(dot3d(g.e13, p3), g.d13);
        double e1[3], e2[3], e3[3];
        for (int k = 0; k < 3; ++k) {
            e1[k] = g.e21[k] * s1 - p1[k];
            e2[k] = g.e32[k] * s2 - p2[k];
            e3[k] = g.e13[k] * s3 - p3[k];
        }
        d1 = fmin_d(fmin_d(dot3d(e1, e1), dot3d(e2, e2)), dot3d(e3, e3));
    } else {
        const double dn = dot3d(g.nor, p1);
        const double a = dn * dn;
        // fmin_d(d0, a / dnor) is d0 when d0 < 0 (the quotient is >= +0 or NaN) or when
        // a > RN(RN(d0 * dnor) * (1 + 2^-40)): then a / dnor > d0 (1 + 2^-41) and the
        // rounded quotient stays above d0 (d0 > 2^-900 keeps the product normal).
        // +inf stands in for the quotient there (same fmin_d result, same bits); a
        // NaN d0 fails both tests.  A wave whose lanes all see the box closer skips
        // the division sequence.
        const bool box_wins = (d0 < 0.0) | ((d0 > 0x1p-900) & (a > (d0 * g.dnor) * (1.0 + 0x1p-40)));
        if (box_wins)
            d1 = __builtin_huge_val();
        else
            d1 = a / g.dnor;
    }
    double d2 = fmin_d(d0, d1);
    d2 -= 0.2;
    return d2;
}

// Both sBox calls of one trace (entry.frag:85-110, 857-859) with txx =
// translate(-centre), sharing the per-ray m = 1/rd (hoisted by the caller).
// The second call's ray is -rd: 1/(-x) == -(1/x), (-m)*roo == -(m*roo) and
// |-m| == |m| exactly in IEEE arithmetic, so its t1 = -n' - k' is n - k bit for
// bit.  Returns false on the first call's miss (tN > tF || tF < 0).
__device__ __forceinline__ bool sdf_slabs(const double ro[3], const double m[3], const double am[3], const SdfK& g,
                                          double& tIn, double& tOut) {
    double t1[3], t2[3], u1[3];
    for (int k = 0; k < 3; ++k) {
        const double roo = ro[k] - g.ac[k];
        const double n = m[k] * roo;
        const double kk = am[k] * g.ae[k];
        t1[k] = -n - kk;
        t2[k] = -n + kk;
        u1[k] = n - kk;
    }
    const double tN = fmax_d(fmax_d(t1[0], t1[1]), t1[2]);
    const double tF = fmin_d(fmin_d(t2[0], t2[1]), t2[2]);
    tIn = (tN > tF || tF < 0.0) ? -1.0 : tN;
    tOut = -fmax_d(fmax_d(u1[0], u1[1]), u1[2]);
    return tIn >= 0.0;
}

// The implicit-surface branch of bvhProcessLeafHit (entry.frag:842-905):
// t of the hit or -1, and the sdNormalFast normal.  m = 1/rd, am = |m|.
// NEAR (the render kernels): zb is the pixel's nearest surface so far, and the
// caller accepts a hit only at t < zb (entry.frag:908-917).  t starts at the AABB
// entry tIn and only grows (a step adds a distance >= 0.03), so once t >= zb neither
// a later hit nor a miss can change the pixel: the trace stops there and reports a
// miss -- the same pixel, without the steps (and the normal) that could not count.
// The counting kernel (rtm_render_stats) keeps every step the shader takes.
template <bool NEAR = false>
__device__ __forceinline__ double sdf_trace(const SdfK& g, const double ro[3], const double rd[3], const double m[3],
                                            const double am[3], double n[3], uint32_t& evals, double zb = 0.0) {
    double tIn, tOut;
    if (!sdf_slabs(ro, m, am, g, tIn, tOut)) return -1.0;
    double t = tIn;
    bool hit = false;
    for (int step = 0; step < g.steps; ++step) {
        if (NEAR && !(t < zb)) break;  // (a NaN t never hits either)
        const double p[3] = {ro[0] + rd[0] * t, ro[1] + rd[1] * t, ro[2] + rd[2] * t};
        const double dist = sdf_dist(g, p);
        ++evals;
        if (dist < 0.03) {
            hit = true;
            break;
        }
        if (t > tOut) break;
        t += dist;
    }
    if (!hit) return -1.0;
    evals += 4;
    const double p[3] = {ro[0] + rd[0] * t, ro[1] + rd[1] * t, ro[2] + rd[2] * t};
    const double h = 0.001;
    const double ks[4][3] = {{1.0, -1.0, -1.0}, {-1.0, -1.0, 1.0}, {-1.0, 1.0, -1.0}, {1.0, 1.0, 1.0}};
    double tap[4];
    for (int j = 0; j < 4; ++j) {
        const double q[3] = {p[0] + ks[j][0] * h, p[1] + ks[j][1] * h, p[2] + ks[j][2] * h};
        tap[j] = sdf_dist(g, q);
    }
    double v[3];
    for (int k = 0; k < 3; ++k) v[k] = ((ks[0][k] * tap[0] + ks[1][k] * tap[1]) + ks[2][k] * tap[2]) + ks[3][k] * tap[3];
    const double inv = 1.0 / sqrt(dot3d(v, v));
    for (int k = 0; k < 3; ++k) n[k] = v[k] * inv;
    return t;
}

// The ray-traced part of one eye pixel: planes, then cylinders, in scene order
// (main.rs:573-638), then the row f-4 SDFs.  zb is the depth after the sphere
// rasterize; kind/rid/t/n are updated in place when a primitive takes the pixel.
// A hit's scene id indexes the frame's shading tables (a.shade, rt->pl / cy, sdf->s
// by id, as renderColorImage indexes the scene's vectors, main.rs:748, 773, 791).  The
// host validated every id against its table (rtm_api.cpp validate_scene), and the
// kernels check it again where the id is taken -- a wave-uniform (scalar) id against
// the frame's count: an id past the table is counted in `oob` (rtm_ctx_oob_reads) and
// replaced by 0, so no id-indexed read can leave its table.
__device__ __forceinline__ int checked_id(int id, int n, bool& oob) {
    if ((unsigned)id < (unsigned)n) return id;
    oob = true;
    return 0;
}

struct RtHit {
    int kind;  // 0 none, 1 sphere, 2 circle plane, 3 capped cylinder, 4 SDF
    int id;
    double t;
    double n[3];
};

template <bool NEAR = false>
__device__ __forceinline__ void trace_sdfs(const SdfTabK* __restrict__ sdf, const double o[3], const double d[3],
                                           double zb, RtHit& hit, uint32_t& evals, bool& oob) {
    const int ns = sdf->n;
    const double m[3] = {1.0 / d[0], 1.0 / d[1], 1.0 / d[2]};
    const double am[3] = {fabs(m[0]), fabs(m[1]), fabs(m[2])};
    for (int i = 0; i < ns; ++i) {
        double n[3];
        const double t = sdf_trace<NEAR>(sdf->s[i], o, d, m, am, n, evals, zb);
        if (!(t > 0.0) || !(t < zb)) continue;  // the shader's acceptance (entry.frag:908-917)
        hit.kind = 4;
        hit.id = checked_id(sdf->s[i].id, ns, oob);
        hit.t = t;
        hit.n[0] = n[0];
        hit.n[1] = n[1];
        hit.n[2] = n[2];
        zb = t;
    }
}

// Per-wave cull of the ray-traced primitives under a PERSPECTIVE eye (all lanes
// active).  The wave's rays (one row, columns [xb, xe]) leave the camera origin
// inside a cone: axis the bisector of its two end rays, half-angle theta to
// them.  Every hit a primitive can report lies within a bounding sphere (C, R):
//   circle plane: |o + d t - pos| <= radius            -> (pos, radius)
//   capped cone:  on the frustum between pa and pb     -> ((pa+pb)/2, |ba|/2 + max|r|)
// and only at t >= 0 (both tests reject t < 0), so a primitive whose inflated
// sphere lies outside the cone -- angle(axis, C - o) > theta + asin(R/|C - o|)
// -- cannot be hit by any ray of the wave.  Inflation (R*1.001 + 1e-7, cosine
// margin 1e-7) dwarfs the f64 rounding of the exact tests.  Kept (never culled):
// non-finite data (every comparison is false), origins inside a sphere, and
// near-cylinders (|rb - ra| < 1e-3 max|r|: the cone formula's cancellation, main.rs:2924-2936).
struct RayCone {
    double ax[3];  // unit axis
    double ct, st; // cos / sin of the half-angle
};

__device__ __forceinline__ RayCone ray_cone(const CamK& c, int xb, int xe, int yi, int W, int H) {
    const double s0 = ndc(xb, W), s1 = ndc(xe, W), u = ndc(yi, H);
    double n0[3], n1[3];
    RayCone k;
    double m0 = 0.0, m1 = 0.0;
    for (int j = 0; j < 3; ++j) {
        n0[j] = (c.dir[j] + c.side[j] * s0) + c.up[j] * u;
        n1[j] = (c.dir[j] + c.side[j] * s1) + c.up[j] * u;
        m0 += n0[j] * n0[j];
        m1 += n1[j] * n1[j];
    }
    m0 = 1.0 / sqrt(m0);
    m1 = 1.0 / sqrt(m1);
    double ma = 0.0;
    for (int j = 0; j < 3; ++j) {
        n0[j] *= m0;
        n1[j] *= m1;
        k.ax[j] = n0[j] + n1[j];
        ma += k.ax[j] * k.ax[j];
    }
    ma = 1.0 / sqrt(ma);
    double ct = 0.0;
    for (int j = 0; j < 3; ++j) {
        k.ax[j] *= ma;
        ct += k.ax[j] * n0[j];
    }
    k.ct = fmin(ct, 1.0);
    k.st = sqrt(1.0 - k.ct * k.ct);
    return k;
}

// The cone of an 8 x 8 pixel block's rays ([x0, x1] x [y0, y1]): the rays of a rectangle
// of pixels lie in the convex hull of its four corner rays, so a cone (half-angle below
// 90 degrees, a convex set) holding the four holds them all.  Axis: the normalised sum of
// the corners' unit rays; half-angle: the largest angle to a corner.
__device__ __forceinline__ RayCone ray_cone_block(const CamK& c, int x0, int x1, int y0, int y1, int W, int H) {
    const double sx[2] = {ndc(x0, W), ndc(x1, W)}, uy[2] = {ndc(y0, H), ndc(y1, H)};
    double n[4][3];
    RayCone k;
    double sum[3] = {0.0, 0.0, 0.0};
    for (int q = 0; q < 4; ++q) {
        double m = 0.0;
        for (int j = 0; j < 3; ++j) {
            n[q][j] = (c.dir[j] + c.side[j] * sx[q & 1]) + c.up[j] * uy[q >> 1];
            m += n[q][j] * n[q][j];
        }
        m = 1.0 / sqrt(m);
        for (int j = 0; j < 3; ++j) {
            n[q][j] *= m;
            sum[j] += n[q][j];
        }
    }
    const double ma = 1.0 / sqrt(sum[0] * sum[0] + sum[1] * sum[1] + sum[2] * sum[2]);
    for (int j = 0; j < 3; ++j) k.ax[j] = sum[j] * ma;
    double ct = 1.0;
    for (int q = 0; q < 4; ++q) ct = fmin(ct, k.ax[0] * n[q][0] + k.ax[1] * n[q][1] + k.ax[2] * n[q][2]);
    k.ct = ct;
    k.st = sqrt(1.0 - k.ct * k.ct);
    return k;
}

// Bounding sphere of primitive slot l (l < 16: circle plane l; 16 + i: cylinder i);
// cullable false for an empty slot and for near-cylinders.
__device__ __forceinline__ void rt_bound(const RtK* __restrict__ rt, int l, double C[3], double& R, bool& cullable) {
    C[0] = C[1] = C[2] = 0.0;
    R = 0.0;
    cullable = false;
    if (l < rt->n_pl) {
        const PlaneK& p = rt->pl[l];
        C[0] = p.cx;
        C[1] = p.cy;
        C[2] = p.cz;
        R = p.radius;
        cullable = true;
    } else if (l >= 16 && l - 16 < rt->n_cy) {
        const CylK& q = rt->cy[l - 16];
        const double rmax = fmax(fabs(q.ra), fabs(q.rb));
        for (int j = 0; j < 3; ++j) C[j] = (q.pa[j] + q.pb[j]) * 0.5;
        R = sqrt(q.baba) * 0.5 + rmax;
        cullable = fabs(q.rb - q.ra) >= 1e-3 * rmax;
    }
}

__device__ __forceinline__ bool cone_culls(const RayCone& k, const CamK& c, const double C[3], double R, bool cullable) {
    const double Ri = R * 1.001 + 1e-7;
    double w[3], L2 = 0.0, aw = 0.0;
    for (int j = 0; j < 3; ++j) {
        w[j] = C[j] - c.pos[j];
        L2 += w[j] * w[j];
        aw += k.ax[j] * w[j];
    }
    const double L = sqrt(L2);
    const double sb = Ri / L;                          // sin(beta)
    const double cb = sqrt(fmax(1.0 - sb * sb, 0.0));
    const double thr = k.ct * cb - k.st * sb - 1e-7;   // cos(theta + beta), less the margin
    return cullable & (L > Ri) & (sb < 1.0) & (aw < thr * L);
}

// The capsule bound of a capped cone (pa, pb, R = max|r|: every point of its caps and
// body lies within R of the segment pa-pb), against the wave's ray cone: no ray of the
// cone meets the capsule when gamma, the least angle between the cone's axis and the
// directions (from the apex) of the segment's points, exceeds theta + beta, beta =
// asin(Ri / dmin) the angular radius of the capsule's cross-section at its least
// distance dmin from the apex.  gamma: the nearer endpoint, or -- when the axis's
// projection on the plane of the segment's directions falls on the arc between them
// -- the angle to that plane.  The same inflation and margins as cone_culls; a long,
// thin cylinder (main()'s scene: |ba| = 10, R = 0.3) is bounded 10x tighter than by
// its sphere.  Non-finite data and a capsule holding the apex are kept.
//
// Everything but the cone's axis and angle is the slot's own (the apex is the camera
// position): CullK holds those terms, computed once per slot and frame (cull_prepare:
// by 32 lanes into LDS in rt_cull_kernel), and cull_test is what remains per wave.
struct CullK {
    double w[3], L, sb, cb;      // bounding sphere: C - apex, |C - apex|, sin / cos of its angular radius
    double u0[3], u1[3], nh[3];  // capsule: unit directions of its ends, the unit normal of their plane
    double csb, ccb;             // sin / cos of the capsule's angular radius at dmin
    int32_t sph, cap, has_n, pad;
};

__device__ __forceinline__ void cull_prepare(const RtK* __restrict__ rt, int l, const CamK& c, CullK& q) {
    double C[3], R;
    bool cullable;
    rt_bound(rt, l, C, R, cullable);
    const double Ri = R * 1.001 + 1e-7;
    double L2 = 0.0;
    for (int j = 0; j < 3; ++j) {
        q.w[j] = C[j] - c.pos[j];
        L2 += q.w[j] * q.w[j];
    }
    q.L = sqrt(L2);
    q.sb = Ri / q.L;  // sin(beta)
    q.cb = sqrt(fmax(1.0 - q.sb * q.sb, 0.0));
    q.sph = cullable & (q.L > Ri) & (q.sb < 1.0);
    q.cap = 0;
    q.has_n = 0;
    q.csb = q.ccb = 0.0;
    for (int j = 0; j < 3; ++j) q.u0[j] = q.u1[j] = q.nh[j] = 0.0;
    if (l >= 16 && l - 16 < rt->n_cy) {
        const CylK& cy = rt->cy[l - 16];
        const double Rc = fmax(fabs(cy.ra), fabs(cy.rb)) * 1.001 + 1e-7;
        double p0[3], p1[3], e[3], pe = 0.0, ee = 0.0;
        for (int j = 0; j < 3; ++j) {
            p0[j] = cy.pa[j] - c.pos[j];
            e[j] = cy.pb[j] - cy.pa[j];
            pe += p0[j] * e[j];
            ee += e[j] * e[j];
        }
        const double t = ee > 0.0 ? fmin(fmax(-pe / ee, 0.0), 1.0) : 0.0;
        double q2 = 0.0, l0 = 0.0, l1 = 0.0;
        for (int j = 0; j < 3; ++j) {
            p1[j] = p0[j] + e[j];
            const double qj = p0[j] + e[j] * t;
            q2 += qj * qj;
            l0 += p0[j] * p0[j];
            l1 += p1[j] * p1[j];
        }
        const double dmin = sqrt(q2);
        l0 = sqrt(l0);
        l1 = sqrt(l1);
        // (the apex inside the capsule, and non-finite data, keep the slot)
        if (dmin > Rc && __builtin_isfinite(dmin) && __builtin_isfinite(l0) && __builtin_isfinite(l1)) {
            q.csb = Rc / dmin;
            q.ccb = sqrt(fmax(1.0 - q.csb * q.csb, 0.0));
            for (int j = 0; j < 3; ++j) {
                q.u0[j] = p0[j] / l0;
                q.u1[j] = p1[j] / l1;
            }
            double n[3] = {q.u0[1] * q.u1[2] - q.u0[2] * q.u1[1], q.u0[2] * q.u1[0] - q.u0[0] * q.u1[2],
                           q.u0[0] * q.u1[1] - q.u0[1] * q.u1[0]};
            const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
            if (nn > 1e-12) {  // (else the arc is a point within 1e-12 rad: its endpoints decide)
                for (int j = 0; j < 3; ++j) q.nh[j] = n[j] / nn;
                q.has_n = 1;
            }
            q.cap = cullable;
        }
    }
}

// Slot culled for the wave's cone: its bounding sphere (cone_culls' test) or, a cylinder,
// its capsule.  NaN anywhere compares false: kept.
__device__ __forceinline__ bool cull_test(const RayCone& k, const CullK& q) {
    if (q.sph) {
        const double aw = k.ax[0] * q.w[0] + k.ax[1] * q.w[1] + k.ax[2] * q.w[2];
        const double thr = k.ct * q.cb - k.st * q.sb - 1e-7;  // cos(theta + beta), less the margin
        if (aw < thr * q.L) return true;
    }
    if (!q.cap) return false;
    const double thr = k.ct * q.ccb - k.st * q.csb - 1e-7;
    const double c0 = k.ax[0] * q.u0[0] + k.ax[1] * q.u0[1] + k.ax[2] * q.u0[2];
    const double c1 = k.ax[0] * q.u1[0] + k.ax[1] * q.u1[1] + k.ax[2] * q.u1[2];
    double cg = c0 > c1 ? c0 : c1;  // (cos of the angle to the nearer endpoint; a NaN axis: both NaN, kept)
    if (q.has_n) {
        const double an = k.ax[0] * q.nh[0] + k.ax[1] * q.nh[1] + k.ax[2] * q.nh[2];
        double ap[3];
        for (int j = 0; j < 3; ++j) ap[j] = k.ax[j] - an * q.nh[j];
        // (u0 x ap).n and (ap x u1).n: the projection between the endpoints (a loose
        // bound: counting a projection just outside the arc only raises cg)
        const double w0 = (q.u0[1] * ap[2] - q.u0[2] * ap[1]) * q.nh[0] + (q.u0[2] * ap[0] - q.u0[0] * ap[2]) * q.nh[1] +
                          (q.u0[0] * ap[1] - q.u0[1] * ap[0]) * q.nh[2];
        const double w1 = (ap[1] * q.u1[2] - ap[2] * q.u1[1]) * q.nh[0] + (ap[2] * q.u1[0] - ap[0] * q.u1[2]) * q.nh[1] +
                          (ap[0] * q.u1[1] - ap[1] * q.u1[0]) * q.nh[2];
        if (!(w0 < -1e-6) && !(w1 < -1e-6)) {
            const double cp = sqrt(fmax(1.0 - an * an, 0.0));
            cg = cp > cg ? cp : cg;
        }
    }
    return cg < thr;
}

// Slot l culled for the wave's cone (all terms per call: the lane-parallel cull below).
__device__ __forceinline__ bool rt_culls(const RtK* __restrict__ rt, int l, const RayCone& k, const CamK& c) {
    CullK q;
    cull_prepare(rt, l, c, q);
    return cull_test(k, q);
}

// Lane-parallel form inside a kernel (all lanes active): lane l tests slot l.
__device__ __forceinline__ uint32_t rt_wave_mask(const RtK* __restrict__ rt, const CamK& c, int xb, int xe, int yi,
                                                 int W, int H, int ye = -1) {
    // (ye >= 0: the wave is the block of rows [yi, ye])
    const RayCone k = ye >= 0 ? ray_cone_block(c, xb, xe, yi, ye, W, H) : ray_cone(c, xb, xe, yi, W, H);
    const int l = threadIdx.x & 63;
    const bool culled = rt_culls(rt, l, k, c);
#if defined(RTM_TEST_REVERT_SLOT_MASKS)  // (tools/bounds_demo.sh only: the pre-dfafeba mask, every slot set)
    return ~(uint32_t)__ballot(culled);
#else
    const bool exists = l < 16 ? l < rt->n_pl : l - 16 < rt->n_cy;
    return (uint32_t)__ballot(exists & !culled);  // lane i < 16: plane i; 16 + i: cylinder i
#endif
}

// The slot bits of a frame's existing primitives (bits 0-15 planes, 16-31 cylinders):
// the masks' producers (rt_slots as the default, rt_wave_mask, rt_cull_wave) set no
// other bit; rt_exist is the exact set trace_pixel checks them against.
__device__ __forceinline__ uint32_t rt_exist(int n_pl, int n_cy) {
    return ((1u << n_pl) - 1u) | (((1u << n_cy) - 1u) << 16);
}
__device__ __forceinline__ uint32_t rt_slots(int n_pl, int n_cy) {
#if defined(RTM_TEST_REVERT_SLOT_MASKS)
    return ~0u;
#else
    return rt_exist(n_pl, n_cy);
#endif
}

// The primitives of `mask` (wave-uniform; bits 0-15 planes, 16-31 cylinders, set only
// for existing slots: rt_slots, or rt_wave_mask / rt_cull_wave, which also clear the
// primitives no ray of the wave can hit), in the reference's order (main.rs:575-642):
// planes by index, then cylinders by index.  A skipped primitive is one no ray of the
// wave can hit, so zb and the hit are what the full loop would leave.
// PERSP: the rays start at the PERSPECTIVE camera position and rt holds its
// origin-only constants (RtK::persp; a compile-time choice, so the kernel carries
// one path).
// A mask bit of a slot the frame does not fill (a producer's bug: no producer sets
// one) is counted in `oob` and dropped, so the walk never visits an empty slot.
template <bool PERSP>
__device__ __forceinline__ void trace_pixel(const RtK* __restrict__ rt, const double o[3], const double d[3],
                                            double& zb_io, RtHit& hit, uint32_t mask, bool& oob) {
    const uint32_t exist = rt_exist(rt->n_pl, rt->n_cy);
    if (mask & ~exist) {  // (wave-uniform)
        oob = true;
        mask &= exist;
    }
    double zb = zb_io;
    constexpr bool persp = PERSP;
    for (uint32_t m = mask & 0xFFFFu; m; m &= m - 1u) {
        const int i = __builtin_ctz(m);
        double t;
        if (persp ? plane_hit_persp(rt->pl[i], o, d, zb, t) : plane_hit(rt->pl[i], o, d, zb, t)) {
            hit.kind = 2;
            hit.id = checked_id(rt->pl[i].id, rt->n_pl, oob);
            hit.t = t;
            zb = t;
        }
    }
    int cyi = -1, cypart = 0;  // the cylinder that takes the pixel: its normal afterwards
    for (uint32_t m = mask >> 16; m; m &= m - 1u) {
        const int i = __builtin_ctz(m);
        int part = 0;
        const double t = persp ? icapped_persp_t(rt->cy[i], d, part) : icapped_t(rt->cy[i], o, d, part);
        if (t < 0.0) continue;  // behind the camera (and misses)
        if (t > zb) continue;   // behind a known intersection
        hit.kind = 3;
        hit.id = checked_id(rt->cy[i].id, rt->n_cy, oob);
        hit.t = t;
        cyi = i;
        cypart = part;
        zb = t;
    }
    if (cyi >= 0) {
        if (persp) icapped_persp_normal(rt->cy[cyi], d, hit.t, cypart, hit.n);
        else icapped_normal(rt->cy[cyi], o, d, hit.t, cypart, hit.n);
    }
    zb_io = zb;
}

// ---- statistics (rtm_render_stats only; never in the timed kernels) ----
__device__ __forceinline__ unsigned long long wave_sum(unsigned long long v) {
    for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
    return v;
}
__device__ __forceinline__ void stat_add(unsigned long long* ctr, unsigned long long v) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, v);
}

struct ShadowCounts {
    unsigned long long tests = 0, iters = 0, hits = 0, inrange = 0;
};

// One shadow-map texel (any shadow camera): shadow viewport rasterize (face BACK,
// main.rs:1569) then processRaymarchingRays (main.rs:1571) with a strict-min
// update (main.rs:559).  [xb, xe] x yw is the pixel set the caller's wave
// covers (for the per-wave cull).
template <bool COUNT>
__device__ __forceinline__ double shadow_texel(const ShadowPart& a, int xi, int yi, int xb, int xe, int yw,
                                               ShadowCounts& c, int& code) {
    double zb = INFINITY;
    code = -1;  // +INF
    if (!(a.flags & RTM_FLAG_NO_SHADOW_RASTER) && union_may_cover(a, xb, xe, yw, yw)) {
        const double x = a.tab.nx[xi];
        const double y = a.tab.ny[yi];
        for (int i = 0; i < a.n_spheres; ++i) {
            if (!may_cover(a.sph[i], xb, xe, yw)) continue;
            double h;
            if (cover(a.sph[i], x, y, h)) {
                if (COUNT) ++c.tests;
                const double depth = a.sph[i].z + h * a.sph[i].r;  // EnumFace::BACK (main.rs:243)
                if (depth < zb) {
                    zb = depth;
                    code = a.steps + i;
                }
            }
        }
    }
    if (!(a.flags & RTM_FLAG_NO_MARCH) && a.n_patches > 0) {
        if (a.tab.d0) {
            // separable axis-aligned shadow camera: the texel's domain-mapped start
            // and surface depth come from per-column / per-row tables
            const double py = a.tab.py[yi];
            const bool inr0 = a.tab.ok[xi] && a.tab.ok[a.W + yi];
            const double oz = a.tab.z[0];
            const double sz = a.cam.dir[2] * 0.03;
            for (int k = 0; k < a.n_patches; ++k) {
                const double D = a.tab.d0[k * a.W + xi] + a.tab.dd[k * a.W + xi] * py;
                MarchResult m = march_axis<COUNT>(D, inr0, oz, sz, a.steps, a.tab);
                if (COUNT) {
                    c.iters += m.iters;
                    c.hits += m.hit;
                    c.inrange += inr0;
                }
                if (m.hit && m.t < zb) {
                    zb = m.t;
                    code = m.k;
                }
            }
        } else {
            double o[3], d[3];
            cam_ray(a.cam, a.tab.nx[xi], a.tab.ny[yi], o, d);
            for (int k = 0; k < a.n_patches; ++k) {
                MarchResult m = march<COUNT>(o[0], o[1], o[2], d[0], d[1], d[2], a.patch[k], a.steps, a.tab);
                if (COUNT) {
                    c.iters += m.iters;
                    c.hits += m.hit;
                    c.inrange += in01((o[0] + 1.0) * 0.5) && in01((o[1] + 1.0) * 0.5);
                }
                if (m.hit && m.t < zb) {
                    zb = m.t;
                    code = m.k;
                }
            }
        }
    }
    return zb;
}
template <bool COUNT>
__device__ __forceinline__ double shadow_texel(const ShadowPart& a, int xi, int yi, int xb, int xe, int yw,
                                               ShadowCounts& c) {
    int code;
    return shadow_texel<COUNT>(a, xi, yi, xb, xe, yw, c, code);
}

// Value of a coded shadow-map texel (ShadowPart::smap_fmt != SMAP_F64): what the
// shadow pass computed there, recomputed from its code with the writer's
// operations (t_after; cover + the BACK-face depth of the lean and generic
// tiles), so the same bits.
// The code of texel (tx, ty) of a coded map: its block byte, or with span records
// (rtm_kernels.h) the span's record, both loaded together.
__device__ __forceinline__ uint32_t smap_code(const ShadowPart& sh, const void* __restrict__ map, int tx, int ty) {
    const int64_t e = smap_code_index(tx, ty, sh.smap_bw);
    if (sh.smap_fmt != SMAP_U8) return (uint32_t)((const uint16_t*)map)[e];
    const uint32_t dense = (uint32_t)((const uint8_t*)map)[e];
    if (!sh.smap_spans) return dense;
    const uint32_t rec = ((const uint32_t*)((const uint8_t*)map + smap_span_offset(sh.W, sh.H)))
        [smap_span_index(tx, ty, sh.smap_bw)];
    const uint32_t run = (uint32_t)(ty & (SPAN_ROWS - 1)) < ((rec >> 16) & 0xFFu) ? rec & 0xFFu : (rec >> 8) & 0xFFu;
    return rec == SPAN_DENSE ? dense : run;
}

__device__ __forceinline__ double smap_decode(const ShadowPart& sh, const void* __restrict__ map, int tx, int ty) {
    const uint32_t code = smap_code(sh, map, tx, ty);
    const uint32_t inf = sh.smap_fmt == SMAP_U8 ? 0xFFu : 0xFFFFu;
    if (code == inf) return INFINITY;
    if ((int)code < sh.steps) return t_after(sh.tab, (int)code);
    if ((int)code - sh.steps >= sh.n_spheres) {  // (no writer stores such a code: counted, read as +INF)
        note_oob();
        return INFINITY;
    }
    const RasterSphereK& sp = sh.sph[(int)code - sh.steps];
    const double pa = ((sh.tab.nx[tx] - sp.cx) * sp.n) / sp.m;
    const double pb = ((sh.tab.ny[ty] - sp.cy) * sp.n) / sp.m;
    const double d = sqrt(pa * pa + pb * pb);
    const double h = sqrt(1.0 - d * d);
    return sp.z + h * sp.r;
}

// smap_decode for the eye pass's lookups (the active lanes of a wave, each with
// its own texel): the code and the texel's NDC coordinates are loaded together
// (no chain of dependent loads), and sphere codes are resolved one sphere at a
// time with that sphere's constants as wave-uniform (scalar) values instead of a
// per-lane indexed load of them.  Same operations as smap_decode: same bits.
// oob: set when the code names no sphere of the frame (reported by the caller after its
// last load, see eye_tile).
__device__ __forceinline__ double smap_decode_wave(const ShadowPart& sh, const void* __restrict__ map, int tx, int ty,
                                                   bool& oob) {
    const bool u8 = sh.smap_fmt == SMAP_U8;
    const uint32_t code = smap_code(sh, map, tx, ty);
    const double xs = sh.tab.nx[tx];
    const double ys = sh.tab.ny[ty];
    const uint32_t inf = u8 ? 0xFFu : 0xFFFFu;
    const int steps = sh.steps;
    double v = INFINITY;
    if (code != inf && (int)code < steps) v = t_after(sh.tab, (int)code);
    int si = (code != inf && (int)code >= steps) ? (int)code - steps : -1;
    if (si >= sh.n_spheres) {  // (no writer stores such a code: counted, read as +INF)
        oob = true;
        si = -1;
    }
    while (__any(si >= 0)) {
        const unsigned long long b = __ballot(si >= 0);
        const int i = __builtin_amdgcn_readfirstlane(__shfl(si, __builtin_ctzll(b)));
        const RasterSphereK& sp = sh.sph[i];
        if (si == i) {
            const double pa = ((xs - sp.cx) * sp.n) / sp.m;
            const double pb = ((ys - sp.cy) * sp.n) / sp.m;
            const double d = sqrt(pa * pa + pb * pb);
            const double h = sqrt(1.0 - d * d);
            v = sp.z + h * sp.r;
            si = -1;
        }
    }
    return v;
}

// Generic shadow tile: 64 x TILE_Y texels, one wave per row.
template <bool COUNT>
__device__ __forceinline__ void shadow_tile_generic(const ShadowPart& a, double* __restrict__ smap, int bx, int by,
                                                    StatsK* __restrict__ st) {
    const int xb = bx * TILE_X;
    const int xi = xb + (threadIdx.x & (TILE_X - 1));
    const int yi = __builtin_amdgcn_readfirstlane(by * TILE_Y + (threadIdx.x >> 6));  // wave-uniform row
    ShadowCounts c;
    if (xi < a.W && yi < a.H) {
        int code;
        const double zb = shadow_texel<COUNT>(a, xi, yi, xb, xb + TILE_X - 1, yi, c, code);
        if (COUNT || a.smap_fmt == SMAP_F64)
            smap[(int64_t)yi * a.W + xi] = zb;
        else if (a.smap_fmt == SMAP_U8)
            ((uint8_t*)smap)[smap_code_index(xi, yi, a.smap_bw)] = (uint8_t)code;  // -1: 0xFF = +INF
        else
            ((uint16_t*)smap)[smap_code_index(xi, yi, a.smap_bw)] = (uint16_t)code;
    }
    if (COUNT) {
        stat_add(&st->shadow_sphere_tests, c.tests);
        stat_add(&st->march_iterations, c.iters);
        stat_add(&st->march_hits, c.hits);
        stat_add(&st->march_in_range, c.inrange);
    }
}

typedef float f32x4 __attribute__((ext_vector_type(4)));

// Tile row of workgroup row b (of n) with the rows [h0, h1] that the spheres'
// pixel-range union reaches dispatched first: their waves carry the raster work,
// and started last they would be the kernel's tail.
__device__ __forceinline__ int hot_rows_first(int b, int n, int h0, int h1) {
    if (h0 > h1) return b;
    const int nh = h1 - h0 + 1;
    if (b < nh) return h0 + b;
    const int r = b - nh;
    return r < h0 ? r : r + nh;
}

// Batched forms: frame blockIdx.z of a BatchFrame table in device memory.  The
// table is read through the constant address space, so its fields become scalar
// loads exactly like kernel arguments.
using CBatch = const __attribute__((address_space(4))) BatchFrame;

// The coded shadow tile (every coded map whose march has host-built records,
// rtm_kernels.h; launch_coded): a wave owns a strip of 128 columns x 16 rows (lane l:
// columns xb + 2l, +1), stored as four 128 x 4 blocks of the coded map.
//
// The first-crossing check of one texel (code_check): with the host's records
// (ZRecK / ColRecK / RowRecK),
//   D = d0 + dd*py (exact, 2 f64 ops); "D finite and nonzero" (one class test);
//   f = ceil(clamp(g0 + g1*py, 1, steps)) (an f32 index guess, checked below; ceil,
//     not trunc(x) + 1: an x that rounds to an integer in f32 is common and would be
//     mis-guessed by one);
//   one LDS record T[f] = (z_{f-1}, z_f, t_f), and with P(z) = INC ? !(z < D) : (z < D)
//   okA = !P(z_{f-1}), okB = P(z_f), entry = !P(z_0)   (P monotone over the table)
//   hit  = fastD & okA & okB & f < steps   -> code f (t_f), else NONE (+INF)
//   slow = !fastD | (entry & !(okA & okB))  -> the check cannot decide: exact march_axis
//
// Monotone codes (the per-strip shortcut).  Down a column, py rises (or falls) with
// the row and D = fl(d0 + fl(dd*py)) is monotone in py (rounding is monotone), so D is
// monotone down the strip.  For a fixed D the reference's answer is: NONE when the
// entry test fails, else the first k with P(z_k) (NONE if there is none before
// `steps`) -- a monotone function of D on each side of the entry threshold.  So when
// both ends of a column's strip are decided by the check, lie on the same side of the
// entry threshold and have D of the same sign (every D between is then finite and
// nonzero), the column's 16 codes are a monotone sequence from the top code to the
// bottom code: equal end codes fill the column; different ones are located by a
// binary search over the rows (4 checks) for the first row whose code differs, and
// when that row's code is the bottom code the column has one boundary (the usual
// case: a code changes every ~100 rows at 3840x2160).  A wave takes the shortcut when
// every lane's columns qualify and every search check decides; otherwise the wave
// checks every texel (the fallback, which is also the path for strips with rows that
// do not march).  Per 16 x 2 texels of a lane: 4 checks, + 4 per column with a boundary.
//
// Spheres (PART 0 / 2, strips meeting the frame's sphere box) are rasterized after the
// march codes, block by block (4 rows): the strict minimum over the spheres in scene
// order, then the march wins only where its t is strictly below it (main.rs:559) --
// the reference's rasterize-then-march order.
// Needs 1 <= steps <= CODED_MAX_STEPS (LDS) when marching, and a coded map.
constexpr int CODED_MAX_STEPS = 1023;  // (steps + 1) * 32 B <= 32 KiB of LDS
constexpr int CODED_ROWS = 16;          // rows per strip (a wave's rows in PART 0 / 1)
constexpr int CODED_TILE_ROWS = CODED_ROWS * TILE_Y;
// PART 2 (the sphere strips of a split launch) runs 4-row waves, a strip per
// workgroup: the sphere raster is most of its work and 16-row waves left it with too
// few waves to hide its latency (2,800 per 8-frame launch at config 3: 37.9 instead of
// 24 us, profiles/r04_v3_*); its march codes take the per-texel check.
template <int PART>
constexpr int coded_wave_rows = PART == 2 ? 4 : CODED_ROWS;
// PART 1 waves loop over P1_STRIPS consecutive 16-row strips (the prologue -- frame
// header, the LDS table fill and its barrier, the row records -- paid once per wave).
// 4 strips (a wave per 128 x 64 texels, a quarter of the waves): config 3 340 -> 348,
// config 2 333 -> 341 Gpix/s in the 4-lane frame, same box, interleaved (the one-lane
// raster-free launch is slower, 27.5 -> 30.9 us per 8 frames: a quarter of the waves fill
// the chip 1.2 times; in the lanes the other frames' kernels fill the rest)
// (profiles/r05_ab_shadow_strips.txt).  The whole-span shortcut below then takes the
// raster-free launch to 21.6 us one-lane and config 3 345 -> 359 Gpix/s in the lanes
// (profiles/r05_ab_span.txt).
constexpr int P1_STRIPS = 4;
static_assert(P1_STRIPS * CODED_ROWS == SPAN_ROWS, "a PART 1 wave covers one span of the map's records (and its row records are one per lane)");
template <int PART>
constexpr int coded_wave_strips = PART == 1 ? P1_STRIPS : 1;
template <int PART>
constexpr int coded_wave_span = coded_wave_rows<PART> * coded_wave_strips<PART>;  // rows a wave covers
template <int PART>
constexpr int coded_tile_rows = coded_wave_span<PART> * TILE_Y;
constexpr uint32_t CODE_NONE = 0xFFFFu;  // packed-code +INF (also the U8 map's 0xFF)
// The BACK-face depth range of a sphere's covered texels: fl(z + fl(h*r)), h in (0, 1].
__device__ __forceinline__ void sphere_range(const RasterSphereK& s, double& lo, double& hi) {
    const double e = s.z + s.r;
    lo = s.r >= 0.0 ? s.z : e;
    hi = s.r >= 0.0 ? e : s.z;
}
// Two 16-bit codes per register (low: column 0, high: column 1), element-wise min.
typedef unsigned short ushort2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_min_u16(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_elementwise_min(__builtin_bit_cast(ushort2_t, a),
                                                                  __builtin_bit_cast(ushort2_t, b)));
}

// A wave's row record in LDS (the binary search's per-lane row lookups).
struct RowLdsK {
    double py;
    float pyf;
    int32_t pad;
};
// Dynamic LDS of the coded tile: the 4 waves' row records, then the ZRecK table.
constexpr size_t CODED_ROW_LDS = sizeof(RowLdsK) * CODED_TILE_ROWS * (P1_STRIPS > 1 ? P1_STRIPS : 1);

template <bool INC>
__device__ __forceinline__ uint32_t code_check(const ZRecK* __restrict__ T, double D, float pyf, float g0, float g1,
                                               float fsteps, double oz, int steps, bool& slow, bool& entry) {
    const bool fastD = __builtin_amdgcn_class(D, 0x198);  // finite, nonzero
    // g0, g1, pyf are host-bounded finite values: the median and the conversion of a
    // value in [1, steps] are exact and defined
    const int f = (int)ceilf(__builtin_amdgcn_fmed3f(__builtin_fmaf(g1, pyf, g0), 1.0f, fsteps));
    const double zp = T[f].zprev, zf = T[f].z;
    // bitwise & | on the predicates: no short-circuit, so no divergent branches
    const bool okA = INC ? (zp < D) : !(zp < D);
    const bool okB = INC ? !(zf < D) : (zf < D);
    entry = INC ? (oz < D) : !(oz < D);
    slow = !fastD | (entry & !(okA & okB));
    return (fastD & okA & okB & (f < steps)) ? (uint32_t)f : CODE_NONE;
}

// Does a sphere of the frame cover a texel of the 128 x 16 strip of columns [xb, xb + 127]
// and rows [s0, s0 + 15]?  A conservative test (wave-uniform): the sphere's exact pixel
// ranges, then its disc -- coverage is pa^2 + pb^2 < 1 with |pa| = |x - cx| / |r| (n / m =
// r / r^2, rtm_kernels.h), so no texel of the strip's NDC rectangle is covered when the
// rectangle's nearest point lies farther than |r| from the centre; a 1e-6 relative margin
// absorbs the rounding of both forms, and NaN / INF never reject.  The split launch gives
// a strip to the raster part (PART 2) exactly when this holds, and both parts evaluate it
// alike: round 5 used the union of the pixel ranges, which at config 3 also sent the empty
// strips between the orbiting sphere and the other two to PART 2's per-texel path.
__device__ __forceinline__ bool strip_rasters(const ShadowPart& a, int xb, int s0) {
    const int xe = min(xb + 127, a.W - 1), ye = min(s0 + CODED_ROWS - 1, a.H - 1);
    if ((a.flags & RTM_FLAG_NO_SHADOW_RASTER) || !union_may_cover(a, xb, xe, s0, ye)) return false;
    uint32_t m = wave_sphere_mask(a.sph, a.n_spheres, xb, xe, s0, ye);
    if (!m) return false;
    const double X0 = a.tab.nx[xb], X1 = a.tab.nx[xe], Y0 = a.tab.ny[s0], Y1 = a.tab.ny[ye];
    for (; m; m &= m - 1u) {
        const RasterSphereK& s = a.sph[__builtin_ctz(m)];
        const double dx = s.cx - fmin(fmax(s.cx, X0), X1), dy = s.cy - fmin(fmax(s.cy, Y0), Y1);
        if (!(dx * dx + dy * dy > (s.r * s.r) * (1.0 + 1e-6))) return true;
    }
    return false;
}

// PART (the split launch, launch_coded): 0 every strip; 1 only strips no sphere covers
// (strip_rasters; no raster code); 2 only the others.
template <bool INC, int CODE, int PART>
__device__ __forceinline__ void shadow_tile_coded(const ShadowPart& a, void* __restrict__ map, int bx, int by,
                                                  ZRecK* __restrict__ T, RowLdsK* __restrict__ RL) {
    constexpr int NR = coded_wave_rows<PART>;
    constexpr int NS = coded_wave_strips<PART>;  // strips per wave
    constexpr int SPAN = coded_wave_span<PART>;
    const int lane = threadIdx.x & (TILE_X - 1);
    const int wv = threadIdx.x >> 6;
    const int xb = bx * 128;
    const int x0 = xb + lane * 2;
    const int yw = __builtin_amdgcn_readfirstlane(by * coded_tile_rows<PART> + wv * SPAN);  // the wave's first row
    const int W = a.W, H = a.H, steps = a.steps;
    const bool march = !(a.flags & RTM_FLAG_NO_MARCH) && a.n_patches > 0 && steps > 0;
    // the LDS records: one per thread, loaded now, written before the barrier
    // (as double2 halves: a ZRecK value would be kept in scratch)
    const double2* zsrc = reinterpret_cast<const double2*>(a.tab.zrec);
    double2 rec0 = make_double2(0.0, 0.0), rec1 = rec0;
    const int fid = (int)threadIdx.x;  // this thread's first record
    if (march && fid <= steps) {
        rec0 = zsrc[2 * fid];
        rec1 = zsrc[2 * fid + 1];
    }
    const int xs0 = min(x0, W - 1), xs1 = min(x0 + 1, W - 1);
    ColRecK c00{}, c10{};  // patch 0's column records
    RowRecK rl{};  // lane < SPAN: row yw + lane's record (the wave's LDS row table)
    if (march) {
        if (NS == 1) {
            c00 = a.tab.col[xs0];
            c10 = a.tab.col[xs1];
        }
        // (the host pads the row table with non-marching rows to a multiple of 64 rows:
        // the wave's rows are inside it unless SPAN > 64; checked all the same)
        if (lane < SPAN) {
            if (yw + lane < a.tab.row_recs) rl = a.tab.row[yw + lane];
            else if (yw + lane < H) note_oob();  // (rows past H need no record: no strip reads them)
        }
    }
    if (march) {
        double2* T2 = reinterpret_cast<double2*>(T);
        if (fid <= steps) {
            T2[2 * fid] = rec0;
            T2[2 * fid + 1] = rec1;
        }
        for (int k = fid + BLOCK; k <= steps; k += BLOCK) {
            T2[2 * k] = zsrc[2 * k];
            T2[2 * k + 1] = zsrc[2 * k + 1];
        }
        if (lane < SPAN) RL[wv * SPAN + lane] = RowLdsK{rl.py, rl.pyf, 0};
        __syncthreads();
    }
    // wave-uniform: bit r = row yw + r marches (inRange01 and < H)
    const uint64_t rowbits_w = __ballot((lane < SPAN) & (rl.ok != 0));
    // bit st: strip st of the wave is the raster part's (strip_rasters; wave-uniform)
    // (a PART 2 workgroup runs only when its strip rasterizes: shadow_coded_block tested it)
    uint32_t boxbits = PART == 2 ? 1u : 0u;
#pragma unroll
    for (int st = 0; st < NS && PART != 2; ++st) {
        const int s0 = (yw + NR * st) & ~(CODED_ROWS - 1);
        if (s0 < H && strip_rasters(a, xb, s0)) boxbits |= 1u << st;
    }
    // The whole span's shortcut (PART 1, one patch, every one of the wave's SPAN rows
    // marching): a column's codes over the span are one monotone sequence by the strip
    // argument (D is monotone down the whole column), so both ends, decided on one side of
    // the entry threshold with D of one sign, and one binary search over the span locate
    // its single boundary -- one chain of log2(SPAN) checks instead of one per strip.
    // Any column it cannot decide sends the wave to the per-strip path.
    bool span_ok = false;
    uint32_t stop[2] = {CODE_NONE, CODE_NONE}, sbot[2] = {CODE_NONE, CODE_NONE};
    int sbnd[2] = {SPAN, SPAN};
    if (PART == 1 && NS > 1 && march && a.n_patches == 1 && rowbits_w == (SPAN >= 64 ? ~0ull : ((1ull << (SPAN & 63)) - 1))) {
        int i0 = xs0, i1 = xs1;
        asm volatile("" : "+v"(i0), "+v"(i1));
        const ColRecK q0 = a.tab.col[i0], q1 = a.tab.col[i1];
        const double d0[2] = {q0.d0, q1.d0};
        const double dd[2] = {q0.dd, q1.dd};
        const float g0[2] = {q0.g0, q1.g0};
        const float g1[2] = {q0.g1, q1.g1};
        const double oz = a.tab.z0;
        const float fsteps = (float)steps;
        const RowLdsK* RS = RL + __builtin_amdgcn_readfirstlane(wv * SPAN);
        bool ok = true;
#pragma unroll
        for (int c = 0; c < 2; ++c) {
            const RowLdsK rt = RS[0], rb = RS[SPAN - 1];
            const double Dt = d0[c] + dd[c] * rt.py;
            const double Db = d0[c] + dd[c] * rb.py;
            bool st_, et, sb, eb;
            stop[c] = code_check<INC>(T, Dt, rt.pyf, g0[c], g1[c], fsteps, oz, steps, st_, et);
            sbot[c] = code_check<INC>(T, Db, rb.pyf, g0[c], g1[c], fsteps, oz, steps, sb, eb);
            ok = ok & !st_ & !sb & (et == eb) & (__builtin_signbit(Dt) == __builtin_signbit(Db));
        }
        span_ok = __all(ok);
        if (span_ok) {
            const bool need[2] = {stop[0] != sbot[0], stop[1] != sbot[1]};
            if (__any(need[0] | need[1])) {
                // The boundary as a threshold on D (no code evaluation per step).  With entry
                // alike over the span, a row's code is the first k with P(z_k) (NONE = steps:
                // none before `steps`; P monotone over the table), so "code != top" is one
                // compare: !P(z_top) when the codes rise down the column, P(z_{top-1}) when they
                // fall -- monotone in D, hence in the row.  The first such row hi: a guess
                // from the ends' D (interpolated, f32), confirmed by rows hi - 1 and hi, else
                // a binary search on the same compare.  Row hi's code is the bottom code when
                // the two codes are adjacent (monotone codes strictly between none); otherwise
                // one check at hi confirms it (any other code: the span is no single run).
                const double Dt0 = d0[0] + dd[0] * RS[0].py, Db0 = d0[0] + dd[0] * RS[SPAN - 1].py;
                const double Dt1 = d0[1] + dd[1] * RS[0].py, Db1 = d0[1] + dd[1] * RS[SPAN - 1].py;
                const double Dt[2] = {Dt0, Dt1}, Db[2] = {Db0, Db1};
                int lo[2], hi[2];
                double zt[2];
                bool rise[2];
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int ct = stop[c] == CODE_NONE ? steps : (int)stop[c];
                    const int cb = sbot[c] == CODE_NONE ? steps : (int)sbot[c];
                    rise[c] = cb > ct;
                    zt[c] = T[rise[c] ? ct : ct - 1].z;  // (need: ct != cb, so ct < steps when rising, >= 1 falling)
                    // the guess: D runs from Dt to Db over rows 0 .. SPAN - 1
                    float fr = (float)(zt[c] - Dt[c]) * __builtin_amdgcn_rcpf((float)(Db[c] - Dt[c]));
                    fr = fr == fr ? fr * (float)(SPAN - 1) : 1.0f;
                    const int g = (int)ceilf(__builtin_amdgcn_fmed3f(fr, 1.0f, (float)(SPAN - 1)));
                    const double Da = d0[c] + dd[c] * RS[g - 1].py, Dg = d0[c] + dd[c] * RS[g].py;
                    // differs(D): the row's code is not the top code
                    const bool pa = INC ? !(zt[c] < Da) : (zt[c] < Da), pg = INC ? !(zt[c] < Dg) : (zt[c] < Dg);
                    const bool da = rise[c] ? !pa : pa, dg = rise[c] ? !pg : pg;
                    const bool hitg = need[c] & !da & dg;
                    lo[c] = hitg ? g - 1 : 0;
                    hi[c] = hitg ? g : SPAN - 1;
                }
                constexpr int HALVINGS = SPAN <= 16 ? 4 : SPAN <= 32 ? 5 : 6;
#pragma unroll
                for (int it = 0; it < HALVINGS; ++it) {
                    const bool act0 = need[0] & (hi[0] - lo[0] > 1), act1 = need[1] & (hi[1] - lo[1] > 1);
                    if (!__any(act0 | act1)) break;
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const bool act = c ? act1 : act0;
                        const int mid = (lo[c] + hi[c]) >> 1;
                        const double Dm = d0[c] + dd[c] * RS[act ? mid : 0].py;
                        const bool pm = INC ? !(zt[c] < Dm) : (zt[c] < Dm);
                        const bool dm = rise[c] ? !pm : pm;
                        lo[c] = (act & !dm) ? mid : lo[c];
                        hi[c] = (act & dm) ? mid : hi[c];
                    }
                }
                bool bad = false;
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const int ct = stop[c] == CODE_NONE ? steps : (int)stop[c];
                    const int cb = sbot[c] == CODE_NONE ? steps : (int)sbot[c];
                    const bool adj = (cb - ct == 1) | (ct - cb == 1);
                    if (__any(need[c] & !adj)) {
                        const RowLdsK rr = RS[hi[c]];
                        bool sm, em;
                        const uint32_t cm = code_check<INC>(T, d0[c] + dd[c] * rr.py, rr.pyf, g0[c], g1[c], fsteps, oz,
                                                            steps, sm, em);
                        bad |= need[c] & !adj & (sm | (cm != sbot[c]));
                    }
                    sbnd[c] = need[c] ? hi[c] : SPAN;
                }
                span_ok = !__any(bad);
            }
        }
    }
    // The span records (rtm_kernels.h).  A span's record is written by the one wave that
    // owns it: the PART 1 wave when no strip of its span is the raster part's (its codes
    // then need no block bytes at all when span_ok), else wave 0 of each PART 2 workgroup
    // of the span (the same SPAN_DENSE from each), or of the PART 0 workgroup (64 rows).
    if (CODE == SMAP_U8 && a.smap_spans && yw < H) {
        const bool own = PART == 1 ? boxbits == 0u : wv == 0;
        if (own) {
            const bool run = PART == 1 && span_ok;
            const uint32_t r0 = run ? (stop[0] & 0xFFu) | ((sbot[0] & 0xFFu) << 8) | ((uint32_t)sbnd[0] << 16) : SPAN_DENSE;
            const uint32_t r1 = run ? (stop[1] & 0xFFu) | ((sbot[1] & 0xFFu) << 8) | ((uint32_t)sbnd[1] << 16) : SPAN_DENSE;
            uint32_t lane_r;
            asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_r));
            uint32_t* rec = (uint32_t*)((uint8_t*)map + smap_span_offset(W, H)) + smap_span_index(xb, yw, a.smap_bw);
            *reinterpret_cast<uint2*>(rec + 2 * lane_r) = make_uint2(r0, r1);
            if (run) return;  // the record is the span's whole store
        }
    }
#pragma unroll 1
    for (int st = 0; st < NS; ++st) {
    const int y0 = yw + NR * st;  // this strip's first row
    if (NS > 1 && y0 >= H) break;  // (wave-uniform)
    // patch 0's column records: the prologue's for the first strip; a later strip reloads
    // them (L1/L2-hot) rather than keep them live across the loop (registers)
    ColRecK c0 = c00, c1 = c10;
    if (NS > 1 && march) {
        // (opaque copies of the column indices: the 64-bit record offsets are formed here,
        // not kept live across the loop -- held across it they were spilled to scratch)
        int i0 = xs0, i1 = xs1;
        asm volatile("" : "+v"(i0), "+v"(i1));
        c0 = a.tab.col[i0];
        c1 = a.tab.col[i1];
    }
    // this wave's strip is left to the other part of a split launch (wave-uniform); a
    // skipping wave still fills its records and meets the workgroup barrier.  The
    // split is decided per 16-row strip (a PART 2 wave's 4 rows lie in one)
    const bool strip_box = (boxbits >> st) & 1u;
    const bool skipw = (PART == 1 && strip_box) || (PART == 2 && !strip_box);
    // a row's two codes packed in one register (low: column 0), NONE = 0xFFFF
    uint32_t cdp[NR];
#pragma unroll
    for (int r = 0; r < NR; ++r) cdp[r] = 0xFFFFFFFFu;
    if (span_ok && !skipw) {
        // rows [0, sbnd) of the span hold the top code, [sbnd, SPAN) the bottom one
#pragma unroll
        for (int r = 0; r < NR; ++r) {
            const int row = NR * st + r;
            cdp[r] = (row < sbnd[0] ? stop[0] : sbot[0]) | ((row < sbnd[1] ? stop[1] : sbot[1]) << 16);
        }
    } else if (march && !skipw) {
        const double oz = a.tab.z0;
        const float fsteps = (float)steps;
        // the strip's rows (uniform reads are broadcasts; the wave's base as a scalar: held in a
        // VGPR across the strips it was spilled in the single-frame kernel)
        const RowLdsK* RW = RL + __builtin_amdgcn_readfirstlane(wv * SPAN) + NR * st;
        // wave-uniform: bit r = row y0 + r marches (inRange01 and < H)
        const uint32_t rowbits = (uint32_t)(rowbits_w >> (NR * st)) & ((1u << NR) - 1u);
        for (int k = 0; k < a.n_patches; ++k) {
            if (k > 0) {
                c0 = a.tab.col[k * W + xs0];
                c1 = a.tab.col[k * W + xs1];
            }
            const double d0[2] = {c0.d0, c1.d0};
            const double dd[2] = {c0.dd, c1.dd};
            const float g0[2] = {c0.g0, c1.g0};
            const float g1[2] = {c0.g1, c1.g1};
            // A column outside inRange01 has the host record d0 = "before the start"
            // (finite), dd = 0: entry and okA are false there, so it neither hits nor
            // goes slow -- no per-texel in-range test.
            // -- the shortcut: both ends of each column's strip
            bool sc = NR == CODED_ROWS && rowbits == (1u << NR) - 1u;  // every row marches (wave-uniform)
            uint32_t top[2] = {CODE_NONE, CODE_NONE}, bot[2] = {CODE_NONE, CODE_NONE};
            int bnd[2] = {NR, NR};  // first row with the bottom code (NR: none)
            if (sc) {
                bool ok = true;
#pragma unroll
                for (int c = 0; c < 2; ++c) {
                    const RowLdsK rt = RW[0], rb = RW[NR - 1];
                    const double Dt = d0[c] + dd[c] * rt.py;
                    const double Db = d0[c] + dd[c] * rb.py;
                    bool st, et, sb, eb;
                    top[c] = code_check<INC>(T, Dt, rt.pyf, g0[c], g1[c], fsteps, oz, steps, st, et);
                    bot[c] = code_check<INC>(T, Db, rb.pyf, g0[c], g1[c], fsteps, oz, steps, sb, eb);
                    ok = ok & !st & !sb & (et == eb) & (__builtin_signbit(Dt) == __builtin_signbit(Db));
                }
                sc = __all(ok);
            }
            if (sc) {
                const bool need0 = top[0] != bot[0], need1 = top[1] != bot[1];
                if (__any(need0 | need1)) {
                    // binary search, both columns side by side: code(lo) == top, code(hi) != top
                    int lo[2] = {0, 0}, hi[2] = {NR - 1, NR - 1};
                    uint32_t chi[2] = {bot[0], bot[1]};
                    const bool need[2] = {need0, need1};
                    bool bad = false;
#pragma unroll
                    for (int it = 0; it < 4; ++it) {  // 15 rows: 4 halvings (NR == 16 here)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const bool act = need[c] & (hi[c] - lo[c] > 1);
                            const int mid = (lo[c] + hi[c]) >> 1;
                            const RowLdsK rr = RW[act ? mid : 0];
                            const double Dm = d0[c] + dd[c] * rr.py;
                            bool sm, em;
                            const uint32_t cm = code_check<INC>(T, Dm, rr.pyf, g0[c], g1[c], fsteps, oz, steps, sm, em);
                            bad |= act & sm;
                            const bool same = cm == top[c];
                            lo[c] = (act & same) ? mid : lo[c];
                            hi[c] = (act & !same) ? mid : hi[c];
                            chi[c] = (act & !same) ? cm : chi[c];
                        }
                    }
                    // one boundary per column: the first differing row already has the bottom code
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        bad |= need[c] & (chi[c] != bot[c]);
                        bnd[c] = need[c] ? hi[c] : NR;
                    }
                    sc = !__any(bad);
                }
            }
            if (sc) {
                // rows [0, bnd) hold the top code, [bnd, NR) the bottom one
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    const uint32_t v = (r < bnd[0] ? top[0] : bot[0]) | ((r < bnd[1] ? top[1] : bot[1]) << 16);
                    cdp[r] = k == 0 ? v : pk_min_u16(cdp[r], v);
                }
                continue;
            }
            // -- the fallback: every texel's check (MASKED: skip rows outside inRange01 or
            // past H, wave-uniform; the common case runs without the row tests)
            bool sany = false;  // a texel the check cannot decide
            auto check = [&](auto masked) {
                constexpr bool MASKED = decltype(masked)::value;
                // (an opaque copy of the row bits per call: the row tests are not hoisted
                // out of the patch loop as NR live lane masks)
                uint32_t rb = rowbits;
                if (MASKED) asm volatile("" : "+s"(rb));
#pragma unroll
                for (int r = 0; r < NR; ++r) {
                    if (MASKED && !((rb >> r) & 1u)) continue;
                    const RowLdsK rr = RW[r];
                    uint32_t vv[2];
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        bool sl, en;
                        vv[c] = code_check<INC>(T, d0[c] + dd[c] * rr.py, rr.pyf, g0[c], g1[c], fsteps, oz, steps, sl,
                                                en);
                        sany |= sl;
                    }
                    cdp[r] = pk_min_u16(cdp[r], vv[0] | (vv[1] << 16));
                }
            };
            if (rowbits == (1u << NR) - 1u) check(std::false_type{});
            else check(std::true_type{});
            if (__any(sany)) {
                // exact per-texel march (march_axis) for the texels the check cannot decide
                // (sz: the host's dir.z * 0.03, the same product)
                const double sz = a.tab.sz;
#pragma unroll 1
                for (int q = 0; q < NR * 2; ++q) {
                    const int qr = q >> 1, qc = q & 1;
                    const RowLdsK rq = RW[qr];
                    const double pyq = rq.py;
                    const float pyfq = rq.pyf;
                    // (selects, not indexing: a dynamically indexed array would live in scratch)
                    const double d0q = qc ? d0[1] : d0[0], ddq = qc ? dd[1] : dd[0];
                    const float g0q = qc ? g0[1] : g0[0], g1q = qc ? g1[1] : g1[0];
                    const double Dv = d0q + ddq * pyq;
                    bool sl, en;
                    (void)code_check<INC>(T, Dv, pyfq, g0q, g1q, fsteps, oz, steps, sl, en);
                    sl = sl & (((rowbits >> qr) & 1u) != 0u);
                    if (!__any(sl)) continue;
                    MarchResult m{false, 0.0, 0, 0};
                    if (sl) m = march_axis<false>(Dv, true, oz, sz, steps, a.tab);
#pragma unroll
                    for (int r = 0; r < NR; ++r)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const unsigned cur = (cdp[r] >> (16 * c)) & 0xFFFFu;
                            if (q == r * 2 + c && sl && m.hit && (unsigned)m.k < min(cur, (unsigned)steps))
                                cdp[r] = (cdp[r] & ~(0xFFFFu << (16 * c))) | ((unsigned)m.k << (16 * c));
                        }
                }
            }
        }
    }
    // shadow viewport rasterize, face BACK (main.rs:1569, 243), 4 rows at a time: the
    // strict minimum over the spheres in scene order, then the march code only where its
    // t is strictly below that minimum (main.rs:559).
    //
    // A covered texel's BACK-face depth is fl(z + fl(h*r)) with h = sqrt(1 - d*d) in
    // (0, 1], so it lies in the sphere's range [z, fl(z + r)] (rounding is monotone; the
    // ends swap for r < 0), and coverage d < 1 is exactly s2 < 1 (sqrt is monotone and
    // the square root of the double below 1 is below 1).  When the ranges of a wave's
    // spheres are pairwise disjoint (wave-uniform), the nearest covering sphere is the
    // one with the lowest range -- the strict minimum in scene order picks it too -- and
    // the march beats it exactly when its t is below the range, loses when t is at or
    // above the range's top: no square root is taken.  Only a texel whose t falls inside
    // its winner's range, and waves with overlapping ranges, evaluate the depths.
    if (PART != 1 && strip_box && !skipw) {
        const uint32_t live0 = wave_sphere_mask(a.sph, a.n_spheres, xb, xb + 127, y0, y0 + NR - 1);
        if (live0) {
            const double xc[2] = {a.tab.nx[xs0], a.tab.nx[xs1]};
            bool disjoint = true;  // (wave-uniform)
            for (uint32_t li = live0; li && disjoint; li &= li - 1u) {
                double loi, hii;
                sphere_range(a.sph[__builtin_ctz(li)], loi, hii);
                disjoint = __builtin_isfinite(loi) & __builtin_isfinite(hii);
                for (uint32_t lj = li & (li - 1u); lj && disjoint; lj &= lj - 1u) {
                    double loj, hij;
                    sphere_range(a.sph[__builtin_ctz(lj)], loj, hij);
                    disjoint = (hii < loj) | (hij < loi);
                }
            }
#pragma unroll
            for (int b = 0; b < NR / 4; ++b) {
                const int yb = y0 + 4 * b;
                if (yb >= H) break;  // (wave-uniform)
                if (disjoint) {
                    // t of each texel's march code (NONE: T[steps].t = +INF; no march: +INF)
                    double tm[4][2];
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const uint32_t mc = (cdp[4 * b + r] >> (16 * c)) & 0xFFFFu;
                            tm[r][c] = march ? T[min(mc, (uint32_t)steps)].t : INFINITY;
                        }
                    uint32_t wc[4];     // packed winner codes (NONE: not covered)
                    uint32_t dec = 0u;  // 2 bits per texel (r, c) at 4r + 2c: 0 march, 1 sphere, 2 undecided
#pragma unroll
                    for (int r = 0; r < 4; ++r) wc[r] = 0xFFFFFFFFu;
                    bool any = false;
                    // farthest range first: a nearer covering sphere overwrites
                    for (uint32_t rem = live0; rem;) {
                        int i = __builtin_ctz(rem);
                        double best = -INFINITY;
                        for (uint32_t l = rem; l; l &= l - 1u) {
                            double lo, hi;
                            sphere_range(a.sph[__builtin_ctz(l)], lo, hi);
                            if (lo > best) {
                                best = lo;
                                i = __builtin_ctz(l);
                            }
                        }
                        rem &= ~(1u << i);
                        const RasterSphereK& sp = a.sph[i];
                        if (yb + 3 < sp.iy0 || yb > sp.iy1) continue;  // wave-uniform
                        double lo, hi;
                        sphere_range(sp, lo, hi);
                        // Coverage s2 = pa*pa + pb*pb < 1 with pa = (rel*n)/m: evaluated with
                        // 1/m (one wave-uniform division per sphere) in place of the divisions,
                        // the approximate s2 is within ~8 ulp of the reference's, so away from 1
                        // (|s2' - 1| > 1e-13) it decides exactly; a row where any texel lies
                        // closer takes the reference's divisions (the coverage rim, rare)
                        const double inv_m = 1.0 / sp.m;
                        double qa[2], pa2[2];
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            qa[c] = (xc[c] - sp.cx) * sp.n;
                            const double pa = qa[c] * inv_m;
                            pa2[c] = pa * pa;
                        }
#pragma unroll
                        for (int r = 0; r < 4; ++r) {
                            const int y = yb + r;
                            if (y >= H || y < sp.iy0 || y > sp.iy1) continue;  // wave-uniform
                            const double qb = (((cdouble*)a.tab.ny)[y] - sp.cy) * sp.n;
                            const double pbq = qb * inv_m;
                            const double pb2 = pbq * pbq;
                            bool inr[2], unsure = false;
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                const double s2 = pa2[c] + pb2;
                                inr[c] = s2 < 1.0;
                                unsure |= fabs(s2 - 1.0) <= 1e-13;
                            }
                            if (__builtin_expect(__any(unsure), 0)) {
                                const double pb = qb / sp.m;
#pragma unroll
                                for (int c = 0; c < 2; ++c) {
                                    const double pa = qa[c] / sp.m;
                                    inr[c] = pa * pa + pb * pb < 1.0;  // d = sqrt(pa*pa + pb*pb) < 1
                                }
                            }
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                const bool in = inr[c];
                                any |= in;
                                const uint32_t sh16 = 16u * (uint32_t)c, sh2 = 4u * (uint32_t)r + 2u * (uint32_t)c;
                                const uint32_t v = tm[r][c] < lo ? 0u : tm[r][c] >= hi ? 1u : 2u;
                                wc[r] = in ? (wc[r] & ~(0xFFFFu << sh16)) | ((uint32_t)(steps + i) << sh16) : wc[r];
                                dec = in ? (dec & ~(3u << sh2)) | (v << sh2) : dec;
                            }
                        }
                    }
                    if (!__any(any)) continue;
                    // texels whose t lies inside their winner's range: that sphere's depth
                    uint32_t amb = 0u;
#pragma unroll
                    for (int q = 0; q < 8; ++q) amb |= ((dec >> (2 * q)) & 3u) == 2u ? 1u << q : 0u;
                    if (__any(amb != 0u)) {
                        for (uint32_t l = live0; l; l &= l - 1u) {
                            const int j = __builtin_ctz(l);
                            const RasterSphereK& sp = a.sph[j];
                            double pa[2];
#pragma unroll
                            for (int c = 0; c < 2; ++c) pa[c] = ((xc[c] - sp.cx) * sp.n) / sp.m;
#pragma unroll
                            for (int r = 0; r < 4; ++r)
#pragma unroll
                                for (int c = 0; c < 2; ++c) {
                                    const uint32_t sh16 = 16u * (uint32_t)c;
                                    const bool mine = ((amb >> (2 * r + c)) & 1u) &&
                                                      ((wc[r] >> sh16) & 0xFFFFu) == (uint32_t)(steps + j);
                                    if (!__any(mine)) continue;
                                    const double pb = ((((cdouble*)a.tab.ny)[yb + r] - sp.cy) * sp.n) / sp.m;
                                    const double d = sqrt(pa[c] * pa[c] + pb * pb);
                                    const double h = sqrt(1.0 - d * d);
                                    const double depth = sp.z + h * sp.r;
                                    const uint32_t sh2 = 4u * (uint32_t)r + 2u * (uint32_t)c;
                                    const uint32_t v = tm[r][c] < depth ? 0u : 1u;
                                    dec = mine ? (dec & ~(3u << sh2)) | (v << sh2) : dec;
                                }
                        }
                    }
#pragma unroll
                    for (int r = 0; r < 4; ++r)
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const uint32_t sh16 = 16u * (uint32_t)c;
                            const bool sph = ((wc[r] >> sh16) & 0xFFFFu) != CODE_NONE &&
                                             ((dec >> (4 * r + 2 * c)) & 3u) == 1u;
                            cdp[4 * b + r] = sph ? (cdp[4 * b + r] & ~(0xFFFFu << sh16)) | (wc[r] & (0xFFFFu << sh16))
                                                 : cdp[4 * b + r];
                        }
                    continue;
                }
                // overlapping ranges: every covering sphere's depth, the strict minimum (zs, cs)
                double zs[4][2];
                uint32_t cs[4];  // packed sphere codes, NONE = no sphere covers
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    cs[r] = 0xFFFFFFFFu;
                    zs[r][0] = zs[r][1] = INFINITY;
                }
                bool any = false;
                uint32_t live = live0;
                while (live) {
                    const int i = __builtin_ctz(live);
                    live &= live - 1u;
                    const RasterSphereK& sp = a.sph[i];
                    if (yb + 3 < sp.iy0 || yb > sp.iy1) continue;  // wave-uniform
                    const double inv_m = 1.0 / sp.m;
                    double pa[2];
#pragma unroll
                    for (int c = 0; c < 2; ++c) pa[c] = ((xc[c] - sp.cx) * sp.n) / sp.m;
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int y = yb + r;
                        if (y >= H || y < sp.iy0 || y > sp.iy1) continue;  // wave-uniform
                        const double qb = (((cdouble*)a.tab.ny)[y] - sp.cy) * sp.n;
                        {  // the division-free filter (see the disjoint path): a row no texel of
                           // which can be covered needs no exact coverage
                            const double pbq = qb * inv_m;
                            bool maybe = false;
#pragma unroll
                            for (int c = 0; c < 2; ++c) {
                                const double paq = ((xc[c] - sp.cx) * sp.n) * inv_m;
                                maybe |= paq * paq + pbq * pbq < 1.0 + 1e-13;
                            }
                            if (!__any(maybe)) continue;
                        }
                        const double pb = qb / sp.m;
                        double s2[2];
                        bool in = false;
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            s2[c] = pa[c] * pa[c] + pb * pb;
                            in |= s2[c] < 1.0;
                        }
                        if (!__any(in)) continue;  // (d < 1 <=> s2 < 1: no covered texel in this row)
                        any = true;
#pragma unroll
                        for (int c = 0; c < 2; ++c) {
                            const double d = sqrt(s2[c]);
                            const double h = sqrt(1.0 - d * d);
                            const double depth = sp.z + h * sp.r;
                            const bool win = (d < 1.0) & (depth < zs[r][c]);
                            zs[r][c] = win ? depth : zs[r][c];
                            const uint32_t sh16 = 16u * (uint32_t)c;
                            cs[r] = win ? (cs[r] & ~(0xFFFFu << sh16)) | ((uint32_t)(steps + i) << sh16) : cs[r];
                        }
                    }
                }
                if (!any) continue;
#pragma unroll
                for (int r = 0; r < 4; ++r)
#pragma unroll
                    for (int c = 0; c < 2; ++c) {
                        const uint32_t sh16 = 16u * (uint32_t)c;
                        const uint32_t sc16 = (cs[r] >> sh16) & 0xFFFFu;
                        if (sc16 == CODE_NONE) continue;
                        const uint32_t mc = (cdp[4 * b + r] >> sh16) & 0xFFFFu;
                        // t of the march code (NONE: T[steps].t = +INF); no march: +INF
                        const double tm = march ? T[min(mc, (uint32_t)steps)].t : INFINITY;
                        if (!(tm < zs[r][c]))
                            cdp[4 * b + r] = (cdp[4 * b + r] & ~(0xFFFFu << sh16)) | (sc16 << sh16);
                    }
            }
        }
    }
    if (skipw) continue;
    // the lane's 4 rows x 2 columns of each block as one 8- (U8) or 16-byte (U16)
    // store: element lane*8 + r*2 + c of block (y >> 2, xb >> 7) (rows past H hold
    // codes no reader looks up; a block wholly past H does not exist).  The lane id is
    // recomputed here (mbcnt): kept live across the march, the batched raster-free kernel
    // spilled it to scratch, and its reload was a memory round trip ahead of the stores
    // (plus 12 B of scratch traffic per lane: the 1.29x HBM writes of the r04 PMC view)
    uint32_t lane_st;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane_st));
#pragma unroll
    for (int b = 0; b < NR / 4; ++b) {
        const int yb = y0 + 4 * b;
        if (yb >= H) break;
        const int64_t blk = (int64_t)(yb >> 2) * a.smap_bw + (xb >> 7);
        if (CODE == SMAP_U8) {
            // bytes (r, c) at 8*((r & 1)*2 + c) of word r >> 1: the low bytes of two rows' codes
            const uint32_t w0 = __builtin_amdgcn_perm(cdp[4 * b + 1], cdp[4 * b], 0x06040200u);
            const uint32_t w1 = __builtin_amdgcn_perm(cdp[4 * b + 3], cdp[4 * b + 2], 0x06040200u);
            *reinterpret_cast<uint2*>((uint8_t*)map + blk * 512 + lane_st * 8) = make_uint2(w0, w1);
        } else {
            *reinterpret_cast<uint4*>((uint8_t*)map + blk * 1024 + lane_st * 16) =
                make_uint4(cdp[4 * b], cdp[4 * b + 1], cdp[4 * b + 2], cdp[4 * b + 3]);
        }
    }
    }  // strips
}

// One workgroup tile (bx, by) of a split launch's part: it leaves at once (workgroup-
// uniform, before its barrier) when none of its strips is this part's, by the waves' own
// test, strip_rasters.
template <bool INC, int CODE, int PART>
__device__ __forceinline__ void shadow_split_block(const ShadowPart& sh, void* __restrict__ map, char* __restrict__ lds,
                                                   int bx, int by) {
    constexpr int TR = coded_tile_rows<PART>;
    const int ya = by * TR, xa = bx * 128;
    if (PART == 2) {  // (one 16-row strip per workgroup)
        if (!strip_rasters(sh, xa, ya)) return;
    } else if (!(sh.flags & RTM_FLAG_NO_SHADOW_RASTER) && union_may_cover(sh, xa, xa + 127, ya, ya + CODED_ROWS - 1) &&
               union_may_cover(sh, xa, xa + 127, ya + TR - CODED_ROWS, ya + TR - 1)) {
        // (the union reaches both end strips: every strip may be PART 2's)
        bool all = true;
        for (int s0 = ya; s0 < ya + TR && s0 < sh.H && all; s0 += CODED_ROWS) all = strip_rasters(sh, xa, s0);
        if (all) return;
    }
    shadow_tile_coded<INC, CODE, PART>(sh, map, bx, by, reinterpret_cast<ZRecK*>(lds + CODED_ROW_LDS),
                                       reinterpret_cast<RowLdsK*>(lds));
}

template <bool INC, int CODE, int PART>
__device__ __forceinline__ void shadow_coded_block(const ShadowPart& sh, void* __restrict__ map, char* __restrict__ lds,
                                                   int4 org) {
    constexpr int TR = coded_tile_rows<PART>;
    int bx = (int)blockIdx.x, by;
    if (PART == 0) {
        const int n = (int)gridDim.y;
        const int h0 = max(sh.cull_y0, 0) / TR;
        const int h1 = min(min(sh.cull_y1, sh.H - 1) / TR, n - 1);
        const bool none = sh.cull_x0 > sh.cull_x1 || sh.cull_y0 > sh.cull_y1 || sh.cull_y1 < 0;
        by = none ? (int)blockIdx.y : hot_rows_first((int)blockIdx.y, n, h0, h1);
    } else {
        shadow_split_block<INC, CODE, PART>(sh, map, lds, bx + org.x, (int)blockIdx.y + org.y);
        return;
    }
    shadow_tile_coded<INC, CODE, PART>(sh, map, bx, by, reinterpret_cast<ZRecK*>(lds + CODED_ROW_LDS),
                                       reinterpret_cast<RowLdsK*>(lds));
}

// waves per SIMD the register allocator must keep: 6 for the raster-free part (round 3:
// uncapped, fewer spilled SGPRs cost 90 VGPRs and 5 waves; round 5: the span shortcut's
// registers spilled 16 B to scratch under 7, none under 6 -- 80 VGPRs, and 6 waves of
// 4-strip waves still fill the chip), else free
template <int PART>
constexpr int CODED_MIN_WAVES = PART == 1 ? 6 : 1;

template <bool INC, int CODE, int PART>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(CODED_MIN_WAVES<PART>, 8))) void
shadow_coded_kernel(const FrameArgs a, double* __restrict__ smap, int4 org) {
    extern __shared__ char lds_coded[];
    shadow_coded_block<INC, CODE, PART>(a.sh, smap, lds_coded, org);
}

template <bool INC, int CODE, int PART>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(CODED_MIN_WAVES<PART>, 8))) void
shadow_coded_batch_kernel(CBatch* __restrict__ fr, int4 org) {
    extern __shared__ char lds_coded[];
    CBatch* f = fr + blockIdx.z;
    shadow_coded_block<INC, CODE, PART>(*(const ShadowPart*)&f->a.sh, f->smap, lds_coded, org);
}

constexpr int SPLIT_MIN_WAVES = 5;
// Both parts of a batch's split launch as ONE launch (round 6): workgroups [0, org.w) of a
// frame are PART 2's tiles over the box (org.z of them per row, from (org.x, org.y)), the
// rest PART 1's over the whole map, row-major.  One launch's fixed cost instead of two
// (an empty launch of either part took ~4.2 us one-lane at config 3, profiles/r06_ab_shadow.txt);
// the sphere tiles come first, so their longer waves start first.
template <bool INC, int CODE>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(SPLIT_MIN_WAVES, 8))) void
shadow_split_batch_kernel(CBatch* __restrict__ fr, int4 org) {
    extern __shared__ char lds_coded[];
    CBatch* f = fr + blockIdx.z;
    const ShadowPart& sh = *(const ShadowPart*)&f->a.sh;
    const int id = (int)blockIdx.x;
    if (id < org.w) {
        shadow_split_block<INC, CODE, 2>(sh, f->smap, lds_coded, org.x + id % org.z, org.y + id / org.z);
    } else {
        const int j = id - org.w, gx = (sh.W + 127) >> 7;
        shadow_split_block<INC, CODE, 1>(sh, f->smap, lds_coded, j % gx, j / gx);
    }
}


// Eye tile: 64 x TILE_Y pixels: eye viewport rasterize (face FRONT, main.rs:1616)
// [+ processRaytracingRays when RT, main.rs:1035] + renderColorImage
// (main.rs:714-898).  FUSED evaluates the looked-up shadow texel on demand from
// `sh` (same frame) instead of reading `smap`.
// RT: 0 spheres only, 1 + ray-traced planes/cylinders and PERSPECTIVE spheres,
// 2 + SDFs (its own instantiation: the sphere-trace loop's registers would
// otherwise lower the occupancy of every ray-traced frame).
// Image row of the launch's local row j (EyePart: contiguous rows or cyclic stripes).
__device__ __forceinline__ int eye_row(int row_begin, int S, int stride, int phase, int j) {
    return S > 0 ? phase + (j / S) * stride + j % S : row_begin + j;
}

template <class T>
__device__ __forceinline__ const T* const_table(const T* p) {
    return (const T*)(const __attribute__((address_space(4))) T*)p;
}

// BLK: the waves are 8 x 8 pixel blocks (workgroup bx: 4 blocks side by side, block row
// by: 8 rows), for the batched RT 3 frames without shadows and without stripes: a compact
// primitive touches fewer blocks than 64 x 1 rows, and a block's cone is narrower.
template <bool FUSED, bool COUNT, int RT, int FMT = RTM_FORMAT_RGBA32F, bool NOSH = false, bool BLK = false>
__device__ __forceinline__ void eye_tile(const EyePart& a, const ShadowPart& sh, const double* __restrict__ smap,
                                         void* __restrict__ out, int bx, int by, StatsK* __restrict__ st,
                                         const DevTabs tabs, bool KMB = false, uint32_t kmw = 0u,
                                         bool km_in = false) {
    static_assert(!BLK || ((RT == 3 || RT == 2) && FMT == RTM_FORMAT_RGBA32F && !COUNT), "8 x 8 blocks: RT 3 / 2, RGBA f32");
    // RT 3: RT 1 under a PERSPECTIVE eye, with the host's origin-only primitive
    // constants (RtK::persp) and the per-wave primitive masks of rt_cull_kernel
    constexpr bool RTP = RT == 3;
    constexpr int RTB = RTP ? 1 : RT;
    // the frame's tables through constant-address-space pointers: their reads are scalar
    // loads wherever the address is uniform, whatever the kernel stored before them
    const RtK* rt_ = tabs.rt;
    const PerspK* __restrict__ psp = const_table(tabs.psp);
    const SdfTabK* __restrict__ sdf = const_table(tabs.sdf);
    // the workgroup's 4 waves stacked (64 x 4 pixels)
    const int wv_ = (int)(threadIdx.x >> 6), ln_ = (int)(threadIdx.x & (TILE_X - 1));
    // (BLK: bx is the wave's block column)
    const int xb = __builtin_amdgcn_readfirstlane(BLK ? bx * 8 : bx * TILE_X);
    const int xi = xb + (BLK ? (ln_ & 7) : ln_);
    // (BLK: the lane's own row; else the wave's)
    const int yl = BLK ? by * 8 + (ln_ >> 3) : __builtin_amdgcn_readfirstlane(by * TILE_Y + wv_);
    const int yl0 = BLK ? __builtin_amdgcn_readfirstlane(by * 8) : yl;  // the wave's first row
    // the header fields the prologue needs, read before any branch so their scalar loads
    // issue as one group: one wait instead of a chain of dependent round trips (the
    // short waves of small frames are latency-bound: config 7 +6 %, profiles/r04_ab_eye_prologue.txt)
    int W_ = a.W, H_ = a.H, rb_ = a.row_begin, re_ = a.row_end, og_ = a.out_global;
    int S_ = a.stripe_rows, ss_ = a.stripe_stride, sp_ = a.stripe_phase;
    const uint32_t* rtm_ = tabs.rtmask;
    int ns_ = a.n_spheres, cx0_ = a.cull_x0, cx1_ = a.cull_x1, cy0_ = a.cull_y0, cy1_ = a.cull_y1;
    const double* nx_ = a.nx;
    const double* ny_ = a.ny;
    int rtw_ = tabs.rtmask_words;
    // (an empty asm that passes them through -- not volatile, no memory operand, so it
    // does not count as a write that would turn the later table loads into vector loads
    // -- makes every load complete here, together, under one wait; for the ray-traced
    // instantiations only: it pushes the SDF one to 155 spilled VGPRs and the sphere-only
    // one from 60 to 66 VGPRs, profiles/r04_ab_eye_prologue.txt)
    // (with the batch kernel's mask word, the primitive table and the frame; the pointers
    // pass as global-address-space ones: an asm's generic output pointer loses its address
    // space, and the primitive table's reads became flat vector loads -- config 6 -29 %)
    typedef const __attribute__((address_space(4))) RtK* RtG;
    typedef __attribute__((address_space(1))) char* OutG;
    RtG rtg = (RtG)rt_;
    OutG outg = (OutG)out;
    if (RT == 1 || RT == 3)
        asm("" : "+s"(W_), "+s"(H_), "+s"(rb_), "+s"(re_), "+s"(og_), "+s"(S_), "+s"(ss_), "+s"(sp_), "+s"(rtm_),
            "+s"(ns_), "+s"(cx0_), "+s"(cx1_), "+s"(cy0_), "+s"(cy1_), "+s"(nx_), "+s"(ny_), "+s"(rtw_), "+s"(kmw),
            "+s"(rtg), "+s"(outg));
    const RtK* __restrict__ rt = (const RtK*)rtg;
    out = (void*)outg;
    const int yi = BLK ? rb_ + yl : __builtin_amdgcn_readfirstlane(eye_row(rb_, S_, ss_, sp_, yl));
    const int yo = og_ ? yi : yl;  // the output row
    const bool live = (xi < W_) & (rb_ + yl < re_) & (yi < H_);
    // the wave's image rows [ya, ye] and columns [xb, xe]
    const int ya = BLK ? rb_ + yl0 : yi, ye = BLK ? ya + 7 : yi;
    const int xe = xb + (BLK ? 7 : TILE_X - 1);
    // (union_may_cover on the loaded fields; an empty union (x0 > x1) meets nothing)
    const bool um_ = (cx0_ <= cx1_) & (ye >= cy0_) & (ya <= cy1_) & (xe >= cx0_) & (xb <= cx1_);
    // An out-of-range side-table read is counted once the tile's last load is done: the
    // counter's atomic is a global write, and one ahead of a load makes the compiler treat
    // the load as clobbered -- the primitive tables would go through vector instead of
    // scalar loads (config 6 eye pass 77 -> 96 us per frame before this was noticed).
    bool oob = false;
    unsigned long long n_tests = 0, n_hit = 0, n_lit = 0, n_pl_tests = 0, n_cy_tests = 0;
    ShadowCounts sc;
    int hit_kind = 0, hit_id = -1;
    uint32_t n_evals = 0;
    // the wave's spheres (all lanes active here); ascending bit order = scene order
    uint32_t smask = um_ ? wave_sphere_mask(a.sph, ns_, xb, xe, ya, ye) : 0u;
    // the wave's ray-traced primitives (PERSPECTIVE eye; all lanes active here)
    uint32_t rmask = 0u;
#if defined(RTM_TEST_REVERT_MASK_GUARD)  // (tools/bounds_demo.sh only: the round-3 over-read, to show tests/test_bounds.py catches it)
    if (RTP && rtm_) {
#else
    if (RTP && KMB) {
        // (the batch kernel's word, loaded with the header; nw = gx * rows words, so
        // km_in is the row guard; a frame without primitives has no word, and rt == null)
        if (km_in) rmask = kmw;
        else if (rb_ + yl < re_ && rt) {
            oob = true;
            rmask = rt_slots(rt->n_pl, rt->n_cy);
        }
    } else if (RTP && rtm_ && rb_ + yl < re_) {  // (no mask word for rows past the part)
#endif
        const int widx = yl * ((a.W + TILE_X - 1) / TILE_X) + (xb / TILE_X);  // (wave-uniform)
        if (widx < rtw_) {  // (the prologue's grouped copies of tabs.rtmask_words / tabs.rtmask)
            rmask = ((const __attribute__((address_space(4))) uint32_t*)rtm_)[widx];
        } else {
            oob = true;
            rmask = rt_slots(rt->n_pl, rt->n_cy);  // (every primitive: the result stays exact)
        }
    } else if (RTB == 1 && rt && a.eye.type == RTM_CAMERA_PERSPECTIVE) {
        rmask = BLK ? rt_wave_mask(rt, a.eye, min(xb, a.W - 1), min(xe, a.W - 1), min(ya, a.H - 1), a.W, a.H,
                                   min(ye, a.H - 1))
                    : rt_wave_mask(rt, a.eye, min(xb, a.W - 1), min(xb + TILE_X - 1, a.W - 1), min(yi, a.H - 1), a.W, a.H);
    } else if (RTB && rt) {
        rmask = rt_slots(rt->n_pl, rt->n_cy);
    }
    float4 c = make_float4(0.0f, 0.2f, 0.2f, 1.0f);  // (0.0, 0.2, 0.2) as f32 (main.rs:718-720)
    bool shaded = false;
    // a wave no sphere, primitive or SDF can reach is background: no NDC loads, no rays
    // (its pixels keep the background colour, as the full loop would leave them)
    const bool reach = smask != 0u || (RTB && rt && rmask != 0u) || (RT == 2 && sdf);
    if (live && reach) {
        const double x = a.nx[xi];
        const double y = a.ny[yi];
        // z-test over spheres in scene order, strict '<' against +INF init (main.rs:318)
        double best = INFINITY, bh = 0.0, bz = 0.0;
        int bid = -1;
        while (smask) {
            const int i = __builtin_ctz(smask);
            smask &= smask - 1u;
            double h;
            // (RT variant only: a PERSPECTIVE eye with spheres, row f-3; psp is wave-uniform)
            if ((RTB && psp) ? cover_persp(psp->s[i], x, y, h) : cover(a.sph[i], x, y, h)) {
                if (COUNT) ++n_tests;
                const double depth = a.sph[i].z - h * a.sph[i].r;  // EnumFace::FRONT (main.rs:239)
                if (depth < best) {
                    best = depth;
                    bh = h;
                    bz = a.sph[i].z;
                    bid = a.sph[i].id & (RTM_MAX_SPHERES - 1);  // (a.shade has RTM_MAX_SPHERES entries)
                }
            }
        }
        RtHit hit;
        hit.kind = bid >= 0 ? 1 : 0;
        hit.id = bid;
        double o[3], d[3];
        if (RTB) {
            cam_ray(a.eye, x, y, o, d);
            double zb = best;
            if (rt) {
                trace_pixel<RTP>(rt, o, d, zb, hit, rmask, oob);
                if (COUNT) {
                    n_pl_tests = __builtin_popcount(rmask & ((1u << rt->n_pl) - 1u));
                    n_cy_tests = __builtin_popcount((rmask >> 16) & ((1u << rt->n_cy) - 1u));
                }
            }
            // (a batch mixes frames with and without SDFs)
            if (RT == 2 && sdf) trace_sdfs<!COUNT>(sdf, o, d, zb, hit, n_evals, oob);
        }
        if (hit.kind) {
            shaded = true;
            if (!RTB) cam_ray(a.eye, x, y, o, d);
            // world position and normal per surface kind (main.rs:729-796)
            double wx, wy, wz, nx, ny, nz, cr, cg, cb;
            // (the tables below are indexed by the hit's scene id, checked where it was
            // taken: checked_id)
            if (!RTB || hit.kind == 1) {
                const ShadeSphereK& s = a.shade[bid];
                const double depth = bz - bh * s.r;  // calcDepth (main.rs:160-162)
                wx = o[0] + d[0] * depth;
                wy = o[1] + d[1] * depth;
                wz = o[2] + d[2] * depth;
                nx = (wx - s.px) * s.inv_r;
                ny = (wy - s.py) * s.inv_r;
                nz = (wz - s.pz) * s.inv_r;
                cr = s.cr;
                cg = s.cg;
                cb = s.cb;
            } else {
                wx = o[0] + d[0] * hit.t;  // calcDepth = rayT (main.rs:166-171)
                wy = o[1] + d[1] * hit.t;
                wz = o[2] + d[2] * hit.t;
                const int id = hit.id;
                if (hit.kind == 2) {
                    const PlaneK& p = rt->pl[id];
                    nx = p.nx;
                    ny = p.ny;
                    nz = p.nz;
                    cr = p.cr;
                    cg = p.cg;
                    cb = p.cb;
                } else {  // capped cylinder or SDF: the normal came with the hit
                    nx = hit.n[0];
                    ny = hit.n[1];
                    nz = hit.n[2];
                    if (RT != 2 || hit.kind == 3) {  // (kind 4, an SDF, only with RT 2)
                        cr = rt->cy[id].cr;
                        cg = rt->cy[id].cg;
                        cb = rt->cy[id].cb;
                    } else {
                        cr = sdf->s[id].cr;
                        cg = sdf->s[id].cg;
                        cb = sdf->s[id].cb;
                    }
                }
            }
            // light (1,0,0).scale(-1.0) (main.rs:810-813)
            const double Lx = 1.0 * -1.0, Ly = 0.0 * -1.0, Lz = 0.0 * -1.0;
            const double diffuse = fmax(nx * Lx + ny * Ly + nz * Lz, 0.0);
            // reflect(L, n) = L - n*(-2 dot(L,n))  (main.rs:2872-2875, sign as written)
            const double k2 = -2.0 * (Lx * nx + Ly * ny + Lz * nz);
            const double Rx = Lx - nx * k2, Ry = Ly - ny * k2, Rz = Lz - nz * k2;
            // retViewDirOfPixel (main.rs:1981-2013): -dir (ORTHOGONAL) or -normalize(ray) (PERSPECTIVE)
            double vx, vy, vz;
            if (!RTB || (!RTP && a.eye.type == RTM_CAMERA_ORTHOGONAL)) {
                vx = a.eye.dir[0] * -1.0;
                vy = a.eye.dir[1] * -1.0;
                vz = a.eye.dir[2] * -1.0;
            } else {
                vx = d[0] * -1.0;
                vy = d[1] * -1.0;
                vz = d[2] * -1.0;
            }
            double sp = fmax(vx * Rx + vy * Ry + vz * Rz, 0.0);
            sp = sp * sp;  // powi(32): five squarings (compiler-rt __powidf2)
            sp = sp * sp;
            sp = sp * sp;
            sp = sp * sp;
            sp = sp * sp;
            // shadow mapping (main.rs:836-856)
            const double dfx = wx - a.shadow.pos[0], dfy = wy - a.shadow.pos[1], dfz = wz - a.shadow.pos[2];
            const double qx = dfx * a.shadow.side[0] + dfy * a.shadow.side[1] + dfz * a.shadow.side[2];
            const double qy = dfx * a.shadow.up[0] + dfy * a.shadow.up[1] + dfz * a.shadow.up[2];
            const double qz = dfx * a.shadow.dir[0] + dfy * a.shadow.dir[1] + dfz * a.shadow.dir[2];
            const int64_t hw = a.Ws / 2, hh = a.Hs / 2;
            const int64_t tx = tex_index(hw, qx * (double)hw);
            const int64_t ty = tex_index(hh, qy * (double)hh);
            double dsm = INFINITY;  // (NOSH: an all-+INF shadow viewport, no lookup)
            if (!NOSH && ty >= 0 && ty < a.Hs && tx >= 0 && tx < a.Ws) {
                if (FUSED)
                    dsm = shadow_texel<COUNT>(sh, (int)tx, (int)ty, (int)tx, (int)tx, (int)ty, sc);
                else if (sh.smap_fmt == SMAP_F64)
                    dsm = smap[ty * a.Ws + tx];
                else
                    dsm = smap_decode_wave(sh, smap, (int)tx, (int)ty, oob);
            }
            const bool lit = dsm > qz - 0.0;
            const double lm = lit ? 1.0 : 0.25;
            const double base = diffuse + sp;
            c.x = (float)((base * lm) * cr);
            c.y = (float)((base * lm) * cg);
            c.z = (float)((base * lm) * cb);
            if (COUNT) {
                n_hit = 1;
                n_lit = lit;
                hit_kind = hit.kind;
                hit_id = hit.id;
            }
        }
    }
    // the frame store (all lanes converged): RGBA f32, or writeColorImage's bytes
    if (FMT == RTM_FORMAT_RGBA32F) {
        float4* o = reinterpret_cast<float4*>(out);
        // non-temporal: the frame is not re-read, and at 7680x4320 its 531 MB would
        // otherwise evict the shadow map the pass gathers from (eye 120 -> 85 us)
        if (live)
            __builtin_nontemporal_store(f32x4{c.x, c.y, c.z, c.w}, reinterpret_cast<f32x4*>(&o[(int64_t)yo * a.W + xi]));
    } else {
        uint32_t e = tabs.bg;  // background: one host-encoded constant
        if (shaded) {
            const float* T = reinterpret_cast<const float*>(tabs.enc);
            const uint8_t* B = reinterpret_cast<const uint8_t*>(tabs.enc) + 1024;
            e = enc_byte(c.x, T, B) | (enc_byte(c.y, T, B) << 8) | (enc_byte(c.z, T, B) << 16);
        }
        if (FMT == RTM_FORMAT_RGBA8) {  // alpha 1.0 -> 255; one dword per pixel, 256 B per wave
            uint32_t* o = reinterpret_cast<uint32_t*>(out);
            if (live) __builtin_nontemporal_store(e | 0xFF000000u, &o[(int64_t)yo * a.W + xi]);
        } else {  // RGB8: the wave's 64 pixels are 192 contiguous bytes = 48 dwords
            uint8_t* row = reinterpret_cast<uint8_t*>(out) + (int64_t)yo * a.W * 3;
            if (tabs.fmt & FMT_RGB8_DWORDS) {
                // dword j of the wave's segment: bytes 4j..4j+3 = the tail of pixel L (from
                // byte o = 4j - 3L) and the head of pixel L + 1
                const int j = threadIdx.x & (TILE_X - 1);
                const int L = min((4 * j) / 3, TILE_X - 1);
                const int o = min(4 * j - 3 * L, 2);  // (lanes j >= 48, clamped, store nothing)
                const uint32_t p0 = (uint32_t)__shfl((int)e, L);
                const uint32_t p1 = (uint32_t)__shfl((int)e, min(L + 1, TILE_X - 1));
                const uint32_t w = (p0 >> (8 * o)) | (p1 << (8 * (3 - o)));
                const int nv = min(TILE_X, a.W - xb);  // W % 4 == 0 (host-checked): 3*nv/4 whole dwords
                if (a.row_begin + yl < a.row_end && yi < a.H && j < (3 * nv) >> 2)
                    __builtin_nontemporal_store(w, reinterpret_cast<uint32_t*>(row + 3 * (int64_t)xb) + j);
            } else if (live) {
                row[3 * (int64_t)xi + 0] = (uint8_t)e;
                row[3 * (int64_t)xi + 1] = (uint8_t)(e >> 8);
                row[3 * (int64_t)xi + 2] = (uint8_t)(e >> 16);
            }
        }
    }
    // the sphere ids a hit shades with (a.shade[id]): the host validated them (checked_id);
    // the frame's first wave checks them again (here, after the tile's stores: earlier it
    // cost the tile 8 VGPRs) and counts any past the table, and every read above masks
    // the id into the 16-entry table, so none can leave it
    if (bx == 0 && by == 0 && (BLK || threadIdx.x < TILE_X)) {  // (wave-uniform; BLK: the block at (0, 0))
        const int l = threadIdx.x & (TILE_X - 1);
        if (__ballot(l < ns_ && (unsigned)a.sph[min(l, RTM_MAX_SPHERES - 1)].id >= (unsigned)ns_)) oob = true;
    }
    if (__builtin_expect(oob, 0)) note_oob();  // (after the tile's last load, see above)
    if (COUNT) {
        stat_add(&st->eye_sphere_tests, n_tests);
        stat_add(&st->eye_hit_pixels, n_hit);
        stat_add(&st->lit_pixels, n_lit);
        for (int i = 0; i < a.n_spheres; ++i) stat_add(&st->eye_hits[i], hit_kind == 1 && hit_id == i);
        if (RTB) {
            stat_add(&st->eye_circle_plane_pixels, hit_kind == 2);
            stat_add(&st->eye_capped_cylinder_pixels, hit_kind == 3);
            stat_add(&st->eye_plane_tests, n_pl_tests);
            stat_add(&st->eye_cylinder_tests, n_cy_tests);
            if (RT == 2) {
                stat_add(&st->eye_sdf_pixels, hit_kind == 4);
                stat_add(&st->sdf_distance_evals, n_evals);
            }
        }
        if (FUSED) {
            stat_add(&st->shadow_sphere_tests, sc.tests);
            stat_add(&st->march_iterations, sc.iters);
            stat_add(&st->march_hits, sc.hits);
            stat_add(&st->march_in_range, sc.inrange);
        }
    }
}

template <bool COUNT>
__global__ __launch_bounds__(BLOCK) void shadow_pass_kernel(const FrameArgs a, double* __restrict__ smap,
                                                            StatsK* __restrict__ st) {
    shadow_tile_generic<COUNT>(a.sh, smap, blockIdx.x, blockIdx.y, st);
}

__global__ __launch_bounds__(BLOCK) void shadow_pass_batch_kernel(CBatch* __restrict__ fr) {
    CBatch* f = fr + blockIdx.z;
    shadow_tile_generic<false>(*(const ShadowPart*)&f->a.sh, f->smap, blockIdx.x, blockIdx.y, nullptr);
}

template <bool FUSED, bool COUNT, int RT, int FMT, bool NOSH = false>
__global__ __launch_bounds__(BLOCK) void eye_pass_kernel(const FrameArgs a, const double* __restrict__ smap,
                                                         void* __restrict__ out, StatsK* __restrict__ st,
                                                         const DevTabs tabs) {
    eye_tile<FUSED, COUNT, RT, FMT, NOSH>(a.ey, a.sh, smap, out, blockIdx.x, blockIdx.y, st, tabs);
}

// The sphere-only eye pass (RT 0, materialised map) held to 8 waves per SIMD: the
// coded map's decode (smap_decode_wave) would otherwise take it to 66 VGPRs, 7 waves.
template <int FMT>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(8, 8))) void eye_pass8_kernel(
    const FrameArgs a, const double* __restrict__ smap, void* __restrict__ out, const DevTabs tabs) {
    eye_tile<false, false, 0, FMT>(a.ey, a.sh, smap, out, blockIdx.x, blockIdx.y, nullptr, tabs);
}

// The SDF eye instantiation (row f-4) with a register cap: WPE waves per SIMD at least.
template <int WPE, int FMT, bool NOSH = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void eye_sdf_kernel(
    const FrameArgs a, const double* __restrict__ smap, void* __restrict__ out, const DevTabs tabs) {
    eye_tile<false, false, 2, FMT, NOSH>(a.ey, a.sh, smap, out, blockIdx.x, blockIdx.y, nullptr, tabs);
}

// NOSH: frames whose shadow viewport is all +INF (no shadow raster, no march): the
// lookup is skipped (lit = +INF > qz, as the fused texel would give)
// RT 3: the batch's per-wave primitive masks, addressed from the kernel arguments
// (frame z's nw words at km + z * nw, nw = gx * rows) so that their load issues with the
// frame header's, not after it
// A RT 3 frame without shadows (main()'s scene and row f-1's bench, configs 6 and 7)
// has short waves: its batched workgroups render 4 tiles one after
// another, held to 8 waves per SIMD (62 VGPRs): configs 6 / 7 +1.5 % against one tile
// (profiles/r05_ab_eye_tiles.txt).  The table reads stay scalar loads after a tile's
// stores because the tables are read through constant-address-space pointers
// (const_table); the frame pointer is opaque per tile, so the header is re-read from the
// scalar cache rather than held in registers across the tiles (68 -> 62 VGPRs).
template <int RT, bool NOSH>
constexpr int eye_batch_tiles = RT == 3 && NOSH ? 4 : 1;
// The sphere-only batched eye pass on the materialised map (the headline kernel) is held
// to 8 waves per SIMD as well: 62 VGPRs, no scratch (the compiler's own allocation gave
// 68, 7 waves): configs 3 / 2 / 4 +2 % (profiles/r05_ab_eye_tiles.txt).  The fused one
// stays free: held to 8 it spills 20 B.
// block rows per workgroup in the 8 x 8 mode, one after another: config 7 294 -> 317
// Gpix/s against one (2: no gain; profiles/r05_ab_eye_blocks.txt)
constexpr int EYE_BLK_NT = 4;
template <bool FUSED, int RT, bool NOSH>
constexpr int eye_batch_wpe = RT == 3 && NOSH ? 8 : RT == 0 && !FUSED ? 8 : 1;
template <bool FUSED, int RT, int FMT, bool NOSH = false, bool BLK = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(eye_batch_wpe<FUSED, RT, NOSH>, 8))) void eye_batch_kernel(
    CBatch* __restrict__ fr, const uint32_t* __restrict__ km, int km_nw, int km_gx, int km_fs) {
    if (BLK) {
        // 8 x 8 blocks (eye_tile<BLK>): workgroup (bx, by) holds blocks 4 bx .. 4 bx + 3 of
        // block rows by + t * gridDim.y; km_gx = blocks per row; every block of the frame
        // has its word.  (Strided rows, not EYE_BLK_NT adjacent ones: a compact primitive's
        // blocks -- main()'s vertical cylinder -- no longer fall to the same wave one after
        // another, whose 4 traced tiles made the launch's tail: config 7's eye pass 0.97 ->
        // 0.90 us per frame one-lane, profiles/r06_ab_eye_variants.txt)
        const int col = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
        if (col >= km_gx) return;  // (wave-uniform: a block past the frame's right edge; no barrier follows)
        const int gy8 = (((const EyePart*)&fr[blockIdx.z].a.ey)->row_end - ((const EyePart*)&fr[blockIdx.z].a.ey)->row_begin + 7) / 8;
#pragma unroll 1
        for (int t = 0; t < EYE_BLK_NT; ++t) {
            const int by = (int)blockIdx.y + t * (int)gridDim.y;
            if (by >= gy8) break;  // (wave-uniform)
            CBatch* f = fr + blockIdx.z;
            if (EYE_BLK_NT > 1) asm volatile("" : "+s"(f));
            const DevTabs tabs = *(const DevTabs*)&f->tabs;
            const int widx = __builtin_amdgcn_readfirstlane(by * km_gx + col);
            const uint32_t kmw = ((const __attribute__((address_space(4))) uint32_t*)km)[(size_t)blockIdx.z * km_fs + widx];
            eye_tile<FUSED, false, RT, FMT, NOSH, BLK>(*(const EyePart*)&f->a.ey, *(const ShadowPart*)&f->a.sh, f->smap,
                                                       f->out, col, by, nullptr, tabs, true, kmw, true);
        }
        return;
    }
    constexpr int NT = eye_batch_tiles<RT, NOSH>;
#pragma unroll 1
    for (int t = 0; t < NT; ++t) {
        CBatch* f = fr + blockIdx.z;
        if (NT > 1) asm volatile("" : "+s"(f));
        const int by = (int)blockIdx.y * NT + t;
        const DevTabs tabs = *(const DevTabs*)&f->tabs;
        uint32_t kmw = 0u;
        int widx = 0;
        if (RT == 3) {
            widx = __builtin_amdgcn_readfirstlane((by * TILE_Y + (int)(threadIdx.x >> 6)) * km_gx + (int)blockIdx.x);
            kmw = ((const __attribute__((address_space(4))) uint32_t*)km)[(size_t)blockIdx.z * km_fs + min(widx, km_nw - 1)];
        }
        eye_tile<FUSED, false, RT, FMT, NOSH>(*(const EyePart*)&f->a.ey, *(const ShadowPart*)&f->a.sh, f->smap, f->out,
                                              blockIdx.x, by, nullptr, tabs, true, kmw, widx < km_nw);
    }
}

template <int WPE, int FMT, bool NOSH = false, bool BLK = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(WPE, 8))) void eye_sdf_batch_kernel(
    CBatch* __restrict__ fr, int gx8) {
    if (BLK) {  // 8 x 8 blocks, 4 across per workgroup, one block row (a row loop spills 360 B)
        const int col = (int)blockIdx.x * 4 + (int)(threadIdx.x >> 6);
        if (col >= gx8) return;  // (wave-uniform; no barrier follows)
        CBatch* f = fr + blockIdx.z;
        const DevTabs tabs = *(const DevTabs*)&f->tabs;
        eye_tile<false, false, 2, FMT, NOSH, BLK>(*(const EyePart*)&f->a.ey, *(const ShadowPart*)&f->a.sh, f->smap,
                                                   f->out, col, blockIdx.y, nullptr, tabs);
        return;
    }
    CBatch* f = fr + blockIdx.z;
    const DevTabs tabs = *(const DevTabs*)&f->tabs;
    eye_tile<false, false, 2, FMT, NOSH>(*(const EyePart*)&f->a.ey, *(const ShadowPart*)&f->a.sh, f->smap, f->out,
                                   blockIdx.x, blockIdx.y, nullptr, tabs);
}

// launch_upload: one 8-byte word per thread from the kernarg copy.
constexpr int UPLOAD_WORDS = 496;  // 3968 bytes: the chunk plus its two arguments fit 4 KiB of kernarg
struct UploadChunk {
    uint64_t w[UPLOAD_WORDS];
};
__global__ void upload_kernel(const UploadChunk k, uint64_t* __restrict__ dst, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = k.w[i];
}

// launch_pull: a batch table pulled from pinned host memory by the device, in the
// lane's stream order (16 bytes per thread, vector loads over PCIe, vector stores):
// one launch instead of an async copy, which goes to a copy engine (with its
// cross-queue waits) once the table passes a few tens of KB.
__global__ __launch_bounds__(BLOCK) void pull_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, int n) {
    for (int i = blockIdx.x * BLOCK + threadIdx.x; i < n; i += gridDim.x * BLOCK) dst[i] = src[i];
}

// Per-wave primitive masks of an eye pass under a PERSPECTIVE eye (RT 3): the
// cone cull of rt_wave_mask, one thread per wave of the eye pass (wave (bx, yl):
// pixels bx*64 .. bx*64+63 of row row_begin + yl), so the cone set-up and the
// bounding-sphere tests run once per wave instead of on every lane of it.  The
// same operations, hence the same masks.
// BLK: one thread per 8 x 8 pixel block of the eye pass (eye_batch_kernel<BLK>; no stripes)
template <bool BLK = false>
__device__ __forceinline__ void rt_cull_wave(const CamK& c, const RtK* __restrict__ rt, int W, int H, int row_begin,
                                             int rows, int4 stripes, uint32_t* __restrict__ masks, int t) {
    // the frame's slot terms, once per workgroup (lane l: slot l), then one wave per thread
    __shared__ CullK cq[32];
    const uint32_t slots = rt_slots(rt->n_pl, rt->n_cy);
    if (threadIdx.x < 32 && ((slots >> threadIdx.x) & 1u)) cull_prepare(rt, (int)threadIdx.x, c, cq[threadIdx.x]);
    __syncthreads();
    RayCone k;
    if (BLK) {
        const int gx8 = (W + 7) / 8, gy8 = (rows + 7) / 8;
        if (t >= gx8 * gy8) return;
        const int x0 = (t % gx8) * 8, y0 = row_begin + (t / gx8) * 8;
        const int y1 = min(min(y0 + 7, row_begin + rows - 1), H - 1);
        k = ray_cone_block(c, min(x0, W - 1), min(x0 + 7, W - 1), min(y0, H - 1), y1, W, H);
    } else {
        const int gx = (W + TILE_X - 1) / TILE_X;
        if (t >= gx * rows) return;
        const int xb = (t % gx) * TILE_X, yi = eye_row(row_begin, stripes.x, stripes.y, stripes.z, t / gx);
        k = ray_cone(c, min(xb, W - 1), min(xb + TILE_X - 1, W - 1), min(yi, H - 1), W, H);
    }
    uint32_t m = slots;
    for (uint32_t b = slots; b; b &= b - 1u) {
        const int l = __builtin_ctz(b);
        if (cull_test(k, cq[l])) m &= ~(1u << l);
    }
    masks[t] = m;
}

__global__ __launch_bounds__(BLOCK) void rt_cull_kernel(const CamK c, const RtK* __restrict__ rt, int W, int H,
                                                        int row_begin, int rows, int4 stripes,
                                                        uint32_t* __restrict__ masks) {
    rt_cull_wave(c, rt, W, H, row_begin, rows, stripes, masks, blockIdx.x * BLOCK + threadIdx.x);
}

// rt_cull_kernel for a batch: frame blockIdx.z's masks (frames with ray-traced
// primitives under a PERSPECTIVE eye get a mask buffer from the host; the others
// have none and skip).
template <bool BLK = false>
__global__ __launch_bounds__(BLOCK) void rt_cull_batch_kernel(CBatch* __restrict__ fr) {
    CBatch* f = fr + blockIdx.z;
    uint32_t* masks = f->tabs.rtmask;
    const RtK* rt = f->tabs.rt;
    if (!masks || !rt) return;
    const EyePart& e = *(const EyePart*)&f->a.ey;
    rt_cull_wave<BLK>(e.eye, rt, e.W, e.H, e.row_begin, e.row_end - e.row_begin,
                 make_int4(e.stripe_rows, e.stripe_stride, e.stripe_phase, 0), masks, blockIdx.x * BLOCK + threadIdx.x);
}

// ---- reference-seam kernels ----

// Viewport::rasterize (main.rs:445-547): spheres in order against the viewport's
// current zBuffer / G-buffer (rasterizeSphere, main.rs:304-330).
__global__ __launch_bounds__(BLOCK) void vp_rasterize_kernel(const RasterArgs a, double* __restrict__ zbuf,
                                                             double* __restrict__ gh, double* __restrict__ gz,
                                                             int32_t* __restrict__ gid) {
    const int xb = blockIdx.x * TILE_X;
    const int xi = xb + (threadIdx.x & (TILE_X - 1));
    const int yi = __builtin_amdgcn_readfirstlane(blockIdx.y * TILE_Y + (threadIdx.x >> 6));
    if (xi >= a.W || yi >= a.H) return;
    const int64_t idx = (int64_t)yi * a.W + xi;
    const double x = ndc(xi, a.W), y = ndc(yi, a.H);
    double zb = zbuf[idx];
    bool wrote = false;
    double wh = 0.0, wz = 0.0;
    int32_t wid = 0;
    for (int i = 0; i < a.n_spheres; ++i) {
        if (!may_cover(a.sph[i], xb, xb + TILE_X - 1, yi)) continue;
        double h;
        if (a.persp ? cover_persp(a.psp[i], x, y, h) : cover(a.sph[i], x, y, h)) {
            const double hr = h * a.sph[i].r;
            const double depth = a.face == RTM_FACE_FRONT ? a.sph[i].z - hr : a.sph[i].z + hr;
            if (depth < zb) {
                zb = depth;
                wrote = true;
                wh = h;
                wz = a.sph[i].z;
                wid = a.sph[i].id;
            }
        }
    }
    if (wrote) {
        zbuf[idx] = zb;
        gh[idx] = wh;
        gz[idx] = wz;
        gid[idx] = wid;
    }
}

// Viewport::processRaymarchingRays (main.rs:551-565)
__global__ __launch_bounds__(BLOCK) void vp_march_kernel(const MarchArgs a, double* __restrict__ zbuf) {
    const int xi = blockIdx.x * TILE_X + (threadIdx.x & (TILE_X - 1));
    const int yi = blockIdx.y * TILE_Y + (threadIdx.x >> 6);
    if (xi >= a.W || yi >= a.H) return;
    const int64_t idx = (int64_t)yi * a.W + xi;
    double o[3], d[3];
    cam_ray(a.cam, a.tab.nx[xi], a.tab.ny[yi], o, d);
    double zb = zbuf[idx];
    const double z0 = zb;
    for (int k = 0; k < a.n_patches; ++k) {
        MarchResult m = march<false>(o[0], o[1], o[2], d[0], d[1], d[2], a.patch[k], a.steps, a.tab);
        if (m.hit && m.t < zb) zb = m.t;
    }
    if (!(zb == z0)) zbuf[idx] = zb;
}

// Viewport::processRaytracingRays (main.rs:569-642) against the viewport's
// current zBuffer / G-buffer.
__global__ __launch_bounds__(BLOCK) void vp_trace_kernel(const TraceArgs a, double* __restrict__ zbuf,
                                                         double* __restrict__ gh, int32_t* __restrict__ gid,
                                                         double* __restrict__ gn) {
    const int xi = blockIdx.x * TILE_X + (threadIdx.x & (TILE_X - 1));
    const int yi = blockIdx.y * TILE_Y + (threadIdx.x >> 6);
    if (xi >= a.W || yi >= a.H) return;
    const int64_t idx = (int64_t)yi * a.W + xi;
    double o[3], d[3];
    cam_ray(a.cam, ndc(xi, a.W), ndc(yi, a.H), o, d);
    RtHit hit;
    hit.kind = 0;
    hit.id = 0;
    double zb = zbuf[idx];
    bool oob = false;
    if (a.rt) {
        const uint32_t slots = rt_slots(a.rt->n_pl, a.rt->n_cy);
        if (a.rt->persp) trace_pixel<true>(a.rt, o, d, zb, hit, slots, oob);
        else trace_pixel<false>(a.rt, o, d, zb, hit, slots, oob);
    }
    uint32_t evals = 0;
    if (a.sdf) trace_sdfs(a.sdf, o, d, zb, hit, evals, oob);
    if (__builtin_expect(oob, 0)) note_oob();
    if (hit.kind) {
        zbuf[idx] = hit.t;
        gh[idx] = hit.t;
        gid[idx] = (hit.kind == 2 ? GID_PLANE : hit.kind == 3 ? GID_CYLINDER : GID_SDF) | hit.id;
        if (hit.kind >= 3)
            for (int k = 0; k < 3; ++k) gn[3 * idx + k] = hit.n[k];
    }
}

// renderColorImage (main.rs:710-902) from a G-buffer.
__global__ __launch_bounds__(BLOCK) void vp_shade_kernel(const ShadeArgs a, const double* __restrict__ szbuf,
                                                         const double* __restrict__ gh,
                                                         const double* __restrict__ gz,
                                                         const int32_t* __restrict__ gid, float4* __restrict__ out) {
    const int xi = blockIdx.x * TILE_X + (threadIdx.x & (TILE_X - 1));
    const int yi = blockIdx.y * TILE_Y + (threadIdx.x >> 6);
    if (xi >= a.W || yi >= a.H) return;
    const int64_t idx = (int64_t)yi * a.W + xi;
    float4 c = make_float4(0.0f, 0.2f, 0.2f, 1.0f);
    const int32_t g = gid[idx];
    // the G-buffer id's table must hold it (the host checked the scene against what the
    // viewport holds, rtm_render_color_image; checked again per pixel: an id past its
    // table, or a null table, is counted and the pixel left as background)
    const int32_t gk = g >> 16, gi = g & 0xFFFF;
    const int32_t gn_ = gk == 0 ? a.n_spheres : gk == 1 ? (a.rt ? a.rt->n_pl : 0)
                      : gk == 2 ? (a.rt ? a.rt->n_cy : 0) : gk == 3 ? (a.sdf ? a.sdf->n : 0) : 0;
    const bool bad = g >= 0 && gi >= gn_;
    if (__builtin_expect(bad, 0)) note_oob();
    if (g >= 0 && !bad) {
        const int32_t kind = gk, id = gi;
        const double s01 = ndc(xi, a.W), u01 = ndc(yi, a.H);
        double o[3], d[3];
        cam_ray(a.eye, s01, u01, o, d);
        double view[3];
        if (a.eye.type == RTM_CAMERA_ORTHOGONAL) {
            for (int k = 0; k < 3; ++k) view[k] = a.eye.dir[k] * -1.0;
        } else {
            for (int k = 0; k < 3; ++k) view[k] = d[k] * -1.0;  // retViewDirOfPixel == -ray dir
        }
        double wx, wy, wz, nx, ny, nz, cr, cg, cb;
        if (kind == 0) {
            const ShadeSphereK& s = a.shade[id];
            const double depth = gz[idx] - gh[idx] * s.r;
            wx = o[0] + d[0] * depth;
            wy = o[1] + d[1] * depth;
            wz = o[2] + d[2] * depth;
            nx = (wx - s.px) * s.inv_r;
            ny = (wy - s.py) * s.inv_r;
            nz = (wz - s.pz) * s.inv_r;
            cr = s.cr;
            cg = s.cg;
            cb = s.cb;
        } else {
            const double depth = gh[idx];  // rayT
            wx = o[0] + d[0] * depth;
            wy = o[1] + d[1] * depth;
            wz = o[2] + d[2] * depth;
            if (kind == 1) {
                const PlaneK& p = a.rt->pl[id];
                nx = p.nx;
                ny = p.ny;
                nz = p.nz;
                cr = p.cr;
                cg = p.cg;
                cb = p.cb;
            } else {
                nx = a.gn[3 * idx];
                ny = a.gn[3 * idx + 1];
                nz = a.gn[3 * idx + 2];
                if (kind == 2) {
                    cr = a.rt->cy[id].cr;
                    cg = a.rt->cy[id].cg;
                    cb = a.rt->cy[id].cb;
                } else {
                    cr = a.sdf->s[id].cr;
                    cg = a.sdf->s[id].cg;
                    cb = a.sdf->s[id].cb;
                }
            }
        }
        const double Lx = 1.0 * -1.0, Ly = 0.0 * -1.0, Lz = 0.0 * -1.0;
        const double diffuse = fmax(nx * Lx + ny * Ly + nz * Lz, 0.0);
        const double k2 = -2.0 * (Lx * nx + Ly * ny + Lz * nz);
        const double Rx = Lx - nx * k2, Ry = Ly - ny * k2, Rz = Lz - nz * k2;
        double sp = fmax(view[0] * Rx + view[1] * Ry + view[2] * Rz, 0.0);
        sp = sp * sp;
        sp = sp * sp;
        sp = sp * sp;
        sp = sp * sp;
        sp = sp * sp;
        const double dfx = wx - a.shadow.pos[0], dfy = wy - a.shadow.pos[1], dfz = wz - a.shadow.pos[2];
        const double qx = dfx * a.shadow.side[0] + dfy * a.shadow.side[1] + dfz * a.shadow.side[2];
        const double qy = dfx * a.shadow.up[0] + dfy * a.shadow.up[1] + dfz * a.shadow.up[2];
        const double qz = dfx * a.shadow.dir[0] + dfy * a.shadow.dir[1] + dfz * a.shadow.dir[2];
        const int64_t hw = a.Ws / 2, hh = a.Hs / 2;
        const int64_t tx = tex_index(hw, qx * (double)hw);
        const int64_t ty = tex_index(hh, qy * (double)hh);
        double dsm = INFINITY;
        if (ty >= 0 && ty < a.Hs && tx >= 0 && tx < a.Ws) dsm = szbuf[ty * a.Ws + tx];
        const double lm = (dsm > qz - 0.0) ? 1.0 : 0.25;
        const double base = diffuse + sp;
        c.x = (float)((base * lm) * cr);
        c.y = (float)((base * lm) * cg);
        c.z = (float)((base * lm) * cb);
    }
    out[idx] = c;
}

__global__ void fill_kernel(double* __restrict__ p, int64_t n, double v, int32_t* __restrict__ ip, int32_t iv) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
        if (p) p[i] = v;
        if (ip) ip[i] = iv;
    }
}

}  // namespace

namespace {

inline dim3 grid_for(int w, int h) { return dim3((unsigned)((w + TILE_X - 1) / TILE_X), (unsigned)((h + TILE_Y - 1) / TILE_Y)); }

inline int launched() { return hipGetLastError() == hipSuccess ? 0 : RTM_ERR_HIP; }

}  // namespace

// Can the coded shadow tile render this frame's shadow pass?  It needs a coded map
// and, when the frame marches, the host-built records (a separable march camera with
// a monotone shared z table, rtm_api.cpp ensure_tables) and at most CODED_MAX_STEPS
// steps (its LDS table).  Everything else takes the generic tile.
static bool coded_ok(const ShadowPart& sh) {
    const bool march = !(sh.flags & RTM_FLAG_NO_MARCH) && sh.n_patches > 0 && sh.steps > 0;
    return sh.smap_fmt != SMAP_F64 &&
           (!march || (sh.tab.zrec && sh.tab.col && sh.tab.row && sh.steps <= CODED_MAX_STEPS));
}

// Launch the coded tile for one frame (FrameArgs) or a batch (fr != nullptr, n frames).
// box: the union over the frames of their spheres' pixel boxes (x0, x1, y0, y1), for the
// split launch (nullptr: sh's own).  The split: the workgroup tiles meeting the box run
// the full tile (PART 2), the others a raster-free instantiation with fewer registers
// (PART 1), when the box covers at most RTM_CODED_SPLIT_MAX (default 0.3) of the tiles
// (configs 2-4 split; config 5's 16 spheres span more: one launch there, measured as
// fast in the 4-lane frame and faster one-lane, profiles/r03_ab_coded_split.txt).
static void launch_coded(const ShadowPart& sh, const FrameArgs* a, double* smap, CBatch* fr, int n, hipStream_t s,
                         const int32_t* box = nullptr, bool one_launch = false) {
    const bool march = !(sh.flags & RTM_FLAG_NO_MARCH) && sh.n_patches > 0 && sh.steps > 0;
    const size_t lsm = march ? CODED_ROW_LDS + sizeof(ZRecK) * (size_t)(sh.steps + 1) : 0;
    constexpr int TR = CODED_TILE_ROWS;
    const int gx = (sh.W + 127) / 128, gy = (sh.H + TR - 1) / TR;
    dim3 g((unsigned)gx, (unsigned)gy, (unsigned)(fr ? n : 1));
    const bool inc = sh.tab.zmono >= 0;  // (no march: either instantiation is exact)
    const int4 org0 = make_int4(0, 0, TR, 0);
    // the split: workgroup tiles [bx0, bx1] x [by0, by1] meet some frame's box
    const int32_t bx_[4] = {sh.cull_x0, sh.cull_x1, sh.cull_y0, sh.cull_y1};
    const int32_t* b = box ? box : bx_;
    const bool raster = !(sh.flags & RTM_FLAG_NO_SHADOW_RASTER) && b[0] <= b[1] && b[2] <= b[3];
    const int bx0 = raster ? std::max(b[0], 0) / 128 : 0, bx1 = raster ? std::min(b[1] / 128, gx - 1) : -1;
    const int by0 = raster ? std::max(b[2], 0) / TR : 0;
    const int by1 = raster ? std::min(std::max(b[3], 0) / TR, gy - 1) : -1;
    const double box_frac = raster ? (double)std::max(bx1 - bx0 + 1, 0) * (double)std::max(by1 - by0 + 1, 0) /
                                         ((double)gx * (double)gy)
                                   : 0.0;
    // PART 2's workgroup tiles (one 16-row strip each) over the box's rows
    constexpr int TR2 = coded_tile_rows<2>;
    const int gy2 = (sh.H + TR2 - 1) / TR2;
    const int c0 = raster ? std::max(b[2], 0) / TR2 : 0;
    const int c1 = raster ? std::min(std::max(b[3], 0) / TR2, gy2 - 1) : -1;
    static const double split_max = [] {
        const char* e = getenv("RTM_CODED_SPLIT_MAX");
        return e ? atof(e) : 0.3;
    }();
    const bool split = box_frac <= split_max;
    dim3 gb((unsigned)std::max(bx1 - bx0 + 1, 0), (unsigned)std::max(c1 - c0 + 1, 0), g.z);
    const int4 orgb = make_int4(bx0, c0, TR2, 0);
#define RTM_CK(I, M, P, G, O)                                                                                     \
    do {                                                                                                        \
        if (fr) hipLaunchKernelGGL((shadow_coded_batch_kernel<I, M, P>), G, dim3(BLOCK), lsm, s, fr, O);          \
        else hipLaunchKernelGGL((shadow_coded_kernel<I, M, P>), G, dim3(BLOCK), lsm, s, *a, smap, O);            \
    } while (0)
    // PART 1's workgroup tiles: coded_tile_rows<1> rows (P1_STRIPS strips per wave)
    constexpr int TR1 = coded_tile_rows<1>;
    const dim3 g1(g.x, (unsigned)((sh.H + TR1 - 1) / TR1), g.z);
    // a batch whose lane runs alone: one launch of both parts (shadow_split_batch_kernel).
    // One-lane at config 3 it takes 29.7 us per 8-frame launch against 17.8 + 16.8 us for
    // the two launches; with 4 lanes the other lanes' kernels fill the gap between the two
    // launches and the merged kernel's registers (84 VGPRs for PART 2's waves, 62 alone)
    // cost 1-4 % of the frame rate, so lanes keep two (profiles/r06_ab_shadow.txt)
    const int n2 = (int)(gb.x * gb.y);
    const dim3 gs((unsigned)(n2 + (int)(g1.x * g1.y)), 1u, g.z);
    const int4 orgs = make_int4(bx0, c0, (int)gb.x, n2);
#define RTM_CKB(I, M)                                                                                        \
    do {                                                                                                     \
        if (split && fr && one_launch) {                                                                                \
            hipLaunchKernelGGL((shadow_split_batch_kernel<I, M>), gs, dim3(BLOCK), lsm, s, fr, orgs);         \
        } else if (split) {                                                                                  \
            if (gb.x > 0 && gb.y > 0) RTM_CK(I, M, 2, gb, orgb);                                             \
            RTM_CK(I, M, 1, g1, org0);                                                                       \
        } else {                                                                                             \
            RTM_CK(I, M, 0, g, org0);                                                                        \
        }                                                                                                    \
    } while (0)
    if (sh.smap_fmt == SMAP_U8) {
        if (inc) RTM_CKB(true, SMAP_U8);
        else RTM_CKB(false, SMAP_U8);
    } else {
        if (inc) RTM_CKB(true, SMAP_U16);
        else RTM_CKB(false, SMAP_U16);
    }
#undef RTM_CKB
#undef RTM_CK
}

int launch_shadow_pass(const FrameArgs& a, double* smap, void* stream, StatsK* stats) {
    hipStream_t s = (hipStream_t)stream;
    if (!stats && coded_ok(a.sh)) {
        launch_coded(a.sh, &a, smap, nullptr, 1, s);
        return launched();
    }
    if (stats)
        hipLaunchKernelGGL(shadow_pass_kernel<true>, grid_for(a.sh.W, a.sh.H), dim3(BLOCK), 0, s, a, smap, stats);
    else
        hipLaunchKernelGGL(shadow_pass_kernel<false>, grid_for(a.sh.W, a.sh.H), dim3(BLOCK), 0, s, a, smap, stats);
    return launched();
}

// Eye kernel of one frame (or of a batch: FR != nullptr, n frames, every frame with
// frame 0's shapes, flags, tables and variant):
//   * an all-+INF shadow viewport (fused, no shadow raster, no march; rtm_api.cpp
//     trivial_shadow): NOSH, no lookup at all (lit = +INF > qz, the fused texel's value);
//   * SDFs (row f-4) on the materialised map or NOSH: the SDF kernel held to 5 waves
//     per SIMD (95 VGPRs, no spill: eye 582 -> 565 us at config 8); fused: RT 2;
//   * ray-traced primitives under a PERSPECTIVE eye (row f-1): RT 3 (host-hoisted
//     origin terms, per-wave primitive masks); other ray-traced frames and PERSPECTIVE
//     spheres (row f-3): RT 1;
//   * spheres only on the materialised map: one frame held to 8 waves per SIMD
//     (eye_pass8_kernel); batched, the compiler's allocation (the headline kernel).
template <int FMT>
static void launch_eye_fmt(const FrameArgs& a, const double* smap, void* o, hipStream_t s, dim3 g, bool fused,
                           const DevTabs& tabs, CBatch* fr, bool blk = false, bool mask_shared = false) {
    struct {
        const uint32_t* p;
        int nw, gx, fs;
    } km{nullptr, 1, 1, 0};
    // (fs: frame z's words at z * fs; 0 when the batch's frames share one set, launch_eye_batch)
    if (fr && tabs.rtmask) km = {tabs.rtmask, tabs.rtmask_words, (int)g.x, mask_shared ? 0 : tabs.rtmask_words};
    // 8 x 8 blocks (eye_block_mode): 4 blocks per workgroup across, 8 rows
    const int rows_ = a.ey.row_end - a.ey.row_begin;
    const int gx8 = (a.ey.W + 7) / 8;
    const dim3 gblk((unsigned)((gx8 + 3) / 4), (unsigned)(((rows_ + 7) / 8 + EYE_BLK_NT - 1) / EYE_BLK_NT), g.z);
#define RTM_EYE(F, R, N)                                                                                           \
    do {                                                                                                        \
        constexpr bool B_ = R == 3 && N && FMT == RTM_FORMAT_RGBA32F;                                           \
        if (fr && B_ && blk)                                                                                    \
            hipLaunchKernelGGL((eye_batch_kernel<F, R, FMT, N, B_>), gblk, dim3(BLOCK), 0, s, fr, km.p, km.nw, gx8, km.fs); \
        else if (fr) hipLaunchKernelGGL((eye_batch_kernel<F, R, FMT, N>), dim3(g.x, (g.y + eye_batch_tiles<R, N> - 1) / eye_batch_tiles<R, N>, g.z), \
                                   dim3(BLOCK), 0, s, fr, km.p, km.nw, km.gx, km.fs);                              \
        else hipLaunchKernelGGL((eye_pass_kernel<F, false, R, FMT, N>), g, dim3(BLOCK), 0, s, a, smap, o, nullptr, tabs); \
    } while (0)
    // the SDF frames' batched eye pass in 8 x 8 pixel blocks as well (RGBA f32, no stripes):
    // neighbouring rays in two dimensions march alike, config 8 21.5 -> 22.6 Gpix/s
    // (profiles/r05_ab_eye_blocks.txt); one block row per workgroup (a row loop spills 360 B)
    const bool sblk = fr && FMT == RTM_FORMAT_RGBA32F && a.ey.stripe_rows == 0;
#define RTM_EYE_SDF(N)                                                                                              \
    do {                                                                                                        \
        constexpr bool SB_ = FMT == RTM_FORMAT_RGBA32F;                                                         \
        if (fr && SB_ && sblk) hipLaunchKernelGGL((eye_sdf_batch_kernel<5, FMT, N, SB_>), dim3(gblk.x, (rows_ + 7) / 8, g.z), \
                                                  dim3(BLOCK), 0, s, fr, gx8);                                   \
        else if (fr) hipLaunchKernelGGL((eye_sdf_batch_kernel<5, FMT, N>), g, dim3(BLOCK), 0, s, fr, gx8);       \
        else hipLaunchKernelGGL((eye_sdf_kernel<5, FMT, N>), g, dim3(BLOCK), 0, s, a, smap, o, tabs);            \
    } while (0)
    const int both = RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER;
    const bool nosh = fused && (a.sh.flags & both) == both;
    const int rt = tabs.sdf ? 2 : (tabs.rt && tabs.rt_persp) ? 3 : (tabs.rt || tabs.psp) ? 1 : 0;
    if (nosh) {
        if (rt == 2) RTM_EYE_SDF(true);
        else if (rt == 3) RTM_EYE(false, 3, true);
        else if (rt == 1) RTM_EYE(false, 1, true);
        else RTM_EYE(false, 0, true);
    } else if (rt == 2) {
        if (fused) RTM_EYE(true, 2, false);
        else RTM_EYE_SDF(false);
    } else if (rt == 3) {
        if (fused) RTM_EYE(true, 3, false);
        else RTM_EYE(false, 3, false);
    } else if (rt == 1) {
        if (fused) RTM_EYE(true, 1, false);
        else RTM_EYE(false, 1, false);
    } else if (fused) {
        RTM_EYE(true, 0, false);
    } else if (fr) {
        RTM_EYE(false, 0, false);
    } else {
        hipLaunchKernelGGL((eye_pass8_kernel<FMT>), g, dim3(BLOCK), 0, s, a, smap, o, tabs);
    }
#undef RTM_EYE_SDF
#undef RTM_EYE
}

int launch_eye_pass(const FrameArgs& a, const double* smap, void* out, void* stream, StatsK* stats,
                    const DevTabs& tabs) {
    hipStream_t s = (hipStream_t)stream;
    const int rows = a.ey.row_end - a.ey.row_begin;
    dim3 g = grid_for(a.ey.W, rows);
    const bool fused = (a.ey.flags & RTM_FLAG_FUSED_SHADOW) != 0;
    const int fmt = tabs.fmt & FMT_MASK;
    if (stats) {  // counting kernels: RGBA f32 output only
        if (fmt != RTM_FORMAT_RGBA32F) return RTM_ERR_INVALID;
#define RTM_EYE(F, R) \
    hipLaunchKernelGGL((eye_pass_kernel<F, true, R, RTM_FORMAT_RGBA32F>), g, dim3(BLOCK), 0, s, a, smap, out, stats, tabs)
        const int rt = tabs.sdf ? 2 : (tabs.rt || tabs.psp) ? 1 : 0;
        if (rt == 2) {
            if (fused) RTM_EYE(true, 2);
            else RTM_EYE(false, 2);
        } else if (rt == 1) {
            if (fused) RTM_EYE(true, 1);
            else RTM_EYE(false, 1);
        } else {
            if (fused) RTM_EYE(true, 0);
            else RTM_EYE(false, 0);
        }
#undef RTM_EYE
        return launched();
    }
    DevTabs t = tabs;
    if (t.rt && t.rt_persp && !t.sdf && t.rtmask) {
        // the per-wave primitive masks (RT 3): one thread per wave of the eye pass
        const int n = ((a.ey.W + TILE_X - 1) / TILE_X) * rows;
        hipLaunchKernelGGL(rt_cull_kernel, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, a.ey.eye,
                           t.rt, a.ey.W, a.ey.H, a.ey.row_begin, rows,
                           make_int4(a.ey.stripe_rows, a.ey.stripe_stride, a.ey.stripe_phase, 0), t.rtmask);
    } else {
        t.rtmask = nullptr;
    }
    if (fmt == RTM_FORMAT_RGBA8) launch_eye_fmt<RTM_FORMAT_RGBA8>(a, smap, out, s, g, fused, t, nullptr);
    else if (fmt == RTM_FORMAT_RGB8) launch_eye_fmt<RTM_FORMAT_RGB8>(a, smap, out, s, g, fused, t, nullptr);
    else launch_eye_fmt<RTM_FORMAT_RGBA32F>(a, smap, out, s, g, fused, t, nullptr);
    return launched();
}

int launch_shadow_batch(const BatchFrame* dev, int n, const FrameArgs& a0, void* stream, const int32_t* box,
                        bool one_launch) {
    hipStream_t s = (hipStream_t)stream;
    CBatch* fr = (CBatch*)dev;
    const ShadowPart& sh = a0.sh;
    if (coded_ok(sh)) {
        launch_coded(sh, nullptr, nullptr, fr, n, s, box, one_launch);
        return launched();
    }
    dim3 g = grid_for(sh.W, sh.H);
    g.z = (unsigned)n;
    hipLaunchKernelGGL(shadow_pass_batch_kernel, g, dim3(BLOCK), 0, s, fr);
    return launched();
}

// The shadow map's storage for these arguments (rtm_kernels.h): coded when every code
// fits (steps + n_spheres codes plus +INF) -- the coded tile and the generic tile both
// write codes -- else f64; RTM_SMAP=f64 forces the 8-byte map (tests/test_smap_codes.py:
// the generic tile's f64 map must give the same image).
int32_t shadow_map_format(const ShadowPart& sh) {
    static const bool f64_env = [] {
        const char* e = getenv("RTM_SMAP");
        return e && (std::string(e) == "f64" || std::string(e) == "0");
    }();
    if (f64_env) return SMAP_F64;
    const int64_t codes = (int64_t)sh.steps + sh.n_spheres;  // + the all-ones +INF code
    if (codes <= 254) return SMAP_U8;
    if (codes <= 65534 && sh.tab.t) return SMAP_U16;
    return SMAP_F64;
}

// Span records come with a U8 map whose shadow pass is the coded tile (launch_coded): its
// waves write them (shadow_tile_coded); the generic tile writes block bytes only.
int32_t shadow_map_spans(const ShadowPart& sh) { return sh.smap_fmt == SMAP_U8 && coded_ok(sh) ? 1 : 0; }

__global__ __launch_bounds__(BLOCK) void smap_decode_kernel(const ShadowPart sh, const void* __restrict__ codes,
                                                            double* __restrict__ out) {
    const int x = blockIdx.x * BLOCK + threadIdx.x;
    const int y = blockIdx.y;
    if (x < sh.W) out[(int64_t)y * sh.W + x] = smap_decode(sh, codes, x, y);
}

int launch_smap_decode(const ShadowPart& sh, const void* codes, double* out, void* stream) {
    if (sh.smap_fmt == SMAP_F64 || sh.W < 1 || sh.H < 1) return RTM_ERR_INVALID;
    hipLaunchKernelGGL(smap_decode_kernel, dim3((unsigned)((sh.W + BLOCK - 1) / BLOCK), (unsigned)sh.H), dim3(BLOCK),
                       0, (hipStream_t)stream, sh, codes, out);
    return launched();
}

// The batch's eye pass in 8 x 8 pixel blocks (eye_tile<BLK>) for frames below 1 Mpixel:
// RT 3 frames without shadows (the NOSH kernel), RGBA f32, no stripes, and every block's
// mask word inside the frame's mask slot (ceil(W/8) * ceil(rows/8) <= ceil(W/64) * rows
// words).  main()'s scene at 512 x 512 (config 7): its cylinder meets 2.4 % of the blocks
// against 13.6 % of the 64 x 1 rows, and the eye kernel runs a 64-frame launch in 66 instead
// of 113 us one lane: 234 -> 293 Gpix/s, 317 with 4 block rows per workgroup.  At 3840 x
// 2160 (config 6: 13 primitives) blocks at 4 rows per workgroup match the 64 x 1 rows (one
// block row: 3 % slower); larger frames keep rows (profiles/r05_ab_eye_blocks.txt).
static bool eye_block_mode(const FrameArgs& a0, const DevTabs& t0, bool fused) {
    const int both = RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER;
    const bool nosh = fused && (a0.sh.flags & both) == both;
    const int rows = a0.ey.row_end - a0.ey.row_begin;
    const int64_t nw8 = (int64_t)((a0.ey.W + 7) / 8) * ((rows + 7) / 8);
    return nosh && t0.rt && t0.rt_persp && !t0.sdf && t0.rtmask && (t0.fmt & FMT_MASK) == RTM_FORMAT_RGBA32F &&
           a0.ey.stripe_rows == 0 && nw8 <= (int64_t)t0.rtmask_words &&
           (int64_t)a0.ey.W * rows < (1 << 20);
}

int launch_eye_batch(const BatchFrame* dev, int n, const FrameArgs& a0, const DevTabs& t0, void* stream,
                     int* blocks, bool mask_shared, bool cull) {
    hipStream_t s = (hipStream_t)stream;
    CBatch* fr = (CBatch*)dev;
    const int rows = a0.ey.row_end - a0.ey.row_begin;
    const bool fused = (a0.ey.flags & RTM_FLAG_FUSED_SHADOW) != 0;
    const bool blk = eye_block_mode(a0, t0, fused);
    // (the SDF batches take blocks under their own rule, launch_eye_fmt's sblk)
    const bool sdf_blk = t0.sdf && (t0.fmt & FMT_MASK) == RTM_FORMAT_RGBA32F && a0.ey.stripe_rows == 0 &&
                         !(fused && !((a0.sh.flags & (RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER)) ==
                                      (RTM_FLAG_NO_MARCH | RTM_FLAG_NO_SHADOW_RASTER)));
    if (blocks) *blocks = blk || sdf_blk;
    if (t0.rtmask && cull) {  // the batch's per-wave primitive masks first (RT 3)
        // (mask_shared: every frame has frame 0's camera and primitive table, so frame 0's
        // masks are every frame's: one frame's cull)
        const int nm = mask_shared ? 1 : n;
        if (blk) {
            const int nw8 = ((a0.ey.W + 7) / 8) * ((rows + 7) / 8);
            hipLaunchKernelGGL(rt_cull_batch_kernel<true>, dim3((unsigned)((nw8 + BLOCK - 1) / BLOCK), 1, (unsigned)nm),
                               dim3(BLOCK), 0, s, fr);
        } else {
            const int nw = ((a0.ey.W + TILE_X - 1) / TILE_X) * rows;
            hipLaunchKernelGGL(rt_cull_batch_kernel<false>, dim3((unsigned)((nw + BLOCK - 1) / BLOCK), 1, (unsigned)nm),
                               dim3(BLOCK), 0, s, fr);
        }
        if (launched()) return RTM_ERR_HIP;
    }
    dim3 g = grid_for(a0.ey.W, rows);
    g.z = (unsigned)n;
    const int fmt = t0.fmt & FMT_MASK;
    if (fmt == RTM_FORMAT_RGBA8) launch_eye_fmt<RTM_FORMAT_RGBA8>(a0, nullptr, nullptr, s, g, fused, t0, fr, false, mask_shared);
    else if (fmt == RTM_FORMAT_RGB8) launch_eye_fmt<RTM_FORMAT_RGB8>(a0, nullptr, nullptr, s, g, fused, t0, fr, false, mask_shared);
    else launch_eye_fmt<RTM_FORMAT_RGBA32F>(a0, nullptr, nullptr, s, g, fused, t0, fr, blk, mask_shared);
    return launched();
}


int read_oob_reads(unsigned long long* count, void* stream) {
    const unsigned long long zero = 0ull;
    if (hipMemcpyFromSymbolAsync(count, HIP_SYMBOL(g_oob_reads), sizeof zero, 0, hipMemcpyDeviceToHost,
                                 (hipStream_t)stream) != hipSuccess ||
        hipMemcpyToSymbolAsync(HIP_SYMBOL(g_oob_reads), &zero, sizeof zero, 0, hipMemcpyHostToDevice,
                               (hipStream_t)stream) != hipSuccess ||
        hipStreamSynchronize((hipStream_t)stream) != hipSuccess)
        return RTM_ERR_HIP;
    return 0;
}

int launch_pull(const void* src_host, size_t bytes, void* dst, void* stream) {
    if (bytes % 16 || ((uintptr_t)src_host & 15) || ((uintptr_t)dst & 15)) return RTM_ERR_INVALID;
    const int n = (int)(bytes / 16);
    if (n == 0) return 0;
    const int blocks = std::min((n + BLOCK - 1) / BLOCK, 64);
    hipLaunchKernelGGL(pull_kernel, dim3((unsigned)blocks), dim3(BLOCK), 0, (hipStream_t)stream,
                       (const uint4*)src_host, (uint4*)dst, n);
    return launched();
}

int launch_upload(const void* src, size_t bytes, void* dst, void* stream) {
    if (bytes % 8) return RTM_ERR_INVALID;
    const uint64_t* s8 = static_cast<const uint64_t*>(src);
    uint64_t* d8 = static_cast<uint64_t*>(dst);
    for (size_t w = 0, nw = bytes / 8; w < nw; w += UPLOAD_WORDS) {
        UploadChunk c;
        const int n = (int)std::min<size_t>(UPLOAD_WORDS, nw - w);
        std::copy(s8 + w, s8 + w + n, c.w);
        hipLaunchKernelGGL(upload_kernel, dim3(1), dim3(512), 0, (hipStream_t)stream, c, d8 + w, n);
        if (launched()) return RTM_ERR_HIP;
    }
    return 0;
}


int launch_vp_rasterize(const RasterArgs& a, double* zbuf, double* gh, double* gz, int32_t* gid, void* stream) {
    hipLaunchKernelGGL(vp_rasterize_kernel, grid_for(a.W, a.H), dim3(BLOCK), 0, (hipStream_t)stream, a, zbuf, gh,
                       gz, gid);
    return launched();
}

int launch_vp_march(const MarchArgs& a, double* zbuf, void* stream) {
    hipLaunchKernelGGL(vp_march_kernel, grid_for(a.W, a.H), dim3(BLOCK), 0, (hipStream_t)stream, a, zbuf);
    return launched();
}

int launch_vp_shade(const ShadeArgs& a, const double* szbuf, const double* gh, const double* gz, const int32_t* gid,
                    float* out, void* stream) {
    hipLaunchKernelGGL(vp_shade_kernel, grid_for(a.W, a.H), dim3(BLOCK), 0, (hipStream_t)stream, a, szbuf, gh, gz,
                       gid, reinterpret_cast<float4*>(out));
    return launched();
}

int launch_vp_trace(const TraceArgs& a, double* zbuf, double* gh, int32_t* gid, double* gn, void* stream) {
    hipLaunchKernelGGL(vp_trace_kernel, grid_for(a.W, a.H), dim3(BLOCK), 0, (hipStream_t)stream, a, zbuf, gh, gid, gn);
    return launched();
}

int launch_fill(double* p, int64_t n, double v, int32_t* ip, int32_t iv, void* stream) {
    if (n <= 0) return 0;
    int64_t blocks = (n + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    hipLaunchKernelGGL(fill_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, p, n, v, ip, iv);
    return launched();
}

}  // namespace rtm
