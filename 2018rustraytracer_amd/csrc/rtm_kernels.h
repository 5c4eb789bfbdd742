// rtm_kernels.h — kernel-argument structs shared by the host library and the
// HIP kernels.  Every scene constant the reference recomputes per pixel but
// that depends only on (camera, sphere) is evaluated once on the host, in the
// reference's floating-point operation order, and travels to the GPU as a
// kernel argument (constant memory, read through the scalar cache into SGPRs).
#pragma once

#include <stdint.h>

#include "../../include/rtm.h"

namespace rtm {

// One sphere as seen by one ORTHOGONAL camera (Viewport::rasterize, main.rs:449-470).
// axisA=(r,0), axisB=(0,r): axisA.normalized()=(n, 0*(1/m)), axisB.normalized()=(0*(1/m), n),
// |axisA|=|axisB|=m (main.rs:2849-2850, 2098-2109).  The 0*(1/m) terms only ever add
// a signed zero (or turn an already-missing pixel into NaN), which cannot change
// d = sqrt(pa^2 + pb^2) < 1, so pa = (rel.x*n)/m and pb = (rel.y*n)/m.
struct RasterSphereK {
    double cx, cy;  // Camera::project(pos).xy (main.rs:455, 464)
    double z;       // calcDepthOfProjectedPoint(pos) (main.rs:450)
    double r;       // the r rasterizeSphere multiplies relativeHeight by (main.rs:541, 316)
    double n;       // r*(1/m)
    double m;       // sqrt(r*r + 0*0)
    int32_t id;     // PrimitiveSphere.id -> G-buffer (main.rs:189)
    // Pixel-index ranges outside which no pixel can be covered (the reference's
    // screen-space bbox, main.rs:256-300, made exact): column xi can be covered
    // only if ix0 <= xi <= ix1, row yi only if iy0 <= yi <= iy1.  Empty: ix0 > ix1.
    int32_t ix0, ix1, iy0, iy1;
    int32_t pad;
};
static_assert(sizeof(RasterSphereK) == 72, "RasterSphereK layout");

// Per-sphere shading constants, indexed by id (renderColorImage, main.rs:748-759).
struct ShadeSphereK {
    double px, py, pz;  // pos
    double r;           // calcDepth's primitiveSphere.r (main.rs:160)
    double inv_r;       // 1.0/r (main.rs:752)
    double cr, cg, cb;  // shading
};

struct CamK {  // ORTHOGONAL or PERSPECTIVE camera (main.rs:1887-1898)
    double pos[3], dir[3], up[3], side[3];
    int32_t type;
    int32_t pad;
};

// Bilinear patch with the linear() differences b-a precomputed (main.rs:2066-2068).
struct PatchK {
    double a0, d0;  // _0.a, _0.b - _0.a
    double a1, d1;  // _1.a, _1.b - _1.a
};

// Host-built lookup tables (device memory, owned by the context), all computed
// with the reference's operations in its order:
//   t[k]   = t after k march advances: t_0 = 0.0, t_{k+1} = t_k + 0.03 (main.rs:2237, 2273)
//   nx[i]  = ((i as f64) / (W as f64)) * 2.0 - 1.0  (main.rs:306, 1903-1906), ny likewise
//   z[k]   = p.z after k advances when every shadow texel starts at the same z
//            (z_0 = z0, z_{k+1} = z_k + step.z, main.rs:2272)
// Separable shadow camera (host-proved: p.x of the domain-mapped ray start depends
// only on the column and p.y only on the row, bit for bit):
//   py[j]          = p.y of row j                        (main.rs:2188)
//   d0[k*W + i]    = _0.a + (_0.b - _0.a) * p.x(i)       (linear, main.rs:2074)
//   dd[k*W + i]    = (_1.a + (_1.b - _1.a) * p.x(i)) - d0 (main.rs:2075, 2077 diff)
//   ok[i] / ok[W+j] = inRange01(p.x(i)) / inRange01(p.y(j)) (main.rs:2249)
//   so the surface depth is D = d0 + dd * py (main.rs:2077, one mul + one add).
// z_{k+1} = fl(z_k + step.z) is monotone in k (rounding is monotone), which the
// host re-checks entry by entry before setting zmono.
// Records of the coded shadow tile (shadow_tile_coded), host-built with the tables
// below when the march camera is separable and the z table monotone:
//   ZRecK[k], k in [0, steps]: (z_{k-1}, z_k, t_k) -- one LDS read yields both table
//     entries the first-crossing check compares and the hit's t.  k == steps holds
//     z = +-INF (the side "past the surface" for the table's direction) and t = +INF,
//     so a guess of `steps` is never a winning hit and needs no separate test.
//   ColRecK[p*W + i]: patch p's column terms d0, dd (below) + the f32 guess terms
//     g0 = (d0 - z0)/sz, g1 = dd/sz (index guess ceil(g0 + g1*py) ~ the first k with
//     z_k past D: a guess only, checked against the table) + inRange01 of the column.
//   RowRecK[j]: py[j], (f32) py[j], inRange01 of the row; the table is padded to a
//     multiple of 64 rows with rows that do not march (ok = 0).
struct ZRecK {
    double zprev, z, t, pad;
};
struct ColRecK {
    double d0, dd;
    float g0, g1;
    int32_t ok, pad;
};
struct RowRecK {
    double py;
    float pyf;
    int32_t ok;
};
struct RowRec4K {  // the 4 rows of a coded-map block: one 64-byte scalar load
    RowRecK r[4];
};
static_assert(sizeof(ZRecK) == 32 && sizeof(ColRecK) == 32 && sizeof(RowRecK) == 16 && sizeof(RowRec4K) == 64,
              "record layouts");

struct Tables {
    const ZRecK* zrec;    // coded-tile records (see above), or nullptr
    const ColRecK* col;   // n_patches*W, or nullptr
    const RowRecK* row;   // H rounded up to 64 (padding: ok = 0), or nullptr
    const double* t;   // steps entries, or nullptr when steps > RTM_T_TABLE_MAX
    const double* nx;  // W entries
    const double* ny;  // H entries
    const double* z;   // steps entries, or nullptr (no shared z sequence)
    const double* py;  // H entries, or nullptr (not separable)
    const double* d0;  // n_patches*W
    const double* dd;  // n_patches*W
    const int32_t* ok; // W + H
    int32_t zmono;     // z table (first `steps` entries) is non-decreasing (+1) / non-increasing (-1)
    int32_t row_recs;  // RowRecK entries (H rounded up to 64; every read is bounds-checked against it)
    double z0;         // z[0] when z != nullptr (a kernarg copy: no dependent global load for it)
    double inv_sz;     // 1.0 / step.z when z != nullptr (the first-crossing guess's scale)
    double sz;         // step.z = dir.z * 0.03 when z != nullptr (main.rs:2233; a kernarg: an SGPR pair, not
                       // a VGPR-held f64 literal the coded tile would spill)
};
#define RTM_T_TABLE_MAX 65536

// What the shadow pass of one frame reads (shadow viewport rasterize + march).
struct ShadowPart {
    RasterSphereK sph[RTM_MAX_SPHERES];  // shadow camera projection
    PatchK patch[RTM_MAX_PATCHES];
    CamK cam;                            // shadow camera
    Tables tab;                          // shadow-map dims
    int32_t W, H;                        // shadow map (== eye image dims)
    int32_t n_spheres, n_patches;
    int32_t steps, flags;
    int32_t cull_x0, cull_x1, cull_y0, cull_y1;  // union of the spheres' pixel ranges (see EyePart)
    int32_t smap_fmt;  // SMAP_F64 / SMAP_U8 / SMAP_U16: how the shadow pass stores the map (shadow_map_format)
    // (two 16-bit fields: FrameArgs must not grow, see the kernarg check below)
    int16_t smap_bw;     // coded maps: blocks per block row, ceil(W / 128) <= 256
    int16_t smap_spans;  // 1: the U8 map carries span records after its codes (shadow_map_spans)
};

// The shadow map's storage.  Every texel's value is one of +INF, a sphere's
// back-face depth at that texel, or t_k (the march's t after k advances, a table
// entry), so a coded map stores WHICH: code k < steps = t_k, steps + i = sphere i's
// depth there (recomputed by the reader with the writer's operations: same bits),
// all ones = +INF.  The codes are tiled in blocks of 128 columns x 4 rows, one
// block per shadow wave: texel (x, y) is element
//   ((y >> 2) * smap_bw + (x >> 7)) * 512 + ((x & 127) >> 1) * 8 + (y & 3) * 2 + (x & 1)
// (the coded tile's lane holds 4 rows x 2 columns = 8 codes, stored as 8 or 16
// contiguous bytes).  1 or 2 bytes per texel instead of 8.
constexpr int32_t SMAP_F64 = 0, SMAP_U8 = 1, SMAP_U16 = 2;
constexpr int64_t smap_code_index(int x, int y, int bw) {
    return ((int64_t)(y >> 2) * bw + (x >> 7)) * 512 + ((x & 127) >> 1) * 8 + (y & 3) * 2 + (x & 1);
}
// Span records (round 6; a U8 map written by the coded tile, ShadowPart::smap_spans).
// Down a column of a strip that marches one patch and meets no sphere, the codes are one
// monotone run (shadow_tile_coded): over a 64-row span they are a top code, a bottom code
// and the row where the bottom code starts.  Such a span is stored as that record alone,
// 4 bytes per column instead of 64 -- the raster-free waves, most of the map, then store
// 1/16 of the bytes.  Every other span has the record SPAN_DENSE and its codes in the
// blocks above.  Record of column x in span s = y >> 6: element s * (smap_bw * 128) + x of
// the table that starts at smap_span_offset; value top | bottom << 8 | boundary << 16
// (rows [0, boundary) of the span hold top).  A reader loads the record and the block
// byte together and keeps the byte only for SPAN_DENSE: the same code, so the same bits.
constexpr int SPAN_ROWS = 64;
constexpr uint32_t SPAN_DENSE = 0xFFFFFFFFu;
constexpr int64_t smap_span_index(int x, int y, int bw) { return (int64_t)(y >> 6) * bw * 128 + x; }
constexpr int64_t smap_span_offset(int32_t W, int32_t H) {
    return ((int64_t)((W + 127) / 128) * ((H + 3) / 4) * 512 + 255) & ~(int64_t)255;
}
// bytes of a shadow map of W x H texels in format fmt (spans: with span records)
inline int64_t smap_bytes(int32_t fmt, int32_t W, int32_t H, int32_t spans = 0) {
    if (fmt == SMAP_F64) return (int64_t)W * H * 8;
    if (fmt == SMAP_U8 && spans)
        return smap_span_offset(W, H) + (int64_t)((H + SPAN_ROWS - 1) / SPAN_ROWS) * ((W + 127) / 128) * 128 * 4;
    return (int64_t)((W + 127) / 128) * ((H + 3) / 4) * 512 * (fmt == SMAP_U8 ? 1 : 2);
}

// What the eye pass of one frame reads (eye viewport rasterize + renderColorImage).
struct EyePart {
    RasterSphereK sph[RTM_MAX_SPHERES];  // eye camera projection
    ShadeSphereK shade[RTM_MAX_SPHERES];
    CamK eye, shadow;                    // shadow: Camera::project for the lookup (main.rs:836)
    const double* nx;                    // eye NDC tables (Tables::nx / ny)
    const double* ny;
    int32_t W, H;                        // eye image
    int32_t Ws, Hs;                      // shadow map
    int32_t n_spheres, flags;
    int32_t row_begin, row_end;
    // union of the spheres' pixel ranges (empty: cull_x0 > cull_x1): a wave
    // outside it skips the per-sphere culls
    int32_t cull_x0, cull_x1, cull_y0, cull_y1;
    // [row_begin, row_end) are the launch's local rows; local row j renders image row
    // eye_row(j) = row_begin + j, or with cyclic stripes (stripe_rows > 0: the multi-GPU
    // frame's balanced partition, rtm_group) stripe_phase + (j / stripe_rows) *
    // stripe_stride + j % stripe_rows, clipped to H.  out_global: the output is the
    // whole image (row eye_row(j) of it), else the launch's rows (row j).
    int32_t stripe_rows, stripe_stride, stripe_phase, out_global;
};

// One launch's arguments: the shadow pass and the eye pass of one frame.  Kept
// < 4 KiB (kernarg limit).
struct FrameArgs {
    ShadowPart sh;
    EyePart ey;
};
static_assert(sizeof(FrameArgs) <= 4096, "FrameArgs must fit the 4 KiB kernarg segment");

// Ray-traced primitives of one frame (row f-1: processRaytracingRays,
// main.rs:569-642), with the ray-independent parts of calcRayPlane /
// iCappedCone evaluated once on the host in the reference's operation order.
// Lives in device memory (too large to share the 4 KiB kernarg segment with
// FrameArgs); written per frame by a stream-ordered upload kernel.
// With a PERSPECTIVE eye every ray starts at the camera position (main.rs:1922-1939),
// so every term of calcRayPlane / iCappedCone that involves only the origin is a
// per-(camera, primitive) constant: the host evaluates it once, in the reference's
// operation order (RtK::persp), and the kernel keeps only the terms with the ray
// direction -- the same bits, about half the per-pixel work.
struct PlaneK {            // PrimitiveCirclePlane (main.rs:370-380)
    double cx, cy, cz;     // pos (Plane.center)
    double nx, ny, nz;     // n
    double radius;
    double r2max;          // largest s with sqrt(s) <= radius (host libm sqrt): the radius test
                           // !(sqrt(s) > radius) is exactly !(s > r2max), no device sqrt
    double cr, cg, cb;     // shading
    double num;            // persp: dot(pos - origin, n), calcRayPlane's numerator (main.rs:2402)
    int32_t id, pad;
};
struct CylK {              // PrimitiveCappedCylinder (main.rs:382-391)
    double pa[3], pb[3];
    double ba[3];          // pb - pa                   (main.rs:2906)
    double ra, rb;
    double baba;           // dot(ba, ba)               (main.rs:2910)
    double rr;             // rb - ra                   (main.rs:2933)
    double hy;             // baba + rr*rr              (main.rs:2934)
    double isq;            // inversesqrt(baba) = 1.0/sqrt(baba) (main.rs:2919, 2963)
    double cr, cg, cb;
    // persp: the origin-only terms of iCappedCone (main.rs:2907-2936)
    double oa[3], ob[3];   // ro - pa, ro - pb
    double oaba, obba;     // dot(oa, ba), dot(ob, ba)
    double oc[3];          // oa*rb - ob*ra
    double ocba;           // dot(oc, ba)
    double bb;             // baba*baba
    double k0;             // baba*baba*dot(oc, oc) - hy*ocba*ocba
    int32_t id, pad;
};
struct RtK {
    PlaneK pl[RTM_MAX_CIRCLE_PLANES];
    CylK cy[RTM_MAX_CAPPED_CYLINDERS];
    int32_t n_pl, n_cy;
    int32_t persp, pad;    // the persp fields hold the eye camera's constants (PERSPECTIVE eye)
};
static_assert(sizeof(PlaneK) == 104 && sizeof(CylK) == 264, "RtK layout");
static_assert(sizeof(RtK) % 8 == 0, "RtK is uploaded in 8-byte words");

// One sphere as seen by a PERSPECTIVE camera (row f-3; Viewport::rasterize,
// main.rs:473-524 + projectSphere, main.rs:2796-2837): the ellipse centre and
// its two (perpendicular, not axis-aligned) axes as calcEllipseDistToCenter uses
// them (main.rs:2848-2852): n = axis.normalized(), m = axis.magnitude().
// z, r, id and the pixel ranges stay in the RasterSphereK of the same index.
struct PerspSphK {
    double cx, cy;
    double nAx, nAy, nBx, nBy;
    double mA, mB;
};
struct PerspK {
    PerspSphK s[RTM_MAX_SPHERES];
};

// The GL preview's SDF implicit surface (row f-4, entry.frag:416-442, 842-905),
// with udTriangleSingle's point-independent terms precomputed on the host in
// the restatement's operation order (oracle/rtm_oracle.c).
struct SdfK {
    double box[3];                       // descriptor vecs[0]
    double v1[3], v2[3], v3[3];          // triangle
    double e21[3], e32[3], e13[3];       // v2-v1, v3-v2, v1-v3
    double nor[3];                       // cross(v21, v13)
    double c1[3], c2[3], c3[3];          // cross(v21,nor), cross(v32,nor), cross(v13,nor)
    double d21, d32, d13, dnor;          // dot2 of the edges and of nor
    double ac[3], ae[3];                 // AABB centre / extent
    double cr, cg, cb;
    int32_t id, steps;
};
struct SdfTabK {
    SdfK s[RTM_MAX_SDFS];
    int32_t n, pad;
};
static_assert(sizeof(PerspK) % 8 == 0 && sizeof(SdfTabK) % 8 == 0, "device tables are uploaded in 8-byte words");


// The device tables a frame may carry beside FrameArgs (each nullptr when absent),
// and the eye pass's output format.
struct DevTabs {
    const RtK* rt;        // circle planes + capped cylinders (f-1)
    const PerspK* psp;    // PERSPECTIVE eye sphere projections (f-3)
    const SdfTabK* sdf;   // SDF implicit surfaces (f-4)
    // writeColorImage's encode (row f-2) as the eye pass's epilogue: the device
    // EncodeTable (rtm_encode.h: t at +0, bucket at +1024) when fmt != RGBA32F
    const void* enc;
    int32_t fmt;          // RTM_FORMAT_* | FMT_RGB8_DWORDS (RGB8 rows start 4-byte aligned)
    uint32_t bg;          // the encoded background pixel (0.0, 0.2, 0.2) (main.rs:718-720), R | G<<8 | B<<16
    // PERSPECTIVE eye with ray-traced primitives: rt holds the origin-only constants
    // (rt_persp) and rtmask is scratch for the per-wave primitive masks,
    // rtmask_words = ceil(W/64) * rows words (launch_eye_pass fills it first; nullptr:
    // in-kernel cull); every read of it is bounds-checked against rtmask_words
    uint32_t* rtmask;
    int32_t rt_persp, rtmask_words;
};
// eye_pass_kernel's explicit arguments (FrameArgs, smap, out, stats, DevTabs) share the
// 4 KiB kernarg segment: past it the launch reads arguments the runtime never copied
// (round 6: ShadowPart grew by 8 bytes and the single-frame eye pass read a stale tail of
// DevTabs -- an illegal memory access in the RGB8 stripes test)
static_assert(sizeof(FrameArgs) + 3 * sizeof(void*) + sizeof(DevTabs) <= 4096,
              "eye_pass_kernel's explicit kernel arguments must fit the 4 KiB kernarg segment");
constexpr int32_t FMT_MASK = 0xff;
constexpr int32_t FMT_RGB8_DWORDS = 0x100;

// One frame of a batched launch (rtm_render_frames_async on small frames): every
// workgroup of blockIdx.z == frame reads its constants from here (device memory,
// scalar loads like a kernel argument), so one launch per pass covers a batch of
// frames instead of one launch per frame.
struct BatchFrame {
    FrameArgs a;
    double* smap;  // the frame's shadow map (W*H f64)
    void* out;     // the frame's output (rows [row_begin, row_end) in tabs.fmt)
    DevTabs tabs;  // its device tables (rt/psp/sdf inside the batch upload)
};

// Reference-seam kernels (one per reference function).
struct RasterArgs {
    RasterSphereK sph[RTM_MAX_SPHERES];
    PerspSphK psp[RTM_MAX_SPHERES];  // used when persp != 0
    int32_t n_spheres, face, W, H;
    int32_t persp, pad;
};

struct MarchArgs {
    PatchK patch[RTM_MAX_PATCHES];
    CamK cam;
    int32_t n_patches, steps, W, H;
    Tables tab;
};

struct ShadeArgs {
    ShadeSphereK shade[RTM_MAX_SPHERES];
    CamK eye, shadow;
    int32_t W, H, Ws, Hs;
    int32_t n_spheres, pad;
    const RtK* rt;      // plane / cylinder shading constants (device; nullptr: none)
    const double* gn;   // cylinder / SDF hit normals, 3 per pixel (nullptr: none)
    const SdfTabK* sdf; // SDF shading constants (device; nullptr: none)
};

struct TraceArgs {      // processRaytracingRays of one viewport
    CamK cam;
    int32_t W, H;
    const RtK* rt;
    const SdfTabK* sdf;
};

// Staged G-buffer id encoding: sphere id | GID_PLANE | GID_CYLINDER | GID_SDF (kind in bits 16+).
constexpr int32_t GID_PLANE = 1 << 16;
constexpr int32_t GID_CYLINDER = 2 << 16;
constexpr int32_t GID_SDF = 3 << 16;

// Device counters for rtm_render_stats (layout == rtm_stats).
struct StatsK {
    unsigned long long eye_hits[RTM_MAX_SPHERES];
    unsigned long long eye_hit_pixels, lit_pixels, eye_sphere_tests, shadow_sphere_tests;
    unsigned long long march_iterations, march_hits, march_in_range;
    unsigned long long eye_circle_plane_pixels, eye_capped_cylinder_pixels, eye_sdf_pixels;
    unsigned long long sdf_distance_evals;
    unsigned long long eye_plane_tests, eye_cylinder_tests;
};
static_assert(sizeof(StatsK) == sizeof(rtm_stats), "StatsK layout");

// Launchers (rtm_kernels.hip).  All asynchronous on `stream`.
int launch_shadow_pass(const FrameArgs& a, double* smap, void* stream, StatsK* stats);
// The map format the (non-counting) shadow pass writes for these arguments: a
// coded map (SMAP_U8 when steps + n_spheres <= 254, SMAP_U16 up to 65534), else
// f64 (and with RTM_SMAP=f64).  Set a.sh.smap_fmt / smap_bw before both passes launch.
int32_t shadow_map_format(const ShadowPart& sh);
// 1 when the shadow pass of sh (smap_fmt set) writes span records (a U8 map by the coded
// tile): set a.sh.smap_spans from it and size the map with smap_bytes(..., spans).
int32_t shadow_map_spans(const ShadowPart& sh);
// f64 values of a coded map (rtm_ctx_shadow_map's view of it), async on stream.
int launch_smap_decode(const ShadowPart& sh, const void* codes, double* out, void* stream);
// rt / psp != nullptr: the frame has ray-traced primitives / a PERSPECTIVE eye
// with spheres (device RtK / PerspK, see launch_upload); either selects the
// general eye kernel.
// out: (row_end-row_begin)*W pixels in tabs.fmt's format (RTM_FORMAT_RGBA32F: 16-byte aligned).
int launch_eye_pass(const FrameArgs& a, const double* smap, void* out, void* stream, StatsK* stats,
                    const DevTabs& tabs = DevTabs{});
// Batched passes over n frames (gridDim.z = n) whose BatchFrame table is at dev
// (device memory); a0 / t0: the host copy of frame 0's arguments (every frame of
// a batch shares the shapes, flags, tables and kernel variant).
// box: the union of the batch's sphere pixel boxes (x0, x1, y0, y1) for the split coded launch
// one_launch: a split coded pass as one launch of both parts (shadow_split_batch_kernel; the
// caller's choice when the batch's lane runs alone, rtm_api.cpp enqueue_batch)
int launch_shadow_batch(const BatchFrame* dev, int n, const FrameArgs& a0, void* stream, const int32_t* box = nullptr,
                        bool one_launch = false);
// blocks (optional): set to 1 when the launch ran 8 x 8-pixel blocks (eye_block_mode), else 0.
// mask_shared: the frames' primitive masks are one set, frame 0's (its words at t0.rtmask;
// every frame has frame 0's eye camera, rows and primitive table: rtm_api.cpp enqueue_batch)
// cull false: the shared masks are in place already (the lane's last cull had the same inputs).
int launch_eye_batch(const BatchFrame* dev, int n, const FrameArgs& a0, const DevTabs& t0, void* stream,
                     int* blocks = nullptr, bool mask_shared = false, bool cull = true);
// Stream-ordered copy of host bytes into device memory by kernels whose
// arguments carry the bytes (<= 3968 per launch), so the host copy is consumed
// at launch: no pinned staging, no host synchronisation.  bytes % 8 == 0.
int launch_upload(const void* src, size_t bytes, void* dst, void* stream);
// bytes (a multiple of 16, 16-byte aligned) from pinned, device-accessible host memory
int launch_pull(const void* src_host, size_t bytes, void* dst, void* stream);
int launch_vp_rasterize(const RasterArgs& a, double* zbuf, double* gh, double* gz, int32_t* gid,
                        void* stream);
int launch_vp_march(const MarchArgs& a, double* zbuf, void* stream);
int launch_vp_shade(const ShadeArgs& a, const double* szbuf, const double* gh, const double* gz,
                    const int32_t* gid, float* out, void* stream);
int launch_vp_trace(const TraceArgs& a, double* zbuf, double* gh, int32_t* gid, double* gn, void* stream);
int launch_fill(double* p, int64_t n, double v, int32_t* ip, int32_t iv, void* stream);
// The device's count of out-of-range side-table reads (skipped, not performed), then
// cleared; blocking on `stream`.
int read_oob_reads(unsigned long long* count, void* stream);

}  // namespace rtm
