/*
 * rtm.h — C ABI of the MI355X-native ray-trace / ray-march renderer ("rtm").
 *
 * Drop-in boundary for the CPU render loop of PtrMan/2018RustRayTracer
 * (reference: src/main.rs).  The reference has no FFI; the seams this ABI
 * replaces are the three Rust calls its scene drivers make
 * (testscene_closelyOrbitingSphere, main.rs:1568-1628; testscene_raytracingPlane0,
 * main.rs:1033-1045):
 *
 *   Viewport::rasterize(&mut self, &Scene)              main.rs:445-547
 *   Viewport::processRaymarchingRays(&mut self)         main.rs:551-565
 *   Viewport::processRaytracingRays(&mut self, &Scene)  main.rs:569-642
 *   renderColorImage(&Scene, &Viewport, &Viewport)      main.rs:710-902
 *
 * Two API levels:
 *   1. rtm_render / rtm_render_async — the whole two-viewport frame
 *      (shadow viewport rasterize + march, eye viewport rasterize + shade) in
 *      two HIP kernels; output RGBA f32.
 *   2. rtm_viewport_* / rtm_render_color_image — one call per reference seam,
 *      for callers that drive the passes themselves as the reference does.
 *
 * Conventions
 *   - All geometry is IEEE f64 (reference Vec3 is f64, main.rs:59-63); the
 *     framebuffer is RGBA f32 row-major, index y*width+x (Map2d, main.rs:2351-2373;
 *     Color32 main.rs:647-651; alpha is always 1.0).
 *   - Every entry point returns 0 (RTM_OK) or a negative RTM_ERR_* code; no
 *     exceptions or aborts cross the ABI (the reference panics instead,
 *     main.rs:700, 1949).  rtm_last_error() gives a thread-local message.
 *   - The caller owns every pointer it passes.  Host-pointer calls block until
 *     the output is written.  A context is not reentrant.
 *   - The 512x512 resolution the reference hard-codes (main.rs:306-307, 553-554,
 *     711-716, 840-841) is generalised to width x height for both viewports;
 *     at 512x512 the output is the reference's.
 */
#ifndef RTM_H
#define RTM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RTM_ABI_VERSION 11

/* ---- limits: scene constants travel as kernel arguments (SGPR path) ---- */
#define RTM_MAX_SPHERES 16
#define RTM_MAX_PATCHES 4
#define RTM_MAX_CIRCLE_PLANES 16
#define RTM_MAX_CAPPED_CYLINDERS 16
#define RTM_MAX_SDFS 8
#define RTM_MAX_DIM 32768

/* ---- status codes ---- */
#define RTM_OK 0
#define RTM_ERR_INVALID -1     /* bad argument (null, size, id out of range, ...) */
#define RTM_ERR_UNSUPPORTED -2 /* valid in the reference but not on this path (a non-orthographic shadow camera) */
#define RTM_ERR_HIP -3         /* a HIP runtime call failed */
#define RTM_ERR_NO_DEVICE -4   /* no usable gfx950 device */
#define RTM_ERR_OOM -5         /* device allocation failed */
#define RTM_ERR_COMM -6        /* RCCL unavailable, or a collective failed / timed out (the group is then aborted) */

/* ---- enums (values mirror the reference's enum order) ---- */
#define RTM_CAMERA_ORTHOGONAL 0 /* EnumCameraType::ORTHOGONAL main.rs:1882 */
#define RTM_CAMERA_PERSPECTIVE 1 /* EnumCameraType::PERSPECTIVE main.rs:1883 */
#define RTM_FACE_FRONT 0 /* EnumFace::FRONT main.rs:226 */
#define RTM_FACE_BACK 1  /* EnumFace::BACK  main.rs:227 */

/* ---- render flags ---- */
#define RTM_FLAG_NO_MARCH 0x1         /* skip processRaymarchingRays (BASELINE config 1; scenes whose
                                         shadow pass is commented out, main.rs:1399-1403) */
#define RTM_FLAG_NO_SHADOW_RASTER 0x2 /* skip the shadow viewport's sphere rasterize (main.rs:1400) */
#define RTM_FLAG_FUSED_SHADOW 0x4     /* evaluate each shadow texel on demand inside the eye pass
                                         instead of materialising the shadow map; same image bits */

/* ---- frame output formats (ABI v6) ----
 * RGBA32F: the reference's Map2d<Color32> (main.rs:709-716, 896-898) as RGBA f32,
 *          alpha 1.0, 16 bytes per pixel (the default everywhere).
 * RGBA8:   writeColorImage's bytes (main.rs:674-684: clamp, powf(1/2.2), *255 as
 *          i64) per channel + alpha 255, 4 bytes per pixel, computed in the eye
 *          pass's epilogue (no f32 frame is written).
 * RGB8:    the same bytes packed R,G,B: exactly the PPM's pixel data, 3 bytes per
 *          pixel.
 * Every byte equals writeColorImage of the RGBA32F frame, bit for bit. */
#define RTM_FORMAT_RGBA32F 0
#define RTM_FORMAT_RGBA8 1
#define RTM_FORMAT_RGB8 2

/* PrimitiveSphere (main.rs:343-349) + Shading (main.rs:336-340). 64 bytes. */
typedef struct rtm_sphere {
    int64_t id;      /* must be a valid index into the sphere array (the reference indexes
                        scene.spherePrimitives[id], main.rs:158, 748) */
    double pos[3];   /* Point */
    double r;        /* radius */
    double color[3]; /* colorR, colorG, colorB */
} rtm_sphere;

/* Bilinear{_0: Linear{a,b}, _1: Linear{a,b}} (main.rs:2134-2142): the implicit
 * surface f(p) = p.z - bilinear(p.xy) marched by raymarchPatch (main.rs:2219). */
typedef struct rtm_patch {
    double a0, b0; /* _0 */
    double a1, b1; /* _1 */
} rtm_patch;

/* Camera (main.rs:1887-1898).  resolutionX/Y come from the viewport size. */
typedef struct rtm_camera {
    int32_t type; /* RTM_CAMERA_* */
    int32_t reserved;
    double pos[3];  /* position */
    double dir[3];  /* dirNormalized */
    double up[3];   /* upNormalized */
    double side[3]; /* sideNormalized */
} rtm_camera;

/* PrimitiveCirclePlane (main.rs:370-380): a disc of `radius` around `pos` in the
 * plane through `pos` with normal `n`.  88 bytes. */
typedef struct rtm_circle_plane {
    int64_t id;      /* index into the circle-plane array: renderColorImage shades a hit with
                        circlePlanePrimitives[id]'s colour and normal (main.rs:773-776) */
    double pos[3];   /* pos: the disc centre (Plane.center, main.rs:578-581) */
    double n[3];     /* n: plane normal, used as given (the scenes normalise it, main.rs:913-914) */
    double radius;
    double color[3]; /* shading colorR, colorG, colorB */
} rtm_circle_plane;

/* PrimitiveCappedCylinder (main.rs:382-391): a capped cone from pA (radius
 * radiusA) to pB (radius radiusB), intersected by iCappedCone (main.rs:2889-2959). 96 bytes. */
typedef struct rtm_capped_cylinder {
    int64_t id;      /* index into the cylinder array (shading lookup, main.rs:791) */
    double pa[3];    /* pA */
    double pb[3];    /* pB */
    double ra, rb;   /* radiusA, radiusB */
    double color[3];
} rtm_capped_cylinder;

/* The signed-distance implicit surface of the reference's GL preview (BASELINE
 * row f-4; entry.frag:842-947 sphere trace, 416-442 distanceFn0, 290-298 sdBox,
 * 312-340 udTriangleSingle, 85-110 sBox, 356-364 sdNormalFast): the union of a
 * box of half-extents (0.4, 0.2, 0.2) centred at box_center and the triangle
 * tri_anchor + {(0.8,0.8,0.8), (1.3,0.8,0.8), (1.0,0.7,0.2)} (udTriangleSingle's
 * SQUARED distance, as written), thickened by 0.2; sphere-traced from the ray's
 * entry into the axis-aligned box aabb_center +- aabb_extent, hit when the
 * distance drops below 0.03, at most max_steps steps (the shader: 180).  The
 * shader runs it in f32 on the GPU; here it is restated in f64 (parity against
 * the oracle's restatement, not against main.rs).  136 bytes. */
typedef struct rtm_sdf {
    int64_t id;             /* index into the sdf array (shading lookup) */
    double box_center[3];   /* descriptor vecs[0] (entry.frag:878) */
    double tri_anchor[3];   /* descriptor vecs[2] (entry.frag:880) */
    double aabb_center[3];  /* entry.frag:850 */
    double aabb_extent[3];  /* entry.frag:851 */
    double color[3];
    int32_t max_steps;      /* entry.frag:887: 180 */
    int32_t reserved;
} rtm_sdf;

/* Scene (main.rs:404-410).  Spheres are rasterized and patches marched (the
 * reference marches one hard-coded patch, main.rs:2024-2031; here n_patches
 * patches are marched in order, each with a strict-min depth update, main.rs:559).
 * Circle planes and capped cylinders are ray traced into the eye viewport after
 * its rasterize (processRaytracingRays, main.rs:569-642); the reference never
 * traces them into the shadow map (main.rs:998-1003).  ABI v2 added the
 * primitive fields, v3 the SDFs. */
typedef struct rtm_scene {
    const rtm_sphere* spheres;
    const rtm_patch* patches;
    int32_t n_spheres;
    int32_t n_patches;
    const rtm_circle_plane* circle_planes;
    const rtm_capped_cylinder* capped_cylinders;
    int32_t n_circle_planes;
    int32_t n_capped_cylinders;
    const rtm_sdf* sdfs; /* ABI v3: traced after the cylinders (row f-4) */
    int32_t n_sdfs;
    int32_t reserved;
} rtm_scene;

/* Per-call statistics (filled by rtm_render_stats on the GPU). */
typedef struct rtm_stats {
    int64_t eye_hits[RTM_MAX_SPHERES]; /* eye pixels whose front surface is sphere i */
    int64_t eye_hit_pixels;            /* pixels with any hit */
    int64_t lit_pixels;                /* hit pixels that pass the shadow test */
    int64_t eye_sphere_tests;          /* (pixel, sphere) pairs with d < 1 in the eye pass */
    int64_t shadow_sphere_tests;       /* (texel, sphere) pairs with d < 1 in the shadow pass */
    int64_t march_iterations;          /* loop iterations executed by raymarchPatch, all texels/patches */
    int64_t march_hits;                /* texels*patches where the march returned Some(t) */
    int64_t march_in_range;            /* texels*patches whose start is inside the [0,1]^2 domain */
    int64_t eye_circle_plane_pixels;   /* eye pixels whose front surface is a circle plane */
    int64_t eye_capped_cylinder_pixels; /* ... a capped cylinder */
    int64_t eye_sdf_pixels;            /* ... an SDF implicit surface (row f-4) */
    int64_t sdf_distance_evals;        /* distanceFn0 calls of the eye's SDF traces (march steps + 4 normal taps per hit) */
    /* (pixel, primitive) ray tests the eye pass ran: the oracle tests every
     * primitive at every pixel; the GPU skips primitives its per-wave cull proves
     * unreachable (ABI v4) */
    int64_t eye_plane_tests;
    int64_t eye_cylinder_tests;
} rtm_stats;

/* ---- library ---- */
int32_t rtm_abi_version(void);
const char* rtm_last_error(void);
/* number of visible HIP devices (0 when none); never fails */
int32_t rtm_device_count(void);

/* ---- context (one per device; owns the stream, the shadow map and events) ---- */
typedef struct rtm_ctx rtm_ctx;
int rtm_ctx_create(int32_t device, rtm_ctx** out);
/* Drains the stream and frees the context.  Viewports created on it stay
 * valid handles: every call on them then fails (RTM_ERR_INVALID) except
 * rtm_viewport_destroy, which still frees them. */
void rtm_ctx_destroy(rtm_ctx* ctx);
/* hipStream_t the context enqueues on (as void*) */
void* rtm_ctx_stream(rtm_ctx* ctx);
int rtm_ctx_synchronize(rtm_ctx* ctx);
/* ABI v10: device memory on the context's device for a host that has no HIP
 * binding of its own (the Rust crate's swap chain of output frames for
 * rtm_render_frames_async).  rtm_ctx_free first waits for the context's stream.
 * rtm_ctx_copy_to_host: `bytes` from device memory into host memory in the
 * context's stream order, blocking (after the frames enqueued before it). */
int rtm_ctx_alloc(rtm_ctx* ctx, int64_t bytes, void** out_dev);
int rtm_ctx_free(rtm_ctx* ctx, void* dev);
int rtm_ctx_copy_to_host(rtm_ctx* ctx, const void* dev, void* host, int64_t bytes);
/* ABI v10, diagnostic: the kernels check every read of their host-built side tables
 * (per-wave primitive masks, row records) against the table's length and skip an
 * out-of-range one.  *count receives how many were skipped on the context's device
 * since the last call (every kernel enqueued before it included), and the count is
 * cleared.  0 on a correct library; tests/test_bounds.py requires it. */
int rtm_ctx_oob_reads(rtm_ctx* ctx, int64_t* count);
/* Durations in ms of the last render's two kernels, from HIP events recorded on
 * the context stream around each launch (valid after rtm_ctx_synchronize). */
int rtm_ctx_last_kernel_ms(rtm_ctx* ctx, float* shadow_pass_ms, float* eye_pass_ms);
/* Keep HIP events for the last `capacity` renders (0 disables; default 1).  After
 * rtm_ctx_synchronize, rtm_ctx_kernel_ms_history writes up to `max` per-render
 * durations, oldest first, and the number written to *count. */
int rtm_ctx_set_timing_capacity(rtm_ctx* ctx, int32_t capacity);
/* Record events only for every `stride`-th render (default 1).  Each event is a
 * barrier packet on the stream (~3-4 us per frame for four), so throughput runs
 * sample kernel durations instead of timing every frame. */
int rtm_ctx_set_timing_stride(rtm_ctx* ctx, int32_t stride);
int rtm_ctx_kernel_ms_history(rtm_ctx* ctx, float* shadow_pass_ms, float* eye_pass_ms, int32_t max,
                              int32_t* count);
/* Lanes of rtm_render_frames_async: independent frames spread over `lanes`
 * streams of the context (own shadow map each), so one frame's kernels run
 * beside another's; the call still completes in ctx's stream order.  0 = auto
 * (RTM_LANES from the environment, else 4; 3 from 16 Mpixel up);
 * 1 = strictly one frame after another; at most 8.  With several lanes the
 * kernel durations of rtm_ctx_kernel_ms_history overlap (each is the kernel's
 * time beside the other lanes).  rtm_ctx_last_lanes: lanes the last
 * rtm_render_frames_async call used. */
int rtm_ctx_set_lanes(rtm_ctx* ctx, int32_t lanes);
int rtm_ctx_last_lanes(rtm_ctx* ctx, int32_t* lanes);
/* Frames per launch of rtm_render_frames_async (ABI v6): consecutive frames with
 * the same patches share ONE launch per pass (the frame index is the grid's z
 * dimension; each frame's constants come from a table uploaded per batch), so
 * small frames stop paying a launch per pass per frame.  0 = auto (as many
 * frames as make 64 Mpixel, at most 64 below 1 Mpixel (64 at 512x512) and 32
 * from 1 Mpixel up (32 at 1920x1080, 8 at 3840x2160, 2 at 7680x4320));
 * 1 = one frame per launch; at most 64.  Frames with overlapping outputs never share a launch (a repeated output
 * pointer still ends with the later frame).  Batches are spread over the lanes.  Kernel durations of
 * rtm_ctx_kernel_ms_history are then per launch, i.e. per batch;
 * rtm_ctx_last_batch: frames per launch of the last call. */
int rtm_ctx_set_batch(rtm_ctx* ctx, int32_t frames);
int rtm_ctx_last_batch(rtm_ctx* ctx, int32_t* frames);

/* ---- whole frame, host output (blocking) ----
 * Equivalent of: shadow viewport (ORTHO, face BACK, zBuffer=+INF) rasterize +
 * processRaymarchingRays; eye viewport (face FRONT) rasterize +
 * processRaytracingRays; renderColorImage (main.rs:1568-1628, 1033-1045).
 * Cameras: the shadow camera must be ORTHOGONAL (Camera::project asserts it,
 * main.rs:1949 -> RTM_ERR_UNSUPPORTED); the eye camera may be ORTHOGONAL or
 * PERSPECTIVE (spheres then project through nalgebra's Perspective3 and
 * projectSphere, main.rs:473-530, 2796-2837, with the aspect 512/512
 * generalised to width/height).  out_rgba: width*height*4 floats. Uses a
 * per-thread default context on device 0. */
int rtm_render(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
               int32_t width, int32_t height, int32_t march_steps, int32_t flags,
               float* out_rgba);
/* The same frame on devices 0..n_gpus-1 of this process (SURVEY.md §8b-1's
 * rtm_render_multi): row bands of ceil(height/n_gpus) rows, one per device,
 * each evaluating the shadow texels it reads (RTM_FLAG_FUSED_SHADOW when
 * n_gpus > 1: same image bits), each copied from its device straight into its
 * slice of out_rgba.  Blocking.  n_gpus in [1, rtm_device_count()].  (The
 * one-process-per-GPU form is rtm_render_async per rank, see bench.py.) */
int rtm_render_multi(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                     int32_t width, int32_t height, int32_t march_steps, int32_t flags,
                     float* out_rgba, int32_t n_gpus);

/* ABI v6: rtm_render / rtm_render_multi with an output format (RTM_FORMAT_*):
 * out_host receives width*height*rtm_format_bytes(format) bytes.  Host buffers
 * registered with rtm_host_register are written by direct DMA from each device
 * (rtm_render_multi_ex: the devices' copies run side by side on their own PCIe
 * links); unregistered (pageable) buffers are copied through the runtime's
 * staging, one host thread per device. */
int rtm_render_ex(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow, int32_t width,
                  int32_t height, int32_t march_steps, int32_t flags, int32_t format, void* out_host);
int rtm_render_multi_ex(const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                        int32_t width, int32_t height, int32_t march_steps, int32_t flags, int32_t format,
                        void* out_host, int32_t n_gpus);
/* bytes per pixel of a format (16, 4, 3), 0 for an unknown format */
int32_t rtm_format_bytes(int32_t format);
/* Page-lock a caller-owned host buffer for all devices (hipHostRegister,
 * portable) so frame copies into it are direct DMA; undo with
 * rtm_host_unregister before freeing it.  A Rust host registers its output
 * Vec once and renders many frames into it. */
int rtm_host_register(void* ptr, int64_t bytes);
int rtm_host_unregister(void* ptr);

/* ---- whole frame, device output (asynchronous on ctx's stream) ----
 * Renders eye rows [row_begin, row_end) into out_rgba_dev (device memory,
 * (row_end-row_begin)*width*4 floats, row-major, row 0 = row_begin).  The
 * shadow map is full size unless RTM_FLAG_FUSED_SHADOW. */
int rtm_render_async(rtm_ctx* ctx, const rtm_scene* scene, const rtm_camera* eye,
                     const rtm_camera* shadow, int32_t width, int32_t height,
                     int32_t march_steps, int32_t flags, int32_t row_begin, int32_t row_end,
                     float* out_rgba_dev);
/* ABI v6: the same with an output format; out_dev holds (row_end-row_begin)*width
 * pixels of rtm_format_bytes(format) bytes (RGBA32F: 16-byte aligned). */
int rtm_render_rows_async(rtm_ctx* ctx, const rtm_scene* scene, const rtm_camera* eye,
                          const rtm_camera* shadow, int32_t width, int32_t height, int32_t march_steps,
                          int32_t flags, int32_t format, int32_t row_begin, int32_t row_end, void* out_dev);
/* A sequence of frames (e.g. the animation of testscene_closelyOrbitingSphere,
 * main.rs:1469), asynchronous on ctx's stream: frame i is scenes[i] rendered
 * into out_rgba_dev[i] (full frames; pointers may repeat), two kernels per
 * frame, spread over the context's lanes (rtm_ctx_set_lanes) when no two frames
 * of different lanes share output memory; the context's shadow map ends up
 * holding the last frame's shadow pass either way.  Each frame's output is
 * bit-identical to rtm_render.  Frames are validated as they are
 * enqueued: on an error return, the frames before the failing one may already
 * be on the stream.  The march tables (built from the patches, the shadow camera
 * and march_steps) are shared by all lanes: when a frame's tables differ from the
 * previous frame's, the host waits for every lane's earlier work before rebuilding
 * them, so a sequence whose patches change from frame to frame serialises the
 * call (still correct, no longer asynchronous). */
int rtm_render_frames_async(rtm_ctx* ctx, int32_t n_frames, const rtm_scene* scenes,
                            const rtm_camera* eye, const rtm_camera* shadow, int32_t width,
                            int32_t height, int32_t march_steps, int32_t flags,
                            float* const* out_rgba_dev);
/* Device pointer of the context's shadow map (width*height f64) after a
 * non-fused render (NULL before the first one).  The shadow pass stores a coded
 * map (which source won each texel, 1 or 2 bytes) unless
 * RTM_SMAP=f64: this call then decodes it into an f64 buffer of the context on
 * its stream and waits (blocking), so the values are the shadow viewport's
 * zBuffer bit for bit either way. */
const double* rtm_ctx_shadow_map(rtm_ctx* ctx);
/* ABI v7: bytes per texel the last non-fused frame's shadow pass stored: 8 (f64),
 * 2 or 1 (coded map); 0 before any, and 0 after a frame with RTM_FLAG_NO_MARCH |
 * RTM_FLAG_NO_SHADOW_RASTER: its shadow viewport is all +INF, so no shadow pass runs
 * (the eye pass evaluates its +INF texels on demand; rtm_ctx_shadow_map still
 * returns the +INF map). */
int32_t rtm_ctx_shadow_map_texel_bytes(rtm_ctx* ctx);
/* ABI v11: bytes the last non-fused frame's shadow pass stored.  A 1-byte map written by
 * the coded tile stores a span of 64 rows of a column whose march codes are one monotone
 * run as a 4-byte record instead of 64 bytes (span records), so this is
 * the span records plus the bytes of the spans stored texel by texel; other maps: their
 * texel bytes.  *span_records (may be NULL): 1 when the map carries span records (an eye
 * lookup then reads a record beside its byte).  Blocking (reads the records).  0 where
 * rtm_ctx_shadow_map_texel_bytes is 0. */
int rtm_ctx_shadow_map_stored_bytes(rtm_ctx* ctx, int64_t* bytes, int32_t* span_records);
/* ABI v11: the plan rtm_render_frames_async makes for n_frames frames of width x rows with
 * distinct outputs on this context (its rtm_ctx_set_lanes / rtm_ctx_set_batch, RTM_LANES):
 * the lanes and the frames per launch.  Host only. */
int rtm_ctx_frames_plan(rtm_ctx* ctx, int32_t width, int32_t rows, int32_t n_frames, int32_t* lanes,
                        int32_t* frames_per_launch);
/* ABI v11: the eye pass's wave shape in the last frame or batch this context launched:
 * 0 = 64 x 1-pixel rows, 1 = 8 x 8-pixel blocks (small ray-traced frames). */
int rtm_ctx_last_eye_blocks(rtm_ctx* ctx, int32_t* blocks);

/* Counting variant of the frame (separate, untimed kernels): the per-pass
 * work counts behind the roofline's algorithmic flop count. */
int rtm_render_stats(rtm_ctx* ctx, const rtm_scene* scene, const rtm_camera* eye,
                     const rtm_camera* shadow, int32_t width, int32_t height,
                     int32_t march_steps, int32_t flags, rtm_stats* out);

/* ---- multi-GPU frame over RCCL (BASELINE north star) ----
 * A group is N ranks, one device each, joined by one RCCL communicator.  A frame
 * is tile-partitioned over the N ranks: 8-row cyclic stripes by default, or N row
 * bands of ceil(H/N) rows (rtm_group_set_partition); every rank renders its rows (each band evaluates
 * the shadow texels it reads: RTM_FLAG_FUSED_SHADOW, same image bits), and ONE
 * gather (ncclSend/ncclRecv in one ncclGroupStart/End, rccl.h:700-745: RCCL's own
 * ncclGather is this same pattern, but needs equal counts and the last band may
 * be short) assembles the frame in the root's device buffer.  The root renders
 * its own band in place; the other ranks' bands go through double-buffered
 * device staging on a communication stream, so frame i+1 renders while frame i
 * is in flight.  RCCL is loaded at the first group call (librccl.so.1; the copy
 * torch.distributed already loaded, if any); without it group calls fail with
 * RTM_ERR_COMM and nothing else in the library needs it.
 *
 * Two ways to form a group:
 *   rtm_group_create        one process drives devices[0..n-1] (NULL: 0..n-1):
 *                           ncclCommInitAll (rccl.h:236);
 *   rtm_group_create_rank   one process per GPU: rank r of n_ranks on `device`,
 *                           with the 128-byte id rank 0 made by rtm_group_unique_id
 *                           and handed to the others by the caller (e.g.
 *                           torch.distributed.broadcast): ncclCommInitRank (rccl.h:220). */
typedef struct rtm_group rtm_group;
int rtm_group_unique_id(uint8_t id[128]);
int rtm_group_create(int32_t n_devices, const int32_t* devices, rtm_group** out);
int rtm_group_create_rank(int32_t device, int32_t n_ranks, int32_t rank, const uint8_t id[128],
                          rtm_group** out);
/* Waits for the group's work, then frees it (communicators destroyed).  The wait is
 * bounded (600 s by default; RTM_GROUP_DESTROY_TIMEOUT_MS, 0 = none): past it the
 * communicators are aborted instead, so a lost peer cannot hang the caller.  Bound
 * it tighter with rtm_group_synchronize(g, timeout_ms) first. */
void rtm_group_destroy(rtm_group* g);
/* n_ranks in the group, members driven by this process, the first one's rank */
int rtm_group_info(rtm_group* g, int32_t* n_ranks, int32_t* n_local, int32_t* first_rank);
/* context of local member i (its device's stream; owned by the group) */
rtm_ctx* rtm_group_ctx(rtm_group* g, int32_t local);
/* One frame, tile-partitioned and gathered: out_dev is the root's device buffer of
 * width*height pixels of rtm_format_bytes(format) bytes, on the root's device
 * (ignored on a process that does not hold the root).  Asynchronous: the frame is
 * complete in the order of the root's rtm_group_stream.  RGBA8 / RGB8 gather 4 / 3
 * bytes per pixel instead of 16.  A frame's out_dev must not be reused before that
 * frame is complete (the root's next band may already be rendering). */
int rtm_group_render_async(rtm_group* g, const rtm_scene* scene, const rtm_camera* eye,
                           const rtm_camera* shadow, int32_t width, int32_t height, int32_t march_steps,
                           int32_t flags, int32_t format, int32_t root, void* out_dev);
/* A sequence of frames, frame i into out_dev[i] (entries ignored off the root);
 * every frame's inputs are validated before the first is enqueued.  Each member
 * renders its parts in chunks of frames (one launch per pass per chunk), spread over
 * its context's lanes as rtm_render_frames_async spreads its batches. */
int rtm_group_render_frames_async(rtm_group* g, int32_t n_frames, const rtm_scene* scenes,
                                  const rtm_camera* eye, const rtm_camera* shadow, int32_t width, int32_t height,
                                  int32_t march_steps, int32_t flags, int32_t format, int32_t root,
                                  void* const* out_dev);
/* ABI v8: the drop-in form for a host that owns no device memory (the Rust
 * crate): one frame, tile-partitioned over the group and gathered to rank 0 as
 * above, into a device buffer the group owns on rank 0's device, then copied
 * into out_host (width*height pixels of rtm_format_bytes(format) bytes; direct
 * DMA when registered with rtm_host_register).  Blocking: returns when out_host
 * holds the frame (on the process holding rank 0; elsewhere when this rank's
 * band has been sent, out_host ignored). */
int rtm_group_render(rtm_group* g, const rtm_scene* scene, const rtm_camera* eye, const rtm_camera* shadow,
                     int32_t width, int32_t height, int32_t march_steps, int32_t flags, int32_t format,
                     void* out_host);
/* hipStream_t (as void*) in whose order a frame gathered to rank 0 is complete on
 * this process (the root's transfer stream; on other ranks, where their sends run) */
void* rtm_group_stream(rtm_group* g);
/* Wait for every local member's work (renders and transfers).  timeout_ms > 0:
 * give up after that long, abort the communicators (ncclCommAbort) and return
 * RTM_ERR_COMM; the group then fails every call but rtm_group_destroy.
 * timeout_ms <= 0: wait indefinitely. */
int rtm_group_synchronize(rtm_group* g, int32_t timeout_ms);
/* Test hook: 1 = the root also stages its band and sends it to itself through
 * RCCL (exercises the transfer path on a one-device group); 0 = in place (default). */
int rtm_group_set_root_staging(rtm_group* g, int32_t on);
/* ABI v9: the frame's partition over the group's ranks.  stripe_rows = S > 0: cyclic
 * S-row stripes (stripe j = rows [j*S, (j+1)*S) goes to rank j % N; each rank renders
 * its stripes compact and the root places them: a 2-D copy per part); 0: contiguous
 * bands of ceil(H/N) rows (SURVEY.md §8e's first form); -1: the default, 8-row
 * stripes for N > 1 (bands measured 1.26-1.56x max/mean band time at N = 4-8, the
 * spheres sit mid-frame; stripes even it out).  Collective: in a one-process-per-GPU
 * group every rank must set the same value before its next frame (the default
 * depends on the rank count only).  stripe_rows * n_ranks <= 8 * RTM_MAX_DIM.  Waits
 * for the group's work first.  rtm_group_partition: the S in use. */
int rtm_group_set_partition(rtm_group* g, int32_t stripe_rows);
int32_t rtm_group_partition(rtm_group* g);
/* ABI v11: the plan of rtm_group_render_frames_async for n_frames frames with distinct
 * outputs: frames per chunk (one launch per pass per chunk on every member) and the lanes
 * of the member that holds rank `root` (local member 0 if this process does not).  An
 * output ring that is a multiple of chunk x lanes frames keeps the root on its lanes.
 * Host only. */
int rtm_group_frames_plan(rtm_group* g, int32_t width, int32_t height, int32_t n_frames, int32_t root,
                          int32_t* frames_per_chunk, int32_t* lanes);
/* ABI v9: part `part` of n_parts of the frame under stripe_rows-row cyclic stripes
 * (the rows a group rank renders), compact rows into out_dev (rtm_stripe_rows(...)
 * rows), on ctx's stream; rtm_stripe_rows: that row count (-1: bad arguments). */
int rtm_render_stripes_async(rtm_ctx* ctx, const rtm_scene* scene, const rtm_camera* eye,
                             const rtm_camera* shadow, int32_t width, int32_t height, int32_t march_steps,
                             int32_t flags, int32_t format, int32_t stripe_rows, int32_t n_parts, int32_t part,
                             void* out_dev);
int32_t rtm_stripe_rows(int32_t height, int32_t stripe_rows, int32_t n_parts, int32_t part);
/* ABI v9, test transport: a group of n_members ranks in this process whose gather
 * runs as device copies on the root's transfer stream (the matched send/receive
 * pairs' completion order kept with events) instead of RCCL, so members may share
 * a device (devices NULL: all on device 0).  Exercises the N-rank band, staging and
 * receive paths of the frame calls on one GPU; not a transport for production. */
int rtm_group_create_loopback(int32_t n_members, const int32_t* devices, rtm_group** out);
/* ABI v9: 1 = rtm_group_render delivers the frame over N host links: every member
 * renders its band and copies it from its own device straight into its rows of
 * out_host (registered with rtm_host_register: DMA on each device's PCIe link), no
 * gather -- the Rust host's multi-GPU frame at N links' rate (main.rs:710, 896-901).
 * Needs every rank in this process (rtm_group_create / _loopback; else
 * RTM_ERR_UNSUPPORTED).  0 = gather to rank 0, then one copy (default). */
int rtm_group_set_host_direct(rtm_group* g, int32_t on);

/* ---- output encoding: writeColorImage (main.rs:660-704), BASELINE row f-2 ----
 * Per channel: c.max(0.0).min(1.0), f32::powf(v, 1.0/2.2), (v * 255.0) as i64,
 * evaluated exactly via 255 thresholds computed with the platform powf. */
/* RGBA f32 (device, n_pixels*4, 16-byte aligned) -> packed RGB8 (device,
 * n_pixels*3, any alignment), async on ctx's stream. */
int rtm_encode_rgb8_async(rtm_ctx* ctx, const float* rgba_dev, int64_t n_pixels, uint8_t* rgb_dev);
/* Upper bound of the PPM text size for a width x height image (header included). */
int64_t rtm_ppm_max_bytes(int32_t width, int32_t height);
/* The whole P3 file text ("P3\n{W} {H}\n255\n" + "{r} {g} {b}  " per pixel + "\n"
 * per row) of a device RGBA f32 frame, generated on the GPU, into host memory
 * `out` (no terminating NUL).  rgba_dev 16-byte aligned.  Blocking.  *length receives the text size; if it
 * exceeds `capacity` nothing is written and RTM_ERR_INVALID is returned. */
int rtm_write_ppm(rtm_ctx* ctx, const float* rgba_dev, int32_t width, int32_t height, char* out,
                  int64_t capacity, int64_t* length);
/* The 256 encode thresholds in use (T[k] = smallest v with byte(v) >= k). */
int rtm_encode_thresholds(float out[256]);

/* ---- reference-seam API (one call per reference function) ---- */
typedef struct rtm_viewport rtm_viewport;
/* Viewport{rasterized: vec![None; w*h], zBuffer: +INF, face, camera} (main.rs:426-439, 951-983) */
int rtm_viewport_create(rtm_ctx* ctx, int32_t width, int32_t height, int32_t face,
                        const rtm_camera* camera, rtm_viewport** out);
void rtm_viewport_destroy(rtm_viewport* vp);
/* Viewport::rasterize (main.rs:445): ORTHOGONAL (main.rs:452-471) or
 * PERSPECTIVE (main.rs:473-524) projection of every sphere, then
 * rasterizeSphere into the viewport's zBuffer / G-buffer. */
int rtm_viewport_rasterize(rtm_viewport* vp, const rtm_scene* scene);
/* Viewport::processRaytracingRays (main.rs:569-642): every pixel's camera ray
 * against the circle planes, then the capped cylinders, in scene order; a hit
 * with 0 <= t <= zBuffer replaces the pixel's surface and depth. */
int rtm_viewport_process_raytracing_rays(rtm_viewport* vp, const rtm_scene* scene);
/* Viewport::processRaymarchingRays (main.rs:551) generalised: the reference's
 * hard-coded patch {0.1,0.1,0.1,0.1} and 500 steps (main.rs:2024-2031) become
 * arguments; patches are marched in order. */
int rtm_viewport_process_raymarching_rays(rtm_viewport* vp, const rtm_patch* patches,
                                          int32_t n_patches, int32_t steps);
/* renderColorImage (main.rs:710): viewport and shadow viewport must share a
 * context; the shadow camera must be ORTHOGONAL (Camera::project asserts it,
 * main.rs:1949).  out_rgba: host, vp width*height*4 floats. */
int rtm_render_color_image(const rtm_scene* scene, const rtm_viewport* vp,
                           const rtm_viewport* shadow_vp, float* out_rgba);
/* Copy the viewport's zBuffer (width*height f64) to host memory. */
int rtm_viewport_read_zbuffer(const rtm_viewport* vp, double* out);

#ifdef __cplusplus
}
#endif

#endif /* RTM_H */
