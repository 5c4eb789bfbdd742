//! Raw bindings of `include/rtm.h` (librtm.so, RTM_ABI_VERSION 11) for the
//! PtrMan/2018RustRayTracer crate.  Every function and struct of the header is
//! bound here, in header order; `tests/test_rust_ffi.py` parses this file and the
//! header and fails on any drift (names, argument counts and C types, return types,
//! struct fields and layout, constants).  Rust is not installed in the image that
//! builds librtm, so this file is checked by that parser, not by rustc.
#![allow(non_camel_case_types)]
#![allow(dead_code)]

use std::os::raw::{c_char, c_void};

pub const RTM_ABI_VERSION: i32 = 11;

// limits: scene constants travel as kernel arguments
pub const RTM_MAX_SPHERES: i32 = 16;
pub const RTM_MAX_PATCHES: i32 = 4;
pub const RTM_MAX_CIRCLE_PLANES: i32 = 16;
pub const RTM_MAX_CAPPED_CYLINDERS: i32 = 16;
pub const RTM_MAX_SDFS: i32 = 8;
pub const RTM_MAX_DIM: i32 = 32768;

// status codes (the reference panics instead, main.rs:700, 1949)
pub const RTM_OK: i32 = 0;
pub const RTM_ERR_INVALID: i32 = -1;
pub const RTM_ERR_UNSUPPORTED: i32 = -2;
pub const RTM_ERR_HIP: i32 = -3;
pub const RTM_ERR_NO_DEVICE: i32 = -4;
pub const RTM_ERR_OOM: i32 = -5;
pub const RTM_ERR_COMM: i32 = -6;

pub const RTM_CAMERA_ORTHOGONAL: i32 = 0; // EnumCameraType::ORTHOGONAL (main.rs:1882)
pub const RTM_CAMERA_PERSPECTIVE: i32 = 1; // EnumCameraType::PERSPECTIVE (main.rs:1883)
pub const RTM_FACE_FRONT: i32 = 0; // EnumFace::FRONT (main.rs:226)
pub const RTM_FACE_BACK: i32 = 1; // EnumFace::BACK (main.rs:227)

pub const RTM_FLAG_NO_MARCH: i32 = 0x1;
pub const RTM_FLAG_NO_SHADOW_RASTER: i32 = 0x2;
pub const RTM_FLAG_FUSED_SHADOW: i32 = 0x4;

pub const RTM_FORMAT_RGBA32F: i32 = 0; // Map2d<Color32> + alpha 1.0, 16 B/px
pub const RTM_FORMAT_RGBA8: i32 = 1; // writeColorImage's bytes + 255, 4 B/px (main.rs:660-704)
pub const RTM_FORMAT_RGB8: i32 = 2; // writeColorImage's bytes, 3 B/px

/// PrimitiveSphere (main.rs:343-349) + Shading (main.rs:336-340), 64 bytes.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rtm_sphere {
    pub id: i64,
    pub pos: [f64; 3],
    pub r: f64,
    pub color: [f64; 3],
}

/// Bilinear{_0: Linear{a,b}, _1: Linear{a,b}} (main.rs:2134-2142), 32 bytes.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rtm_patch {
    pub a0: f64,
    pub b0: f64,
    pub a1: f64,
    pub b1: f64,
}

/// Camera (main.rs:1887-1898), 104 bytes.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rtm_camera {
    pub type_: i32,
    pub reserved: i32,
    pub pos: [f64; 3],
    pub dir: [f64; 3],
    pub up: [f64; 3],
    pub side: [f64; 3],
}

/// PrimitiveCirclePlane (main.rs:370-380), 88 bytes.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rtm_circle_plane {
    pub id: i64,
    pub pos: [f64; 3],
    pub n: [f64; 3],
    pub radius: f64,
    pub color: [f64; 3],
}

/// PrimitiveCappedCylinder (main.rs:382-391), 96 bytes.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rtm_capped_cylinder {
    pub id: i64,
    pub pa: [f64; 3],
    pub pb: [f64; 3],
    pub ra: f64,
    pub rb: f64,
    pub color: [f64; 3],
}

/// The GL preview's SDF (entry.frag:416-442, 842-947; row f-4), 136 bytes.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rtm_sdf {
    pub id: i64,
    pub box_center: [f64; 3],
    pub tri_anchor: [f64; 3],
    pub aabb_center: [f64; 3],
    pub aabb_extent: [f64; 3],
    pub color: [f64; 3],
    pub max_steps: i32,
    pub reserved: i32,
}

/// Scene (main.rs:404-410), 64 bytes; the caller owns the arrays.
#[repr(C)]
#[derive(Clone, Copy, Debug)]
pub struct rtm_scene {
    pub spheres: *const rtm_sphere,
    pub patches: *const rtm_patch,
    pub n_spheres: i32,
    pub n_patches: i32,
    pub circle_planes: *const rtm_circle_plane,
    pub capped_cylinders: *const rtm_capped_cylinder,
    pub n_circle_planes: i32,
    pub n_capped_cylinders: i32,
    pub sdfs: *const rtm_sdf,
    pub n_sdfs: i32,
    pub reserved: i32,
}

/// Per-call statistics (rtm_render_stats), 232 bytes.
#[repr(C)]
#[derive(Clone, Copy, Debug, Default)]
pub struct rtm_stats {
    pub eye_hits: [i64; 16],
    pub eye_hit_pixels: i64,
    pub lit_pixels: i64,
    pub eye_sphere_tests: i64,
    pub shadow_sphere_tests: i64,
    pub march_iterations: i64,
    pub march_hits: i64,
    pub march_in_range: i64,
    pub eye_circle_plane_pixels: i64,
    pub eye_capped_cylinder_pixels: i64,
    pub eye_sdf_pixels: i64,
    pub sdf_distance_evals: i64,
    pub eye_plane_tests: i64,
    pub eye_cylinder_tests: i64,
}

/// Opaque handles (the library owns the device buffers, streams and RCCL comms).
#[repr(C)]
pub struct rtm_ctx {
    _private: [u8; 0],
}
#[repr(C)]
pub struct rtm_group {
    _private: [u8; 0],
}
#[repr(C)]
pub struct rtm_viewport {
    _private: [u8; 0],
}

#[link(name = "rtm")]
extern "C" {
    // ---- library ----
    pub fn rtm_abi_version() -> i32;
    pub fn rtm_last_error() -> *const c_char;
    pub fn rtm_device_count() -> i32;

    // ---- context ----
    pub fn rtm_ctx_create(device: i32, out: *mut *mut rtm_ctx) -> i32;
    pub fn rtm_ctx_destroy(ctx: *mut rtm_ctx);
    pub fn rtm_ctx_stream(ctx: *mut rtm_ctx) -> *mut c_void;
    pub fn rtm_ctx_synchronize(ctx: *mut rtm_ctx) -> i32;
    pub fn rtm_ctx_alloc(ctx: *mut rtm_ctx, bytes: i64, out_dev: *mut *mut c_void) -> i32;
    pub fn rtm_ctx_free(ctx: *mut rtm_ctx, dev: *mut c_void) -> i32;
    pub fn rtm_ctx_copy_to_host(ctx: *mut rtm_ctx, dev: *const c_void, host: *mut c_void, bytes: i64) -> i32;
    pub fn rtm_ctx_oob_reads(ctx: *mut rtm_ctx, count: *mut i64) -> i32;
    pub fn rtm_ctx_last_kernel_ms(ctx: *mut rtm_ctx, shadow_pass_ms: *mut f32, eye_pass_ms: *mut f32) -> i32;
    pub fn rtm_ctx_set_timing_capacity(ctx: *mut rtm_ctx, capacity: i32) -> i32;
    pub fn rtm_ctx_set_timing_stride(ctx: *mut rtm_ctx, stride: i32) -> i32;
    pub fn rtm_ctx_kernel_ms_history(ctx: *mut rtm_ctx, shadow_pass_ms: *mut f32, eye_pass_ms: *mut f32, max: i32,
                                     count: *mut i32) -> i32;
    pub fn rtm_ctx_set_lanes(ctx: *mut rtm_ctx, lanes: i32) -> i32;
    pub fn rtm_ctx_last_lanes(ctx: *mut rtm_ctx, lanes: *mut i32) -> i32;
    pub fn rtm_ctx_set_batch(ctx: *mut rtm_ctx, frames: i32) -> i32;
    pub fn rtm_ctx_last_batch(ctx: *mut rtm_ctx, frames: *mut i32) -> i32;

    // ---- whole frame, host output (blocking) ----
    pub fn rtm_render(scene: *const rtm_scene, eye: *const rtm_camera, shadow: *const rtm_camera, width: i32,
                      height: i32, march_steps: i32, flags: i32, out_rgba: *mut f32) -> i32;
    pub fn rtm_render_multi(scene: *const rtm_scene, eye: *const rtm_camera, shadow: *const rtm_camera, width: i32,
                            height: i32, march_steps: i32, flags: i32, out_rgba: *mut f32, n_gpus: i32) -> i32;
    pub fn rtm_render_ex(scene: *const rtm_scene, eye: *const rtm_camera, shadow: *const rtm_camera, width: i32,
                         height: i32, march_steps: i32, flags: i32, format: i32, out_host: *mut c_void) -> i32;
    pub fn rtm_render_multi_ex(scene: *const rtm_scene, eye: *const rtm_camera, shadow: *const rtm_camera,
                               width: i32, height: i32, march_steps: i32, flags: i32, format: i32,
                               out_host: *mut c_void, n_gpus: i32) -> i32;
    pub fn rtm_format_bytes(format: i32) -> i32;
    pub fn rtm_host_register(ptr: *mut c_void, bytes: i64) -> i32;
    pub fn rtm_host_unregister(ptr: *mut c_void) -> i32;

    // ---- whole frame, device output (asynchronous on ctx's stream) ----
    pub fn rtm_render_async(ctx: *mut rtm_ctx, scene: *const rtm_scene, eye: *const rtm_camera,
                            shadow: *const rtm_camera, width: i32, height: i32, march_steps: i32, flags: i32,
                            row_begin: i32, row_end: i32, out_rgba_dev: *mut f32) -> i32;
    pub fn rtm_render_rows_async(ctx: *mut rtm_ctx, scene: *const rtm_scene, eye: *const rtm_camera,
                                 shadow: *const rtm_camera, width: i32, height: i32, march_steps: i32, flags: i32,
                                 format: i32, row_begin: i32, row_end: i32, out_dev: *mut c_void) -> i32;
    /// The headline call: a sequence of frames (testscene_closelyOrbitingSphere's
    /// animation, main.rs:1469-1633), frame i = scenes[i] into out_rgba_dev[i].
    pub fn rtm_render_frames_async(ctx: *mut rtm_ctx, n_frames: i32, scenes: *const rtm_scene,
                                   eye: *const rtm_camera, shadow: *const rtm_camera, width: i32, height: i32,
                                   march_steps: i32, flags: i32, out_rgba_dev: *const *mut f32) -> i32;
    pub fn rtm_ctx_shadow_map(ctx: *mut rtm_ctx) -> *const f64;
    pub fn rtm_ctx_shadow_map_texel_bytes(ctx: *mut rtm_ctx) -> i32;
    pub fn rtm_ctx_shadow_map_stored_bytes(ctx: *mut rtm_ctx, bytes: *mut i64, span_records: *mut i32) -> i32;
    pub fn rtm_ctx_frames_plan(ctx: *mut rtm_ctx, width: i32, rows: i32, n_frames: i32, lanes: *mut i32,
                               frames_per_launch: *mut i32) -> i32;
    pub fn rtm_ctx_last_eye_blocks(ctx: *mut rtm_ctx, blocks: *mut i32) -> i32;
    pub fn rtm_render_stats(ctx: *mut rtm_ctx, scene: *const rtm_scene, eye: *const rtm_camera,
                            shadow: *const rtm_camera, width: i32, height: i32, march_steps: i32, flags: i32,
                            out: *mut rtm_stats) -> i32;

    // ---- multi-GPU frame over RCCL ----
    pub fn rtm_group_unique_id(id: *mut u8) -> i32; // 128 bytes
    pub fn rtm_group_create(n_devices: i32, devices: *const i32, out: *mut *mut rtm_group) -> i32;
    pub fn rtm_group_create_rank(device: i32, n_ranks: i32, rank: i32, id: *const u8, out: *mut *mut rtm_group)
                                 -> i32;
    pub fn rtm_group_destroy(g: *mut rtm_group);
    pub fn rtm_group_info(g: *mut rtm_group, n_ranks: *mut i32, n_local: *mut i32, first_rank: *mut i32) -> i32;
    pub fn rtm_group_ctx(g: *mut rtm_group, local: i32) -> *mut rtm_ctx;
    pub fn rtm_group_render_async(g: *mut rtm_group, scene: *const rtm_scene, eye: *const rtm_camera,
                                  shadow: *const rtm_camera, width: i32, height: i32, march_steps: i32, flags: i32,
                                  format: i32, root: i32, out_dev: *mut c_void) -> i32;
    pub fn rtm_group_render_frames_async(g: *mut rtm_group, n_frames: i32, scenes: *const rtm_scene,
                                         eye: *const rtm_camera, shadow: *const rtm_camera, width: i32,
                                         height: i32, march_steps: i32, flags: i32, format: i32, root: i32,
                                         out_dev: *const *mut c_void) -> i32;
    pub fn rtm_group_render(g: *mut rtm_group, scene: *const rtm_scene, eye: *const rtm_camera,
                            shadow: *const rtm_camera, width: i32, height: i32, march_steps: i32, flags: i32,
                            format: i32, out_host: *mut c_void) -> i32;
    pub fn rtm_group_stream(g: *mut rtm_group) -> *mut c_void;
    pub fn rtm_group_synchronize(g: *mut rtm_group, timeout_ms: i32) -> i32;
    pub fn rtm_group_set_root_staging(g: *mut rtm_group, on: i32) -> i32;
    pub fn rtm_group_set_partition(g: *mut rtm_group, stripe_rows: i32) -> i32;
    pub fn rtm_group_partition(g: *mut rtm_group) -> i32;
    pub fn rtm_group_frames_plan(g: *mut rtm_group, width: i32, height: i32, n_frames: i32, root: i32,
                                 frames_per_chunk: *mut i32, lanes: *mut i32) -> i32;
    pub fn rtm_render_stripes_async(ctx: *mut rtm_ctx, scene: *const rtm_scene, eye: *const rtm_camera,
                                    shadow: *const rtm_camera, width: i32, height: i32, march_steps: i32,
                                    flags: i32, format: i32, stripe_rows: i32, n_parts: i32, part: i32,
                                    out_dev: *mut c_void) -> i32;
    pub fn rtm_stripe_rows(height: i32, stripe_rows: i32, n_parts: i32, part: i32) -> i32;
    pub fn rtm_group_create_loopback(n_members: i32, devices: *const i32, out: *mut *mut rtm_group) -> i32;
    pub fn rtm_group_set_host_direct(g: *mut rtm_group, on: i32) -> i32;

    // ---- writeColorImage (main.rs:660-704) ----
    pub fn rtm_encode_rgb8_async(ctx: *mut rtm_ctx, rgba_dev: *const f32, n_pixels: i64, rgb_dev: *mut u8) -> i32;
    pub fn rtm_ppm_max_bytes(width: i32, height: i32) -> i64;
    pub fn rtm_write_ppm(ctx: *mut rtm_ctx, rgba_dev: *const f32, width: i32, height: i32, out: *mut c_char,
                         capacity: i64, length: *mut i64) -> i32;
    pub fn rtm_encode_thresholds(out: *mut f32) -> i32; // 256 floats

    // ---- reference-seam API (one call per reference function) ----
    pub fn rtm_viewport_create(ctx: *mut rtm_ctx, width: i32, height: i32, face: i32, camera: *const rtm_camera,
                               out: *mut *mut rtm_viewport) -> i32;
    pub fn rtm_viewport_destroy(vp: *mut rtm_viewport);
    pub fn rtm_viewport_rasterize(vp: *mut rtm_viewport, scene: *const rtm_scene) -> i32;
    pub fn rtm_viewport_process_raytracing_rays(vp: *mut rtm_viewport, scene: *const rtm_scene) -> i32;
    pub fn rtm_viewport_process_raymarching_rays(vp: *mut rtm_viewport, patches: *const rtm_patch, n_patches: i32,
                                                 steps: i32) -> i32;
    pub fn rtm_render_color_image(scene: *const rtm_scene, vp: *const rtm_viewport, shadow_vp: *const rtm_viewport,
                                  out_rgba: *mut f32) -> i32;
    pub fn rtm_viewport_read_zbuffer(vp: *const rtm_viewport, out: *mut f64) -> i32;
}
