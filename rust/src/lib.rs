//! rtm for PtrMan/2018RustRayTracer: the CPU render loop of `src/main.rs`
//! (Viewport::rasterize + processRaymarchingRays + renderColorImage) on MI355X,
//! behind librtm.so's C ABI (`include/rtm.h`).  `rtm_ffi` is the raw binding;
//! this module is the thin safe layer the crate's scene drivers call.
pub mod rtm_ffi;

use rtm_ffi::*;
use std::ffi::CStr;
use std::os::raw::c_void;

#[derive(Debug)]
pub struct Error {
    pub code: i32,
    pub message: String,
}

/// The reference panics on a bad frame (main.rs:700, 1949); the ABI returns a
/// status code and a thread-local message instead.
pub fn check(rc: i32) -> Result<(), Error> {
    if rc == RTM_OK {
        return Ok(());
    }
    let message = unsafe { CStr::from_ptr(rtm_last_error()) }.to_string_lossy().into_owned();
    Err(Error { code: rc, message })
}

/// The reference's `Scene` (main.rs:404-410: spherePrimitives, circlePlanePrimitives,
/// cappedCylinderPrimitives) plus the implicit patches its march takes as data
/// (rayEntry_ShadowRay_testing's hard-coded one, main.rs:2024-2029) and the GL
/// preview's SDFs.  Owns its primitives; `raw` borrows them for one call.
#[derive(Clone, Default)]
pub struct Scene {
    pub spheres: Vec<rtm_sphere>,
    pub patches: Vec<rtm_patch>,
    pub circle_planes: Vec<rtm_circle_plane>,
    pub capped_cylinders: Vec<rtm_capped_cylinder>,
    pub sdfs: Vec<rtm_sdf>,
}

fn ptr_or_null<T>(v: &[T]) -> *const T {
    if v.is_empty() { std::ptr::null() } else { v.as_ptr() }
}

impl Scene {
    /// The C view of the scene (valid while `self` is borrowed and unchanged).
    pub fn raw(&self) -> rtm_scene {
        rtm_scene {
            spheres: ptr_or_null(&self.spheres),
            patches: ptr_or_null(&self.patches),
            n_spheres: self.spheres.len() as i32,
            n_patches: self.patches.len() as i32,
            circle_planes: ptr_or_null(&self.circle_planes),
            capped_cylinders: ptr_or_null(&self.capped_cylinders),
            n_circle_planes: self.circle_planes.len() as i32,
            n_capped_cylinders: self.capped_cylinders.len() as i32,
            sdfs: ptr_or_null(&self.sdfs),
            n_sdfs: self.sdfs.len() as i32,
            reserved: 0,
        }
    }
}

/// The reference's `Camera` (main.rs:1887-1898; the resolution comes with the call).
pub type Camera = rtm_camera;

/// One device's context: its stream, shadow maps and lanes.
pub struct Context {
    raw: *mut rtm_ctx,
    // the device frame `render` renders into before its copy to the host (reused)
    frame: std::cell::Cell<(*mut c_void, i64)>,
}

impl Context {
    pub fn new(device: i32) -> Result<Context, Error> {
        if unsafe { rtm_abi_version() } != RTM_ABI_VERSION {
            return Err(Error { code: RTM_ERR_INVALID, message: "librtm ABI version mismatch".into() });
        }
        let mut raw = std::ptr::null_mut();
        check(unsafe { rtm_ctx_create(device, &mut raw) })?;
        Ok(Context { raw, frame: std::cell::Cell::new((std::ptr::null_mut(), 0)) })
    }

    /// The reference's whole frame -- shadow viewport rasterize + processRaymarchingRays,
    /// eye viewport rasterize + processRaytracingRays, renderColorImage (main.rs:1568-1628)
    /// -- as its `Map2d<Color32>`: width*height RGBA f32 in row order, in host memory.
    /// Blocking.  The same frame as rtm_render, on this context's device and stream.
    pub fn render(&self, scene: &Scene, eye: &Camera, shadow: &Camera, width: i32, height: i32,
                  march_steps: i32, flags: i32) -> Result<Vec<f32>, Error> {
        if width <= 0 || height <= 0 {
            return Err(Error { code: RTM_ERR_INVALID, message: "image size must be positive".into() });
        }
        let n = width as usize * height as usize * 4;
        let bytes = (n * 4) as i64;
        let (mut dev, cap) = self.frame.get();
        if cap < bytes {
            if !dev.is_null() {
                check(unsafe { rtm_ctx_free(self.raw, dev) })?;
                self.frame.set((std::ptr::null_mut(), 0));
            }
            check(unsafe { rtm_ctx_alloc(self.raw, bytes, &mut dev) })?;
            self.frame.set((dev, bytes));
        }
        let sc = scene.raw();
        check(unsafe {
            rtm_render_async(self.raw, &sc, eye, shadow, width, height, march_steps, flags, 0, height,
                             dev as *mut f32)
        })?;
        let mut out = vec![0f32; n];
        self.copy_to_host(dev as *const f32, &mut out)?;
        Ok(out)
    }

    /// `Viewport{rasterized: None.., zBuffer: +INF, face, camera}` (main.rs:426-439) of
    /// width x height on this context: the reference's per-seam calls.
    pub fn viewport(&self, width: i32, height: i32, face: i32, camera: &Camera) -> Result<Viewport<'_>, Error> {
        let mut raw = std::ptr::null_mut();
        check(unsafe { rtm_viewport_create(self.raw, width, height, face, camera, &mut raw) })?;
        Ok(Viewport { _ctx: self, raw, width, height })
    }

    pub fn raw(&self) -> *mut rtm_ctx {
        self.raw
    }

    /// Streams a frame sequence spreads over (0 = auto) and frames per launch (0 = auto).
    pub fn set_lanes(&self, lanes: i32) -> Result<(), Error> {
        check(unsafe { rtm_ctx_set_lanes(self.raw, lanes) })
    }
    pub fn set_batch(&self, frames: i32) -> Result<(), Error> {
        check(unsafe { rtm_ctx_set_batch(self.raw, frames) })
    }

    /// `n` device frames of width x height RGBA f32 (a swap chain for `render_frames`).
    pub fn alloc_frames(&self, n: usize, width: i32, height: i32) -> Result<FrameRing<'_>, Error> {
        let bytes = width as i64 * height as i64 * 16;
        let mut ring = FrameRing { ctx: self, frames: Vec::with_capacity(n), bytes };
        for _ in 0..n {
            let mut p: *mut c_void = std::ptr::null_mut();
            check(unsafe { rtm_ctx_alloc(self.raw, bytes, &mut p) })?;
            ring.frames.push(p as *mut f32);
        }
        Ok(ring)
    }

    /// Frame i = scenes[i] rendered into outs[i] (device frames), asynchronous on the
    /// context's stream: rtm_render_frames_async, the timed call of bench.py.
    pub fn render_frames(&self, scenes: &[rtm_scene], eye: &rtm_camera, shadow: &rtm_camera, width: i32,
                         height: i32, march_steps: i32, flags: i32, outs: &[*mut f32]) -> Result<(), Error> {
        assert_eq!(scenes.len(), outs.len());
        check(unsafe {
            rtm_render_frames_async(self.raw, scenes.len() as i32, scenes.as_ptr(), eye, shadow, width, height,
                                    march_steps, flags, outs.as_ptr())
        })
    }

    pub fn synchronize(&self) -> Result<(), Error> {
        check(unsafe { rtm_ctx_synchronize(self.raw) })
    }

    /// A device frame into host memory (Map2d<Color32> order, RGBA), after the frames
    /// enqueued before it.
    pub fn copy_to_host(&self, frame_dev: *const f32, host: &mut [f32]) -> Result<(), Error> {
        check(unsafe {
            rtm_ctx_copy_to_host(self.raw, frame_dev as *const c_void, host.as_mut_ptr() as *mut c_void,
                                 (host.len() * 4) as i64)
        })
    }

    /// writeColorImage (main.rs:660-704) of a device frame: the PPM file's text.
    pub fn ppm_text(&self, frame_dev: *const f32, width: i32, height: i32) -> Result<Vec<u8>, Error> {
        let cap = unsafe { rtm_ppm_max_bytes(width, height) };
        let mut text = vec![0u8; cap as usize];
        let mut len = 0i64;
        check(unsafe {
            rtm_write_ppm(self.raw, frame_dev, width, height, text.as_mut_ptr() as *mut std::os::raw::c_char, cap,
                          &mut len)
        })?;
        text.truncate(len as usize);
        Ok(text)
    }
}

impl Drop for Context {
    fn drop(&mut self) {
        let (dev, _) = self.frame.get();
        if !dev.is_null() {
            unsafe { rtm_ctx_free(self.raw, dev) };
        }
        unsafe { rtm_ctx_destroy(self.raw) }
    }
}

/// The reference's `Viewport` (main.rs:426-643) on the device: its zBuffer and
/// G-buffer stay in device memory between the seams.  Borrowing the context keeps
/// the viewport from outliving it.
pub struct Viewport<'a> {
    _ctx: &'a Context,
    raw: *mut rtm_viewport,
    pub width: i32,
    pub height: i32,
}

impl Viewport<'_> {
    /// Viewport::rasterize (main.rs:445): every sphere projected and rasterized into
    /// the zBuffer / G-buffer (face as created).
    pub fn rasterize(&mut self, scene: &Scene) -> Result<(), Error> {
        let sc = scene.raw();
        check(unsafe { rtm_viewport_rasterize(self.raw, &sc) })
    }

    /// Viewport::processRaymarchingRays (main.rs:551): the patches marched in order,
    /// `steps` steps of 0.03 (the reference hard-codes its patch and 500 steps,
    /// main.rs:2024-2031: pass those for its frame).
    pub fn process_raymarching_rays(&mut self, patches: &[rtm_patch], steps: i32) -> Result<(), Error> {
        check(unsafe {
            rtm_viewport_process_raymarching_rays(self.raw, ptr_or_null(patches), patches.len() as i32, steps)
        })
    }

    /// Viewport::processRaytracingRays (main.rs:569): circle planes, then capped
    /// cylinders, against every pixel's camera ray.
    pub fn process_raytracing_rays(&mut self, scene: &Scene) -> Result<(), Error> {
        let sc = scene.raw();
        check(unsafe { rtm_viewport_process_raytracing_rays(self.raw, &sc) })
    }

    /// The zBuffer (width*height f64, row order).
    pub fn z_buffer(&self) -> Result<Vec<f64>, Error> {
        let mut z = vec![0f64; self.width as usize * self.height as usize];
        check(unsafe { rtm_viewport_read_zbuffer(self.raw, z.as_mut_ptr()) })?;
        Ok(z)
    }
}

impl Drop for Viewport<'_> {
    fn drop(&mut self) {
        unsafe { rtm_viewport_destroy(self.raw) }
    }
}

/// renderColorImage(&scene, &viewport, &shadowViewport) (main.rs:710): the shaded
/// image, width*height RGBA f32 in host memory (its `Map2d<Color32>`).
pub fn render_color_image(scene: &Scene, vp: &Viewport<'_>, shadow_vp: &Viewport<'_>) -> Result<Vec<f32>, Error> {
    let mut out = vec![0f32; vp.width as usize * vp.height as usize * 4];
    let sc = scene.raw();
    check(unsafe { rtm_render_color_image(&sc, vp.raw, shadow_vp.raw, out.as_mut_ptr()) })?;
    Ok(out)
}

/// Device frames owned through a context (freed after its stream drains).
pub struct FrameRing<'a> {
    ctx: &'a Context,
    pub frames: Vec<*mut f32>,
    pub bytes: i64,
}

impl Drop for FrameRing<'_> {
    fn drop(&mut self) {
        for &p in &self.frames {
            unsafe { rtm_ctx_free(self.ctx.raw, p as *mut c_void) };
        }
    }
}

/// The north star's multi-GPU frame: N devices of this process
/// joined by one RCCL communicator (rtm_group_create: ncclCommInitAll).  Each frame is
/// tile-partitioned over the devices (8-row cyclic stripes by default), every device
/// renders its part -- evaluating the shadow texels it reads, so the image is the same
/// bits -- and ONE gather over xGMI assembles it on device 0, from where it is copied into
/// the caller's host buffer.  It replaces the reference's per-frame render in its
/// animation loop (main.rs:1469-1633).
pub struct Group {
    raw: *mut rtm_group,
    /// bound on the wait in `Drop` before the communicators are aborted
    pub drop_timeout_ms: i32,
}

impl Group {
    /// A group over `devices` (empty: every device, 0..rtm_device_count()).
    pub fn new(devices: &[i32]) -> Result<Group, Error> {
        if unsafe { rtm_abi_version() } != RTM_ABI_VERSION {
            return Err(Error { code: RTM_ERR_INVALID, message: "librtm ABI version mismatch".into() });
        }
        let n = if devices.is_empty() { unsafe { rtm_device_count() } } else { devices.len() as i32 };
        let mut raw = std::ptr::null_mut();
        check(unsafe { rtm_group_create(n, ptr_or_null(devices), &mut raw) })?;
        Ok(Group { raw, drop_timeout_ms: 120_000 })
    }

    /// Devices (ranks) in the group.
    pub fn len(&self) -> Result<i32, Error> {
        let (mut n, mut local, mut first) = (0i32, 0i32, 0i32);
        check(unsafe { rtm_group_info(self.raw, &mut n, &mut local, &mut first) })?;
        Ok(n)
    }

    /// One frame of the animation as `format` pixels (RTM_FORMAT_RGBA32F: the reference's
    /// Map2d<Color32> + alpha; RGBA8 / RGB8: writeColorImage's bytes), width*height pixels
    /// in row order, in host memory.  Blocking: rtm_group_render.
    pub fn render(&self, scene: &Scene, eye: &Camera, shadow: &Camera, width: i32, height: i32, march_steps: i32,
                  flags: i32, format: i32) -> Result<Vec<u8>, Error> {
        let mut out = Vec::new();
        self.render_into(scene, eye, shadow, width, height, march_steps, flags, format, &mut out)?;
        Ok(out)
    }

    /// `render` into a caller-owned buffer (resized to the frame), e.g. one registered once
    /// with rtm_host_register for direct DMA and reused by every frame of the loop.
    pub fn render_into(&self, scene: &Scene, eye: &Camera, shadow: &Camera, width: i32, height: i32,
                       march_steps: i32, flags: i32, format: i32, out: &mut Vec<u8>) -> Result<(), Error> {
        let bpp = unsafe { rtm_format_bytes(format) };
        if bpp <= 0 || width <= 0 || height <= 0 {
            return Err(Error { code: RTM_ERR_INVALID, message: "bad format or image size".into() });
        }
        out.resize(width as usize * height as usize * bpp as usize, 0);
        let sc = scene.raw();
        check(unsafe {
            rtm_group_render(self.raw, &sc, eye, shadow, width, height, march_steps, flags, format,
                             out.as_mut_ptr() as *mut c_void)
        })
    }

    /// true: every device copies its part straight into its rows of the host frame (N PCIe
    /// links, no gather); false: gather on device 0, then one copy (the default).
    pub fn set_host_direct(&self, on: bool) -> Result<(), Error> {
        check(unsafe { rtm_group_set_host_direct(self.raw, on as i32) })
    }

    /// The partition: stripe_rows > 0 cyclic stripes of that many rows, 0 contiguous
    /// bands of ceil(H/N) rows, -1 the default (8-row stripes).
    pub fn set_partition(&self, stripe_rows: i32) -> Result<(), Error> {
        check(unsafe { rtm_group_set_partition(self.raw, stripe_rows) })
    }

    /// Wait for every device's work; timeout_ms > 0 bounds the wait (RTM_ERR_COMM past it,
    /// with the communicators aborted).
    pub fn synchronize(&self, timeout_ms: i32) -> Result<(), Error> {
        check(unsafe { rtm_group_synchronize(self.raw, timeout_ms) })
    }

    pub fn raw(&self) -> *mut rtm_group {
        self.raw
    }
}

impl Drop for Group {
    fn drop(&mut self) {
        // a bounded wait first: a lost device cannot hang the drop (rtm_group_destroy then
        // aborts the communicators instead of waiting on them)
        unsafe {
            let _ = rtm_group_synchronize(self.raw, self.drop_timeout_ms);
            rtm_group_destroy(self.raw)
        }
    }
}
