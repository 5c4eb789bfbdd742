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

/// One device's context: its stream, shadow maps and lanes.
pub struct Context {
    raw: *mut rtm_ctx,
}

impl Context {
    pub fn new(device: i32) -> Result<Context, Error> {
        if unsafe { rtm_abi_version() } != RTM_ABI_VERSION {
            return Err(Error { code: RTM_ERR_INVALID, message: "librtm ABI version mismatch".into() });
        }
        let mut raw = std::ptr::null_mut();
        check(unsafe { rtm_ctx_create(device, &mut raw) })?;
        Ok(Context { raw })
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
        unsafe { rtm_ctx_destroy(self.raw) }
    }
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
