"""Host-side mirror of the reference's render interface over the HIP C ABI.

Reference surface (src/main.rs) -> this module:
    Viewport{rasterized, zBuffer, face, camera}   main.rs:426-439  -> Viewport
    Viewport::rasterize(&Scene)                   main.rs:445      -> Viewport.rasterize
    Viewport::processRaymarchingRays()            main.rs:551      -> Viewport.processRaymarchingRays
    Viewport::processRaytracingRays(&Scene)       main.rs:569      -> Viewport.processRaytracingRays
    renderColorImage(&Scene,&Viewport,&Viewport)  main.rs:710      -> renderColorImage
    writeColorImage(&Map2d<Color32>, &path)       main.rs:660      -> writeColorImage / Context.write_ppm
    the whole two-viewport frame of a scene script (main.rs:1533-1628) -> render_frame / Context.render_async

Errors surface as abi.RtmError (the reference panics).  There is no CPU
fallback: every call goes through librtm.so.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import abi
from .scenes import EnumFace, REFERENCE_MARCH_STEPS, REFERENCE_PATCH, Camera, Scene  # noqa: F401


def _lib():
    return abi.load_library()


def device_count() -> int:
    return int(_lib().rtm_device_count())


class Context:
    """One device: stream, shadow map, events (rtm_ctx)."""

    def __init__(self, device: int = 0):
        self.device = device
        self._h = C.c_void_p()
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_create(device, C.byref(self._h)), "rtm_ctx_create")

    @property
    def handle(self):
        return self._h

    @property
    def stream(self) -> int:
        return _lib().rtm_ctx_stream(self._h) or 0

    def synchronize(self):
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_synchronize(self._h), "rtm_ctx_synchronize")

    def last_kernel_ms(self):
        s, e = C.c_float(), C.c_float()
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_last_kernel_ms(self._h, C.byref(s), C.byref(e)), "rtm_ctx_last_kernel_ms")
        return float(s.value), float(e.value)

    def set_timing_capacity(self, n: int):
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_set_timing_capacity(self._h, n), "rtm_ctx_set_timing_capacity")

    def set_timing_stride(self, n: int):
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_set_timing_stride(self._h, n), "rtm_ctx_set_timing_stride")

    def set_lanes(self, n: int):
        """Lanes of render_frames_async (0 = auto, 1 = one frame after another)."""
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_set_lanes(self._h, n), "rtm_ctx_set_lanes")

    def set_batch(self, n: int):
        """Frames per launch of render_frames_async (0 = auto, 1 = one frame per launch)."""
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_set_batch(self._h, n), "rtm_ctx_set_batch")

    def last_batch(self) -> int:
        n = C.c_int32()
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_last_batch(self._h, C.byref(n)), "rtm_ctx_last_batch")
        return int(n.value)

    def last_lanes(self) -> int:
        n = C.c_int32()
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_last_lanes(self._h, C.byref(n)), "rtm_ctx_last_lanes")
        return int(n.value)

    def last_eye_blocks(self) -> bool:
        """rtm_ctx_last_eye_blocks: the last eye launch ran 8 x 8-pixel blocks (else 64 x 1 rows)."""
        n = C.c_int32()
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_last_eye_blocks(self._h, C.byref(n)), "rtm_ctx_last_eye_blocks")
        return bool(n.value)

    def frames_plan(self, width: int, rows: int, n_frames: int):
        """rtm_ctx_frames_plan: (lanes, frames per launch) render_frames_async picks for
        n_frames frames of width x rows with distinct outputs on this context."""
        ln, b = C.c_int32(), C.c_int32()
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_frames_plan(self._h, width, rows, n_frames, C.byref(ln), C.byref(b)),
                  "rtm_ctx_frames_plan")
        return int(ln.value), int(b.value)

    def kernel_ms_history(self, n: int):
        """Per-render (shadow_pass_ms, eye_pass_ms) from HIP events, oldest first."""
        sm = (C.c_float * max(n, 1))()
        em = (C.c_float * max(n, 1))()
        cnt = C.c_int32()
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_kernel_ms_history(self._h, sm, em, n, C.byref(cnt)), "rtm_ctx_kernel_ms_history")
        return [float(v) for v in sm[:cnt.value]], [float(v) for v in em[:cnt.value]]

    def render_async(self, scene: Scene, eye: Camera, shadow: Camera, width: int, height: int,
                     steps: int, flags: int, out_ptr: int, row_begin: int = 0, row_end: int | None = None):
        """Enqueue one frame; out_ptr is a device pointer (e.g. tensor.data_ptr())
        to (row_end-row_begin)*width*4 floats."""
        row_end = height if row_end is None else row_end
        sc, keep = scene.to_c()
        e, s = eye.to_c(), shadow.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_render_async(self._h, C.byref(sc), C.byref(e), C.byref(s), width, height,
                                            steps, flags, row_begin, row_end, C.c_void_p(out_ptr)),
                  "rtm_render_async")

    def render_rows_async(self, scene: Scene, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
                          flags: int, fmt: int, out_ptr: int, row_begin: int = 0, row_end: int | None = None):
        """rtm_render_rows_async: rows [row_begin, row_end) in output format `fmt`
        (abi.RTM_FORMAT_*) into the device buffer at out_ptr."""
        row_end = height if row_end is None else row_end
        sc, keep = scene.to_c()
        e, s = eye.to_c(), shadow.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_render_rows_async(self._h, C.byref(sc), C.byref(e), C.byref(s), width, height, steps,
                                                 flags, fmt, row_begin, row_end, C.c_void_p(out_ptr)),
                  "rtm_render_rows_async")

    def render_stripes_async(self, scene: Scene, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
                             flags: int, fmt: int, stripe_rows: int, n_parts: int, part: int, out_ptr: int):
        """rtm_render_stripes_async: part `part` of n_parts under stripe_rows-row cyclic
        stripes, compact rows (stripe_rows_of(...) of them) into the device buffer."""
        sc, keep = scene.to_c()
        e, s = eye.to_c(), shadow.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_render_stripes_async(self._h, C.byref(sc), C.byref(e), C.byref(s), width, height,
                                                    steps, flags, fmt, stripe_rows, n_parts, part,
                                                    C.c_void_p(out_ptr)), "rtm_render_stripes_async")

    def prepare_frames(self, scenes):
        """ctypes array of rtm_scene for render_frames_async (+ keepalive)."""
        arr = (abi.rtm_scene * len(scenes))()
        keep = []
        conv = {}  # a scene repeated in the sequence is converted once
        for i, s in enumerate(scenes):
            if id(s) not in conv:
                conv[id(s)] = s.to_c()
                keep.append(conv[id(s)][1])
            arr[i] = conv[id(s)][0]
        return arr, keep

    def render_frames_async(self, scenes, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
                            flags: int, out_ptrs, prepared=None):
        """Enqueue len(scenes) frames (batched and spread over the context's lanes);
        frame i goes to device pointer out_ptrs[i]."""
        arr, keep = prepared if prepared is not None else self.prepare_frames(scenes)  # scenes unused if prepared
        n = len(arr)
        outs = Context.out_array(out_ptrs)
        if len(outs) != n:
            raise ValueError(f"{len(outs)} output pointers for {n} frames")
        e, s = eye.to_c(), shadow.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_render_frames_async(self._h, n, arr, C.byref(e), C.byref(s), width, height, steps,
                                                   flags, outs), "rtm_render_frames_async")

    @staticmethod
    def out_array(out_ptrs):
        """The float* const* of rtm_render_frames_async: a ctypes array built once
        (a swap chain reused call after call) passes through as it is."""
        if isinstance(out_ptrs, C.Array):
            return out_ptrs
        return (C.c_void_p * len(out_ptrs))(*[C.c_void_p(p) for p in out_ptrs])

    def shadow_map_ptr(self) -> int:
        return _lib().rtm_ctx_shadow_map(self._h) or 0

    def shadow_map_texel_bytes(self) -> int:
        """Bytes per texel of the last shadow pass's map: 8 (f64), 2 or 1 (coded)."""
        return int(_lib().rtm_ctx_shadow_map_texel_bytes(self._h))

    def shadow_map_stored_bytes(self):
        """rtm_ctx_shadow_map_stored_bytes: (bytes the last shadow pass stored -- span
        records + the spans stored texel by texel for a 1-byte coded map, else the texel
        bytes -- and whether the map carries span records)."""
        n, sr = C.c_int64(), C.c_int32()
        lib = _lib()
        abi.check(lib, lib.rtm_ctx_shadow_map_stored_bytes(self._h, C.byref(n), C.byref(sr)),
                  "rtm_ctx_shadow_map_stored_bytes")
        return int(n.value), bool(sr.value)

    def stats(self, scene: Scene, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
              flags: int = 0) -> dict:
        sc, keep = scene.to_c()
        e, s = eye.to_c(), shadow.to_c()
        st = abi.rtm_stats()
        lib = _lib()
        abi.check(lib, lib.rtm_render_stats(self._h, C.byref(sc), C.byref(e), C.byref(s), width, height,
                                            steps, flags, C.byref(st)), "rtm_render_stats")
        return st.as_dict()

    def encode_rgb8_async(self, rgba_dev: int, n_pixels: int, rgb_dev: int):
        """writeColorImage's per-pixel encode (main.rs:674-684) of a device RGBA f32
        buffer into device RGB8 (3 bytes per pixel), on this context's stream."""
        lib = _lib()
        abi.check(lib, lib.rtm_encode_rgb8_async(self._h, C.c_void_p(rgba_dev), n_pixels, C.c_void_p(rgb_dev)),
                  "rtm_encode_rgb8_async")

    def write_ppm(self, rgba_dev: int, width: int, height: int) -> bytes:
        """writeColorImage's P3 text (main.rs:660-688) of a device RGBA f32 image."""
        lib = _lib()
        cap = int(lib.rtm_ppm_max_bytes(width, height))
        buf = C.create_string_buffer(max(cap, 1))
        n = C.c_int64()
        abi.check(lib, lib.rtm_write_ppm(self._h, C.c_void_p(rgba_dev), width, height, buf, cap, C.byref(n)),
                  "rtm_write_ppm")
        return buf.raw[:n.value]

    def close(self):
        if self._h:
            _lib().rtm_ctx_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def render_frame(scene: Scene, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
                 flags: int = 0) -> np.ndarray:
    """rtm_render: the full frame into host memory, (height, width, 4) f32."""
    out = np.empty((height, width, 4), np.float32)
    sc, keep = scene.to_c()
    e, s = eye.to_c(), shadow.to_c()
    lib = _lib()
    abi.check(lib, lib.rtm_render(C.byref(sc), C.byref(e), C.byref(s), width, height, steps, flags,
                                  out.ctypes.data_as(C.POINTER(C.c_float))), "rtm_render")
    return out


def render_frame_multi(scene: Scene, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
                       flags: int = 0, n_gpus: int = 1) -> np.ndarray:
    """rtm_render_multi: the frame as row bands on devices 0..n_gpus-1 of this
    process, assembled in host memory, (height, width, 4) f32."""
    out = np.empty((height, width, 4), np.float32)
    sc, keep = scene.to_c()
    e, s = eye.to_c(), shadow.to_c()
    lib = _lib()
    abi.check(lib, lib.rtm_render_multi(C.byref(sc), C.byref(e), C.byref(s), width, height, steps, flags,
                                        out.ctypes.data_as(C.POINTER(C.c_float)), n_gpus), "rtm_render_multi")
    return out


def _unknown_format(fmt: int):
    # the library's answer to an unknown format (RTM_ERR_INVALID), before any buffer is sized
    return abi.RtmError(abi.RTM_ERR_INVALID, "host frame", f"unknown output format {fmt}")


def _host_frame(height: int, width: int, fmt: int) -> np.ndarray:
    if fmt not in abi.FORMAT_BYTES:
        raise _unknown_format(fmt)
    if fmt == abi.RTM_FORMAT_RGBA32F:
        return np.empty((height, width, 4), np.float32)
    return np.empty((height, width, abi.FORMAT_BYTES[fmt]), np.uint8)


def _check_host_out(out, height: int, width: int, fmt: int) -> np.ndarray:
    """A caller-supplied host frame: the C side writes width*height*bytes(fmt)
    contiguous bytes through its base pointer, so a short, strided or mistyped
    buffer would be overrun or scattered.  Raise instead."""
    if fmt not in abi.FORMAT_BYTES:
        raise _unknown_format(fmt)
    if not isinstance(out, np.ndarray):
        raise ValueError("out must be a numpy array")
    want = np.float32 if fmt == abi.RTM_FORMAT_RGBA32F else np.uint8
    if out.dtype != want:
        raise ValueError(f"out has dtype {out.dtype}, format {fmt} needs {np.dtype(want)}")
    if not out.flags.c_contiguous:
        raise ValueError("out must be C-contiguous")
    need = width * height * abi.FORMAT_BYTES[fmt]
    if out.nbytes < need:
        raise ValueError(f"out holds {out.nbytes} bytes, the frame needs {need}")
    return out


def render_frame_ex(scene: Scene, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
                    flags: int = 0, fmt: int = abi.RTM_FORMAT_RGBA32F, n_gpus: int = 0, out=None) -> np.ndarray:
    """rtm_render_ex (n_gpus == 0) or rtm_render_multi_ex: the frame in output format
    `fmt` into host memory: (H, W, 4) f32, (H, W, 4) u8 (RGBA8) or (H, W, 3) u8 (RGB8)."""
    out = _host_frame(height, width, fmt) if out is None else _check_host_out(out, height, width, fmt)
    sc, keep = scene.to_c()
    e, s = eye.to_c(), shadow.to_c()
    lib = _lib()
    if n_gpus:
        abi.check(lib, lib.rtm_render_multi_ex(C.byref(sc), C.byref(e), C.byref(s), width, height, steps, flags, fmt,
                                               C.c_void_p(out.ctypes.data), n_gpus), "rtm_render_multi_ex")
    else:
        abi.check(lib, lib.rtm_render_ex(C.byref(sc), C.byref(e), C.byref(s), width, height, steps, flags, fmt,
                                         C.c_void_p(out.ctypes.data)), "rtm_render_ex")
    return out


class HostRegistration:
    """rtm_host_register / rtm_host_unregister of a numpy array (context manager)."""

    def __init__(self, arr: np.ndarray):
        self.arr = arr
        lib = _lib()
        abi.check(lib, lib.rtm_host_register(C.c_void_p(arr.ctypes.data), arr.nbytes), "rtm_host_register")

    def close(self):
        if self.arr is not None:
            lib = _lib()
            abi.check(lib, lib.rtm_host_unregister(C.c_void_p(self.arr.ctypes.data)), "rtm_host_unregister")
            self.arr = None

    def __enter__(self):
        return self.arr

    def __exit__(self, *exc):
        self.close()


class Group:
    """rtm_group: N ranks, one device each, one RCCL communicator; frames are
    tile-partitioned into row bands and gathered into the root's device buffer
    (SURVEY.md §8e).  Group(n_devices=N) drives devices 0..N-1 from this process
    (ncclCommInitAll); Group(device=d, n_ranks=N, rank=r, uid=bytes) joins one
    process per GPU (ncclCommInitRank, uid from Group.unique_id() on rank 0)."""

    def __init__(self, n_devices: int | None = None, devices=None, *, device: int | None = None,
                 n_ranks: int | None = None, rank: int | None = None, uid: bytes | None = None,
                 loopback: bool = False):
        self._h = C.c_void_p()
        lib = _lib()
        if loopback:
            # test transport (rtm_group_create_loopback): device copies instead of RCCL,
            # members may share a device (devices None: all on device 0)
            n = n_devices if n_devices is not None else len(devices)
            devs = (C.c_int32 * n)(*devices) if devices is not None else None
            abi.check(lib, lib.rtm_group_create_loopback(n, devs, C.byref(self._h)), "rtm_group_create_loopback")
        elif device is not None:
            u = (C.c_uint8 * 128).from_buffer_copy(uid)
            abi.check(lib, lib.rtm_group_create_rank(device, n_ranks, rank, u, C.byref(self._h)),
                      "rtm_group_create_rank")
        else:
            n = n_devices if n_devices is not None else len(devices)
            devs = (C.c_int32 * n)(*devices) if devices is not None else None
            abi.check(lib, lib.rtm_group_create(n, devs, C.byref(self._h)), "rtm_group_create")

    @property
    def handle(self):
        return self._h

    @staticmethod
    def unique_id() -> bytes:
        u = (C.c_uint8 * 128)()
        lib = _lib()
        abi.check(lib, lib.rtm_group_unique_id(u), "rtm_group_unique_id")
        return bytes(u)

    def info(self):
        n, loc, first = C.c_int32(), C.c_int32(), C.c_int32()
        lib = _lib()
        abi.check(lib, lib.rtm_group_info(self._h, C.byref(n), C.byref(loc), C.byref(first)), "rtm_group_info")
        return int(n.value), int(loc.value), int(first.value)

    def frames_plan(self, width: int, height: int, n_frames: int, root: int = 0):
        """rtm_group_frames_plan: (frames per chunk, lanes of the root's member) that
        render_frames_async uses for n_frames frames with distinct outputs."""
        b, ln = C.c_int32(), C.c_int32()
        lib = _lib()
        abi.check(lib, lib.rtm_group_frames_plan(self._h, width, height, n_frames, root, C.byref(b), C.byref(ln)),
                  "rtm_group_frames_plan")
        return int(b.value), int(ln.value)

    def member_lanes(self, local: int = 0) -> int:
        """Lanes local member `local`'s context used for the last frame call."""
        lib = _lib()
        n = C.c_int32()
        abi.check(lib, lib.rtm_ctx_last_lanes(lib.rtm_group_ctx(self._h, local), C.byref(n)), "rtm_ctx_last_lanes")
        return int(n.value)

    def ctx_stream(self, local: int = 0) -> int:
        lib = _lib()
        c = lib.rtm_group_ctx(self._h, local)
        return lib.rtm_ctx_stream(c) or 0

    def set_root_staging(self, on: bool):
        lib = _lib()
        abi.check(lib, lib.rtm_group_set_root_staging(self._h, 1 if on else 0), "rtm_group_set_root_staging")

    def set_partition(self, stripe_rows: int):
        """rtm_group_set_partition: S-row cyclic stripes (S > 0), contiguous bands (0),
        the library default (-1: 8-row stripes for N > 1)."""
        lib = _lib()
        abi.check(lib, lib.rtm_group_set_partition(self._h, stripe_rows), "rtm_group_set_partition")

    @property
    def partition(self) -> int:
        return int(_lib().rtm_group_partition(self._h))

    def set_host_direct(self, on: bool):
        """rtm_group_set_host_direct: render() copies every band from its own device
        straight into the host frame (N links) instead of gathering to rank 0."""
        lib = _lib()
        abi.check(lib, lib.rtm_group_set_host_direct(self._h, 1 if on else 0), "rtm_group_set_host_direct")

    def render_async(self, scene: Scene, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
                     flags: int, fmt: int, root: int, out_ptr: int, prepared=None):
        sc, keep = prepared if prepared is not None else scene.to_c()
        e, s = eye.to_c(), shadow.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_group_render_async(self._h, C.byref(sc), C.byref(e), C.byref(s), width, height,
                                                  steps, flags, fmt, root, C.c_void_p(out_ptr)),
                  "rtm_group_render_async")

    def render_frames_async(self, scenes, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
                            flags: int, fmt: int, root: int, out_ptrs, prepared=None):
        """rtm_group_render_frames_async: frame i into out_ptrs[i] (ignored off the root)."""
        arr, keep = prepared if prepared is not None else Context.prepare_frames(None, scenes)
        n = len(arr)
        if len(out_ptrs) != n:
            raise ValueError(f"{len(out_ptrs)} output pointers for {n} frames")
        outs = (C.c_void_p * n)(*[C.c_void_p(p or 0) for p in out_ptrs])
        e, s = eye.to_c(), shadow.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_group_render_frames_async(self._h, n, arr, C.byref(e), C.byref(s), width, height,
                                                         steps, flags, fmt, root, outs),
                  "rtm_group_render_frames_async")

    @property
    def stream(self) -> int:
        """hipStream_t in whose order a gathered frame is complete on this process."""
        return _lib().rtm_group_stream(self._h) or 0

    def synchronize(self, timeout_ms: int = 0):
        lib = _lib()
        abi.check(lib, lib.rtm_group_synchronize(self._h, timeout_ms), "rtm_group_synchronize")

    def render(self, scene: Scene, eye: Camera, shadow: Camera, width: int, height: int, steps: int,
               flags: int = 0, fmt: int = abi.RTM_FORMAT_RGBA32F, out=None):
        """rtm_group_render: the tile-partitioned, gathered frame in host memory
        (blocking): (H, W, 4) float32 for RGBA32F, (H, W, 4|3) uint8 for RGBA8 / RGB8."""
        out = _host_frame(height, width, fmt) if out is None else _check_host_out(out, height, width, fmt)
        sc, keep = scene.to_c()
        e, s = eye.to_c(), shadow.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_group_render(self._h, C.byref(sc), C.byref(e), C.byref(s), width, height, steps,
                                            flags, fmt, out.ctypes.data_as(C.c_void_p)), "rtm_group_render")
        return out

    # the garbage collector's and interpreter exit's bound on the wait for queued group work:
    # past it the communicators are aborted (a peer that died with a transfer unmatched
    # cannot hang interpreter exit)
    DEL_TIMEOUT_MS = 120_000

    def close(self, timeout_ms: int = 0):
        """Waits for the group's queued frames, then frees it.  timeout_ms <= 0 (default):
        as long as they take; > 0: at most that long, then the communicators are aborted.
        Raises RtmError when the wait failed or timed out (the group is freed all the same):
        frames enqueued before close may then be incomplete."""
        if self._h:
            lib = _lib()
            rc = lib.rtm_group_synchronize(self._h, timeout_ms)
            msg = lib.rtm_last_error() if rc != abi.RTM_OK else None
            lib.rtm_group_destroy(self._h)
            self._h = C.c_void_p()
            if rc != abi.RTM_OK:
                raise abi.RtmError(rc, "Group.close", (msg.decode() if msg else "") +
                                   "; frames enqueued before close may be incomplete")

    def __del__(self):
        try:
            self.close(self.DEL_TIMEOUT_MS)
        except Exception:
            pass


def encode_thresholds() -> np.ndarray:
    """T[k] = least f32 v in [0,1] whose writeColorImage byte is >= k (T[0] = 0)."""
    t = (C.c_float * 256)()
    lib = _lib()
    abi.check(lib, lib.rtm_encode_thresholds(t), "rtm_encode_thresholds")
    return np.array(t[:], np.float32)


def writeColorImage(ctx: Context, rgba_dev: int, width: int, height: int, path: str):
    """main.rs:660 — encode on the GPU, write the P3 file (the reference panics on
    an I/O error; this raises)."""
    data = ctx.write_ppm(rgba_dev, width, height)
    with open(path, "wb") as f:
        f.write(data)


class Viewport:
    """Reference Viewport (main.rs:426-439) with device-resident zBuffer / G-buffer."""

    def __init__(self, ctx: Context, width: int, height: int, face: int, camera: Camera):
        self.ctx, self.width, self.height, self.face, self.camera = ctx, width, height, face, camera
        self._h = C.c_void_p()
        c = camera.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_viewport_create(ctx.handle, width, height, face, C.byref(c), C.byref(self._h)),
                  "rtm_viewport_create")

    def rasterize(self, scene: Scene):  # main.rs:445
        sc, keep = scene.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_viewport_rasterize(self._h, C.byref(sc)), "rtm_viewport_rasterize")

    def processRaytracingRays(self, scene: Scene):  # main.rs:569
        sc, keep = scene.to_c()
        lib = _lib()
        abi.check(lib, lib.rtm_viewport_process_raytracing_rays(self._h, C.byref(sc)),
                  "rtm_viewport_process_raytracing_rays")

    def processRaymarchingRays(self, patches=(REFERENCE_PATCH,), steps: int = REFERENCE_MARCH_STEPS):  # main.rs:551
        arr = (abi.rtm_patch * max(len(patches), 1))()
        for i, p in enumerate(patches):
            arr[i].a0, arr[i].b0, arr[i].a1, arr[i].b1 = p._0.a, p._0.b, p._1.a, p._1.b
        lib = _lib()
        abi.check(lib, lib.rtm_viewport_process_raymarching_rays(self._h, arr, len(patches), steps),
                  "rtm_viewport_process_raymarching_rays")

    def zBuffer(self) -> np.ndarray:
        out = np.empty((self.height, self.width), np.float64)
        lib = _lib()
        abi.check(lib, lib.rtm_viewport_read_zbuffer(self._h, out.ctypes.data_as(C.POINTER(C.c_double))),
                  "rtm_viewport_read_zbuffer")
        return out

    def close(self):
        if self._h:
            _lib().rtm_viewport_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def renderColorImage(scene: Scene, viewport: Viewport, viewportShadowmapping: Viewport) -> np.ndarray:
    """main.rs:710 — returns the (height, width, 4) f32 image (Color32 + alpha 1)."""
    out = np.empty((viewport.height, viewport.width, 4), np.float32)
    sc, keep = scene.to_c()
    lib = _lib()
    abi.check(lib, lib.rtm_render_color_image(C.byref(sc), viewport._h, viewportShadowmapping._h,
                                              out.ctypes.data_as(C.POINTER(C.c_float))),
              "rtm_render_color_image")
    return out
