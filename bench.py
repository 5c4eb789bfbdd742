#!/usr/bin/env python3
"""Benchmark: Mpixels/s of the full two-pass frame (shadow viewport rasterize +
march, eye viewport rasterize + shade) at BASELINE config 3 — 3840x2160,
3 spheres + 1 implicit patch, 64 march steps.

One process per GPU (torch.distributed.run); prints ONE JSON line on rank 0.

A step is one segment of the animation: --frames-per-step frames (auto: at least 8
and at least 512 Mpixel worth, so 64 at 3840x2160) enqueued by one
rtm_render_frames_async call into a ring of output frames.  `value` is pixels of all
timed frames / the timed region's wall time; `ms_per_step` is per segment and
`ms_per_frame` per frame.

Modes (--mode):
  frames       (default) frame-parallel: rank r renders animation frames
               r, r+N, ... of the orbiting-sphere sequence; each frame is
               independent, no data-path collective ("scaling": "weak").
  tile-gather  one frame per step, rows split into N bands, each rank renders
               its band, then ONE RCCL gather (librtm's rtm_group, RCCL over
               xGMI) assembles the frame in rank 0's device memory
               ("scaling": "strong").  --format picks what is gathered: the
               RGBA f32 frame (16 B/px) or writeColorImage's bytes (RGBA8,
               4 B/px, encoded in the eye pass's epilogue).

Whatever the mode, the line also carries `tile_gather`: the strong-scaling
tile-partitioned frame (the north star's assembled framebuffer) measured in the
same run for RGBA f32 and RGBA8, so every N of a scaling sweep reports both the
weak (frames) and the strong (tile-gather) figure.  With --dist-backend gloo
(several ranks rehearsing on one GPU) the bands are gathered on the CPU by gloo
instead of RCCL.
"""
from __future__ import annotations

import argparse
import glob
import importlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "Mpixels/s at 3840×2160, 64 march steps; 1/2/4/8-GPU scaling"
# configs 6/7 measure BASELINE "next" row f-1 (ray-traced primitives), not the headline
METRIC_F1 = "Mpixels/s, ray-traced circle planes + capped cylinders (row f-1)"
METRIC_F4 = "Mpixels/s, sphere-traced GL-preview SDFs (row f-4)"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # a step is one segment of the animation: --frames-per-step frames rendered by one
    # rtm_render_frames_async call (the renderer's swap chain); 100 steps x 32 frames x
    # ~31 us: the timed region is ~100 ms at config 3
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--frames-per-step", type=int, default=0,
                    help="frames of one step (0 = auto: at least 8 and at least 8 Gpixel worth, at most 4096)")
    ap.add_argument("--config", type=int, default=3,
                    help="scenes.CONFIGS id: 1-5 BASELINE, 6-7 row f-1, 8 row f-4, 9 general march (tilted sun)")
    ap.add_argument("--mode", choices=["frames", "tile-gather"], default="frames")
    ap.add_argument("--fused", action="store_true", help="evaluate shadow texels on demand (same image)")
    ap.add_argument("--per-frame-calls", action="store_true",
                    help="frames mode: one rtm_render_async call per frame instead of one rtm_render_frames_async")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=1)
    ap.add_argument("--no-alt", action="store_true", help="skip the secondary fused-shadow measurement")
    ap.add_argument("--dist-backend", choices=["nccl", "gloo"], default="nccl",
                    help="nccl (= RCCL, the multi-GPU run); gloo only to rehearse the N>1 paths "
                         "with several ranks on one GPU (timing tensors and tile-gather bands on the CPU)")
    ap.add_argument("--format", choices=["rgba32f", "rgba8"], default="rgba32f",
                    help="tile-gather mode: what is rendered and gathered")
    ap.add_argument("--tile-gather-steps", type=int, default=-1,
                    help="frames of the secondary tile-gather measurement (0 = skip it; -1 = auto: "
                         "at least 2048 and at least 16 Gpixel, at most 16384)")
    ap.add_argument("--tile-gather-timeout-s", type=float, default=240.0,
                    help="watchdog of the secondary tile-gather measurement (group set-up included)")
    # The clocks ramp for tens of ms after an idle GPU: a time-based pre-roll before the
    # counted warmup makes a short --steps/--warmup run read the steady state.
    ap.add_argument("--preroll-ms", type=float, default=300.0)
    ap.add_argument("--no-host-output", action="store_true",
                    help="skip the secondary host-output (PCIe-inclusive drop-in) measurement")
    return ap.parse_args()


FORMATS = {"rgba32f": 0, "rgba8": 1}


WATCHDOG_EXIT = 3  # the status of a run whose secondary measurement stalled


class _Watchdog:
    """Bounds a secondary measurement: if it has not finished after `seconds`, rank 0
    prints the line it already holds (the secondary field marked as timed out), and
    every rank leaves with status WATCHDOG_EXIT: the headline line survives a stalled
    peer, and the caller still sees that the run did not finish cleanly."""

    def __init__(self, seconds: float, res: dict | None, field: str):
        import threading
        self._t = threading.Timer(seconds, self._fire, args=(res, field, seconds))
        self._t.daemon = True
        self._t.start()

    @staticmethod
    def _fire(res, field, seconds):
        if res is not None:
            res[field] = {"error": f"watchdog: not finished after {seconds:.0f} s"}
            print(json.dumps(res), flush=True)
        sys.stderr.write(f"bench.py: {field} watchdog fired after {seconds:.0f} s; exiting with status "
                         f"{WATCHDOG_EXIT}\n")
        sys.stderr.flush()
        os._exit(WATCHDOG_EXIT)

    def cancel(self):
        self._t.cancel()


def band_times(rtm, lib, ctx, world, rank, dist, tdev, c_scene, eye, shadow, W, H, K, flags, fmt, stripe=0,
               reps=6):
    """Every rank's own part of the tile-partitioned frame (its band, or with stripe
    > 0 its cyclic stripes: what the group renders on it, each part evaluating the
    shadow texels it reads), timed alone with HIP events on its context's stream;
    rank 0 gets the list (SURVEY.md §8e-1 imbalance)."""
    import ctypes as C
    import torch

    shard = importlib.import_module("2018rustraytracer_amd.shard")
    r0, r1 = shard.row_band(H, world, rank)
    rows = shard.stripe_rows_of(H, world, stripe, rank) if stripe > 0 and world > 1 else r1 - r0
    ms = 0.0
    if rows > 0:
        e_c, s_c = eye.to_c(), shadow.to_c()
        buf = torch.empty(rows * W * rtm.abi.FORMAT_BYTES[fmt] + 16, dtype=torch.uint8,
                          device=torch.device("cuda", torch.cuda.current_device()))
        st = torch.cuda.ExternalStream(ctx.stream)
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        fl = flags | (rtm.abi.RTM_FLAG_FUSED_SHADOW if world > 1 else 0)
        for it in range(2 + reps):
            if it == 2:
                ev0.record(st)
            if stripe > 0 and world > 1:
                rc = lib.rtm_render_stripes_async(ctx.handle, C.byref(c_scene[0]), C.byref(e_c), C.byref(s_c), W, H,
                                                  K, fl, fmt, stripe, world, rank, C.c_void_p(buf.data_ptr()))
            else:
                rc = lib.rtm_render_rows_async(ctx.handle, C.byref(c_scene[0]), C.byref(e_c), C.byref(s_c), W, H, K,
                                               fl, fmt, r0, r1, C.c_void_p(buf.data_ptr()))
            rtm.abi.check(lib, rc, "band render")
        ev1.record(st)
        ev1.synchronize()
        ms = ev0.elapsed_time(ev1) / reps
    if world == 1:
        return [ms]
    t = torch.zeros(world, dtype=torch.float64, device=tdev)
    t[rank] = ms
    dist.all_reduce(t)
    return [float(v) for v in t.cpu()]


def tile_gather(rtm, lib, ctx, group, world, rank, dist, tdev, c_scenes, eye, shadow, W, H, K, flags, fmt, steps,
                warmup, timeout_ms=120000, bands=False):
    """The tile-partitioned frame: N row bands, one gather into rank
    0.  RCCL (librtm rtm_group) with the nccl backend; with gloo the bands go to the
    CPU and gloo gathers them (the rehearsal of this path on one GPU)."""
    import ctypes as C
    import torch

    shard = importlib.import_module("2018rustraytracer_amd.shard")
    bpp = rtm.abi.FORMAT_BYTES[fmt]
    dev = torch.device("cuda", torch.cuda.current_device())
    r0, r1 = shard.row_band(H, world, rank)
    e_c, s_c = eye.to_c(), shadow.to_c()
    if group is not None:
        # a swap chain of output frames on the root: every member renders its part of a
        # chunk of frames per launch (distinct outputs), chunks spread over its lanes, and
        # frame i+1.. render while frame i is gathered.  The ring is a multiple of the
        # chunk frames x lanes the library picks for rank 0's part (rtm_api.cpp
        # frame_batch / lanes_plan), so frames that share a buffer render on one lane and
        # the root keeps its lanes (rtm_group.cpp chunks_clash_across_lanes: a ring of 32
        # at 512x512, 64 frames per chunk, would leave it one lane)
        # (the library's own plan, rtm_group_frames_plan: VERDICT r05 ADVICE)
        b0, l0 = group.frames_plan(W, H, max(steps, warmup, 1))
        n_out = b0 * l0 * -(-32 // (b0 * l0))
        outs = ([torch.empty(W * H * bpp, dtype=torch.uint8, device=dev) for _ in range(n_out)] if rank == 0
                else [None] * n_out)
        ptrs = [C.c_void_p(o.data_ptr() if o is not None else 0) for o in outs]

        def prep(first, n):  # the call's scene and output arrays (built before the clock, like frames mode)
            if n <= 0:
                return None
            return ((rtm.abi.rtm_scene * n)(*[c_scenes[(first + j) % len(c_scenes)][0] for j in range(n)]),
                    (C.c_void_p * n)(*[ptrs[(first + j) % n_out] for j in range(n)]))

        def run(first, n, pre=None):  # ONE rtm_group_render_frames_async call over the n frames
            if n <= 0:
                return
            arr, ov = pre if pre is not None else prep(first, n)
            rc = lib.rtm_group_render_frames_async(group.handle, n, arr, C.byref(e_c), C.byref(s_c), W, H, K,
                                                   flags, fmt, 0, ov)
            rtm.abi.check(lib, rc, "rtm_group_render_frames_async")

        def drain():
            group.synchronize(timeout_ms)
    else:
        band = shard.band_rows(H, world)
        dbuf = torch.empty(max(r1 - r0, 1) * W * bpp, dtype=torch.uint8, device=dev)
        hbuf = torch.zeros(band * W * bpp, dtype=torch.uint8)
        fl = flags | (rtm.abi.RTM_FLAG_FUSED_SHADOW if world > 1 else 0)

        def step(i):
            sc_c = c_scenes[i % len(c_scenes)][0]
            if r1 > r0:
                rc = lib.rtm_render_rows_async(ctx.handle, C.byref(sc_c), C.byref(e_c), C.byref(s_c), W, H, K, fl,
                                               fmt, r0, r1, C.c_void_p(dbuf.data_ptr()))
                rtm.abi.check(lib, rc, "rtm_render_rows_async")
                ctx.synchronize()
                hbuf[: (r1 - r0) * W * bpp].copy_(dbuf[: (r1 - r0) * W * bpp])
            if world > 1:
                shard.gather_bands(hbuf.view(band, W * bpp), rank, world, H, dist)

        def drain():
            ctx.synchronize()

        def prep(first, n):
            return None

        def run(first, n, pre=None):
            for i in range(first, first + n):
                step(i)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    run(0, warmup)
    drain()
    pre = prep(warmup, steps)
    barrier()
    t0 = time.perf_counter()
    run(warmup, steps, pre)
    t_enq = time.perf_counter() - t0  # the host's enqueue of the frames (the calls returned)
    drain()
    barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    r00, r01 = shard.row_band(H, world, 0)
    if group is None:
        gather = "gloo gather of CPU-staged bands (rehearsal, not RCCL)"
    elif world == 1:
        gather = "none: one band, rendered in place into the output (no transfer at N = 1)"
    else:
        gather = "RCCL: ncclSend/ncclRecv in one group into rank 0's device buffer (librtm rtm_group)"
    stripe = group.partition if group is not None else 0
    extra = {"partition": (f"{stripe}-row cyclic stripes" if stripe > 0 and world > 1 else
                           f"contiguous bands of ceil(H/{world}) rows")}
    if group is not None:
        # the lanes the root's member actually used in the timed call, beside the plan the
        # output ring was sized for (fewer: its frames clashed across lanes)
        extra.update({"root_lanes_used": group.member_lanes(0), "root_lanes_planned": l0,
                      "frames_per_chunk": b0, "output_ring": n_out})
    if bands:
        bt = band_times(rtm, lib, ctx, world, rank, dist, tdev, c_scenes[0], eye, shadow, W, H, K, flags, fmt,
                        stripe if group is not None else 0)
        mean = sum(bt) / len(bt)
        extra.update({"band_ms": [round(v, 4) for v in bt],
                      "band_max_over_mean": round(max(bt) / mean, 4) if mean > 0 else None,
                      "band_note": "each rank's own part alone (fused shadow), HIP events on its context stream"})
    return {"value": round(W * H * steps / el / 1e6, 2), "unit": "Mpixels/s", "frames": steps,
            "ms_per_step": round(el / steps * 1e3, 5), "scaling": "strong",
            "host_enqueue_ms_per_frame": round(t_enq / max(steps, 1) * 1e3, 5),
            "format": {0: "RGBA32F", 1: "RGBA8", 2: "RGB8"}[fmt], "bytes_per_pixel": bpp,
            "root_ingress_bytes_per_frame": int(W * (H - (shard.stripe_rows_of(H, world, stripe, 0)
                                                          if stripe > 0 and world > 1 else r01 - r00)) * bpp),
            "gather": gather,
            "shadow": ("fused: each band evaluates the shadow texels it reads" if world > 1 or flags & 4
                       else "two-pass (one band: the whole shadow map)"), **extra}


def tile_scaling(tile: dict, res: dict, world: int) -> None:
    """The assembled frame's strong-scaling figures, stated in the line itself (VERDICT r05
    item 5): per format, `scaling_vs_n1` = the tile-gather frame rate over ONE GPU's fused
    frame rate in the same run (alt_fused_shadow / N: every rank renders whole fused frames
    there; without it the two-pass `value` / N), and `root_ingress_GBps` = the bytes the
    root receives per frame over the time per frame.  The frames-mode `value` beside it is
    the weak curve; these two read the strong one without DESIGN.md §7's model."""
    alt = res.get("alt_fused_shadow") or {}
    base, basis = (alt.get("value"), "alt_fused_shadow") if alt.get("value") else (res.get("value"), "value")
    for name, t in tile.items():
        if not isinstance(t, dict) or "value" not in t:
            continue
        if base:
            t["scaling_vs_n1"] = round(t["value"] / (base / world), 6)
            t["scaling_basis"] = (f"{name} tile-gather Mpix/s / ({basis} / {world}): the assembled frame's speed-up "
                                  f"over one GPU's frame rate in this run ({'fused' if basis != 'value' else 'two-pass'})")
        ms = t.get("ms_per_step")
        if ms:
            t["root_ingress_GBps"] = round(t["root_ingress_bytes_per_frame"] / (ms * 1e-3) / 1e9, 3)


def make_group(rtm, world, rank, local, dist, backend):
    """librtm's group: one rank per process over RCCL (ncclCommInitRank, the 128-byte id
    from rank 0 handed over by torch.distributed).  At N = 1 there is nothing to gather
    (the one band renders in place), so no communicator is formed: the one-member group
    of the device-copy transport runs the same render path (a process that formed and
    destroyed one-device RCCL communicators later met illegal memory accesses on this
    pool, tests/test_zz_rccl_groups.py)."""
    import torch
    if backend != "nccl":
        return None
    if world == 1:
        return rtm.Group(n_devices=1, devices=[local], loopback=True)
    uid = torch.zeros(128, dtype=torch.uint8, device=f"cuda:{local}")
    if rank == 0:
        uid.copy_(torch.frombuffer(bytearray(rtm.Group.unique_id()), dtype=torch.uint8))
    dist.broadcast(uid, src=0)
    return rtm.Group(device=local, n_ranks=world, rank=rank, uid=bytes(uid.cpu().numpy().tobytes()))


def host_output(rtm, scene, eye, shadow, W, H, K, flags, frames=8, n_gpus=0):
    """The drop-in's host-output rate (PCIe included; never `value`): rtm_render_ex
    into pageable and registered host memory, RGBA f32 and writeColorImage's RGB8.
    n_gpus > 0: rtm_render_multi_ex over devices 0..n_gpus-1 from this process (the
    Rust host's multi-GPU frame, = rtm_group_render with rtm_group_set_host_direct):
    every device renders its row band and copies it over its own PCIe link into its
    rows of the host frame, no device-to-device hop."""
    import numpy as np
    res = {}
    for fmt, name in ((0, "rgba32f"), (2, "rgb8")):
        for reg in (False, True):
            buf = np.empty((H, W, 4), np.float32) if fmt == 0 else np.empty((H, W, 3), np.uint8)
            r = rtm.HostRegistration(buf) if reg else None
            try:
                kw = {"n_gpus": n_gpus} if n_gpus else {}
                rtm.render_frame_ex(scene, eye, shadow, W, H, K, flags, fmt, out=buf, **kw)
                t0 = time.perf_counter()
                for _ in range(frames):
                    rtm.render_frame_ex(scene, eye, shadow, W, H, K, flags, fmt, out=buf, **kw)
                el = (time.perf_counter() - t0) / frames
            finally:
                if r is not None:
                    r.close()
            res[f"{name}_{'registered' if reg else 'pageable'}"] = {
                "value": round(W * H / el / 1e6, 2), "unit": "Mpixels/s", "ms_per_frame": round(el * 1e3, 4),
                "bytes_per_frame": int(buf.nbytes), "GB_per_s": round(buf.nbytes / el / 1e9, 2)}
    res["note"] = ((f"rtm_render_multi_ex over {n_gpus} devices (row bands, fused shadow, each band over its "
                    "own device's PCIe link)" if n_gpus else "rtm_render_ex")
                   + ": blocking, the frame copied to host memory by every call, one frame at a time "
                   f"({frames} frames); registered = a buffer pinned once with rtm_host_register (direct DMA)")
    return res


def librtm_build_id() -> str:
    """sha256 (first 16 hex digits) of the librtm.so this run loads: the build a PMC
    summary must have profiled for its counters to describe the benched code."""
    import hashlib
    with open(os.path.join(ROOT, "2018rustraytracer_amd", "librtm.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()[:16]


def _latest_pmc(cfg_id: int, kernel: str, frames_per_launch: int = 1):
    """(file, per-launch counters) of `kernel` from the newest committed PMC summary
    (tools/profile_pmc.sh) of THIS librtm.so build (its `librtm_build_id` stamp,
    tools/pmc_summary.py) whose launches held `frames_per_launch` frames
    (`frames_per_launch` in the summary, 1 when absent); (None, None) if none: a
    summary of another build is never cited."""
    want = librtm_build_id()
    cands = []
    for f in glob.glob(os.path.join(ROOT, "profiles", "*pmc*.json")):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if (d.get("librtm_build_id") == want and d.get("config") == cfg_id and kernel in d.get("kernels", {})
                and d.get("frames_per_launch", 1) == frames_per_launch):
            cands.append((d.get("generated_unix", 0), f, d))
    if not cands:
        return None, None
    _, f, d = max(cands, key=lambda c: c[0])  # newest by the summary's own time stamp
    return os.path.relpath(f, ROOT), d["kernels"][kernel]


def _latest_traffic(cfg_id: int, kernel: str, frames_per_launch: int = 1):
    """HBM bytes per launch from the newest committed PMC summary (see _latest_pmc)."""
    _, k = _latest_pmc(cfg_id, kernel, frames_per_launch)
    return k.get("hbm_bytes_per_launch") if k else None


def pmc_fractions(cfg_id: int, kernel: str, frames_per_launch: int, alg_ops: int):
    """The counters' view of a kernel next to the algorithmic roofline (VERDICT r02
    item 6): issued f64 lane-ops (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F64 x 64) over the
    PMC run's own average duration against the non-FMA f64 peak, and the VALU issue
    fraction: issued wave-instructions x 2 cycles / (1024 SIMDs x 2.4 GHz x duration), and
    the VALU busy fraction with the f64 instructions at 4 cycles."""
    src, k = _latest_pmc(cfg_id, kernel, frames_per_launch)
    if not k or not k.get("avg_duration_ns_profiled"):
        return {"source": None, "librtm_build_id": librtm_build_id(),
                "note": "no committed PMC summary of this librtm.so build for this config and frames per launch"}
    dur = k["avg_duration_ns_profiled"] * 1e-9
    f64 = 64.0 * sum(k.get(c, 0.0) for c in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                              "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
    valu = k.get("SQ_INSTS_VALU", 0.0)
    f64_wi = f64 / 64.0
    waves = k.get("SQ_WAVES", 0.0) or 1.0
    return {"source": src, "librtm_build_id": librtm_build_id(), "kernel_name": k.get("kernel_name"),
            "duration_ns": round(k["avg_duration_ns_profiled"]),
            "issued_f64_lane_ops": int(f64), "issued_f64_frac": round(f64 / dur / 39.3e12, 4),
            "valu_issue_frac": round(valu * 2 / (1024 * 2.4e9 * dur), 4),
            # f64 wave-instructions hold the SIMD 4 cycles (16 f64 lanes per clock), the rest 2
            "valu_busy_frac": round((f64_wi * 4 + (valu - f64_wi) * 2) / (1024 * 2.4e9 * dur), 4),
            "valu_insts_per_wave": round(valu / waves, 1), "salu_insts_per_wave": round(k.get("SQ_INSTS_SALU", 0.0) / waves, 1),
            "algorithmic_over_issued_f64": round(alg_ops / f64, 3) if f64 else None,
            "note": "counters from the committed PMC summary of this config (same kernel, same frames per launch)"}


def available_cores():
    """The CPUs this process may actually run on, measured: the
    scheduler affinity mask, capped by the cgroup v2 CPU quota (cpu.max) when one is
    set, and by the job's CPU share in OMP_NUM_THREADS.  os.cpu_count() reports the
    whole machine and is recorded beside it."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    # the GPU box grants each GPU job a CPU share through OMP_NUM_THREADS (16 there)
    # without an affinity mask or quota: the share is honoured, and named as the limit
    omp = os.environ.get("OMP_NUM_THREADS", "")
    omp = int(omp) if omp.isdigit() and int(omp) > 0 else None
    lims = {"sched_getaffinity": aff, "cgroup_cpu_max": int(quota) if quota else None, "OMP_NUM_THREADS": omp}
    src, n = min(((k, v) for k, v in lims.items() if v), key=lambda kv: kv[1])
    return max(1, n), {"sched_getaffinity": aff, "cgroup_cpu_max_cpus": quota, "OMP_NUM_THREADS": omp,
                       "os_cpu_count": os.cpu_count(), "limited_by": src}


def cpu_baseline(scene, eye, shadow, w, h, k, flags, threads, what):
    """The CPU oracle (f64 C restatement of main.rs) on the host cores, rank 0 only:
    `threads` threads (default 1, the reference's sequential loops), plus the
    all-cores mode of BASELINE.md (OpenMP over row bands on every CPU the process
    may run on: available_cores(), measured, not assumed)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # checker / CPU baseline only

    oracle.lib()

    def best_of(n, nt):
        best = None
        for _ in range(n):
            t0 = time.perf_counter()
            oracle.render(scene, eye, shadow, w, h, k, flags, nthreads=nt)
            dt = time.perf_counter() - t0
            best = dt if best is None else min(best, dt)
        return best

    # a bounded sample, ~10 s of CPU work at config 3 (7 single-thread frames + 10 all-core frames)
    n_one, n_all = 7, 10
    best = best_of(n_one, threads)
    all_cores, core_probe = available_cores()
    best_all = best_of(n_all, all_cores)
    model = None  # log the host CPU model and hardware concurrency
    try:
        with open("/proc/cpuinfo") as f:
            model = next((l.split(":", 1)[1].strip() for l in f if l.startswith("model name")), None)
    except OSError:
        pass
    return dict(value=round(w * h / best / 1e6, 3), unit="Mpixels/s", cores=threads, kind="port",
                sample=f"full {w}x{h} frame, K={k}, {what}, best of {n_one}, {threads} thread(s)",
                cpu_model=model, hardware_concurrency=os.cpu_count(),
                seconds_per_frame=round(best, 3),
                all_cores={"value": round(w * h / best_all / 1e6, 3), "cores": all_cores,
                           "cores_probe": core_probe,
                           "seconds_per_frame": round(best_all, 4),
                           "sample": f"same frame, OpenMP over 8-row bands, best of {n_all}"})


def main():
    a = parse()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # one rank per GPU; a rehearsal with more ranks than GPUs (gloo) shares them round-robin
    local = local % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    if world > 1:
        if a.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group("gloo")
    tdev = f"cuda:{local}" if a.dist_backend == "nccl" else "cpu"  # where the timing reductions run

    rtm = importlib.import_module("2018rustraytracer_amd")
    sc = importlib.import_module("2018rustraytracer_amd.scenes")
    shard = importlib.import_module("2018rustraytracer_amd.shard")
    metrics = importlib.import_module("2018rustraytracer_amd.metrics")
    cfg = sc.CONFIGS[a.config]
    W, H, K = cfg["width"], cfg["height"], cfg["steps"]
    # frames per step: a step renders F frames of the sequence (at least 8, and at least
    # 8 Gpixel, at most 4096 frames: 1035 at 3840x2160, ~25 ms), so the driver's
    # --steps 20 run times >= 0.5 s of frames, the lanes' start and drain are a small
    # share of it, and a box's clock and noise average out over it (r03: 512 Mpixel,
    # a 33 ms timed region)
    F = a.frames_per_step or min(4096, max(8, (8 << 30) // (W * H)))
    nW, nS = a.warmup * F, a.steps * F  # warmup / timed frames
    tile_mode = a.mode == "tile-gather"
    # tile-gather: each band evaluates only the shadow texels it reads (no cross-rank shadow map)
    fused = a.fused or tile_mode
    flags = cfg["flags"] | (rtm.abi.RTM_FLAG_FUSED_SHADOW if fused else 0)
    eye, shadow = cfg.get("eye", sc.eye_camera)(), cfg.get("shadow", sc.shadow_camera)()
    ctx = rtm.Context(local)
    lib = rtm.load_library()
    # kernel durations: HIP events on every TIMING_STRIDE-th frame of the timed region
    # (an event is a barrier packet; timing every frame would cost ~15% throughput)
    timing_stride = max(10, nS // 1000)  # (at most ~1000 sampled launches: events cost host time to create)
    ctx.set_timing_capacity(max(1, nS // timing_stride))

    def scene_for(frame_index: int):
        if a.config >= 5:
            return cfg["scene"]()  # static scenes
        if a.config == 1:
            return sc.closely_orbiting_sphere(100 + frame_index)
        return sc.scene_a_bench(100 + frame_index)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def max_over_ranks(v: float) -> float:
        if world == 1:
            return v
        t = torch.tensor([v], dtype=torch.float64, device=tdev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    total = nW + nS
    # inputs prepared before the timed region: one scene per frame this rank renders
    # (frames mode: frames rank, rank+N, ...; tile-gather: every rank renders a band of every
    # frame), the animation cycling through its first 600 frames (the reference animates 300)
    n_distinct = min(total, 600)
    distinct = [scene_for(i if tile_mode else i * world + rank) for i in range(n_distinct)]
    scenes = [distinct[i % n_distinct] for i in range(total)]
    c_distinct = [s.to_c() for s in distinct]
    c_scenes = [c_distinct[i % n_distinct] for i in range(total)]
    # the RCCL group of the tile-partitioned frame: up front when it is the primary
    # measurement; for the secondary `tile_gather` field only after the headline frames
    # (a group that cannot be formed must never cost the headline line)
    group = make_group(rtm, world, rank, local, dist, a.dist_backend) if tile_mode else None

    # a ring of output frames (a renderer's swap chain): consecutive frames write
    # different buffers, so the library may run them side by side (rtm_api.cpp
    # frame_lanes puts frame i on lane (n-1-i) % L: the ring must be a multiple of L)
    # and batch (several frames per launch, rtm_ctx_set_batch: frames of one launch need
    # distinct outputs; batch b runs on lane (n_batches-1-b) % L, so the ring must be a
    # multiple of frames-per-launch x lanes): 48 frames from 4 Mpixel up (the auto
    # batches of 2-8 frames on 2-3 lanes; 25 GB at 7680x4320, of 288 GB), 128 below
    # (batches of up to 64 frames on 2 lanes)
    n_ring = 48 if W * H >= (4 << 20) else 128
    # the library's own plan for the timed call (rtm_ctx_frames_plan: its lanes and batch rules)
    plan_lanes, plan_batch = ctx.frames_plan(W, H, max(nS, 1))
    m = plan_lanes * plan_batch
    n_ring = n_ring if n_ring % m == 0 else m * ((n_ring + m - 1) // m)
    ring = ([torch.empty((H, W, 4), dtype=torch.float32, device=f"cuda:{local}") for _ in range(n_ring)]
            if not tile_mode else [])
    sequence = not tile_mode and not a.per_frame_calls

    import ctypes as C
    e_c, s_c = eye.to_c(), shadow.to_c()

    def frames_step(i: int):  # --per-frame-calls / --fused: one rtm_render_async per frame
        rc = lib.rtm_render_async(ctx.handle, C.byref(c_scenes[i][0]), C.byref(e_c), C.byref(s_c), W, H, K, flags,
                                  0, H, C.c_void_p(ring[i % n_ring].data_ptr()))
        rtm.abi.check(lib, rc, "rtm_render_async")

    if sequence:
        # the whole timed region is ONE rtm_render_frames_async call over the animation
        # frames (two kernels per frame or per batch of frames)
        warm = ctx.prepare_frames(scenes[:nW])
        timed = ctx.prepare_frames(scenes[nW:])
        outp = [ring[i % n_ring].data_ptr() for i in range(max(nW, nS, 1))]

    # clock ramp: frames for at least --preroll-ms of wall time before the counted warmup
    # (in chunks of one step, so its launches carry full batches like the timed ones: the
    # PMC passes average a kernel's counters over all of its launches)
    preroll_frames, t_pre = 0, time.perf_counter()
    n_pre = min(F, total)
    pre = ctx.prepare_frames(scenes[:n_pre]) if sequence and not tile_mode else None
    while (time.perf_counter() - t_pre) * 1e3 < a.preroll_ms and not tile_mode:
        if sequence:
            ctx.render_frames_async([0] * n_pre, eye, shadow, W, H, K, flags, outp[:n_pre], pre)
        else:
            for i in range(n_pre):
                frames_step(i)
        ctx.synchronize()
        preroll_frames += n_pre
    preroll = {"ms": round((time.perf_counter() - t_pre) * 1e3, 1), "frames": preroll_frames,
               "note": "untimed frames before the counted warmup, so the clocks have ramped (time-based)"}

    tg_primary = None
    if tile_mode:
        fmt = FORMATS[a.format]
        t_pre = time.perf_counter()
        while (time.perf_counter() - t_pre) * 1e3 < a.preroll_ms:  # clock ramp
            tile_gather(rtm, lib, ctx, group, world, rank, dist, tdev, c_scenes, eye, shadow, W, H, K, flags, fmt,
                        50, 0)
            preroll_frames += 50
        preroll["ms"], preroll["frames"] = round((time.perf_counter() - t_pre) * 1e3, 1), preroll_frames
        tg_primary = tile_gather(rtm, lib, ctx, group, world, rank, dist, tdev, c_scenes, eye, shadow, W, H, K,
                                 flags, fmt, nS, nW, bands=True)
        tile_scaling({a.format: tg_primary}, {}, world)  # (root ingress; no one-GPU rate in this mode)
        elapsed = tg_primary["ms_per_step"] * nS / 1e3
    else:
        if sequence:
            if nW:
                ctx.render_frames_async([0] * nW, eye, shadow, W, H, K, flags, outp[:nW], warm)
        else:
            for i in range(nW):
                frames_step(i)
        if sequence:  # the swap chain's pointer array, built before the clock starts like the scenes
            outs_timed = ctx.out_array(outp[:nS])
        barrier()
        ctx.set_timing_stride(timing_stride)  # restarts the stride count: launch 0 of the timed region is timed
        t0 = time.perf_counter()
        if sequence:
            ctx.render_frames_async([0] * nS, eye, shadow, W, H, K, flags, outs_timed, timed)
        else:
            for i in range(nW, total):
                frames_step(i)
        barrier()
        elapsed = max_over_ranks(time.perf_counter() - t0)

    # the shadow map's storage in the timed frames (coded: 1-2 B per texel; fused: none).
    # A frame without shadow raster and march (config 7, main()'s scene) has an all-+INF
    # shadow viewport: the library runs no shadow pass and its eye pass evaluates the
    # +INF texels on demand (rtm_api.cpp trivial_shadow), i.e. the fused frame's work
    trivial = (flags & 3) == 3 and not fused
    map_bytes = ctx.shadow_map_texel_bytes() or 8
    # what the last timed frame's shadow pass stored (span records: DESIGN.md §5)
    map_stored, span_records = ctx.shadow_map_stored_bytes() if not (fused or trivial) else (0, False)
    # per-kernel HIP-event durations over the timed region (ctx stream)
    n_launches = nS
    sh_ms, eye_ms = ctx.kernel_ms_history((n_launches + timing_stride - 1) // timing_stride)
    if tile_mode:  # the group's own contexts ran the bands: one timed pass of rank 0's band on ctx
        ctx.set_timing_capacity(1)
        r0, r1 = shard.row_band(H, world, rank)
        if r1 > r0:
            tmp = torch.empty(((r1 - r0) * W * rtm.abi.FORMAT_BYTES[FORMATS[a.format]] + 15) // 16 * 4,
                              dtype=torch.float32, device=f"cuda:{local}")
            for _ in range(3):
                ctx.render_rows_async(scenes[0], eye, shadow, W, H, K, flags | (0 if world == 1 else 4),
                                      FORMATS[a.format], tmp.data_ptr(), r0, r1)
            ctx.synchronize()
            sh_ms, eye_ms = ctx.kernel_ms_history(1)
        else:
            sh_ms, eye_ms = [0.0], [0.0]

    # batched launches (rtm_ctx_set_batch: several frames per launch): the events
    # time a launch, i.e. a batch of frames; the per-kernel figures are per frame
    batch = ctx.last_batch() if sequence else 1
    launch_batch = batch  # frames per launch of the kernels the roofline prices
    if batch > 1:
        sh_ms, eye_ms = [v / batch for v in sh_ms], [v / batch for v in eye_ms]

    # With several lanes (rtm_ctx_set_lanes: independent frames on side-by-side
    # streams) the kernels of the timed region overlap, and each event duration is
    # a kernel's time BESIDE other frames' kernels.  The kernel roofline is taken
    # from a one-lane pass over the same frames right after it (each kernel alone on
    # the chip); the headline value stays the timed region's.
    lanes = ctx.last_lanes() if sequence else 1
    in_lanes, one_lane = None, None
    if lanes > 1:
        avg = lambda v: sum(v) / max(len(v), 1)
        in_lanes = {"lanes": lanes, "shadow_pass_ms": round(avg(sh_ms), 5), "eye_pass_ms": round(avg(eye_ms), 5),
                    "note": "HIP-event kernel durations in the timed region, kernels of other lanes alongside"}
        n1 = min(nS, 400)
        ctx.set_lanes(1)
        ctx.render_frames_async([0] * min(nW, F), eye, shadow, W, H, K, flags, outp[:min(nW, F)],
                                ctx.prepare_frames(scenes[:min(nW, F)]))
        ctx.set_timing_capacity(n1)  # every launch of this short pass timed
        one = ctx.prepare_frames(scenes[nW:nW + n1])
        outs_one = ctx.out_array(outp[:n1])
        barrier()
        ctx.set_timing_stride(1)
        t1 = time.perf_counter()
        ctx.render_frames_async([0] * n1, eye, shadow, W, H, K, flags, outs_one, one)
        barrier()
        el1 = time.perf_counter() - t1
        sh_ms, eye_ms = ctx.kernel_ms_history(n1)
        b1 = ctx.last_batch()
        launch_batch = b1
        sh_ms, eye_ms = [v / b1 for v in sh_ms], [v / b1 for v in eye_ms]
        ctx.set_lanes(0)
        one_lane = {"value": round(W * H * n1 / el1 / 1e6, 2), "unit": "Mpixels/s", "frames": n1,
                    "ms_per_step": round(el1 / n1 * 1e3, 5),
                    "note": "same frames, one lane (one frame after another): the per-kernel durations "
                            "of `kernels` and `roofline` come from this pass"}

    # Secondary measurement, same run and frames (not the headline value): the
    # fused-shadow frame (RTM_FLAG_FUSED_SHADOW), which evaluates only the shadow
    # texels the eye pass looks up instead of materialising the whole shadow map.
    # Bit-identical image (tests/test_gpu_parity.py::test_fused_shadow_identical).
    alt_fused = None
    if sequence and not a.no_alt and not fused and not trivial:
        fflags = flags | rtm.abi.RTM_FLAG_FUSED_SHADOW
        ctx.set_timing_capacity(max(1, nS // timing_stride))
        ctx.render_frames_async([0] * min(nW, F), eye, shadow, W, H, K, fflags, outp[:min(nW, F)],
                                ctx.prepare_frames(scenes[:min(nW, F)]))
        barrier()
        ctx.set_timing_stride(timing_stride)
        t1 = time.perf_counter()
        ctx.render_frames_async([0] * nS, eye, shadow, W, H, K, fflags, outs_timed, timed)
        barrier()
        el_f = max_over_ranks(time.perf_counter() - t1)
        _, f_eye = ctx.kernel_ms_history((nS + timing_stride - 1) // timing_stride)
        f_eye = [v / max(ctx.last_batch(), 1) for v in f_eye]  # per frame
        alt_fused = {"value": round(W * H * nS * world / el_f / 1e6, 2), "unit": "Mpixels/s",
                     "ms_per_step": round(el_f / a.steps * 1e3, 5), "ms_per_frame": round(el_f / nS * 1e3, 5),
                     "fused_eye_pass_ms_in_lanes": round(sum(f_eye) / max(len(f_eye), 1), 5),
                     "lanes": ctx.last_lanes(),
                     "note": "RTM_FLAG_FUSED_SHADOW (shadow texels evaluated on demand in the eye pass, "
                             "bit-identical image); secondary measurement, not the headline value"}

    avg_sh = sum(sh_ms) / max(len(sh_ms), 1)
    avg_eye = sum(eye_ms) / max(len(eye_ms), 1)

    res = None
    if rank == 0:
        rows = shard.row_band(H, world, rank) if tile_mode else (0, H)
        pixels = W * H * nS * (1 if tile_mode else world)
        value = pixels / elapsed / 1e6
        s0 = scenes[nW] if nW < len(scenes) else scenes[0]
        band_h = rows[1] - rows[0]
        st = ctx.stats(s0, eye, shadow, W, H, K, flags)
        sep = metrics.shared_z_separable(shadow)
        def frame_work(fused_):
            return metrics.frame_work(st, W, H, len(s0.spherePrimitives), len(s0.patches), flags, fused=fused_,
                                      sep=sep, n_planes=len(s0.circlePlanePrimitives),
                                      n_cyls=len(s0.cappedCylinderPrimitives),
                                      perspective=eye.type_ == sc.PERSPECTIVE,
                                      search=sep,
                                      n_sdfs=len(s0.sdfPrimitives), map_texel_bytes=map_bytes,
                                      map_stored_bytes=map_stored if map_stored else None,
                                      span_records=span_records,
                                      moving=(shadow.dirNormalized[0] * 0.03 != 0.0
                                              or shadow.dirNormalized[1] * 0.03 != 0.0))

        work = frame_work(fused or trivial)
        if alt_fused is not None and band_h == H:
            # the fused frame is one kernel (the eye pass evaluating the shadow texels its
            # hit pixels read): its algorithmic bytes and ops per frame over its wall time
            # per frame in the same run
            rf = dict(metrics.roofline("eye_pass", frame_work(True), alt_fused["ms_per_frame"]))
            rf.pop("traffic", None)
            rf["kernel"] = "frame (fused shadow: one eye-pass kernel per frame)"
            rf["note"] = ("algorithmic bytes per frame (16 B/px store, no map) / wall time per frame "
                          f"of the alt_fused_shadow run ({alt_fused['lanes']} lanes); PMC: profiles/*pmc_fused*")
            alt_fused["roofline_frame"] = rf
        if band_h != H:  # rank 0 renders one band: scale the frame's work to it (approximate)
            for kk in work.values():
                kk["ops"] = int(kk["ops"] * band_h / H)
                kk["bytes"] = int(kk["bytes"] * band_h / H)
        # the whole frame (both passes' algorithmic bytes) over the headline time per frame
        passes = [work[k] for k in ("shadow_pass", "eye_pass") if k in work]
        work["frame"] = {"ops": sum(w["ops"] for w in passes), "bytes": sum(w["bytes"] for w in passes)}
        roof_frame = dict(metrics.roofline("frame", work, elapsed / nS * 1e3))  # per GPU
        roof_frame.pop("traffic", None)
        roof_frame["note"] = ("both passes' algorithmic bytes per frame / wall time per frame of the timed region"
                              + (f" ({lanes} lanes)" if lanes > 1 else ""))
        # the kernel rooflines are per LAUNCH (what rocprofv3 and the PMC passes see): a
        # launch of B frames (rtm_ctx_set_batch) moves B frames' bytes in its duration
        nb = max(launch_batch, 1)
        work_l = {k: {"ops": v["ops"] * nb, "bytes": v["bytes"] * nb} for k, v in work.items()}

        def kroof(kernel, ms_per_frame):
            fpl = nb if kernel in ("eye_pass", "shadow_pass") else 1
            r = dict(metrics.roofline(kernel, work_l, ms_per_frame * nb, _latest_traffic(a.config, kernel, fpl)))
            r["frames_per_launch"] = nb
            r["pmc"] = pmc_fractions(a.config, kernel, fpl, work_l[kernel]["ops"])
            return r

        dom = "eye_pass" if (fused or trivial or avg_eye >= avg_sh) else "shadow_pass"
        dom_ms = avg_eye if dom == "eye_pass" else avg_sh
        roof = kroof(dom, dom_ms)
        other = "shadow_pass" if dom == "eye_pass" else "eye_pass"
        other_ms = avg_sh if other == "shadow_pass" else avg_eye
        roof_other = kroof(other, other_ms) if other_ms > 0 and not trivial else None
        res = {
            "metric": cfg.get("metric", METRIC if a.config <= 5 else METRIC_F1 if a.config <= 7 else METRIC_F4),
            "value": round(value, 2),
            "unit": "Mpixels/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 5),
            "frames_per_step": F,
            "ms_per_frame": round(elapsed / nS * 1e3, 5),
            "higher_is_better": True,
            "scaling": "strong" if tile_mode else "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic: Scene A-bench (SURVEY.md §8d-2) animation frames 100+i, f64 scene built on host"
                     if a.config in (2, 3, 4) else "synthetic: SURVEY.md §8d-2 scene" if a.config <= 5
                     else "synthetic: row f-1 scene (scenes.py), f64 scene built on host" if a.config <= 7
                     else "synthetic: row f-4 Scene S-bench (scenes.py), f64 scene built on host" if a.config == 8
                     else "synthetic: " + cfg["desc"]),
            "config": {"workload": cfg["desc"], "config_id": a.config, "width": W, "height": H,
                       "march_steps": K, "mode": a.mode, "shadow": ("fused" if fused else "none: all-+INF viewport (no shadow raster or march), "
                                 "eye pass only" if trivial else "two-pass"),
                       "parallelism": (f"frame-parallel x{world}" if not tile_mode
                                       else f"row-bands x{world} + one gather ({a.format})"),
                       "rows_rank0": band_h},
            "kernels": {"shadow_pass_ms": round(avg_sh, 5), "eye_pass_ms": round(avg_eye, 5),
                        "frame_kernel_ms": round(avg_sh + avg_eye, 5)},
            "roofline": roof,
            "roofline_other_kernel": roof_other,
            "roofline_frame": roof_frame,
            "shadow_map_texel_bytes": None if (fused or trivial) else map_bytes,
            "shadow_map_stored_bytes_per_frame": None if (fused or trivial) else map_stored,
            "shadow_map_span_records": None if (fused or trivial) else span_records,
            "lanes": lanes,
            "frames_per_launch": batch,
            "kernels_in_lanes": in_lanes,
            "one_lane": one_lane,
            "preroll": preroll,
            "alt_fused_shadow": alt_fused,
            "tile_gather": tg_primary if tile_mode else None,
            "host_output": None,
            "parity": ("bit-exact vs CPU oracle (tests/test_gpu_parity.py)" if a.config <= 5
                       else "bit-exact vs CPU oracle (tests/test_raytrace.py)" if a.config <= 8
                       else "bit-exact vs CPU oracle (tests/test_general_march.py)"),
        }

    # Secondary: the tile-partitioned, gathered frame (strong scaling) in RGBA f32 and RGBA8
    tile = None
    if not tile_mode and a.tile_gather_steps != 0:
        tile = {}
        # a watchdog for the secondary measurement: RCCL over several ranks is exercised
        # here for the first time in a run; if it stalls, rank 0 still prints the line
        watchdog = _Watchdog(a.tile_gather_timeout_s, res, "tile_gather")
        try:
            group = make_group(rtm, world, rank, local, dist, a.dist_backend)
        except Exception as ex:
            tile["error"] = f"group: {str(ex)[:300]}"
        tg_scenes = [scene_for(i) for i in range(min(total, 64))]
        tg_c = [s.to_c() for s in tg_scenes]
        # every band count renders the same algorithm: each band evaluates the shadow
        # texels it reads (N = 1 included, so the N = 1 figure is the strong-scaling base)
        tflags = cfg["flags"] | rtm.abi.RTM_FLAG_FUSED_SHADOW
        # (auto: at least 2048 frames and 16 Gpixel, at most 16384 -- 2048 frames, ~50 ms at
        # 3840x2160: a 512-frame call read 1-2 % low from the lanes' start and drain)
        tg_steps = (a.tile_gather_steps if a.tile_gather_steps >= 0
                    else min(16384, max(2048, (16 << 30) // (W * H))))
        for name, fmt in FORMATS.items():
            if "error" in tile:
                break
            try:
                # (warmup: one call of the same shape, so every lane's table slots and
                # pinned buffers are allocated before the clock, as in frames mode)
                tile[name] = tile_gather(rtm, lib, ctx, group, world, rank, dist, tdev, tg_c, eye, shadow, W, H, K,
                                         tflags, fmt, tg_steps, tg_steps,
                                         bands=name == "rgba32f")
            except Exception as ex:  # a failed secondary measurement must not lose the headline line
                tile[name] = {"error": str(ex)[:300]}
                break
        watchdog.cancel()
        if res is not None:
            tile_scaling(tile, res, world)
            res["tile_gather"] = tile
    if group is not None:
        try:
            group.close(120_000)  # (bounded: a stalled peer cannot hang the run's exit)
        except Exception as ex:
            if res is not None:
                res["group_close_error"] = str(ex)[:300]

    if world > 1 and not a.no_host_output and a.config in (3, 4):
        # the N-link host frame: rank 0 drives all N devices while the others wait
        barrier()
        if rank == 0:
            if torch.cuda.device_count() >= world:
                try:
                    res["host_output"] = host_output(rtm, scenes[0], eye, shadow, W, H, K, cfg["flags"],
                                                     n_gpus=world)
                except Exception as ex:
                    res["host_output"] = {"error": str(ex)[:300]}
            else:
                res["host_output"] = {"skipped": f"{torch.cuda.device_count()} visible devices < {world} ranks"}
        barrier()
    if rank == 0:
        if world == 1 and not a.no_host_output and a.config == 3:
            res["host_output"] = host_output(rtm, scenes[0], eye, shadow, W, H, K, cfg["flags"])
        if world == 1 and not a.no_cpu_baseline:
            what = ("Scene A-bench frame 100" if a.config in (2, 3, 4) else cfg["desc"].split(", ", 1)[1])
            res["cpu_baseline"] = cpu_baseline(s0, eye, shadow, W, H, K, flags, a.cpu_threads, what)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
