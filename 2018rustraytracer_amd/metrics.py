"""Algorithmic work per frame and the MI355X roofs it is priced against.

Counting rules: every f64 add/sub/mul/div/sqrt/compare is one
flop (no FMA: contraction is off), per-(camera, sphere) constants are hoisted.

  eye pass     per pixel  6 + 15*S   (+6 per covering sphere, +89 per hit pixel)
  shadow pass  per texel  6 + 15*S   (+6 per covering sphere)
               per (texel, patch) 31 (march setup + final compare)
               per march iteration 22 (main.rs:2247-2274)

Algorithmic HBM bytes (what the two-kernel design must move):
  shadow pass  8 B per texel            (f64 shadow-map store)
  eye pass     16 B per pixel           (RGBA f32 store)
             + 8 B per hit pixel        (f64 shadow-map lookup)
"""
from __future__ import annotations

# MI355X peaks (/opt/skills/guides/MI355X_MICROARCH.md; FP64 vector is the datasheet
# value, FMA counted as 2 flops — this path issues no FMA, so its VALU ceiling
# in these units is half of it).
PEAK_HBM_GBS = 8000.0
PEAK_FP64_VECTOR_TFLOPS = 78.6


def frame_work(stats: dict, width: int, height: int, n_spheres: int, n_patches: int, flags: int = 0,
               fused: bool = False) -> dict:
    px = width * height
    no_march = bool(flags & 0x1)
    no_sraster = bool(flags & 0x2)
    eye_flops = px * (6 + 15 * n_spheres) + 6 * stats["eye_sphere_tests"] + 89 * stats["eye_hit_pixels"]
    texels = px if not fused else stats["eye_hit_pixels"]
    sh_flops = 0
    if not no_sraster:
        sh_flops += texels * (6 + 15 * n_spheres) + 6 * stats["shadow_sphere_tests"]
    if not no_march:
        sh_flops += texels * n_patches * 31 + 22 * stats["march_iterations"]
    sh_bytes = 0 if fused else 8 * px
    eye_bytes = 16 * px + (0 if fused else 8 * stats["eye_hit_pixels"])
    return dict(shadow_pass=dict(flops=sh_flops, bytes=sh_bytes),
                eye_pass=dict(flops=eye_flops + (sh_flops if fused else 0), bytes=eye_bytes))


def roofline(kernel: str, work: dict, ms: float, traffic_bytes=None) -> dict:
    """Both roofs for one kernel; `bound` is the one it sits closer to."""
    w = work[kernel]
    s = ms * 1e-3
    gbs = w["bytes"] / s / 1e9 if s > 0 else 0.0
    tfl = w["flops"] / s / 1e12 if s > 0 else 0.0
    hbm = dict(bound="hbm", achieved=round(gbs, 2), peak=PEAK_HBM_GBS, unit="GB/s",
               frac=round(gbs / PEAK_HBM_GBS, 4))
    alu = dict(bound="valu_fp64", achieved=round(tfl, 3), peak=PEAK_FP64_VECTOR_TFLOPS, unit="TFLOP/s",
               frac=round(tfl / PEAK_FP64_VECTOR_TFLOPS, 4))
    main, other = (hbm, alu) if hbm["frac"] >= alu["frac"] else (alu, hbm)
    main = dict(main)
    main["kernel"] = kernel
    main["traffic"] = traffic_bytes
    main["other_roof"] = other
    main["algorithmic_bytes_per_launch"] = w["bytes"]
    main["algorithmic_flops_per_launch"] = w["flops"]
    main["avg_launch_ms"] = round(ms, 5)
    return main
