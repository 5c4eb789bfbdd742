"""State carried across frames on one context: long seeded
random frame sequences through rtm_render_frames_async on ONE reused context,
compared frame by frame with the oracle.

Round 3 shipped a bug of exactly this class: with shadow raster on and no sphere
covering the map, the empty sphere union "met" the top-left strip and the split
shadow launch left it to a part it never ran, so that strip kept the previous
frame's codes (fixed in 270eecd, pinned by tests/test_empty_sphere_union.py).  The
frames here vary everything a context keeps between frames:

  * 0-16 spheres, ids permuted; spheres wholly off the shadow and eye viewports
    (an empty union), spheres covering the whole map, ordinary ones;
  * patch sets changing between frames and calls (the march tables are rebuilt
    mid-sequence, and frames with different patches split a batch);
  * circle planes in front of the eye, so a hit looks up the shadow map where no
    sphere is (the stale strip of the round-3 bug is visible only that way);
  * march steps from 8 to 250, so 1- and 2-byte map codes alternate on a context;
  * the auto lanes and frames per launch, and forced 1-4 lanes x 1-8 frames;
  * flags: the two-pass frame, no march, no shadow raster, neither (the all-+INF
    viewport, no shadow pass), an ORTHOGONAL and a PERSPECTIVE eye;
  * image sizes that are no multiple of the tiles (rebuilt tables, ragged tiles).

After every call: every frame's RGBA f32 image and the last frame's shadow map
equal the oracle's bit for bit, and no side-table read left its table
(rtm_ctx_oob_reads == 0).  Seeded splitmix64 (seed 0x2018): the sequence is the
same on every run.  References: testscene_closelyOrbitingSphere's animation loop
(main.rs:1468-1633) renders such a sequence frame after frame on one set of
viewports; Viewport::rasterize / processRaymarchingRays / renderColorImage
(main.rs:445, 551, 710)."""
import ctypes
import os

import numpy as np
import pytest

from conftest import bits_equal, first_mismatch
from test_bounds import oob

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)
SEED = 0x2018
M64 = (1 << 64) - 1


class SplitMix64:
    def __init__(self, seed: int):
        self.s = seed & M64

    def next(self) -> int:
        self.s = (self.s + 0x9E3779B97F4A7C15) & M64
        z = self.s
        z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
        z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
        return z ^ (z >> 31)

    def below(self, n: int) -> int:
        return self.next() % n

    def unit(self) -> float:  # [0, 1)
        return (self.next() >> 11) * (1.0 / (1 << 53))

    def uniform(self, a: float, b: float) -> float:
        return a + (b - a) * self.unit()

    def pick(self, seq):
        return seq[self.below(len(seq))]


def _patch_sets(scenes):
    P = scenes
    return [[], [P.BENCH_PATCH], [P.REFERENCE_PATCH], [P.BENCH_PATCH, P.SCENE_B_PATCH2],
            [P.Bilinear(P.Linear(0.2, 1.4), P.Linear(0.6, 2.2))]]


def _sphere(scenes, rng, kind: str, sid: int):
    col = scenes.Shading(rng.uniform(0.02, 1.0), rng.uniform(0.02, 1.0), rng.uniform(0.02, 1.0))
    if kind == "off":  # off the shadow map (|x| or |y| > 1 + r) and off the eye's view (|y| > 1 + r)
        y = rng.pick([-1.0, 1.0]) * rng.uniform(1.6, 3.0)
        return scenes.PrimitiveSphere(sid, col, (rng.uniform(-3.0, 3.0), y, rng.uniform(-0.8, 0.8)), 0.2)
    if kind == "cover":  # covers every texel of the map
        return scenes.PrimitiveSphere(sid, col, (0.0, 0.0, rng.uniform(1.5, 2.5)), rng.uniform(2.0, 3.0))
    return scenes.PrimitiveSphere(sid, col, (rng.uniform(-0.9, 0.9), rng.uniform(-0.9, 0.9), rng.uniform(-0.9, 0.9)),
                                  rng.uniform(0.02, 0.35))


def _scene(scenes, rng, patches):
    mode = rng.below(8)
    ns = 0 if mode == 0 else rng.pick([1, 2, 3, 4, 7, 16]) if mode < 7 else 16
    kinds = []
    for _ in range(ns):
        r = rng.below(10)
        kinds.append("off" if r < 3 else "cover" if r == 3 else "normal")
    if mode == 1:
        kinds = ["off"] * ns  # every sphere off the map: an empty union with raster on
    ids = list(range(ns))
    for i in range(ns - 1, 0, -1):  # Fisher-Yates with the seeded stream
        j = rng.below(i + 1)
        ids[i], ids[j] = ids[j], ids[i]
    s = scenes.Scene([_sphere(scenes, rng, k, ids[i]) for i, k in enumerate(kinds)], list(patches))
    if rng.below(3) == 0:  # circle planes facing the orthographic eye (and visible to the perspective one)
        n = 1 + rng.below(3)
        s.circlePlanePrimitives = [
            scenes.PrimitiveCirclePlane(
                i, scenes.Shading(rng.uniform(0.1, 1.0), rng.uniform(0.1, 1.0), rng.uniform(0.1, 1.0)),
                rng.uniform(0.1, 0.6),
                # the first one over the map's top-left corner (texels x < 128, y < 16)
                (rng.uniform(-0.99, 0.9), -0.97 if i == 0 else rng.uniform(-0.9, 0.9), rng.uniform(-0.9, 0.9)),
                scenes.normalize((-1.0, rng.uniform(-0.3, 0.3), rng.uniform(-0.3, 0.3))))
            for i in range(n)]
    return s


def _smap(ctx, w, h):
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    m = np.empty((h, w), np.float64)
    p = ctx.shadow_map_ptr()
    assert p, "no shadow map"
    assert hip.hipMemcpy(m.ctypes.data, p, w * h * 8, 2) == 0
    return m


SIZES = [(256, 192), (200, 136), (384, 100), (130, 70)]
STEPS = [8, 16, 64, 250]  # 250 + 16 spheres: 2-byte codes
FLAGS = [0, 0, 0, 1, 2, 3]  # two-pass (most), no march, no shadow raster, neither


@pytest.mark.parametrize("chunk", range(4))
def test_random_frame_sequences_on_one_context(rtm, oracle, scenes, chunk):
    """chunk c: calls 12c .. 12c+11 of the seeded sequence (the stream is advanced over
    the earlier chunks' draws, so every chunk is the same on every run and the four
    chunks run on one context in order)."""
    import torch
    rng = SplitMix64(SEED)
    patch_sets = _patch_sets(scenes)
    sh_cam = scenes.shadow_camera()
    ctx = _ctx(rtm)
    n_calls = 12
    checked = 0
    for call in range(n_calls * (chunk + 1)):
        w, h = rng.pick(SIZES)
        k = rng.pick(STEPS)
        flags = rng.pick(FLAGS)
        persp = rng.below(4) == 0
        eye = scenes.perspective_eye_camera() if persp else scenes.eye_camera()
        n = 1 + rng.below(12)
        lanes, batch = (0, 0) if rng.below(3) == 0 else (1 + rng.below(4), 1 + rng.below(8))
        frames, ps = [], rng.pick(patch_sets)
        for i in range(n):
            if rng.below(4) == 0:
                ps = rng.pick(patch_sets)  # the patch set changes mid-call
            frames.append(_scene(scenes, rng, ps))
        same_out = rng.below(8) == 0  # every frame into one buffer: the last one must land last
        if call < n_calls * chunk:
            continue  # (an earlier chunk's call: the draws above keep the stream in step)
        outs = [torch.full((h, w, 4), float("nan"), dtype=torch.float32, device="cuda")
                for _ in range(1 if same_out else n)]
        ptrs = [outs[0].data_ptr()] * n if same_out else [o.data_ptr() for o in outs]
        ctx.set_lanes(lanes)
        ctx.set_batch(batch)
        torch.cuda.synchronize()
        ctx.render_frames_async(frames, eye, sh_cam, w, h, k, flags, ptrs)
        ctx.synchronize()
        what = f"call {call}: {w}x{h} K={k} flags={flags} persp={persp} n={n} lanes={lanes} batch={batch}"
        assert oob(rtm, ctx) == 0, what
        check = [n - 1] if same_out else range(n)
        for i in check:
            want = oracle.render(frames[i], eye, sh_cam, w, h, k, flags, nthreads=NT, want_shadow=i == n - 1)
            got = (outs[0] if same_out else outs[i]).cpu().numpy()
            assert bits_equal(got, want["rgba"]), f"{what}, frame {i}: {first_mismatch(got, want['rgba'])}"
            if i == n - 1:
                m = _smap(ctx, w, h)
                assert bits_equal(m, want["shadow"]), f"{what}, last map: {first_mismatch(m, want['shadow'])}"
            checked += 1
        del outs
    ctx.set_lanes(0)
    ctx.set_batch(0)
    assert checked > 0


_CTX = {}


def _ctx(rtm):
    """ONE context for every chunk of the sequence (state carried across chunks)."""
    if "c" not in _CTX:
        _CTX["c"] = rtm.Context(0)
        assert oob(rtm, _CTX["c"]) >= 0  # (clears the device-wide count)
    return _CTX["c"]
