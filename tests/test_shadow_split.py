"""The split coded shadow launch: per batch (when the batch's sphere box
covers at most 0.3 of the map), the 16-row tiles that meet a frame's sphere box run
the full tile and every other texel is written by a raster-free instantiation with
16-row waves that skip the rows of the box; both decide on the same 16-row blocks, so
each texel is written once.  These cases stress the partition: spheres that move
between the frames of one launch (the sphere grid spans the batch's union box, a
tile outside its own frame's box leaves), spheres partly or wholly outside the
viewport, frames without spheres beside frames with them, heights and widths that
are not multiples of the tiles, 1- and 2-byte codes.  Every frame's image and
every frame's shadow map (each frame rendered last once, by rotating the batch)
== the oracle's, bit for bit."""
import dataclasses
import os

import pytest

from conftest import bits_equal, first_mismatch
from test_headline_mode import _smap

pytestmark = pytest.mark.gpu

NT = min(16, os.cpu_count() or 1)


def _moved(s, dx, dy):
    """The scene with every sphere shifted by (dx, dy) in the shadow viewport's plane."""
    sp = [dataclasses.replace(p, pos=(p.pos[0] + dx, p.pos[1] + dy, p.pos[2])) for p in s.spherePrimitives]
    return dataclasses.replace(s, spherePrimitives=sp)


def _frames(scenes, which):
    a = scenes.scene_a_bench
    b = scenes.scene_b()
    bare = scenes.Scene([], list(b.patches))
    if which == "moving":  # the orbiting sphere at four times: one union box, four frame boxes
        return [a(100), a(140), a(180), a(220)]
    if which == "edges":  # spheres across the left/right/top/bottom edges and wholly outside
        s = a(100)
        return [_moved(s, -0.9, 0.0), _moved(s, 0.9, 0.3), _moved(s, 0.2, -0.95), _moved(s, 3.0, 3.0)]
    if which == "mixed":  # 16 spheres, none, 16 moved, none (K = 240: 2-byte codes)
        return [b, bare, _moved(b, 0.3, -0.2), bare]
    raise ValueError(which)


CASES = [
    # (frames, width, height, K)
    ("moving", 3840, 2160, 64),
    ("moving", 333, 97, 33),
    ("edges", 770, 203, 64),
    ("edges", 1000, 515, 90),
    ("mixed", 517, 299, 240),
]


@pytest.mark.parametrize("case", CASES, ids=[f"{c[0]}-{c[1]}x{c[2]}-K{c[3]}" for c in CASES])
def test_split_launch_every_frame_and_map(rtm, oracle, scenes, case):
    import torch
    which, w, h, k = case
    frames = _frames(scenes, which)
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    want = [oracle.render(s, eye, sh, w, h, k, 0, nthreads=NT, want_shadow=True) for s in frames]
    ctx = rtm.Context(0)
    outs = [torch.empty((h, w, 4), dtype=torch.float32, device="cuda") for _ in frames]
    try:
        ctx.set_batch(len(frames))
        ctx.set_lanes(1)
        for r in range(len(frames)):
            order = [(r + 1 + i) % len(frames) for i in range(len(frames))]  # frame r last
            torch.cuda.synchronize()
            ctx.render_frames_async([frames[i] for i in order], eye, sh, w, h, k, 0,
                                    [outs[i].data_ptr() for i in order])
            ctx.synchronize()
            assert ctx.last_batch() == len(frames)
            if r == 0:
                for i, o in enumerate(outs):
                    got = o.cpu().numpy()
                    assert bits_equal(got, want[i]["rgba"]), (i, first_mismatch(got, want[i]["rgba"]))
            m = _smap(ctx, w, h)
            assert bits_equal(m, want[r]["shadow"]), ("map", r, first_mismatch(m, want[r]["shadow"]))
    finally:
        ctx.close()
        torch.cuda.empty_cache()


CHILD = r'''
import importlib, os, sys
sys.path.insert(0, %(root)r)
sys.path.insert(0, %(root)r + "/oracle")
sys.path.insert(0, %(root)r + "/tests")
import oracle
rtm = importlib.import_module("2018rustraytracer_amd")
scenes = importlib.import_module("2018rustraytracer_amd.scenes")
import test_shadow_split as t
for case in [("mixed", 517, 299, 240), ("edges", 770, 203, 64)]:
    t.test_split_launch_every_frame_and_map(rtm, oracle, scenes, case)
print("CHILD_OK")
'''


@pytest.mark.parametrize("bound", ["1.0", "0"])
def test_split_forced_on_and_off_in_subprocess(bound):
    """The same partition checks with the split forced for any box (the 16-sphere frames
    too; RTM_CODED_SPLIT_MAX=1.0) and with one launch for every batch (0), in child
    processes (the bound is read once per process)."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RTM_CODED_SPLIT_MAX=bound)
    r = subprocess.run([sys.executable, "-c", CHILD % {"root": root}], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0 and "CHILD_OK" in r.stdout, r.stdout[-2000:] + r.stderr[-3000:]
