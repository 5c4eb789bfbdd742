"""writeColorImage (main.rs:660-704) on the GPU: RGB8 encode + P3 text.

The product encodes with 255 host-computed thresholds (rtm_api.cpp encode_table)
instead of calling powf per channel.  That is bit-identical to the reference's
`(powf(clamp(c), 1/2.2) * 255) as i64` iff the composition is monotone in c;
test_encode_exhaustive_monotone proves it over every f32 in [0, 1] with the
oracle's libm powf (the function the Rust binary links).
"""
import ctypes as C
import ctypes.util

import numpy as np
import pytest

from conftest import bits_equal  # noqa: F401


def _edge_values(thresholds):
    """Every threshold, its f32 neighbours, and the clamp/NaN/inf corner cases."""
    t = thresholds[1:].astype(np.float32)
    v = [t, np.nextafter(t, np.float32(-1)), np.nextafter(t, np.float32(2))]
    special = np.array([0.0, -0.0, 1.0, np.nextafter(np.float32(1), np.float32(0)), 1.0000001, 2.0, -1.0,
                        1e-45, 1e-38, 1e15, -1e15, 3.4e38, np.inf, -np.inf, np.nan, -np.nan], np.float32)
    snan = np.array([0x7F800001, 0xFF800001, 0x7FBFFFFF], np.uint32).view(np.float32)
    return np.concatenate(v + [special, snan]).astype(np.float32)


def _image(h, w, values, seed=0):
    rng = np.random.default_rng(seed)
    img = rng.choice(values, size=(h, w, 4)).astype(np.float32)
    img[..., 3] = 1.0
    return img


def test_encode_exhaustive_monotone(oracle, rtm):
    """All 1,065,353,217 f32 in [+0, 1]: the libm byte map never decreases, and
    its thresholds are exactly the product library's table."""
    violations, t = oracle.encode_scan(8)
    assert violations == 0
    assert bits_equal(t, rtm.encode_thresholds())
    assert t[0] == 0.0 and t[255] <= 1.0 and np.all(np.diff(t) > 0)


def test_oracle_encode_matches_libm_powf(oracle):
    """oracle.encode_rgb8 == clamp -> libm powf(v, 1f/2.2f) -> (v*255f) as i64, per channel."""
    libm = C.CDLL(ctypes.util.find_library("m"))
    libm.powf.restype = C.c_float
    libm.powf.argtypes = [C.c_float, C.c_float]
    e = np.float32(1.0) / np.float32(2.2)
    rng = np.random.default_rng(3)
    vals = np.concatenate([rng.uniform(-0.2, 1.2, 3000).astype(np.float32),
                           np.array([0.0, 1.0, np.nan, np.inf, -np.inf, 1e15], np.float32)])
    img = np.zeros((len(vals), 4), np.float32)
    img[:, 0] = vals
    got = oracle.encode_rgb8(img)[:, 0]
    for v, g in zip(vals, got):
        c = np.float32(0.0) if np.isnan(v) else np.float32(min(max(v, np.float32(0)), np.float32(1)))
        p = np.float32(libm.powf(float(c), float(e)))
        assert g == int(np.float32(p * np.float32(255.0))), (v, g)


def test_threshold_rank_equals_oracle(oracle, rtm):
    """The product's rule (rank among thresholds) on every edge value == oracle."""
    t = rtm.encode_thresholds()
    vals = _edge_values(t)
    img = np.zeros((len(vals), 4), np.float32)
    img[:, 0] = vals
    want = oracle.encode_rgb8(img)[:, 0]
    c = np.where(np.isnan(vals), np.float32(0), np.clip(vals, 0, 1)).astype(np.float32)
    rank = np.searchsorted(t, c, side="right") - 1
    assert np.array_equal(rank, want)


def test_oracle_ppm_text_format(oracle):
    """rtmo_write_ppm == the reference's format!() sequence rebuilt in Python."""
    img = _image(3, 5, np.array([0.0, 0.5, 1.0, 0.001, 0.9, np.nan], np.float32))
    b = oracle.encode_rgb8(img)
    want = "P3\n5 3\n255\n" + "".join(
        "".join(f"{b[y, x, 0]} {b[y, x, 1]} {b[y, x, 2]}  " for x in range(5)) + "\n" for y in range(3))
    assert oracle.write_ppm(img) == want.encode()


def test_ppm_max_bytes(rtm):
    lib = rtm.load_library()
    assert lib.rtm_ppm_max_bytes(0, 5) == 0
    assert lib.rtm_ppm_max_bytes(2, 1) >= len(b"P3\n2 1\n255\n255 255 255  255 255 255  \n")
    w, h = 32768, 32768
    assert lib.rtm_ppm_max_bytes(w, h) >= len(f"P3\n{w} {h}\n255\n") + w * h * 13 + h


# --------------------------------------------------------------------------- GPU


def _dev(img):
    import torch
    return torch.from_numpy(np.ascontiguousarray(img)).to("cuda:0")


@pytest.mark.gpu
def test_gpu_encode_rgb8_edges(gpu_ctx, oracle, rtm):
    import torch
    vals = _edge_values(rtm.encode_thresholds())
    img = np.zeros((len(vals), 4), np.float32)
    img[:, 0] = vals
    img[:, 1] = vals[::-1]
    img[:, 2] = np.roll(vals, 7)
    d = _dev(img)
    out = torch.empty(len(vals) * 3, dtype=torch.uint8, device="cuda:0")
    gpu_ctx.encode_rgb8_async(d.data_ptr(), len(vals), out.data_ptr())
    gpu_ctx.synchronize()
    assert np.array_equal(out.cpu().numpy().reshape(-1, 3), oracle.encode_rgb8(img).astype(np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("n,rgb_off", [(1, 0), (3, 1), (5, 2), (4097, 3), (100003, 1), (65536, 0)])
def test_gpu_encode_rgb8_ragged_unaligned(gpu_ctx, oracle, rtm, n, rgb_off):
    """n % 4 tails and byte-aligned RGB destinations (the byte-store path)."""
    import torch
    vals = _edge_values(rtm.encode_thresholds())
    img = _image(1, n, vals, seed=n)[0]
    d = _dev(img)
    buf = torch.full((n * 3 + 8,), 0xAB, dtype=torch.uint8, device="cuda:0")
    torch.cuda.synchronize()
    gpu_ctx.encode_rgb8_async(d.data_ptr(), n, buf.data_ptr() + rgb_off)
    gpu_ctx.synchronize()
    got = buf.cpu().numpy()
    assert np.array_equal(got[rgb_off:rgb_off + 3 * n].reshape(n, 3), oracle.encode_rgb8(img).astype(np.uint8))
    assert np.all(got[:rgb_off] == 0xAB) and np.all(got[rgb_off + 3 * n:] == 0xAB)


@pytest.mark.gpu
def test_gpu_encode_rejects_misaligned_rgba(gpu_ctx, rtm):
    import torch
    lib = rtm.load_library()
    d = torch.zeros(64, dtype=torch.float32, device="cuda:0")
    o = torch.zeros(64, dtype=torch.uint8, device="cuda:0")
    assert lib.rtm_encode_rgb8_async(gpu_ctx.handle, C.c_void_p(d.data_ptr() + 4), 4, C.c_void_p(o.data_ptr())) == -1
    assert b"aligned" in lib.rtm_last_error()


@pytest.mark.gpu
def test_gpu_encode_rgb8_every_float_in_range(gpu_ctx, oracle, rtm):
    """Every f32 bit pattern in [0, 1] (1.07e9 values, device-resident), encoded
    on the GPU, equals the threshold rank — checked on the GPU by comparing with
    the thresholds' step function (searchsorted on device)."""
    import torch
    t = torch.from_numpy(rtm.encode_thresholds()).to("cuda:0")
    top = 0x3F800000
    chunk = 1 << 26
    rgb = torch.empty(chunk * 3, dtype=torch.uint8, device="cuda:0")
    for b0 in range(0, top + 1, chunk):
        n = min(chunk, top + 1 - b0)
        bits = torch.arange(b0, b0 + n, dtype=torch.int64, device="cuda:0").to(torch.int32)
        v = bits.view(torch.float32)
        img = torch.zeros((n, 4), dtype=torch.float32, device="cuda:0")
        img[:, 0] = v
        torch.cuda.synchronize()  # img is written on torch's stream, encoded on the context's
        gpu_ctx.encode_rgb8_async(img.data_ptr(), n, rgb.data_ptr())
        want = torch.searchsorted(t, v, right=True) - 1
        gpu_ctx.synchronize()
        got = rgb[: 3 * n].view(n, 3)[:, 0].to(torch.int64)
        assert torch.equal(got, want), f"mismatch in chunk starting at bits {b0:#x}"


@pytest.mark.gpu
@pytest.mark.parametrize("w,h", [(1, 1), (5, 3), (255, 2), (256, 2), (257, 3), (300, 7), (1000, 1)])
def test_gpu_write_ppm_ragged(gpu_ctx, oracle, rtm, w, h):
    vals = _edge_values(rtm.encode_thresholds())
    img = _image(h, w, vals, seed=w * 7 + h)
    d = _dev(img)
    assert gpu_ctx.write_ppm(d.data_ptr(), w, h) == oracle.write_ppm(img)


@pytest.mark.gpu
@pytest.mark.parametrize("fill", [0.0, 1.0])
def test_gpu_write_ppm_min_max_length(gpu_ctx, oracle, rtm, fill):
    w, h = 640, 480
    img = np.full((h, w, 4), fill, np.float32)
    d = _dev(img)
    txt = gpu_ctx.write_ppm(d.data_ptr(), w, h)
    assert txt == oracle.write_ppm(img)
    if fill == 1.0:
        lib = rtm.load_library()
        assert len(txt) <= lib.rtm_ppm_max_bytes(w, h)
        assert len(txt) == len(f"P3\n{w} {h}\n255\n") + w * h * 13 + h


@pytest.mark.gpu
def test_gpu_write_ppm_rendered_reference_frame(gpu_ctx, oracle, rtm, scenes, tmp_path):
    """Frame 0 of the reference scene, rendered AND encoded on the GPU, written
    through writeColorImage == the oracle's render + writeColorImage."""
    import torch
    sc = scenes.closely_orbiting_sphere(0)
    eye, sh = scenes.eye_camera(), scenes.shadow_camera()
    w = h = 512
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda:0")
    gpu_ctx.render_async(sc, eye, sh, w, h, 500, 0, out.data_ptr())
    path = tmp_path / "frame0.ppm"
    rtm.writeColorImage(gpu_ctx, out.data_ptr(), w, h, str(path))
    ref = oracle.render(sc, eye, sh, w, h, 500)["rgba"]
    assert path.read_bytes() == oracle.write_ppm(ref)


@pytest.mark.gpu
def test_gpu_encode_4k_frame(gpu_ctx, oracle, rtm, scenes):
    """BASELINE config 3 frame (3840x2160, huge reflect values included)."""
    import torch
    cfg = scenes.CONFIGS[3]
    sc = cfg["scene"]()
    w, h, k = cfg["width"], cfg["height"], cfg["steps"]
    out = torch.empty((h, w, 4), dtype=torch.float32, device="cuda:0")
    gpu_ctx.render_async(sc, scenes.eye_camera(), scenes.shadow_camera(), w, h, k, cfg["flags"], out.data_ptr())
    rgb = torch.empty(w * h * 3, dtype=torch.uint8, device="cuda:0")
    gpu_ctx.encode_rgb8_async(out.data_ptr(), w * h, rgb.data_ptr())
    gpu_ctx.synchronize()
    img = out.cpu().numpy()
    assert np.array_equal(rgb.cpu().numpy().reshape(h, w, 3), oracle.encode_rgb8(img).astype(np.uint8))


@pytest.mark.gpu
def test_gpu_write_ppm_capacity_error(gpu_ctx, rtm):
    import torch
    lib = rtm.load_library()
    w, h = 16, 4
    d = torch.ones((h, w, 4), dtype=torch.float32, device="cuda:0")
    buf = C.create_string_buffer(10)
    n = C.c_int64()
    rc = lib.rtm_write_ppm(gpu_ctx.handle, C.c_void_p(d.data_ptr()), w, h, buf, 10, C.byref(n))
    assert rc == -1  # RTM_ERR_INVALID, with the needed length reported
    assert n.value == len(f"P3\n{w} {h}\n255\n") + w * h * 13 + h
    assert b"capacity" in lib.rtm_last_error()
