"""CPU tests of the C-ABI boundary: librtm.so loads, exports every function
include/rtm.h declares, struct layouts match, and argument validation fails
cleanly.  No kernel is launched here (no GPU in this container)."""
import ctypes as C
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rtm.h")


def declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(rtm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_expected_surface():
    names = declared_functions()
    for n in ("rtm_render", "rtm_render_async", "rtm_viewport_rasterize",
              "rtm_viewport_process_raymarching_rays", "rtm_render_color_image", "rtm_last_error"):
        assert n in names


def test_library_exports_every_declared_symbol(rtm):
    lib = rtm.load_library()
    for n in declared_functions():
        assert hasattr(lib, n), f"librtm.so does not export {n}"
    py = {name for name, _, _ in rtm.abi.ABI_SYMBOLS}
    assert py == set(declared_functions()), "abi.py symbol table out of sync with rtm.h"


def test_library_is_gfx950_code_object(rtm):
    data = open(rtm.abi.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_struct_sizes(rtm):
    abi = rtm.abi
    assert C.sizeof(abi.rtm_sphere) == 64
    assert C.sizeof(abi.rtm_camera) == 104
    assert C.sizeof(abi.rtm_patch) == 32
    assert C.sizeof(abi.rtm_circle_plane) == 88
    assert C.sizeof(abi.rtm_capped_cylinder) == 96
    assert C.sizeof(abi.rtm_sdf) == 136
    assert C.sizeof(abi.rtm_scene) == 64


def test_struct_layout_matches_header(rtm, tmp_path):
    """Every ctypes struct's size and field offsets == the C compiler's view of include/rtm.h."""
    import subprocess
    abi = rtm.abi
    structs = [abi.rtm_sphere, abi.rtm_patch, abi.rtm_camera, abi.rtm_circle_plane, abi.rtm_capped_cylinder,
               abi.rtm_sdf, abi.rtm_scene, abi.rtm_stats]
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "rtm.h"', "int main(void) {"]
    for st in structs:
        n = st.__name__
        lines.append(f'printf("{n} %zu\\n", sizeof({n}));')
        for f, _ in st._fields_:
            lines.append(f'printf("{n}.{f} %zu\\n", offsetof({n}, {f}));')
    lines.append("return 0; }")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(l.split() for l in subprocess.run([str(exe)], check=True, capture_output=True,
                                                   text=True).stdout.splitlines())
    for st in structs:
        n = st.__name__
        assert int(got[n]) == C.sizeof(st), n
        for f, _ in st._fields_:
            assert int(got[f"{n}.{f}"]) == getattr(st, f).offset, (n, f)


def test_abi_version_and_device_count(rtm):
    lib = rtm.load_library()
    assert lib.rtm_abi_version() == rtm.abi.RTM_ABI_VERSION
    assert lib.rtm_device_count() >= 0


def test_argument_validation_without_gpu(rtm, scenes):
    """Invalid arguments are rejected before any device work."""
    lib = rtm.load_library()
    abi = rtm.abi
    sc, keep = scenes.scene_a_bench().to_c()
    e, s = scenes.eye_camera().to_c(), scenes.shadow_camera().to_c()
    out = (C.c_float * 16)()
    assert lib.rtm_render(None, C.byref(e), C.byref(s), 2, 2, 1, 0, out) == abi.RTM_ERR_INVALID
    assert lib.rtm_render_multi(C.byref(sc), C.byref(e), C.byref(s), 2, 2, 1, 0, None, 1) == abi.RTM_ERR_INVALID
    assert lib.rtm_render(C.byref(sc), C.byref(e), C.byref(s), 0, 2, 1, 0, out) == abi.RTM_ERR_INVALID
    assert lib.rtm_render(C.byref(sc), C.byref(e), C.byref(s), 2, 2, -1, 0, out) == abi.RTM_ERR_INVALID
    assert lib.rtm_render(C.byref(sc), C.byref(e), C.byref(s), 2, 2, 1, 0x80, out) == abi.RTM_ERR_INVALID
    assert b"flags" in lib.rtm_last_error()
    p = scenes.Camera(scenes.PERSPECTIVE, (0, 0, 0), (0, 0, 1), (0, 1, 0), (1, 0, 0)).to_c()
    # a perspective shadow camera: Camera::project asserts ORTHOGONAL (main.rs:1949)
    assert lib.rtm_render(C.byref(sc), C.byref(e), C.byref(p), 2, 2, 1, 0, out) == abi.RTM_ERR_UNSUPPORTED
    h = C.c_void_p()
    rc = lib.rtm_ctx_create(0, C.byref(h))
    if lib.rtm_device_count() == 0:
        assert rc == abi.RTM_ERR_NO_DEVICE
        assert lib.rtm_render(C.byref(sc), C.byref(e), C.byref(s), 2, 2, 1, 0, out) == abi.RTM_ERR_NO_DEVICE
        assert lib.rtm_render_multi(C.byref(sc), C.byref(e), C.byref(s), 2, 2, 1, 0, out, 1) == abi.RTM_ERR_NO_DEVICE
    else:
        assert rc == 0
        lib.rtm_ctx_destroy(h)


def test_product_package_does_not_import_oracle():
    """The product path must never route through the oracle: no import, no
    link, no symbol reference from the package or librtm.so."""
    pkg = os.path.join(ROOT, "2018rustraytracer_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                txt = open(os.path.join(dirpath, f)).read()
                for bad in ("import oracle", "from oracle", "librtm_oracle", "rtmo_"):
                    assert bad not in txt, (f, bad)
    so = open(os.path.join(pkg, "librtm.so"), "rb").read()
    assert b"rtmo_" not in so and b"librtm_oracle" not in so


def test_package_ships_only_the_product_library():
    """The product package holds one shared library, librtm.so:
    A/B variants and the bounds demos' revert builds go to build/ (tools/ab_lib.sh,
    tools/bounds_demo.sh), and the product source defines no A/B switch."""
    pkg = os.path.join(ROOT, "2018rustraytracer_amd")
    libs = sorted(f for f in os.listdir(pkg) if f.endswith(".so"))
    assert libs == ["librtm.so"], libs
    csrc = os.path.join(pkg, "csrc")
    for f in os.listdir(csrc):
        if f.endswith((".hip", ".cpp", ".h")):
            assert "RTM_AB_" not in open(os.path.join(csrc, f)).read(), f
    for tool in ("ab_lib.sh", "bounds_demo.sh"):
        assert "build/" in open(os.path.join(ROOT, "tools", tool)).read(), tool
