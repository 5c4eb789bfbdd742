"""Shared test setup.  `gpu`-marked tests need an MI355X and the built
librtm.so; everything else runs on CPU.  The oracle (oracle/) is loaded only
here, as the checker."""
import importlib
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
ORACLE_DIR = os.path.join(ROOT, "oracle")
if ORACLE_DIR not in sys.path:
    sys.path.insert(0, ORACLE_DIR)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) and librtm.so")
    config.addinivalue_line("markers", "rccl: forms an RCCL communicator (runs in its own process, "
                                       "tests/test_zz_rccl_groups.py)")


# Tests that form RCCL communicators run in a child process of their own
# (tests/test_zz_rccl_groups.py, last): on this pool a process that had formed and destroyed
# one-device RCCL communicators later met an illegal memory access in unrelated kernels --
# the round-5 tree's own suite as well (gpurun_out/r06_control), none in two suites without
# those tests (r06_norccl).  In the parent process they are skipped with that reason.
RCCL_CHILD = os.environ.get("RTM_RCCL_CHILD") == "1"


def pytest_collection_modifyitems(config, items):
    if RCCL_CHILD:
        return
    skip = pytest.mark.skip(reason="forms an RCCL communicator: run in its own process by test_zz_rccl_groups.py")
    for item in items:
        if item.get_closest_marker("rccl"):
            item.add_marker(skip)


@pytest.fixture(scope="session")
def rtm():
    return importlib.import_module("2018rustraytracer_amd")


@pytest.fixture(scope="session")
def scenes():
    return importlib.import_module("2018rustraytracer_amd.scenes")


@pytest.fixture(scope="session")
def oracle():
    import oracle as O  # noqa: E402  (test infrastructure only)
    O.lib()
    return O


@pytest.fixture(scope="session")
def gpu_ctx(rtm):
    if rtm.device_count() < 1:
        pytest.fail("gpu test without a visible GPU")
    ctx = rtm.Context(0)
    yield ctx
    ctx.close()


def bits_equal(a, b):
    """Bit-exact equality of float arrays (NaN-safe, distinguishes -0.0)."""
    a = np.ascontiguousarray(a)
    b = np.ascontiguousarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    v = {4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    return bool(np.array_equal(a.view(v), b.view(v)))


def first_mismatch(a, b):
    v = {4: np.uint32, 8: np.uint64}[a.dtype.itemsize]
    idx = np.argwhere(a.view(v) != b.view(v))
    if len(idx) == 0:
        return None
    i = tuple(idx[0])
    return f"{len(idx)} mismatches, first at {i}: got {a[i]!r} want {b[i]!r}"


def device_smap(ctx, w, h):
    """The context's last shadow map as f64 values (rtm_ctx_shadow_map: decoded from the
    coded map on the device), copied to the host."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    m = np.empty((h, w), np.float64)
    p = ctx.shadow_map_ptr()
    assert p, "no shadow map"
    assert hip.hipMemcpy(m.ctypes.data, p, w * h * 8, 2) == 0
    return m
