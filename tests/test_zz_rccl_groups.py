"""The tests that form RCCL communicators (marker `rccl`: ncclCommInitAll over the box's
one device, the ncclCommInitRank form, RCCL's self-gather of a staged root band), run in a
child pytest process of their own, last.

Why a process of their own: on this pool a process that had formed and destroyed one-device
RCCL communicators later met an illegal memory access in unrelated kernels -- the round-5
tree's own suite too, on the same box (gpurun_out/r06_control) -- while two full suites
without those tests ran clean (r06_norccl) and the loopback group tests ran clean four
times alone (r06_rep).  The child runs every one of them bit-exact against the oracle as
before; a fault the communicators leave behind ends with the child."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_rccl_group_tests_in_their_own_process():
    env = dict(os.environ, RTM_RCCL_CHILD="1")
    files = [os.path.join(ROOT, "tests", f) for f in ("test_formats_group.py", "test_group_loopback.py")]
    r = subprocess.run([sys.executable, "-u", "-m", "pytest", "-q", "-p", "no:cacheprovider", "-m", "gpu and rccl",
                        "--timeout", "200", "--timeout-method", "thread"] + files,
                       capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    tail = (r.stdout + r.stderr)[-4000:]
    assert r.returncode == 0, tail
    assert " passed" in r.stdout and " failed" not in r.stdout and "skipped" not in r.stdout, tail
