"""Host-side sanitizer run of the extension's launch-planning code: the native
check (tests/native/host_check.cpp) is built with ASan + UBSan on the host side
(ops/build.build_host_check; no GPU needed) and must finish clean. UBSan is set to halt on
the first error, so undefined behaviour fails the test instead of only printing."""

import os
import shutil
import subprocess

import pytest

from distributed_learning_simulator_amd.ops import build


@pytest.mark.skipif(shutil.which(build.HIPCC) is None and not os.path.exists(build.HIPCC), reason="no hipcc")
def test_host_code_under_asan_ubsan():
    exe = build.build_host_check()
    env = dict(os.environ, UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1",
               ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr
    assert "0 failures" in r.stdout
