"""Sanitizer job (CPU only - GPU ASan / XNACK runs are not available on the
MI355X pool).

* tests/sanitize/_build/san_driver: the C driver (lbfgs_driver.c) and the C++ drop-in shim
  (lbfgs_cxx.cpp) built with -fsanitize=address,undefined -fno-sanitize-recover=all over a host
  test double of the device layer (tests/sanitize/host_device_double.c, canonical-order
  reductions from the oracle; never part of the product library). Every line search, objective,
  the batched / one-pass-per-step / unfused modes, host callbacks in both call orders, the
  stepping and primitive APIs and the error paths; every trajectory bit-exact with the oracle's
  ORC_CANON run, and no sanitizer report (any report aborts).
* the oracle's own golden tests against an ASan + UBSan build of oracle/lbfgs_oracle.c, loaded
  into a Python whose allocator is the ASan runtime (LD_PRELOAD).
"""
import os
import shutil
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "sanitize")


def _gcc_lib(name):
    try:
        p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True, timeout=30).stdout.strip()
    except (OSError, subprocess.SubprocessError):
        return None
    return p if p and os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def built():
    if shutil.which("gcc") is None or shutil.which("make") is None or _gcc_lib("libasan.so") is None:
        pytest.skip("no gcc / make / ASan runtime here")
    p = subprocess.run(["make", "-C", SAN, "-j4"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-2000:] + p.stderr[-2000:]
    return SAN


def test_driver_and_shim_under_asan_ubsan(built):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    p = subprocess.run([os.path.join(built, "_build", "san_driver")], capture_output=True, text=True, timeout=600,
                       env=env)
    tail = p.stdout[-1500:] + p.stderr[-3000:]
    assert p.returncode == 0, tail
    assert "sanitizer job: all checks passed" in p.stdout, tail
    assert "ERROR: AddressSanitizer" not in p.stderr and "runtime error" not in p.stderr, tail


def test_oracle_golden_under_asan_ubsan(built):
    env = dict(os.environ, LD_PRELOAD=_gcc_lib("libasan.so"), ASAN_OPTIONS="detect_leaks=0",
               ORACLE_LIB=os.path.join(built, "_build", "liboracle_san.so"))
    p = subprocess.run([sys.executable, "-m", "pytest", os.path.join(HERE, "test_oracle_golden.py"), "-q",
                        "-p", "no:cacheprovider"], capture_output=True, text=True, timeout=600, env=env)
    tail = p.stdout[-1500:] + p.stderr[-3000:]
    assert p.returncode == 0, tail
    assert "runtime error" not in p.stdout + p.stderr, tail
