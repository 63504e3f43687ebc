"""Sanitizer builds of the host code (race detection / sanitizers; CPU only -- GPU
sanitizers are not available on the MI355X pool):
  * oracle/kkt_ref.c (the C restatement behind the CPU baseline) under AddressSanitizer +
    UndefinedBehaviorSanitizer, every supported shape and the edge cases (N = 1, empty batch,
    indefinite Quu, invalid dimensions), `make -C oracle sanitize`;
  * the C-ABI's host-side argument validation (csrc/noc_abi.hip's host code instrumented with
    -Xarch_host -fsanitize=address,undefined, device code untouched) driven by
    tests/abi_sanitize.cpp, `make -C ip-parallel-optimal-control_amd abi-sanitize`.
Any out-of-bounds access or undefined behaviour aborts the driver (-fno-sanitize-recover)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "ip-parallel-optimal-control_amd")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1", OMP_NUM_THREADS="2")


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_kkt_ref_under_asan_ubsan():
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle"), "sanitize"], check=True,
                   capture_output=True)
    p = subprocess.run([os.path.join(ROOT, "oracle", "_build", "kkt_ref_sanitize")], env=ENV,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, p.stdout + p.stderr[-3000:]


@pytest.mark.skipif(not os.path.exists("/opt/rocm/bin/hipcc"), reason="hipcc not available")
def test_abi_argument_validation_under_asan_ubsan():
    subprocess.run(["make", "-C", PKG, "-j", "8", "abi-sanitize"], check=True, capture_output=True,
                   timeout=1500)
    p = subprocess.run([os.path.join(PKG, "build", "abi_sanitize")], env=ENV, capture_output=True,
                       text=True, timeout=300)
    assert p.returncode == 0 and "ok" in p.stdout, p.stdout + p.stderr[-3000:]
