"""Host sanitizer builds ("host ASan/UBSan build of the oracle and the C ABI"):
tests/native/Makefile builds the oracle under ASan+UBSan and under TSan (the row-parallel
loop of RayTracer.cs:898-901 writes disjoint pixels, :1038), and rt_api.cpp's host code under
host-side ASan+UBSan (scene packing, view set-up and screen boxes, camera input, PPM, wire
layout, argument checks).  CPU only: no device call is reached."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
NATIVE = os.path.join(ROOT, "tests", "native")
BUILD = os.path.join(NATIVE, "build")


@pytest.fixture(scope="module")
def built():
    subprocess.run(["make", "-s", "-j4", "-C", NATIVE], check=True, timeout=600)
    return BUILD


def _run(cmd, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    # a preloaded library (if any) stays: ASan is told not to insist on coming first
    env["ASAN_OPTIONS"] = ":".join(x for x in (env.get("ASAN_OPTIONS", ""), "verify_asan_link_order=0") if x)
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    for marker in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer"):
        assert marker not in out, out[-4000:]
    return out


def test_oracle_asan_ubsan(built):
    out = _run([os.path.join(built, "san_oracle_asan"), "60"], {"UBSAN_OPTIONS": "print_stacktrace=1"})
    assert "0 failures" in out


def test_oracle_tsan_disjoint_rows(built):
    out = _run([os.path.join(built, "san_oracle_tsan"), "20"], {"TSAN_OPTIONS": "halt_on_error=1"})
    assert "0 failures" in out


def test_host_api_asan_ubsan(built):
    out = _run([os.path.join(built, "san_host_asan")], {"UBSAN_OPTIONS": "print_stacktrace=1"})
    assert "san_host: 0 failures" in out
