"""Sanitizer builds of the CPU code ("Race detection / sanitizers"), CPU only.

tests/sanitize/Makefile builds three drivers and every report aborts its run (-fno-sanitize-recover=all):
  * san_oracle       oracle/bls_oracle.c under AddressSanitizer + UndefinedBehaviorSanitizer: every oc_* entry
                     point with its known answers and edge cases (tests/sanitize/san_oracle.c);
  * san_oracle_tsan  the same oracle under ThreadSanitizer, driving its pthread registry paths (registry
                     generation, batch signing, registry-resident FastAggregateVerify in both modes);
  * san_hostcheck    the host build of the device headers the gfx950 kernels compile (tests/hostcheck/*.cpp,
                     the digit form with its column / value checks) under ASan + UBSan, checked against
                     algebraic identities (tests/sanitize/san_hostcheck.cpp).
GPU code is not sanitized: GPU AddressSanitizer / xnack+ runs are not available on the MI355X pool.
"""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
SAN = os.path.join(HERE, "sanitize")
ENV = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1",
           TSAN_OPTIONS="halt_on_error=1")


def _build(target):
    subprocess.check_call(["make", "-j3", "-C", SAN, target], timeout=2400, stdout=subprocess.DEVNULL)
    return os.path.join(SAN, target)


def _run(path, *args):
    p = subprocess.run([path, *args], env=ENV, capture_output=True, text=True, timeout=600)
    report = p.stdout + p.stderr
    assert p.returncode == 0, report[-4000:]
    for marker in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer"):
        assert marker not in report, report[-4000:]
    return report


def test_oracle_asan_ubsan():
    assert "san_oracle ok" in _run(_build("san_oracle"))


def test_oracle_tsan_threads():
    assert "san_oracle ok (threads)" in _run(_build("san_oracle_tsan"), "threads")


@pytest.mark.slow
def test_device_headers_host_asan_ubsan():
    assert "san_hostcheck ok" in _run(_build("san_hostcheck"))
