"""The codec's host code under AddressSanitizer + UndefinedBehaviorSanitizer.

tests/host_check/host_check_asan (built by build() / tests/host_check/Makefile)
links the product's gfx950 kernel objects with the host side of
snappy_device.hip and snappy_host.c instrumented, and checks every result
against the oracle.  Without a GPU it covers the varint helpers and every host
entry point's error path; on the GPU, the buffer and FILE* pipelines (ragged
sizes, a three-chunk input), the sidecar index (and a corrupted one), malformed
streams and pooled host contexts from four threads.  Any sanitizer report
fails the run (halt_on_error, a nonzero exit code).
"""
import os
import subprocess

import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "host_check")
BIN = os.path.join(HERE, "build", "host_check_asan")


def _run(mode, timeout):
    assert os.path.exists(BIN), "host_check_asan is not built (run build() / make -C tests/host_check)"
    env = dict(os.environ,
               ASAN_OPTIONS="halt_on_error=1:abort_on_error=0:exitcode=23:detect_leaks=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1:exitcode=24",
               LSAN_OPTIONS="suppressions=" + os.path.join(HERE, "lsan.supp"))
    r = subprocess.run([BIN, mode], env=env, capture_output=True, text=True, timeout=timeout)
    out = r.stdout + r.stderr
    assert r.returncode == 0, f"host_check_asan {mode}: rc {r.returncode}\n{out[-4000:]}"
    assert f"host_check {mode}: ok" in out, out[-4000:]
    for bad in ("ERROR: AddressSanitizer", "runtime error:", "ERROR: LeakSanitizer"):
        assert bad not in out, out[-4000:]


def test_host_code_sanitized_without_device():
    # (re)made here on every CPU run: a harness that no longer builds fails this
    # test instead of leaving a stale binary to pass it (build() only warns)
    r = subprocess.run(["make", "-C", HERE], capture_output=True, text=True)
    assert r.returncode == 0, "tests/host_check does not build:\n" + (r.stdout + r.stderr)[-4000:]
    env_gpu = os.environ.get("HIP_VISIBLE_DEVICES")
    try:
        os.environ["HIP_VISIBLE_DEVICES"] = "-1"  # no device even on a GPU box
        _run("nodev", 120)
    finally:
        if env_gpu is None:
            os.environ.pop("HIP_VISIBLE_DEVICES", None)
        else:
            os.environ["HIP_VISIBLE_DEVICES"] = env_gpu


@pytest.mark.gpu
def test_host_code_sanitized_on_gpu():
    _run("gpu", 300)
