"""The adapter layer's host C under sanitizers: tests/sanitize/Makefile builds the picoquic
stand-in (tests/host/mini_host.c) with the product's protoops.c, fec_core.c, batch.c, frames.c and cc.c,
the oracle and a CPU stand-in for the engine's entry points (tests/sanitize/fecgpu_cpu_stub.c, never in
the product), once with AddressSanitizer + UndefinedBehaviorSanitizer and once with ThreadSanitizer.
The protoop, batching, frame and CC suites then run against each build in a child process with the
sanitizer runtime preloaded (PQUIC_TEST_MINIHOST points the suites at it): every reference fixture
through the synchronous adapters and through the batcher -- stagers, engine threads, the arena registry
with 1100 connections registered and unregistered, ordered completions -- must pass with no sanitizer
report.  CPU only: the stand-in computes through the oracle."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
SAN = os.path.join(ROOT, "tests", "sanitize")
SUITES = ["tests/test_protoops_gpu.py", "tests/test_batch_gpu.py", "tests/test_frames.py",
          "tests/test_frames_differential.py", "tests/test_cc.py", "tests/test_cc_differential.py"]
REPORTS = ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer", "ERROR: LeakSanitizer")


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


@pytest.fixture(scope="module")
def built():
    if shutil.which("gcc") is None:
        pytest.skip("gcc not present")
    r = subprocess.run(["make", "-s", "-C", SAN, "all"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    return os.path.join(SAN, "_build")


def _sanitizer_logs(tmp_path):
    """the reports the sanitizer runtimes wrote to their log_path files (one per process)"""
    return "".join(p.read_text(errors="replace") for p in sorted(tmp_path.glob("san.*")))


def _run_suites(lib, preload, extra_env, tmp_path, deselect=()):
    env = dict(os.environ)
    env.update(extra_env)
    # reports also go to files: a runtime that ends the process can lose what it wrote to a pipe
    for var in ("ASAN_OPTIONS", "UBSAN_OPTIONS", "TSAN_OPTIONS"):
        if var in env:
            env[var] += f":log_path={tmp_path / 'san'}"
    env["LD_PRELOAD"] = preload
    env["PQUIC_TEST_MINIHOST"] = lib
    env["PYTHONMALLOC"] = "malloc"
    cmd = [sys.executable, "-m", "pytest", "-x", "-q", "-p", "no:cacheprovider", "-m", "gpu or not gpu",
           "--deselect", "tests/test_frames.py::test_device_repair_frames"]
    for d in deselect:
        cmd += ["--deselect", d]
    r = subprocess.run(cmd + SUITES, cwd=ROOT, env=env, capture_output=True, text=True, timeout=1800)
    out = r.stdout + r.stderr + _sanitizer_logs(tmp_path)
    (tmp_path / "log.txt").write_text(out)
    assert r.returncode == 0, out[-6000:]
    found = [m for m in REPORTS if m in out]
    assert not found, out[-6000:]
    return out


def _canary(lib, preload, extra_env, kind, report):
    """the build's sanitizer is live: a deliberate defect (san_canary) is reported"""
    env = dict(os.environ)
    env.update(extra_env)
    env["LD_PRELOAD"] = preload
    code = f"import ctypes; ctypes.CDLL({lib!r}).san_canary({kind})"
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert any(m in r.stderr for m in report), r.stderr[-3000:]


def test_host_c_under_asan_ubsan(built, tmp_path):
    rt = _runtime("libasan.so")
    if not rt:
        pytest.skip("libasan not present")
    env = {"ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:abort_on_error=1",
           "UBSAN_OPTIONS": "halt_on_error=1:print_stacktrace=1"}
    lib = os.path.join(built, "asan", "libminihost.so")
    # the read past the block: UBSan's object-size check or ASan's redzone, whichever fires first
    _canary(lib, rt, env, 1, ("ERROR: AddressSanitizer: heap-buffer-overflow", "runtime error: load of address"))
    out = _run_suites(lib, rt, env, tmp_path)
    assert " passed" in out


def test_batcher_under_tsan(built, tmp_path):
    rt = _runtime("libtsan.so")
    if not rt:
        pytest.skip("libtsan not present")
    env = {"TSAN_OPTIONS": "halt_on_error=1:second_deadlock_stack=1"}
    lib = os.path.join(built, "tsan", "libminihost.so")
    _canary(lib, rt, env, 2, ("WARNING: ThreadSanitizer: data race",))
    out = _run_suites(lib, rt, env, tmp_path)
    assert " passed" in out
