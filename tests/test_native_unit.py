"""Runs the native C++ unit tests (csrc/tests/native_tests.cc): Quantity,
JSON, GPU-ledger aggregates vs brute force, pod heap, queue backoff/flush
under a fake clock, timers, CycleState memo invalidation, store watch."""
import subprocess

from flex_gpu_scheduler_amd import build_ext


def test_native_unit_tests_pass():
    exe = build_ext.build_tests(verbose=False)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failed" in r.stdout
