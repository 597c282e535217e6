"""SURVEY §5 race detection / sanitizers: the CPU oracle and the engine's host-side table builders
(csrc/rmx_tables.cpp, the same source librmx.so links) built with -fsanitize=address,undefined
(oracle/Makefile `asan`) and driven over every BASELINE config, every golden scenario, the randomised worlds
and corrupted configs (tests/asan_driver.py).  Clean means: exit 0, no sanitizer report."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _runtime(name):
    p = subprocess.run(["gcc", f"-print-file-name={name}"], capture_output=True, text=True).stdout.strip()
    return p if os.path.isabs(p) and os.path.exists(p) else None


def _drive(*args):
    asan = _runtime("libasan.so")
    if asan is None:
        pytest.skip("gcc has no AddressSanitizer runtime")
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "asan"], check=True)
    env = dict(os.environ, LD_PRELOAD=asan, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1",
               UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1",
               RMX_ORACLE_LIB=os.path.join(ROOT, "oracle", "_asan", "liboracle.so"), OMP_NUM_THREADS="2")
    return subprocess.run([sys.executable, os.path.join(ROOT, "tests", "asan_driver.py"), *args], capture_output=True,
                          text=True, env=env, timeout=900)


def test_sanitizer_is_live():
    """Negative control: an out-of-bounds table read in the host builders is caught and aborts."""
    r = _drive("--control")
    assert r.returncode != 0 and "CONTROL_NOT_CAUGHT" not in r.stdout
    assert "heap-buffer-overflow" in r.stderr, r.stderr[-3000:]


def test_oracle_and_table_builders_clean_under_asan_ubsan():
    r = _drive()
    report = r.stdout[-3000:] + r.stderr[-6000:]
    assert r.returncode == 0, report
    assert "ASAN_DRIVER_OK" in r.stdout, report
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, report
