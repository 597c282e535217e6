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


def host_run_reference(tab, n, steps, seed):
    """rmxh_host_run's sequence (oracle/asan/rmxh_entry.cpp) through librmx.so's host handle (HostRMEnv): the
    statistics and the FNV digest of the final pos_x, pos_y, rm_q, flags, t columns."""
    import numpy as np

    from rmx.engine import HostRMEnv
    env = HostRMEnv(tab, n)
    env.reset(seed=seed)
    A = tab.n_agents
    for s in range(steps):
        if s % 97 == 5:
            act = ((s + np.arange(A * n)) % 4).astype(np.int32)
            act[A * n // 2] = 9
            env.step(act.reshape(A, n))
        else:
            env.step_hashed(seed, s)
    A_N = A * n  # the driver's garbage columns (oracle/asan/rmxh_entry.cpp), then 5 steps, a reset and 5 more
    k = np.arange(A_N, dtype=np.uint64)
    env.pos_x[...] = (((k * 2654435761) & 0xFFFFFFFF).astype(np.uint32).view(np.int32) ^ 0x7ffff).reshape(A, n)
    env.pos_y[...] = (-(k.astype(np.int64)) - 300).astype(np.int32).reshape(A, n)
    env.rm_q[...] = ((k * 40503) & 0xFFFFFFFF).astype(np.uint32).view(np.int32).reshape(A, n)
    env.flags[...] = ((k * 2246822519) & 0xFFFFFFFF).astype(np.uint32).reshape(A, n)
    e = np.arange(n, dtype=np.uint64)
    env.t[...] = (((e * 7919) & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64) - 100000).astype(np.int32)
    env.t[0] = 0x7fffffff
    for it in range(5):
        env.step_hashed(seed, 777 + it)
    env.reset(seed=seed)
    for it in range(5):
        env.step_hashed(seed, 900 + it)
    bad = 0
    try:
        env.check_errors()
    except ValueError:
        bad = 1
    mask = np.zeros(n, np.uint8)
    mask[::3] = 1
    env.reset(mask=mask, seed=seed + 1)
    for it in range(16):
        env.step_hashed(seed, steps + it)
    d = 0xcbf29ce484222325
    for col in (env.pos_x, env.pos_y, env.rm_q, env.flags, env.t):
        for byte in np.ascontiguousarray(col).tobytes():
            d = ((d ^ byte) * 0x100000001b3) & (2**64 - 1)
    return list(env.stats()) + [float(d >> 12), float(bad)]


def test_oracle_host_path_and_table_builders_clean_under_asan_ubsan():
    """The driver runs clean under the sanitizers, and the sanitizer build of the host path (rmxh_host_run) ends every
    config exactly where librmx.so's host handle does on the same inputs (the same source, another compiler)."""
    import json

    from rmx import tables as T
    from test_random_maps_gpu import CASES, random_tables
    r = _drive()
    report = r.stdout[-3000:] + r.stderr[-6000:]
    assert r.returncode == 0, report
    assert "ASAN_DRIVER_OK" in r.stdout, report
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, report
    n, steps, seed = next(tuple(int(v) for v in ln.split()[1:]) for ln in r.stdout.splitlines()
                          if ln.startswith("HOSTRUN_PARAMS"))
    runs = {ln.split()[1]: json.loads(ln.split(None, 2)[2]) for ln in r.stdout.splitlines()
            if ln.startswith("HOSTRUN ")}
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        descs = json.load(f)
    assert len(runs) >= 4 + len(descs) + len(CASES)
    for name, got in runs.items():
        if name.startswith("baseline"):
            tab = T.compile_scenario(T.baseline_scenario(int(name[len("baseline"):])))
        elif name in descs:
            tab = T.compile_scenario(descs[name])
        else:
            tab = random_tables(*CASES[name])
        want = host_run_reference(tab, n, steps, seed)
        assert got[1:] == want[1:], (name, got, want)
        assert abs(got[0] - want[0]) <= 1e-9 * max(1.0, abs(want[0])), (name, got, want)
