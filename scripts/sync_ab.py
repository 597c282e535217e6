"""Same-process timing of the synchronous host-boundary call (rmx_step_sync, N = 1, BASELINE config 1) for the
library named by RMX_LIB (default: the in-tree build): the raw ctypes call in a loop, and with a diagnostic build
(make -C multiagent-rl-rm_amd/csrc diag) the device-side span of each request (request seen -> outputs complete)
from rmx_diag_sync_span.  One JSON line.  Run one process per library for a same-box A/B:
    for l in a.so b.so; do RMX_LIB=$l python scripts/sync_ab.py; done
"""
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))

from rmx import compat as CP  # noqa: E402
from rmx import tables as T  # noqa: E402


def main():
    env, agents = CP.scenario_objects(T.baseline_scenario(1))
    w = CP.RMEnvironmentWrapper(env, agents)
    w.reset(0)
    lib = w._engine.lib
    span = getattr(lib, "rmx_diag_sync_span", None)
    if span is not None:
        span.restype, span.argtypes = C.c_int, [C.c_void_p, C.POINTER(C.c_ulonglong)]
    buf = (C.c_ulonglong * 4)()
    fn, h, a, b = w._step_fn, w._h, w._act_p, w._bufs_p
    M = 20000
    best = 1e9
    spans = []
    for rep in range(3):
        t0 = time.perf_counter()
        for _ in range(M):
            fn(h, a, 1, b, None)
        best = min(best, (time.perf_counter() - t0) / M * 1e6)
    if span is not None:
        for _ in range(2000):
            fn(h, a, 1, b, None)
            span(h, buf)
            spans.append(((buf[1] - buf[0]) / (buf[2] / 1e3), buf[3] / 1e3))
    sv = lib.rmx_step_variant
    t0 = time.perf_counter()
    for _ in range(M):
        sv(h)
    ctypes_us = (time.perf_counter() - t0) / M * 1e6  # a trivial C-ABI call from the same ctypes binding
    out = {"lib": os.path.basename(os.environ.get("RMX_LIB", "librmx.so")), "us_per_sync_call": best,
           "us_trivial_ctypes_call": ctypes_us}
    if spans:
        dev = sorted(x[0] for x in spans)
        host = sorted(x[1] for x in spans)
        out["device_span_us_median"] = dev[len(dev) // 2]
        out["host_post_to_ack_us_median"] = host[len(host) // 2]
        out["host_post_to_ack_us_p10"] = host[len(host) // 10]
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
