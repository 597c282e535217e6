"""Where a K-step queue window's time goes, on one clock: the HSA system timestamp read on the host around the call
and the command processor's stamps of the window's first and last packets (rmx_queue_timing with a stride >= K).

    python scripts/window_timeline.py --config 2 --k 20 --windows 200

Per window (medians over the windows, µs): call -> packet 0 starts; packet 0 start -> last packet start (K - 1
dispatches); the last packet (the fused report); its completion -> the call returns; torch.cuda.synchronize after
it; and the call's wall time."""
import argparse
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--windows", type=int, default=200)
    ap.add_argument("--n-envs", type=int, default=65536)
    a = ap.parse_args()
    import numpy as np
    import torch
    from rmx import _capi, engine as E, tables as T

    _capi.load_library()
    hsa = C.CDLL("libhsa-runtime64.so.1")  # the runtime librmx.so is bound to (one per process)
    assert hsa.hsa_init() == 0  # reference-counted: the HIP runtime's own init is unaffected
    freq = C.c_uint64()
    hsa.hsa_system_get_info(3, C.byref(freq))  # HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY
    tick = C.c_uint64()

    def now_ns():
        hsa.hsa_system_get_info(2, C.byref(tick))  # HSA_SYSTEM_INFO_TIMESTAMP
        return tick.value * 1e9 / freq.value

    tab = T.compile_scenario(T.baseline_scenario(a.config))
    env = E.VecRMEnv(tab, a.n_envs, with_renv=False)
    K = a.k
    acts = env.fill_actions(3, 0, K)
    rep = torch.zeros(4, dtype=torch.float64, device="cuda")
    seq = env.seq_window(acts, out=rep)
    for _ in range(max(200, 20000 // K)):  # spin-up
        seq()
    torch.cuda.synchronize()
    env.queue_timing(K)  # stamps: packet 0 and the last
    rows = []
    for _ in range(a.windows):
        h0 = now_ns()
        seq()
        h1 = now_ns()
        torch.cuda.synchronize()
        h2 = now_ns()
        ts = env.queue_times().astype(np.float64)
        assert ts[0, 0] == 0 and ts[-1, 0] == K - 1
        rows.append({"call_to_first_start": ts[0, 1] - h0, "dispatches": ts[-1, 1] - ts[0, 1],
                     "last_packet": ts[-1, 2] - ts[-1, 1], "completion_to_return": h1 - ts[-1, 2],
                     "synchronize": h2 - h1, "wall": h2 - h0})
    env.queue_timing(0)
    med = {k: statistics.median(r[k] for r in rows) / 1e3 for k in rows[0]}
    med["per_dispatch"] = med["dispatches"] / (K - 1)
    print(json.dumps({"config": a.config, "k": K, "windows": a.windows, "median_us": med}))


if __name__ == "__main__":
    main()
