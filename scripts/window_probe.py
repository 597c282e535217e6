"""Where does the fixed cost of a short timed window go?  (diagnostic, GPU box)

For BASELINE config 2 at 65,536 envs, times a K-step window several ways and prints one JSON line per case:
host time of graph.replay(), event-timed window, wall window (sync to sync), the stats report alone.
    python scripts/window_probe.py [K ...]
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))

import torch  # noqa: E402

from rmx import tables as T  # noqa: E402
from rmx.engine import VecRMEnv  # noqa: E402


def main():
    Ks = [int(k) for k in sys.argv[1:]] or [20, 100, 1000]
    tab = T.compile_scenario(T.baseline_scenario(int(os.environ.get("CFG", "2"))))
    N, W = 65536, 5
    env = VecRMEnv(tab, N, device=0, with_renv=False, with_env_done=True)
    st = torch.cuda.current_stream()
    for K in Ks:
        acts = env.fill_actions(0, 0, W + K)
        g = torch.cuda.CUDAGraph()
        s0 = torch.cuda.Stream()
        s0.wait_stream(st)
        with torch.cuda.stream(s0):
            with torch.cuda.graph(g, stream=s0):
                for s in range(K):
                    env.step(acts[W + s])
        st.wait_stream(s0)
        torch.cuda.synchronize()
        for rep in range(4):
            env.reset()
            env.clear_stats()
            for s in range(W):
                env.step(acts[s])
            torch.cuda.synchronize()
            e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
            t0 = time.perf_counter()
            e0.record(st)
            g.replay()
            t1 = time.perf_counter()
            e1.record(st)
            env.stats_tensor()
            e2.record(st)
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(json.dumps({"K": K, "rep": rep, "mode": "graph", "host_replay_us": (t1 - t0) * 1e6,
                              "ev_steps_us_per_step": e0.elapsed_time(e1) * 1e3 / K,
                              "ev_stats_us": e1.elapsed_time(e2) * 1e3,
                              "wall_us_per_step": (t2 - t0) * 1e6 / K}), flush=True)
        # eager launches
        for rep in range(3):
            env.reset()
            env.clear_stats()
            for s in range(W):
                env.step(acts[s])
            torch.cuda.synchronize()
            e0, e1 = (torch.cuda.Event(enable_timing=True) for _ in range(2))
            t0 = time.perf_counter()
            e0.record(st)
            for s in range(K):
                env.step(acts[W + s])
            t1 = time.perf_counter()
            e1.record(st)
            env.stats_tensor()
            torch.cuda.synchronize()
            t2 = time.perf_counter()
            print(json.dumps({"K": K, "rep": rep, "mode": "eager", "host_issue_us": (t1 - t0) * 1e6,
                              "ev_steps_us_per_step": e0.elapsed_time(e1) * 1e3 / K,
                              "wall_us_per_step": (t2 - t0) * 1e6 / K}), flush=True)
        # empty sync round trip
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        torch.cuda.synchronize()
        print(json.dumps({"sync_idle_us": (time.perf_counter() - t0) * 1e6}), flush=True)
        del g, acts
    env.check_errors()


if __name__ == "__main__":
    main()
