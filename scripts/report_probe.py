"""The statistics report inside a K-step window: separate launch (rmx_step + rmx_stats_device) vs fused into the
K-th step (rmx_step_report).  Per chain, one captured graph replayed --reps times; event time of the graph
(us) and bench.py's wall window (graph + device sync, us).  Config 2, 65,536 envs unless given."""
import argparse
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n-envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--reps", type=int, default=41)
    args = ap.parse_args()
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    tab = T.compile_scenario(T.baseline_scenario(args.config))
    env = VecRMEnv(tab, args.n_envs, with_renv=False)
    K = args.steps
    acts = env.fill_actions(0, 0, K)
    out = torch.zeros(4, dtype=torch.float64, device="cuda")

    chains = {
        "steps": lambda: [env.step(acts[s]) for s in range(K)],
        "steps+stats": lambda: ([env.step(acts[s]) for s in range(K)], env.stats_tensor()),
        "steps+fused": lambda: ([env.step(acts[s]) for s in range(K - 1)], env.step_report(acts[K - 1], out=out)),
        "reports": lambda: [env.step_report(acts[s], out=out) for s in range(K)],
        "stats_only": lambda: [env.stats_tensor() for _ in range(K)],
    }
    res = {"config": args.config, "n_envs": args.n_envs, "K": K, "fused": env.report_fused}
    graphs = {}
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        for name, fn in chains.items():
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s0):
                fn()
            graphs[name] = g
    torch.cuda.current_stream().wait_stream(s0)
    for g in graphs.values():
        g.replay()
    torch.cuda.synchronize()
    t_end = time.perf_counter() + 0.3  # clocks up
    while time.perf_counter() < t_end:
        graphs["steps"].replay()
        torch.cuda.synchronize()
    for rnd in range(2):
        for name, g in graphs.items():
            ev, wall = [], []
            for r in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                g.replay()
                e1.record()
                torch.cuda.synchronize()
                ev.append(e0.elapsed_time(e1) * 1e3)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                g.replay()
                torch.cuda.synchronize()
                wall.append((time.perf_counter() - t0) * 1e6)
            res[f"{name}#{rnd}"] = {"ev_us": round(statistics.median(ev), 2), "wall_us": round(statistics.median(wall), 2)}
    # eager launches from a raw ctypes loop (no graph): host launch cost vs the graph's launch latency
    from rmx.engine import _ptr
    lib, h, st = env.lib, env._h, env._stream()
    ptrs = [_ptr(acts[s]) for s in range(K)]
    for rnd in range(2):
        ev, wall = [], []
        for r in range(args.reps):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for s in range(K):
                lib.rmx_step(h, ptrs[s], 1, st)
            e1.record()
            torch.cuda.synchronize()
            ev.append(e0.elapsed_time(e1) * 1e3)
            t0 = time.perf_counter()
            for s in range(K):
                lib.rmx_step(h, ptrs[s], 1, st)
            torch.cuda.synchronize()
            wall.append((time.perf_counter() - t0) * 1e6)
        res[f"eager_ctypes#{rnd}"] = {"ev_us": round(statistics.median(ev), 2), "wall_us": round(statistics.median(wall), 2)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
