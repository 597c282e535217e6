"""Diagnostic (not product): the step kernel at the bench's back-to-back cadence, for a kernel trace.

One BASELINE config at 65,536 envs: windows of K steps on the engine's own AQL queue (rmx_step_seq: K dispatch packets,
one doorbell, each packet behind the previous one), after a 1-s spin-up.  Run under
    rocprofv3 --kernel-trace --stats -- python3 scripts/trace_window.py --config 2 --k 500 --windows 20
the tracer sees K dependent dispatches submitted together, so each starts as the previous ends (not on an idle GPU, as
eager launches under the tracer do: profiles/r05_ab_log.md trace).  Prints one JSON line: the wall-clock time per step
of the same windows (host clock around each blocking rmx_step_seq, median), to set beside the trace's per-dispatch
durations (scripts/summarize_trace.py).
"""
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
    ap.add_argument("--k", type=int, default=500)
    ap.add_argument("--windows", type=int, default=20)
    ap.add_argument("--n-envs", type=int, default=65536)
    ap.add_argument("--spin-s", type=float, default=1.0)
    args = ap.parse_args()
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    tab = T.compile_scenario(T.baseline_scenario(args.config))
    env = VecRMEnv(tab, args.n_envs, with_renv=False, with_env_done=True)
    assert env.step_variant == "fast"
    acts = env.fill_actions(0, 0, args.k)
    run = env.seq_window(acts)
    torch.cuda.synchronize()
    t_end = time.perf_counter() + args.spin_s
    spins = 0
    while time.perf_counter() < t_end:
        run()
        spins += 1
    walls = []
    for _ in range(args.windows):
        t0 = time.perf_counter()
        run()  # blocking: returns once the K steps are complete
        walls.append((time.perf_counter() - t0) / args.k * 1e6)
    env.check_errors()
    q = env.queue_info()
    print(json.dumps({"config": args.config, "n_envs": args.n_envs, "k": args.k, "windows": args.windows,
                      "spin_windows": spins, "us_per_step_wall_median": statistics.median(walls),
                      "us_per_step_wall_min": min(walls), "dispatch": q["dispatch"], "queue_state": q["state"],
                      "kernel": "rmx::step_fast_kernel"}), flush=True)


if __name__ == "__main__":
    main()
