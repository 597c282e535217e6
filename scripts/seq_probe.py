"""Diagnostic (not product): host time of a K-step window at BASELINE config 2, 65,536 envs, by how its launches are
issued — a HIP graph replay + device sync (the round-3 bench), rmx_step_seq through VecRMEnv.step_seq (+ sync), and
the bare C call — median of --reps windows after a 1-s spin-up, K in --ks.  Prints one JSON line per K.
    python scripts/seq_probe.py --ks 1,20,100
"""
import argparse
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ks", default="1,20,100")
    ap.add_argument("--reps", type=int, default=300)
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n-envs", type=int, default=65536)
    args = ap.parse_args()
    import torch
    from rmx import tables as T
    from rmx.engine import VecRMEnv

    tab = T.compile_scenario(T.baseline_scenario(args.config))
    env = VecRMEnv(tab, args.n_envs, with_renv=False, with_env_done=True)
    report = torch.zeros(4, dtype=torch.float64, device="cuda")
    stream = torch.cuda.current_stream()
    clk = time.perf_counter
    for K in [int(k) for k in args.ks.split(",")]:
        acts = env.fill_actions(0, 0, K)
        g = torch.cuda.CUDAGraph()
        s0 = torch.cuda.Stream()
        s0.wait_stream(stream)
        with torch.cuda.stream(s0):
            with torch.cuda.graph(g, stream=s0):
                for s in range(K - 1):
                    env.step(acts[s])
                env.step_report(acts[K - 1], out=report)
        stream.wait_stream(s0)
        torch.cuda.synchronize()
        lib, h, sp = env.lib, env._h, env._stream()
        aptr, optr = C.c_void_p(acts.data_ptr()), C.c_void_p(report.data_ptr())
        stride = env.A * env.N

        def graph():
            g.replay()
            torch.cuda.synchronize()

        def seq():
            env.step_seq(acts, out=report)
            torch.cuda.synchronize()

        def seq_bare():
            lib.rmx_step_seq(h, aptr, stride, K, 1, optr, sp)

        def seq_same_slice():  # every step reads actions[0] (the floors' chain form)
            lib.rmx_step_seq(h, aptr, 0, K, 1, optr, sp)

        def seq_noreport():
            lib.rmx_step_seq(h, aptr, stride, K, 1, None, sp)

        W = 5
        wacts = env.fill_actions(0, 0, W)

        def bench_pre():  # what bench.py does between its timed windows: reset, statistics cleared, W eager steps
            env.reset()
            env.clear_stats()
            for s in range(W):
                env.step(wacts[s])
            torch.cuda.synchronize()

        def sync_only():
            torch.cuda.synchronize()

        res = {"K": K}
        for name, fn, pre in (("graph", graph, None), ("seq", seq, None), ("seq_bare", seq_bare, None),
                              ("seq_same_slice", seq_same_slice, None), ("seq_noreport", seq_noreport, None),
                              ("seq_benchlike", seq, bench_pre), ("sync_idle", sync_only, None),
                              ("graph", graph, None), ("seq", seq, None)):
            t_end = clk() + 1.0
            while clk() < t_end:
                fn()
            w = []
            for _ in range(args.reps):
                if pre is not None:
                    pre()
                t0 = clk()
                fn()
                w.append(clk() - t0)
            res[f"{name}_us"] = round(statistics.median(w) * 1e6, 2)
        res["queue"] = env.queue_counters()
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
