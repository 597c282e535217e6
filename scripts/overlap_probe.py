"""Probe: do S independent env shards on S HIP streams overlap their step chains on one GPU?

The envs of a batch are independent (a step of env e reads and writes env e's columns only), so a K-step window over
N envs can be S chains over N/S envs each, every chain keeping its own step-to-step dependency.  One chain's
dependent-launch boundary could then overlap another chain's kernel.  This measures it with the existing engine: S
VecRMEnv shards (env_offset = i * N / S, n_envs_global = N, the bench's columns), each with a K-step HIP graph
captured on its own stream (distinct action slices per step), replayed concurrently; µs per step of the whole batch =
elapsed / K.  "main" is the bench's own event-window form (one graph over all N envs replayed on the current
stream).  All variants of a config are built first, spun up together (an idle-clocked GPU runs 30-50 % slower), then
timed interleaved, ROUNDS times; one JSON line per (config, variant) with the median and the spread.

    python scripts/overlap_probe.py --configs 2,3,4 --shards 1,2,4 --steps 500
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
    ap.add_argument("--configs", default="2,3,4")
    ap.add_argument("--shards", default="1,2,4")
    ap.add_argument("--n-envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--spin-ms", type=float, default=500.0)
    a = ap.parse_args()
    import torch
    from rmx import engine as E
    from rmx import tables as T

    assert torch.cuda.is_available()
    N, K = a.n_envs, a.steps
    main_s = torch.cuda.current_stream()
    for cfg in [int(c) for c in a.configs.split(",")]:
        tab = T.compile_scenario(T.baseline_scenario(cfg))
        variants = {}  # name -> (envs, runner)
        keep = []
        for S in [0] + [int(s) for s in a.shards.split(",")]:  # 0: the bench's form
            n = N // max(S, 1)
            envs = [E.VecRMEnv(tab, n, env_offset=i * n, n_envs_global=N, with_renv=False) for i in range(max(S, 1))]
            acts = []
            for env in envs:
                env.reset(seed=7)
                acts.append(env.fill_actions(11, 0, K))
            streams = [torch.cuda.Stream() for _ in envs]
            graphs = []
            for i, env in enumerate(envs):
                g = torch.cuda.CUDAGraph()
                streams[i].wait_stream(main_s)
                with torch.cuda.stream(streams[i]):
                    with torch.cuda.graph(g, stream=streams[i]):
                        for k in range(K):
                            env.step(acts[i][k])
                main_s.wait_stream(streams[i])
                graphs.append(g)
            torch.cuda.synchronize()
            keep.append((envs, acts, graphs))

            def run(S=S, graphs=graphs, streams=streams):
                if S == 0:
                    graphs[0].replay()  # on the current stream, as bench.py's event windows
                    return
                for s in streams:
                    s.wait_stream(main_s)
                for s, g in zip(streams, graphs):
                    with torch.cuda.stream(s):
                        g.replay()
                for s in streams:
                    main_s.wait_stream(s)
            variants["main" if S == 0 else f"S{S}"] = (envs, run)

        def timed(run):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main_s)
            run()
            e1.record(main_s)
            torch.cuda.synchronize()
            return e0.elapsed_time(e1) * 1e3 / K

        t_end = time.perf_counter() + a.spin_ms / 1e3
        while time.perf_counter() < t_end:
            for _, run in variants.values():
                timed(run)
        res = {v: [] for v in variants}
        for _ in range(a.rounds):
            for v, (_, run) in variants.items():
                res[v].append(timed(run))
        for v, (envs, _) in variants.items():
            for env in envs:
                env.check_errors()
            xs = sorted(res[v])
            med = statistics.median(xs)
            print(json.dumps({"config": cfg, "variant": v, "shards": len(envs), "steps": K, "us_per_step_median": med,
                              "us_per_step_min": xs[0], "us_per_step_max": xs[-1],
                              "Gsteps": N * tab.n_agents / med / 1e3}), flush=True)
        del variants, keep
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
