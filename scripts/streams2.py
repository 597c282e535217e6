"""Concurrency experiment 2: split N envs into S independent shards, each with its OWN captured graph
(K steps) on its OWN stream, replayed concurrently.  Per-env step order is unchanged; shards only
overlap each other's launch boundaries.  (streams.py captured all shards in ONE graph with fork/join,
which the runtime serialises.)"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--n-envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--shards", default="1,2,4")
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    tab = T.compile_scenario(T.baseline_scenario(args.config))
    N, K = args.n_envs, args.steps
    ref = None
    for S in [int(x) for x in args.shards.split(",")]:
        n = N // S
        envs = [VecRMEnv(tab, n, env_offset=i * n, n_envs_global=N, with_renv=False) for i in range(S)]
        acts = [e.fill_actions(0, 0, K) for e in envs]
        streams = [torch.cuda.Stream() for _ in range(S)]
        graphs = []
        torch.cuda.synchronize()
        for i in range(S):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.stream(streams[i]):
                with torch.cuda.graph(g, stream=streams[i]):
                    for s in range(K):
                        envs[i].step(acts[i][s])
            graphs.append(g)
        torch.cuda.synchronize()
        times = []
        for r in range(args.reps):
            for e in envs:
                e.reset()
            torch.cuda.synchronize()
            main = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            for i in range(S):
                streams[i].wait_stream(main)
                with torch.cuda.stream(streams[i]):
                    graphs[i].replay()
            for i in range(S):
                main.wait_stream(streams[i])
            e1.record(main)
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / K)
        st = torch.cat([e.pos_x for e in envs], dim=1).cpu()
        if ref is None:
            ref = st
        same = bool(torch.equal(st, ref))
        best = min(times)
        print(json.dumps({"config": args.config, "shards": S, "us_per_step": best, "median": sorted(times)[len(times) // 2],
                          "Gsteps": N * tab.n_agents / best / 1e3, "state_equal_to_S1": same}), flush=True)
        del graphs


if __name__ == "__main__":
    main()
