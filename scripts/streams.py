"""Concurrency experiment: split N envs into S independent shards, each stepped on its own HIP stream,
all captured in one graph (fork/join).  Per-env step order is unchanged (env e's step s+1 still follows
its step s on the same stream); different shards overlap each other's launch boundaries."""
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
    ap.add_argument("--shards", default="1,2,4,8")
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
        main_s = torch.cuda.Stream()
        g = torch.cuda.CUDAGraph()
        main_s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(main_s):
            with torch.cuda.graph(g, stream=main_s):
                for i in range(S):
                    streams[i].wait_stream(main_s)
                    with torch.cuda.stream(streams[i]):
                        for s in range(K):
                            envs[i].step(acts[i][s])
                for i in range(S):
                    main_s.wait_stream(streams[i])
        torch.cuda.current_stream().wait_stream(main_s)
        for e in envs:
            e.reset()
        torch.cuda.synchronize()
        times = []
        for r in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) * 1e3 / K)
        # state after the last replay == reps x K steps from reset; compare across S
        st = torch.cat([e.pos_x for e in envs], dim=1).cpu()
        q = torch.cat([e.rm_q for e in envs], dim=1).cpu()
        for e in envs:
            e.reset()
        if ref is None:
            ref = None
        best = min(times)
        print(json.dumps({"config": args.config, "shards": S, "us_per_step": best,
                          "Gsteps": N * tab.n_agents / best / 1e3, "median": sorted(times)[len(times) // 2]}),
              flush=True)
        del g


if __name__ == "__main__":
    main()
