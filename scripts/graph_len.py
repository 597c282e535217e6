"""Per-step time of the config-2 step chain vs the number of steps captured per HIP graph: K = 1000 steps
as K/L graphs of L steps each (every graph its own slice of the action array, replayed in order), timed
with HIP events on the launch stream, best and median of R repetitions on continuing state."""
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
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--lens", default="1000,500,250,200,100,50,25")
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    tab = T.compile_scenario(T.baseline_scenario(args.config))
    K = args.steps
    env = VecRMEnv(tab, args.n_envs, with_renv=False)
    acts = env.fill_actions(0, 0, K)
    stream = torch.cuda.current_stream()
    for L in [int(x) for x in args.lens.split(",")]:
        graphs = []
        for g0 in range(0, K, L):
            g = torch.cuda.CUDAGraph()
            s0 = torch.cuda.Stream()
            s0.wait_stream(stream)
            with torch.cuda.stream(s0):
                with torch.cuda.graph(g, stream=s0):
                    for s in range(g0, min(K, g0 + L)):
                        env.step(acts[s])
            stream.wait_stream(s0)
            graphs.append(g)
        torch.cuda.synchronize()
        times = []
        for r in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for g in graphs:
                g.replay()
            e1.record(stream)
            torch.cuda.synchronize()
            times.append(round(e0.elapsed_time(e1) * 1e3 / K, 4))
        print(json.dumps({"config": args.config, "steps_per_graph": L, "graphs": len(graphs),
                          "us_per_step_by_rep": times, "best": min(times),
                          "median": sorted(times)[len(times) // 2]}), flush=True)
        del graphs
    env.close()


if __name__ == "__main__":
    main()
