"""Where the bench's per-step time differs from scripts/variants.py: per-replay timing of one captured
K-step graph (replays 1..R on continuing state), with the action array sized for K or for W + K steps,
and with / without the env_done byte column.  Prints one JSON line per case."""
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
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    tab = T.compile_scenario(T.baseline_scenario(args.config))
    K = args.steps
    for extra, env_done in ((0, True), (100, True), (1100, True), (100, False)):
        env = VecRMEnv(tab, args.n_envs, with_renv=False, with_env_done=env_done)
        acts = env.fill_actions(0, 0, K + extra)
        for s in range(min(extra, 100)):
            env.step(acts[s])
        g = torch.cuda.CUDAGraph()
        s0 = torch.cuda.Stream()
        s0.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s0):
            with torch.cuda.graph(g, stream=s0):
                for s in range(K):
                    env.step(acts[extra + s])
        torch.cuda.current_stream().wait_stream(s0)
        torch.cuda.synchronize()
        times = []
        for r in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            g.replay()
            e1.record()
            torch.cuda.synchronize()
            times.append(round(e0.elapsed_time(e1) * 1e3 / K, 4))
        print(json.dumps({"config": args.config, "action_steps": K + extra, "env_done": env_done,
                          "us_per_step_by_replay": times}), flush=True)
        env.close()
        del g


if __name__ == "__main__":
    main()
