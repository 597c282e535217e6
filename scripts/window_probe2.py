"""Fixed cost of a short timed window, by variant (diagnostic, GPU box).  Config 2, 65,536 envs, K steps:
  A  graph(K steps); stats launch; device sync          (bench.py's window)
  B  graph(K steps + stats); device sync
  C  graph(K steps + stats); event sync
  E  A with events around steps / stats (GPU time of each part)
Prints the median wall us per window of 11 windows per variant."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))
import torch  # noqa: E402

from rmx import tables as T  # noqa: E402
from rmx.engine import VecRMEnv  # noqa: E402


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    W = 5
    tab = T.compile_scenario(T.baseline_scenario(2))
    env = VecRMEnv(tab, 65536, device=0, with_renv=False, with_env_done=True)
    st = torch.cuda.current_stream()
    acts = env.fill_actions(0, 0, W + K)
    graphs = {}
    for with_stats in (False, True):
        g = torch.cuda.CUDAGraph()
        s0 = torch.cuda.Stream()
        s0.wait_stream(st)
        with torch.cuda.stream(s0):
            with torch.cuda.graph(g, stream=s0):
                for s in range(K):
                    env.step(acts[W + s])
                if with_stats:
                    env.stats_tensor()
        st.wait_stream(s0)
        g.replay()
        torch.cuda.synchronize()
        graphs[with_stats] = g
    res = {}
    for var in ("A", "B", "C", "E", "A", "B", "C"):
        walls, parts = [], []
        for w in range(11):
            env.reset()
            env.clear_stats()
            for s in range(W):
                env.step(acts[s])
            evs = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if var == "A":
                graphs[False].replay()
                env.stats_tensor()
                torch.cuda.synchronize()
            elif var == "B":
                graphs[True].replay()
                torch.cuda.synchronize()
            elif var == "C":
                graphs[True].replay()
                evs[2].record(st)
                evs[2].synchronize()
            else:
                evs[0].record(st)
                graphs[False].replay()
                evs[1].record(st)
                env.stats_tensor()
                evs[2].record(st)
                torch.cuda.synchronize()
                parts.append((evs[0].elapsed_time(evs[1]) * 1e3, evs[1].elapsed_time(evs[2]) * 1e3))
            walls.append((time.perf_counter() - t0) * 1e6)
        r = {"variant": var, "K": K, "wall_us_median": statistics.median(walls), "wall_us_min": min(walls)}
        if parts:
            r["steps_us_median"] = statistics.median(p[0] for p in parts)
            r["stats_us_median"] = statistics.median(p[1] for p in parts)
        print(json.dumps(r), flush=True)
    t0 = time.perf_counter()
    torch.cuda.synchronize()
    print(json.dumps({"idle_sync_us": (time.perf_counter() - t0) * 1e6}))


if __name__ == "__main__":
    main()
