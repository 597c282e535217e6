"""FrozenLake slip rollout throughput: the fused fast rollout (rollout_fast_kernel<..., SLIP>) vs the generic
rollout kernel (RMX_FAST_SKIP=1 routes a slip handle to the generic kernels).  65,536 envs x 2,000 steps,
event-timed, median of 5.  Prints one JSON line."""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv
    with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
        cfgs = json.load(f)
    N, Tn = 65536, 2000
    res = {"n_envs": N, "steps": Tn}
    for name in ("fl2_slip", "fl2_delay"):
        for mode in ("fast", "generic"):
            if mode == "generic":
                os.environ["RMX_FAST_SKIP"] = "1"
            else:
                os.environ.pop("RMX_FAST_SKIP", None)
            env = VecRMEnv(T.compile_scenario(cfgs[name]), N)
            env.reset(seed=3)
            env.rollout(1, 0, 50)
            ts = []
            for r in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize()
                e0.record()
                env.rollout(1, 50 + r * Tn, Tn)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e3 / Tn)
            us = statistics.median(ts)
            res[f"{name}/{mode}"] = {"us_per_step": round(us, 3), "agent_steps_per_s": round(N * env.A / us * 1e6)}
            del env
    os.environ.pop("RMX_FAST_SKIP", None)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
