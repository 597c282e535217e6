"""Time the REFERENCE Python step loop in the build container (it cannot travel to the GPU box).

Same workload as bench.py's default (BASELINE config 2: FrozenLake map1, 2 agents, built-in A->B->C
RM, uniform random actions, autoreset per frozen_lake_main.py:336-376), one process, ~N seconds.
Writes profiles/reference_cpu_container.json.  Run from /tmp:

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/time_reference.py
"""
import json
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import gen_golden as G  # noqa: E402  (installs the stubs, imports the reference)


def run(cfg_name, seconds):
    cfg = G.CONFIGS[cfg_name]
    rm_env, agents, _ = G.make_env(cfg)
    A = len(agents)
    names = [ag.name for ag in agents]
    acts = [G.ActionRL(n) for n in G.ACTION_NAMES]
    # pre-generated uniform actions (kept out of the timed loop, like bench.py's HBM-resident inputs)
    import numpy as np
    pre = np.random.default_rng(0).integers(0, 4, size=(400_000, A)).tolist()
    steps = 0
    t = 0
    need_reset = True
    t0 = time.perf_counter()
    while True:
        if need_reset:
            rm_env.reset(0)
            need_reset = False
        row = pre[t % len(pre)]
        actions = {names[i]: acts[row[i]] for i in range(A)}
        _, _, terms, truncs, _ = rm_env.step(actions)
        steps += 1
        t += 1
        if all(terms.values()) or all(truncs.values()):
            need_reset = True
        if steps % 2000 == 0 and time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"config": cfg_name, "env_steps": steps, "seconds": dt, "value": steps * A / dt,
            "unit": "(env x agent)-steps/s", "cores": 1}


if __name__ == "__main__":
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    res = {"kind": "reference", "where": "build container (no GPU), 1 process, stub imports of SURVEY §8(c)",
           "cpu": platform.processor() or platform.machine(), "python": platform.python_version(),
           "runs": [run("fl2", secs), run("ow1", secs), run("ow3", secs), run("fl4", secs)]}
    out = os.path.join(os.path.dirname(os.path.dirname(HERE)), "profiles", "reference_cpu_container.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))
