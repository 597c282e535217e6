"""Time the REFERENCE Python step loop in the build container (it cannot travel to the GPU box).

Same workload as bench.py's default (BASELINE config 2: FrozenLake map1, 2 agents, built-in A->B->C
RM, uniform random actions, autoreset per frozen_lake_main.py:336-376) and the other BASELINE shapes, ~N seconds
each, in one process and in one process per core (1 and 8 processes).
Also times the port's drop-in (rmx.compat on the engine's host path) head to head with the reference's loop,
alternating in this process (head_to_head).  Writes profiles/reference_cpu_container.json.  Run from /tmp:

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


class _PlainLearner:
    """The bench workload emits no QRM counterfactuals (the headline kernel's outputs are the step's own), so
    the timed reference loop runs the wrapper without them (use_qrm False: rm_environment_wrapper.py:78)."""
    use_qrm = False


def run(cfg_name, seconds):
    cfg = G.CONFIGS[cfg_name]
    rm_env, agents, _ = G.make_env(cfg)
    for ag in agents:
        ag.set_learning_algorithm(_PlainLearner())
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


def run_rmx_host(cfg_name, seconds):
    """The same loop through the port's drop-in, rmx.compat.RMEnvironmentWrapper on the engine's host path
    (device="cpu": the host handle of librmx.so), on the same scenario (tests/golden/configs.json, the configs the
    reference goldens were recorded from), agents with the same use_qrm-False learner."""
    import numpy as np

    root = os.path.dirname(os.path.dirname(HERE))
    sys.path.insert(0, os.path.join(root, "multiagent-rl-rm_amd"))
    from rmx import compat as CP
    with open(os.path.join(HERE, "configs.json")) as f:
        desc = json.load(f)[cfg_name]
    env, agents = CP.scenario_objects(desc)
    for ag in agents:
        ag.set_learning_algorithm(_PlainLearner())
    w = CP.RMEnvironmentWrapper(env, agents, device="cpu")
    A = len(agents)
    names = [ag.name for ag in agents]
    acts = [CP.ActionRL(n) for n in G.ACTION_NAMES]
    pre = np.random.default_rng(0).integers(0, 4, size=(400_000, A)).tolist()
    steps = t = 0
    need_reset = True
    t0 = time.perf_counter()
    while True:
        if need_reset:
            w.reset(0)
            need_reset = False
        row = pre[t % len(pre)]
        _, _, terms, truncs, _ = w.step({names[i]: acts[row[i]] for i in range(A)})
        steps += 1
        t += 1
        if all(terms.values()) or all(truncs.values()):
            need_reset = True
        if steps % 2000 == 0 and time.perf_counter() - t0 > seconds:
            break
    dt = time.perf_counter() - t0
    return {"config": cfg_name, "env_steps": steps, "seconds": dt, "value": steps * A / dt,
            "unit": "(env x agent)-steps/s", "cores": 1, "engine": "rmx host path (device=\"cpu\")"}


def head_to_head(cfg_name, seconds, rounds=5):
    """The reference loop and the port's host-path loop back to back in this process, `rounds` times alternating
    (the container's speed drifts by 2x over minutes: a ratio of neighbouring runs is what holds); the median ratio."""
    import statistics
    pairs = []
    for _ in range(rounds):
        r, p = run(cfg_name, seconds), run_rmx_host(cfg_name, seconds)
        pairs.append({"reference": r["value"], "rmx_host": p["value"], "ratio": p["value"] / r["value"]})
    return {"config": cfg_name, "seconds_each": seconds, "rounds": pairs,
            "median_ratio": statistics.median(x["ratio"] for x in pairs)}


def _one(args):
    return run(*args)


def run_parallel(cfg_name, seconds, procs):
    """procs independent copies of the loop, one per process (the reference is single-threaded Python: its
    only parallelism is more processes); value = the sum of the per-process rates."""
    import multiprocessing as mp

    with mp.get_context("fork").Pool(procs) as pool:
        res = pool.map(_one, [(cfg_name, seconds)] * procs)
    return {"config": cfg_name, "env_steps": sum(r["env_steps"] for r in res),
            "seconds": max(r["seconds"] for r in res), "value": sum(r["value"] for r in res),
            "unit": "(env x agent)-steps/s", "cores": procs, "per_process": [r["value"] for r in res]}


def cpu_model():
    try:
        import subprocess
        for ln in subprocess.run(["lscpu"], capture_output=True, text=True).stdout.splitlines():
            if ln.startswith("Model name:"):
                return ln.split(":", 1)[1].strip()
    except Exception:
        pass
    return platform.processor() or platform.machine()


if __name__ == "__main__":
    secs = float(sys.argv[1]) if len(sys.argv) > 1 else 10.0
    procs = os.cpu_count() or 1
    cfgs = ("fl2", "ow1", "ow3", "fl4")
    sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
    from bench import python_speed_probe  # the fixed workload bench.py times on the GPU box's host as well
    probe = python_speed_probe()
    res = {"kind": "reference",
           "where": f"build container (no GPU), stub imports of SURVEY §8(c); 1 process, then {procs} processes "
                    f"(one per core, os.cpu_count())",
           "cpu": cpu_model(), "cpu_count": procs, "python": platform.python_version(),
           "python_probe_us": probe,
           "runs": [run(c, secs) for c in cfgs],
           "head_to_head": head_to_head("fl2", min(secs, 4.0)),
           "runs_all_cores": [run_parallel(c, secs, procs) for c in cfgs]}
    out = os.path.join(os.path.dirname(os.path.dirname(HERE)), "profiles", "reference_cpu_container.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))
