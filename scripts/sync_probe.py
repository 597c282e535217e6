"""Diagnostic (not product): BASELINE config 1 through the dict API (rmx.compat.RMEnvironmentWrapper) and the bare
synchronous C call it rests on (rmx_step_sync at N = 1), median over --reps blocks of --calls calls, after a warm-up.
RMX_LIB selects the library (same-box A/B).  Prints one JSON line.
    python scripts/sync_probe.py --reps 7 --calls 20000
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
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--calls", type=int, default=20000)
    args = ap.parse_args()
    import numpy as np
    from rmx import compat as CP
    from rmx import tables as T

    desc = T.baseline_scenario(1)
    env, agents = CP.scenario_objects(desc)
    w = CP.RMEnvironmentWrapper(env, agents)
    names = [ag.name for ag in agents]
    A = len(agents)
    acts = [CP.ActionRL(n) for n in ("up", "down", "left", "right")]
    pre = np.random.default_rng(0).integers(0, 4, size=(100_000, A)).tolist()
    w.reset(0)

    def dict_block(n):
        t0 = time.perf_counter()
        for s in range(n):
            row = pre[s % len(pre)]
            _, _, terms, truncs, _ = w.step({names[i]: acts[row[i]] for i in range(A)})
            if all(terms.values()) or all(truncs.values()):
                w.reset(0)
        return (time.perf_counter() - t0) / n * 1e6

    def bare_block(n):
        f, h, a, b = w._step_fn, w._h, w._act_p, w._bufs_p
        t0 = time.perf_counter()
        for _ in range(n):
            f(h, a, 1, b, None)
        return (time.perf_counter() - t0) / n * 1e6

    dict_block(5000)
    bare_block(5000)
    res = {"dict_us": [], "bare_us": []}
    for _ in range(args.reps):
        res["dict_us"].append(dict_block(args.calls))
        res["bare_us"].append(bare_block(args.calls))
    out = {k + "_median": round(statistics.median(v), 3) for k, v in res.items()}
    out.update({k: [round(x, 3) for x in v] for k, v in res.items()})
    out["lib"] = os.path.basename(os.environ.get("RMX_LIB", "librmx.so"))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
