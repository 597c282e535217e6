"""Diagnostic (not product): host time of one eager VecRMEnv.step call (Python wrapper + rmx_step's parameter block +
the HIP launch), back to back without synchronising, against a torch in-place add on a 4-element tensor and the bare
C call; config 2, 65,536 envs.  Prints one JSON line."""
import ctypes as C
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    import torch
    from rmx import tables as T
    from rmx.engine import VecRMEnv

    env = VecRMEnv(T.compile_scenario(T.baseline_scenario(2)), 65536)
    acts = env.fill_actions(0, 0, 1)[0]
    x = torch.zeros(4, device="cuda")
    lib, h, ap = env.lib, env._h, C.c_void_p(acts.data_ptr())
    sp = env._stream()
    res = {}
    for name, fn in (("torch_add", lambda: x.add_(1)), ("step", lambda: env.step(acts)),
                     ("bare_rmx_step", lambda: lib.rmx_step(h, ap, 1, sp))):
        per = []
        for rep in range(7):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(200):
                fn()
            per.append((time.perf_counter() - t0) / 200 * 1e6)
            torch.cuda.synchronize()
        res[f"{name}_host_us"] = round(statistics.median(per), 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
