"""Debug probe: masked rmx_reset with a new base seed under random starts, stepwise vs the oracle, printing which
envs diverge (masked or not, step of first divergence)."""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "multiagent-rl-rm_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")):
    sys.path.insert(0, p)
import oracle as O  # noqa: E402
from conftest import derived_configs  # noqa: E402
from rmx import tables as T  # noqa: E402
from rmx.engine import VecRMEnv  # noqa: E402

with open(os.path.join(ROOT, "tests", "golden", "configs.json")) as f:
    C = json.load(f)
C.update(derived_configs(C))


def run(name, N, mode, reset_at=250, steps=600, seed=23):
    tab = T.compile_scenario(C[name])
    env = VecRMEnv(tab, N)
    orc = O.OracleEnv(tab, N)
    env.reset(seed=7)
    orc.reset(seed=7)
    mask = (np.arange(N) % 3 == 1).astype(np.uint8)
    first = None
    for s in range(steps):
        if s == reset_at:
            m = None if mode == "nomask" else mask
            sd = 7 if mode == "sameseed" else 1234567
            env.reset(mask=m, seed=sd)
            orc.reset(mask=m, seed=sd)
        env.step_hashed(seed, s)
        orc.step(O.hash_actions(seed, s, 1, N, 0, N, tab.n_agents)[0])
        bad = np.nonzero((env.pos_x.cpu().numpy() != orc.pos_x).any(0) | (env.pos_y.cpu().numpy() != orc.pos_y).any(0))[0]
        if len(bad) and first is None:
            first = s
            e = int(bad[0])
            print(json.dumps({"name": name, "N": N, "mode": mode, "first_bad_step": s, "n_bad": int(len(bad)),
                              "envs": bad[:12].tolist(), "masked": [int(mask[i]) for i in bad[:12]],
                              "env_t": env.t.cpu().numpy()[bad[:12]].tolist(), "orc_t": orc.t[bad[:12]].tolist(),
                              "env_ep": env.episode.cpu().numpy()[bad[:12]].tolist(),
                              "orc_ep": orc.episode[bad[:12]].tolist(),
                              "env_xy": [env.pos_x.cpu().numpy()[:, e].tolist(), env.pos_y.cpu().numpy()[:, e].tolist()],
                              "orc_xy": [orc.pos_x[:, e].tolist(), orc.pos_y[:, e].tolist()]}), flush=True)
            break
    if first is None:
        print(json.dumps({"name": name, "N": N, "mode": mode, "ok": True}), flush=True)
    env.close()


for name in ("fl2_randstart", "fl2_randstart_slip_fixed", "fl2_randstart_slip"):
    for N in (4115, 4096):
        for mode in ("mask", "nomask", "sameseed"):
            run(name, N, mode)
