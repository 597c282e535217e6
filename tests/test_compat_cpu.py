"""The dict API on the CPU (rmx.compat.RMEnvironmentWrapper with device="cpu"): the engine's host path
(csrc/rmx_hoststep.cpp behind a host handle of the same C ABI) replays the reference's golden trajectories, through
the C step path (csrc/rmx_dictstep.c) and the Python one, dict for dict.

No GPU and no stand-in: the host handle IS the product path of BASELINE config 1 (the reference's one-env CPU case);
the golden fixtures (recorded from the reference by tests/golden/gen_golden.py) are the checker."""
import ctypes as C
import os

import numpy as np
import pytest

from rmx import _capi
from rmx import _dictstep
from rmx import compat as CP
from rmx import engine as E
from rmx import tables as T


class CountingStep:
    """_dictstep with its step calls counted (which steps the C path served)."""

    def __init__(self):
        self.calls = 0
        self.SOURCE_HASH, self.CTX_ITEMS = _dictstep.SOURCE_HASH, _dictstep.CTX_ITEMS

    def step(self, ctx, actions):
        r = _dictstep.step(ctx, actions)
        self.calls += r is not None
        return r


@pytest.fixture
def counting(monkeypatch):
    c = CountingStep()
    monkeypatch.setattr(CP, "_dictstep_module", lambda: c)
    return c


def _golden_seed(desc, base, e, k):
    scale, es, ks = desc.get("seed_schedule") or ((1, 1, 0) if desc["kind"] == "frozen_lake" else (1000, 1000, 1))
    return (base * scale + e * es + k * ks) % 2**64


def _wrapper(desc, python_path):
    env, agents = CP.scenario_objects(desc)
    env.frozen_lake_stochastic = env.stochastic = bool(desc.get("stochastic", False))
    env.delay_action = bool(desc.get("delay_action", False))
    env.all_slip = bool(desc.get("all_slip", False))
    env.high_prob = desc.get("high_prob", 0.8)
    if desc["kind"] == "frozen_lake":
        env.random_start_positions = bool(desc.get("random_start_positions", False))
    w = CP.RMEnvironmentWrapper(env, agents, device="cpu")
    w.use_c_step = not python_path
    return w, env, agents


def _strip(infos):
    """infos with the RM objects by identity class only (the two wrappers hold different RM objects)."""
    return {n: [(k, type(v).__name__ if k == "reward_machine" else v) for k, v in d.items()] for n, d in infos.items()}


@pytest.mark.parametrize("name,env_index", [("fl2", 0), ("fl2_quirks", 3), ("ow2_final", 1), ("ow2_fail", 0),
                                            ("fl2_slip", 2), ("ow2_allslip", 1), ("fl2_randstart", 4), ("fl4", 1),
                                            ("ow1", 2), ("ow3", 0), ("ow1_map3", 1), ("fl2_initfinal", 0),
                                            ("ow3_slip", 2), ("fl4_randstart_open", 5)])
def test_dict_api_c_and_python_paths_replay_golden(name, env_index, configs, golden_dir, counting):
    g = dict(np.load(os.path.join(golden_dir, f"traj_{name}.npz")))
    desc = configs[name]
    wc, envc, agc = _wrapper(desc, False)
    wp, envp, agp = _wrapper(desc, True)
    base, episode = int(g["seed"]), 0
    for w in (wc, wp):
        w.reset(seed=_golden_seed(desc, base, env_index, episode))
    names = ["up", "down", "left", "right"]
    steps = min(200, g["actions"].shape[0])
    for s in range(steps):
        outs = []
        for w, agents in ((wc, agc), (wp, agp)):
            acts = {ag.name: CP.ActionRL(names[int(g["actions"][s, i, env_index])]) for i, ag in enumerate(agents)}
            outs.append(w.step(acts))
        (oc, rc, tc, uc, ic), (op, rp, tp, up_, ip) = outs
        assert oc == op and rc == rp and tc == tp and uc == up_ and _strip(ic) == _strip(ip), s
        for i, ag in enumerate(agc):
            assert oc[ag.name] == {"pos_x": int(g["pos_x"][s, i, env_index]), "pos_y": int(g["pos_y"][s, i, env_index])}
            assert abs(rc[ag.name] - g["reward"][s, i, env_index]) <= 1e-6
            assert tc[ag.name] is bool(g["term"][s, i, env_index])
            assert uc[ag.name] is bool(g["trunc"][s, i, env_index])
            rm = ag.get_reward_machine()
            assert rm.get_state_index(ic[ag.name]["q"]) == int(g["q"][s, i, env_index])
            assert ic[ag.name]["reward_machine"] is rm
            assert envc.active_agents[ag.name] is bool(g["active"][s, i, env_index])
        assert envc.timestep == int(g["t"][s, env_index]) == envp.timestep
        assert envc.agent_steps == envp.agent_steps and envc.agent_fail == envp.agent_fail
        if g["env_done"][s, env_index]:
            episode += 1
            for w in (wc, wp):
                w.reset(seed=_golden_seed(desc, base, env_index, episode))
    # the host handle stepped them, and the C path served every step of the C-path wrapper (no Python fallback)
    assert isinstance(wc._engine, E.HostRMEnv) and wc._engine.step_variant == "host"
    assert counting.calls == steps


def test_c_path_falls_back_to_python_where_it_must(configs):
    """A learner with use_qrm, an int action and FrozenLake slip's "wait" take the Python path (which raises the
    reference's KeyError for the latter); a plain step takes the C path."""
    desc = configs["fl2_slip"]
    w, env, agents = _wrapper(desc, False)
    w.reset(seed=3)
    ctx = w._ctx
    a0, a1 = agents[0].name, agents[1].name
    assert _dictstep.step(ctx, {a0: CP.ActionRL("up"), a1: CP.ActionRL("wait")}) is None
    with pytest.raises(KeyError):
        w.step({a0: CP.ActionRL("up"), a1: CP.ActionRL("wait")})
    assert _dictstep.step(ctx, {a0: 0, a1: CP.ActionRL("up")}) is None
    assert _dictstep.step(ctx, {a0: CP.ActionRL("nope"), a1: CP.ActionRL("up")}) is None
    with pytest.raises(KeyError):
        w.step({a0: CP.ActionRL("nope"), a1: CP.ActionRL("up")})

    class Learner:
        use_qrm = True
    agents[0].set_learning_algorithm(Learner())
    assert _dictstep.step(ctx, {a0: CP.ActionRL("up"), a1: CP.ActionRL("up")}) is None
    agents[0].set_learning_algorithm(None)
    r = _dictstep.step(ctx, {a0: CP.ActionRL("up"), a1: CP.ActionRL("up")})
    assert isinstance(r, tuple) and len(r) == 5 and set(r[0]) == {a0, a1}


def test_c_path_survives_an_action_that_removes_itself(configs):
    """An action whose `.name` property deletes its own entry from the actions dict (the dict held the only reference):
    the C path keeps the object alive while the property runs and steps as the Python path does."""
    desc = configs["fl2"]
    outs = []
    for python_path in (False, True):
        w, env, agents = _wrapper(desc, python_path)
        w.reset(seed=3)
        acts = {}

        class Vanishing:
            @property
            def name(self):
                acts.pop(agents[0].name, None)
                return "down"
        acts[agents[0].name] = Vanishing()
        acts[agents[1].name] = CP.ActionRL("right")
        outs.append(w.step(acts)[:4])
    assert outs[0] == outs[1]


def test_qrm_experiences_c_and_python_paths(configs, golden_dir, counting):
    """A use_qrm learner (rm_environment_wrapper.py:78-89): the C step path builds infos["qrm_experience"] from the QRM
    columns; it equals the Python path's tuples and the reference's own (the fl2 golden's qrm_* fields)."""
    g = dict(np.load(os.path.join(golden_dir, "traj_fl2.npz")))
    desc = configs["fl2"]
    keys = ("qrm_s", "qrm_a", "qrm_r", "qrm_sn", "qrm_done", "qrm_pos", "qrm_q", "qrm_npos", "qrm_nq", "qrm_hr")

    class Learner:
        use_qrm = True

    ws = []
    for python_path in (False, True):
        w, env, agents = _wrapper(desc, python_path)
        for ag in agents:
            ag.set_learning_algorithm(Learner())
        w.reset(seed=0)
        ws.append((w, agents))
    (wc, agc), (wp, agp) = ws
    names = ["up", "down", "left", "right"]
    calls0 = counting.calls
    for s in range(120):
        outs = []
        for w, agents in ws:
            acts = {ag.name: CP.ActionRL(names[int(g["actions"][s, i, 0])]) for i, ag in enumerate(agents)}
            outs.append(w.step(acts))
        ic, ip = outs[0][4], outs[1][4]
        assert _strip(ic) == _strip(ip), s
        for i, ag in enumerate(agc):
            exps = ic[ag.name]["qrm_experience"]
            assert list(ic[ag.name]) == list(ip[agp[i].name])  # the info keys in the reference's order
            assert len(exps) == len(ag.get_reward_machine().get_all_states()) - 1
            for j, x in enumerate(exps):
                ref = tuple(g[k][s, i, j, 0] for k in keys)
                assert x[0] == ref[0] and x[1] == ref[1] and x[3] == ref[3] and x[4] is bool(ref[4])
                assert x[5:9] == tuple(int(v) for v in ref[5:9])
                assert abs(x[2] - ref[2]) <= 1e-6 and abs(x[9] - ref[9]) <= 1e-6
        if g["env_done"][s, 0]:
            for w, _ in ws:
                w.reset(seed=0)
    assert counting.calls - calls0 == 120  # every step on the C path


def test_failed_rebuild_leaves_no_stale_c_context(configs, monkeypatch):
    """A rebuild that replaces the engine and then fails (here: restoring the episode state raises) must not leave the
    C step path's context pointing at the closed engine: the next step takes the Python path on the new engine (or
    raises a Python exception), never a freed handle.  (rmx/compat.py _build / _agent_cache.)"""
    desc = configs["fl2"]
    w, env, agents = _wrapper(desc, False)
    w.reset(seed=1)
    a0, a1 = agents[0].name, agents[1].name
    acts = {a0: CP.ActionRL("right"), a1: CP.ActionRL("down")}
    w.step(acts)
    old = w._engine

    def boom(self, snap):
        raise RuntimeError("injected restore failure")
    monkeypatch.setattr(E.HostRMEnv, "load_snapshot", boom)
    w.reward_modifier = 2  # the next step rebuilds the tables (and the engine) before it steps
    with pytest.raises(RuntimeError, match="injected"):
        w.step(acts)
    assert w._engine is not old and old._h is None  # the old handle is closed ...
    assert w._ctx is None  # ... and no context refers to it
    monkeypatch.undo()
    obs, rew, terms, truncs, infos = w.step(acts)  # the Python path on the new engine
    assert set(obs) == {a0, a1} and w._ctx is None
    w.reset(seed=1)  # the next reset installs the context for the new engine
    assert w._ctx is not None and w._cstep is not CP._no_c_step
