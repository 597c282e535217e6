"""The dict API's host logic on the CPU (rmx.compat.RMEnvironmentWrapper): the C step path (csrc/rmx_dictstep.c) and
the Python one replay the reference's golden trajectories and agree dict for dict.

No GPU here: the engine's synchronous entry points (rmx_reset_sync, rmx_step_sync_begin, rmx_sync_wait) are stood in
for by C-callable functions that step the CPU oracle at N = 1 and write the output record the resident workgroup
writes.  That is test infrastructure (the oracle as the checker's stand-in for the device): it pins the host
plumbing — action mapping, the record layout, the five dicts and their keys, the RM labels, the env mirrors,
positions — while tests/test_compat.py pins the same replays on the GPU."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle as O
from rmx import _capi
from rmx import _dictstep
from rmx import compat as CP
from rmx import engine as E
from rmx import tables as T

BEGIN = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p)
WAIT = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p)
RESET = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p)
STEP = C.CFUNCTYPE(C.c_int, C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p)


class OracleDevice:
    """VecRMEnv's interface as the dict API uses it, over the CPU oracle at N = 1."""

    def __init__(self, tables, n_envs, device=0, with_qrm=False):
        assert n_envs == 1
        self.orc = O.OracleEnv(tables, 1)
        self.A, self.n_qrm_max, self.qrm_s = tables.n_agents, 0, None
        if with_qrm and self.orc.qrm_s is not None:  # the QRM columns (the oracle computes them whenever it can)
            self.n_qrm_max, self.qrm_s = int(self.orc.qrm_s.shape[1]), self.orc.qrm_s
        self._h = C.c_void_p(1)
        self._acts = np.zeros(self.A, np.int32)
        self.calls = {"begin": 0, "wait": 0, "reset": 0}

        def write(bufs_p):
            b = C.cast(bufs_p, C.POINTER(_capi.RmxBuffers)).contents
            o = self.orc
            for name, src, ct in (("pos_x", o.pos_x, C.c_int32), ("pos_y", o.pos_y, C.c_int32),
                                  ("rm_q", o.rm_q, C.c_int32), ("flags", o.flags.view(np.int32), C.c_int32),
                                  ("reward", o.reward, C.c_float), ("renv", o.renv, C.c_float)):
                dst = getattr(b, name)
                if dst:
                    C.memmove(dst, np.ascontiguousarray(src[:, 0]).ctypes.data, 4 * self.A)
            if b.t:
                C.memmove(b.t, o.t.ctypes.data, 4)
            if b.qrm_s and o.qrm_s is not None:  # [A][Qx] at N = 1
                for name, src in (("qrm_s", o.qrm_s), ("qrm_sn", o.qrm_sn), ("qrm_rq", o.qrm_rq), ("qrm_done", o.qrm_done)):
                    a = np.ascontiguousarray(src[:, :, 0])
                    C.memmove(getattr(b, name), a.ctypes.data, a.nbytes)

        def begin(h, act, autoreset, stream):
            C.memmove(self._acts.ctypes.data, act, 4 * self.A)
            self.calls["begin"] += 1
            return 0

        def wait(h, bufs):
            self.orc.step(self._acts.reshape(self.A, 1), autoreset=False)
            write(bufs)
            self.calls["wait"] += 1
            return 0

        def reset(h, seed, bufs, stream):
            self.orc.reset(seed=seed)
            write(bufs)
            self.calls["reset"] += 1
            return 0

        def step(h, act, autoreset, bufs, stream):
            begin(h, act, autoreset, stream)
            return wait(h, bufs)

        self._keep = (BEGIN(begin), WAIT(wait), RESET(reset), STEP(step))
        self.lib = type("Lib", (), {})()
        self.lib.rmx_step_sync_begin, self.lib.rmx_sync_wait, self.lib.rmx_reset_sync, self.lib.rmx_step_sync = \
            self._keep

    def close(self):
        pass

    def sync_end(self):
        pass


@pytest.fixture
def oracle_device(monkeypatch):
    monkeypatch.setattr(E, "VecRMEnv", OracleDevice)


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
    w = CP.RMEnvironmentWrapper(env, agents)
    w.use_c_step = not python_path
    return w, env, agents


def _strip(infos):
    """infos with the RM objects by identity class only (the two wrappers hold different RM objects)."""
    return {n: [(k, type(v).__name__ if k == "reward_machine" else v) for k, v in d.items()] for n, d in infos.items()}


@pytest.mark.parametrize("name,env_index", [("fl2", 0), ("fl2_quirks", 3), ("ow2_final", 1), ("ow2_fail", 0),
                                            ("fl2_slip", 2), ("ow2_allslip", 1), ("fl2_randstart", 4), ("fl4", 1),
                                            ("ow1", 2), ("ow3", 0), ("ow1_map3", 1), ("fl2_initfinal", 0),
                                            ("ow3_slip", 2), ("fl4_randstart_open", 5)])
def test_dict_api_c_and_python_paths_replay_golden(name, env_index, configs, golden_dir, oracle_device, monkeypatch):
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
    # the C path served the steps (one begin / wait pair each, no Python-path fallback)
    assert wc._engine.calls["begin"] == steps == wc._engine.calls["wait"]


def test_c_path_falls_back_to_python_where_it_must(configs, oracle_device):
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


def test_qrm_experiences_c_and_python_paths(configs, golden_dir, oracle_device):
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
    calls0 = wc._engine.calls["begin"]
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
    assert wc._engine.calls["begin"] - calls0 == 120  # every step on the C path
