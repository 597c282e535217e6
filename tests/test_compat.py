"""Reference-shaped dict API (rmx.compat.RMEnvironmentWrapper): tables built from reference-style
objects equal the scenario compiler's; on the GPU the dict API replays a golden trajectory and the
reference's unit KATs (test_ma_frozen_lake.py:46-58, test_rm_environment_wrapper.py:70-90) — on the GPU (the
resident workgroup, gpu-marked) and on the engine's host path (device="cpu", the CPU suite)."""
import os

import numpy as np
import pytest

from rmx import compat as CP
from rmx import tables as T


def _objects(desc):
    return CP.scenario_objects(desc)


def _fl_objects(desc):
    return CP.scenario_objects(desc)


def _ow_objects(desc):
    return CP.scenario_objects(desc)


@pytest.mark.parametrize("name", ["fl2", "fl2_quirks", "fl2_open", "ow1", "ow2_fail", "ow1_map3"])
def test_tables_from_objects_equal_scenario_compiler(name, configs):
    desc = configs[name]
    env, agents = _objects(desc)
    a = CP.tables_from_objects(env, agents)
    b = T.compile_scenario(desc)
    b_gamma = a.gamma  # the dict API reports per-step rewards only; discounting is the loop's business
    for k in ("kind", "width", "height", "n_agents", "n_rm_states", "n_events", "hazard_fail", "wall_fail",
              "max_t"):
        assert getattr(a, k) == getattr(b, k), k
    assert a.hazard_penalty == b.hazard_penalty and a.wall_penalty == b.wall_penalty and b_gamma == 1.0
    for k in ("cell", "cell_event", "next_q", "rm_reward", "init_q", "final_q", "start_xy"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)


def test_stochastic_flags_feed_slip_tables():
    env, agents = _fl_objects(T.baseline_scenario(2))
    env.frozen_lake_stochastic = True
    tab = CP.tables_from_objects(env, agents)
    assert tab.stochastic == 1 and list(tab.slip_n) == [3, 3, 3, 3] and tab.seed_schedule == (1, 0, 0)
    env.delay_action = True
    assert list(CP.tables_from_objects(env, agents).slip_n) == [4, 4, 4, 4]


def test_random_start_flag_is_read():
    """random_start_positions (ma_frozen_lake.py:37-39) reaches the tables; it is not silently dropped."""
    env, agents = _fl_objects(T.baseline_scenario(2))
    assert CP.tables_from_objects(env, agents).random_starts == 0
    env.random_start_positions = True
    assert CP.tables_from_objects(env, agents).random_starts == 1


def test_unmodelled_env_switch_is_refused():
    """A dynamics switch the engine does not model raises instead of being ignored."""
    env, agents = _fl_objects(T.baseline_scenario(2))
    env.some_new_dynamics_flag = True
    with pytest.raises(NotImplementedError, match="some_new_dynamics_flag"):
        CP.tables_from_objects(env, agents)
    env.some_new_dynamics_flag = False  # unset switches change nothing
    CP.tables_from_objects(env, agents)
    env2, agents2 = _ow_objects(T.baseline_scenario(3))
    env2.random_start_positions = True  # a FrozenLake switch: the reference OfficeWorld ignores it too
    assert CP.tables_from_objects(env2, agents2).random_starts == 0


def test_reward_modifier_scales_rm_reward():
    env, agents = _fl_objects(T.baseline_scenario(2))
    a = CP.tables_from_objects(env, agents, reward_modifier=2)
    b = CP.tables_from_objects(env, agents)
    # the modifier scales the wrapper reward in-kernel; the raw table also feeds the QRM experiences
    np.testing.assert_array_equal(a.rm_reward, b.rm_reward)
    assert a.reward_modifier == 2.0 and b.reward_modifier == 1.0


# ------------------------------------------------------------------------------------- GPU and host path
DEVICES = [pytest.param(0, marks=pytest.mark.gpu, id="gpu"), pytest.param("cpu", id="host")]


def _wrapper(env, agents, device):
    """The dict API on `device`; the engine it got is checked (a GPU case never runs on the host path)."""
    from rmx import engine as E
    w = CP.RMEnvironmentWrapper(env, agents, device=device)
    w._build()
    assert isinstance(w._engine, E.HostRMEnv if device == "cpu" else E.VecRMEnv)
    return w


def _golden_seed(desc, base, e, k):
    scale, es, ks = desc.get("seed_schedule") or ((1, 1, 0) if desc["kind"] == "frozen_lake" else (1000, 1000, 1))
    return (base * scale + e * es + k * ks) % 2**64


@pytest.mark.parametrize("device", DEVICES)
@pytest.mark.parametrize("name,env_index", [("fl2", 0), ("fl2_quirks", 3), ("ow2_final", 1), ("ow2_fail", 0),
                                            ("fl2_slip", 2), ("ow2_allslip", 1), ("fl2_delay", 5),
                                            ("fl2_randstart", 4), ("fl2_randstart_slip", 7), ("fl4", 1), ("ow1", 2),
                                            ("ow3", 0), ("ow1_map3", 1), ("fl2_initfinal", 0), ("fl2_finalnt", 3),
                                            ("fl2_open", 1), ("ow1_slip", 3), ("ow2_delay", 0), ("ow3_slip", 2),
                                            ("fl4_randstart_open", 5)])
def test_dict_api_replays_golden(name, env_index, device, configs, golden_dir):
    g = dict(np.load(os.path.join(golden_dir, f"traj_{name}.npz")))
    desc = configs[name]
    env, agents = _objects(desc)
    env.frozen_lake_stochastic = env.stochastic = bool(desc.get("stochastic", False))
    env.delay_action = bool(desc.get("delay_action", False))
    env.all_slip = bool(desc.get("all_slip", False))
    env.high_prob = desc.get("high_prob", 0.8)
    if desc["kind"] == "frozen_lake":
        env.random_start_positions = bool(desc.get("random_start_positions", False))
    base, episode = int(g["seed"]), 0
    w = _wrapper(env, agents, device)
    obs, infos = w.reset(seed=_golden_seed(desc, base, env_index, episode))
    assert set(obs) == {ag.name for ag in agents} and all(infos[n] == {} for n in infos)
    if "reset_xy" in g:
        assert [(o["pos_x"], o["pos_y"]) for o in obs.values()] == \
            [tuple(int(v) for v in g["reset_xy"][0, :, i, env_index]) for i in range(len(agents))]
    names = ["up", "down", "left", "right"]
    steps = min(300, g["actions"].shape[0])
    for s in range(steps):
        acts = {ag.name: CP.ActionRL(names[int(g["actions"][s, i, env_index])]) for i, ag in enumerate(agents)}
        obs, rew, term, trunc, info = w.step(acts)
        for i, ag in enumerate(agents):
            assert obs[ag.name] == {"pos_x": int(g["pos_x"][s, i, env_index]), "pos_y": int(g["pos_y"][s, i, env_index])}
            assert abs(rew[ag.name] - g["reward"][s, i, env_index]) <= 1e-6
            assert term[ag.name] is bool(g["term"][s, i, env_index])
            assert trunc[ag.name] is bool(g["trunc"][s, i, env_index])
            rm = ag.get_reward_machine()
            assert rm.get_state_index(info[ag.name]["q"]) == int(g["q"][s, i, env_index])
            assert abs(info[ag.name]["RQ"] - g["rq"][s, i, env_index]) <= 1e-6
            assert env.active_agents[ag.name] is bool(g["active"][s, i, env_index])
        assert env.timestep == int(g["t"][s, env_index])
        if g["env_done"][s, env_index]:
            episode += 1
            obs, infos = w.reset(seed=_golden_seed(desc, base, env_index, episode))


@pytest.mark.parametrize("device", DEVICES)
def test_frozen_lake_boundary_kat(device):
    # test_ma_frozen_lake.py:46-58 on a 2x2 lake through the engine
    env = CP.MultiAgentFrozenLake(width=2, height=2, holes=[])
    ag = CP.AgentRL("a", env)
    ag.set_initial_position(0, 0)
    ag.set_reward_machine(CP.RewardMachine({("q0", (9, 9)): ("qf", 1)}, CP.PositionEventDetector({(9, 9)})))
    env.add_agent(ag)
    w = _wrapper(env, [ag], device)
    w.reset(123)
    for a, pos in [("left", (0, 0)), ("up", (0, 0)), ("right", (1, 0)), ("down", (1, 1))]:
        w.step({"a": CP.ActionRL(a)})
        assert ag.get_position() == pos


@pytest.mark.parametrize("device", DEVICES)
def test_wrapper_reward_merge_and_rm_termination_kat(device):
    # test_rm_environment_wrapper.py:70-90 restated on a grid: env penalty -0.5 on a hole cell that is
    # also the RM goal event -> reward = -0.5 + 1.0, terminated by the RM, prev_q/q labels
    env = CP.MultiAgentFrozenLake(width=2, height=1, holes=[(1, 0)])
    env.penalty_amount = -0.5
    ag = CP.AgentRL("agent", env)
    ag.set_initial_position(0, 0)
    ag.set_reward_machine(CP.RewardMachine({("q0", (1, 0)): ("qf", 1.0)}, CP.PositionEventDetector({(1, 0)})))
    env.add_agent(ag)
    w = _wrapper(env, [ag], device)
    w.reset(seed=123)
    obs, rew, term, trunc, info = w.step({"agent": CP.ActionRL("right")})
    assert obs["agent"]["pos_x"] == 1
    assert rew["agent"] == 0.5
    assert term["agent"] is True and trunc["agent"] is False
    assert info["agent"]["prev_q"] == "q0" and info["agent"]["q"] == "qf"
    assert info["agent"]["Renv"] == -0.5 and info["agent"]["RQ"] == 1.0
    assert w.check_terminations() == {"agent": True}
    # reward_modifier = 2 (test_rm_environment_wrapper.py:110-150)
    w.reset(seed=0)
    w.reward_modifier = 2
    _, rew, _, _, _ = w.step({"agent": CP.ActionRL("right")})
    assert rew["agent"] == -0.5 + 2.0


@pytest.mark.parametrize("device", DEVICES)
def test_dict_api_qrm_experience_tuples(device, configs, golden_dir):
    """infos["qrm_experience"] for a use_qrm learner equals the reference's tuples (fl2, env 0)."""
    g = dict(np.load(os.path.join(golden_dir, "traj_fl2.npz")))
    env, agents = _objects(configs["fl2"])

    class L:
        use_qrm = True

    for ag in agents:
        ag.set_learning_algorithm(L())
    w = _wrapper(env, agents, device)
    w.reset(seed=0)
    names = ["up", "down", "left", "right"]
    keys = ("qrm_s", "qrm_a", "qrm_r", "qrm_sn", "qrm_done", "qrm_pos", "qrm_q", "qrm_npos", "qrm_nq", "qrm_hr")
    for s in range(120):
        acts = {ag.name: CP.ActionRL(names[int(g["actions"][s, i, 0])]) for i, ag in enumerate(agents)}
        _, _, _, _, info = w.step(acts)
        for i, ag in enumerate(agents):
            exps = info[ag.name]["qrm_experience"]
            assert len(exps) == len(ag.get_reward_machine().get_all_states()) - 1
            for j, x in enumerate(exps):
                ref = tuple(g[k][s, i, j, 0] for k in keys)
                assert x[0] == ref[0] and x[1] == ref[1] and x[3] == ref[3] and x[4] == bool(ref[4])
                assert x[5:9] == tuple(int(v) for v in ref[5:9])
                assert abs(x[2] - ref[2]) <= 1e-6 and abs(x[9] - ref[9]) <= 1e-6
        if g["env_done"][s, 0]:
            w.reset(seed=0)


@pytest.mark.parametrize("device", DEVICES)
def test_get_mdp_kat_small_lake(device):
    """test_ma_frozen_lake.py:86-102: 2x2 lake with a 2-state RM -> 8 states, 4 actions, keyed by name."""
    env = CP.MultiAgentFrozenLake(width=2, height=2, holes=[])
    ag = CP.AgentRL("a", env)
    ag.set_initial_position(0, 0)
    ag.set_reward_machine(CP.RewardMachine({("q0", (1, 0)): ("qf", 1)}, CP.PositionEventDetector({(1, 0)})))
    env.add_agent(ag)
    all_p, all_ns, all_na = _wrapper(env, [ag], device).get_mdp(seed=123)
    assert all_ns["a"] == 8 and all_na["a"] == 4 and set(all_p) == {"a"}


@pytest.mark.parametrize("device", DEVICES)
def test_frozen_lake_slip_wait_raises_keyerror_before_stepping(device, configs):
    """Under FrozenLake slip the reference's stochastic action map has no "wait" entry: get_stochastic_action raises
    KeyError (ma_frozen_lake.py:122, 257) for an agent the env steps.  The dict API raises it on the host before the
    request goes out, so the device state and the host copies stay in step; the handle keeps working.
    This asserts the PORT's behaviour on the error path, which intentionally differs from the reference's: the
    reference raises inside its agent loop (ma_frozen_lake.py:106-124), after earlier agents (here a0) have moved,
    drawn from the rng and counted a step; the port refuses the whole step, so no agent moves."""
    desc = configs["fl2_slip"]
    env, agents = _objects(desc)
    env.frozen_lake_stochastic = True
    w = _wrapper(env, agents, device)
    w.reset(seed=5)
    a0, a1 = agents[0].name, agents[1].name
    before = [ag.get_position() for ag in agents]
    with pytest.raises(KeyError):
        w.step({a0: CP.ActionRL("up"), a1: CP.ActionRL("wait")})
    assert [ag.get_position() for ag in agents] == before and env.timestep == 0
    obs, _, _, _, _ = w.step({a0: CP.ActionRL("up"), a1: CP.ActionRL("left")})
    assert env.timestep == 1 and set(obs) == {a0, a1}
    # the same action is fine in the deterministic env ("wait" is a legal move there)
    env2, agents2 = _objects(desc)
    env2.frozen_lake_stochastic = False
    w2 = _wrapper(env2, agents2, device)
    w2.reset(seed=5)
    w2.step({agents2[0].name: CP.ActionRL("wait"), agents2[1].name: CP.ActionRL("wait")})
    assert env2.timestep == 1
