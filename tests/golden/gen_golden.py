"""Generate golden vectors by running the REFERENCE hot path (build container only).

This script imports the read-only reference at ``/root/reference`` (with the
offline stubs of ``_refstubs.py`` for pettingzoo / gymnasium / unified_planning),
drives ``RMEnvironmentWrapper.step`` -> ``MultiAgent{FrozenLake,OfficeWorld}.step``
-> ``RewardMachine.step`` on hash-generated uniform actions with the reference's
own episode loop rules, and writes small fixtures next to this file:

* ``configs.json``   -- the scenario descriptions (shared with the build's table compiler)
* ``tables.json``    -- the reference's own parse / RM-index / final-state / potential results
* ``traj_<cfg>.npz`` -- per-step trajectories (inputs = actions, outputs = state/reward/flags)
* ``episodes_<cfg>.npz`` -- per-episode summaries (return, length, success) for the stats path

The reference never travels to the GPU box: only the fixtures do.  Run from /tmp:

    cd /tmp && PYTHONDONTWRITEBYTECODE=1 python /root/repo/tests/golden/gen_golden.py

Reference call sites followed (paths relative to /root/reference):
  loop rules   multiagent_rlrm/environments/frozen_lake/frozen_lake_main.py:336-376
               multiagent_rlrm/environments/office_world/office_main.py:1696-1749
  success      multiagent_rlrm/environments/utils_envs/evaluation_metrics.py:248-267
  OW setup     multiagent_rlrm/environments/office_world/office_main.py:400-440,539-545
"""
import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _refstubs  # noqa: E402

_refstubs.install()
sys.path.insert(0, "/root/reference")

from multiagent_rlrm.environments.frozen_lake.ma_frozen_lake import MultiAgentFrozenLake  # noqa: E402
from multiagent_rlrm.environments.frozen_lake.detect_event import PositionEventDetector  # noqa: E402
from multiagent_rlrm.environments.frozen_lake.config_frozen_lake import config as fl_config  # noqa: E402
from multiagent_rlrm.environments.office_world.ma_office import MultiAgentOfficeWorld  # noqa: E402
from multiagent_rlrm.environments.office_world.config_office import config as ow_config  # noqa: E402
from multiagent_rlrm.environments.office_world.config_office import get_experiment_for_map  # noqa: E402
from multiagent_rlrm.multi_agent.agent_rl import AgentRL  # noqa: E402
from multiagent_rlrm.multi_agent.action_rl import ActionRL  # noqa: E402
from multiagent_rlrm.multi_agent.reward_machine import RewardMachine  # noqa: E402
from multiagent_rlrm.multi_agent.wrappers.rm_environment_wrapper import RMEnvironmentWrapper  # noqa: E402
from multiagent_rlrm.utils.utils import parse_map_emoji, parse_office_world  # noqa: E402
from multiagent_rlrm.environments.frozen_lake.state_encoder_frozen_lake import StateEncoderFrozenLake  # noqa: E402
from multiagent_rlrm.environments.frozen_lake.action_encoder_frozen_lake import ActionEncoderFrozenLake  # noqa: E402
from multiagent_rlrm.environments.office_world.state_encoder_office import StateEncoderOfficeWorld  # noqa: E402
from multiagent_rlrm.environments.office_world.action_encoder_office_world import ActionEncoderOfficeWorld  # noqa: E402


class _QRMLearner:
    """Stand-in learner exposing only the flag the wrapper reads (rm_environment_wrapper.py:78)."""
    use_qrm = True

ACTION_NAMES = ["up", "down", "left", "right"]
M64 = (1 << 64) - 1
GOLDEN_RATIO = 0x9E3779B97F4A7C15


def _spec_dict(name, states_order=None):
    with open(os.path.join(HERE, "specs", f"{name}.json")) as f:
        d = json.load(f)
    if states_order:
        d["states"] = list(states_order)
    return d




def splitmix64(x):
    z = (x + GOLDEN_RATIO) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def hash_action(seed, t, n_global, e, n_agents, i):
    """SURVEY.md §8(d) synthetic-action hash (restated in rmx/actions.py)."""
    ctr = (((t * n_global + e) * n_agents + i) * GOLDEN_RATIO) & M64
    return splitmix64((seed ^ ctr) & M64) >> 62


# ---------------------------------------------------------------------------
# Scenario descriptions.  Events are symbolic: FrozenLake goal letters; for
# OfficeWorld goal letters plus coffee0/coffee1/letter0 (config_office.py exps).
# ---------------------------------------------------------------------------
FL_ABC = [["state0", "A", "state1", 10], ["state1", "B", "state2", 15], ["state2", "C", "state3", 20]]
OW_ACBD = [["state0", "A", "state1", 0], ["state1", "C", "state2", 0],
           ["state2", "B", "state3", 0], ["state3", "D", "state4", 1]]
# exp5 in insertion order of config_office.py:363-388
OW_EXP5 = [["state0", "A", "state1", 0], ["state1", "B", "state2", 0], ["state2", "C", "state3", 0],
           ["state3", "D", "state4", 0], ["state4", "coffee0", "state5", 0], ["state4", "coffee1", "state5", 0],
           ["state4", "letter0", "state6", 0], ["state6", "coffee0", "state7", 0], ["state6", "coffee1", "state7", 0],
           ["state5", "letter0", "state7", 0], ["state7", "O", "state8", 1]]
# None-event self loop with a fractional reward, and a rewarding self loop on the
# final state's own event cell: pins "RM stepped for every agent, frozen or not".
FL_SELFLOOP = [["state0", "A", "state1", 10], ["state0", None, "state0", -0.25], ["state1", "A", "state1", 1]]
# completed-spec quirks (reward_machine.py:152-163): final = to_state of the LAST inserted row
FL_INIT_IS_FINAL = [["q0", "A", "q1", 1], ["q1", "B", "q0", 0]]
FL_FINAL_NOT_TERMINAL = [["q2", "A", "q0", 0], ["q0", "B", "q1", 1], ["q1", "C", "q2", 0], ["q1", None, "q1", 0.5]]
FL_ZIGZAG = [[f"s{k}", "A" if k % 2 == 0 else "B", f"s{k + 1}", float(k + 1)] for k in range(8)]
FL_AB = [["s0", "A", "s1", 1], ["s1", "B", "s2", 3]]
OPEN_LAKE = """
A 🟩 🟩 🟩 🟩 🟩
🟩 🟩 🟩 🟩 🟩 🟩
🟩 🟩 🟩 🟩 🟩 🟩
🟩 🟩 🟩 🟩 🟩 🟩
🟩 🟩 🟩 🟩 🟩 B
"""
FL_CBA = [["q0", "C", "q1", 1], ["q1", "B", "q2", 2], ["q2", "A", "q3", 4]]
OW_SHORT0 = [["state0", "coffee0", "state1", 1]]
OW_SHORT1 = [["state0", "letter0", "state1", 0], ["state1", "O", "state2", 5]]

CONFIGS = {
    "fl2": {"kind": "frozen_lake", "map": "map1", "penalty": 0.0,
            "agents": [{"start": [5, 0], "rm": FL_ABC}, {"start": [0, 0], "rm": FL_ABC}]},
    "fl4": {"kind": "frozen_lake", "map": "map1", "penalty": 0.0,
            "agents": [{"start": [5, 0], "rm": FL_ABC}, {"start": [0, 0], "rm": FL_ABC},
                       {"start": [9, 0], "rm": FL_ABC}, {"start": [9, 9], "rm": FL_ABC}]},
    "fl2_quirks": {"kind": "frozen_lake", "map": "map1", "penalty": -1.0,
                   "agents": [{"start": [4, 3], "rm": FL_SELFLOOP}, {"start": [4, 9], "rm": FL_CBA}]},
    "fl2_initfinal": {"kind": "frozen_lake", "map": "map1", "penalty": 0.0,
                      "agents": [{"start": [1, 1], "rm": FL_INIT_IS_FINAL}, {"start": [1, 0], "rm": FL_FINAL_NOT_TERMINAL}]},
    "fl2_finalnt": {"kind": "frozen_lake", "map": "map1", "penalty": 0.0,
                    "agents": [{"start": [1, 0], "rm": FL_FINAL_NOT_TERMINAL}, {"start": [4, 3], "rm": FL_ABC}]},
    "fl2_open": {"kind": "frozen_lake", "layout": OPEN_LAKE, "penalty": 0.0,
                 "agents": [{"start": [2, 2], "rm": FL_ZIGZAG}, {"start": [3, 1], "rm": FL_AB}]},
    "ow1_map3": {"kind": "office_world", "map": "map3", "plants_penalty": -100.0, "wall_penalty": -2.0,
                 "terminate_on_plants": False, "terminate_hit_walls": False, "gamma": 0.95,
                 "agents": [{"start": [2, 7], "rm": OW_ACBD}]},
    "ow1": {"kind": "office_world", "map": "map1", "plants_penalty": -100.0, "wall_penalty": 0.0,
            "terminate_on_plants": False, "terminate_hit_walls": False, "gamma": 0.9,
            "agents": [{"start": [2, 7], "rm": OW_ACBD}]},
    "ow3": {"kind": "office_world", "map": "map1", "plants_penalty": -100.0, "wall_penalty": 0.0,
            "terminate_on_plants": False, "terminate_hit_walls": False, "gamma": 0.9, "shaping_gamma": 0.9,
            "agents": [{"start": [2, 7], "rm": OW_EXP5}, {"start": [0, 0], "rm": OW_EXP5},
                       {"start": [11, 8], "rm": OW_EXP5}]},
    "ow2_final": {"kind": "office_world", "map": "map1", "plants_penalty": -100.0, "wall_penalty": 0.0,
                  "terminate_on_plants": False, "terminate_hit_walls": False, "gamma": 0.9,
                  "agents": [{"start": [3, 1], "rm": OW_SHORT0}, {"start": [6, 4], "rm": OW_SHORT1}]},
    "ow2_fail": {"kind": "office_world", "map": "map1", "plants_penalty": -100.0, "wall_penalty": -1.0,
                 "terminate_on_plants": True, "terminate_hit_walls": True, "gamma": 0.9,
                 "agents": [{"start": [2, 7], "rm": OW_ACBD}, {"start": [5, 1], "rm": OW_SHORT1}]},
}

# --rm-spec scenarios: the reference's own fixture specs, completed under two `states` orders (the
# completion order decides the "final" state: [q2, q0, q1] makes q1 "final").
CONFIGS["fl2_spec"] = {"kind": "frozen_lake", "map": "map1", "penalty": 0.0, "agents": [
    {"start": [4, 3], "rm_spec": {"spec": _spec_dict("frozenlake_linear"), "complete": True, "default_reward": 0.0}},
    {"start": [1, 0], "rm_spec": {"spec": _spec_dict("frozenlake_linear", ["q2", "q0", "q1"]), "complete": True,
                                  "default_reward": -0.5, "terminal_reward_must_be_zero": False}}]}
CONFIGS["ow2_spec"] = {"kind": "office_world", "map": "map1", "plants_penalty": -100.0, "wall_penalty": 0.0,
                       "terminate_on_plants": False, "terminate_hit_walls": False, "gamma": 0.9, "agents": [
    {"start": [2, 7], "rm_spec": {"spec": {"name": "ow_coffee_office", "env_id": "officeworld", "version": "1.0",
                                           "states": ["q0", "q1", "q2"], "initial_state": "q0",
                                           "terminal_states": ["q2"], "event_vocabulary": ["coffee", "at(O)", "email"],
                                           "transitions": [
                                               {"from_state": "q0", "event": "coffee", "to_state": "q1", "reward": 0},
                                               {"from_state": "q1", "event": "at(O)", "to_state": "q2", "reward": "r1"}]},
                                  "complete": True}},
    {"start": [8, 5], "rm_spec": {"spec": _spec_dict("officeworld_simple") | {
        "event_vocabulary": ["at(A)", "at(B)", "at(D)"],
        "transitions": [{"from_state": "q0", "event": "at(A)", "to_state": "q1", "reward": 0.0},
                        {"from_state": "q1", "event": "at(D)", "to_state": "q2", "reward": 1.0}]},
        "complete": False}}]}

# stochastic slip scenarios (ma_frozen_lake.py:244-298, ma_office.py:327-379)
CONFIGS["fl2_slip"] = dict(CONFIGS["fl2"], stochastic=True)
CONFIGS["fl2_delay"] = dict(CONFIGS["fl2_quirks"], stochastic=True, delay_action=True)
CONFIGS["ow1_slip"] = dict(CONFIGS["ow1"], stochastic=True)
CONFIGS["ow2_allslip"] = dict(CONFIGS["ow2_final"], stochastic=True, all_slip=True, high_prob=0.9, wall_penalty=-1.0)
CONFIGS["ow2_delay"] = dict(CONFIGS["ow2_fail"], stochastic=True, delay_action=True, terminate_hit_walls=False)
CONFIGS["ow3_slip"] = dict(CONFIGS["ow3"], stochastic=True, seed_schedule=[7, 3, 11])
# FrozenLake random_start_positions (ma_frozen_lake.py:37-39, 59-64, 156-172): the shuffle of the free cells
# consumes the freshly seeded env rng before any slip draw of the episode
CONFIGS["fl2_randstart"] = dict(CONFIGS["fl2"], random_start_positions=True)
CONFIGS["fl2_randstart_slip"] = dict(CONFIGS["fl2_quirks"], stochastic=True, random_start_positions=True,
                                     seed_schedule=[5, 7, 3])
CONFIGS["fl4_randstart_open"] = dict(CONFIGS["fl2_open"], random_start_positions=True, seed_schedule=[1, 1, 1],
                                     agents=CONFIGS["fl2_open"]["agents"] + CONFIGS["fl2_open"]["agents"])

TRAJ = {  # cfg -> (n_envs, n_steps, seed)
    "fl2": (32, 1100, 0), "fl4": (16, 1100, 1), "fl2_quirks": (32, 1100, 2), "fl2_initfinal": (8, 300, 4),
    "fl2_finalnt": (16, 1100, 5), "fl2_open": (16, 2500, 6), "ow1_map3": (8, 1100, 8), "fl2_spec": (32, 1100, 9),
    "ow2_spec": (12, 1100, 10), "fl2_slip": (32, 1100, 11), "fl2_delay": (32, 1100, 12), "ow1_slip": (12, 1100, 13),
    "ow2_allslip": (12, 1100, 14), "ow2_delay": (24, 800, 15), "ow3_slip": (8, 1100, 16),
    "fl2_randstart": (32, 1100, 17), "fl2_randstart_slip": (32, 1100, 18), "fl4_randstart_open": (16, 1100, 19),
    "ow1": (16, 1100, 0), "ow3": (12, 1100, 1), "ow2_final": (16, 1100, 2), "ow2_fail": (32, 600, 3),
}
EPISODES = {"fl2": (256, 2000, 7), "ow1": (32, 2200, 7)}


def resolve_events(cfg):
    """Symbol -> position map for a scenario, using the REFERENCE parsers."""
    if cfg["kind"] == "frozen_lake":
        holes, goals, dims = parse_map_emoji(cfg.get("layout") or fl_config["maps"][cfg["map"]]["layout"])
        sym = dict(goals)
        return sym, {"holes": holes, "goals": goals, "dims": dims}
    layout = ow_config["maps"][cfg["map"]]["layout"]
    coords, goals, walls = parse_office_world(layout)
    sym = dict(goals)
    for k in ("coffee", "letter"):
        for j, p in enumerate(coords[k]):
            sym[f"{k}{j}"] = p
    return sym, {"coords": coords, "goals": goals, "walls": walls}


def build_rm_from_spec(rs, cfg, detector):
    """The --rm-spec path of the runners: compile_reward_machine with the env's event mapping."""
    from multiagent_rlrm.rmgen.io import compile_reward_machine
    from multiagent_rlrm.rmgen.spec import RMSpec
    _, parsed = resolve_events(cfg)
    mapping = {}
    for label, pos in parsed["goals"].items():  # frozen_lake_main.py:125-130 / office_main.py:461-466
        mapping[f"at({label})"] = pos
        mapping[label] = pos
    if cfg["kind"] == "office_world":  # office_main.py:467-485
        coords = parsed["coords"]
        if "O" in parsed["goals"]:
            mapping["office"] = mapping["at(office)"] = parsed["goals"]["O"]
        if coords.get("coffee"):
            mapping["coffee"] = list(coords["coffee"])
            mapping["at(coffee)"] = list(coords["coffee"])
        if coords.get("letter"):
            for k in ("letter", "email", "at(letter)", "at(email)"):
                mapping[k] = list(coords["letter"])
    return compile_reward_machine(RMSpec.from_dict(json.loads(json.dumps(rs["spec"]))), event_detector=detector,
                                  event_mapping=mapping, complete_missing_transitions=rs.get("complete", False),
                                  default_reward=rs.get("default_reward", 0.0),
                                  terminal_self_loop=rs.get("terminal_self_loop", True),
                                  terminal_reward_must_be_zero=rs.get("terminal_reward_must_be_zero", True))


def build_rm(rows, sym, detector):
    trans = {}
    for fr, ev, to, r in rows:
        key_ev = None if ev is None else sym[ev]
        trans[(fr, key_ev)] = (to, r)
    return RewardMachine(trans, detector)


def make_env(cfg):
    sym, parsed = resolve_events(cfg)
    if cfg["kind"] == "frozen_lake":
        holes, goals, (w, h) = parsed["holes"], parsed["goals"], parsed["dims"]
        env = MultiAgentFrozenLake(width=w, height=h, holes=holes)  # frozen_lake_main.py:207-214
        env.frozen_lake_stochastic = bool(cfg.get("stochastic", False))
        env.penalty_amount = cfg["penalty"]
        env.delay_action = bool(cfg.get("delay_action", False))
        env.random_start_positions = bool(cfg.get("random_start_positions", False))
        detector = PositionEventDetector(set(goals.values()))  # frozen_lake_main.py:226
    else:
        mc = ow_config["maps"][cfg["map"]]
        coords, goals, walls = parse_office_world(mc["layout"])
        walls = walls + [(b, a) for (a, b) in walls]  # office_main.py:416
        env = MultiAgentOfficeWorld(
            width=mc["grid_size"][1], height=mc["grid_size"][0],
            plants=coords["plant"], coffee=coords["coffee"], letters=coords["letter"], walls=walls,
            plants_penalty_value=cfg["plants_penalty"], wall_penalty_value=cfg["wall_penalty"],
            terminate_on_plants=cfg["terminate_on_plants"], terminate_hit_walls=cfg["terminate_hit_walls"])
        env.stochastic = bool(cfg.get("stochastic", False))
        env.all_slip = bool(cfg.get("all_slip", False))
        env.high_prob = cfg.get("high_prob", 0.8)
        env.delay_action = bool(cfg.get("delay_action", False))
        det_pos = set(mc["position_map"](coords, goals))  # office_main.py:414,438
        if any("rm_spec" in ac for ac in cfg["agents"]):  # office_main.py:487-495
            det_pos |= set(goals.values()) | set(coords["coffee"]) | set(coords["letter"])
        detector = PositionEventDetector(det_pos)
    agents = []
    for i, ac in enumerate(cfg["agents"]):
        ag = AgentRL(f"a{i + 1}", env)
        ag.set_initial_position(*ac["start"])
        if cfg["kind"] == "frozen_lake":
            ag.add_state_encoder(StateEncoderFrozenLake(ag))
            ag.add_action_encoder(ActionEncoderFrozenLake(ag))
        else:
            ag.add_state_encoder(StateEncoderOfficeWorld(ag))
            ag.add_action_encoder(ActionEncoderOfficeWorld(ag))
        ag.set_learning_algorithm(_QRMLearner())  # the wrapper then emits infos["qrm_experience"]
        rm = build_rm_from_spec(ac["rm_spec"], cfg, detector) if "rm_spec" in ac else build_rm(ac["rm"], sym, detector)
        if "shaping_gamma" in cfg:
            with contextlib.redirect_stdout(io.StringIO()):
                rm.add_reward_shaping(cfg["shaping_gamma"], cfg["shaping_gamma"])  # office_main.py:543-545
        ag.set_reward_machine(rm)
        env.add_agent(ag)
        agents.append(ag)
    return RMEnvironmentWrapper(env, agents), agents, detector


def seed_for(cfg, base, e, k):
    """Reset seed of env e's k-th episode: base*scale + e*env_stride + k*episode_stride (mod 2^64).
    Defaults follow the runners: FrozenLake reset(args.seed) every episode (+ env offset for the batch),
    OfficeWorld reset(seed*1000 + episode) (frozen_lake_main.py:337, office_main.py:1699)."""
    scale, es, ks = cfg.get("seed_schedule") or ((1, 1, 0) if cfg["kind"] == "frozen_lake" else (1000, 1000, 1))
    return (base * scale + e * es + k * ks) & M64


def run(cfg_name, n_envs, n_steps, seed, record_traj=True):
    cfg = CONFIGS[cfg_name]
    A = len(cfg["agents"])
    ow = cfg["kind"] == "office_world"
    gamma = cfg.get("gamma", 1.0)
    acts = np.zeros((n_steps, A, n_envs), np.int8)
    out = {k: np.zeros((n_steps, A, n_envs), dt) for k, dt in [
        ("pos_x", np.int8), ("pos_y", np.int8), ("q", np.int8), ("reward", np.float64), ("shaping", np.float64),
        ("renv", np.float64), ("rq", np.float64), ("term", np.bool_), ("trunc", np.bool_), ("active", np.bool_)]}
    env_done = np.zeros((n_steps, n_envs), np.bool_)
    # positions right after each reset (-1 where no reset preceded the step): pins random start positions
    reset_xy = np.full((n_steps, 2, A, n_envs), -1, np.int8)
    tcol = np.zeros((n_steps, n_envs), np.int16)
    probe, _, _ = make_env(cfg)
    QX = max(len(ag.get_reward_machine().get_all_states()) - 1 for ag in probe.agents)
    # QRM experience tuples (rm_environment_wrapper.py:168-179): enc_s, a, r, enc_sn, done, s, q, sn, qn, hr
    qrm = {k: np.full((n_steps, A, max(QX, 1), n_envs), -1 if dt != np.float64 else np.nan, dt) for k, dt in [
        ("qrm_s", np.int32), ("qrm_a", np.int32), ("qrm_r", np.float64), ("qrm_sn", np.int32), ("qrm_done", np.int8),
        ("qrm_pos", np.int32), ("qrm_q", np.int32), ("qrm_npos", np.int32), ("qrm_nq", np.int32),
        ("qrm_hr", np.float64)]}
    ep = {k: [] for k in ("env", "agent", "ret", "length", "success", "final_q", "end_step")}
    for e in range(n_envs):
        rm_env, agents, _ = make_env(cfg)
        env = rm_env.env
        need_reset = True
        ret = [0.0] * A
        cum_gamma = 1.0
        episode = 0
        for t in range(n_steps):
            if need_reset:
                rm_env.reset(seed_for(cfg, seed, e, episode))
                for i, ag in enumerate(agents):
                    reset_xy[t, 0, i, e], reset_xy[t, 1, i, e] = ag.state["pos_x"], ag.state["pos_y"]
                ret = [0.0] * A
                cum_gamma = 1.0
                need_reset = False
            actions = {}
            for i, ag in enumerate(agents):
                a = hash_action(seed, t, n_envs, e, A, i)
                acts[t, i, e] = a
                actions[ag.name] = ag.actions_dix()[a]  # the agent's own ActionRL (actions_idx identity)
            prev_labels = [ag.get_reward_machine().get_current_state() for ag in agents]
            obs, rewards, terms, truncs, infos = rm_env.step(actions)
            for i, ag in enumerate(agents):
                rm = ag.get_reward_machine()
                out["pos_x"][t, i, e] = obs[ag.name]["pos_x"]
                out["pos_y"][t, i, e] = obs[ag.name]["pos_y"]
                out["q"][t, i, e] = rm.get_state_index(rm.get_current_state())
                out["reward"][t, i, e] = rewards[ag.name]
                out["renv"][t, i, e] = infos[ag.name].get("Renv", 0)
                out["rq"][t, i, e] = infos[ag.name]["RQ"]
                out["term"][t, i, e] = bool(terms[ag.name])
                out["trunc"][t, i, e] = bool(truncs[ag.name])
                out["active"][t, i, e] = bool(env.active_agents[ag.name])
                for j, x in enumerate(infos[ag.name].get("qrm_experience", [])):
                    for f, key in enumerate(("qrm_s", "qrm_a", "qrm_r", "qrm_sn", "qrm_done", "qrm_pos", "qrm_q",
                                             "qrm_npos", "qrm_nq", "qrm_hr")):
                        qrm[key][t, i, j, e] = x[f]
                if rm.potentials is not None:  # qlearning.py:60-65 formula on labels
                    g = cfg["shaping_gamma"]
                    out["shaping"][t, i, e] = g * rm.potentials.get(rm.get_current_state(), 0) - \
                        rm.potentials.get(prev_labels[i], 0)
                ret[i] += (cum_gamma if ow else 1.0) * rewards[ag.name]
            tcol[t, e] = env.timestep
            if ow:
                cum_gamma *= gamma
            done = all(terms.values()) or all(truncs.values())
            env_done[t, e] = done
            if done:
                for i, ag in enumerate(agents):
                    rm = ag.get_reward_machine()
                    succ = bool(terms[ag.name]) and rm.get_current_state() == rm.get_final_state() and ret[i] > 0
                    ep["env"].append(e); ep["agent"].append(i); ep["ret"].append(ret[i])
                    ep["length"].append(env.timestep); ep["success"].append(succ)
                    ep["final_q"].append(rm.get_state_index(rm.get_current_state())); ep["end_step"].append(t)
                need_reset = True
                episode += 1
    ep = {k: np.asarray(v) for k, v in ep.items()}
    out.update(qrm)
    out["reset_xy"] = reset_xy
    return acts, out, env_done, tcol, ep


def spec_fixture():
    """compile_reward_machine on the reference's fixture specs: map, indices, initial, final; errors."""
    from multiagent_rlrm.rmgen.io import compile_reward_machine, load_rmspec
    from multiagent_rlrm.rmgen.validator import ValidationError
    out = {}
    cases = [("frozenlake_linear", None, False, 0.0, True), ("frozenlake_linear", None, True, 0.0, True),
             ("frozenlake_linear", ["q2", "q0", "q1"], True, 0.0, True),
             ("frozenlake_linear", ["q1", "q2", "q0"], True, 0.25, False),
             ("officeworld_simple", None, False, 0.0, True), ("officeworld_simple", None, True, 0.0, True),
             ("warehouse_pickup_delivery", None, False, 0.0, True),
             ("warehouse_pickup_delivery", None, True, 0.0, True),
             ("nondeterministic_rm", None, False, 0.0, True), ("invalid_schema_rm", None, False, 0.0, True)]
    for name, order, complete, dr, tsl in cases:
        key = f"{name}|{','.join(order) if order else '-'}|{int(complete)}|{dr}|{int(tsl)}"
        spec = load_rmspec(os.path.join(HERE, "specs", f"{name}.json"))
        if order:
            spec.states = list(order)
        try:
            rm = compile_reward_machine(spec, complete_missing_transitions=complete, default_reward=dr,
                                        terminal_self_loop=tsl, terminal_reward_must_be_zero=False)
            out[key] = {"rows": [[k[0], k[1], v[0], v[1]] for k, v in rm.transitions.items()],
                        "state_indices": rm.state_indices, "initial": rm.initial_state,
                        "final": rm.get_final_state(), "numbers_state": rm.numbers_state(),
                        "all_states": rm.get_all_states()}
        except (ValidationError, ValueError) as exc:
            out[key] = {"error": type(exc).__name__}
    return out


def tables_fixture():
    tab = {}
    # map parses
    holes, goals, dims = parse_map_emoji(fl_config["maps"]["map1"]["layout"])
    tab["fl_map1"] = {"holes": holes, "goals": goals, "dims": dims}
    for m in ("map0", "map1", "map2", "map3", "map4"):
        mc = ow_config["maps"][m]
        coords, goals, walls = parse_office_world(mc["layout"])
        tab[f"ow_{m}"] = {"coords": coords, "goals": goals, "walls": walls, "grid_size": mc["grid_size"],
                          "position_map": sorted(mc["position_map"](coords, goals))}
        tab[f"ow_{m}_experiments"] = {}
        for x in ("exp0", "exp0_simply", "exp1", "exp2", "exp3", "exp4", "exp5", "exp6", "exp7"):
            ex = get_experiment_for_map(m, x)
            tab[f"ow_{m}_experiments"][x] = [[k[0], list(k[1]), v[0], v[1]] for k, v in ex["transitions"].items()]
    # RM indexing / final / potentials for every scenario RM and some quirky dicts
    rms = {"fl_abc": FL_ABC, "ow_acbd": OW_ACBD, "ow_exp5": OW_EXP5, "fl_selfloop": FL_SELFLOOP,
           "fl_cba": FL_CBA, "ow_short1": OW_SHORT1,
           "sorted_quirk": [["s0", "A", "s10", 1], ["s10", "B", "s2", 2], ["s2", "C", "s1", 3]],
           "final_not_terminal": [["q2", "A", "q0", 0], ["q0", "B", "q1", 1], ["q1", "C", "q2", 0],
                                  ["q1", None, "q1", 0]],
           "initial_is_final": [["q0", "A", "q1", 1], ["q1", "B", "q0", 0]]}
    sym = {k: (i, 100 + i) for i, k in enumerate("ABCDEO")}
    sym.update({"coffee0": (50, 1), "coffee1": (50, 2), "letter0": (50, 3)})
    tab["rmspec"] = spec_fixture()
    tab["rm"] = {}
    for name, rows in rms.items():
        rm = build_rm(rows, sym, None)
        with contextlib.redirect_stdout(io.StringIO()):
            rm.add_reward_shaping(0.9, 0.9)
        pots = dict(rm.potentials)
        rm2 = build_rm(rows, sym, None)
        rm2.add_distance_reward_shaping(0.9, 0.9, alpha=100)
        tab["rm"][name] = {"rows": rows, "state_indices": rm.state_indices, "final": rm.get_final_state(),
                           "initial": rm.initial_state, "numbers_state": rm.numbers_state(),
                           "all_states": rm.get_all_states(), "potentials": pots,
                           "distance_potentials": rm2.potentials}
    return tab


MDP_CONFIGS = ["fl2", "fl2_quirks", "ow1", "ow3", "ow2_fail", "ow2_final", "ow1_map3", "fl2_spec", "ow2_spec"]


def mdp_fixture(name):
    """RMEnvironmentWrapper.get_mdp (rm_environment_wrapper.py:185-283) as dense arrays per agent:
    next[S][4] (-1: no entry), reward[S][4], done[S][4]; every reference entry is a single outcome."""
    cfg = CONFIGS[name]
    rm_env, agents, _ = make_env(cfg)
    with contextlib.redirect_stdout(io.StringIO()):
        P, ns, na = rm_env.get_mdp(seed=0)
    out = {}
    for i, ag in enumerate(agents):
        S, Na = ns[ag.name], na[ag.name]
        nxt = np.full((S, Na), -1, np.int32)
        rew = np.zeros((S, Na), np.float64)
        done = np.zeros((S, Na), np.int8)
        for s_ in range(S):
            for a in range(Na):
                ent = P[ag.name][s_][a]
                assert len(ent) <= 1, "deterministic dynamics give at most one outcome"
                if ent:
                    prob, sn, r, d = ent[0]
                    assert prob == 1.0
                    nxt[s_, a], rew[s_, a], done[s_, a] = sn, r, int(bool(d))
        out[f"a{i}_next"], out[f"a{i}_reward"], out[f"a{i}_done"] = nxt, rew, done
    return out


def _jsonable(o):
    if isinstance(o, dict):
        return {str(k): _jsonable(v) for k, v in o.items()}
    if isinstance(o, (list, tuple)):
        return [_jsonable(v) for v in o]
    if isinstance(o, (np.integer,)):
        return int(o)
    if isinstance(o, (np.floating,)):
        return float(o)
    return o


def _savez(path, **arrays):
    """np.savez_compressed with a fixed entry timestamp and order, so a re-run reproduces every fixture byte for byte
    (numpy's own writer stamps each entry with the current time).  np.load reads it as any .npz."""
    import zipfile
    with zipfile.ZipFile(path, "w", compression=zipfile.ZIP_DEFLATED) as z:
        for name, arr in arrays.items():
            buf = io.BytesIO()
            np.lib.format.write_array(buf, np.asanyarray(arr), allow_pickle=False)
            info = zipfile.ZipInfo(name + ".npy", date_time=(1980, 1, 1, 0, 0, 0))
            info.compress_type = zipfile.ZIP_DEFLATED
            info.external_attr = 0o600 << 16
            z.writestr(info, buf.getvalue(), compresslevel=6)


def main(only=None):
    """Regenerate every fixture, or with names on the command line only those trajectories (configs.json is
    always rewritten: it is the scenario list)."""
    with open(os.path.join(HERE, "configs.json"), "w") as f:
        json.dump(CONFIGS, f, indent=1)
    if only:
        for name in only:
            n, T, seed = TRAJ[name]
            acts, out, env_done, tcol, _ = run(name, n, T, seed)
            _savez(os.path.join(HERE, f"traj_{name}.npz"), actions=acts, env_done=env_done, t=tcol,
                                seed=np.int64(seed), **out)
            print(name, "episodes done:", int(env_done.sum()))
        return
    with open(os.path.join(HERE, "tables.json"), "w") as f:
        json.dump(_jsonable(tables_fixture()), f, indent=0)
    for name, (n, T, seed) in TRAJ.items():
        acts, out, env_done, tcol, _ = run(name, n, T, seed)
        _savez(os.path.join(HERE, f"traj_{name}.npz"), actions=acts, env_done=env_done, t=tcol,
                            seed=np.int64(seed), **out)
        print(name, "episodes done:", int(env_done.sum()))
    for name in MDP_CONFIGS:
        _savez(os.path.join(HERE, f"mdp_{name}.npz"), **mdp_fixture(name))
        print(name, "mdp recorded")
    for name, (n, T, seed) in EPISODES.items():
        _, _, _, _, ep = run(name, n, T, seed)
        _savez(os.path.join(HERE, f"episodes_{name}.npz"), n_envs=np.int64(n), n_steps=np.int64(T),
                            seed=np.int64(seed), **ep)
        print(name, "episode records:", len(ep["ret"]))


if __name__ == "__main__":
    main(sys.argv[1:])
