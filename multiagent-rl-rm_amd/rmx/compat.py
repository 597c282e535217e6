"""Reference-shaped dict API over the GPU engine — the drop-in for code written against
multiagent_rlrm's ``RMEnvironmentWrapper`` (rm_environment_wrapper.py:4-120).

``RMEnvironmentWrapper(env, agents)`` accepts either the configuration classes below or the
reference's own objects (duck-typed: ``env.holes`` / ``env.plants`` + ``env.walls``,
``agent.initial_position``, ``agent.get_reward_machine().transitions`` and
``.event_detector.positions``).  ``reset(seed)`` / ``step(actions)`` / ``check_terminations()`` return
the reference's five dicts and info keys; each call runs ONE environment (N = 1) through the engine's C ABI:
``device=<ordinal>`` the resident gfx950 workgroup behind rmx_step_sync (the same rules as the batched
``VecRMEnv``), ``device="cpu"`` a host handle (csrc/rmx_hoststep.cpp: the engine's CPU path over the same compiled
tables, no GPU and no PCIe round trip per call — the reference's own config, BASELINE config 1), and the default
``device=None`` the GPU when one is visible, else the host handle.  After every step the agent positions, RM labels
and the env's ``active_agents`` / ``agent_fail`` / ``agent_steps`` / ``timestep`` mirrors are updated so
reference-style loops (frozen_lake_main.py:336-376, office_main.py:1696-1749) run unchanged.

The configuration classes only hold what the reference constructors take; stepping happens in the engine,
including the stochastic slip dynamics (ma_frozen_lake.py:244-298, ma_office.py:327-379) with the env rng reseeded
by every reset(seed) exactly like numpy's default_rng(seed).
"""
from __future__ import annotations

import ctypes as C
import struct
from typing import Dict, List

import numpy as np

from . import _capi
from .tables import FROZEN_LAKE, OFFICE_WORLD, RewardMachineSpec, compile_tables

ACTION_INDEX = {"up": 0, "down": 1, "left": 2, "right": 3, "wait": 4}
MAX_T = 1000  # ma_frozen_lake.py:202 / ma_office.py:254 hard-code 1000


class ActionRL:
    """Symbolic action (action_rl.py:1-28): only the name matters to the grid dynamics."""

    def __init__(self, name, preconditions=None, effects=None):
        self.name = name
        self.preconditions = preconditions or []
        self.effects = effects or []


class PositionEventDetector:
    """Configuration of the position detector (detect_event.py:4-16): the set of event cells."""

    def __init__(self, positions):
        self.positions = positions


class RewardMachine(RewardMachineSpec):
    """RewardMachine(transitions, event_detector) (reward_machine.py:5-18): structure + current label.
    The transition itself is taken on the GPU by the wrapper's step."""

    def __init__(self, transitions, event_detector):
        super().__init__(transitions)
        self.event_detector = event_detector
        self.current_state = self.initial_state

    def get_current_state(self):
        return self.current_state

    def reset_to_initial_state(self):
        self.current_state = self.initial_state
        return self.initial_state


class AgentRL:
    """The position / RM plumbing of AgentRL (agent_rl.py:11-42, 229-235, 340-384)."""

    def __init__(self, name, ma_problem=None, reward_machine=None):
        self.name = name
        self.ma_problem = ma_problem
        self.reward_machine = reward_machine
        self.position = None
        self.initial_position = None
        self.state: Dict = {}
        self.actions_: List[ActionRL] = []

    def set_initial_position(self, x, y):
        self.initial_position = (x, y)
        self.set_position(x, y)

    def set_position(self, x, y):
        self.position = (x, y)
        self.state = {"pos_x": x, "pos_y": y}

    def get_position(self):
        return self.position

    def get_state(self):
        return self.state

    def set_reward_machine(self, rm):
        self.reward_machine = rm

    def get_reward_machine(self):
        return self.reward_machine

    def set_learning_algorithm(self, algorithm):
        self.learning_algorithm = algorithm

    def get_learning_algorithm(self):
        return getattr(self, "learning_algorithm", None)

    def add_action(self, action):
        self.actions_.append(action)

    def get_actions(self):
        return self.actions_


class _GridEnv:
    def __init__(self, width, height):
        self.grid_width = width
        self.grid_height = height
        self.map_width = width
        self.map_height = height
        self._agents: List = []
        self.active_agents: Dict = {}
        self.agent_fail: Dict = {}
        self.agent_steps: Dict = {}
        self.timestep = 0

    @property
    def agents(self):
        return self._agents

    def add_agent(self, agent):
        if any(a.name == agent.name for a in self._agents):
            raise ValueError(f"duplicate agent {agent.name}")
        self._agents.append(agent)


class MultiAgentFrozenLake(_GridEnv):
    """Configuration mirror of MultiAgentFrozenLake(width, height, holes) (ma_frozen_lake.py:12-41)."""

    def __init__(self, width, height, holes):
        super().__init__(width, height)
        self.holes = holes
        self.penalty_amount = 0
        self.frozen_lake_stochastic = False
        self.delay_action = False
        self.random_start_positions = False  # ma_frozen_lake.py:37-39: agents start in random free cells


class MultiAgentOfficeWorld(_GridEnv):
    """Configuration mirror of MultiAgentOfficeWorld(...) (ma_office.py:20-75)."""

    def __init__(self, width, height, plants, coffee, letters, walls, plants_penalty_value, wall_penalty_value,
                 terminate_on_plants, terminate_hit_walls, all_slip=False):
        super().__init__(width, height)
        self.plants, self.coffee, self.letters, self.walls = plants, coffee, letters, walls
        self.plants_penalty_value = plants_penalty_value
        self.wall_penalty_value = wall_penalty_value
        self.terminate_on_plants = terminate_on_plants
        self.terminate_hit_walls = terminate_hit_walls
        self.all_slip = all_slip
        self.stochastic = False
        self.delay_action = False


# Dynamics switches of the reference envs.  Each env class reads only its own (a FrozenLake ignores an
# OfficeWorld switch set on it, and vice versa, exactly as the reference classes do); any other switch that
# is set (truthy) is refused rather than ignored, since a silently different dynamics would void parity.
_FL_FLAGS = ("frozen_lake_stochastic", "delay_action", "random_start_positions", "penalty_amount")
_OW_FLAGS = ("stochastic", "delay_action", "all_slip", "high_prob", "terminate_on_plants", "terminate_hit_walls",
             "plants_penalty_value", "wall_penalty_value")
# attributes of the reference envs that carry no dynamics (bookkeeping / rng / unused: epsilon is never read)
_INERT = {"grid_width", "grid_height", "map_width", "map_height", "holes", "plants", "coffee", "letters", "walls",
          "wait_action", "possible_actions", "rewards", "active_agents", "agent_fail", "agent_steps", "timestep",
          "epsilon", "rng", "_agents", "agents"}


def _check_modelled(env):
    """Raise for a set (truthy) boolean / numeric switch on the env that no reference env class reads."""
    for k, v in vars(env).items():
        if k in _FL_FLAGS or k in _OW_FLAGS or k in _INERT or k.startswith("_") or callable(v):
            continue
        if isinstance(v, (bool, int, float)) and v:
            raise NotImplementedError(f"env attribute {k!r} = {v!r} is not modelled by the rmx engine")


def tables_from_objects(env, agents, reward_modifier=1.0):
    """Compile the dense tables from reference-shaped env / agent / RM objects.  Stochastic slip and random
    start positions read the env's own flags (frozen_lake_stochastic / stochastic, delay_action, all_slip,
    high_prob, random_start_positions); each reset(seed) reseeds the env rng exactly like default_rng(seed)
    (seed schedule (1, 0, 0)), and the random starts consume it before any slip draw (ma_frozen_lake.py:59-64)."""
    rms, dets, starts = [], [], []
    for ag in agents:
        rm = ag.get_reward_machine()
        spec = RewardMachineSpec(rm.transitions, initial_state=getattr(rm, "initial_state", None))
        if hasattr(rm, "state_indices"):
            spec.state_indices = dict(rm.state_indices)  # honour compile_reward_machine's override (io.py:167-170)
        rms.append(spec)
        dets.append(set(getattr(rm.event_detector, "positions", ()) or ()))
        pos = getattr(ag, "initial_position", None) or ag.get_position()
        starts.append(tuple(pos))
    if hasattr(env, "holes"):
        _check_modelled(env)
        slip = {"stochastic": bool(getattr(env, "frozen_lake_stochastic", False)),
                "delay_action": bool(getattr(env, "delay_action", False)), "seed_schedule": (1, 0, 0),
                "random_starts": bool(getattr(env, "random_start_positions", False))}
        return compile_tables(FROZEN_LAKE, env.grid_width, env.grid_height, env.holes, (), starts, rms, dets,
                              hazard_penalty=getattr(env, "penalty_amount", 0) or 0, hazard_fail=True, gamma=1.0,
                              reward_modifier=reward_modifier, max_t=MAX_T, **slip)
    if hasattr(env, "plants"):
        _check_modelled(env)
        slip = {"stochastic": bool(getattr(env, "stochastic", False)),
                "delay_action": bool(getattr(env, "delay_action", False)),
                "all_slip": bool(getattr(env, "all_slip", False)), "high_prob": getattr(env, "high_prob", 0.8),
                "seed_schedule": (1, 0, 0)}
        return compile_tables(OFFICE_WORLD, env.grid_width, env.grid_height, env.plants, env.walls, starts, rms, dets,
                              hazard_penalty=env.plants_penalty_value, wall_penalty=env.wall_penalty_value,
                              hazard_fail=env.terminate_on_plants, wall_fail=env.terminate_hit_walls, gamma=1.0,
                              reward_modifier=reward_modifier, max_t=MAX_T, **slip)
    raise TypeError("env must be a FrozenLake (holes) or OfficeWorld (plants, walls) grid environment")


def _learner(agent):
    get = getattr(agent, "get_learning_algorithm", None)
    return get() if get else getattr(agent, "learning_algorithm", None)


def _same_tables(a, b):
    if a.random_starts != b.random_starts:
        return False
    if a.stochastic != b.stochastic or (a.stochastic and not (np.array_equal(a.slip_out, b.slip_out)
                                                              and np.array_equal(a.slip_cdf, b.slip_cdf))):
        return False
    keys = ("cell", "cell_event", "next_q", "rm_reward", "init_q", "final_q") + (() if a.random_starts else ("start_xy",))
    scal = ("kind", "width", "height", "hazard_penalty", "wall_penalty", "hazard_fail", "wall_fail", "max_t",
            "reward_modifier")
    return (all(getattr(a, k) == getattr(b, k) for k in scal)
            and all(np.array_equal(getattr(a, k), getattr(b, k)) for k in keys))


# env attributes that change while an episode runs (bookkeeping, rng) and never feed the tables
_VOLATILE = {"active_agents", "agent_fail", "agent_steps", "timestep", "rng", "rewards", "epsilon", "agents"}


_ATOMIC = frozenset((int, float, bool, str, type(None)))


def _freeze(v):
    """A comparable snapshot of a table input (containers copied into tuples, arrays into bytes).  A container whose
    items are all hashable (tuples of numbers and strings: holes, transitions, positions) is snapshotted as one tuple
    in C; hashable values are immutable by convention, so the tuple cannot change under the snapshot."""
    t = type(v)
    if t in _ATOMIC:  # the common case (flags, penalties, sizes): the value itself
        return v
    if t is list or t is tuple:
        tv = tuple(v)
        try:
            hash(tv)
            return tv
        except TypeError:
            return tuple(_freeze(x) for x in tv)
    if t is dict:
        items = tuple(v.items())
        try:
            hash(items)
            return items
        except TypeError:
            return tuple((k, _freeze(x)) for k, x in items)
    if isinstance(v, dict):
        return tuple((k, _freeze(x)) for k, x in v.items())
    if isinstance(v, (list, tuple)):
        return tuple(_freeze(x) for x in v)
    if isinstance(v, (set, frozenset)):
        return frozenset(v)
    if isinstance(v, np.ndarray):
        return (v.dtype.str, v.shape, v.tobytes())
    return v


def _fingerprint(env, agents, reward_modifier, want_qrm):
    """Everything tables_from_objects reads, frozen: equal fingerprints compile to equal tables, so reset() skips
    the ~0.3-0.4 ms table compile while nothing changed.  With random starts the agents' start cells are drawn
    at every reset and are no table input."""
    fe = tuple([(k, _freeze(v)) for k, v in vars(env).items()
                if k not in _VOLATILE and k[:1] != "_" and not callable(v)])
    rs = hasattr(env, "holes") and bool(getattr(env, "random_start_positions", False))
    fa = []
    for ag in agents:
        rm = ag.get_reward_machine()
        det = getattr(rm, "event_detector", None)
        fa.append((id(rm), _freeze(rm.transitions), getattr(rm, "initial_state", None),
                   _freeze(getattr(rm, "state_indices", None)), _freeze(getattr(det, "positions", None)),
                   None if rs else (getattr(ag, "initial_position", None) or ag.get_position())))
    return fe, tuple(fa), reward_modifier, bool(want_qrm)


def _action_index(a):
    if isinstance(a, (int, np.integer)):
        return int(a)
    name = getattr(a, "name", a)
    if name not in ACTION_INDEX:
        raise KeyError(f"unknown action {name!r}")
    return ACTION_INDEX[name]


def scenario_objects(desc):
    """Reference-shaped env / agents / RMs (the classes above) for a scenario dict of tables.compile_scenario,
    built the way frozen_lake_main.py:199-267 / office_main.py:400-440 build theirs (rm rows only)."""
    from . import maps
    from .tables import scenario_symbols

    sym, parsed = scenario_symbols(desc)
    if desc["kind"] == "frozen_lake":
        w, h = parsed["dims"]
        env = MultiAgentFrozenLake(width=w, height=h, holes=parsed["holes"])
        env.penalty_amount = desc.get("penalty", 0)
        det = PositionEventDetector(set(parsed["goals"].values()))
    else:
        gh, gw = parsed["grid_size"]
        coords = parsed["coords"]
        walls = list(parsed["walls"]) + [(b, a) for (a, b) in parsed["walls"]]
        env = MultiAgentOfficeWorld(gw, gh, coords["plant"], coords["coffee"], coords["letter"], walls,
                                    desc["plants_penalty"], desc["wall_penalty"], desc["terminate_on_plants"],
                                    desc["terminate_hit_walls"])
        det = PositionEventDetector({sym[k] for k in maps.OFFICE_WORLD_EVENT_SYMBOLS})
    agents = []
    for i, ac in enumerate(desc["agents"]):
        ag = AgentRL(f"a{i + 1}", env)
        ag.set_initial_position(*ac["start"])
        trans = {(fr, None if ev is None else sym[ev]): (to, r) for fr, ev, to, r in ac["rm"]}
        ag.set_reward_machine(RewardMachine(trans, det))
        env.add_agent(ag)
        agents.append(ag)
    return env, agents


def _no_c_step(ctx, actions):
    """The C step path is off (use_c_step False, no engine yet, or an engine being replaced): step() runs in Python."""
    return None


_DICTSTEP = []  # the checked module (or None), once per process


def _dictstep_module():
    """csrc/rmx_dictstep.c's extension, checked against this tree's source once per process (a stale build is refused:
    the context layout is part of the source), or None when it is not built for this interpreter (the Python step
    path runs)."""
    if not _DICTSTEP:
        _DICTSTEP.append(_load_dictstep())
    return _DICTSTEP[0]


def _load_dictstep():
    import hashlib
    import os

    try:
        from . import _dictstep
    except ImportError:
        return None
    src = os.path.join(_capi.CSRC, "rmx_dictstep.c")
    if os.path.exists(src):
        with open(src, "rb") as f:
            want = hashlib.sha256(f.read()).hexdigest()[:16]
        if getattr(_dictstep, "SOURCE_HASH", None) != want:
            raise RuntimeError(f"{_dictstep.__file__} was built from another rmx_dictstep.c (rebuild: "
                               "__graft_entry__.build())")
    if getattr(_dictstep, "CTX_ITEMS", None) != _CTX_ITEMS:
        raise RuntimeError(f"{_dictstep.__file__}: context layout {getattr(_dictstep, 'CTX_ITEMS', None)}, "
                           f"rmx.compat builds {_CTX_ITEMS}")
    return _dictstep


_CTX_ITEMS = 20  # the step context tuple (_agent_cache; rmx_dictstep.c CTX_ITEMS)


def default_device():
    """The dict API's engine when none is named: GPU 0 when the process sees one, else the host path."""
    return 0 if _capi.device_count() > 0 else "cpu"


class RMEnvironmentWrapper:
    """reset(seed) / step(actions) / check_terminations() of rm_environment_wrapper.py on the engine.

    Every reset / step is one synchronous call of the C ABI (rmx_reset_sync / rmx_step_sync): on a GPU the actions go
    into the handle's pinned mailbox, the resident workgroup steps the env and writes the outputs back into host
    memory; on a host handle (device="cpu") the call steps the env itself.  One ``struct.unpack_from`` (or the C step
    path) turns the output record into Python numbers.  The QRM counterfactual columns are computed only while a
    learner has ``use_qrm`` (rm_environment_wrapper.py:78)."""

    # the per-step host path in C (csrc/rmx_dictstep.c); False: the Python implementation of step() (A/B, tests)
    use_c_step = True

    def __init__(self, env, agents, device=None):
        self.env = env
        self.agents = agents
        self.reward_modifier = 1
        self.device = default_device() if device is None else device
        self._cstep, self._ctx, self._ctx_key = _no_c_step, None, None
        self._engine = None
        self.tables = None
        self._modifier_compiled = None
        self._qrm_on = False
        self._qrm_req = False
        self._fp = None

    # -- engine lifecycle --------------------------------------------------------------------------
    def _want_qrm(self):
        return any(getattr(_learner(ag), "use_qrm", False) for ag in self.agents)

    def _build(self, want_qrm=None):
        from . import engine as E

        want_qrm = self._want_qrm() if want_qrm is None else want_qrm
        fp = _fingerprint(self.env, self.agents, self.reward_modifier, want_qrm)
        if self._engine is not None and fp == self._fp:
            return
        tab = tables_from_objects(self.env, self.agents, float(self.reward_modifier))
        self._fp = fp
        if self._engine is not None and _same_tables(tab, self.tables) and want_qrm <= self._qrm_req:
            self._modifier_compiled = self.reward_modifier  # (a modifier change that compiles to the same tables)
            return  # objects unchanged since the last build: keep the device handle
        self.tables = tab
        # the C step path's context holds the old engine's handle and buffer addresses: off until _agent_cache
        # rebuilds it for the new engine (a failure before that leaves step() on the Python path, never on freed memory)
        self._cstep, self._ctx, self._ctx_key = _no_c_step, None, None
        if self._engine is not None:
            self._engine.close()
            self._engine = None
        self._engine = E.make_env(self.tables, 1, device=self.device, with_qrm=want_qrm)
        self._modifier_compiled = self.reward_modifier
        self._qrm_on = self._engine.qrm_s is not None
        # what was asked for: with n_qrm_max == 0 there are no QRM columns to bind, and a learner's use_qrm must not
        # make every step rebuild (want_qrm > _qrm_on would hold forever)
        self._qrm_req = bool(want_qrm)
        self._io_setup()

    def _io_setup(self):
        """One host output record for the synchronous calls: x, y, q, flags [A] i32, reward, renv [A] f32, t i32,
        then (QRM on) s, sn [A][Qx] i32, rq [A][Qx] f32, done [A][Qx] u8 — the rmx_buffers columns at N = 1."""
        eng = self._engine
        A, Qx = eng.A, (eng.n_qrm_max if self._qrm_on else 0)
        self._A, self._Qx = A, Qx
        head = 4 * (6 * A + 1)
        nbytes = head + 4 * 3 * A * Qx + A * Qx
        self._out = (C.c_char * max(nbytes, 1))()
        base = C.addressof(self._out)
        b = _capi.RmxBuffers()
        for k, name in enumerate(("pos_x", "pos_y", "rm_q", "flags", "reward", "renv")):
            setattr(b, name, base + 4 * A * k)
        b.t = base + 4 * 6 * A
        if Qx:
            b.qrm_s, b.qrm_sn, b.qrm_rq = (base + head + 4 * A * Qx * k for k in range(3))
            b.qrm_done = base + head + 12 * A * Qx
        self._bufs = b
        self._bufs_p = C.pointer(b)
        self._fmt = struct.Struct(f"<{4 * A}i{2 * A}fi")
        self._fmt_q = struct.Struct(f"<{2 * A * Qx}i{A * Qx}f{A * Qx}B") if Qx else None
        self._act = (C.c_int32 * A)()
        self._act_p = C.cast(self._act, C.c_void_p)
        lib = eng.lib
        self._step_fn, self._reset_fn = lib.rmx_step_sync, lib.rmx_reset_sync
        self._begin_fn, self._wait_fn = lib.rmx_step_sync_begin, lib.rmx_sync_wait
        self._h = eng._h
        self._fl_kind = self.tables.kind == FROZEN_LAKE
        self._fl_slip = self._fl_kind and bool(self.tables.stochastic)
        # RM-state labels by index (RewardMachine.get_state_from_index), per agent
        self._labels = [{v: k for k, v in rm.state_indices.items()} for rm in self.tables.rms]

    def _sync_call(self, rc, what):
        if rc != _capi.RMX_OK:
            _capi.check(rc, what)

    def _label(self, a, q):
        return self.tables.rms[a].get_state_from_index(int(q))

    # -- reference API -------------------------------------------------------------------------------
    def reset(self, seed=123):
        """env.reset(seed) (ma_frozen_lake.py:43-94, ma_office.py:77-120).  seed=None: the reference draws a
        fresh default_rng(); here a fresh 64-bit seed from OS entropy, so an unseeded run matches the
        reference in distribution (not stream for stream)."""
        self._build()
        self._agent_cache()
        if seed is None:
            seed = int(np.random.SeedSequence().entropy) & (2**64 - 1)
        self._sync_call(self._reset_fn(self._h, int(seed) & (2**64 - 1), self._bufs_p, None), "rmx_reset_sync")
        v = self._fmt.unpack_from(self._out)
        A = self._A
        e = self.env
        e.timestep = 0
        obs, infos = {}, {}
        active, fail, steps = e.active_agents, e.agent_fail, e.agent_steps
        rs = self.tables.random_starts
        for i, (ag, name, rm) in enumerate(zip(self.agents, self._names, self._rms)):
            if rs:  # _sample_start_positions -> agent.set_initial_position
                ag.set_initial_position(v[i], v[A + i])
            else:
                ag.set_position(v[i], v[A + i])
            rm.current_state = rm.initial_state
            active[name] = True
            fail[name] = False
            steps[name] = 0
            obs[name] = ag.state
            infos[name] = {}
        return obs, infos

    def _agent_cache(self):
        """Per-agent objects the per-step path reads, refreshed at every reset (an agent's RM object is a table input:
        a new one is picked up by the reset's fingerprint, as before), and the context of the C step path
        (csrc/rmx_dictstep.c: the same calls as step() below, without the interpreter loop).  The context holds raw
        addresses of this engine's handle and of the ctypes buffers below; the engine and those buffers stay referenced
        by the wrapper (self._engine, self._act, self._bufs, self._out) for as long as the context is installed."""
        agents = self.agents
        key = (self._engine, self._fp, tuple(map(id, agents)), tuple(ag.name for ag in agents), self.use_c_step)
        if self._ctx is not None and key == self._ctx_key:
            return  # the same engine, agents and tables as the installed context
        self._cstep, self._ctx, self._ctx_key = _no_c_step, None, None
        self._names = [ag.name for ag in agents]
        self._rms = [ag.get_reward_machine() for ag in agents]
        self._getl = [getattr(ag, "get_learning_algorithm", None) for ag in agents]
        labels = [[d.get(i) for i in range(max(d) + 1)] if d else [] for d in self._labels]
        lib = self._engine.lib
        addr = lambda f: C.cast(f, C.c_void_p).value  # noqa: E731
        tab, A = self.tables, len(agents)
        n_qrm = [int(v) for v in tab.n_qrm] if tab.n_qrm is not None else [0] * A
        enc_nq = [int(v) for v in tab.enc_nq] if tab.enc_nq is not None else [1] * A
        self._ctx = (self._h.value or 0, addr(lib.rmx_step_sync_begin), addr(lib.rmx_sync_wait),
                     C.addressof(self._act), C.addressof(self._bufs), C.addressof(self._out), self._fl_kind,
                     self._fl_slip, self._names, list(agents), self._rms, labels, self._getl, self.env, ACTION_INDEX,
                     bool(self._qrm_req), int(self._Qx), n_qrm, enc_nq, AgentRL)
        mod = _dictstep_module() if self.use_c_step else None
        self._cstep = mod.step if mod is not None else _no_c_step
        self._ctx_key = key

    def _use_qrm(self):
        """rm_environment_wrapper.py:78, read every step: getattr(agent.get_learning_algorithm(), "use_qrm", False)."""
        out = []
        for g, ag in zip(self._getl, self.agents):
            out.append(getattr(g() if g is not None else getattr(ag, "learning_algorithm", None), "use_qrm", False))
        return out

    def step(self, actions):
        if self._engine is None:
            raise RuntimeError("call reset() before step()")
        if self.reward_modifier == self._modifier_compiled:  # the C path (rmx_dictstep.c); None: this one
            r = self._cstep(self._ctx, actions)
            if r is not None:
                if r.__class__ is int:
                    _capi.check(r, "rmx_step_sync")
                return r
        agents = self.agents
        use_qrm = self._use_qrm()
        want_qrm = True in use_qrm
        if self.reward_modifier != self._modifier_compiled or want_qrm > self._qrm_req:
            eng = self._engine  # rebuild tables / outputs, keep the episode state
            eng.sync_end()
            snap = eng.snapshot()
            self._build(want_qrm)
            self._engine.load_snapshot(snap)
            self._agent_cache()
        act = self._act
        fl_slip = self._fl_slip
        names, rms = self._names, self._rms
        for i, name in enumerate(names):
            a = actions[name]
            try:
                k = ACTION_INDEX[a.name]
            except AttributeError:
                k = _action_index(a)
            except KeyError:
                raise KeyError(f"unknown action {a.name!r}") from None
            if not 0 <= k <= 4:
                raise ValueError("actions must be up/down/left/right/wait")
            if k == 4 and fl_slip:  # the slip map has no "wait" entry (ma_frozen_lake.py:122, 257): KeyError
                # Intentional difference on this error path: the reference raises inside its agent loop
                # (ma_frozen_lake.py:106-124), after the agents before this one have moved, drawn from the rng and
                # counted a step; here the whole step is refused before any agent moves (the env state is the
                # pre-step state).  The exception type and key are the reference's.
                rm = rms[i]  # for an agent the env steps (active, RM not final: :107-114)
                if self.env.active_agents.get(name, True) and rm.get_current_state() != rm.get_final_state():
                    raise KeyError("wait")
            act[i] = k
        # the request goes out first; the host-side bookkeeping of the previous state overlaps its round trip
        rc = self._begin_fn(self._h, self._act_p, 0, None)
        if rc != _capi.RMX_OK:
            _capi.check(rc, "rmx_step_sync_begin")
        env = self.env
        active, fail, steps = env.active_agents, env.agent_fail, env.agent_steps
        prev = [dict(ag.state) for ag in agents]
        prev_q = [rm.current_state for rm in rms]
        labels = self._labels
        # OW skips inactive agents before filling infos (ma_office.py:143-144); FrozenLake fills them all
        full = None if self._fl_kind else [active.get(n, True) for n in names]
        A = self._A
        qrm = None
        rc = self._wait_fn(self._h, self._bufs_p)
        if rc != _capi.RMX_OK:
            _capi.check(rc, "rmx_sync_wait")
        v = self._fmt.unpack_from(self._out)
        if want_qrm and self._Qx:
            qv = self._fmt_q.unpack_from(self._out, 4 * (6 * A + 1))
            n = A * self._Qx
            qrm = (qv[:n], qv[n:2 * n], qv[2 * n:3 * n], qv[3 * n:])
        obs, rewards, terms, truncs, infos = {}, {}, {}, {}, {}
        # the record: x [A], y [A], q [A], flags [A], reward [A], renv [A], t
        for i in range(A):
            name, ag, rm = names[i], agents[i], rms[i]
            f, reward, renv = v[3 * A + i], v[4 * A + i], v[5 * A + i]
            ag.set_position(v[i], v[A + i])
            q = rm.current_state = labels[i][v[2 * A + i]]
            state = ag.state
            obs[name] = state
            rewards[name] = reward
            terms[name] = (f & 4) != 0  # RMX_F_TERM
            truncs[name] = (f & 8) != 0  # RMX_F_TRUNC
            if full is None or full[i]:
                info = {"prev_s": prev[i], "s": dict(state), "Renv": renv, "RQ": reward - renv, "prev_q": prev_q[i],
                        "q": q, "reward_machine": rm}
            else:
                info = {"RQ": reward - renv, "prev_q": prev_q[i], "q": q, "reward_machine": rm}
            if qrm is not None and use_qrm[i]:  # rm_environment_wrapper.py:78-89
                info["qrm_experience"] = self._qrm_tuples(i, act[i], renv, qrm)
            info["env_terminated"] = (f & 16) != 0  # RMX_F_ENV_TERM
            info["rm_terminated"] = (f & 32) != 0  # RMX_F_RM_TERM
            infos[name] = info
            active[name] = (f & 1) != 0  # RMX_F_ACTIVE
            fail[name] = (f & 2) != 0  # RMX_F_FAIL
            steps[name] = f >> 16  # RMX_F_STEPS_SHIFT
        env.timestep = v[6 * A]
        return obs, rewards, terms, truncs, infos

    def _qrm_tuples(self, i, action_index, renv, qrm):
        """The ten-field experience tuples of rm_environment_wrapper.py:168-179 for agent i (qrm: the flat
        [A][Qx] s, sn, rq, done columns of the step)."""
        qs, qsn, qrq, qdone = qrm
        nq = int(self.tables.enc_nq[i])
        o = i * self._Qx
        out = []
        for j in range(int(self.tables.n_qrm[i])):
            s_, sn, hr = qs[o + j], qsn[o + j], qrq[o + j]
            out.append((s_, action_index, renv + hr, sn, bool(qdone[o + j]), s_ // nq, s_ % nq, sn // nq, sn % nq, hr))
        return out

    def get_mdp(self, seed=123, fix_frozen_lake=False):
        """rm_environment_wrapper.py:185-283 on the GPU: one launch per agent over all (state, action)
        pairs.  Like the reference it switches OfficeWorld to deterministic dynamics permanently and
        leaves the wrapper reset.  fix_frozen_lake=False keeps the reference's FrozenLake quirk."""
        if hasattr(self.env, "stochastic"):
            self.env.stochastic = False  # :196-197
        self._build()
        self._engine.sync_end()
        P, ns, na = self._engine.get_mdp(fix_frozen_lake=fix_frozen_lake)  # (HostRMEnv: the host path's get_mdp)
        names = [ag.name for ag in self.agents]
        out = ({names[i]: v for i, v in P.items()}, {names[i]: v for i, v in ns.items()},
               {names[i]: v for i, v in na.items()})
        self.reset(seed)
        return out

    def check_terminations(self):
        out = {}
        for ag in self.agents:
            rm = ag.get_reward_machine()
            out[ag.name] = rm.get_current_state() == rm.get_final_state()
        return out
