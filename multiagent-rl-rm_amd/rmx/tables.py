"""Host-side table compiler: map layouts + Reward Machines -> the dense tables of ``rmx_config``.

This runs once per engine construction (never per step).  It restates, from scratch, the parts of
the reference that define the static structure the step kernel consults (paths relative to
Alee08/multiagent-rl-rm):

* ``parse_map_emoji``            multiagent_rlrm/utils/utils.py:169-203
* ``parse_office_world``         multiagent_rlrm/utils/utils.py:206-240
* ``find_disconnected_pairs``    multiagent_rlrm/utils/utils.py:300-364 (incl. the x==1,y==3 quirk)
* wall symmetrisation            multiagent_rlrm/environments/office_world/office_main.py:416
* ``can_move_*``                 multiagent_rlrm/environments/office_world/config_office.py:12-39
* FrozenLake boundary clamp      multiagent_rlrm/environments/frozen_lake/ma_frozen_lake.py:224-242
* RM indexing / initial / final  multiagent_rlrm/multi_agent/reward_machine.py:20-39,130-177
* potential shaping (VI)         multiagent_rlrm/multi_agent/reward_machine.py:197-214,308-345
* distance shaping (BFS)         multiagent_rlrm/multi_agent/reward_machine.py:216-278

Pinned against the reference's own results in tests/golden/tables.json.
"""
from __future__ import annotations

import math
import string
import textwrap
from collections import deque
from dataclasses import dataclass, field
from typing import Dict, Hashable, List, Optional, Sequence, Tuple

import numpy as np

from . import maps as _maps

FROZEN_LAKE = 0
OFFICE_WORLD = 1

CAN_UP, CAN_DOWN, CAN_LEFT, CAN_RIGHT, HAZARD = 0x01, 0x02, 0x04, 0x08, 0x10

Pos = Tuple[int, int]


# --------------------------------------------------------------------------------------------------
# Map parsers
# --------------------------------------------------------------------------------------------------
def parse_map_emoji(map_string: str):
    """FrozenLake emoji layout -> (holes, goals, (width, height)).  utils.py:169-203."""
    lines = textwrap.dedent(map_string).strip().splitlines()
    holes: List[Pos] = []
    goals: Dict[str, Pos] = {}
    widths = []
    for y, raw in enumerate(lines):
        cells = [ch for ch in raw if ch != " "]
        widths.append(len(cells))
        for x, ch in enumerate(cells):
            if ch == "⛔":
                holes.append((x, y))
            elif ch.isdigit() or ch.isalpha():
                goals[ch] = (x, y)
    return holes, goals, (max(widths), len(lines))


_OW_SYMBOLS = {"🟩": "empty_cell", "🪴": "plant", "🥤": "coffee", "✉️": "letter"}


def find_disconnected_pairs(office_world: str) -> List[Tuple[Pos, Pos]]:
    """Wall pairs between compact cells separated by a ⛔ in the full layout.  utils.py:300-364."""
    grid = [line.strip().split() for line in office_world.strip().split("\n")]
    rows = len(grid)
    cols = len(grid[0]) if rows else 0
    is_barrier = lambda c: c in ("⛔", "🚪")  # noqa: E731

    y_off = [0] * rows
    k = 0
    for y in range(rows):
        if all(is_barrier(c) for c in grid[y]):
            y_off[y] = 1  # barrier rows get offset 1 (never used as a source; kept as in the reference)
        else:
            y_off[y] = k
            k += 1
    x_off = [0] * cols
    k = 0
    for x in range(cols):
        if all(is_barrier(grid[y][x]) for y in range(rows)):
            x_off[x] = 1
        else:
            x_off[x] = k
            k += 1

    pairs = []
    for y in range(rows):
        for x in range(cols):
            if is_barrier(grid[y][x]):
                continue
            if x < cols - 2 and grid[y][x + 1] == "⛔" and grid[y][x + 2] != "⛔":
                pairs.append(((x_off[x], y_off[y]), (x_off[x + 2], y_off[y])))
            if (y < rows - 2 and grid[y + 1][x] == "⛔" and grid[y + 2][x] != "⛔"
                    and not (x == 1 and y == 3 and grid[1][4] == "🪴")):
                pairs.append(((x_off[x], y_off[y]), (x_off[x], y_off[y + 2])))
    return pairs


def parse_office_world(office_world: str):
    """OfficeWorld layout -> (coordinates, goals, walls).  utils.py:206-240."""
    lines = [ln.replace("⛔", "").replace("🚪", "").strip().split() for ln in office_world.strip().split("\n")]
    lines = [ln for ln in lines if ln]
    keys = string.ascii_uppercase + string.digits
    goals_all: Dict[str, List[Pos]] = {c: [] for c in keys}
    coords: Dict[str, List[Pos]] = {"plant": [], "coffee": [], "letter": [], "empty_cell": []}
    for y, row in enumerate(lines):
        for x, cell in enumerate(row):
            if cell in _OW_SYMBOLS:
                coords[_OW_SYMBOLS[cell]].append((x, y))
            elif cell in keys:
                goals_all[cell].append((x, y))
    goals = {k: v[0] for k, v in goals_all.items() if v}
    return coords, goals, find_disconnected_pairs(office_world)


# --------------------------------------------------------------------------------------------------
# Reward Machine structure (construction-time API of the reference RewardMachine)
# --------------------------------------------------------------------------------------------------
class RewardMachineSpec:
    """Static structure of a Reward Machine given its transitions dict.

    ``transitions``: ``{(from_state, event): (to_state, reward)}`` in insertion order, exactly the
    reference constructor argument (reward_machine.py:5-18).  Events are position tuples, ``None``
    (the detector's "no event") or anything hashable (never detected by a position detector).
    """

    def __init__(self, transitions: Dict[Tuple[Hashable, Hashable], Tuple[Hashable, float]],
                 initial_state: Optional[Hashable] = None):
        self.transitions = dict(transitions)
        if initial_state is None:  # source of the first inserted transition (reward_machine.py:165-177)
            initial_state = next(iter(self.transitions))[0] if self.transitions else None
        self.initial_state = initial_state
        self.state_indices = self._state_indices()
        self.potentials: Optional[Dict[Hashable, float]] = None

    def _state_indices(self):  # reward_machine.py:20-39: initial first, the rest in sorted() order
        states = set()
        for (u1, _e), (u2, _r) in self.transitions.items():
            states.add(u1)
            states.add(u2)
        states.add(self.initial_state)
        ordered = sorted(states)
        ordered.remove(self.initial_state)
        ordered.insert(0, self.initial_state)
        return {s: i for i, s in enumerate(ordered)}

    def get_state_index(self, s):
        return self.state_indices[s]

    def get_state_from_index(self, i):
        inv = {v: k for k, v in self.state_indices.items()}
        if i not in inv:
            raise ValueError(f"Index {i} not present in RewardMachine.state_indices")
        return inv[i]

    def get_final_state(self):  # reward_machine.py:152-163: to_state of the LAST inserted transition
        if not self.transitions:
            return None
        return next(reversed(self.transitions.values()))[0]

    def numbers_state(self):  # reward_machine.py:130-138
        states = set()
        for (u1, _e), (u2, _r) in self.transitions.items():
            states.add(u1)
            states.add(u2)
        return len(states)

    def get_all_states(self):  # reward_machine.py:95-111: first-appearance order
        seen, out = set(), []
        for (u1, _e), (u2, _r) in self.transitions.items():
            for s in (u1, u2):
                if s not in seen:
                    seen.add(s)
                    out.append(s)
        return out

    def get_delta_u(self):  # reward_machine.py:280-292
        d: Dict = {}
        for (u1, ev), (u2, _r) in self.transitions.items():
            d.setdefault(u1, {})
            d.setdefault(u2, {})
            d[u1][u2] = ev
        return d

    def get_delta_r(self):  # reward_machine.py:294-306 (constant rewards only)
        d: Dict = {}
        for (u1, _ev), (u2, r) in self.transitions.items():
            d.setdefault(u1, {})
            d.setdefault(u2, {})
            d[u1][u2] = r
        return d

    @staticmethod
    def value_iteration(U, delta_u, delta_r, terminal_u, gamma):
        """Gauss-Seidel VI in U order until the max change <= 1e-7 (reward_machine.py:308-345)."""
        V = {u: 0 for u in U}
        V[terminal_u] = 0
        err = 1
        while err > 0.0000001:
            err = 0
            for u1 in U:
                if not delta_u[u1]:
                    continue
                q = [delta_r[u1][u2] + gamma * V[u2] for u2 in delta_u[u1]]
                if q:
                    v = max(q)
                    err = max([err, abs(v - V[u1])])
                    V[u1] = v
        return V

    def add_reward_shaping(self, gamma, rs_gamma):  # reward_machine.py:197-214
        self.gamma = gamma
        V = self.value_iteration(list(self.state_indices.keys()), self.get_delta_u(), self.get_delta_r(),
                                 self.get_final_state(), rs_gamma)
        self.potentials = {u: -v for u, v in V.items()}

    def get_distance(self, start):  # reward_machine.py:242-278
        final = self.get_final_state()
        if start == final:
            return 0
        queue, seen = deque([(start, 0)]), {start}
        while queue:
            cur, d = queue.popleft()
            if cur == final:
                return d
            for (u, _ev), (v, _r) in self.transitions.items():
                if u == cur and v not in seen:
                    seen.add(v)
                    queue.append((v, d + 1))
        return 999999

    def add_distance_reward_shaping(self, gamma, rs_gamma, alpha=100):  # reward_machine.py:216-240
        final = self.get_final_state()
        self.potentials = {u: (0 if u == final else -alpha * self.get_distance(u)) for u in self.get_all_states()}


# --------------------------------------------------------------------------------------------------
# Compiled tables
# --------------------------------------------------------------------------------------------------
@dataclass
class CompiledTables:
    """Everything ``rmx_config`` needs, as numpy arrays (host)."""
    kind: int
    width: int
    height: int
    n_agents: int
    n_rm_states: int
    n_events: int
    cell: np.ndarray          # uint16 [H*W]
    cell_event: np.ndarray    # uint8  [A][H*W]
    next_q: np.ndarray        # uint8  [A][Q][E]
    rm_reward: np.ndarray     # float32 [A][Q][E]
    shape: Optional[np.ndarray]  # float32 [A][Q][E] or None
    init_q: np.ndarray        # int32 [A]
    final_q: np.ndarray       # int32 [A]
    start_xy: np.ndarray      # int32 [A][2]
    hazard_penalty: float = 0.0
    wall_penalty: float = 0.0
    hazard_fail: int = 1
    wall_fail: int = 0
    gamma: float = 1.0
    max_t: int = 1000
    reward_modifier: float = 1.0
    # QRM (rm_environment_wrapper.py:122-183): per agent the state indices of get_all_states()[:-1]
    n_qrm: Optional[np.ndarray] = None       # int32 [A]
    qrm_states: Optional[np.ndarray] = None  # uint8 [A][Qx]
    enc_nq: Optional[np.ndarray] = None      # int32 [A] numbers_state() (encoder stride)
    # stochastic slip (ma_frozen_lake.py:244-298, ma_office.py:327-379)
    stochastic: int = 0
    slip_n: Optional[np.ndarray] = None      # int32 [4]
    slip_out: Optional[np.ndarray] = None    # int32 [4][4] outcome action ids
    slip_cdf: Optional[np.ndarray] = None    # float64 [4][4]
    seed_schedule: Tuple[int, int, int] = (1, 1, 0)  # seed = base*scale + e*env_stride + k*episode_stride
    # FrozenLake random_start_positions (ma_frozen_lake.py:37-39, 59-64, 156-172): every reset shuffles the
    # non-hole cells with the freshly seeded env rng and starts the agents on the first A (start_xy unused)
    random_starts: int = 0
    rms: List[RewardMachineSpec] = field(default_factory=list)
    event_cells: List[Pos] = field(default_factory=list)  # event id k>=1 -> cell

    def label_of(self, agent: int, q_index: int):
        return self.rms[agent].get_state_from_index(int(q_index))


_ACT = {"up": 0, "down": 1, "left": 2, "right": 3, "wait": 4}


def slip_mapping(kind: int, delay_action=False, all_slip=False, high_prob=0.8):
    """{intended: (outcomes, probabilities)} of the stochastic dynamics, exactly the reference lists:
    FrozenLake _stochastic_action_probability_mapping (ma_frozen_lake.py:279-298), OfficeWorld
    get_action_probability_mapping (ma_office.py:327-366)."""
    if delay_action:
        return {"left": (["wait", "left", "up", "down"], [0.6, 0.36, 0.02, 0.02]),
                "right": (["wait", "right", "up", "down"], [0.6, 0.36, 0.02, 0.02]),
                "up": (["wait", "up", "left", "right"], [0.6, 0.36, 0.02, 0.02]),
                "down": (["wait", "down", "left", "right"], [0.6, 0.36, 0.02, 0.02])}
    if kind == FROZEN_LAKE:
        return {"left": (["left", "up", "down"], [0.8, 0.1, 0.1]), "right": (["right", "up", "down"], [0.8, 0.1, 0.1]),
                "up": (["up", "left", "right"], [0.8, 0.1, 0.1]), "down": (["down", "left", "right"], [0.8, 0.1, 0.1])}
    hp = high_prob
    if all_slip:
        lp = (1 - hp) / 3
        return {"left": (["left", "right", "up", "down"], [hp, lp, lp, lp]),
                "right": (["right", "left", "up", "down"], [hp, lp, lp, lp]),
                "up": (["up", "down", "left", "right"], [hp, lp, lp, lp]),
                "down": (["down", "up", "left", "right"], [hp, lp, lp, lp])}
    lp = (1 - hp) / 2
    return {"left": (["left", "up", "down"], [hp, lp, lp]), "right": (["right", "up", "down"], [hp, lp, lp]),
            "up": (["up", "left", "right"], [hp, lp, lp]), "down": (["down", "left", "right"], [hp, lp, lp])}


def slip_tables(mapping):
    """Outcome ids and the cdf numpy's Generator.choice builds: p.cumsum(); cdf /= cdf[-1]."""
    n = np.zeros(4, np.int32)
    out = np.full((4, 4), 4, np.int32)
    cdf = np.ones((4, 4), np.float64)
    for name, (outs, probs) in mapping.items():
        i = _ACT[name]
        c = np.asarray(probs, dtype=np.double).cumsum()
        c /= c[-1]
        n[i] = len(outs)
        out[i, :len(outs)] = [_ACT[o] for o in outs]
        cdf[i, :len(outs)] = c
    return n, out, cdf


def cell_tile(kind: int, width: int, height: int, hazards: Sequence[Pos], walls: Sequence[Tuple[Pos, Pos]] = ()):
    """uint16 per cell: can_move bits in the kind's own direction convention + hazard bit."""
    wall_set = set((tuple(a), tuple(b)) for a, b in walls)
    haz = set(tuple(p) for p in hazards)
    tile = np.zeros(width * height, np.uint16)
    up = -1 if kind == FROZEN_LAKE else +1  # FL up = y-1 (ma_frozen_lake.py:233), OW up = y+1 (ma_office.py:280)
    for y in range(height):
        for x in range(width):
            bits = 0
            for k, (dx, dy) in enumerate(((0, up), (0, -up), (-1, 0), (1, 0))):
                nx, ny = x + dx, y + dy
                if 0 <= nx < width and 0 <= ny < height and ((x, y), (nx, ny)) not in wall_set:
                    bits |= 1 << k
            if (x, y) in haz:
                bits |= HAZARD
            tile[y * width + x] = bits
    return tile


def compile_tables(kind: int, width: int, height: int, hazards, walls, starts: Sequence[Pos],
                   rms: Sequence[RewardMachineSpec], detector_positions: Sequence[Sequence[Pos]], *,
                   hazard_penalty=0.0, wall_penalty=0.0, hazard_fail=None, wall_fail=False, gamma=1.0,
                   shaping_gamma: Optional[float] = None, reward_modifier=1.0, max_t=1000, stochastic=False,
                   delay_action=False, all_slip=False, high_prob=0.8, seed_schedule=None,
                   random_starts=False) -> CompiledTables:
    """Dense per-agent tables.

    ``detector_positions[a]`` is the position set of agent a's PositionEventDetector
    (detect_event.py:18-33: a position in the set -> that position is the event, else None).
    A transition keyed on an event the detector can never emit is dead and gets no table entry, but
    still counts for state indexing and the final state, as in the reference.
    """
    A = len(rms)
    if not (1 <= A <= 8):
        raise ValueError("1..8 agents supported")
    if len(starts) != A or len(detector_positions) != A:
        raise ValueError("one start and one detector per agent")
    if random_starts:
        if kind != FROZEN_LAKE:
            raise ValueError("random_start_positions is a FrozenLake option (ma_frozen_lake.py:37-39)")
        haz = {tuple(p) for p in hazards}
        if width * height - len({p for p in haz if 0 <= p[0] < width and 0 <= p[1] < height}) < A:
            raise ValueError("Not enough free cells to place all agents.")  # ma_frozen_lake.py:169-170
    cells = width * height
    ev_cells = sorted({tuple(p) for ps in detector_positions for p in ps
                       if 0 <= p[0] < width and 0 <= p[1] < height})
    ev_id = {p: i + 1 for i, p in enumerate(ev_cells)}
    E = 1 + len(ev_cells)
    Q = max(len(rm.state_indices) for rm in rms)
    if Q > 255 or E > 255:
        raise ValueError("RM tables exceed the uint8 index range")
    cell_event = np.zeros((A, cells), np.uint8)
    for a, ps in enumerate(detector_positions):
        for p in ps:
            p = tuple(p)
            if p in ev_id:
                cell_event[a, p[1] * width + p[0]] = ev_id[p]
    from .rmspec import DenseRM

    next_q = np.zeros((A, Q, E), np.uint8)
    rr = np.zeros((A, Q, E), np.float64)
    shape = np.zeros((A, Q, E), np.float64) if shaping_gamma is not None else None
    init_q = np.zeros(A, np.int32)
    final_q = np.zeros(A, np.int32)
    for a, rm in enumerate(rms):
        # this agent's detector emits only its own cells; any other event (None aside) makes a dead row
        cols = {tuple(p): ev_id[tuple(p)] for p in detector_positions[a] if tuple(p) in ev_id}
        d = DenseRM.build(rm, cols, E, n_states=Q)
        next_q[a], rr[a], init_q[a], final_q[a] = d.next_q, d.reward, d.init_q, d.final_q
        if shape is not None:
            if rm.potentials is None:
                rm.add_reward_shaping(shaping_gamma, shaping_gamma)
            inv = {v: k for k, v in rm.state_indices.items()}
            phi = np.array([rm.potentials.get(inv.get(q), 0) if q in inv else 0.0 for q in range(Q)], np.float64)
            # shaping = gamma * Phi(q') - Phi(q) (qlearning.py:60-65, 99-105), f64 then f32
            shape[a] = shaping_gamma * phi[next_q[a].astype(np.int64)] - phi[:, None]
    if hazard_fail is None:
        hazard_fail = kind == FROZEN_LAKE
    qlists = [[rm.state_indices[u] for u in rm.get_all_states()[:-1]] for rm in rms]
    qx = max(len(ql) for ql in qlists)
    qrm_states = np.zeros((A, max(qx, 1)), np.uint8)
    for a, ql in enumerate(qlists):
        qrm_states[a, :len(ql)] = ql
    slip = slip_tables(slip_mapping(kind, delay_action, all_slip, high_prob)) if stochastic else (None, None, None)
    if seed_schedule is None:  # the runners' reset seeds: FL reset(seed) each episode; OW seed*1000+episode
        seed_schedule = (1, 1, 0) if kind == FROZEN_LAKE else (1000, 1000, 1)
    return CompiledTables(
        stochastic=int(bool(stochastic)), slip_n=slip[0], slip_out=slip[1], slip_cdf=slip[2],
        random_starts=int(bool(random_starts)),
        seed_schedule=tuple(int(v) for v in seed_schedule),
        kind=kind, width=width, height=height, n_agents=A, n_rm_states=Q, n_events=E,
        cell=cell_tile(kind, width, height, hazards, walls), cell_event=cell_event, next_q=next_q,
        rm_reward=rr.astype(np.float32), shape=None if shape is None else shape.astype(np.float32),
        init_q=init_q, final_q=final_q, start_xy=np.asarray(starts, np.int32).reshape(A, 2),
        hazard_penalty=float(hazard_penalty), wall_penalty=float(wall_penalty), hazard_fail=int(bool(hazard_fail)),
        wall_fail=int(bool(wall_fail)), gamma=float(gamma), max_t=int(max_t), reward_modifier=float(reward_modifier),
        n_qrm=np.array([len(ql) for ql in qlists], np.int32), qrm_states=qrm_states,
        enc_nq=np.array([rm.numbers_state() for rm in rms], np.int32), rms=list(rms), event_cells=ev_cells)


# --------------------------------------------------------------------------------------------------
# Scenario descriptions (the JSON-able form used by tests, bench and the golden generator)
# --------------------------------------------------------------------------------------------------
def _rm_from_rows(rows, sym: Dict[str, Pos]) -> RewardMachineSpec:
    trans = {}
    for fr, ev, to, r in rows:
        key = None if ev is None else tuple(sym[ev]) if isinstance(ev, str) else tuple(ev)
        trans[(fr, key)] = (to, r)
    return RewardMachineSpec(trans)


def scenario_symbols(desc) -> Tuple[Dict[str, Pos], dict]:
    kind = desc["kind"]
    if kind == "frozen_lake":
        layout = desc.get("layout") or _maps.FROZEN_LAKE_LAYOUTS[desc["map"]]
        holes, goals, dims = parse_map_emoji(layout)
        return dict(goals), {"holes": holes, "goals": goals, "dims": dims}
    m = _maps.OFFICE_WORLD_MAPS[desc["map"]]
    coords, goals, walls = parse_office_world(m["layout"])
    sym = dict(goals)
    for k in ("coffee", "letter"):
        for j, p in enumerate(coords[k]):
            sym[f"{k}{j}"] = p
    return sym, {"coords": coords, "goals": goals, "walls": walls, "grid_size": m["grid_size"]}


def _rm_from_spec(rs, mapping) -> RewardMachineSpec:
    """An agent's ``rm_spec`` entry: {"spec": RMSpec dict | "path": file, "complete": bool,
    "default_reward": float, "terminal_self_loop": bool} compiled like the --rm-spec runners."""
    from . import rmspec as R

    spec = R.RMSpec.from_dict(rs["spec"]) if "spec" in rs else R.load_rmspec(rs["path"])
    return R.compile_reward_machine(spec, event_mapping=mapping,
                                    complete_missing_transitions=rs.get("complete", False),
                                    default_reward=rs.get("default_reward", 0.0),
                                    terminal_self_loop=rs.get("terminal_self_loop", True),
                                    terminal_reward_must_be_zero=rs.get("terminal_reward_must_be_zero", True))


def _slip_kw(desc):
    return {"stochastic": desc.get("stochastic", False), "delay_action": desc.get("delay_action", False),
            "all_slip": desc.get("all_slip", False), "high_prob": desc.get("high_prob", 0.8),
            "seed_schedule": desc.get("seed_schedule"), "random_starts": desc.get("random_start_positions", False)}


def compile_scenario(desc, max_t: int = 1000) -> CompiledTables:
    """Compile a scenario dict (see tests/golden/configs.json) exactly as the reference entry points
    build their objects (frozen_lake_main.py:199-267, office_main.py:400-440,539-545); agents may give
    an ``rm_spec`` instead of ``rm`` rows (frozen_lake_main.py:133-183, office_main.py:442-532)."""
    from . import rmspec as R

    sym, parsed = scenario_symbols(desc)
    agents = desc["agents"]
    if desc["kind"] == "frozen_lake":
        mapping = R.frozenlake_event_mapping(parsed["goals"])
    else:
        mapping = R.officeworld_event_mapping(parsed["coords"], parsed["goals"])
    rms = [_rm_from_spec(ag["rm_spec"], mapping) if "rm_spec" in ag else _rm_from_rows(ag["rm"], sym) for ag in agents]
    starts = [tuple(ag["start"]) for ag in agents]
    sg = desc.get("shaping_gamma")
    if desc["kind"] == "frozen_lake":
        w, h = parsed["dims"]
        det = [set(parsed["goals"].values())] * len(agents)  # frozen_lake_main.py:226
        return compile_tables(FROZEN_LAKE, w, h, parsed["holes"], (), starts, rms, det,
                              hazard_penalty=desc.get("penalty", 0.0), gamma=1.0, shaping_gamma=sg, max_t=max_t,
                              reward_modifier=desc.get("reward_modifier", 1.0), **_slip_kw(desc))
    gh, gw = parsed["grid_size"]  # office_main.py:420-421: width = grid_size[1], height = grid_size[0]
    walls = list(parsed["walls"]) + [(b, a) for (a, b) in parsed["walls"]]  # office_main.py:416
    positions = {sym[s] for s in _maps.OFFICE_WORLD_EVENT_SYMBOLS if s in sym}
    if any("rm_spec" in ag for ag in agents):  # office_main.py:487-495: mapped positions join the detector
        positions = R.officeworld_detector_positions(parsed["coords"], parsed["goals"], positions)
    det = [positions] * len(agents)
    return compile_tables(OFFICE_WORLD, gw, gh, parsed["coords"]["plant"], walls, starts, rms, det,
                          hazard_penalty=desc.get("plants_penalty", -100.0), wall_penalty=desc.get("wall_penalty", 0.0),
                          hazard_fail=desc.get("terminate_on_plants", False), wall_fail=desc.get("terminate_hit_walls", False),
                          gamma=desc.get("gamma", 0.9), shaping_gamma=sg, max_t=max_t,
                          reward_modifier=desc.get("reward_modifier", 1.0), **_slip_kw(desc))


def baseline_scenario(config: int) -> dict:
    """BASELINE.json configs 1..5 as scenario dicts (SURVEY.md §8 'Concrete values')."""
    abc = [list(r) for r in _maps.FROZEN_LAKE_ABC]
    if config in (1, 2):
        return {"kind": "frozen_lake", "map": "map1", "penalty": 0.0,
                "agents": [{"start": [5, 0], "rm": abc}, {"start": [0, 0], "rm": abc}]}
    if config == 3:
        return {"kind": "office_world", "map": "map1", "plants_penalty": -100.0, "wall_penalty": 0.0,
                "terminate_on_plants": False, "terminate_hit_walls": False, "gamma": 0.9,
                "agents": [{"start": [2, 7], "rm": [list(r) for r in _maps.office_world_experiment("map1", "acbd")]}]}
    if config == 4:
        return {"kind": "frozen_lake", "map": "map1", "penalty": 0.0,
                "agents": [{"start": s, "rm": abc} for s in ([5, 0], [0, 0], [9, 0], [9, 9])]}
    if config == 5:
        exp5 = [list(r) for r in _maps.office_world_experiment("map1", "exp5")]
        return {"kind": "office_world", "map": "map1", "plants_penalty": -100.0, "wall_penalty": 0.0,
                "terminate_on_plants": False, "terminate_hit_walls": False, "gamma": 0.9, "shaping_gamma": 0.9,
                "agents": [{"start": s, "rm": exp5} for s in ([2, 7], [0, 0], [11, 8])]}
    raise ValueError(f"unknown BASELINE config {config}")
