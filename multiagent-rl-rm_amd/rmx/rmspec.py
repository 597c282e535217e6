"""Reward-Machine spec files -> the dense RM tables the step kernels read.

SURVEY.md §8(f) #3.  A spec (JSON / YAML, the reference's RMSpec format: name, env_id, version, states,
initial_state, terminal_states, event_vocabulary, transitions, notes) goes through one pipeline of pure
functions over immutable rows:

    read_spec / spec_from_mapping          the document -> RMSpec (rows are Transition tuples)
    spec_problems                          every rule the spec breaks, in a fixed order (empty: valid)
    completion_rows                        the self loops that close states x vocabulary
    expand_rows                            spec events -> environment events (grid cells), one row each
    DenseRM.build                          rows -> next_q [Q][E], reward [Q][E], init / final indices

``compile_reward_machine`` chains them into the RM structure the table compiler consumes
(tables.RewardMachineSpec); ``compile_dense`` goes straight to the arrays.  The names a caller of the reference
uses are kept (``load_rmspec``, ``RMSpec``, ``TransitionSpec``, ``ValidationError``, ``compile_reward_machine``,
``complete_missing_transitions``, ``validate_spec`` / ``validate_semantics``, ``compile_transition_map``); the
behaviour they pin is the reference's (paths relative to multiagent_rlrm/):

* reward literals "r0.5" / 0.5, booleans refused                          rmgen/spec.py:5-49
* JSON first, YAML (safe loader) as fallback unless the file says .json   rmgen/io.py:39-77
* completion: states x vocabulary order, terminal self loops optional     rmgen/completion.py:6-38
* an event mapped to a list of cells expands to one row per cell         rmgen/io.py:80-123
* RM indexing: the spec's initial state first, the rest in sorted() order; the "final" state is the target
  of the LAST row of the compiled map (so after completion: a self loop in `states` order, which can be a
  non-terminal state) — rmgen/io.py:126-171 over reward_machine.py:20-39,152-163; DESIGN.md §1 a10.

The LLM authoring / normalisation parts of rmgen are out of scope.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, Iterable, Iterator, List, Mapping, NamedTuple, Optional, Sequence, Tuple, Union

import numpy as np

from .tables import RewardMachineSpec


class ValidationError(ValueError):
    """The spec breaks a structural or semantic rule (the reference's rmgen ValidationError)."""


# --------------------------------------------------------------------------------------------------------------
# rows and rewards
# --------------------------------------------------------------------------------------------------------------
def parse_reward(value: Any, where: Any = None) -> float:
    """A reward literal: a number, or a string with an optional leading r / R ("r1", " 0.5 ")."""
    if isinstance(value, (int, float)) and not isinstance(value, bool):
        return float(value)
    if isinstance(value, str):
        body = value.strip()
        body = body[1:] if body[:1] in ("r", "R") else body
        try:
            return float(body)
        except ValueError:
            pass
    raise ValueError(f"reward {value!r} is not a number or an r<number> literal ({where})")


class Transition(NamedTuple):
    """One spec row: from_state --event / reward--> to_state."""
    from_state: str
    event: Any
    to_state: str
    reward: float

    @classmethod
    def from_mapping(cls, row: Mapping[str, Any]) -> "Transition":
        return cls(row["from_state"], row["event"], row["to_state"], parse_reward(row["reward"], row))

    def to_dict(self) -> Dict[str, Any]:
        return dict(self._asdict())


TransitionSpec = Transition  # the reference's name for a spec row


_FIELDS = ("name", "env_id", "version", "states", "initial_state", "terminal_states", "event_vocabulary",
           "transitions", "notes")


@dataclass
class RMSpec:
    """A parsed spec.  `states` and `transitions` are plain lists (completion appends rows in place, and a
    caller may reorder `states`, which decides the completion order)."""
    name: str
    env_id: str
    version: str
    states: List[str]
    initial_state: str
    terminal_states: List[str]
    event_vocabulary: List[str]
    transitions: List[Transition] = field(default_factory=list)
    notes: Optional[str] = None

    @classmethod
    def from_dict(cls, doc: Mapping[str, Any]) -> "RMSpec":
        return spec_from_mapping(doc)

    def to_dict(self) -> Dict[str, Any]:
        out = {k: getattr(self, k) for k in _FIELDS}
        out["transitions"] = [t.to_dict() for t in self.transitions]
        return out

    def rows(self) -> List[Transition]:
        return list(self.transitions)


def spec_from_mapping(doc: Mapping[str, Any]) -> RMSpec:
    """The spec document (already decoded) -> RMSpec; a missing required key raises KeyError."""
    return RMSpec(name=doc["name"], env_id=str(doc["env_id"]).strip().lower(), version=doc["version"],
                  states=list(doc["states"]), initial_state=doc["initial_state"],
                  terminal_states=list(doc.get("terminal_states") or []),
                  event_vocabulary=list(doc["event_vocabulary"]),
                  transitions=[Transition.from_mapping(r) for r in doc.get("transitions") or []],
                  notes=doc.get("notes"))


def read_spec(path: Union[str, Path]) -> RMSpec:
    """Decode a spec file: JSON, or YAML (safe loader, executes nothing) when it is not JSON and not named
    *.json.  Every decode / shape problem is a ValueError naming the file; a missing file FileNotFoundError."""
    p = Path(path)
    if not p.exists():
        raise FileNotFoundError(f"no RM spec at {p}")
    if not p.is_file():
        raise ValueError(f"{p} is not a file")
    text = p.read_text(encoding="utf-8")
    try:
        doc = json.loads(text)
    except json.JSONDecodeError as err:
        if p.suffix.lower() == ".json":
            raise ValueError(f"{p}: not valid JSON ({err})") from err
        import yaml

        try:
            doc = yaml.safe_load(text)
        except yaml.YAMLError as err2:
            raise ValueError(f"{p}: neither JSON nor YAML ({err2})") from err2
    if not isinstance(doc, dict):
        raise ValueError(f"{p}: the spec must be a mapping at the top level")
    try:
        return spec_from_mapping(doc)
    except KeyError as err:
        raise ValueError(f"{p}: required field {err} is missing") from err
    except ValueError as err:
        raise ValueError(f"{p}: {err}") from err


load_rmspec = read_spec


# --------------------------------------------------------------------------------------------------------------
# rules
# --------------------------------------------------------------------------------------------------------------
def _dupes(items: Sequence[Any]) -> List[Any]:
    seen, out = set(), []
    for x in items:
        if x in seen:
            out.append(x)
        seen.add(x)
    return out


def spec_problems(spec: RMSpec) -> Iterator[str]:
    """Every structural rule the spec breaks, in a fixed order: non-empty and duplicate-free state list,
    vocabulary and row list; initial / terminal states declared; every row between declared states on a
    declared event; the initial state touched by some row; at most one target per (state, event)."""
    states, vocab = set(spec.states), set(spec.event_vocabulary)
    if not spec.states:
        yield "no states declared"
    for s in _dupes(spec.states):
        yield f"state {s!r} declared twice"
    if spec.initial_state not in states:
        yield f"initial state {spec.initial_state!r} is not a declared state"
    for s in spec.terminal_states:
        if s not in states:
            yield f"terminal state {s!r} is not a declared state"
    for s in _dupes(spec.terminal_states):
        yield f"terminal state {s!r} listed twice"
    if not spec.event_vocabulary:
        yield "empty event vocabulary"
    for e in _dupes(spec.event_vocabulary):
        yield f"event {e!r} declared twice"
    if not spec.transitions:
        yield "no transitions"
    for t in spec.transitions:
        for what, s in (("source", t.from_state), ("target", t.to_state)):
            if s not in states:
                yield f"row {tuple(t)}: {what} state {s!r} is not declared"
        if t.event not in vocab:
            yield f"row {tuple(t)}: event {t.event!r} is not in the vocabulary"
    if spec.transitions and not any(spec.initial_state in (t.from_state, t.to_state) for t in spec.transitions):
        yield f"no row enters or leaves the initial state {spec.initial_state!r}"
    target: Dict[Tuple[str, Any], str] = {}
    for t in spec.transitions:
        prev = target.setdefault((t.from_state, t.event), t.to_state)
        if prev != t.to_state:
            yield f"({t.from_state!r}, {t.event!r}) leads to both {prev!r} and {t.to_state!r}"


def reward_problems(spec: RMSpec, *, max_positive_reward_transitions: Optional[int] = None,
                    terminal_reward_must_be_zero: bool = True) -> Iterator[str]:
    """Reward rules: at most N rewarding rows; no reward on rows leaving a terminal state."""
    if max_positive_reward_transitions is not None:
        n = sum(1 for t in spec.transitions if t.reward > 0)
        if n > max_positive_reward_transitions:
            yield f"{n} rows carry a positive reward, the limit is {max_positive_reward_transitions}"
    if terminal_reward_must_be_zero:
        term = set(spec.terminal_states)
        for t in spec.transitions:
            if t.from_state in term and t.reward != 0:
                yield f"row {tuple(t)} leaves terminal state {t.from_state!r} with reward {t.reward}"


def _raise_first(problems: Iterable[str]) -> None:
    for msg in problems:
        raise ValidationError(msg)


def validate_spec(spec: RMSpec) -> None:
    _raise_first(spec_problems(spec))


def validate_semantics(spec: RMSpec, *, max_positive_reward_transitions: Optional[int] = None,
                       terminal_reward_must_be_zero: bool = True) -> None:
    _raise_first(reward_problems(spec, max_positive_reward_transitions=max_positive_reward_transitions,
                                 terminal_reward_must_be_zero=terminal_reward_must_be_zero))


# --------------------------------------------------------------------------------------------------------------
# completion and event expansion
# --------------------------------------------------------------------------------------------------------------
def completion_rows(spec: RMSpec, default_reward: float = 0.0, terminal_self_loop: bool = True) -> List[Transition]:
    """The self loops (reward `default_reward`) that give every (state, event) of states x vocabulary a row,
    in that nested order; terminal states get none unless `terminal_self_loop`."""
    have = {(t.from_state, t.event) for t in spec.transitions}
    term = set(spec.terminal_states)
    return [Transition(s, e, s, float(default_reward)) for s in spec.states for e in spec.event_vocabulary
            if (s, e) not in have and (terminal_self_loop or s not in term)]


def complete_missing_transitions(spec: RMSpec, default_reward: float = 0.0, terminal_self_loop: bool = True):
    """Append completion_rows(spec) to the spec (in place); returns (spec, {"added": n})."""
    rows = completion_rows(spec, default_reward, terminal_self_loop)
    spec.transitions.extend(rows)
    return spec, {"added": len(rows)}


def _targets(event: Any, mapping: Mapping[str, object]) -> List[Any]:
    if event not in mapping:
        raise ValueError(f"event {event!r} has no entry in the event mapping (mapped: {sorted(mapping)})")
    tgt = mapping[event]
    cells = list(tgt) if isinstance(tgt, (list, set, frozenset)) else [tgt]
    if tgt is None or not cells:
        raise ValueError(f"event {event!r} maps to nothing")
    for c in cells:
        try:
            hash(c)
        except TypeError as err:
            raise ValueError(f"event {event!r} maps to an unhashable {c!r}") from err
    return cells


def expand_rows(rows: Iterable[Transition], mapping: Optional[Mapping[str, object]]) -> Dict[Tuple[Any, Any], Tuple[str, float]]:
    """Rows -> the RM transition map {(state, env_event): (state', reward)} in row order.  With a mapping every
    spec event becomes its cell (or one row per cell of a list); two rows that land on one key must agree."""
    out: Dict[Tuple[Any, Any], Tuple[str, float]] = {}
    for t in rows:
        for ev in (_targets(t.event, mapping) if mapping else [t.event]):
            key, val = (t.from_state, ev), (t.to_state, t.reward)
            if mapping and key in out and out[key] != val:
                raise ValueError(f"{key} maps to both {out[key]} and {val}")
            out[key] = val
    return out


def compile_transition_map(spec: RMSpec, event_mapping: Optional[Mapping[str, object]] = None):
    return expand_rows(spec.transitions, event_mapping)


def compile_reward_machine(spec: RMSpec, *, event_mapping: Optional[Mapping[str, object]] = None,
                           complete_missing_transitions: bool = False, default_reward: float = 0.0,
                           terminal_self_loop: bool = True, max_positive_reward_transitions: Optional[int] = None,
                           terminal_reward_must_be_zero: bool = True) -> RewardMachineSpec:
    """complete (optional) -> rules -> event expansion -> the RM structure, indexed from the spec's initial
    state (the order the reference's compile_reward_machine applies them in)."""
    if complete_missing_transitions:
        spec.transitions.extend(completion_rows(spec, default_reward, terminal_self_loop))
    validate_spec(spec)
    validate_semantics(spec, max_positive_reward_transitions=max_positive_reward_transitions,
                       terminal_reward_must_be_zero=terminal_reward_must_be_zero)
    return RewardMachineSpec(expand_rows(spec.transitions, event_mapping), initial_state=spec.initial_state)


# --------------------------------------------------------------------------------------------------------------
# dense tables
# --------------------------------------------------------------------------------------------------------------
@dataclass
class DenseRM:
    """One agent's RM as the kernels read it: next_q / reward per (state index, event column); a missing
    (state, event) is a zero-reward self loop (reward_machine.py:45-59).  Column 0 is the detector's None."""
    labels: List[Any]        # state label of each index (initial first, the rest sorted)
    next_q: np.ndarray       # uint8 [Q][E]
    reward: np.ndarray       # float64 [Q][E]
    init_q: int
    final_q: int             # -1 when the map is empty

    @classmethod
    def build(cls, rm: RewardMachineSpec, event_column: Mapping[Any, int], n_events: int,
              n_states: Optional[int] = None) -> "DenseRM":
        idx = rm.state_indices
        Q = n_states or len(idx)
        nq = np.repeat(np.arange(Q, dtype=np.uint8)[:, None], n_events, axis=1)
        rw = np.zeros((Q, n_events), np.float64)
        for (src, ev), (dst, r) in rm.transitions.items():
            col = 0 if ev is None else event_column.get(ev)
            if col is None:
                continue  # an event this agent's detector never emits: a dead row (still indexed)
            nq[idx[src], col] = idx[dst]
            rw[idx[src], col] = float(r)
        fs = rm.get_final_state()
        labels = [None] * len(idx)
        for s, i in idx.items():
            labels[i] = s
        return cls(labels, nq, rw, idx[rm.initial_state], idx[fs] if fs in idx else -1)


def compile_dense(spec: RMSpec, event_column: Mapping[Any, int], n_events: int, **compile_kw) -> DenseRM:
    """Spec -> dense tables in one call (compile_reward_machine's options, e.g. event_mapping / completion)."""
    return DenseRM.build(compile_reward_machine(spec, **compile_kw), event_column, n_events)


# --------------------------------------------------------------------------------------------------------------
# the entry points' event vocabularies
# --------------------------------------------------------------------------------------------------------------
def frozenlake_event_mapping(goals: Mapping[str, tuple]) -> Dict[str, object]:
    """Each goal letter L as "L" and "at(L)" -> its cell (frozen_lake_main.py:125-130)."""
    return {k: tuple(pos) for label, pos in goals.items() for k in (f"at({label})", label)}


def officeworld_event_mapping(coords: Mapping[str, list], goals: Mapping[str, tuple]) -> Dict[str, object]:
    """Goal letters as in FrozenLake, "office" / "at(office)" -> O, "coffee" / "at(coffee)" -> every coffee
    cell, "letter" / "email" / "at(letter)" / "at(email)" -> every letter cell (office_main.py:461-485)."""
    out = frozenlake_event_mapping(goals)
    if "O" in goals:
        out.update({"office": tuple(goals["O"]), "at(office)": tuple(goals["O"])})
    groups = (("coffee", ("coffee", "at(coffee)")), ("letter", ("letter", "email", "at(letter)", "at(email)")))
    for kind, names in groups:
        cells = [tuple(p) for p in (coords.get(kind) or [])]
        if cells:
            out.update({n: list(cells) for n in names})
    return out


def officeworld_detector_positions(coords, goals, base_positions) -> set:
    """The OfficeWorld runner's detector with an --rm-spec: its position_map plus every mapped cell
    (office_main.py:487-495)."""
    cells = {tuple(p) for p in base_positions}
    for tgt in officeworld_event_mapping(coords, goals).values():
        cells.update(tgt if isinstance(tgt, list) else [tgt])
    return cells
