"""On-disk Reward Machine specs (JSON / YAML ``RMSpec``) -> the structure the table compiler consumes.

SURVEY.md §8(f) #3: the spec -> transition-map compile that lets ``--rm-spec`` RMs feed the kernel
tables.  Restated from (paths relative to multiagent_rlrm/):

* ``RMSpec`` / ``TransitionSpec`` (reward coercion "r0.5" -> 0.5)      rmgen/spec.py:5-98
* ``load_rmspec`` (JSON, YAML via safe_load)                          rmgen/io.py:17-77
* ``validate_schema`` / ``ensure_deterministic`` / ``validate_semantics`` rmgen/validator.py:18-103
* ``complete_missing_transitions`` (states x vocabulary self loops)     rmgen/completion.py:6-38
* ``_compile_transition_map`` (event -> position(s) expansion)          rmgen/io.py:80-123
* ``compile_reward_machine`` (initial-state override, re-indexing)      rmgen/io.py:126-171
* the FrozenLake / OfficeWorld event mappings of the entry points
  (frozen_lake_main.py:125-130, office_main.py:461-485)

The LLM authoring / normalisation parts of rmgen are out of scope.
Note the reference's final-state rule applies to the compiled map: the "final" state is the target of
the LAST inserted row, which after completion is a self loop in ``states`` order.
"""
from __future__ import annotations

import json
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, Dict, List, Mapping, Optional, Tuple, Union

from .tables import RewardMachineSpec


class ValidationError(Exception):
    """An RMSpec failed validation (rmgen/validator.py:6-7)."""


@dataclass
class TransitionSpec:
    from_state: str
    event: str
    to_state: str
    reward: float

    @staticmethod
    def _coerce_reward(raw: Any, data: Dict[str, Any]) -> float:
        if isinstance(raw, bool):
            raise ValueError(f"Invalid reward type '{type(raw)}' in transition {data}")
        if isinstance(raw, (int, float)):
            return float(raw)
        if isinstance(raw, str):
            txt = raw.strip()
            if txt.lower().startswith("r"):
                txt = txt[1:]
            try:
                return float(txt)
            except ValueError as exc:
                raise ValueError(f"Invalid reward value '{raw}' in transition {data}") from exc
        raise ValueError(f"Invalid reward type '{type(raw)}' in transition {data}")

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "TransitionSpec":
        return cls(d["from_state"], d["event"], d["to_state"], cls._coerce_reward(d["reward"], d))

    def to_dict(self):
        return {"from_state": self.from_state, "event": self.event, "to_state": self.to_state, "reward": self.reward}


@dataclass
class RMSpec:
    name: str
    env_id: str
    version: str
    states: List[str]
    initial_state: str
    terminal_states: List[str]
    event_vocabulary: List[str]
    transitions: List[TransitionSpec] = field(default_factory=list)
    notes: Optional[str] = None

    @classmethod
    def from_dict(cls, d: Dict[str, Any]) -> "RMSpec":
        return cls(name=d["name"], env_id=d["env_id"].strip().lower(), version=d["version"], states=list(d["states"]),
                   initial_state=d["initial_state"], terminal_states=list(d.get("terminal_states", [])),
                   event_vocabulary=list(d["event_vocabulary"]),
                   transitions=[TransitionSpec.from_dict(t) for t in d.get("transitions", [])], notes=d.get("notes"))

    def to_dict(self):
        return {"name": self.name, "env_id": self.env_id, "version": self.version, "states": self.states,
                "initial_state": self.initial_state, "terminal_states": self.terminal_states,
                "event_vocabulary": self.event_vocabulary, "transitions": [t.to_dict() for t in self.transitions],
                "notes": self.notes}

    def as_transition_map(self):
        return {(t.from_state, t.event): (t.to_state, t.reward) for t in self.transitions}


def load_rmspec(path: Union[str, Path]) -> RMSpec:
    src = Path(path)
    if not src.exists():
        raise FileNotFoundError(f"RM spec file not found: {src}")
    if not src.is_file():
        raise ValueError(f"RM spec path is not a file: {src}")
    text = src.read_text(encoding="utf-8")
    try:
        data = json.loads(text)
    except json.JSONDecodeError as exc:
        if src.suffix.lower() == ".json":
            raise ValueError(f"Invalid JSON in {src}: {exc}") from exc
        import yaml
        try:
            data = yaml.safe_load(text)
        except Exception as exc2:
            raise ValueError(f"Invalid YAML in {src}: {exc2}") from exc2
    if not isinstance(data, dict):
        raise ValueError(f"RM spec must be a JSON/YAML object at top-level: {src}")
    try:
        return RMSpec.from_dict(data)
    except KeyError as exc:
        raise ValueError(f"RM spec missing required field {exc!s}: {src}") from exc
    except ValueError as exc:
        raise ValueError(f"RM spec has invalid values: {src}: {exc}") from exc


def _unique(items, label):
    seen = set()
    for it in items:
        if it in seen:
            raise ValidationError(f"Duplicate {label}: {it}")
        seen.add(it)


def validate_schema(spec: RMSpec) -> None:
    if not spec.states:
        raise ValidationError("states must be non-empty")
    _unique(spec.states, "state")
    if spec.initial_state not in spec.states:
        raise ValidationError(f"initial_state {spec.initial_state} not in states")
    for s in spec.terminal_states:
        if s not in spec.states:
            raise ValidationError(f"terminal_state {s} not in states")
    _unique(spec.terminal_states, "terminal_state")
    if not spec.event_vocabulary:
        raise ValidationError("event_vocabulary must be non-empty")
    _unique(spec.event_vocabulary, "event")
    if not spec.transitions:
        raise ValidationError("transitions must be non-empty")
    states, events = set(spec.states), set(spec.event_vocabulary)
    for t in spec.transitions:
        if t.from_state not in states:
            raise ValidationError(f"transition from_state {t.from_state} not in states")
        if t.to_state not in states:
            raise ValidationError(f"transition to_state {t.to_state} not in states")
        if t.event not in events:
            raise ValidationError(f"transition event {t.event} not in vocabulary")
    if not any(t.from_state == spec.initial_state or t.to_state == spec.initial_state for t in spec.transitions):
        raise ValidationError(f"initial_state {spec.initial_state} has no incident transitions")


def ensure_deterministic(spec: RMSpec) -> None:
    seen: Dict[Tuple[str, str], str] = {}
    for t in spec.transitions:
        k = (t.from_state, t.event)
        if k in seen and seen[k] != t.to_state:
            raise ValidationError(f"Non-deterministic transitions for {k}: {seen[k]} vs {t.to_state}")
        seen[k] = t.to_state


def validate_spec(spec: RMSpec) -> None:
    validate_schema(spec)
    ensure_deterministic(spec)


def validate_semantics(spec: RMSpec, *, max_positive_reward_transitions: int = None,
                       terminal_reward_must_be_zero: bool = True) -> None:
    if max_positive_reward_transitions is not None:
        pos = [t for t in spec.transitions if t.reward > 0]
        if len(pos) > max_positive_reward_transitions:
            raise ValidationError(f"Positive-reward transitions exceed limit {max_positive_reward_transitions}: {pos}")
    if terminal_reward_must_be_zero:
        term = set(spec.terminal_states)
        bad = [t for t in spec.transitions if t.from_state in term and t.reward != 0]
        if bad:
            raise ValidationError(f"Terminal transitions must have reward 0. Offenders: {bad}")


def complete_missing_transitions(spec: RMSpec, default_reward: float = 0.0, terminal_self_loop: bool = True):
    """Self loops with ``default_reward`` for every missing (state, event) in states x vocabulary order,
    appended in place (completion.py:6-38)."""
    existing = {(t.from_state, t.event) for t in spec.transitions}
    if not spec.states or not spec.event_vocabulary:
        return spec, {"added": 0}
    added = []
    for s in spec.states:
        for ev in spec.event_vocabulary:
            if (s, ev) in existing:
                continue
            if s in spec.terminal_states and not terminal_self_loop:
                continue
            added.append(TransitionSpec(s, ev, s, default_reward))
    spec.transitions.extend(added)
    return spec, {"added": len(added)}


def compile_transition_map(spec: RMSpec, event_mapping: Optional[Mapping[str, object]] = None):
    """Spec rows -> {(state, env_event): (state', reward)}; a mapped list expands to one row per
    position; conflicting expansions raise (io.py:80-123)."""
    if not event_mapping:
        return spec.as_transition_map()
    out: Dict[Tuple[object, object], Tuple[object, object]] = {}
    for t in spec.transitions:
        if t.event not in event_mapping:
            raise ValueError(f"Unknown event '{t.event}' in RMSpec; missing from event mapping "
                             f"(available: {sorted(event_mapping.keys())})")
        mapped = event_mapping[t.event]
        if mapped is None:
            raise ValueError(f"Event mapping for '{t.event}' is None")
        evs = list(mapped) if isinstance(mapped, (list, set, frozenset)) else [mapped]
        if not evs:
            raise ValueError(f"Event mapping for '{t.event}' is empty")
        for ev in evs:
            try:
                hash(ev)
            except TypeError as exc:
                raise ValueError(f"Mapped event for '{t.event}' is not hashable: {ev!r}") from exc
            key, val = (t.from_state, ev), (t.to_state, t.reward)
            if key in out and out[key] != val:
                raise ValueError(f"Event mapping produced conflicting transitions for {key}: {out[key]} vs {val}")
            out[key] = val
    return out


def compile_reward_machine(spec: RMSpec, *, event_mapping: Optional[Mapping[str, object]] = None,
                           complete_missing_transitions: bool = False, default_reward: float = 0.0,
                           terminal_self_loop: bool = True, max_positive_reward_transitions: int = None,
                           terminal_reward_must_be_zero: bool = True) -> RewardMachineSpec:
    """Validate + compile an RMSpec into the RM structure of the tables (io.py:126-171)."""
    if complete_missing_transitions:
        spec, _ = globals()["complete_missing_transitions"](spec, default_reward=default_reward,
                                                           terminal_self_loop=terminal_self_loop)
    validate_spec(spec)
    validate_semantics(spec, max_positive_reward_transitions=max_positive_reward_transitions,
                       terminal_reward_must_be_zero=terminal_reward_must_be_zero)
    trans = compile_transition_map(spec, event_mapping=event_mapping)
    # RewardMachine(transitions, detector), then initial_state/current_state override + re-indexing
    return RewardMachineSpec(trans, initial_state=spec.initial_state)


def frozenlake_event_mapping(goals: Mapping[str, tuple]) -> Dict[str, object]:
    """label and at(label) -> goal cell (frozen_lake_main.py:125-130)."""
    m: Dict[str, object] = {}
    for label, pos in goals.items():
        m[f"at({label})"] = tuple(pos)
        m[label] = tuple(pos)
    return m


def officeworld_event_mapping(coords: Mapping[str, list], goals: Mapping[str, tuple]) -> Dict[str, object]:
    """Goal labels, office / coffee / letter / email aliases (office_main.py:461-485)."""
    m: Dict[str, object] = {}
    for label, pos in goals.items():
        m[f"at({label})"] = tuple(pos)
        m[label] = tuple(pos)
    if "O" in goals:
        m["office"] = tuple(goals["O"])
        m["at(office)"] = tuple(goals["O"])
    coffee = [tuple(p) for p in (coords.get("coffee") or [])]
    if coffee:
        m["coffee"] = list(coffee)
        m["at(coffee)"] = list(coffee)
    letter = [tuple(p) for p in (coords.get("letter") or [])]
    if letter:
        for k in ("letter", "email", "at(letter)", "at(email)"):
            m[k] = list(letter)
    return m


def officeworld_detector_positions(coords, goals, base_positions) -> set:
    """The OW runner's detector: position_map plus every mapped position (office_main.py:487-495)."""
    pos = set(tuple(p) for p in base_positions)
    for v in officeworld_event_mapping(coords, goals).values():
        if isinstance(v, list):
            pos.update(v)
        else:
            pos.add(v)
    return pos
