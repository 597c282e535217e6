"""RMSpec -> RM structure (rmx.rmspec) vs the reference's compile_reward_machine on its own fixture
specs (tests/golden/tables.json["rmspec"], tests/golden/specs/ = the reference's tests/fixtures), plus the
reference's rmgen unit KATs (test_rmgen_completion.py, test_rmspec_io.py)."""
import json
import os

import numpy as np
import pytest

from rmx import rmspec as R
from rmx import tables as T


@pytest.fixture(scope="module")
def ref(golden_dir):
    with open(os.path.join(golden_dir, "tables.json")) as f:
        return json.load(f)["rmspec"]


def _ev(e):
    return tuple(e) if isinstance(e, list) else e


def test_compile_matches_reference(ref, golden_dir):
    for key, want in ref.items():
        name, order, complete, dr, tsl = key.split("|")
        spec = R.load_rmspec(os.path.join(golden_dir, "specs", f"{name}.json"))
        if order != "-":
            spec.states = order.split(",")
        if "error" in want:
            with pytest.raises((R.ValidationError, ValueError)):
                R.compile_reward_machine(spec, complete_missing_transitions=bool(int(complete)),
                                         default_reward=float(dr), terminal_self_loop=bool(int(tsl)),
                                         terminal_reward_must_be_zero=False)
            continue
        rm = R.compile_reward_machine(spec, complete_missing_transitions=bool(int(complete)), default_reward=float(dr),
                                      terminal_self_loop=bool(int(tsl)), terminal_reward_must_be_zero=False)
        rows = [[k[0], _ev(k[1]), v[0], v[1]] for k, v in rm.transitions.items()]
        assert rows == [[a, _ev(b), c, d] for a, b, c, d in want["rows"]], key
        assert rm.state_indices == want["state_indices"], key
        assert rm.initial_state == want["initial"] and rm.get_final_state() == want["final"], key
        assert rm.numbers_state() == want["numbers_state"] and rm.get_all_states() == want["all_states"], key


def _partial():
    return R.RMSpec.from_dict({"name": "partial", "env_id": "env", "version": "1.0", "states": ["q0", "q1"],
                               "initial_state": "q0", "terminal_states": ["q1"], "event_vocabulary": ["e1", "e2"],
                               "transitions": [{"from_state": "q0", "event": "e1", "to_state": "q1", "reward": 1}]})


def test_completion_kats():
    # test_rmgen_completion.py
    spec, report = R.complete_missing_transitions(_partial(), default_reward=0.0)
    assert report["added"] == 3 and len(spec.transitions) == 4
    spec, _ = R.complete_missing_transitions(_partial(), default_reward=0.5)
    assert next(t for t in spec.transitions if t.from_state == "q1" and t.event == "e2").reward == 0.5
    spec, _ = R.complete_missing_transitions(_partial(), terminal_self_loop=True)
    assert any(t.from_state == "q1" and t.event == "e1" and t.to_state == "q1" for t in spec.transitions)
    spec, rep = R.complete_missing_transitions(_partial(), terminal_self_loop=False)
    assert rep["added"] == 1


def test_rmspec_io_kat(golden_dir):
    # test_rmspec_io.py: compile without an event mapping -> string events
    rm = R.compile_reward_machine(R.load_rmspec(os.path.join(golden_dir, "specs", "officeworld_simple.json")))
    assert rm.transitions[("q1", "at(G)")] == ("q2", 1.0)


def test_reward_coercion_and_errors(tmp_path):
    assert R.parse_reward("r0.5") == 0.5 and R.parse_reward(2) == 2.0 and R.parse_reward(" R3 ") == 3.0
    for bad in ("abc", True, None, [1]):
        with pytest.raises(ValueError):
            R.parse_reward(bad)
    p = tmp_path / "spec.yaml"
    p.write_text("name: y\nenv_id: FrozenLake\nversion: '1'\nstates: [a, b]\ninitial_state: a\n"
                 "event_vocabulary: [at(A)]\ntransitions:\n  - {from_state: a, event: at(A), to_state: b, reward: r1}\n")
    spec = R.load_rmspec(p)
    assert spec.env_id == "frozenlake" and spec.transitions[0].reward == 1.0
    with pytest.raises(FileNotFoundError):
        R.load_rmspec(tmp_path / "missing.json")
    bad = tmp_path / "bad.json"
    bad.write_text("{not json")
    with pytest.raises(ValueError):
        R.load_rmspec(bad)


def test_terminal_reward_semantics():
    spec = _partial()
    spec.transitions.append(R.TransitionSpec("q1", "e2", "q1", 1.0))
    with pytest.raises(R.ValidationError):
        R.validate_semantics(spec)
    with pytest.raises(R.ValidationError):
        R.validate_semantics(spec, max_positive_reward_transitions=1, terminal_reward_must_be_zero=False)


def test_event_mapping_expansion_and_conflicts():
    spec = R.RMSpec.from_dict({"name": "m", "env_id": "officeworld", "version": "1", "states": ["q0", "q1"],
                               "initial_state": "q0", "terminal_states": ["q1"], "event_vocabulary": ["coffee"],
                               "transitions": [{"from_state": "q0", "event": "coffee", "to_state": "q1", "reward": 0}]})
    m = R.compile_transition_map(spec, {"coffee": [(3, 2), (8, 6)]})
    assert list(m) == [("q0", (3, 2)), ("q0", (8, 6))]
    with pytest.raises(ValueError):
        R.compile_transition_map(spec, {"other": (1, 1)})


def test_spec_scenarios_compile(configs):
    for name in ("fl2_spec", "ow2_spec"):
        tab = T.compile_scenario(configs[name])
        assert tab.n_agents == 2
    # q1 is the "final" state of the [q2, q0, q1]-ordered completed spec
    tab = T.compile_scenario(configs["fl2_spec"])
    assert tab.rms[1].get_final_state() == "q1" and tab.rms[0].get_final_state() == "q2"


def test_dense_tables_direct(ref, golden_dir, configs):
    """compile_dense: spec -> next_q / reward / init / final arrays, equal to what the table compiler builds from
    the same spec inside a scenario (fl2_spec agent 1: completed under states [q2, q0, q1], so q1 is "final")."""
    desc = configs["fl2_spec"]["agents"][1]["rm_spec"]
    sym, parsed = T.scenario_symbols(configs["fl2_spec"])
    mapping = R.frozenlake_event_mapping(parsed["goals"])
    tab = T.compile_scenario(configs["fl2_spec"])
    cols = {c: i + 1 for i, c in enumerate(tab.event_cells)}
    d = R.compile_dense(R.RMSpec.from_dict(desc["spec"]), cols, tab.n_events, event_mapping=mapping,
                        complete_missing_transitions=True, default_reward=desc["default_reward"],
                        terminal_reward_must_be_zero=False)
    Q = len(d.labels)
    assert (d.next_q == tab.next_q[1, :Q]).all() and np.allclose(d.reward, tab.rm_reward[1, :Q])
    assert d.init_q == tab.init_q[1] and d.final_q == tab.final_q[1] and d.labels[d.final_q] == "q1"


def test_rules_report_every_problem():
    spec = R.RMSpec.from_dict({"name": "bad", "env_id": "x", "version": "1", "states": ["a", "a"],
                               "initial_state": "z", "terminal_states": ["b"], "event_vocabulary": ["e"],
                               "transitions": [{"from_state": "a", "event": "f", "to_state": "c", "reward": 1}]})
    probs = list(R.spec_problems(spec))
    assert len(probs) == 6  # duplicate state, bad initial, bad terminal, bad target, bad event, untouched initial
    with pytest.raises(R.ValidationError):
        R.validate_spec(spec)


def test_officeworld_event_mapping_kat():
    """test_officeworld_event_context.py:65-135 from its normalised spec on (the event normalisation itself is the
    LLM-authoring side, out of scope): the OfficeWorld runner's event mapping over map1 (goal letters as "L" / "at(L)",
    office, every coffee and letter cell under all their names, office_main.py:461-485) compiles "at(A)" to A's cell:
    the RM steps q0 -> q1 with reward 1 there.  A coffee event expands to one row per coffee cell."""
    from rmx import maps
    coords, goals, _walls = T.parse_office_world(maps.OFFICE_WORLD_MAPS["map1"]["layout"])
    mapping = R.officeworld_event_mapping(coords, goals)
    assert mapping["office"] == mapping["at(office)"] == tuple(goals["O"])
    assert sorted(mapping["at(coffee)"]) == sorted(tuple(p) for p in coords["coffee"]) and len(coords["coffee"]) == 2
    assert mapping["email"] == mapping["at(letter)"] == [tuple(p) for p in coords["letter"]]
    spec = R.RMSpec.from_dict({"name": "smoke", "env_id": "officeworld", "version": "1.0", "states": ["q0", "q1"],
                               "initial_state": "q0", "terminal_states": ["q1"], "event_vocabulary": ["at(A)"],
                               "transitions": [{"from_state": "q0", "event": "at(A)", "to_state": "q1", "reward": 1}]})
    rm = R.compile_reward_machine(spec, event_mapping=mapping)
    assert rm.transitions[("q0", tuple(goals["A"]))] == ("q1", 1.0)
    assert rm.get_final_state() == "q1" and rm.state_indices == {"q0": 0, "q1": 1}
    spec = R.RMSpec.from_dict({"name": "c", "env_id": "officeworld", "version": "1.0", "states": ["q0", "q1"],
                               "initial_state": "q0", "terminal_states": ["q1"], "event_vocabulary": ["at(coffee)"],
                               "transitions": [{"from_state": "q0", "event": "at(coffee)", "to_state": "q1",
                                                "reward": 0}]})
    rm = R.compile_reward_machine(spec, event_mapping=mapping)
    assert sorted(ev for (_, ev) in rm.transitions) == sorted(tuple(p) for p in coords["coffee"])
