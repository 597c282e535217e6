"""Host table compiler vs the reference's own parse / index / final-state / potential results
(tests/golden/tables.json, produced by tests/golden/gen_golden.py from the reference)."""
import json
import os

import numpy as np
import pytest

from rmx import maps, tables as T


@pytest.fixture(scope="module")
def ref(golden_dir):
    with open(os.path.join(golden_dir, "tables.json")) as f:
        return json.load(f)


def _tl(v):
    return [tuple(x) for x in v]


def test_frozen_lake_map1_parse(ref):
    holes, goals, dims = T.parse_map_emoji(maps.FROZEN_LAKE_LAYOUTS["map1"])
    r = ref["fl_map1"]
    assert holes == _tl(r["holes"])
    assert {k: tuple(v) for k, v in goals.items()} == {k: tuple(v) for k, v in r["goals"].items()}
    assert dims == tuple(r["dims"]) == (10, 10)


@pytest.mark.parametrize("m", ["map0", "map1", "map2", "map3", "map4"])
def test_office_world_parse(ref, m):
    coords, goals, walls = T.parse_office_world(maps.OFFICE_WORLD_MAPS[m]["layout"])
    r = ref[f"ow_{m}"]
    for k in ("plant", "coffee", "letter", "empty_cell"):
        assert coords[k] == _tl(r["coords"][k]), k
    assert {k: tuple(v) for k, v in goals.items()} == {k: tuple(v) for k, v in r["goals"].items()}
    assert [(tuple(a), tuple(b)) for a, b in walls] == [(tuple(a), tuple(b)) for a, b in r["walls"]]
    assert tuple(maps.OFFICE_WORLD_MAPS[m]["grid_size"]) == tuple(r["grid_size"])


def test_office_world_map1_counts(ref):
    # 39 undirected wall pairs, 6 plants, 2 coffee, 1 letter, 9 event cells
    coords, goals, walls = T.parse_office_world(maps.OFFICE_WORLD_MAPS["map1"]["layout"])
    assert len(walls) == 39 and len(coords["plant"]) == 6 and len(coords["coffee"]) == 2
    assert len(ref["ow_map1"]["position_map"]) == 9


@pytest.mark.parametrize("m", ["map0", "map1", "map2", "map3", "map4"])
def test_office_world_experiments(ref, m):
    sym, _ = T.scenario_symbols({"kind": "office_world", "map": m})
    for ex, rows in ref[f"ow_{m}_experiments"].items():
        mine = maps.office_world_experiment(m, ex)
        assert [(a, tuple(sym[e]), b, r) for a, e, b, r in mine] == [(a, tuple(e), b, r) for a, e, b, r in rows], ex


def _rm(rows):
    sym = {k: (i, 100 + i) for i, k in enumerate("ABCDEO")}
    sym.update({"coffee0": (50, 1), "coffee1": (50, 2), "letter0": (50, 3)})
    return T._rm_from_rows(rows, sym)


def test_rm_structure_matches_reference(ref):
    for name, r in ref["rm"].items():
        rm = _rm(r["rows"])
        assert rm.state_indices == r["state_indices"], name
        assert rm.get_final_state() == r["final"], name
        assert rm.initial_state == r["initial"], name
        assert rm.numbers_state() == r["numbers_state"], name
        assert rm.get_all_states() == r["all_states"], name
        rm.add_reward_shaping(0.9, 0.9)
        for k, v in r["potentials"].items():
            assert rm.potentials[k] == pytest.approx(v, abs=1e-12), (name, k)
        rm.add_distance_reward_shaping(0.9, 0.9, alpha=100)
        assert rm.potentials == r["distance_potentials"], name


def test_exp5_potentials_survey_values():
    sc = T.compile_scenario(T.baseline_scenario(5))
    pots = sc.rms[0].potentials
    assert pots["state0"] == pytest.approx(-0.531441) and pots["state8"] == 0 and pots["state7"] == pytest.approx(-1.0)


def test_reference_rm_unit_kats():
    # test_reward_machine.py:12-41 (structure part), test_reward_machine_shaping.py:9-17,
    # test_reward_machine_extras.py:12-25
    rm = T.RewardMachineSpec({("q0", "a"): ("q1", 1), ("q1", "b"): ("qf", 2)})
    assert rm.numbers_state() == 3 and rm.get_state_index("q0") == 0 and rm.get_state_from_index(1) == "q1"
    rm = T.RewardMachineSpec({("q0", "a"): ("q1", 0), ("q1", "b"): ("qf", 1)})
    rm.add_distance_reward_shaping(gamma=0.9, rs_gamma=0.9, alpha=5)
    assert (rm.potentials["qf"], rm.potentials["q1"], rm.potentials["q0"]) == (0, -5, -10)
    rm = T.RewardMachineSpec({("q0", "a"): ("q1", 0)})
    assert rm.get_distance("q_missing") == 999999
    V = rm.value_iteration(list(rm.state_indices), rm.get_delta_u(), rm.get_delta_r(), rm.get_final_state(), 0.9)
    assert V[rm.get_final_state()] == 0
    with pytest.raises(ValueError):
        rm.get_state_from_index(7)


def test_parse_kats():
    # test_utils_encoding.py:49-69
    holes, goals, dims = T.parse_map_emoji("""
        🟩 🟩
        ⛔ 1
        """)
    assert holes == [(0, 1)] and goals == {"1": (1, 1)} and dims == (2, 2)
    coords, g, walls = T.parse_office_world("""
    🟩 🪴
    🥤 ✉️
    """)
    assert coords["plant"] == [(1, 0)] and coords["coffee"] == [(0, 1)] and coords["letter"] == [(1, 1)]
    assert g == {} and isinstance(walls, list)


def test_cell_tile_boundaries_and_walls():
    # FrozenLake: up = y-1 with boundary clamp (test_ma_frozen_lake.py:46-58)
    tile = T.cell_tile(T.FROZEN_LAKE, 2, 2, [])
    assert tile[0] == T.CAN_DOWN | T.CAN_RIGHT
    assert tile[3] == T.CAN_UP | T.CAN_LEFT
    # OfficeWorld: up = y+1, walls block (config_office.py:12-39)
    tile = T.cell_tile(T.OFFICE_WORLD, 2, 2, [(1, 1)], walls=[((0, 0), (1, 0)), ((1, 0), (0, 0))])
    assert tile[0] == T.CAN_UP
    assert tile[3] == T.CAN_DOWN | T.CAN_LEFT | T.HAZARD


def test_office_map1_tile_matches_can_move(ref):
    sc = T.compile_scenario(T.baseline_scenario(3))
    walls = {(tuple(a), tuple(b)) for a, b in ref["ow_map1"]["walls"]}
    walls |= {(b, a) for a, b in walls}
    W, H = 12, 9
    for y in range(H):
        for x in range(W):
            bits = int(sc.cell[y * W + x])
            assert bool(bits & T.CAN_UP) == (y < H - 1 and ((x, y), (x, y + 1)) not in walls)
            assert bool(bits & T.CAN_DOWN) == (y > 0 and ((x, y), (x, y - 1)) not in walls)
            assert bool(bits & T.CAN_LEFT) == (x > 0 and ((x, y), (x - 1, y)) not in walls)
            assert bool(bits & T.CAN_RIGHT) == (x < W - 1 and ((x, y), (x + 1, y)) not in walls)
    assert sc.n_events == 10 and sc.n_rm_states == 5


def test_dense_rm_table_semantics():
    sc = T.compile_scenario(T.baseline_scenario(2))
    assert (sc.n_rm_states, sc.n_events) == (4, 4)
    assert list(sc.final_q) == [3, 3] and list(sc.init_q) == [0, 0]
    # missing (q, e) is a zero-reward self loop (reward_machine.py:55-59)
    assert np.all(sc.next_q[:, :, 0] == np.arange(4)[None, :])
    assert np.all(sc.rm_reward[:, :, 0] == 0)
    A_id = sc.event_cells.index((4, 4)) + 1
    assert sc.next_q[0, 0, A_id] == 1 and sc.rm_reward[0, 0, A_id] == 10
