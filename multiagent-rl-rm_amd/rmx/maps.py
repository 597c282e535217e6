"""Built-in map layouts (data) and the experiment Reward Machines of the reference configs.

Layouts are the emoji strings of the reference configs, kept verbatim as data:
  FrozenLake  multiagent_rlrm/environments/frozen_lake/config_frozen_lake.py:12-26 (map1)
  OfficeWorld multiagent_rlrm/environments/office_world/config_office.py:49-255 (map0..map4),
              grid_size and the default agent start of each map alongside.
Experiments: symbolic restatement of get_experiment_for_map (config_office.py:275-457);
symbols resolve against the parsed map (goal letters, coffee0/coffee1/letter0).
"""

FROZEN_LAKE_LAYOUTS = {
    'map1': '\n              B 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n             🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n             🟩 🟩 🟩 ⛔ ⛔ 🟩 🟩 🟩 🟩 🟩\n             🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n             🟩 🟩 🟩 🟩 A  🟩 🟩 🟩 🟩 🟩\n             🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n             🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n             ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🟩 ⛔ ⛔\n             🟩 🟩 🟩 🟩  C 🟩 🟩 🟩 🟩 🟩\n             🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n            ',
}

OFFICE_WORLD_MAPS = {
    'map0': {"layout": '\n🥤 🟩 🟩 🟩 🟩 🟩 🟩 🟩 A  🥤\n🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\nC  🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 \n🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\nD  🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 B\n🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\n🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩 🟩\nO  🟩 🟩 🟩 E  🟩 🟩 🟩 🟩 ✉️\n',
             "grid_size": (10, 10), "start": (0, 0)},
    'map1': {"layout": '\n 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n 🟩 B  🟩 🚪 🟩 🪴 🟩 🚪 🟩 🪴 🟩 🚪 🟩 C  🟩\n 🟩 🟩 🟩 ⛔ 🥤 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔ \n 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n 🟩 🪴 🟩 ⛔ 🟩 O  🟩 ⛔ 🟩 ✉️ 🟩 ⛔ 🟩 🪴 🟩\n 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔\n 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🥤 ⛔ 🟩 🟩 🟩\n 🟩 A  🟩 🚪 🟩 🪴 🟩 🚪 🟩 🪴 🟩 🚪 🟩 D  🟩\n E  🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n ',
             "grid_size": (9, 12), "start": (2, 7)},
    'map2': {"layout": '\n  E 🪴 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🟩 🟩\n 🟩 B  🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🟩 🚪 🟩  D 🟩\n 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ 🚪 \n 🪴 🟩 🟩 ⛔ 🥤 🪴 🟩 🚪 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n 🟩 O  🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🪴 🟩\n 🟩 🟩 🟩 ⛔ 🥤 🟩 🟩 🚪 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ 🚪\n 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🪴 🟩 🟩 ⛔ 🟩 🟩 🟩\n 🟩 A  🟩 ⛔ 🟩 🪴 🟩 🚪 🟩 🟩 🟩 ⛔ 🪴 🟩 🟩\n 🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 ⛔ ✉️ 🟩 🪴 ⛔ 🟩 🟩 🟩\n 🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔\n 🟩 🟩 🟩 🚪 🪴 🪴 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n 🟩 🟩 🟩 ⛔ C  🟩 🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🟩\n 🪴 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🪴 🪴\n ',
             "grid_size": (12, 12), "start": (2, 7)},
    'map3': {"layout": '\n🟩 🪴 E  🚪 🟩 🟩 🪴 🚪 🪴 🪴 🪴 🚪 🪴 🟩 🟩 🚪 🟩 🪴 🟩\n🟩 A  🪴 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🪴 🚪 🟩 🟩 🟩 ⛔ 🟩 B  🟩\n🟩 🟩 🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🪴 ⛔ 🟩 🟩 🟩\n⛔ 🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ 🚪 🚪 ⛔\n🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 🚪 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n🟩 🪴 🟩 ⛔ ✉️ 🟩 🟩 ⛔ 🟩 🟩 🥤 ⛔ 🟩 🪴 🪴 ⛔ 🟩 🪴 🟩\n🟩 🟩 🟩 ⛔ 🪴 🪴 🪴 🚪 🟩 🪴 🪴 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n⛔ 🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ 🚪 ⛔\n🪴 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🟩 🟩\n🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 🚪 🟩 🪴 🟩 🚪 🟩 🪴 🟩 ⛔ 🟩 🟩 🟩\n🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 🚪 ⛔ ⛔ ⛔ 🚪 ⛔\n🟩 🟩 🪴 🚪 🪴 🟩 🥤 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🪴 🚪 🟩 🟩 🟩\n🟩 D  🟩 ⛔ 🪴 🟩 🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🪴 ⛔ 🪴 🟩 🟩\n🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔\n🟩 🟩 🟩 🚪 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n🟩 O  🟩 🚪 🟩 🪴 🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🟩 ⛔ 🟩 🟩 C\n🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 🚪 🟩 🟩 🟩\n',
             "grid_size": (15, 15), "start": (2, 7)},
    'map4': {"layout": '\n🟩 🪴 E  🚪 🟩 🟩 🪴 🚪 🪴 🪴 🪴 🚪 🪴 🟩 🟩 🚪 🟩 🪴 🥤\n🟩 A  🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🟩 ⛔ B  🟩 🟩\n🟩 🟩 🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🟩 🚪 🟩 🟩 🪴 ⛔ 🪴 🟩 🟩\n⛔ 🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ 🚪 🚪 ⛔\n🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 🚪 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n🟩 🪴 🟩 ⛔ ✉️ 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🪴 🪴 ⛔ 🪴 🪴 🟩\n🟩 🟩 🟩 ⛔ 🪴 🪴 🪴 🚪 🟩 🪴 🪴 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n⛔ 🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ 🚪 ⛔\n🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🟩 🟩\n🟩 🪴 🟩 ⛔ 🟩 🪴 🟩 🚪 🟩 🪴 🟩 🚪 🟩 🪴 🟩 ⛔ 🟩 🪴 🟩\n🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ 🚪 🚪 ⛔ ⛔ ⛔ 🚪 ⛔\n🟩 🟩 🪴 🚪 🪴 🟩 🥤 ⛔ 🟩 🟩 🪴 ⛔ 🟩 🟩 🪴 🚪 🟩 🟩 🟩\n🟩 D  🟩 ⛔ 🪴 🟩 🟩 ⛔ 🟩 🟩 🟩 🚪 🟩 🟩 🪴 ⛔ 🪴 🟩 🟩\n🟩 🟩 🟩 🚪 🟩 🟩 🟩 ⛔ 🟩 🪴 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n🚪 ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔ ⛔ ⛔ 🚪 ⛔\n🟩 🟩 🟩 🚪 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩\n🟩 O  🟩 🚪 🟩 🪴 🟩 🚪 🟩 🪴 🟩 🚪 🟩 🪴 🟩 ⛔ 🟩 🪴 C\n🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 ⛔ 🟩 🟩 🟩 🚪 🟩 🟩 🟩\n',
             "grid_size": (15, 15), "start": (2, 7)},
}

# position_map of every OfficeWorld map (config_office.py, "position_map" lambdas): the event cells.
OFFICE_WORLD_EVENT_SYMBOLS = ("coffee0", "coffee1", "letter0", "A", "B", "C", "D", "E", "O")

# Experiment RMs as (from_state, event_symbol, to_state, reward) rows in dict insertion order
# (insertion order matters: it fixes the initial and the "final" state, reward_machine.py:152-177).
OFFICE_WORLD_EXPERIMENTS = {
    "exp1": [("state0", "coffee0", "state1", 0), ("state0", "coffee1", "state1", 0), ("state1", "O", "state2", 1)],
    "exp2": [("state0", "letter0", "state1", 0), ("state1", "O", "state2", 1)],
    "exp3": [("state0", "letter0", "state1", 0), ("state0", "coffee0", "state2", 0), ("state0", "coffee1", "state2", 0),
             ("state2", "letter0", "state3", 0), ("state1", "coffee0", "state3", 0), ("state1", "coffee1", "state3", 0),
             ("state3", "O", "state4", 1)],
    "exp4": [("state0", "A", "state1", 0), ("state1", "B", "state2", 0), ("state2", "C", "state3", 0),
             ("state3", "D", "state4", 1)],
    "exp5": [("state0", "A", "state1", 0), ("state1", "B", "state2", 0), ("state2", "C", "state3", 0),
             ("state3", "D", "state4", 0), ("state4", "coffee0", "state5", 0), ("state4", "coffee1", "state5", 0),
             ("state4", "letter0", "state6", 0), ("state6", "coffee0", "state7", 0), ("state6", "coffee1", "state7", 0),
             ("state5", "letter0", "state7", 0), ("state7", "O", "state8", 1)],
    "exp6": [("state0", "A", "state1", 0), ("state1", "B", "state2", 0), ("state2", "C", "state3", 0),
             ("state3", "D", "state4", 0), ("state4", "E", "state5", 0), ("state5", "coffee0", "state6", 0),
             ("state5", "coffee1", "state6", 0), ("state5", "letter0", "state7", 0), ("state7", "coffee0", "state8", 0),
             ("state7", "coffee1", "state8", 0), ("state6", "letter0", "state8", 0), ("state8", "O", "state9", 1)],
    "exp7": [("state0", "coffee0", "state1", 0), ("state0", "coffee1", "state2", 0), ("state1", "O", "state3", 1000),
             ("state2", "O", "state3", 1)],
    "exp0": [("state0", "letter0", "state1", 0), ("state1", "coffee0", "state2", 0), ("state2", "O", "state3", 1)],
    "exp0_simply": [("state0", "letter0", "state1", 1)],
    # BASELINE config 3: exp4 with B and C swapped (README rmgen example), A -> C -> B -> D
    "acbd": [("state0", "A", "state1", 0), ("state1", "C", "state2", 0), ("state2", "B", "state3", 0),
             ("state3", "D", "state4", 1)],
}


def office_world_experiment(map_name, experiment):
    """Experiment rows for a map; map4/exp6 is the paper's exp7 (config_office.py:446-451)."""
    if map_name == "map4" and experiment == "exp6":
        return list(OFFICE_WORLD_EXPERIMENTS["exp7"])
    return list(OFFICE_WORLD_EXPERIMENTS[experiment])


# Built-in FrozenLake RM of frozen_lake_main.py:254-258: reach A -> B -> C (10 / 15 / 20).
FROZEN_LAKE_ABC = [("state0", "A", "state1", 10), ("state1", "B", "state2", 15), ("state2", "C", "state3", 20)]
