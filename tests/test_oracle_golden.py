"""Pin the CPU oracle against golden vectors recorded from the REFERENCE itself.

Inputs: the scenario (configs.json) compiled by rmx.tables + the recorded action sequence.
Outputs compared per step, per (env, agent): positions / RM state / flags / env_done / timestep
bit-exact; reward and shaping within 1e-6 (BASELINE.json north_star tolerance), compared in f64.
"""
import os

import numpy as np
import pytest

import oracle as O
from rmx import tables as T
from rmx._capi import F_ACTIVE, F_TERM, F_TRUNC

REWARD_TOL = 1e-6

TRAJ = ["fl2", "fl4", "fl2_quirks", "fl2_initfinal", "fl2_finalnt", "fl2_open", "ow1_map3", "ow1", "ow3",
        "ow2_final", "ow2_fail", "fl2_spec", "ow2_spec", "fl2_slip", "fl2_delay", "ow1_slip", "ow2_allslip",
        "ow2_delay", "ow3_slip", "fl2_randstart", "fl2_randstart_slip", "fl4_randstart_open"]


def replay_oracle(tab, acts, seed=123):
    Tn, A, N = acts.shape
    env = O.OracleEnv(tab, N)
    env.reset(seed=seed)  # base of the reset-seed schedule (stochastic scenarios)
    rec = {k: np.zeros((Tn, A, N), dt) for k, dt in
           [("pos_x", np.int32), ("pos_y", np.int32), ("q", np.int32), ("reward", np.float32),
            ("shaping", np.float32), ("renv", np.float32), ("flags", np.uint32), ("ep_ret", np.float32)]}
    done = np.zeros((Tn, N), np.uint8)
    tcol = np.zeros((Tn, N), np.int32)
    if env.qrm_s is not None:
        Qx = env.qrm_s.shape[1]
        for k, dt in (("qrm_s", np.int32), ("qrm_sn", np.int32), ("qrm_rq", np.float32), ("qrm_done", np.uint8)):
            rec[k] = np.zeros((Tn, A, Qx, N), dt)
    for s in range(Tn):
        assert env.step(acts[s]) == 0
        rec["pos_x"][s], rec["pos_y"][s], rec["q"][s] = env.pos_x, env.pos_y, env.rm_q
        rec["reward"][s], rec["shaping"][s], rec["renv"][s] = env.reward, env.shaping, env.renv
        rec["flags"][s], rec["ep_ret"][s] = env.flags, env.ep_ret
        done[s], tcol[s] = env.env_done, env.t
        if env.qrm_s is not None:
            rec["qrm_s"][s], rec["qrm_sn"][s], rec["qrm_rq"][s], rec["qrm_done"][s] = \
                env.qrm_s, env.qrm_sn, env.qrm_rq, env.qrm_done
    return rec, done, tcol, env


def check_qrm(tab, rec, g, acts, renv):
    """Engine QRM outputs vs the reference's infos["qrm_experience"] tuples (all ten fields)."""
    Tn, A, Qg, N = g["qrm_s"].shape
    for a in range(A):
        nq = int(tab.n_qrm[a])
        enc = int(tab.enc_nq[a])
        if nq == 0:
            continue
        s_, sn = rec["qrm_s"][:, a, :nq], rec["qrm_sn"][:, a, :nq]
        np.testing.assert_array_equal(s_, g["qrm_s"][:, a, :nq])
        np.testing.assert_array_equal(sn, g["qrm_sn"][:, a, :nq])
        np.testing.assert_array_equal(rec["qrm_done"][:, a, :nq].astype(np.int8), g["qrm_done"][:, a, :nq])
        np.testing.assert_array_equal(s_ // enc, g["qrm_pos"][:, a, :nq])
        np.testing.assert_array_equal(s_ % enc, g["qrm_q"][:, a, :nq])
        np.testing.assert_array_equal(sn // enc, g["qrm_npos"][:, a, :nq])
        np.testing.assert_array_equal(sn % enc, g["qrm_nq"][:, a, :nq])
        assert np.max(np.abs(rec["qrm_rq"][:, a, :nq] - g["qrm_hr"][:, a, :nq])) <= 1e-6
        r = renv[:, a, None, :].astype(np.float64) + rec["qrm_rq"][:, a, :nq]
        assert np.max(np.abs(r - g["qrm_r"][:, a, :nq])) <= 1e-6
        np.testing.assert_array_equal(np.broadcast_to(acts[:, a, None, :], s_.shape), g["qrm_a"][:, a, :nq])


@pytest.mark.parametrize("name", TRAJ)
def test_oracle_matches_reference_trajectory(name, configs, golden_dir):
    g = dict(np.load(os.path.join(golden_dir, f"traj_{name}.npz")))
    tab = T.compile_scenario(configs[name])
    acts = g["actions"].astype(np.int32)
    rec, done, tcol, _ = replay_oracle(tab, acts, int(g["seed"]))
    np.testing.assert_array_equal(rec["pos_x"], g["pos_x"])
    np.testing.assert_array_equal(rec["pos_y"], g["pos_y"])
    np.testing.assert_array_equal(rec["q"], g["q"])
    np.testing.assert_array_equal((rec["flags"] & F_TERM) != 0, g["term"])
    np.testing.assert_array_equal((rec["flags"] & F_TRUNC) != 0, g["trunc"])
    np.testing.assert_array_equal((rec["flags"] & F_ACTIVE) != 0, g["active"])
    np.testing.assert_array_equal(done.astype(bool), g["env_done"])
    np.testing.assert_array_equal(tcol, g["t"])
    assert np.max(np.abs(rec["reward"].astype(np.float64) - g["reward"])) <= REWARD_TOL
    assert np.max(np.abs(rec["renv"].astype(np.float64) - g["renv"])) <= REWARD_TOL
    total = rec["reward"].astype(np.float64) + rec["shaping"].astype(np.float64)
    assert np.max(np.abs(total - (g["reward"] + g["shaping"]))) <= REWARD_TOL
    check_qrm(tab, rec, g, acts, rec["renv"])


@pytest.mark.parametrize("name", ["fl2_randstart", "fl2_randstart_slip", "fl4_randstart_open"])
def test_oracle_reset_positions(name, configs, golden_dir):
    """random_start_positions: the positions right after the first reset(seed) equal the reference's."""
    g = dict(np.load(os.path.join(golden_dir, f"traj_{name}.npz")))
    tab = T.compile_scenario(configs[name])
    assert tab.random_starts
    N = g["actions"].shape[2]
    env = O.OracleEnv(tab, N)
    env.reset(seed=int(g["seed"]))
    np.testing.assert_array_equal(env.pos_x, g["reset_xy"][0, 0])
    np.testing.assert_array_equal(env.pos_y, g["reset_xy"][0, 1])


@pytest.mark.parametrize("shape", [(10, 10, 11, 2), (6, 5, 0, 4), (1, 2, 0, 2), (64, 64, 300, 8), (3, 3, 8, 1)])
def test_random_starts_match_numpy_shuffle(shape):
    """_sample_start_positions restated (oracle) == numpy's own Generator.shuffle of the x-major free-cell
    list (ma_frozen_lake.py:156-172) for random hole sets and seeds, incl. a 4,096-cell map."""
    W, H, n_holes, A = shape
    rs = np.random.RandomState(W * 131 + n_holes)
    cells = [(x, y) for x in range(W) for y in range(H)]
    holes = [cells[i] for i in rs.choice(len(cells), n_holes, replace=False)] if n_holes else []
    rm = T.RewardMachineSpec({("q0", (0, 0)): ("q1", 1)})
    tab = T.compile_tables(T.FROZEN_LAKE, W, H, holes, (), [(0, 0)] * A, [rm] * A, [{(0, 0)}] * A,
                           random_starts=True, seed_schedule=(1, 1, 0))
    N = 37
    env = O.OracleEnv(tab, N)
    base = int(rs.randint(0, 2**31))
    env.reset(seed=base)
    for e in range(N):
        free = [c for c in cells if c not in set(holes)]
        np.random.default_rng(base + e).shuffle(free)
        assert [(int(env.pos_x[a, e]), int(env.pos_y[a, e])) for a in range(A)] == free[:A]


def test_random_starts_need_enough_free_cells():
    rm = T.RewardMachineSpec({("q0", (0, 0)): ("q1", 1)})
    with pytest.raises(ValueError, match="Not enough free cells"):
        T.compile_tables(T.FROZEN_LAKE, 2, 1, [(1, 0)], (), [(0, 0)] * 2, [rm] * 2, [{(0, 0)}] * 2, random_starts=True)
    with pytest.raises(ValueError, match="FrozenLake"):
        T.compile_tables(T.OFFICE_WORLD, 2, 2, [], (), [(0, 0)], [rm], [{(0, 0)}], random_starts=True)


@pytest.mark.parametrize("name", ["fl2", "ow1"])
def test_oracle_episode_summaries(name, configs, golden_dir):
    """Per-episode return / length / success and the 4-scalar stats vector (evaluation_metrics.py:248-267)."""
    ep = dict(np.load(os.path.join(golden_dir, f"episodes_{name}.npz")))
    n, Tn, seed = int(ep["n_envs"]), int(ep["n_steps"]), int(ep["seed"])
    tab = T.compile_scenario(configs[name])
    A = tab.n_agents
    acts = O.hash_actions(seed, 0, Tn, n, 0, n, A)
    env = O.OracleEnv(tab, n)
    got = []
    for s in range(Tn):
        env.step(acts[s])
        for e in np.nonzero(env.env_done)[0]:
            for a in range(A):
                got.append((e, a, float(env.ep_ret[a, e]), int(env.t[e]), s))
    got.sort(key=lambda r: (r[0], r[4], r[1]))
    order = np.lexsort((ep["agent"], ep["end_step"], ep["env"]))
    assert len(got) == len(order)
    g_ret = ep["ret"][order]
    m_ret = np.array([r[2] for r in got])
    # FL returns are integer sums (exact); OW discounted returns accumulate in f32 (rel 1e-5)
    np.testing.assert_allclose(m_ret, g_ret, rtol=1e-5, atol=1e-5)
    np.testing.assert_array_equal([r[3] for r in got], ep["length"][order])
    st = env.stats
    assert st[1] * A == len(order)
    assert st[2] == ep["success"].sum()
    np.testing.assert_allclose(st[0], ep["ret"].sum(), rtol=1e-6, atol=1e-4)
    assert st[3] * A == ep["length"].sum()


def test_hash_actions_match_golden(configs, golden_dir):
    g = dict(np.load(os.path.join(golden_dir, "traj_fl2.npz")))
    Tn, A, N = g["actions"].shape
    acts = O.hash_actions(int(g["seed"]), 0, Tn, N, 0, N, A)
    np.testing.assert_array_equal(acts, g["actions"])


def test_oracle_rollout_equals_stepwise(configs):
    tab = T.compile_scenario(configs["fl2"])
    a = O.OracleEnv(tab, 64)
    b = O.OracleEnv(tab, 64)
    acts = O.hash_actions(3, 0, 300, 64, 0, 64, 2)
    for s in range(300):
        a.step(acts[s])
    b.rollout(3, 0, 300, n_threads=2)
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret"):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k))
    np.testing.assert_array_equal(a.stats, b.stats)


def test_ctypes_layout_matches_header():
    import ctypes as C
    from rmx._capi import RmxBuffers, RmxConfig
    lay = O.config_layout()
    mine = [C.sizeof(RmxConfig), RmxConfig.kind.offset, RmxConfig.n_envs.offset, RmxConfig.env_offset.offset,
            RmxConfig.n_envs_global.offset, RmxConfig.hazard_penalty.offset, RmxConfig.gamma.offset,
            RmxConfig.has_shaping.offset, RmxConfig.cell.offset, RmxConfig.start_xy.offset, C.sizeof(RmxBuffers),
            RmxBuffers.ep_ret.offset, RmxBuffers.renv.offset, RmxConfig.reward_modifier.offset,
            RmxConfig.n_qrm.offset, RmxConfig.enc_nq.offset, RmxBuffers.qrm_s.offset, RmxBuffers.qrm_done.offset,
            RmxConfig.random_starts.offset]
    assert list(lay) == mine


MDP = ["fl2", "fl2_quirks", "ow1", "ow3", "ow2_fail", "ow2_final", "ow1_map3", "fl2_spec", "ow2_spec"]


def check_mdp(tab, a, nxt, rew, done, g):
    """Arrays vs the reference's P[s][a] = [(1.0, s', r, done)] (or [] for no entry)."""
    gn, gr, gd = g[f"a{a}_next"], g[f"a{a}_reward"], g[f"a{a}_done"]
    assert nxt.shape == gn.shape
    np.testing.assert_array_equal(nxt, gn)
    has = gn >= 0
    np.testing.assert_array_equal(done == 255, ~has)
    np.testing.assert_array_equal(done[has].astype(np.int8), gd[has])
    assert np.max(np.abs(rew[has].astype(np.float64) - gr[has]), initial=0.0) <= REWARD_TOL


@pytest.mark.parametrize("name", MDP)
def test_oracle_mdp_matches_reference(name, configs, golden_dir):
    g = dict(np.load(os.path.join(golden_dir, f"mdp_{name}.npz")))
    tab = T.compile_scenario(configs[name])
    for a in range(tab.n_agents):
        check_mdp(tab, a, *O.mdp(tab, a), g)


def test_oracle_mdp_kat_small_lake():
    """test_ma_frozen_lake.py:86-102: 2x2 lake, RM {(q0,(1,0)): (qf,1)} -> 8 states, 4 actions."""
    rm = T.RewardMachineSpec({("q0", (1, 0)): ("qf", 1)})
    tab = T.compile_tables(T.FROZEN_LAKE, 2, 2, [], (), [(0, 0)], [rm], [{(1, 0)}])
    nxt, rew, done = O.mdp(tab, 0)
    assert nxt.shape == (8, 4)
    # corrected decode: the q0 -> right -> (1,0) transition fires the RM
    nxt2, rew2, done2 = O.mdp(tab, 0, fix_fl=True)
    assert nxt2[0, 3] == (0 * 2 + 1) * 2 + 1 and rew2[0, 3] == 1.0 and done2[0, 3] == 1


@pytest.mark.parametrize("seed", [0, 1, 123, 4096, 123007, 2**32 + 5, 2**63 + 12345])
def test_seed_pcg64_matches_numpy_default_rng(seed):
    """SeedSequence -> PCG64 restatement == np.random.default_rng(seed).bit_generator.state."""
    st = np.random.default_rng(seed).bit_generator.state["state"]
    r = [int(v) for v in O.seed_pcg64(seed)]
    assert (r[0] << 64 | r[1]) == st["state"] and (r[2] << 64 | r[3]) == st["inc"]


def test_slip_tables_match_numpy_choice():
    """The per-action cdf tables reproduce Generator.choice(outcomes, p) on the same stream."""
    for kind, kw in [(T.FROZEN_LAKE, {}), (T.FROZEN_LAKE, {"delay_action": True}), (T.OFFICE_WORLD, {"high_prob": 0.7}),
                     (T.OFFICE_WORLD, {"all_slip": True, "high_prob": 0.9})]:
        mp = T.slip_mapping(kind, **kw)
        n, out, cdf = T.slip_tables(mp)
        for name, (outs, probs) in mp.items():
            rng, rng2 = np.random.default_rng(5), np.random.default_rng(5)
            i = T._ACT[name]
            for _ in range(300):
                want = rng.choice(outs, p=probs)
                u = rng2.random()
                got = out[i, int(np.searchsorted(cdf[i, :n[i]], u, side="right"))]
                assert T._ACT[str(want)] == got


def test_state_encoder_kat():
    """test_state_encoder_frozen_lake.py:21-43 restated on the enc_state column of a 4x5 lake.  Single-state RM
    {("q0", None): ("q0", 0)}: q0 is also its final state, so the agent at (1, 2) is frozen there (the reference's
    RM-final freeze) and its index is 2*4+1 = 9.  Two-state RM {("q0","a"): ("q1",1)}: the agent moves down from
    (1, 1) to (1, 2) and stays in q0 -> 9*2 + 0 = 18; the reference's decode(19) = (pos 9, RM index 1) is the
    same stride."""
    from rmx import tables as T
    for transitions, start, want in (({("q0", None): ("q0", 0)}, (1, 2), 9), ({("q0", "a"): ("q1", 1)}, (1, 1), 18)):
        rm = T.RewardMachineSpec(transitions)
        tab = T.compile_tables(T.FROZEN_LAKE, 4, 5, [], [], [start], [rm], [[]])
        orc = O.OracleEnv(tab, 1)
        orc.step(np.array([[1]], np.int32))  # down: y + 1 in FrozenLake
        assert (orc.pos_x[0, 0], orc.pos_y[0, 0]) == (1, 2)
        assert orc.enc_state[0, 0] == want
    assert divmod(19, 2) == (9, 1) and divmod(9, 4) == (2, 1)  # decode(19): pos_index 9 -> (x=1, y=2), q index 1
