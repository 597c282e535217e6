"""GPU parity on randomised worlds: every step-kernel variant against the CPU oracle.

The BASELINE maps exercise one shape each; these cases draw random grids (holes / plants, OfficeWorld
walls), random per-agent event detectors and random Reward Machines (rewards off the integer grid,
`None`-event transitions, reward_modifier != 1, optional shaping, short max_t so truncation is frequent),
and drive them with caller actions including `wait`.  The shapes are picked so that each table mode is
reached: the merged table (small), global tables (larger), lane-resident tables (H*W <= 128) and the
generic kernel (W > 255, where the fast path does not apply).  Bar: bit-exact integer state and rewards,
episode statistics as in test_engine_gpu.py.
"""
import numpy as np
import pytest

import oracle as O
from rmx import tables as T

pytestmark = pytest.mark.gpu

REWARDS = (0.0, 1.0, 2.5, -1.0, 0.75)


def random_rm(rng, Q, event_cells):
    """A random RM over states s0..s{Q-1}: 1-3 outgoing transitions per state on random events."""
    tr = {}
    for q in range(Q):
        for _ in range(int(rng.integers(1, 4))):
            ev = None if rng.random() < 0.15 else tuple(int(v) for v in event_cells[rng.integers(len(event_cells))])
            tr[(f"s{q}", ev)] = (f"s{int(rng.integers(Q))}", float(REWARDS[rng.integers(len(REWARDS))]))
    return T.RewardMachineSpec(tr, initial_state="s0")


def random_tables(seed, kind, W, H, A, Q, n_ev, shaping, wall_p=0.12, **extra):
    rng = np.random.default_rng(seed)
    cells = [(x, y) for y in range(H) for x in range(W)]
    perm = rng.permutation(len(cells))
    hazards = [cells[i] for i in perm[: max(1, len(cells) // 12)]]
    event_cells = [cells[i] for i in perm[len(hazards): len(hazards) + n_ev]]
    free = [cells[i] for i in perm[len(hazards) + n_ev:]]
    starts = [free[i] for i in range(A)]
    walls = []
    if kind == T.OFFICE_WORLD:
        for (x, y) in cells:
            for nx, ny in ((x + 1, y), (x, y + 1)):
                if nx < W and ny < H and rng.random() < wall_p:
                    walls += [((x, y), (nx, ny)), ((nx, ny), (x, y))]
    rms = [random_rm(rng, Q, event_cells) for _ in range(A)]
    detectors = [[c for c in event_cells if rng.random() < 0.8] or event_cells[:1] for _ in range(A)]
    return T.compile_tables(kind, W, H, hazards, walls, starts, rms, detectors, hazard_penalty=-1.5,
                            wall_penalty=-0.25, hazard_fail=None if kind == T.FROZEN_LAKE else bool(seed % 2),
                            wall_fail=bool(seed % 3 == 0), gamma=0.95, shaping_gamma=0.9 if shaping else None,
                            reward_modifier=1.5, max_t=60, **extra)


CASES = {
    # name: (seed, kind, W, H, A, Q, events, shaping)
    "fl_small_merged": (1, T.FROZEN_LAKE, 6, 6, 2, 3, 3, False),
    "ow_regs_eligible": (2, T.OFFICE_WORLD, 12, 10, 4, 6, 7, True),
    "fl_wide_global": (3, T.FROZEN_LAKE, 14, 14, 3, 5, 6, False),
    "ow_one_agent": (4, T.OFFICE_WORLD, 9, 7, 1, 4, 5, True),
    "fl_w300_generic": (5, T.FROZEN_LAKE, 300, 2, 2, 3, 4, False),
}
MODES = {  # env settings per kernel variant (round 5: the step's lost table modes and layouts were removed)
    "default": {},
    "global": {"RMX_FAST_TABLES": "global"},
    "merged": {"RMX_FAST_TABLES": "merged"},
    "merged4": {"RMX_FAST_TABLES": "merged4"},
    "wave_stats": {"RMX_FAST_STATS": "wave"},
    "nt": {"RMX_FAST_SKIP": "3"},
    "merged4_nt": {"RMX_FAST_TABLES": "merged4", "RMX_FAST_SKIP": "3"},
    "global_nt": {"RMX_FAST_TABLES": "global", "RMX_FAST_SKIP": "3"},
    "rollout_l2": {"RMX_ROLLOUT_LDS": "0"},
    "generic": {"RMX_FAST": "0"},
    "generic_skip": {"RMX_FAST": "0", "RMX_GENERIC_SKIP": "1"},
    "generic_lpe": {"RMX_FAST": "0", "RMX_LAYOUT": "lpe"},
}
KNOBS = ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP", "RMX_LAYOUT",
         "RMX_ROLLOUT_LDS")


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    assert _t.cuda.is_available(), "gpu tests need a ROCm device"
    return _t


@pytest.mark.parametrize("mode", list(MODES))
@pytest.mark.parametrize("case", list(CASES))
def test_random_world_vs_oracle(case, mode, torch, monkeypatch):
    from rmx.engine import VecRMEnv

    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    tab = random_tables(*CASES[case])
    N, Tn = 1500, 150
    env = VecRMEnv(tab, N, with_enc_state=True)
    if case == "fl_w300_generic":
        assert env.step_variant == ("lane_per_agent" if mode == "generic_lpe" else "generic")  # W > 255: not fast
    elif mode.startswith("generic"):
        assert env.step_variant == ("lane_per_agent" if mode == "generic_lpe" else "generic")
    else:
        assert env.step_variant == "fast"
    orc = O.OracleEnv(tab, N)
    rng = np.random.default_rng(CASES[case][0] + 100)
    for s in range(Tn):
        a = rng.integers(0, 5, size=(tab.n_agents, N), dtype=np.int32)  # 4 = wait
        env.step(torch.as_tensor(a, device="cuda"))
        orc.step(a)
        if s % 25 == 24 or s == Tn - 1:
            for k in ("pos_x", "pos_y", "rm_q", "t"):
                np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, k), err_msg=k)
            np.testing.assert_array_equal(env.flags.cpu().numpy().view(np.uint32), orc.flags)
            np.testing.assert_array_equal(env.env_done.cpu().numpy(), orc.env_done)
            np.testing.assert_array_equal(env.reward.cpu().numpy(), orc.reward)
            np.testing.assert_array_equal(env.renv.cpu().numpy(), orc.renv)
            np.testing.assert_array_equal(env.enc_state.cpu().numpy(), orc.enc_state)
            np.testing.assert_allclose(env.ep_ret.cpu().numpy(), orc.ep_ret, rtol=1e-5, atol=1e-5)
            if env.shaping is not None:
                np.testing.assert_allclose(env.shaping.cpu().numpy(), orc.shaping, rtol=0, atol=1e-6)
    env.check_errors()
    st, so = env.stats(), orc.stats
    assert st[1] == so[1] and st[2] == so[2] and st[3] == so[3], (st, so)
    np.testing.assert_allclose(st[0], so[0], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("mode", ["default", "global", "merged", "merged4", "nt", "generic", "generic_skip",
                                  "generic_lpe", "qrm"])
def test_garbage_state_is_bounded(mode, torch, monkeypatch):
    """State columns written by a caller with out-of-range values (negative / huge positions, RM states,
    timesteps, flags) must not make any kernel read or write outside its buffers: table reads go through
    range-checked buffer descriptors or LDS, the discount index is clamped.  Values are unspecified."""
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in MODES.get(mode, {}).items():
        monkeypatch.setenv(k, v)
    from rmx.engine import VecRMEnv

    tab = random_tables(*CASES["ow_regs_eligible"])
    N = 2048
    env = VecRMEnv(tab, N, with_qrm=mode == "qrm")
    g = torch.Generator(device="cuda").manual_seed(5)
    for col, lo, hi in (("pos_x", -300, 1 << 20), ("pos_y", -300, 1 << 20), ("rm_q", -5, 1 << 16),
                        ("flags", 0, 1 << 30)):
        getattr(env, col).copy_(torch.randint(lo, hi, getattr(env, col).shape, device="cuda", generator=g,
                                              dtype=torch.int32))
    env.t.copy_(torch.randint(-100000, 100000, env.t.shape, device="cuda", generator=g, dtype=torch.int32))
    for s in range(5):
        env.step_hashed(3, s)
    env.check_errors()
    torch.cuda.synchronize()
    env.reset()  # the engine recovers from a reset
    for s in range(5):
        env.step_hashed(3, s)
    env.check_errors()
    for col in ("pos_x", "pos_y", "rm_q"):  # and the fused rollout from garbage state
        getattr(env, col).copy_(torch.randint(-300, 1 << 20, getattr(env, col).shape, device="cuda", generator=g,
                                              dtype=torch.int32))
    env.rollout(3, 5, 20)
    torch.cuda.synchronize()


@pytest.mark.parametrize("mode", ["default", "global", "merged", "wave_stats", "generic", "generic_lpe"])
@pytest.mark.parametrize("n", [1, 2, 63, 65])
@pytest.mark.parametrize("case", ["fl_small_merged", "ow_regs_eligible"])
def test_tiny_and_ragged_batches(case, n, mode, torch, monkeypatch):
    """Batches of 1, 2, 63 and 65 envs (one partial wave; one full wave plus one lane) in every kernel family,
    bit-exact against the oracle over 150 steps with truncation (max_t = 60)."""
    from rmx.engine import VecRMEnv

    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    for k, v in MODES[mode].items():
        monkeypatch.setenv(k, v)
    tab = random_tables(*CASES[case])
    env = VecRMEnv(tab, n, with_enc_state=True)
    orc = O.OracleEnv(tab, n)
    rng = np.random.default_rng(n + 7)
    for s in range(150):
        a = rng.integers(0, 5, size=(tab.n_agents, n), dtype=np.int32)
        env.step(torch.as_tensor(a, device="cuda"))
        orc.step(a)
    for k in ("pos_x", "pos_y", "rm_q", "t", "enc_state"):
        np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, k), err_msg=k)
    np.testing.assert_array_equal(env.flags.cpu().numpy().view(np.uint32), orc.flags)
    np.testing.assert_array_equal(env.reward.cpu().numpy(), orc.reward)
    env.check_errors()
    st, so = env.stats(), orc.stats
    assert st[1] == so[1] and st[2] == so[2] and st[3] == so[3], (st, so)
    np.testing.assert_allclose(st[0], so[0], rtol=1e-5, atol=1e-4)


SLIP_CASES = {
    # name: (seed, kind, W, H, A, Q, events, shaping, slip options)
    "ow_slip_walls_fail": (6, T.OFFICE_WORLD, 9, 8, 4, 5, 6, False, {}),
    "ow_allslip_delay": (9, T.OFFICE_WORLD, 11, 9, 2, 4, 5, True, {"all_slip": True, "delay_action": True}),
    "ow_slip_highprob": (11, T.OFFICE_WORLD, 8, 8, 3, 4, 4, False, {"high_prob": 0.6}),
    "fl_slip_delay": (8, T.FROZEN_LAKE, 8, 7, 3, 4, 4, False, {"delay_action": True}),
}


def random_slip_tables(seed, kind, W, H, A, Q, n_ev, shaping, opts):
    """random_tables with slip and, for OfficeWorld, a denser wall set (blocked intended moves are frequent)."""
    return random_tables(seed, kind, W, H, A, Q, n_ev, shaping, wall_p=0.3, stochastic=True,
                         seed_schedule=(1000, 1000, 1), **opts)


@pytest.mark.parametrize("mode", ["default", "merged4", "generic"])
@pytest.mark.parametrize("case", list(SLIP_CASES))
def test_random_slip_world_vs_oracle(case, mode, torch, monkeypatch):
    """Slip dynamics on random worlds (dense OfficeWorld walls, so intended moves are often blocked: the wall
    penalty of the intended action, no draw for a blocked one, a slipped move into a wall that just does not move)
    on the fast kernel (16-B and 4-B merged records) and the generic one, stepwise and fused, vs the oracle with
    the rng columns."""
    from rmx.engine import VecRMEnv

    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv(*{"default": ("RMX_FAST", "1"), "merged4": ("RMX_FAST_TABLES", "merged4"),
                         "generic": ("RMX_FAST", "0")}[mode])
    tab = random_slip_tables(*SLIP_CASES[case])
    N, Tn = 1500, 200
    env = VecRMEnv(tab, N, with_enc_state=True)
    assert env.step_variant == ("generic" if mode == "generic" else "fast")
    env.reset(seed=31)
    orc = O.OracleEnv(tab, N)
    orc.reset(seed=31)
    rng = np.random.default_rng(SLIP_CASES[case][0] + 7)
    hi = 5 if tab.kind == T.OFFICE_WORLD else 4  # OfficeWorld: wait is an action (no draw); FrozenLake slip: not
    for s in range(Tn):
        a = rng.integers(0, hi, size=(tab.n_agents, N), dtype=np.int32)
        env.step(torch.as_tensor(a, device="cuda"))
        orc.step(a)
        if s % 40 == 39:
            for k in ("pos_x", "pos_y", "rm_q", "t"):
                np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, k), err_msg=k)
            np.testing.assert_array_equal(env.flags.cpu().numpy().view(np.uint32), orc.flags)
            np.testing.assert_array_equal(env.reward.cpu().numpy(), orc.reward)
            np.testing.assert_array_equal(env.renv.cpu().numpy(), orc.renv)
            np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64), orc.rng)
    env.check_errors()
    env2 = VecRMEnv(tab, N)  # the fused rollout of the same handle kind vs the oracle's rollout
    env2.reset(seed=31)
    orc2 = O.OracleEnv(tab, N)
    orc2.reset(seed=31)
    env2.rollout(5, 0, Tn)
    orc2.rollout(5, 0, Tn)
    for k in ("pos_x", "pos_y", "rm_q", "t"):
        np.testing.assert_array_equal(getattr(env2, k).cpu().numpy(), getattr(orc2, k), err_msg=k)
    np.testing.assert_array_equal(env2.rng.cpu().numpy().view(np.uint64), orc2.rng)
