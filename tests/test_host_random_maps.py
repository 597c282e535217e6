"""The host path (csrc/rmx_hoststep.cpp, rmx.engine.HostRMEnv) on randomised worlds, against the CPU oracle.

The same random grids, event detectors and Reward Machines as tests/test_random_maps_gpu.py (rewards off the integer
grid, `None`-event transitions, reward_modifier != 1, optional shaping, max_t = 60 so truncation is frequent, caller
actions including `wait`), here on the CPU: the host step reads the generic kernels' table blob with its own index
arithmetic, so the shapes that pick different device table modes (merged, global, W > 255) are different blob
layouts to it.  Bar: bit-exact integer state and rewards, the rng columns under slip, statistics as on the device.
"""
import numpy as np
import pytest

import oracle as O
from rmx import tables as T
from rmx.engine import HostRMEnv
from test_random_maps_gpu import CASES, SLIP_CASES, random_slip_tables, random_tables


def _same_state(env, orc, what):
    for k in ("pos_x", "pos_y", "rm_q", "t"):
        np.testing.assert_array_equal(getattr(env, k), getattr(orc, k), err_msg=f"{what} {k}")
    np.testing.assert_array_equal(env.flags.view(np.uint32), orc.flags, err_msg=f"{what} flags")
    np.testing.assert_array_equal(env.reward, orc.reward, err_msg=f"{what} reward")
    np.testing.assert_array_equal(env.renv, orc.renv, err_msg=f"{what} renv")


def _same_stats(env, orc):
    env.check_errors()
    st, so = env.stats(), orc.stats
    assert st[1] == so[1] and st[2] == so[2] and st[3] == so[3], (st, so)
    np.testing.assert_allclose(st[0], so[0], rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("case", list(CASES))
def test_host_random_world_vs_oracle(case):
    tab = random_tables(*CASES[case])
    N, Tn = 1500, 150
    env = HostRMEnv(tab, N, with_enc_state=True)
    orc = O.OracleEnv(tab, N)
    rng = np.random.default_rng(CASES[case][0] + 100)
    for s in range(Tn):
        a = rng.integers(0, 5, size=(tab.n_agents, N), dtype=np.int32)  # 4 = wait
        env.step(a)
        orc.step(a)
        if s % 25 == 24 or s == Tn - 1:
            _same_state(env, orc, s)
            np.testing.assert_array_equal(env.env_done, orc.env_done)
            np.testing.assert_array_equal(env.enc_state, orc.enc_state)
            np.testing.assert_allclose(env.ep_ret, orc.ep_ret, rtol=1e-5, atol=1e-5)
            if env.shaping is not None:
                np.testing.assert_allclose(env.shaping, orc.shaping, rtol=0, atol=1e-6)
    _same_stats(env, orc)


@pytest.mark.parametrize("n", [1, 2, 63, 65])
@pytest.mark.parametrize("case", ["fl_small_merged", "ow_regs_eligible"])
def test_host_tiny_and_ragged_batches(case, n):
    tab = random_tables(*CASES[case])
    env = HostRMEnv(tab, n, with_enc_state=True)
    orc = O.OracleEnv(tab, n)
    rng = np.random.default_rng(n + 7)
    for s in range(150):
        a = rng.integers(0, 5, size=(tab.n_agents, n), dtype=np.int32)
        env.step(a)
        orc.step(a)
    _same_state(env, orc, "end")
    np.testing.assert_array_equal(env.enc_state, orc.enc_state)
    _same_stats(env, orc)


@pytest.mark.parametrize("case", list(SLIP_CASES))
def test_host_random_slip_world_vs_oracle(case):
    """Slip on random worlds with dense OfficeWorld walls (the intended move's wall penalty, no draw for a blocked
    move, a slipped move into a wall that stays put), stepwise and through the fused rollout, with the rng columns."""
    tab = random_slip_tables(*SLIP_CASES[case])
    N, Tn = 1500, 200
    env = HostRMEnv(tab, N, with_enc_state=True)
    env.reset(seed=31)
    orc = O.OracleEnv(tab, N)
    orc.reset(seed=31)
    rng = np.random.default_rng(SLIP_CASES[case][0] + 7)
    hi = 5 if tab.kind == T.OFFICE_WORLD else 4  # FrozenLake's slip map has no wait
    for s in range(Tn):
        a = rng.integers(0, hi, size=(tab.n_agents, N), dtype=np.int32)
        env.step(a)
        orc.step(a)
        if s % 40 == 39:
            _same_state(env, orc, s)
            np.testing.assert_array_equal(env.rng.view(np.uint64), orc.rng)
    _same_stats(env, orc)
    env2, orc2 = HostRMEnv(tab, N), O.OracleEnv(tab, N)
    env2.reset(seed=31)
    orc2.reset(seed=31)
    env2.rollout(5, 0, Tn)
    orc2.rollout(5, 0, Tn)
    for k in ("pos_x", "pos_y", "rm_q", "t"):
        np.testing.assert_array_equal(getattr(env2, k), getattr(orc2, k), err_msg=k)
    np.testing.assert_array_equal(env2.rng.view(np.uint64), orc2.rng)


@pytest.mark.parametrize("qrm", [False, True])
@pytest.mark.parametrize("case", ["ow_regs_eligible", "fl_w300_generic"])
def test_host_garbage_state_is_bounded(case, qrm):
    """Columns a caller overwrote with out-of-range positions, RM states, timesteps and flags index no table outside
    it (the host step resets such an index to 0, as the device's range-checked descriptors keep its reads inside);
    the values that follow are unspecified, but positions and RM states stay in range and a reset recovers the
    oracle's trajectory.  Run under ASan by tests/test_sanitizers.py (oracle/asan/rmxh_entry.cpp)."""
    tab = random_tables(*CASES[case])
    N = 2048
    env = HostRMEnv(tab, N, with_qrm=qrm, with_enc_state=True)
    g = np.random.default_rng(5)
    for col, lo, hi in (("pos_x", -300, 1 << 20), ("pos_y", -300, 1 << 20), ("rm_q", -5, 1 << 16),
                        ("flags", 0, 1 << 30)):
        c = getattr(env, col)
        c[...] = g.integers(lo, hi, c.shape).astype(np.int32).view(c.dtype)
    env.t[...] = g.integers(-100000, 100000, env.t.shape).astype(np.int32)
    for s in range(5):
        env.step_hashed(3, s)
    env.check_errors()
    assert ((env.pos_x >= 0) & (env.pos_x < tab.width)).all() and ((env.pos_y >= 0) & (env.pos_y < tab.height)).all()
    assert ((env.rm_q >= 0) & (env.rm_q < tab.n_rm_states)).all()
    env.reset(seed=9)
    orc = O.OracleEnv(tab, N)
    orc.reset(seed=9)
    env.rollout(3, 0, 40)
    orc.rollout(3, 0, 40)
    for k in ("pos_x", "pos_y", "rm_q", "t"):
        np.testing.assert_array_equal(getattr(env, k), getattr(orc, k), err_msg=k)
