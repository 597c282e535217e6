"""The engine's host path (cfg.device = RMX_DEVICE_HOST, csrc/rmx_hoststep.cpp) as a product, on the CPU: the
reference's golden trajectories and MDPs, the CPU oracle at the BASELINE shapes, slip and random starts with their
rng columns, rollouts, checkpoints, errors — the same bars as the GPU parity tests (tests/test_engine_gpu.py):
bit-exact integer state, rewards / shaping within 1e-6, statistics counts exact and returns within 1e-6."""
import ctypes as C
import os

import numpy as np
import pytest

import oracle as O
from rmx import _capi
from rmx import tables as T
from rmx._capi import F_ACTIVE, F_TERM, F_TRUNC
from rmx.engine import HostRMEnv
from test_engine_gpu import RS_DERIVED, TRAJ
from test_oracle_golden import check_mdp, check_qrm

REWARD_TOL = 1e-6


def _compare_state(env, orc):
    for k in ("pos_x", "pos_y", "rm_q", "t"):
        np.testing.assert_array_equal(getattr(env, k), getattr(orc, k), err_msg=k)
    np.testing.assert_array_equal(env.flags, orc.flags)
    np.testing.assert_array_equal(env.env_done, orc.env_done)
    np.testing.assert_array_equal(env.reward, orc.reward)
    np.testing.assert_allclose(env.ep_ret, orc.ep_ret, rtol=1e-6, atol=1e-6)
    if env.shaping is not None:
        np.testing.assert_allclose(env.shaping, orc.shaping, rtol=0, atol=REWARD_TOL)
    if env.enc_state is not None:
        np.testing.assert_array_equal(env.enc_state, orc.enc_state, err_msg="enc_state")


def _compare_stats(a, b):
    assert a[1] == b[1] and a[2] == b[2] and a[3] == b[3], (a, b)
    np.testing.assert_allclose(a[0], b[0], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("qrm", [False, True])
@pytest.mark.parametrize("name", TRAJ)
def test_host_engine_matches_reference_golden(name, qrm, configs, golden_dir):
    """Every golden scenario (FrozenLake / OfficeWorld, quirks, specs, slip, delay, random starts) stepped by the host
    handle, with and without the QRM columns, against the reference's recorded trajectories."""
    g = dict(np.load(os.path.join(golden_dir, f"traj_{name}.npz")))
    tab = T.compile_scenario(configs[name])
    acts = g["actions"].astype(np.int32)
    Tn, A, N = acts.shape
    env = HostRMEnv(tab, N, with_qrm=qrm)
    assert env.step_variant == "host"
    env.reset(seed=int(g["seed"]))
    np.testing.assert_array_equal(env.pos_x, g["reset_xy"][0, 0])
    np.testing.assert_array_equal(env.pos_y, g["reset_xy"][0, 1])
    keys = ("pos_x", "pos_y", "rm_q", "reward", "renv", "flags", "env_done", "t") + \
        (("qrm_s", "qrm_sn", "qrm_rq", "qrm_done") if env.qrm_s is not None else ())
    rec = {k: [] for k in keys}
    for s in range(Tn):
        env.step(acts[s])
        for k in keys:
            rec[k].append(getattr(env, k).copy())
        if env.shaping is not None:
            rec.setdefault("shaping", []).append(env.shaping.copy())
    env.check_errors()
    r = {k: np.stack(v) for k, v in rec.items()}
    np.testing.assert_array_equal(r["pos_x"], g["pos_x"])
    np.testing.assert_array_equal(r["pos_y"], g["pos_y"])
    np.testing.assert_array_equal(r["rm_q"], g["q"])
    np.testing.assert_array_equal((r["flags"] & F_TERM) != 0, g["term"])
    np.testing.assert_array_equal((r["flags"] & F_TRUNC) != 0, g["trunc"])
    np.testing.assert_array_equal((r["flags"] & F_ACTIVE) != 0, g["active"])
    np.testing.assert_array_equal(r["env_done"].astype(bool), g["env_done"])
    np.testing.assert_array_equal(r["t"], g["t"])
    assert np.max(np.abs(r["reward"].astype(np.float64) - g["reward"])) <= REWARD_TOL
    assert np.max(np.abs(r["renv"].astype(np.float64) - g["renv"])) <= REWARD_TOL
    sh = r["shaping"].astype(np.float64) if "shaping" in r else 0.0
    assert np.max(np.abs(r["reward"] + sh - (g["reward"] + g["shaping"]))) <= REWARD_TOL
    if "qrm_s" in r:
        check_qrm(tab, r, g, acts, r["renv"])


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_host_engine_vs_oracle_baseline_shapes(cfg):
    """BASELINE configs 2-5 (4,096 envs per shard, 1,100 hashed steps: OfficeWorld crosses its t > 1000 truncation),
    state every 100 steps, statistics at the end."""
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 4096, 1100, 11 + cfg
    env = HostRMEnv(tab, N, with_enc_state=True)
    orc = O.OracleEnv(tab, N)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    for s in range(Tn):
        env.step_hashed(seed, s)
        orc.step(acts[s])
        if s % 100 == 99:
            _compare_state(env, orc)
    _compare_stats(env.stats(), orc.stats)


@pytest.mark.parametrize("name", ["fl2_slip", "fl2_delay", "ow1_slip", "ow2_allslip", "ow3_slip", "fl2_randstart",
                                  "fl2_randstart_slip", "fl4_randstart_open"] + RS_DERIVED)
def test_host_engine_stochastic_vs_oracle(name, configs):
    """Slip and random starts at 2,048 envs x 1,100 caller-action steps: state, rng / episode columns (numpy's PCG64
    bit for bit), statistics; then the host rollout from the same reset ends at the same place."""
    tab = T.compile_scenario(configs[name])
    N, Tn, seed, base = 2048, 1100, 41, 77
    env = HostRMEnv(tab, N, with_enc_state=True)
    env.reset(seed=base)
    orc = O.OracleEnv(tab, N)
    orc.reset(seed=base)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    for s in range(Tn):
        env.step(acts[s])
        orc.step(acts[s])
    _compare_state(env, orc)
    np.testing.assert_array_equal(env.rng, orc.rng)
    np.testing.assert_array_equal(env.episode, orc.episode)
    _compare_stats(env.stats(), orc.stats)
    env2 = HostRMEnv(tab, N, with_enc_state=True)
    env2.reset(seed=base)
    env2.rollout(seed, 0, Tn)
    _compare_state(env2, orc)
    np.testing.assert_array_equal(env2.rng, orc.rng)


@pytest.mark.parametrize("name", ["fl2", "fl2_slip", "ow3", "fl2_randstart_slip"])
def test_host_rollout_trace_step_seq_and_report(name, configs):
    """rmx_rollout (with its reward trace), rmx_step_seq and rmx_step_report on a host handle equal single steps."""
    tab = T.compile_scenario(configs[name])
    N, Tn, seed = 777, 300, 9
    a, b, c = (HostRMEnv(tab, N) for _ in range(3))
    for e in (a, b, c):
        e.reset(seed=3)
    trace = b.rollout(seed, 0, Tn, record_rewards=True)
    acts = c.fill_actions(seed, 0, Tn)
    np.testing.assert_array_equal(acts, O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents))
    out = np.zeros(4)
    c.step_seq(acts[:Tn - 1])
    c.step_report(acts[Tn - 1], out=out)
    for s in range(Tn):
        a.step_hashed(seed, s)
        np.testing.assert_array_equal(trace[s], a.reward, err_msg=str(s))
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward") + (("rng", "episode") if a.rng is not None else ()):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
        np.testing.assert_array_equal(getattr(a, k), getattr(c, k), err_msg=k)
    np.testing.assert_array_equal(a.stats(), b.stats())
    np.testing.assert_array_equal(a.stats(), out)
    assert c.queue_info()["dispatch"] == "host" and c.queue_info()["state"] == "unused"


@pytest.mark.parametrize("name", ["fl2", "fl2_slip", "fl2_randstart_slip", "ow3"])
def test_host_save_load_state_resumes_bit_exactly(name, configs):
    tab = T.compile_scenario(configs[name])
    N, seed = 600, 13
    a = HostRMEnv(tab, N)
    a.reset(seed=5)
    for s in range(300):
        a.step_hashed(seed, s)
    blob = a.save_state()
    for s in range(300, 700):
        a.step_hashed(seed, s)
    b = HostRMEnv(tab, N)
    b.load_state(blob)
    for s in range(300, 700):
        b.step_hashed(seed, s)
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward") + (("rng", "episode") if a.rng is not None else ()):
        np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)
    np.testing.assert_array_equal(a.stats()[1:], b.stats()[1:])
    np.testing.assert_allclose(a.stats()[0], b.stats()[0], rtol=1e-12)
    if name == "fl2":  # a blob of another scenario (same agents and envs, other holes / penalty) is refused
        with pytest.raises(ValueError, match="another scenario"):
            HostRMEnv(T.compile_scenario(configs["fl2_quirks"]), N).load_state(blob)


@pytest.mark.parametrize("name", ["fl2", "fl2_quirks", "ow1", "ow3", "ow2_fail", "ow2_final", "ow1_map3", "fl2_spec",
                                  "ow2_spec"])
def test_host_mdp_matches_reference(name, configs, golden_dir):
    g = dict(np.load(os.path.join(golden_dir, f"mdp_{name}.npz")))
    tab = T.compile_scenario(configs[name])
    env = HostRMEnv(tab, 1)
    for a in range(tab.n_agents):
        check_mdp(tab, a, *env.mdp_arrays(a), g)
        for x, y in zip(env.mdp_arrays(a, fix_frozen_lake=True), O.mdp(tab, a, fix_fl=True)):
            np.testing.assert_array_equal(x, y)


def test_host_masked_reset_and_invalid_action():
    tab = T.compile_scenario(T.baseline_scenario(2))
    N = 64
    env = HostRMEnv(tab, N)
    for s in range(20):
        env.step_hashed(1, s)
    t_before = env.t.copy()
    mask = np.zeros(N, np.uint8)
    mask[::3] = 1
    env.reset(mask=mask, seed=4)
    np.testing.assert_array_equal(env.t[::3], 0)
    np.testing.assert_array_equal(env.t[1::3], t_before[1::3])
    bad = np.zeros((2, N), np.int32)
    bad[1, 5] = 7
    env.step(bad)
    with pytest.raises(ValueError, match="outside"):
        env.check_errors()
    env.check_errors()  # cleared
    x = env.step_sync  # the synchronous form reports it at once
    with pytest.raises(ValueError):
        x(bad)


def test_host_handle_queue_timing_is_a_no_op():
    """A host handle has no device queue: timing on/off succeeds and there are never stamps."""
    env = HostRMEnv(T.compile_scenario(T.baseline_scenario(2)), 16)
    env.queue_timing(1)
    env.step_seq(np.zeros((3, 2, 16), np.int32))
    assert env.queue_times().shape == (0, 3)
    env.queue_timing(0)
    with pytest.raises(ValueError):
        env.queue_timing(-1)


def test_host_output_arrays_are_checked_before_c_writes_them():
    """Caller-supplied output arrays reach C as raw addresses: a wrong dtype, size or layout is refused in Python
    (nothing written), a right one is filled."""
    tab = T.compile_scenario(T.baseline_scenario(2))
    N = 32
    env = HostRMEnv(tab, N)
    acts = np.zeros((2, N), np.int32)
    for out in (np.zeros(4, np.float32), np.zeros(2, np.float64), np.zeros((8, 2), np.float64)[:, 0]):
        with pytest.raises(ValueError, match="out must be"):
            env.step_report(acts, out=out)
        with pytest.raises(ValueError, match="out must be"):
            env.step_seq(acts[None], out=out)
    ro = np.zeros(_capi.NSTATS, np.float64)
    ro.flags.writeable = False
    with pytest.raises(ValueError, match="out must be"):
        env.step_report(acts, out=ro)
    for out in (np.zeros((3, 2, N), np.int64), np.zeros((2, 2, N), np.int32)):
        with pytest.raises(ValueError, match="out must be"):
            env.fill_actions(1, 0, 3, out=out)
    ok = np.zeros(_capi.NSTATS, np.float64)
    assert env.step_report(acts, out=ok) is ok and ok[1] >= 0
    fa = env.fill_actions(1, 0, 3, out=np.full((3, 2, N), -1, np.int32))
    assert ((fa >= 0) & (fa < 4)).all()


def test_host_handle_through_raw_c_abi():
    """A host handle from plain ctypes (no rmx.engine): create with RMX_DEVICE_HOST, bind host columns, reset and
    step_sync against the oracle; the queue and variant queries answer for a host handle."""
    lib = _capi.load_library()
    tab = T.compile_scenario(T.baseline_scenario(4))
    N, A = 5, tab.n_agents
    cfg, keep = _capi.make_config(tab, N, device=_capi.DEVICE_HOST)
    h = C.c_void_p()
    assert lib.rmx_create(C.byref(cfg), C.byref(h)) == 0
    try:
        cols = {k: np.zeros((A, N), np.int32) for k in ("pos_x", "pos_y", "rm_q", "flags")}
        cols.update(ep_ret=np.zeros((A, N), np.float32), t=np.zeros(N, np.int32), reward=np.zeros((A, N), np.float32))
        b = _capi.RmxBuffers()
        for k, v in cols.items():
            setattr(b, k, v.ctypes.data)
        assert lib.rmx_bind(h, C.byref(b)) == 0
        assert lib.rmx_step_variant(h) == _capi.VARIANT_HOST
        out = {k: np.zeros_like(v) for k, v in cols.items()}
        ob = _capi.RmxBuffers()
        for k, v in out.items():
            setattr(ob, k, v.ctypes.data)
        assert lib.rmx_reset_sync(h, 9, C.byref(ob), None) == 0
        orc = O.OracleEnv(tab, N)
        orc.reset(seed=9)
        acts = O.hash_actions(2, 0, 200, N, 0, N, A)
        for s in range(200):
            a = np.ascontiguousarray(acts[s])
            assert lib.rmx_step_sync(h, a.ctypes.data, 1, C.byref(ob), None) == 0
            orc.step(acts[s])
            for k in ("pos_x", "pos_y", "rm_q", "t"):
                np.testing.assert_array_equal(out[k], getattr(orc, k), err_msg=k)
            np.testing.assert_array_equal(out["flags"].view(np.uint32), orc.flags)
            np.testing.assert_array_equal(out["reward"], orc.reward)
        info = (C.c_int64 * _capi.QUEUE_INFO_N)()
        assert lib.rmx_queue_info(h, info, _capi.QUEUE_INFO_N) == 0
        assert info[0] == info[1] == info[2] == 0 and _capi.QUEUE_STATES[info[4]] == "unused"
        # a column the handle does not compute is refused, as on a device handle
        sh = np.zeros((A, N), np.float32)
        ob2 = _capi.RmxBuffers(shaping=sh.ctypes.data)
        a = np.zeros((A, N), np.int32)
        assert lib.rmx_step_sync(h, a.ctypes.data, 1, C.byref(ob2), None) == _capi.RMX_E_STATE
        assert b"shaping" in lib.rmx_last_error()
    finally:
        lib.rmx_destroy(h)


def test_device_count_answers_without_a_gpu():
    n = _capi.device_count()
    assert n >= 0
    import torch
    if not torch.cuda.is_available():
        assert n == 0
