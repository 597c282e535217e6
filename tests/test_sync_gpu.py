"""The synchronous host-boundary calls (rmx_reset_sync / rmx_step_sync: the resident workgroup behind the
reference's per-call dict API) against the asynchronous device path and the CPU oracle.

Bar: every output column bit-exact with rmx_reset / rmx_step on the same actions (the two run the same
agent_step / env_step), across resets, autoresets, slip and random starts, QRM outputs, the idle-timeout
relaunch, the one-launch-per-call mode and interleaving with asynchronous calls on the same handle."""
import time

import numpy as np
import pytest

import oracle as O
from rmx import tables as T

pytestmark = pytest.mark.gpu

COLS = ("pos_x", "pos_y", "rm_q", "flags", "ep_ret", "t", "reward", "env_done", "renv")


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    assert _t.cuda.is_available(), "gpu tests need a ROCm device"
    return _t


def _engine(tab, n, **kw):
    from rmx.engine import VecRMEnv
    return VecRMEnv(tab, n, **kw)


def _dev_cols(env):
    d = {k: getattr(env, k).cpu().numpy() for k in COLS}
    d["flags"] = d["flags"].astype(np.uint32)
    if env.shaping is not None:
        d["shaping"] = env.shaping.cpu().numpy()
    if env.qrm_s is not None:
        for k in ("qrm_s", "qrm_sn", "qrm_rq", "qrm_done"):
            d[k] = getattr(env, k).cpu().numpy()
    return d


def _assert_same(host, dev, where, keys=None):
    for k in keys or dev:
        np.testing.assert_array_equal(host[k], dev[k], err_msg=f"{where}: {k}")


def _actions(rng, A, N, wait=False):
    return rng.integers(0, 5 if wait else 4, size=(A, N), dtype=np.int32)


@pytest.mark.parametrize("name,N", [("fl2", 1), ("fl2", 63), ("fl2", 256), ("ow3", 1), ("ow3", 200), ("fl4", 5),
                                    ("fl2_slip", 1), ("fl2_slip", 130), ("fl2_randstart_slip", 1),
                                    ("fl2_randstart", 64), ("ow2_allslip", 1), ("ow3_slip", 17), ("ow1_map3", 3)])
def test_sync_equals_async(name, N, configs, torch):
    """300 steps with autoreset, sync handle vs async handle: every column after every step."""
    tab = T.compile_scenario(configs[name])
    a_env, s_env = _engine(tab, N), _engine(tab, N)
    a_env.reset(seed=11)
    out = s_env.reset_sync(seed=11)
    _assert_same(out, _dev_cols(a_env), "after reset", ("pos_x", "pos_y", "rm_q", "flags", "ep_ret", "t"))
    rng = np.random.default_rng(3)
    for s in range(300):
        acts = _actions(rng, tab.n_agents, N)
        a_env.step(torch.as_tensor(acts, device=a_env.device), autoreset=True)
        out = s_env.step_sync(acts, autoreset=True)
        _assert_same(out, _dev_cols(a_env), f"{name} N={N} step {s}")
    # the resident workgroup's write-back: the device columns of the sync handle continue identically
    s_env.sync_end()
    _assert_same(_dev_cols(s_env), _dev_cols(a_env), "after sync_end")
    if tab.stochastic or tab.random_starts:
        np.testing.assert_array_equal(s_env.rng.cpu().numpy(), a_env.rng.cpu().numpy())
        np.testing.assert_array_equal(s_env.episode.cpu().numpy(), a_env.episode.cpu().numpy())
    np.testing.assert_allclose(s_env.stats(), a_env.stats(), rtol=1e-12)


@pytest.mark.parametrize("name", ["fl2", "ow1"])
def test_sync_qrm_outputs(name, configs, torch):
    tab = T.compile_scenario(configs[name])
    a_env, s_env = _engine(tab, 3, with_qrm=True), _engine(tab, 3, with_qrm=True)
    a_env.reset(seed=5)
    s_env.reset_sync(seed=5)
    rng = np.random.default_rng(8)
    for s in range(200):
        acts = _actions(rng, tab.n_agents, 3)
        a_env.step(torch.as_tensor(acts, device=a_env.device), autoreset=True)
        out = s_env.step_sync(acts, autoreset=True)
        _assert_same(out, _dev_cols(a_env), f"{name} step {s}")


def test_sync_interleaved_with_async_and_oracle(configs, torch):
    """Sync steps, async steps, a sync reset, more sync steps on ONE handle = the oracle on the same actions."""
    tab = T.compile_scenario(configs["fl2_slip"])
    N = 9
    env = _engine(tab, N)
    orc = O.OracleEnv(tab, N)
    env.reset(seed=21)
    orc.reset(seed=21)
    rng = np.random.default_rng(1)
    for s in range(240):
        acts = _actions(rng, tab.n_agents, N)
        orc.step(acts)
        if (s // 40) % 3 == 0:
            out = env.step_sync(acts, autoreset=True)
            np.testing.assert_array_equal(out["pos_x"], orc.pos_x)
            np.testing.assert_array_equal(out["rm_q"], orc.rm_q)
        else:
            env.step(torch.as_tensor(acts, device=env.device), autoreset=True)
        if s == 150:
            out = env.reset_sync(seed=99)
            orc.reset(seed=99)
            np.testing.assert_array_equal(out["pos_x"], orc.pos_x)
    env.sync_end()
    np.testing.assert_array_equal(env.pos_x.cpu().numpy(), orc.pos_x)
    np.testing.assert_array_equal(env.pos_y.cpu().numpy(), orc.pos_y)
    np.testing.assert_array_equal(env.rm_q.cpu().numpy(), orc.rm_q)
    np.testing.assert_array_equal(env.flags.cpu().numpy().astype(np.uint32), orc.flags)


@pytest.mark.parametrize("mode", ["idle", "launch"])
def test_sync_relaunch_paths(mode, configs, torch, monkeypatch):
    """idle: a 30-us idle timeout with pauses between calls, so the workgroup exits and is relaunched (some
    requests land just as it times out); launch: one launch per call.  Both equal the async path."""
    if mode == "idle":
        monkeypatch.setenv("RMX_SYNC_IDLE_US", "30")
    else:
        monkeypatch.setenv("RMX_SYNC", "launch")
    tab = T.compile_scenario(configs["fl2_randstart_slip"])
    a_env, s_env = _engine(tab, 2), _engine(tab, 2)
    a_env.reset(seed=4)
    s_env.reset_sync(seed=4)
    rng = np.random.default_rng(6)
    for s in range(150):
        acts = _actions(rng, tab.n_agents, 2)
        a_env.step(torch.as_tensor(acts, device=a_env.device), autoreset=True)
        out = s_env.step_sync(acts, autoreset=True)
        _assert_same(out, _dev_cols(a_env), f"{mode} step {s}")
        if mode == "idle" and s % 7 == 3:
            time.sleep(rng.uniform(0, 2e-4))


def test_sync_errors(configs, torch):
    tab = T.compile_scenario(configs["fl2"])
    with pytest.raises(ValueError, match="RMX_SYNC_MAX_ENVS"):
        _engine(tab, 257).reset_sync(seed=1)
    env = _engine(tab, 2)
    env.reset_sync(seed=1)
    with pytest.raises(ValueError, match="outside"):
        env.step_sync(np.array([[0, 7], [1, 2]], np.int32))
    with pytest.raises(ValueError):  # the error word is also set for rmx_check_errors
        env.check_errors()
    out = env.step_sync(np.zeros((2, 2), np.int32))  # the handle keeps working
    assert out["t"].tolist() == [2, 2]


@pytest.mark.parametrize("name", ["fl2_randstart", "fl2_randstart_slip_fixed", "fl2_randstart_slip"])
def test_sync_reset_then_async_step_on_another_stream(name, configs, torch):
    """rmx_reset_sync with a new seed while the resident workgroup runs, then asynchronous steps on ANOTHER
    non-blocking stream: the start cache / next-episode precompute of the new seed is in place before the first of
    those steps (it is brought up to date on the stream of the launch that reads it), so every later autoreset
    equals the oracle's."""
    tab = T.compile_scenario(configs[name])
    N = 37
    env = _engine(tab, N)
    orc = O.OracleEnv(tab, N)
    env.reset(seed=3)
    orc.reset(seed=3)
    rng = np.random.default_rng(12)
    side = torch.cuda.Stream()
    for s in range(400):
        acts = _actions(rng, tab.n_agents, N)
        torch.cuda.current_stream().wait_stream(side)  # the caller orders its own streams before a sync call
        if s in (60, 230):
            out = env.reset_sync(seed=1000 + s)
            orc.reset(seed=1000 + s)
            np.testing.assert_array_equal(out["pos_x"], orc.pos_x)
            np.testing.assert_array_equal(out["pos_y"], orc.pos_y)
        orc.step(acts)
        if s % 50 < 10:
            out = env.step_sync(acts, autoreset=True)
            np.testing.assert_array_equal(out["pos_x"], orc.pos_x, err_msg=f"step {s}")
        else:
            with torch.cuda.stream(side):
                env.step(torch.as_tensor(acts, device=env.device), autoreset=True)
    env.sync_end()
    torch.cuda.synchronize()
    for k in ("pos_x", "pos_y", "rm_q"):
        np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, k), err_msg=k)
    np.testing.assert_array_equal(env.flags.cpu().numpy().astype(np.uint32), orc.flags)
    np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64), orc.rng)
    np.testing.assert_array_equal(env.episode.cpu().numpy(), orc.episode)
