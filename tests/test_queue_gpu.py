"""rmx_step_seq: K steps in one submission on the engine's own AQL queue (rmx_queue.cpp).

The window's launches are the ones rmx_step / rmx_step_report would issue (the same step_fast_kernel
instantiations and parameter blocks, recorded instead of launched), written as kernel-dispatch packets into an HSA
queue of the engine's.  Parity: the reference's golden trajectories stepped one window per step, the oracle at the
BASELINE configs' full size, and bit-equality with K rmx_step calls for every kernel family (the families that are
not the thread-per-env fast kernel take the stream path, which the queue counters show)."""
import os

import numpy as np
import pytest

import oracle as O
from rmx import tables as T
from rmx._capi import F_ACTIVE, F_TERM, F_TRUNC

pytestmark = pytest.mark.gpu

REWARD_TOL = 1e-6
COLS = ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward", "env_done", "rng", "episode", "enc_state",
        "shaping", "qrm_s", "qrm_sn", "qrm_rq", "qrm_done")
KNOBS = ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP", "RMX_LAYOUT",
         "RMX_QUEUE")


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    assert _t.cuda.is_available(), "gpu tests need a ROCm device"
    return _t


@pytest.fixture(autouse=True)
def _default_knobs(monkeypatch):
    for k in KNOBS:
        monkeypatch.delenv(k, raising=False)


def _engine(tab, n, **kw):
    from rmx.engine import VecRMEnv
    return VecRMEnv(tab, n, **kw)


def _assert_same(a, b, torch):
    for k in COLS:
        x, y = getattr(a, k, None), getattr(b, k, None)
        if x is not None:
            assert torch.equal(x, y), k


def _delta(before, after):
    return {k: after[k] - before[k] for k in before}


@pytest.mark.parametrize("report", [False, True])
@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_seq_vs_oracle_full_size(cfg, report, torch):
    """The headline path through the queue: 65,536 envs, 1,100 caller-action steps in 20-step windows (the bench's
    K), the last step of each window the fused report when `report`; state vs the oracle every 5 windows,
    statistics (and each window's report vector) vs the oracle."""
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, K, Tn, seed = 65536, 20, 1100, 77
    env = _engine(tab, N)
    assert env.step_variant == "fast" and env.report_fused
    orc = O.OracleEnv(tab, N)
    dev_acts = env.fill_actions(seed, 0, Tn)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    out = torch.zeros(4, dtype=torch.float64, device="cuda")
    c0 = env.queue_counters()
    for w in range(Tn // K):
        env.step_seq(dev_acts[w * K:(w + 1) * K], out=out if report else None)
        for s in range(w * K, (w + 1) * K):
            orc.step(acts[s])
        if report:
            r = out.cpu().numpy()
            assert r[1] == orc.stats[1] and r[2] == orc.stats[2] and r[3] == orc.stats[3], w
            np.testing.assert_allclose(r[0], orc.stats[0], rtol=1e-6, atol=1e-6)
        if w % 5 == 4:
            _compare_state(env, orc)
    _compare_state(env, orc)
    d = _delta(c0, env.queue_counters())
    assert d["windows"] == Tn // K and d["packets"] == Tn - Tn % K  # every window went through the queue
    # every window reads another action slice: only that slot range of the kernargs changes
    assert d["uploads"] <= Tn // K


def _compare_state(env, orc):
    for k in ("pos_x", "pos_y", "rm_q", "t"):
        np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, k), err_msg=k)
    np.testing.assert_array_equal(env.flags.cpu().numpy().view(np.uint32), orc.flags)
    np.testing.assert_array_equal(env.env_done.cpu().numpy(), orc.env_done)
    np.testing.assert_array_equal(env.reward.cpu().numpy(), orc.reward)
    np.testing.assert_allclose(env.ep_ret.cpu().numpy(), orc.ep_ret, rtol=1e-6, atol=1e-6)


TRAJ = ["fl2", "fl4", "fl2_quirks", "fl2_initfinal", "fl2_finalnt", "fl2_open", "ow1_map3", "ow1", "ow3",
        "ow2_fail", "ow2_final", "fl2_spec", "ow2_spec", "fl2_slip", "fl2_delay", "ow1_slip", "ow2_allslip",
        "ow2_delay", "ow3_slip", "fl2_randstart", "fl2_randstart_slip", "fl4_randstart_open"]


@pytest.mark.parametrize("name", TRAJ)
def test_seq_matches_reference_golden(name, configs, golden_dir, torch):
    """The reference-recorded trajectories (tests/golden/traj_*.npz) stepped through the queue, one window per
    step (K = 1) so every step's outputs are compared, then the whole trajectory again as ONE window from the same
    reset, compared at its end."""
    path = os.path.join(golden_dir, f"traj_{name}.npz")
    if not os.path.exists(path):
        pytest.skip(f"no golden {name}")
    g = dict(np.load(path))
    tab = T.compile_scenario(configs[name])
    acts = torch.as_tensor(g["actions"].astype(np.int32), device="cuda").contiguous()
    Tn, A, N = acts.shape
    env = _engine(tab, N)
    env.reset(seed=int(g["seed"]))
    # positions right after reset(seed) as the reference recorded them (every scenario: configured, build-defined
    # and random start positions)
    np.testing.assert_array_equal(env.pos_x.cpu().numpy(), g["reset_xy"][0, 0])
    np.testing.assert_array_equal(env.pos_y.cpu().numpy(), g["reset_xy"][0, 1])
    rec = {k: [] for k in ("pos_x", "pos_y", "q", "reward", "flags", "done", "t")}
    c0 = env.queue_counters()
    for s in range(Tn):
        env.step_seq(acts[s:s + 1])
        rec["pos_x"].append(env.pos_x.clone())
        rec["pos_y"].append(env.pos_y.clone())
        rec["q"].append(env.rm_q.clone())
        rec["reward"].append(env.reward.clone())
        rec["flags"].append(env.flags.clone())
        rec["done"].append(env.env_done.clone())
        rec["t"].append(env.t.clone())
    env.check_errors()
    if env.step_variant == "fast":
        assert _delta(c0, env.queue_counters())["packets"] == Tn
    r = {k: torch.stack(v).cpu().numpy() for k, v in rec.items()}
    np.testing.assert_array_equal(r["pos_x"], g["pos_x"])
    np.testing.assert_array_equal(r["pos_y"], g["pos_y"])
    np.testing.assert_array_equal(r["q"], g["q"])
    np.testing.assert_array_equal((r["flags"] & F_TERM) != 0, g["term"])
    np.testing.assert_array_equal((r["flags"] & F_TRUNC) != 0, g["trunc"])
    np.testing.assert_array_equal((r["flags"] & F_ACTIVE) != 0, g["active"])
    np.testing.assert_array_equal(r["done"].astype(bool), g["env_done"])
    np.testing.assert_array_equal(r["t"], g["t"])
    assert np.max(np.abs(r["reward"].astype(np.float64) - g["reward"])) <= REWARD_TOL
    env.reset(seed=int(g["seed"]))
    env.step_seq(acts)
    np.testing.assert_array_equal(env.pos_x.cpu().numpy(), g["pos_x"][-1])
    np.testing.assert_array_equal(env.pos_y.cpu().numpy(), g["pos_y"][-1])
    np.testing.assert_array_equal(env.rm_q.cpu().numpy(), g["q"][-1])
    np.testing.assert_array_equal(env.t.cpu().numpy(), g["t"][-1])


# (kernel family knobs, scenario, envs): the fast kernel in its table and store modes, with QRM outputs, slip and
# random starts, 256-thread blocks (1M envs) (the queue); the generic kernel and RMX_QUEUE=0 (the stream path)
FAMILIES = [
    ({}, "cfg2", 65536), ({}, "cfg4", 65536), ({}, "cfg3", 65536 + 77), ({}, "cfg5", 65536),
    ({"RMX_FAST_TABLES": "global"}, "cfg3", 4096), ({"RMX_FAST_TABLES": "merged"}, "cfg5", 4096),
    ({"RMX_FAST_TABLES": "merged"}, "cfg2", 4096), ({"RMX_FAST_SKIP": "3"}, "cfg2", 1 << 20), ({}, "cfg4", 1 << 20),
    ({"qrm": True}, "cfg4", 4096),
    ({}, "fl2_slip", 8192 + 37), ({}, "ow3_slip", 8192), ({}, "fl2_randstart", 8192), ({}, "fl2_randstart_slip", 8192),
    ({}, "fl2_randstart_slip_fixed", 8192), ({}, "fl4_randstart", 8192), ({}, "ow1_slip_fixed", 8192),
    ({"RMX_FAST_STATS": "wave"}, "cfg2", 65536), ({"RMX_FAST": "0"}, "cfg5", 8192),
    ({"RMX_FAST": "0", "RMX_LAYOUT": "lpe"}, "cfg2", 8192),
    ({"RMX_QUEUE": "0"}, "cfg2", 65536), ({"RMX_QUEUE": "0"}, "cfg4", 65536),
]


@pytest.mark.parametrize("knobs,scenario,n", FAMILIES,
                         ids=[f"{s}-{'-'.join(f'{k}={v}' for k, v in kn.items()) or 'default'}" for kn, s, _ in FAMILIES])
def test_seq_equals_steps(knobs, scenario, n, configs, torch, monkeypatch):
    """Three 37-step windows (the last with the report) equal 111 rmx_step calls with rmx_step_report last in each
    window: every column bit for bit, the report vectors equal; a masked reset with a new seed between windows
    (random starts: the reset cache goes dirty) and a repeated window on the same action slice (kernargs reused)."""
    qrm = bool(knobs.get("qrm"))
    for k, v in knobs.items():
        if k != "qrm":
            monkeypatch.setenv(k, v)
    desc = T.baseline_scenario(int(scenario[3:])) if scenario.startswith("cfg") else configs[scenario]
    tab = T.compile_scenario(desc)
    K, W, seed = 37, 3, 19
    a = _engine(tab, n, with_qrm=qrm, with_enc_state=not qrm)
    b = _engine(tab, n, with_qrm=qrm, with_enc_state=not qrm)
    for e in (a, b):
        e.reset(seed=5)
    acts = a.fill_actions(seed, 0, K * W)
    ra = torch.zeros(4, dtype=torch.float64, device="cuda")
    rb = torch.zeros(4, dtype=torch.float64, device="cuda")
    on_queue = a.step_variant == "fast" and knobs.get("RMX_QUEUE") != "0"
    c0 = b.queue_counters()
    mask = torch.zeros(n, dtype=torch.uint8, device="cuda")
    mask[::3] = 1
    for w in range(W):
        for s in range(w * K, (w + 1) * K - 1):
            a.step(acts[s])
        a.step_report(acts[(w + 1) * K - 1], out=ra)
        b.step_seq(acts[w * K:(w + 1) * K], out=rb)
        _assert_same(a, b, torch)
        assert torch.equal(ra, rb), (w, ra, rb)
        if w == 0:
            for e in (a, b):
                e.reset(mask=mask, seed=11)
    d = _delta(c0, b.queue_counters())
    assert d["windows"] == (W if on_queue else 0) and d["packets"] == (W * K if on_queue else 0)
    assert d["stream_windows"] == (0 if on_queue else W)
    assert b.queue_info()["dispatch"] == ("queue" if on_queue else "stream:disabled" if knobs.get("RMX_QUEUE") == "0"
                                          else "stream:kernel")
    if on_queue:  # the same slice again: same parameter blocks, nothing recorded or uploaded
        b.step_seq(acts[:K])
        c1 = b.queue_counters()
        b.step_seq(acts[:K])
        d1 = _delta(c1, b.queue_counters())
        assert d1["uploads"] == 0 and d1["recordings"] == 0 and d1["windows"] == 1
        for s in range(K):
            a.step(acts[s])
        for s in range(K):
            a.step(acts[s])
        _assert_same(a, b, torch)
    a.check_errors()
    b.check_errors()


def test_seq_longer_than_the_queue(torch):
    """A 2,500-step window (the queue holds 1,024 packets: the writer waits for room) equals 2,500 rmx_step calls."""
    tab = T.compile_scenario(T.baseline_scenario(4))
    n, K = 1024, 2500
    a, b = _engine(tab, n), _engine(tab, n)
    acts = a.fill_actions(3, 0, K)
    for s in range(K):
        a.step(acts[s])
    c0 = b.queue_counters()
    b.step_seq(acts)
    _assert_same(a, b, torch)
    assert _delta(c0, b.queue_counters())["packets"] == K
    assert torch.equal(a.stats_tensor(), b.stats_tensor())


@pytest.mark.parametrize("K,every", [(1, 1), (1, 50), (2, 50), (64, 1), (1500, 1), (1000, 50), (1000, 7)])
def test_dispatch_timing_stamps_the_strided_packets_and_changes_nothing(K, every, torch):
    """rmx_queue_timing(m): a timed window returns (packet, start, end) for packets 0, m, 2m, ... and the last one, in
    order (start < end; a later stamped packet starts after an earlier one completed: the barrier bit); its results
    equal an untimed window's from the same state; turning timing off leaves no stamps.  1,500 packets cross the
    1,024-packet ring."""
    tab = T.compile_scenario(T.baseline_scenario(2))
    n = 65536
    a, b = _engine(tab, n), _engine(tab, n)
    acts = a.fill_actions(9, 0, K)
    a.step_seq(acts)
    b.queue_timing(every)
    try:
        b.step_seq(acts)
        ts = b.queue_times().astype(np.int64)
    finally:
        b.queue_timing(0)
    _assert_same(a, b, torch)
    assert torch.equal(a.stats_tensor(), b.stats_tensor())
    assert b.queue_info()["dispatch"] == "queue"
    want = sorted(set(list(range(0, K - 1, every)) + [K - 1]))
    assert ts[:, 0].tolist() == want
    dur = ts[:, 2] - ts[:, 1]
    assert (dur > 0).all() and (dur < 10_000_000).all(), dur  # each dispatch 0 < d < 10 ms
    assert (ts[1:, 1] >= ts[:-1, 2]).all()  # a stamped packet starts after the previous stamped one completed
    if len(ts) > 2:  # a short buffer: *n is the full count, only cap triples are written
        import ctypes as C
        buf = np.full(3 * 3, 7, np.uint64)
        n = C.c_int64()
        assert b.lib.rmx_queue_times(b._h, buf.ctypes.data, 2, C.byref(n)) == 0
        assert n.value == len(ts) and (buf[:6].reshape(2, 3) == ts[:2].astype(np.uint64)).all() and (buf[6:] == 7).all()
    b.step_seq(acts)
    assert b.queue_times().shape == (0, 3)


def test_seq_orders_after_stream_work_and_before_later_work(torch):
    """Work enqueued on the caller's stream before the window (a reset, an action fill) runs first; work enqueued
    after it sees the window's results (step_seq returns once the steps are complete)."""
    tab = T.compile_scenario(T.baseline_scenario(2))
    n = 65536
    a, b = _engine(tab, n), _engine(tab, n)
    for w in range(5):
        acts = a.fill_actions(100 + w, 0, 20)  # fresh buffer, filled on the stream right before the window
        a.reset(seed=w)
        b.reset(seed=w)
        for s in range(20):
            a.step(acts[s])
        b.step_seq(acts)
        snapshot = b.pos_x.clone()  # enqueued after the window
        assert torch.equal(a.pos_x, snapshot)
        _assert_same(a, b, torch)


@pytest.mark.parametrize("cfg", [2, 5])
def test_seq_without_autoreset_equals_steps(cfg, torch):
    """autoreset = 0 (a caller that resets finished envs itself): windows equal the same rmx_step calls."""
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    n, K = 8192, 30
    a, b = _engine(tab, n), _engine(tab, n)
    acts = a.fill_actions(5, 0, 3 * K)
    for w in range(3):
        for s in range(w * K, (w + 1) * K):
            a.step(acts[s], autoreset=False)
        b.step_seq(acts[w * K:(w + 1) * K], autoreset=False)
        _assert_same(a, b, torch)
        done = a.env_done.clone()
        a.reset(mask=done)
        b.reset(mask=done)


def test_seq_handles_share_the_device_queue(torch):
    """Two handles (configs 2 and 5) alternate windows on the device's one queue (each window rebuilds the other's
    packets), then run windows from two host threads at once (ctypes releases the GIL: the queue's lock
    serialises them); both equal their own rmx_step calls."""
    import threading
    ta, tb = T.compile_scenario(T.baseline_scenario(2)), T.compile_scenario(T.baseline_scenario(5))
    n, K = 16384, 20
    a, a_ref = _engine(ta, n), _engine(ta, n)
    b, b_ref = _engine(tb, n), _engine(tb, n)
    acts_a, acts_b = a.fill_actions(1, 0, 8 * K), b.fill_actions(2, 0, 8 * K)
    ra, rb = (torch.zeros(4, dtype=torch.float64, device="cuda") for _ in range(2))
    for w in range(4):
        a.step_seq(acts_a[w * K:(w + 1) * K], out=ra)
        b.step_seq(acts_b[w * K:(w + 1) * K], out=rb)
    errors = []

    def run(env, acts, out):
        try:
            for w in range(4, 8):
                env.step_seq(acts[w * K:(w + 1) * K], out=out)
        except Exception as e:  # noqa: BLE001
            errors.append(e)

    th = [threading.Thread(target=run, args=x) for x in ((a, acts_a, ra), (b, acts_b, rb))]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for ref, acts, out in ((a_ref, acts_a, ra), (b_ref, acts_b, rb)):
        ref_out = torch.zeros(4, dtype=torch.float64, device="cuda")
        for s in range(8 * K):
            if s % K == K - 1:
                ref.step_report(acts[s], out=ref_out)
            else:
                ref.step(acts[s])
        assert torch.equal(ref_out, out)
    _assert_same(a, a_ref, torch)
    _assert_same(b, b_ref, torch)


def test_seq_window_is_step_seq(torch):
    """VecRMEnv.seq_window (the bench's bound form) runs the same window as step_seq on the buffers' current contents."""
    tab = T.compile_scenario(T.baseline_scenario(2))
    n, K = 65536, 20
    a, b = _engine(tab, n), _engine(tab, n)
    acts = a.fill_actions(7, 0, K)
    ra = torch.zeros(4, dtype=torch.float64, device="cuda")
    rb = torch.zeros(4, dtype=torch.float64, device="cuda")
    run = b.seq_window(acts, out=rb)
    for w in range(4):
        a.fill_actions(7 + w, 0, K, out=acts)  # refilled in place, as the bench does per window seed
        a.step_seq(acts, out=ra)
        assert run() is rb
        _assert_same(a, b, torch)
        assert torch.equal(ra, rb)
    with pytest.raises(ValueError):
        b.seq_window(acts[0])


def test_seq_rejects_bad_arguments(torch):
    tab = T.compile_scenario(T.baseline_scenario(2))
    env = _engine(tab, 256)
    acts = env.fill_actions(1, 0, 4)
    with pytest.raises(ValueError):
        env.step_seq(acts[0])  # [A, N]: not a window
    with pytest.raises(ValueError):
        env.step_seq(acts.to(torch.int64))
    with pytest.raises(ValueError):
        env.step_seq(acts, out=torch.zeros(4, dtype=torch.float32, device="cuda"))


_INJECT_CHILD = r"""
import sys, numpy as np, torch
sys.path[:0] = [%r, %r]
import oracle as O
from rmx import tables as T
from rmx.engine import VecRMEnv
mode = sys.argv[1]
tab = T.compile_scenario(T.baseline_scenario(2))
N, K = 8192, 20
env = VecRMEnv(tab, N)
orc = O.OracleEnv(tab, N)
acts = O.hash_actions(3, 0, 3 * K, N, 0, N, tab.n_agents)
dev = torch.as_tensor(acts, device="cuda").contiguous()
w0 = 0
if mode == "window":
    try:
        env.step_seq(dev[:K])
        raise SystemExit("the injected window failure did not raise")
    except RuntimeError as e:
        assert "did not complete" in str(e), e
    info = env.queue_info()
    assert info["state"] == "retired" and info["dispatch"] == "queue", info
    env.reset(seed=123)  # the failed window's results are undefined: start again
    w0 = 1
for w in range(w0, 3):
    env.step_seq(dev[w * K:(w + 1) * K])
    info = env.queue_info()
    assert info["dispatch"] == "stream:queue", info
for s in range(w0 * K, 3 * K):
    orc.step(acts[s])
for k in ("pos_x", "pos_y", "rm_q", "t"):
    np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, k), err_msg=k)
np.testing.assert_array_equal(env.flags.cpu().numpy().view(np.uint32), orc.flags)
info = env.queue_info()
assert info["state"] == ("retired" if mode == "window" else "unavailable"), info
assert info["stream_windows"] == 3 - w0, info
assert info["packets"] == 0, info
print("ok", mode, info)
"""


@pytest.mark.parametrize("mode", ["init", "window"])
def test_seq_falls_back_to_the_stream(mode, torch):
    """The queue cannot serve (fault injection, RMX_QUEUE_INJECT, read when the device's queue is set up, so in a
    child process): "init" — set-up fails, every window runs on the stream and equals the oracle; "window" — the
    first window fails as a timed-out one would (RMX_E_HIP, queue retired), later windows run on the stream and
    equal the oracle."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = _INJECT_CHILD % (os.path.join(root, "multiagent-rl-rm_amd"), os.path.join(root, "oracle"))
    env = dict(os.environ, RMX_QUEUE_INJECT=mode)
    r = subprocess.run([sys.executable, "-c", code, mode], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert f"ok {mode}" in r.stdout
