"""GPU parity of rmx_step_report: a step whose launch also produces the episode-statistics report.

Contract (include/rmx.h): rmx_step_report(h, actions, autoreset, out) == rmx_step(h, actions, autoreset)
followed by rmx_stats_device(h, out) on the same stream.  Where the handle runs the default thread-per-env
fast kernel below 1M envs the report is computed inside the step launch (step_fast_kernel<..., RPT>); the
state it leaves must be bit-identical to rmx_step's, the integer statistics identical, and the return sum equal
up to the association of its fixed-order sum.  Everywhere else it is the two launches, bit-identical.
"""
import numpy as np
import pytest

import oracle as O
from rmx import tables as T

pytestmark = pytest.mark.gpu

ENV_KEYS = ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP", "RMX_LAYOUT")
STATE = ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward", "env_done")


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    assert _t.cuda.is_available(), "gpu tests need a ROCm device"
    return _t


def _clean(monkeypatch, extra=None):
    for k in ENV_KEYS:
        monkeypatch.delenv(k, raising=False)
    for k, v in (extra or {}).items():
        monkeypatch.setenv(k, v)


def _engine(tab, n, **kw):
    from rmx.engine import VecRMEnv
    return VecRMEnv(tab, n, **kw)


def _same_state(a, b):
    for k in STATE:
        np.testing.assert_array_equal(getattr(a, k).cpu().numpy(), getattr(b, k).cpu().numpy(), err_msg=k)


def _same_report(got, want, exact):
    got, want = np.asarray(got), np.asarray(want)
    np.testing.assert_array_equal(got[1:], want[1:])  # episodes, successes, length: integers, exact in f64
    if exact:
        np.testing.assert_array_equal(got[0], want[0])
    else:  # the fused report's own fixed association order
        np.testing.assert_allclose(got[0], want[0], rtol=1e-12, atol=1e-9)


@pytest.mark.parametrize("n", [65536, 1500, 63, 1])
@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_step_report_equals_step_then_stats(cfg, n, torch, monkeypatch):
    """Every step reported, several reports queued before the host reads any; against a twin engine that runs
    rmx_step + rmx_stats_device and against the CPU oracle.  Ragged sizes: one partial block (63, 1) and a
    tail block (1500)."""
    _clean(monkeypatch)
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    a, b = _engine(tab, n), _engine(tab, n)
    assert a.report_fused  # the default kernel below 1M envs fuses the report
    orc = O.OracleEnv(tab, n)
    Tn, seed = 260, 11
    acts = a.fill_actions(seed, 0, Tn)
    host = O.hash_actions(seed, 0, Tn, n, 0, n, tab.n_agents)
    pend = []
    for s in range(Tn):
        got = a.step_report(acts[s], out=torch.empty(4, dtype=torch.float64, device="cuda"))
        b.step(acts[s])
        pend.append((got, b.stats_tensor().clone()))
        orc.step(host[s])
        if s % 20 == 19:  # compare the queued reports of the last 20 steps
            for g, w in pend:
                _same_report(g.cpu().numpy(), w.cpu().numpy(), exact=False)
            pend.clear()
            o = orc.stats
            g = got.cpu().numpy()
            assert g[1] == o[1] and g[2] == o[2] and g[3] == o[3], (g, o)
            np.testing.assert_allclose(g[0], o[0], rtol=1e-6, atol=1e-6)
    _same_state(a, b)
    for k in ("pos_x", "pos_y", "rm_q", "t"):  # and the oracle's state
        np.testing.assert_array_equal(getattr(a, k).cpu().numpy(), getattr(orc, k), err_msg=k)
    np.testing.assert_array_equal(a.flags.cpu().numpy().view(np.uint32), orc.flags)
    np.testing.assert_array_equal(a.env_done.cpu().numpy(), orc.env_done)
    a.check_errors()


RNG_SCENARIOS = {  # the fast kernel's SLIP instantiations, reported (round 5: the report fused there too)
    "rs2": (2, {"random_start_positions": True}),            # kRngStarts | kRngFixedSeed (the runner's schedule)
    "rs4": (4, {"random_start_positions": True}),
    "rs2_stride": (2, {"random_start_positions": True, "seed_schedule": (1, 1, 1)}),  # kRngStarts (precompute)
    "slip2": (2, {"stochastic": True}),                      # kRngSlip
    "rsslip2": (2, {"random_start_positions": True, "stochastic": True}),
    "slip5": (5, {"stochastic": True}),                      # OfficeWorld slip
}


@pytest.mark.parametrize("n", [16384, 1500, 1])
@pytest.mark.parametrize("name", sorted(RNG_SCENARIOS))
def test_step_report_with_slip_and_random_starts(name, n, torch, monkeypatch):
    """The reported step of the slip / random-start instantiations: bit-identical state (rng columns included) to
    rmx_step + rmx_stats_device on a twin, the report equal to the twin's, statistics and state equal to the CPU
    oracle's."""
    _clean(monkeypatch)
    cfg, extra = RNG_SCENARIOS[name]
    tab = T.compile_scenario(dict(T.baseline_scenario(cfg), **extra))
    a, b = _engine(tab, n), _engine(tab, n)
    assert a.step_variant == "fast" and a.report_fused, (a.step_variant, a.report_fused)
    orc = O.OracleEnv(tab, n)
    for e in (a, b, orc):
        e.reset(seed=21)
    Tn, seed = 240, 13
    acts = a.fill_actions(seed, 0, Tn)
    host = O.hash_actions(seed, 0, Tn, n, 0, n, tab.n_agents)
    for s in range(Tn):
        got = a.step_report(acts[s], out=torch.empty(4, dtype=torch.float64, device="cuda"))
        b.step(acts[s])
        orc.step(host[s])
        if s % 40 == 39:
            _same_report(got.cpu().numpy(), b.stats_tensor().cpu().numpy(), exact=False)
            g, o = got.cpu().numpy(), orc.stats
            assert g[1] == o[1] and g[2] == o[2] and g[3] == o[3], (s, g, o)
            np.testing.assert_allclose(g[0], o[0], rtol=1e-6, atol=1e-6)
    _same_state(a, b)
    for k in ("rng", "episode"):
        if getattr(a, k, None) is not None:
            np.testing.assert_array_equal(getattr(a, k).cpu().numpy(), getattr(b, k).cpu().numpy(), err_msg=k)
    for k in ("pos_x", "pos_y", "rm_q", "t"):
        np.testing.assert_array_equal(getattr(a, k).cpu().numpy(), getattr(orc, k), err_msg=k)
    np.testing.assert_array_equal(a.flags.cpu().numpy().view(np.uint32), orc.flags)
    if getattr(a, "rng", None) is not None and orc.rng is not None:
        np.testing.assert_array_equal(a.rng.cpu().numpy().view(np.uint64), orc.rng)
    a.check_errors()


@pytest.mark.parametrize("cfg", [2, 5])
def test_step_report_folds_in_the_slab(cfg, torch, monkeypatch):
    """The slab (written by the fused rollout and by a restored checkpoint) is part of the report: a rollout,
    then reported steps, then a save / load into a fresh engine and more reported steps."""
    _clean(monkeypatch)
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    n = 65536
    a, b = _engine(tab, n), _engine(tab, n)
    a.rollout(4, 0, 300)
    b.rollout(4, 0, 300)
    acts = a.fill_actions(4, 300, 40)
    for s in range(40):
        got = a.step_report(acts[s]).clone()
        b.step(acts[s])
        _same_report(got.cpu().numpy(), b.stats(), exact=False)
    blob = a.save_state()
    c = _engine(tab, n)
    c.load_state(blob)
    assert c.report_fused
    more = c.fill_actions(4, 340, 10)
    for s in range(10):
        got = c.step_report(more[s]).clone()
        b.step(more[s])
        _same_report(got.cpu().numpy(), b.stats(), exact=False)
    _same_state(c, b)


def test_step_report_is_repeatable_and_graph_safe(torch, monkeypatch):
    """Two engines on the same actions give bit-identical fused reports; a captured graph of 19 steps + one
    reported step replayed twice equals the same sequence run eagerly (the ticket re-arms inside the graph)."""
    _clean(monkeypatch)
    tab = T.compile_scenario(T.baseline_scenario(2))
    n, K = 65536, 20
    a, b, c = _engine(tab, n), _engine(tab, n), _engine(tab, n)
    acts = a.fill_actions(8, 0, 2 * K)
    for s in range(2 * K):
        ra = a.step_report(acts[s]).clone()
        rb = b.step_report(acts[s]).clone()
        np.testing.assert_array_equal(ra.cpu().numpy(), rb.cpu().numpy())
    out = torch.zeros(4, dtype=torch.float64, device="cuda")
    win = torch.empty((K,) + tuple(acts.shape[1:]), dtype=torch.int32, device="cuda")
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        with torch.cuda.graph(g, stream=s0):
            for s in range(K - 1):
                c.step(win[s])
            c.step_report(win[K - 1], out=out)
    torch.cuda.current_stream().wait_stream(s0)
    c.reset()
    c.clear_stats()
    for w in range(2):
        win.copy_(acts[w * K:(w + 1) * K])
        g.replay()
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out.cpu().numpy(), rb.cpu().numpy() if w == 1 else _report_at(tab, n, acts, K))
    _same_state(c, b)


def _report_at(tab, n, acts, K):
    """The fused report after the first K steps of a fresh engine (eager)."""
    e = _engine(tab, n)
    r = None
    for s in range(K):
        r = e.step_report(acts[s])
    return r.cpu().numpy()


@pytest.mark.parametrize("mode", ["wave_stats", "generic", "generic_lpe", "nt", "qrm"])
def test_step_report_unfused_modes_are_step_then_stats(mode, torch, monkeypatch):
    """Handles whose step kernel does not fuse the report run the step launch then the stats launch: the report
    is bit-identical to rmx_step + rmx_stats_device."""
    extra = {"wave_stats": {"RMX_FAST_STATS": "wave"}, "generic": {"RMX_FAST": "0"},
             "generic_lpe": {"RMX_FAST": "0", "RMX_LAYOUT": "lpe"}, "nt": {"RMX_FAST_SKIP": "3"}, "qrm": {}}[mode]
    _clean(monkeypatch, extra)
    tab = T.compile_scenario(T.baseline_scenario(2))
    n = 4096
    kw = {"with_qrm": True} if mode == "qrm" else {}
    a, b = _engine(tab, n, **kw), _engine(tab, n, **kw)
    assert not a.report_fused
    acts = a.fill_actions(2, 0, 120)
    for s in range(120):
        got = a.step_report(acts[s]).clone()
        b.step(acts[s])
        _same_report(got.cpu().numpy(), b.stats(), exact=True)
    _same_state(a, b)


@pytest.mark.parametrize("cfg,n", [(2, (1 << 20) - 1), (4, 262147)])
def test_step_report_large_grids(cfg, n, torch, monkeypatch):
    """The largest fused grids (just below the 1M-env switch to per-wave slots: 16,384 blocks, 512 arrivals per
    shard counter, several 1,024-block chunks in the last block's partial sum) and a ragged A = 4 size."""
    _clean(monkeypatch)
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    a, b = _engine(tab, n), _engine(tab, n)
    assert a.report_fused
    acts = a.fill_actions(6, 0, 30)
    for s in range(30):
        got = a.step_report(acts[s]).clone()
        b.step(acts[s])
        if s % 10 == 9:
            _same_report(got.cpu().numpy(), b.stats(), exact=False)
    _same_state(a, b)
