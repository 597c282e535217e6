"""GPU parity: the HIP engine (through the C ABI) vs the reference golden vectors and the CPU oracle.

Bar: bit-exact integer state (positions, RM state, flags, timestep, env_done); rewards / shaping within
1e-6 (BASELINE.json north_star); episode statistics: counts exact, return sums within 1e-6 relative.
"""
import os

import numpy as np
import pytest

import oracle as O
from rmx import tables as T
from rmx._capi import F_ACTIVE, F_TERM, F_TRUNC

pytestmark = pytest.mark.gpu

REWARD_TOL = 1e-6
TRAJ = ["fl2", "fl4", "fl2_quirks", "fl2_initfinal", "fl2_finalnt", "fl2_open", "ow1_map3", "ow1", "ow3",
        "ow2_final", "ow2_fail", "fl2_spec", "ow2_spec", "fl2_slip", "fl2_delay", "ow1_slip", "ow2_allslip",
        "ow2_delay", "ow3_slip", "fl2_randstart", "fl2_randstart_slip", "fl4_randstart_open"]
# conftest.derived_configs: the random-start kernel paths the goldens do not reach (zero episode stride with slip,
# A = 4 under the default schedule, a non-zero stride without slip)
RS_DERIVED = ["fl2_randstart_slip_fixed", "fl4_randstart", "fl2_randstart_stride", "fl2_slip_stride", "ow1_slip_fixed"]


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    assert _t.cuda.is_available(), "gpu tests need a ROCm device"
    return _t


def _set_tables(monkeypatch, mode):
    """RMX_FAST_TABLES for a test mode name: fast_global / fast_merged / fast_merged4, else the default; an `_nt`
    suffix also sets RMX_FAST_SKIP=3 (the large-N store mode: rm_q / ep_ret skipped, non-temporal stores), otherwise
    the small-N default (rm_q / ep_ret skipped).  (Round 5 removed the step's LDS, lane-resident, speculative and
    8-B table modes, the lane-per-agent layout and the other store modes: they lost their A/Bs.)"""
    if mode.endswith("_nt"):
        monkeypatch.setenv("RMX_FAST_SKIP", "3")
        mode = mode[: -len("_nt")]
    else:
        monkeypatch.delenv("RMX_FAST_SKIP", raising=False)
    t = {"fast_global": "global", "fast_merged": "merged", "fast_merged4": "merged4"}.get(mode)
    if t:
        monkeypatch.setenv("RMX_FAST_TABLES", t)
    else:
        monkeypatch.delenv("RMX_FAST_TABLES", raising=False)


def _engine(tab, n, **kw):
    from rmx.engine import VecRMEnv
    return VecRMEnv(tab, n, **kw)


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_default_step_kernel(cfg, torch, monkeypatch):
    """BASELINE configs run the thread-per-env fast kernel by default."""
    for k in ("RMX_FAST", "RMX_FAST_TABLES"):
        monkeypatch.delenv(k, raising=False)
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    env = _engine(tab, 1024)
    assert env.step_variant == "fast"
    assert _engine(tab, 1024, with_qrm=True).step_variant == "fast"  # QRM outputs on the fast path too
    assert _engine(tab, 1 << 20).step_variant == "fast"  # bandwidth regime: fast kernel, skipped stores


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_full_size_step_vs_oracle(cfg, torch):
    """The headline path itself: 65,536 envs x 1,100 caller-action steps through rmx_step (default fast
    kernel), state compared every 100 steps, statistics at the end; OfficeWorld (configs 3 and 5) crosses its
    t > 1000 truncation at this size."""
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 65536, 1100, 77
    env = _engine(tab, N)
    assert env.step_variant == "fast"
    orc = O.OracleEnv(tab, N)
    dev_acts = env.fill_actions(seed, 0, Tn)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    for s in range(Tn):
        env.step(dev_acts[s])
        orc.step(acts[s])
        if s % 100 == 99:
            _compare_state(env, orc)
    _compare_stats(env.stats(), orc.stats)


@pytest.mark.parametrize("cfg", [2, 5])
def test_bandwidth_regime_default_vs_oracle(cfg, torch, monkeypatch):
    """The large-N default (2^20 envs: fast kernel, unchanged rm_q / ep_ret words not stored, per-wave stats)
    against the oracle: 120 hashed steps, state compared at 60 and 120, statistics at the end."""
    for k in ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP"):
        monkeypatch.delenv(k, raising=False)
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 1 << 20, 120, 5
    env = _engine(tab, N)
    assert env.step_variant == "fast"
    orc = O.OracleEnv(tab, N)
    # the oracle's rollout entry (the same hashed actions and autoreset, one env's steps in a row, OpenMP over envs:
    # equal to Tn single steps, and ~10x faster than stepping 2^20 envs column-wise)
    threads = min(16, os.cpu_count() or 1)
    for s0 in range(0, Tn, 60):
        for s in range(s0, s0 + 60):
            env.step_hashed(seed, s)
        orc.rollout(seed, s0, 60, n_threads=threads)
        _compare_state(env, orc)
    _compare_stats(env.stats(), orc.stats)


def test_library_is_the_hip_build(torch):
    """The library this GPU run loaded is the in-tree gfx950 build of exactly these sources (digest)."""
    from rmx import _capi
    lib = _capi.load_library()
    assert lib.rmx_abi_version() == _capi.ABI_VERSION
    assert os.path.samefile(lib._name, _capi.LIB_PATH)
    info = _capi.build_info(lib)
    assert info["src"] == _capi.source_hash() and info["arch"] == "gfx950", info


@pytest.mark.parametrize("mode", ["qrm", "qrm_generic", "fast", "fast_global", "fast_merged", "fast_merged4",
                                  "fast_nt", "fast_merged_nt"])
@pytest.mark.parametrize("name", TRAJ)
def test_engine_matches_reference_golden(name, mode, configs, golden_dir, torch, monkeypatch):
    """Deterministic scenarios run the fast kernel (every table and store mode; with QRM outputs its global-table
    instantiation); slip / random-start scenarios the fast kernel in the merged modes, else (and qrm_generic) the
    generic kernel.  Positions right after the first reset are compared too (every scenario: the configured or
    build-defined starts, and random_start_positions)."""
    monkeypatch.delenv("RMX_FAST", raising=False)
    if mode == "qrm_generic":
        monkeypatch.setenv("RMX_FAST", "0")
    _set_tables(monkeypatch, mode)
    g = dict(np.load(os.path.join(golden_dir, f"traj_{name}.npz")))
    tab = T.compile_scenario(configs[name])
    acts = torch.as_tensor(g["actions"].astype(np.int32), device="cuda")
    Tn, A, N = acts.shape
    env = _engine(tab, N, with_qrm=mode.startswith("qrm"))
    # slip and random starts run on the fast path in the default / merged / merged4 table modes with the small-N
    # store mode (rm_q / ep_ret skip stores, no QRM); every other stochastic or random-start case runs the generic
    # kernel
    rng = tab.stochastic or tab.random_starts
    fast_slip = rng and mode in ("fast", "fast_merged", "fast_merged4")
    if mode == "qrm_generic" or (rng and not fast_slip):
        assert env.step_variant == "generic"
    else:
        assert env.step_variant == "fast"
    env.reset(seed=int(g["seed"]))
    # positions right after reset(seed), as the reference recorded them (every scenario records its first reset)
    np.testing.assert_array_equal(g["reset_xy"][0] >= 0, True)
    np.testing.assert_array_equal(env.pos_x.cpu().numpy(), g["reset_xy"][0, 0])
    np.testing.assert_array_equal(env.pos_y.cpu().numpy(), g["reset_xy"][0, 1])
    rec = {k: [] for k in ("pos_x", "pos_y", "q", "reward", "shaping", "renv", "flags", "done", "t",
                           "qrm_s", "qrm_sn", "qrm_rq", "qrm_done")}
    for s in range(Tn):
        env.step(acts[s])
        rec["pos_x"].append(env.pos_x.clone())
        rec["pos_y"].append(env.pos_y.clone())
        rec["q"].append(env.rm_q.clone())
        rec["reward"].append(env.reward.clone())
        rec["shaping"].append(env.shaping.clone() if env.shaping is not None else torch.zeros_like(env.reward))
        rec["renv"].append(env.renv.clone())
        rec["flags"].append(env.flags.clone())
        rec["done"].append(env.env_done.clone())
        rec["t"].append(env.t.clone())
        if env.qrm_s is not None:
            for k in ("qrm_s", "qrm_sn", "qrm_rq", "qrm_done"):
                rec[k].append(getattr(env, k).clone())
    env.check_errors()
    r = {k: torch.stack(v).cpu().numpy() for k, v in rec.items() if v}
    np.testing.assert_array_equal(r["pos_x"], g["pos_x"])
    np.testing.assert_array_equal(r["pos_y"], g["pos_y"])
    np.testing.assert_array_equal(r["q"], g["q"])
    np.testing.assert_array_equal((r["flags"] & F_TERM) != 0, g["term"])
    np.testing.assert_array_equal((r["flags"] & F_TRUNC) != 0, g["trunc"])
    np.testing.assert_array_equal((r["flags"] & F_ACTIVE) != 0, g["active"])
    np.testing.assert_array_equal(r["done"].astype(bool), g["env_done"])
    np.testing.assert_array_equal(r["t"], g["t"])
    assert np.max(np.abs(r["reward"].astype(np.float64) - g["reward"])) <= REWARD_TOL
    assert np.max(np.abs(r["renv"].astype(np.float64) - g["renv"])) <= REWARD_TOL
    tot = r["reward"].astype(np.float64) + r["shaping"].astype(np.float64)
    assert np.max(np.abs(tot - (g["reward"] + g["shaping"]))) <= REWARD_TOL
    if "qrm_s" in r:  # QRM counterfactuals vs the reference's infos["qrm_experience"]
        from test_oracle_golden import check_qrm
        check_qrm(tab, r, g, g["actions"].astype(np.int32), r["renv"])


def _compare_state(env, orc):
    for k, ok in (("pos_x", "pos_x"), ("pos_y", "pos_y"), ("rm_q", "rm_q"), ("t", "t")):
        np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, ok), err_msg=k)
    np.testing.assert_array_equal(env.flags.cpu().numpy().view(np.uint32), orc.flags)
    np.testing.assert_array_equal(env.env_done.cpu().numpy(), orc.env_done)
    np.testing.assert_array_equal(env.reward.cpu().numpy(), orc.reward)
    np.testing.assert_allclose(env.ep_ret.cpu().numpy(), orc.ep_ret, rtol=1e-6, atol=1e-6)
    if env.shaping is not None:
        np.testing.assert_allclose(env.shaping.cpu().numpy(), orc.shaping, rtol=0, atol=REWARD_TOL)
    if env.enc_state is not None:  # learner input column (state_encoder_*.encode of the new observation)
        np.testing.assert_array_equal(env.enc_state.cpu().numpy(), orc.enc_state, err_msg="enc_state")


def _compare_stats(gpu, cpu):
    assert gpu[1] == cpu[1] and gpu[2] == cpu[2] and gpu[3] == cpu[3], (gpu, cpu)
    np.testing.assert_allclose(gpu[0], cpu[0], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("kernel", ["fast", "fast_global", "fast_merged", "fast_merged4", "fast_nt", "fast_global_nt",
                                    "fast_merged_nt", "generic", "generic_skip"])
@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_engine_vs_oracle_stepwise(cfg, kernel, torch, monkeypatch):
    """4,096 envs x 1,100 hashed steps (covers t=1001 truncation), state compared every 50 steps; the fast kernel
    in every table and store mode and the generic one (with its large-N store mode)."""
    monkeypatch.setenv("RMX_FAST", "0" if kernel.startswith("generic") else "1")
    monkeypatch.setenv("RMX_GENERIC_SKIP", "1" if kernel == "generic_skip" else "0")
    _set_tables(monkeypatch, kernel if kernel.startswith("fast") else "generic")
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 4096, 1100, 11 + cfg
    env = _engine(tab, N, with_enc_state=True)
    want = "generic" if kernel.startswith("generic") else "fast"
    assert env.step_variant == want
    orc = O.OracleEnv(tab, N)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    for s in range(Tn):
        env.step_hashed(seed, s)
        orc.step(acts[s])
        if s % 50 == 49 or s == Tn - 1:
            _compare_state(env, orc)
    _compare_stats(env.stats(), orc.stats)


@pytest.mark.parametrize("stats", ["wave", "env"])
@pytest.mark.parametrize("cfg", [2, 5])
def test_fast_stats_modes_vs_oracle(cfg, stats, torch, monkeypatch):
    """Both episode-statistics modes of the fast kernel (per-env atomic slots, per-wave slab) against the
    oracle, mixed with a rollout on the same handle (the slab is shared)."""
    monkeypatch.setenv("RMX_FAST_STATS", stats)
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 3000, 700, 41
    env = _engine(tab, N)
    orc = O.OracleEnv(tab, N)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    for s in range(Tn):
        env.step_hashed(seed, s)
        orc.step(acts[s])
    _compare_state(env, orc)
    _compare_stats(env.stats(), orc.stats)
    env.rollout(seed, Tn, 300)  # rollout kernel on the same handle (slab statistics)
    orc.rollout(seed, Tn, 300)
    _compare_state(env, orc)
    _compare_stats(env.stats(), orc.stats)
    env.clear_stats()
    assert np.all(env.stats() == 0)


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_full_size_rollout_vs_oracle(cfg, torch):
    """BASELINE size: 65,536 envs, 2,000 steps, fused rollout vs oracle rollout, bit-exact state."""
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 65536, 2000, 5
    env = _engine(tab, N, with_enc_state=True)
    env.rollout(seed, 0, Tn)
    orc = O.OracleEnv(tab, N)
    orc.rollout(seed, 0, Tn, n_threads=16)
    _compare_state(env, orc)
    _compare_stats(env.stats(), orc.stats)


@pytest.mark.parametrize("kernel", ["fast", "fast_global", "fast_merged", "fast_l2", "fast_global_l2", "generic"])
@pytest.mark.parametrize("cfg", [2, 3, 5])
def test_rollout_equals_stepwise(cfg, kernel, torch, monkeypatch):
    """The fused rollout (fast path: merged or global tables, staged in LDS or read through L2 (`_l2`);
    generic) ends in the state the step kernel reaches with the same hashed actions, and records the
    same rewards."""
    monkeypatch.setenv("RMX_FAST", "0" if kernel == "generic" else "1")
    monkeypatch.setenv("RMX_ROLLOUT_LDS", "0" if kernel.endswith("_l2") else "1")
    _set_tables(monkeypatch, kernel.replace("_l2", ""))
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 8192 + 37, 1200, 21
    a = _engine(tab, N)
    b = _engine(tab, N)
    for s in range(Tn):
        a.step_hashed(seed, s)
    trace = b.rollout(seed, 0, Tn, record_rewards=True)
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward", "env_done"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    sa, sb = a.stats(), b.stats()  # step and rollout kernels sum the returns in different orders
    np.testing.assert_array_equal(sa[1:], sb[1:])
    np.testing.assert_allclose(sa[0], sb[0], rtol=1e-12)
    # the trace of the rollout equals the per-step rewards (last row = the last step's reward)
    assert torch.equal(trace[-1], a.reward)
    c = _engine(tab, N)
    for s in range(Tn):
        c.step_hashed(seed, s)
        if s % 300 == 7:
            assert torch.equal(trace[s], c.reward), s


@pytest.mark.parametrize("fast", ["1", "global", "merged", "merged4", "0"])
def test_step_with_actions_equals_hashed(fast, torch, monkeypatch):
    monkeypatch.setenv("RMX_FAST", "0" if fast == "0" else "1")
    _set_tables(monkeypatch, "fast_" + fast)
    tab = T.compile_scenario(T.baseline_scenario(2))
    N, Tn, seed = 5000, 300, 9  # N not a multiple of the block size
    a = _engine(tab, N)
    b = _engine(tab, N)
    acts = b.fill_actions(seed, 0, Tn)
    ref = O.hash_actions(seed, 0, Tn, N, 0, N, 2)
    np.testing.assert_array_equal(acts.cpu().numpy(), ref)
    for s in range(Tn):
        a.step_hashed(seed, s)
        b.step(acts[s])
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k


def test_sharded_hash_matches_unsharded(torch):
    """A shard (env_offset, n_envs_global) runs exactly the envs of the unsharded job (§8(e))."""
    tab = T.compile_scenario(T.baseline_scenario(4))
    Ng, Tn, seed = 4096, 500, 2
    full = _engine(tab, Ng)
    lo = _engine(tab, Ng // 2, env_offset=0, n_envs_global=Ng)
    hi = _engine(tab, Ng // 2, env_offset=Ng // 2, n_envs_global=Ng)
    full.rollout(seed, 0, Tn)
    lo.rollout(seed, 0, Tn)
    hi.rollout(seed, 0, Tn)
    for k in ("pos_x", "pos_y", "rm_q", "flags"):
        assert torch.equal(torch.cat([getattr(lo, k), getattr(hi, k)], dim=1), getattr(full, k)), k
    np.testing.assert_allclose(lo.stats() + hi.stats(), full.stats(), rtol=1e-12)


@pytest.mark.parametrize("fast", ["1", "global", "merged", "merged4", "0"])
def test_reset_mask_and_invalid_action(fast, torch, monkeypatch):
    monkeypatch.setenv("RMX_FAST", "0" if fast == "0" else "1")
    _set_tables(monkeypatch, "fast_" + fast)
    tab = T.compile_scenario(T.baseline_scenario(2))
    env = _engine(tab, 256)
    for s in range(5):
        env.step_hashed(1, s)
    mask = torch.zeros(256, dtype=torch.uint8, device="cuda")
    mask[::2] = 1
    env.reset(mask)
    assert torch.all(env.t[::2] == 0) and torch.all(env.t[1::2] == 5)
    assert torch.all(env.pos_x[0, ::2] == 5) and torch.all(env.rm_q[:, ::2] == 0)
    bad = torch.full((2, 256), 7, dtype=torch.int32, device="cuda")
    env.step(bad)
    with pytest.raises(ValueError):
        env.check_errors()
    env.check_errors()  # cleared


def test_stats_clear(torch):
    tab = T.compile_scenario(T.baseline_scenario(2))
    env = _engine(tab, 1024)
    env.rollout(3, 0, 500)
    assert env.stats()[1] > 0
    env.clear_stats()
    assert np.all(env.stats() == 0)


@pytest.mark.parametrize("layout", ["tpe", "lpe"])
@pytest.mark.parametrize("cfg", [2, 5])
def test_both_layouts_match_oracle(layout, cfg, torch, monkeypatch):
    """The generic kernels' thread-per-env and lane-per-agent layouts (RMX_FAST=0, RMX_LAYOUT) for both
    step and rollout."""
    monkeypatch.setenv("RMX_FAST", "0")
    monkeypatch.setenv("RMX_LAYOUT", layout)
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 3000, 1050, 17
    env = _engine(tab, N, with_enc_state=True)
    orc = O.OracleEnv(tab, N)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    for s in range(Tn):
        env.step_hashed(seed, s)
        orc.step(acts[s])
    _compare_state(env, orc)
    _compare_stats(env.stats(), orc.stats)
    env2 = _engine(tab, N, with_enc_state=True)
    env2.rollout(seed, 0, Tn)
    _compare_state(env2, orc)
    _compare_stats(env2.stats(), orc.stats)


@pytest.mark.parametrize("kernel", ["fast", "generic_tpe", "generic_lpe"])
@pytest.mark.parametrize("cfg", [2, 4, 5])
def test_qrm_vs_oracle_large(cfg, kernel, torch, monkeypatch):
    """QRM outputs at 4,096 envs x 600 steps (cfg 5: exp5, 8 experiences per agent-step), on the fast
    kernel and both generic layouts."""
    monkeypatch.setenv("RMX_LAYOUT", "lpe" if kernel == "generic_lpe" else "tpe")
    monkeypatch.setenv("RMX_FAST", "1" if kernel == "fast" else "0")
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, Tn, seed = 4096, 600, 31
    env = _engine(tab, N, with_qrm=True)
    assert env.step_variant == {"fast": "fast", "generic_tpe": "generic", "generic_lpe": "lane_per_agent"}[kernel]
    orc = O.OracleEnv(tab, N)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    for s in range(Tn):
        env.step_hashed(seed, s)
        orc.step(acts[s])
        if s % 100 == 99:
            for k in ("qrm_s", "qrm_sn", "qrm_rq", "qrm_done"):
                np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, k), err_msg=k)
    _compare_state(env, orc)


@pytest.mark.parametrize("name", ["fl2", "fl2_quirks", "ow1", "ow3", "ow2_fail", "ow2_final", "ow1_map3", "fl2_spec",
                                  "ow2_spec"])
def test_mdp_matches_reference(name, configs, golden_dir, torch):
    """get_mdp on the GPU (one launch per agent) vs the reference's P dict, as arrays."""
    from test_oracle_golden import check_mdp
    g = dict(np.load(os.path.join(golden_dir, f"mdp_{name}.npz")))
    tab = T.compile_scenario(configs[name])
    env = _engine(tab, 1)
    for a in range(tab.n_agents):
        nxt, rew, done = (x.cpu().numpy() for x in env.mdp_arrays(a))
        check_mdp(tab, a, nxt, rew, done, g)
        # corrected FrozenLake decode vs the oracle's
        on, orw, od = O.mdp(tab, a, fix_fl=True)
        nxt, rew, done = (x.cpu().numpy() for x in env.mdp_arrays(a, fix_frozen_lake=True))
        np.testing.assert_array_equal(nxt, on)
        np.testing.assert_array_equal(done, od)
        np.testing.assert_array_equal(rew, orw)


@pytest.mark.parametrize("skip", ["generic", "generic_skip", "default"])
@pytest.mark.parametrize("name", ["fl2_slip", "fl2_delay", "ow2_allslip", "ow3_slip", "fl2_randstart", "fl2_randstart_slip",
                                  "fl4_randstart_open"] + RS_DERIVED)
def test_stochastic_large_vs_oracle(name, skip, configs, torch, monkeypatch):
    """Slip dynamics / random start positions at 8,192 envs: stepwise (caller actions) and fused rollout vs
    the oracle; generic_skip is the generic kernel's large-N store mode (unchanged column words not stored), generic
    the generic kernel storing every word, default: slip on the fast path (step_fast_kernel<..., SLIP>)."""
    for k in ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP"):
        monkeypatch.delenv(k, raising=False)
    if skip != "default":
        monkeypatch.setenv("RMX_FAST", "0")
        monkeypatch.setenv("RMX_GENERIC_SKIP", "1" if skip == "generic_skip" else "0")
    tab = T.compile_scenario(configs[name])
    N, Tn, seed, base = 8192, 1100, 41, 77
    env = _engine(tab, N, with_enc_state=True)
    fast_slip = skip == "default"  # slip and random starts: step_fast_kernel<..., SLIP> with the default stores
    assert env.step_variant == ("fast" if fast_slip else "generic")
    env.reset(seed=base)
    orc = O.OracleEnv(tab, N)
    orc.reset(seed=base)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    dacts = torch.as_tensor(acts, device="cuda")
    for s in range(Tn):
        env.step(dacts[s])
        orc.step(acts[s])
    _compare_state(env, orc)
    np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64), orc.rng)
    np.testing.assert_array_equal(env.episode.cpu().numpy(), orc.episode)
    _compare_stats(env.stats(), orc.stats)
    env2 = _engine(tab, N, with_enc_state=True)
    env2.reset(seed=base)
    env2.rollout(seed, 0, Tn)  # slip (default skip): rollout_fast_kernel<..., SLIP>
    _compare_state(env2, orc)
    np.testing.assert_array_equal(env2.rng.cpu().numpy().view(np.uint64), orc.rng)
    np.testing.assert_array_equal(env2.episode.cpu().numpy(), orc.episode)
    s2, so = env2.stats(), orc.stats
    np.testing.assert_array_equal(s2[1:], so[1:])
    np.testing.assert_allclose(s2[0], so[0], rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("name", ["fl2_slip", "fl2_delay", "ow1_slip", "ow2_allslip", "ow3_slip", "fl2_randstart",
                                  "fl2_randstart_slip", "fl4_randstart_open"] + RS_DERIVED)
@pytest.mark.parametrize("lds", ["0", "1"])
def test_slip_rollout_equals_stepwise(name, lds, configs, torch, monkeypatch):
    """Slip: the fused rollout (merged tables in LDS or through L2) ends where the step kernel's
    hashed steps do, rng / episode columns and per-step rewards included; a rollout continues a stepped engine."""
    for k in ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP"):
        monkeypatch.delenv(k, raising=False)
    monkeypatch.setenv("RMX_ROLLOUT_LDS", lds)
    tab = T.compile_scenario(configs[name])
    N, Tn, seed, base = 8192 + 37, 900, 13, 5
    a, b = _engine(tab, N), _engine(tab, N)
    a.reset(seed=base)
    b.reset(seed=base)
    for s in range(Tn):
        a.step_hashed(seed, s)
    trace = b.rollout(seed, 0, Tn - 300, record_rewards=True)
    b.rollout(seed, Tn - 300, 300)
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward", "env_done", "rng", "episode"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    sa, sb = a.stats(), b.stats()
    np.testing.assert_array_equal(sa[1:], sb[1:])
    np.testing.assert_allclose(sa[0], sb[0], rtol=1e-12)
    c = _engine(tab, N)
    c.reset(seed=base)
    for s in range(Tn - 300):
        c.step_hashed(seed, s)
        if s % 150 == 3:
            assert torch.equal(trace[s], c.reward), s


@pytest.mark.parametrize("name", ["fl2", "fl2_slip", "fl2_randstart_slip", "ow3", "fl2_randstart", "fl2_randstart_slip_fixed"])
def test_save_load_state_resumes_bit_exactly(name, configs, torch):
    """rmx_get_state / rmx_set_state (C ABI): a rollout checkpointed at step 400 and resumed in a FRESH engine
    continues exactly like the uninterrupted one (state columns, rng / episode columns, statistics)."""
    tab = T.compile_scenario(configs[name])
    N, seed = 3000, 13
    a = _engine(tab, N)
    a.reset(seed=5)
    for s in range(400):
        a.step_hashed(seed, s)
    blob = a.save_state()
    for s in range(400, 900):
        a.step_hashed(seed, s)
    b = _engine(tab, N)
    b.load_state(blob)
    for s in range(400, 900):
        b.step_hashed(seed, s)
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward") + (("rng", "episode") if a.rng is not None else ()):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    sa, sb = a.stats(), b.stats()
    np.testing.assert_array_equal(sa[1:], sb[1:])
    np.testing.assert_allclose(sa[0], sb[0], rtol=1e-12)
    c = _engine(T.compile_scenario(configs["fl4"]), N)
    with pytest.raises(ValueError):  # shape mismatch (agents) is refused
        c.load_state(blob)


def test_checkpoint_identity_refuses_other_scenario(configs, torch):
    """A blob of fl2 loads into fl2 but not into fl2_quirks (same A, N and columns; other holes / penalty) nor into
    the same scenario with another reward_modifier, nor into another shard of the same scenario
    (evaluation_metrics.py:193-214: checkpoints belong to one scenario); a blob whose columns point outside the
    tables is refused before anything is uploaded."""
    import dataclasses
    N = 512
    tab = T.compile_scenario(configs["fl2"])
    a = _engine(tab, N)
    for s in range(30):
        a.step_hashed(3, s)
    blob = a.save_state()
    _engine(tab, N).load_state(blob)  # same scenario: accepted
    with pytest.raises(ValueError, match="another scenario"):
        _engine(T.compile_scenario(configs["fl2_quirks"]), N).load_state(blob)
    with pytest.raises(ValueError, match="another scenario"):
        _engine(dataclasses.replace(tab, reward_modifier=2.0), N).load_state(blob)
    with pytest.raises(ValueError, match="another shard"):
        _engine(tab, N, env_offset=N, n_envs_global=2 * N).load_state(blob)
    bad = bytearray(blob)
    hdr = len(blob) - 4 * (5 * 2 * N + N)  # the columns follow the header: pos_x [A][N] first
    bad[hdr:hdr + 4] = (99).to_bytes(4, "little")
    b = _engine(tab, N)
    with pytest.raises(ValueError, match="outside"):
        b.load_state(bytes(bad))
    assert int(b.pos_x[0, 0]) != 99  # nothing was uploaded


@pytest.mark.parametrize("n,steps", [(65536, 120), (1 << 20, 24)])
def test_stats_report_every_step_vs_oracle(n, steps, torch):
    """The one-launch report (relaxed ticket, last-block reduction) right after every step, with several reports
    queued back to back on the stream before the host reads any: each equals the oracle's statistics at that
    step (counts exact, returns to 1e-6).  Both stats homes: per-env slots (65,536 envs, 65 blocks) and the
    per-wave slab (2^20 envs, 512 blocks)."""
    tab = T.compile_scenario(T.baseline_scenario(2))
    env = _engine(tab, n)
    orc = O.OracleEnv(tab, n)
    seed = 19
    for s in range(steps):
        env.step_hashed(seed, s)
        orc.step(O.hash_actions(seed, s, 1, n, 0, n, tab.n_agents)[0])
        outs = [env.stats_tensor().clone() for _ in range(3)]  # queued; no host sync in between
        want = orc.stats
        for o in outs:
            _compare_stats(o.cpu().numpy(), want)
    env.check_errors()


def test_stats_report_is_one_launch_and_repeatable(torch):
    """The fused statistics kernel (last-block reduction with a self-re-arming ticket) gives bit-identical
    reports when repeated, at both stats homes."""
    for n in (65536, 1 << 20):
        tab = T.compile_scenario(T.baseline_scenario(2))
        env = _engine(tab, n)
        env.rollout(3, 0, 300)
        for s in range(300, 320):
            env.step_hashed(3, s)
        r = [env.stats() for _ in range(4)]
        for x in r[1:]:
            np.testing.assert_array_equal(x, r[0])
        assert r[0][1] > 0


def test_state_encoder_kat_gpu(torch):
    """test_state_encoder_frozen_lake.py:21-43 through the engine's enc_state column (see the oracle KAT)."""
    from rmx.engine import VecRMEnv
    for transitions, start, want in (({("q0", None): ("q0", 0)}, (1, 2), 9), ({("q0", "a"): ("q1", 1)}, (1, 1), 18)):
        tab = T.compile_tables(T.FROZEN_LAKE, 4, 5, [], [], [start], [T.RewardMachineSpec(transitions)], [[]])
        env = VecRMEnv(tab, 3, with_enc_state=True)
        env.step(torch.ones((1, 3), dtype=torch.int32, device="cuda"))  # down
        assert env.pos_y.cpu().numpy().tolist() == [[2, 2, 2]]
        assert env.enc_state.cpu().numpy().tolist() == [[want] * 3]


@pytest.mark.parametrize("n,variant", [((1 << 29) - 32, "fast"), ((1 << 29) + 32, "generic")])
def test_maximum_sizes_vs_oracle_slices(n, variant, torch, monkeypatch):
    """The largest shards: 2^29 - 32 envs x 2 agents, just inside the fast path's 32-bit column offsets (A*N*4 <
    2^32), and 2^29 + 32, just past it (the generic kernel).  ~30 GB of columns; 4 hashed steps, then the first
    and the last 4,096 envs compared with the oracle run on those slices alone (the action hash uses the global
    env index, so a slice replays exactly)."""
    for k in ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP"):
        monkeypatch.delenv(k, raising=False)
    tab = T.compile_scenario(T.baseline_scenario(2))
    env = _engine(tab, n, with_renv=False)
    assert env.step_variant == variant
    seed, steps, k = 3, 4, 4096
    for s in range(steps):
        env.step_hashed(seed, s)
    env.check_errors()
    for off in (0, n - k):
        orc = O.OracleEnv(tab, k, env_offset=off, n_envs_global=n)
        for s in range(steps):
            orc.step(O.hash_actions(seed, s, 1, n, off, k, tab.n_agents)[0])
        for col in ("pos_x", "pos_y", "rm_q", "flags", "reward"):
            got = getattr(env, col)[:, off:off + k].cpu().numpy()
            want = getattr(orc, col)
            np.testing.assert_array_equal(got.view(want.dtype) if got.dtype != want.dtype else got, want,
                                          err_msg=f"{col} @ {off}")
        np.testing.assert_array_equal(env.t[off:off + k].cpu().numpy(), orc.t)
    del env
    torch.cuda.empty_cache()


@pytest.mark.parametrize("name", ["fl2_slip", "fl2_delay", "ow3_slip", "fl2_randstart", "fl2_randstart_slip",
                                  "fl2_randstart_slip_fixed", "fl4_randstart"])
def test_slip_default_at_2pow20_vs_oracle_slices(name, configs, torch, monkeypatch):
    """The slip default from 2^20 envs on (fast kernel, 256-thread workgroups, per-wave statistics slab): 150
    hashed steps stepwise and as one fused rollout, the first and last 4,096 envs against the oracle run on those
    slices alone (seeds and actions use the global env index), rng / episode columns included."""
    for k in ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP"):
        monkeypatch.delenv(k, raising=False)
    tab = T.compile_scenario(configs[name])
    n, steps, seed, base, k = 1 << 20, 150, 9, 21, 4096
    a = _engine(tab, n, with_renv=False)
    assert a.step_variant == "fast" and not a.report_fused  # per-wave statistics from 2^20 envs: no fused report
    a.reset(seed=base)
    for s in range(steps):
        a.step_hashed(seed, s)
    b = _engine(tab, n, with_renv=False)
    b.reset(seed=base)
    b.rollout(seed, 0, steps)
    a.check_errors()
    b.check_errors()
    for off in (0, n - k):
        orc = O.OracleEnv(tab, k, env_offset=off, n_envs_global=n)
        orc.reset(seed=base)
        for s in range(steps):
            orc.step(O.hash_actions(seed, s, 1, n, off, k, tab.n_agents)[0])
        for env, what in ((a, "step"), (b, "rollout")):
            for col in ("pos_x", "pos_y", "rm_q", "flags"):
                got = getattr(env, col)[:, off:off + k].cpu().numpy()
                want = getattr(orc, col)
                np.testing.assert_array_equal(got.view(want.dtype) if got.dtype != want.dtype else got, want,
                                              err_msg=f"{what} {col} @ {off}")
            np.testing.assert_array_equal(env.t[off:off + k].cpu().numpy(), orc.t)
            np.testing.assert_array_equal(env.rng[:, off:off + k].cpu().numpy().view(np.uint64), orc.rng)
            np.testing.assert_array_equal(env.episode[off:off + k].cpu().numpy(), orc.episode)
    del a, b
    torch.cuda.empty_cache()


@pytest.mark.parametrize("into", ["generic", "wave_stats", "merged", "global"])
@pytest.mark.parametrize("cfg", [2, 5])
def test_checkpoint_moves_between_kernels(cfg, into, torch, monkeypatch):
    """The checkpoint blob is layout-independent: saved from the default kernel at step 300, loaded into an
    engine that runs another kernel family / table mode / statistics home, resumed to step 700, it matches the
    uninterrupted default engine (state) and the oracle (statistics)."""
    for k in ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP"):
        monkeypatch.delenv(k, raising=False)
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    N, seed = 5000, 17
    a = _engine(tab, N)
    for s in range(300):
        a.step_hashed(seed, s)
    blob = a.save_state()
    for s in range(300, 700):
        a.step_hashed(seed, s)
    env_var = {"generic": ("RMX_FAST", "0"), "wave_stats": ("RMX_FAST_STATS", "wave"),
               "merged": ("RMX_FAST_TABLES", "merged"), "global": ("RMX_FAST_TABLES", "global")}[into]
    monkeypatch.setenv(*env_var)
    b = _engine(tab, N)
    b.load_state(blob)
    for s in range(300, 700):
        b.step_hashed(seed, s)
    for k in ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    orc = O.OracleEnv(tab, N)
    for s in range(700):
        orc.step(O.hash_actions(seed, s, 1, N, 0, N, tab.n_agents)[0])
    _compare_stats(b.stats(), orc.stats)


@pytest.mark.parametrize("tables", ["default", "merged", "merged4"])
@pytest.mark.parametrize("hashed", [True, False])
@pytest.mark.parametrize("name", ["fl2_slip", "fl2_delay", "ow1_slip", "ow2_allslip", "ow2_delay", "ow3_slip",
                                  "fl2_randstart", "fl2_randstart_slip", "fl4_randstart_open"] + RS_DERIVED)
def test_fast_slip_tables_vs_oracle(name, hashed, tables, configs, torch, monkeypatch):
    """Slip on the fast kernel, every table mode it runs with (merged 4-B records, 16-B records; OfficeWorld: the
    intended action's record decides the wall penalty and whether a draw happens), in-kernel hashed (rmx_step_hashed)
    or caller actions: 4,096 envs x
    1,100 steps against the oracle (OfficeWorld crosses its t > 1000 truncation), rng / episode columns included."""
    for k in ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_STATS", "RMX_FAST_SKIP", "RMX_GENERIC_SKIP"):
        monkeypatch.delenv(k, raising=False)
    if tables != "default":
        monkeypatch.setenv("RMX_FAST_TABLES", tables)
    tab = T.compile_scenario(configs[name])
    N, Tn, seed, base = 4096, 1100, 29, 11
    env = _engine(tab, N)
    assert env.step_variant == "fast"
    env.reset(seed=base)
    orc = O.OracleEnv(tab, N)
    orc.reset(seed=base)
    acts = O.hash_actions(seed, 0, Tn, N, 0, N, tab.n_agents)
    dacts = None if hashed else torch.as_tensor(acts, device="cuda")
    for s in range(Tn):
        if hashed:
            env.step_hashed(seed, s)
        else:
            env.step(dacts[s])
        orc.step(acts[s])
    _compare_state(env, orc)
    np.testing.assert_array_equal(env.rng.cpu().numpy().view(np.uint64), orc.rng)
    np.testing.assert_array_equal(env.episode.cpu().numpy(), orc.episode)
    _compare_stats(env.stats(), orc.stats)


@pytest.mark.parametrize("name", ["fl2_randstart", "fl2_randstart_slip_fixed", "fl2_randstart_slip", "fl4_randstart",
                                  "fl2_slip", "ow1_slip_fixed"])
def test_masked_reset_new_seed_random_starts_vs_oracle(name, configs, torch):
    """A masked rmx_reset with a NEW base seed moves the seed schedule of every env (the handle's base seed): the envs
    outside the mask keep their episode, and their next autoreset starts from the new seed's shuffle (the fixed-start
    cache is rebuilt for every env, the next-episode precompute restarts).  Stepwise and fused rollout vs the oracle,
    rng / episode columns included."""
    tab = T.compile_scenario(configs[name])
    N, seed = 4096 + 19, 23
    env, env2 = _engine(tab, N), _engine(tab, N)
    orc = O.OracleEnv(tab, N)
    for e in (env, env2, orc):
        e.reset(seed=7)
    mask = (np.arange(N) % 3 == 1).astype(np.uint8)
    for s in range(600):
        if s == 250:
            env.reset(mask=mask, seed=1234567)
            orc.reset(mask=mask, seed=1234567)
        env.step_hashed(seed, s)
        orc.step(O.hash_actions(seed, s, 1, N, 0, N, tab.n_agents)[0])
    env2.rollout(seed, 0, 250)
    env2.reset(mask=mask, seed=1234567)
    env2.rollout(seed, 250, 350)
    for e in (env, env2):
        _compare_state(e, orc)
        np.testing.assert_array_equal(e.rng.cpu().numpy().view(np.uint64), orc.rng)
        np.testing.assert_array_equal(e.episode.cpu().numpy(), orc.episode)
    env.check_errors()


@pytest.mark.parametrize("name", ["fl2_slip", "ow1_slip"])
def test_slip_per_action_cdfs_vs_oracle(name, configs, torch):
    """The draw's general form: intended actions with DIFFERENT cdfs / outcome counts (no reference map has them; the
    shared-cdf fast form covers those).  A table whose action 2 slips 50/25/25 and whose action 3 has four outcomes,
    stepwise and fused rollout against the oracle at 4,096 + 7 envs, rng columns included."""
    import dataclasses
    tab = T.compile_scenario(configs[name])
    cdf, n, out = tab.slip_cdf.copy(), tab.slip_n.copy(), tab.slip_out.copy()
    cdf[2, :3] = [0.5, 0.75, 1.0]
    n[3], out[3], cdf[3] = 4, [3, 0, 1, 4 if tab.kind == T.FROZEN_LAKE else 2], [0.4, 0.7, 0.9, 1.0]
    tab = dataclasses.replace(tab, slip_cdf=cdf, slip_n=n, slip_out=out)
    N, Tn, seed = 4096 + 7, 700, 31
    a, b = _engine(tab, N), _engine(tab, N)
    orc = O.OracleEnv(tab, N)
    for e in (a, b, orc):
        e.reset(seed=3)
    for s in range(Tn):
        a.step_hashed(seed, s)
        orc.step(O.hash_actions(seed, s, 1, N, 0, N, tab.n_agents)[0])
    b.rollout(seed, 0, Tn)
    for e in (a, b):
        _compare_state(e, orc)
        np.testing.assert_array_equal(e.rng.cpu().numpy().view(np.uint64), orc.rng)
    a.check_errors()


def test_output_tensors_are_checked_before_a_kernel_writes_them():
    """fill_actions / step_report / step_seq refuse an `out` of the wrong dtype, device, layout or size in Python,
    before any kernel writes through its address; a right one is filled (hashed actions in 0..3)."""
    import torch
    from rmx.engine import VecRMEnv

    tab = T.compile_scenario(T.baseline_scenario(2))
    N = 256
    env = VecRMEnv(tab, N)
    for out in (torch.zeros((3, 2, N - 1), dtype=torch.int32, device="cuda"),
                torch.zeros((3, 2, N), dtype=torch.int64, device="cuda"),
                torch.zeros((3, 2, N), dtype=torch.int32),
                torch.zeros((3, 2, 2 * N), dtype=torch.int32, device="cuda")[:, :, ::2]):
        with pytest.raises(ValueError, match="out must be"):
            env.fill_actions(1, 0, 3, out=out)
    acts = torch.zeros((2, N), dtype=torch.int32, device="cuda")
    for out in (torch.zeros(3, dtype=torch.float64, device="cuda"), torch.zeros(4, dtype=torch.float32, device="cuda")):
        with pytest.raises(ValueError, match="out must be"):
            env.step_report(acts, out=out)
        with pytest.raises(ValueError, match="out must be"):
            env.step_seq(acts[None], out=out)
    fa = env.fill_actions(1, 0, 3, out=torch.full((3, 2, N), -1, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
    assert bool(((fa >= 0) & (fa < 4)).all())
    env.check_errors()
