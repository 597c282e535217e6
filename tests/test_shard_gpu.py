"""BASELINE config 4's per-rank workload on one GPU: the 8-GPU job (524,288 FrozenLake map1 envs x 4 agents, one
65,536-env shard per rank at env offset g * 65,536) proven against the same job unsharded, on the path bench.py
times at N > 1: rmx_fill_actions (the SURVEY §8(d) counter hash over the GLOBAL env index and the global N) +
rmx_step_seq windows of 20 steps on the engine's queue, the last step of each window the fused statistics report.

The whole job (2.1 M env x agent instances) fits one MI355X, so "8 shards == 1 job" is checked on one box:
- every shard's columns equal the unsharded job's slice of them, bit for bit, after the run;
- the 8 shards' report vectors sum to the unsharded job's report after EVERY window (counts exact; return sums are
  sums of integer-valued FrozenLake returns, so exact too);
- rank 7's shard (the last, non-zero offset) equals the CPU oracle over the same global slice;
- every shard's windows ran on the engine's queue.
Reference semantics per shard are unchanged (ma_frozen_lake.py:96-215, rm_environment_wrapper.py:43-107); what this
pins is the offset / global-N plumbing of the sharded path (rmx/dist.py)."""
import numpy as np
import pytest

import oracle as O
from rmx import dist as RD
from rmx import tables as T

pytestmark = pytest.mark.gpu

COLS = ("pos_x", "pos_y", "rm_q", "flags", "t", "ep_ret", "reward", "env_done")


@pytest.fixture(scope="module")
def torch():
    import torch as _t
    assert _t.cuda.is_available(), "gpu tests need a ROCm device"
    return _t


@pytest.mark.parametrize("steps", [1100])
def test_config4_eight_shards_equal_the_unsharded_job(steps, torch, monkeypatch):
    from rmx.engine import VecRMEnv
    for k in ("RMX_FAST", "RMX_FAST_TABLES", "RMX_FAST_SKIP", "RMX_FAST_STATS", "RMX_GENERIC_SKIP", "RMX_QUEUE"):
        monkeypatch.delenv(k, raising=False)
    tab = T.compile_scenario(T.baseline_scenario(4))
    world, per, K, seed = 8, 65536, 20, 2024
    n_glob = world * per
    whole = VecRMEnv(tab, n_glob, with_renv=False)
    shards = []
    for g in range(world):
        off, n = RD.shard(n_glob, world, g)
        assert (off, n) == (g * per, per)
        shards.append(VecRMEnv(tab, n, env_offset=off, n_envs_global=n_glob, with_renv=False))
    for e in [whole] + shards:
        e.reset(seed=7)
        assert e.step_variant == "fast" and e.report_fused
    # rank 7's slice on the CPU oracle (same global env indices, same global N)
    off7 = 7 * per
    orc = O.OracleEnv(tab, per, env_offset=off7, n_envs_global=n_glob)
    orc.reset(seed=7)
    acts_w = whole.fill_actions(seed, 0, K)
    acts_s = [e.fill_actions(seed, 0, K) for e in shards]
    rep_w = torch.zeros(4, dtype=torch.float64, device="cuda")
    rep_s = [torch.zeros(4, dtype=torch.float64, device="cuda") for _ in shards]
    n_win = steps // K
    for w in range(n_win):
        whole.fill_actions(seed, w * K, K, out=acts_w)
        whole.step_seq(acts_w, out=rep_w)
        for e, a, r in zip(shards, acts_s, rep_s):
            e.fill_actions(seed, w * K, K, out=a)
            e.step_seq(a, out=r)
        tot = torch.stack(rep_s).sum(0).cpu().numpy()
        rw = rep_w.cpu().numpy()
        assert rw[1] == tot[1] and rw[2] == tot[2] and rw[3] == tot[3], (w, rw, tot)
        assert rw[0] == tot[0], (w, rw, tot)  # integer-valued FrozenLake returns: exact in f64
        for s in range(w * K, (w + 1) * K):
            orc.step(O.hash_actions(seed, s, 1, n_glob, off7, per, tab.n_agents)[0])
    whole.check_errors()
    for g, e in enumerate(shards):
        e.check_errors()
        sl = slice(g * per, (g + 1) * per)
        for k in COLS:
            a, b = getattr(whole, k), getattr(e, k)
            assert torch.equal(a[..., sl], b), (g, k)
        info = e.queue_info()
        assert info["dispatch"] == "queue", (g, info)
    # the rank-7 slice against the oracle, after 1,100 steps (crosses FrozenLake's t = 1001 truncation)
    e7 = shards[7]
    for k in ("pos_x", "pos_y", "rm_q", "t"):
        np.testing.assert_array_equal(getattr(e7, k).cpu().numpy(), getattr(orc, k), err_msg=k)
    np.testing.assert_array_equal(e7.flags.cpu().numpy().view(np.uint32), orc.flags)
    np.testing.assert_array_equal(e7.env_done.cpu().numpy(), orc.env_done)
    np.testing.assert_array_equal(e7.reward.cpu().numpy(), orc.reward)
    np.testing.assert_allclose(e7.ep_ret.cpu().numpy(), orc.ep_ret, rtol=1e-6, atol=1e-6)
    r7 = rep_s[7].cpu().numpy()
    assert r7[1] == orc.stats[1] and r7[2] == orc.stats[2] and r7[3] == orc.stats[3]
    np.testing.assert_allclose(r7[0], orc.stats[0], rtol=1e-9)
    assert orc.stats[1] > 0
    # the actions each shard generated are the unsharded job's slice (global env index, global N)
    for g, a in enumerate(acts_s):
        assert torch.equal(acts_w[:, :, g * per:(g + 1) * per], a)
    for e in [whole] + shards:
        e.close()
