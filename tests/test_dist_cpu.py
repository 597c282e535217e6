"""Multi-rank path on CPU: world_size-2 gloo process group, each rank steps its env shard (the CPU
oracle stands in for the per-rank GPU engine here) and the statistics are SUM all-reduced, exactly as
bench.py / rmx.dist do with RCCL on the GPU box.  The sharded job must equal the unsharded one."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from rmx import dist as D
from rmx import tables as T


def test_shard_partition():
    for n, w in [(65536, 8), (10, 3), (7, 7), (524288, 8)]:
        spans = [D.shard(n, w, r) for r in range(w)]
        assert spans[0][0] == 0
        for (o1, n1), (o2, _) in zip(spans, spans[1:]):
            assert o1 + n1 == o2
        assert sum(s[1] for s in spans) == n
        assert max(s[1] for s in spans) - min(s[1] for s in spans) <= 1
    with pytest.raises(ValueError):
        D.shard(3, 4, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, n_global, steps, seed, cfg, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "multiagent-rl-rm_amd"), os.path.join(root, "oracle")]
    import torch
    import torch.distributed as dist

    import oracle as O
    from rmx import dist as RD
    from rmx import tables as RT

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    tab = RT.compile_scenario(RT.baseline_scenario(cfg))
    off, n = RD.shard(n_global, world, rank)
    env = O.OracleEnv(tab, n, env_offset=off, n_envs_global=n_global)
    env.rollout(seed, 0, steps)
    st = torch.tensor(env.stats, dtype=torch.float64)
    RD.allreduce_stats(st)
    out[rank] = (st.numpy().tolist(), env.pos_x.tolist(), env.rm_q.tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("cfg", [4, 5])
def test_gloo_two_ranks_equal_single_process(cfg):
    import oracle as O

    n_global, steps, seed = 1000, 700, 3
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, n_global, steps, seed, cfg, out)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    tab = T.compile_scenario(T.baseline_scenario(cfg))
    full = O.OracleEnv(tab, n_global)
    full.rollout(seed, 0, steps)
    st0, st1 = np.array(out[0][0]), np.array(out[1][0])
    np.testing.assert_array_equal(st0, st1)  # every rank holds the all-reduced aggregate
    np.testing.assert_array_equal(st0[1:], full.stats[1:])
    np.testing.assert_allclose(st0[0], full.stats[0], rtol=1e-12)
    pos = np.concatenate([np.array(out[0][1]), np.array(out[1][1])], axis=1)
    q = np.concatenate([np.array(out[0][2]), np.array(out[1][2])], axis=1)
    np.testing.assert_array_equal(pos, full.pos_x)
    np.testing.assert_array_equal(q, full.rm_q)


class _OracleVecEnv:
    """Stand-in for rmx.engine.VecRMEnv behind the same interface (constructor, rollout, stats_tensor,
    columns), backed by the CPU oracle: the code under test below is rmx.dist itself."""

    def __init__(self, tables, n_envs, device=0, env_offset=0, n_envs_global=None, **kw):
        import oracle as O
        self.o = O.OracleEnv(tables, n_envs, env_offset=env_offset, n_envs_global=n_envs_global)
        self.device = device

    def rollout(self, seed, t0, T, record_rewards=False):
        self.o.rollout(seed, t0, T)

    def stats_tensor(self):
        import torch
        return torch.tensor(self.o.stats, dtype=torch.float64)

    @property
    def pos_x(self):
        return self.o.pos_x

    @property
    def rm_q(self):
        return self.o.rm_q


def _sharded_rank_main(rank, world, port, n_global, steps, seed, cfg, out):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "multiagent-rl-rm_amd"), os.path.join(root, "oracle"),
                    os.path.join(root, "tests")]
    import torch.distributed as dist

    import rmx.engine as E
    from rmx import dist as RD
    from rmx import tables as RT
    from test_dist_cpu import _OracleVecEnv

    E.VecRMEnv = _OracleVecEnv  # the per-rank engine; ShardedVecRMEnv imports it at construction
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    rank_, world_, local_ = RD.init("gloo")
    assert (rank_, world_, local_) == (rank, world, rank)
    tab = RT.compile_scenario(RT.baseline_scenario(cfg))
    env = RD.ShardedVecRMEnv(tab, n_global)  # rank / world / device from the launcher environment
    assert (env.rank, env.world) == (rank, world) and env.offset == RD.shard(n_global, world, rank)[0]
    env.rollout(seed, 0, steps)  # delegated to the per-rank engine
    out[rank] = (env.global_stats().tolist(), env.pos_x.tolist(), env.offset, env.n)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_vec_env_global_stats(world):
    """rmx.dist.ShardedVecRMEnv under a gloo group: shards from the launcher environment, the engine's
    columns through delegation, and global_stats() == the unsharded job's statistics on every rank."""
    import oracle as O

    n_global, steps, seed, cfg = 999, 600, 8, 2
    ctx = mp.get_context("spawn")
    mgr = ctx.Manager()
    out = mgr.dict()
    port = _free_port()
    procs = [ctx.Process(target=_sharded_rank_main, args=(r, world, port, n_global, steps, seed, cfg, out))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    full = O.OracleEnv(T.compile_scenario(T.baseline_scenario(cfg)), n_global)
    full.rollout(seed, 0, steps)
    for r in range(world):
        st = np.array(out[r][0])
        np.testing.assert_array_equal(st[1:], full.stats[1:])
        np.testing.assert_allclose(st[0], full.stats[0], rtol=1e-12)
    pos = np.concatenate([np.array(out[r][1]) for r in range(world)], axis=1)
    np.testing.assert_array_equal(pos, full.pos_x)
    assert sum(out[r][3] for r in range(world)) == n_global
