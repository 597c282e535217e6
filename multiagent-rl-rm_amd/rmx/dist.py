"""One process per GPU: contiguous env shards + ONE all-reduce of the episode statistics.

SURVEY.md §8(e): envs are independent, so rank g of G owns envs [offset_g, offset_g + n_g) with its own
table copy and its own action stream (the counter hash uses the GLOBAL env index, so trajectories
are identical for every G).  The only collective is a SUM all-reduce of the 4 x f64 statistics vector
(sum return, episodes, successes, sum length) at the end of a reporting window — RCCL over xGMI when
the process group backend is "nccl", gloo in the CPU tests.  The reference has no distributed code.
"""
from __future__ import annotations

import os
from typing import Tuple


def shard(n_global: int, world: int, rank: int) -> Tuple[int, int]:
    """(env_offset, n_envs) of `rank`: contiguous, sizes differ by at most one."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError("bad world/rank")
    if n_global < world:
        raise ValueError("fewer envs than ranks")
    base, extra = divmod(n_global, world)
    n = base + (1 if rank < extra else 0)
    off = rank * base + min(rank, extra)
    return off, n


def env_rank():
    """(rank, world, local_rank) from the torchrun environment (1-process defaults)."""
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


# Rendezvous and collective timeout: a rank that dies or hangs makes the others fail with a message well inside a
# driver's 600-s limit instead of sitting in the collective until they are killed (RMX_PG_TIMEOUT_S overrides).
PG_TIMEOUT_S = 120.0


def init(backend: str = "nccl", timeout_s: float = None):
    """Initialise the default process group (MASTER_ADDR/PORT from the launcher) if world > 1, with an explicit
    timeout for the rendezvous and every collective."""
    import datetime

    import torch
    import torch.distributed as dist

    rank, world, local = env_rank()
    if timeout_s is None:
        timeout_s = float(os.environ.get("RMX_PG_TIMEOUT_S", PG_TIMEOUT_S))
    timeout = datetime.timedelta(seconds=timeout_s)
    if world > 1 and not dist.is_initialized():
        if backend == "nccl":
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local), timeout=timeout)
        else:
            dist.init_process_group(backend, timeout=timeout)
    return rank, world, local


def collective_device(backend: str, local: int):
    """Where the collectives' tensors live: this rank's GPU under "nccl" (RCCL reduces device memory over xGMI),
    the host under gloo.  Every caller builds its collective tensors here, so the RCCL run and the gloo rehearsal
    issue the same calls on the same kind of tensor (one resident on the collective's own device)."""
    import torch

    return torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")


def _world():
    import torch.distributed as dist

    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def allreduce_stats(stats, device=None):
    """In-place SUM of a float64[4] statistics tensor over all ranks (no-op when not distributed).  `device`: the
    collective device (collective_device); a tensor elsewhere (a GPU report under the gloo rehearsal) is reduced
    through a copy there.  A tensor already on it — every RCCL call — is reduced in place with no copy."""
    import torch
    import torch.distributed as dist

    if _world() > 1:
        if device is None:
            device = stats.device if dist.get_backend() != "gloo" else "cpu"
        device = torch.device(device)
        x = stats if stats.device == device else stats.to(device)
        dist.all_reduce(x, op=dist.ReduceOp.SUM)
        if x is not stats:
            stats.copy_(x)
    return stats


def max_over_ranks(values, device):
    """The element-wise MAX over ranks of a few host floats (one all-reduce of an f64 tensor on the collective
    device); the values themselves at world 1."""
    import torch
    import torch.distributed as dist

    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if _world() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


class ShardedVecRMEnv:
    """This rank's shard of an n_global-env job on its local GPU (weak or strong scaling)."""

    def __init__(self, tables, n_global: int, rank: int = None, world: int = None, device: int = None, **kw):
        from .engine import VecRMEnv

        r, w, local = env_rank()
        self.rank = r if rank is None else rank
        self.world = w if world is None else world
        self.offset, self.n = shard(n_global, self.world, self.rank)
        self.n_global = n_global
        self.env = VecRMEnv(tables, self.n, device=local if device is None else device, env_offset=self.offset,
                            n_envs_global=n_global, **kw)

    def __getattr__(self, name):
        return getattr(self.env, name)

    def global_stats(self):
        """All-reduced statistics (the job-wide aggregate episodic-return statistic)."""
        st = self.env.stats_tensor()
        allreduce_stats(st)
        return st.cpu().numpy().copy()
