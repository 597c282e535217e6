"""The RCCL path on the one GPU this pool gives: a single-rank "nccl" process group (RCCL, the backend bench.py and
rmx/dist.py use at N > 1) in the same process as the engine and its own AQL queue.

What this pins: RCCL initialises next to the engine's HSA queue (rmx_queue.cpp) on one device; the statistics
all-reduce of rmx/dist.py (ONE SUM all-reduce of the 4 x f64 vector per reporting window) runs on RCCL
between queue windows and returns the window's report; the windows keep running on the queue afterwards and stay
equal to the CPU oracle.  A world of one is the most RCCL allows on one GPU (two ranks on one device are refused by
RCCL, and by bench.py's collective block); the driver's N = 2..8 runs take the same code with one GPU per rank.
Runs in a child process so the process group does not outlive the test."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_CHILD = r"""
import datetime, sys, numpy as np, torch
import torch.distributed as dist
sys.path[:0] = [%r, %r]
import oracle as O
from rmx import dist as RD
from rmx import tables as T
from rmx.engine import VecRMEnv
torch.cuda.set_device(0)
dist.init_process_group("nccl", device_id=torch.device("cuda", 0), rank=0, world_size=1,
                        timeout=datetime.timedelta(seconds=60))
assert dist.get_backend() == "nccl"
tab = T.compile_scenario(T.baseline_scenario(2))
N, K, seed = 65536, 20, 11
env = VecRMEnv(tab, N)
env.reset(seed=5)
orc = O.OracleEnv(tab, N)
orc.reset(seed=5)
acts = env.fill_actions(seed, 0, K)
rep = torch.zeros(4, dtype=torch.float64, device="cuda")
for w in range(6):
    env.fill_actions(seed, w * K, K, out=acts)
    env.step_seq(acts, out=rep)
    mine = rep.clone()
    dist.all_reduce(rep, op=dist.ReduceOp.SUM)  # rmx/dist.py's collective, on RCCL
    torch.cuda.synchronize()
    assert torch.equal(rep, mine), (w, rep, mine)
    info = env.queue_info()
    assert info["dispatch"] == "queue" and info["state"] == "ready", info
    for s in range(w * K, (w + 1) * K):
        orc.step(O.hash_actions(seed, s, 1, N, 0, N, tab.n_agents)[0])
env.check_errors()
for k in ("pos_x", "pos_y", "rm_q", "t"):
    np.testing.assert_array_equal(getattr(env, k).cpu().numpy(), getattr(orc, k), err_msg=k)
np.testing.assert_array_equal(env.flags.cpu().numpy().view(np.uint32), orc.flags)
r = rep.cpu().numpy()
assert r[1] == orc.stats[1] and r[2] == orc.stats[2] and r[3] == orc.stats[3] and r[1] > 0, (r, orc.stats)
np.testing.assert_allclose(r[0], orc.stats[0], rtol=1e-9)
dist.barrier()
dist.destroy_process_group()
print("ok rccl", torch.cuda.nccl.version(), env.queue_counters())
"""


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_single_rank_with_the_engine_queue():
    code = _CHILD % (os.path.join(ROOT, "multiagent-rl-rm_amd"), os.path.join(ROOT, "oracle"))
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), RANK="0", WORLD_SIZE="1",
               LOCAL_RANK="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "ok rccl" in r.stdout, r.stdout[-2000:]
