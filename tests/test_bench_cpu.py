"""bench.py's multi-rank launch on CPU: `--gpus N` starts N ranks itself (torch.distributed.run child, gloo
process group in --dry-run) and rank 0 reports n_gpus == N; a launcher whose world size disagrees with
--gpus is refused."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=180):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, capture_output=True, text=True,
                          env=env, cwd=ROOT, timeout=timeout)


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_gpus_flag_launches_that_many_ranks(n):
    r = _run(["--gpus", str(n), "--dry-run", "--n-envs", "1000"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # rank 0's JSON line and nothing else
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["dry_run"]
    # contiguous weak-scaling shards of --n-envs each, and the statistics summed over every rank
    assert out["shards"] == [[r_ * 1000, 1000] for r_ in range(n)]
    assert out["stats_allreduced"] == [float(n), n * (n + 1) / 2, 0.0, 1000.0 * n]
    if n > 1:  # the aligned window start: rank 0 left its spin at (or just after) the agreed instant
        assert 0.0 <= out["aligned_start_late_s"] < 0.05
    # what the job ran on: backend, world, one entry per rank with its local rank, (fake) device and shard
    c = out["collective"]
    assert c["backend"] == ("gloo" if n > 1 else "none") and c["world"] == n and c["distinct_devices"] == n
    assert [r["rank"] for r in c["ranks"]] == list(range(n)) and [r["local_rank"] for r in c["ranks"]] == list(range(n))
    assert [[r["env_offset"], r["n_envs"]] for r in c["ranks"]] == out["shards"]
    assert len({r["device_pci"] for r in c["ranks"]}) == n
    # every rank's per-config dispatch and queue counters, gathered after the windows (dry run: no queue)
    for r in c["ranks"]:
        d = r["dispatch"]["2"]
        assert d["dispatch"] == "dry-run" and d["queue_state"] == "unused"
        assert set(d["queue_counters"]) == {"windows", "uploads", "packets", "stream_windows", "recordings"}
    assert c["every_rank_on_queue"] is False


@pytest.mark.parametrize("n", [2, 3])
def test_ranks_sharing_a_device_are_refused(n):
    """Under the one-GPU-per-rank check (what RCCL runs get) ranks that report the same device make the job exit
    non-zero, naming the shared device, and no result line is printed."""
    r = _run(["--gpus", str(n), "--dry-run", "--n-envs", "1000", "--dry-run-same-device"], timeout=150)
    assert r.returncode != 0
    assert "distinct devices" in r.stderr and "0000:00:00" in r.stderr, r.stderr[-3000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_world_size_must_match_gpus():
    r = _run(["--gpus", "2", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2 and "--gpus 2" in r.stderr


def test_failed_rank_is_reported_without_hanging():
    """A rank that dies mid-window (before the statistics all-reduce) makes the whole job exit non-zero within
    the process-group timeout, with the failed rank named on stderr (SURVEY §8(e) failure handling)."""
    import time
    t0 = time.time()
    r = _run(["--gpus", "2", "--dry-run", "--n-envs", "1000", "--fail-rank", "1"], {"RMX_PG_TIMEOUT_S": "30"},
             timeout=150)
    assert r.returncode != 0
    assert time.time() - t0 < 120
    assert "failed: rank 1 (--fail-rank)" in r.stderr, r.stderr[-3000:]
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]  # no result line for a failed job


def test_reported_windows_default_to_the_engine_queue():
    """The driver's plain `bench.py --steps 20 --warmup 5` times its reported windows through rmx_step_seq (the
    engine's own AQL queue); `--dispatch graph` keeps the rounds-2/3 HIP graph form for A/B runs."""
    sys.path.insert(0, ROOT)
    import bench
    a = bench.parse_args(["--steps", "20", "--warmup", "5"])
    assert a.dispatch == "queue" and a.graph == 1
    assert bench.parse_args(["--dispatch", "graph"]).dispatch == "graph"
    with pytest.raises(SystemExit):
        bench.parse_args(["--dispatch", "eager"])
