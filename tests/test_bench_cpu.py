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


LINE_KEYS = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
             "vs_baseline", "dtype", "config", "roofline", "cpu_baseline", "parity", "configs", "collective", "detail")


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_gpus_flag_launches_that_many_ranks(n, tmp_path):
    detail_path = str(tmp_path / "detail.json")
    r = _run(["--gpus", str(n), "--dry-run", "--n-envs", "1000", "--detail", detail_path])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # rank 0's JSON line and nothing else
    # the line the driver parses: whole inside its 8 KB stdout tail at every world size, the contract keys present
    assert len(lines[0].encode()) <= 8000, len(lines[0].encode())
    out = json.loads(lines[0])
    assert all(k in out for k in LINE_KEYS), [k for k in LINE_KEYS if k not in out]
    assert out["n_gpus"] == n and out["dry_run"] and out["value"] is None
    for k in ("frac", "achieved", "peak", "unit", "bound", "bytes_per_launch", "avg_launch_us"):
        assert k in out["roofline"], k
    for k in ("value", "cores", "kind", "host"):
        assert k in out["cpu_baseline"], k
    # one summary per other config and random-start leg: value, time per step, roofline fraction, parity rate
    assert set(out["configs"]) == {"1", "3", "4", "5", "rs2", "rs4"}
    for k, c in out["configs"].items():
        assert "value" in c and "parity" in c
        if k != "1":
            assert "ms_per_step" in c and "frac" in c
    # contiguous weak-scaling shards of --n-envs each, and the statistics summed over every rank
    assert out["shards"] == [[r_ * 1000, 1000] for r_ in range(n)]
    assert out["stats_allreduced"] == [float(n), n * (n + 1) / 2, 0.0, 1000.0 * n]
    if n > 1:  # the aligned window start: rank 0 left its spin at (or just after) the agreed instant
        assert 0.0 <= out["aligned_start_late_s"] < 0.05
    # what the job ran on, in the line: backend, world, distinct devices, every rank on its queue
    c = out["collective"]
    assert c["backend"] == ("gloo" if n > 1 else "none") and c["world"] == n and c["distinct_devices"] == n
    assert c["every_rank_on_queue"] is False  # dry run: no queue
    # the per-rank rows are in the detail file the line names: local rank, (fake) device, shard, dispatch per config
    assert out["detail"] == detail_path
    with open(detail_path) as f:
        d = json.load(f)["collective"]
    assert [r["rank"] for r in d["ranks"]] == list(range(n)) and [r["local_rank"] for r in d["ranks"]] == list(range(n))
    assert [[r["env_offset"], r["n_envs"]] for r in d["ranks"]] == out["shards"]
    assert len({r["device_pci"] for r in d["ranks"]}) == n
    for r in d["ranks"]:
        assert set(r["dispatch"]) == {"2", "3", "4", "5", "rs2", "rs4"}
        x = r["dispatch"]["2"]
        assert x["dispatch"] == "dry-run" and x["queue_state"] == "unused"
        assert set(x["queue_counters"]) == {"windows", "uploads", "packets", "stream_windows", "recordings"}


def test_compact_line_of_a_full_detail_stays_small():
    """compact_line over a detail record of the largest shape a GPU run produces (8 ranks, every config, both
    random-start legs, the bandwidth regime, floors, traffic sources): under the driver's 8 KB limit."""
    sys.path.insert(0, ROOT)
    import bench
    args = bench.parse_args(["--steps", "20", "--warmup", "5"])
    world, n = 8, 65536
    head = bench._dry_result(2, n, 2, world, 7e-5, 4e-6, 20)
    head["roofline"]["traffic_source"] = {"summary": "profiles/r06_cfg2_pmc_passes.md and a long name beside it",
                                          "commit": "0123456789ab", "src": "0123456789abcdef",
                                          "kern": "0123456789abcdef", "same_build": True, "same_kernels": True}
    others = {str(c): dict(bench._dry_result(c, n, A, world, 7e-5, 4e-6, 20), parity={"rate": 1.0})
              for c, A in ((3, 1), (4, 4), (5, 3))}
    others["1"] = {"config": 1, "value": 1.0e6, "us_per_env_step": 1.2, "vs_reference_loop_scaled": 4.0,
                   "engine": "host", "reference_loop": {"value": 94868.8}, "gpu_sync": {"value": 3.2e5},
                   "parity": {"rate": 1.0}}
    rs = {c: bench._dry_result(int(c), n, A, world, 7e-5, 4e-6, 20) for c, A in (("2", 2), ("4", 4))}
    ident = {"pci": "0000:75:00", "uuid": "37643637-3537-3636-3435-356438393664", "name": "AMD Instinct MI355X"}
    coll = {"backend": "nccl", "rccl_version": "2.26.6", "world": world, "distinct_devices": world,
            "every_rank_on_queue": True,
            "ranks": [{"rank": r, "local_rank": r, "env_offset": r * n, "n_envs": n, "device_pci": ident["pci"],
                       "device_uuid": ident["uuid"], "device_name": ident["name"], "device_index": r,
                       "dispatch": {k: {"dispatch": "queue", "queue_counters": {"windows": 6, "uploads": 0,
                                                                                "packets": 120, "stream_windows": 0,
                                                                                "recordings": 0},
                                        "queue_state": "ready"} for k in ("2", "3", "4", "5", "rs2", "rs4")}}
                      for r in range(world)]}
    cpu = {"value": 7.4e8, "unit": "(env x agent)-steps/s", "cores": 16, "kind": "port",
           "host": {"model": "AMD EPYC 9575F 64-Core Processor"}, "sample": "x" * 200, "single_thread": {"value": 5e7}}
    large = {"n_envs": 1 << 23, "frac": 0.91, "frac_counter": 0.79, "avg_launch_us": 120.5}
    detail = bench.assemble_detail(args, world, 2, head, others, rs, coll, cpu, {"rate": 1.0, "exact": 1, "instance_steps": 1},
                                   {"value": 1e11}, large, None)
    assert len(json.dumps(detail)) > 8000  # the detail itself would not fit
    line = json.dumps(bench.compact_line(detail, "gpurun_out/bench_detail_n8.json"))
    assert len(line.encode()) <= 4000, len(line.encode())
    back = json.loads(line)
    assert all(k in back for k in LINE_KEYS)
    assert back["configs"]["1"]["vs_reference_loop_scaled"] == 4.0 and back["collective"]["every_rank_on_queue"]


@pytest.mark.parametrize("n", [2, 8])
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


class _FakeTimedEngine:
    """queue_timing / queue_times as the engine's queue answers them: packets 0, m, 2m, ... and the last stamped; each
    dispatch `step_ns` apart, a stamped one `extra_ns` longer (its signalled completion)."""

    def __init__(self, K, step_ns=3000, extra_ns=1200, broken=False):
        self.K, self.step_ns, self.extra_ns, self.broken = K, step_ns, extra_ns, broken
        self.every, self.calls, self.t0 = 0, [], 10_000_000

    def queue_timing(self, every):
        self.calls.append(every)
        self.every = every

    def run(self):
        import numpy as np
        m, K = self.every, self.K
        stamped = sorted(set(range(0, K - 1, m)) | {K - 1}) if m else []
        rows, t = [], self.t0
        for i in range(K):
            dur = self.step_ns + (self.extra_ns if i in stamped else 0)
            if i in stamped:
                rows.append((i, t, t + dur))
            t += dur
        self.t0 = t + 50_000
        self.ts = np.array(rows if not self.broken else rows[1:], dtype=np.uint64).reshape(-1, 3)

    def queue_times(self):
        return self.ts


def test_cp_dispatch_times_span_and_fallbacks(monkeypatch):
    """bench.cp_dispatch_times: the span from packet 0's start to the last packet's start / (K - 1), the stamped
    dispatches' own length, timing switched off afterwards; None without a queue window, for K < 3, or when the
    stamps do not start at packet 0."""
    sys.path.insert(0, ROOT)
    import bench

    import torch
    monkeypatch.setattr(torch.cuda, "synchronize", lambda *a, **k: None)
    K = 1000
    eng = _FakeTimedEngine(K)
    seeds = []
    r = bench.cp_dispatch_times(eng, eng.run, K, seeds.append, reps=3, every=50)
    n_st = len(set(range(0, K - 1, 50)) | {K - 1})
    assert r["stamps_per_window"] == n_st == 21 and r["every"] == 50 and r["windows"] == 3
    # (K - 1) dispatches: 3,000 ns each, plus 1,200 for each stamped one among them (all stamped but the last)
    assert abs(r["dispatch_us"] - (3000 * (K - 1) + 1200 * (n_st - 1)) / (K - 1) / 1e3) < 1e-9
    assert abs(r["stamped_dispatch_us"] - 4.2) < 1e-9
    assert eng.calls == [50, 0] and len(seeds) == 3  # timing on, then off; each window prepared
    assert bench.cp_dispatch_times(eng, None, K, seeds.append) is None
    assert bench.cp_dispatch_times(_FakeTimedEngine(2), eng.run, 2, seeds.append) is None
    bad = _FakeTimedEngine(K, broken=True)
    assert bench.cp_dispatch_times(bad, bad.run, K, seeds.append) is None and bad.calls == [50, 0]
