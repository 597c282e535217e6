"""bench.py — (env x agent)-steps/s of the rmx step engine on BASELINE.json's workload.

Default workload (N=1): BASELINE config 2 — FrozenLake map1, 65,536 envs x 2 agents, built-in
A->B->C RM (Q=4 states, "3-state RM"), uniform synthetic actions from the SURVEY §8(d) counter hash,
pre-generated in HBM before the timed region.  One "step" = one RMEnvironmentWrapper.step of every
env = one launch of the gfx950 step kernel (state round-trips HBM, autoreset on episode end).

Multi-GPU (torchrun, one process per GPU): weak scaling with the same per-GPU workload at every N
(65,536 envs x 2 agents of config 2 per rank, so efficiency compares like with like); BASELINE config 4
(65,536 envs x 4 agents per rank, 524,288 envs over 8 GPUs) is measured by the same protocol and
reported beside it as `config4`.  Each rank owns a contiguous env shard with no data-path collective;
the per-rank episode statistics are summed with ONE RCCL all-reduce (4 x f64) inside the timed window.

Prints ONE JSON line (rank 0) with the driver's contract keys plus `roofline`, `cpu_baseline` and
`parity` (the metric's "CPU-ref parity rate": fraction of (env x agent)-steps of a bounded sample of the
same workload that the default kernel computes bit-exactly against the CPU oracle).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))

METRIC = "env×agent steps/sec at 65,536 envs (1/2/4/8 GPU) + CPU-ref parity rate"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
WORKLOADS = {
    2: "FrozenLake map1, 65,536 envs/GPU x 2 agents, built-in A->B->C RM (3-state RM), random actions",
    3: "OfficeWorld map1, 65,536 envs x 1 agent, A->C->B->D RM (4 RM states)",
    4: "FrozenLake map1, 65,536 envs/GPU x 4 agents, 3-state RM (524,288 envs over 8 GPUs)",
    5: "OfficeWorld map1, 65,536 envs x 3 agents, exp5 8-state RM + reward shaping",
}


KERNEL_NAMES = {"fast": "rmx::step_fast_kernel", "fast_lpe": "rmx::step_fast_lpe_kernel",
                "generic": "rmx::step_kernel", "lane_per_agent": "rmx::step_kernel_lpe"}


def algorithmic_bytes_per_instance_step(A, shaping):
    """B = 48 + 9/A (+4 with the shaping column) bytes per (env x agent)-step.
    reads pos_x,pos_y,rm_q,flags 16 + action 4 + ep_ret 4; writes the same 16 + reward 4 + ep_ret 4;
    per env t r/w 8 + env_done 1 (shared by A agents)."""
    return 48.0 + 9.0 / A + (4.0 if shaping else 0.0)


def pmc_traffic(cfg_id, n_envs):
    """HBM bytes per launch of the default step kernel from the committed rocprofv3 PMC passes of the same
    kernel/config/size (profiles/traffic.json, FETCH_SIZE x2 + WRITE_SIZE; that file documents the gfx950
    correction), or None."""
    tfile = os.environ.get("RMX_TRAFFIC_JSON", os.path.join(ROOT, "profiles", "traffic.json"))
    if os.path.exists(tfile):
        with open(tfile) as f:
            for v in json.load(f).values():
                if isinstance(v, dict) and v.get("config") == cfg_id and v.get("n_envs") == n_envs:
                    return v["bytes_per_launch"]
    return None


def copy_floor(n_envs, launch_us):
    """The achievable floor of the step's access pattern at this size (profiles/floors.json, measured by
    scripts/floor_bench with the same graph-chain method): an empty launch and a pure copy of exactly the
    step's I/O (config-2 shape).  frac_of_copy_floor = copy time / this step's launch time."""
    f = os.path.join(ROOT, "profiles", "floors.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        v = json.load(fh).get(str(n_envs))
    if not v:
        return None
    return {"null_us": v["null_us"], "copy_step_io_us": v["copy_step_io_us"],
            "frac_of_copy_floor": v["copy_step_io_us"] / launch_us, "source": v["source"]}


def bandwidth_regime(tab, n_envs, steps, device, cfg_id):
    """The same step kernel at an HBM-resident size (state >> the 256 MiB Infinity Cache), where the launch
    floor no longer dominates: algorithmic bytes per launch / average launch time over `steps` graph-replayed
    steps (HIP events on the launch stream).  Reported beside the headline roofline, not as `value`."""
    import torch

    from rmx.engine import VecRMEnv

    env = VecRMEnv(tab, n_envs, device=device, with_renv=False, with_env_done=True)
    acts = env.fill_actions(7, 0, steps)
    stream = torch.cuda.current_stream()
    for s in range(2):
        env.step(acts[s])
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()
    s0.wait_stream(stream)
    with torch.cuda.stream(s0):
        with torch.cuda.graph(g, stream=s0):
            for s in range(steps):
                env.step(acts[s])
    stream.wait_stream(s0)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    g.replay()
    e1.record(stream)
    torch.cuda.synchronize()
    env.check_errors()
    launch_s = e0.elapsed_time(e1) / 1e3 / steps
    B = algorithmic_bytes_per_instance_step(tab.n_agents, tab.shape is not None)
    achieved = n_envs * tab.n_agents * B / launch_s / 1e9
    out = {"n_envs": n_envs, "kernel": KERNEL_NAMES[env.step_variant], "achieved": achieved, "peak": HBM_PEAK_GBS,
           "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(cfg_id, n_envs),
           "floor": copy_floor(n_envs, launch_s * 1e6) if cfg_id == 2 else None,
           "avg_launch_us": launch_s * 1e6, "value": n_envs * tab.n_agents / launch_s,
           "note": "same kernel at an HBM-resident size (bandwidth regime); secondary"}
    del g, env, acts
    torch.cuda.empty_cache()
    return out


def cpu_baseline(tab, n_envs, seconds, threads):
    """The CPU oracle (scalar C restatement, 'port') on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O

    env = O.OracleEnv(tab, n_envs)
    T0 = 50
    t = time.perf_counter()
    env.rollout(123, 0, T0, n_threads=threads)
    dt = time.perf_counter() - t
    T = max(50, int(T0 * seconds / max(dt, 1e-6)))
    env2 = O.OracleEnv(tab, n_envs)
    t = time.perf_counter()
    env2.rollout(123, 0, T, n_threads=threads)
    dt = time.perf_counter() - t
    return {"value": n_envs * tab.n_agents * T / dt, "unit": "(env x agent)-steps/s", "cores": threads,
            "kind": "port",
            "sample": f"CPU oracle (C restatement, oracle/rmx_oracle.c) {n_envs} envs x {tab.n_agents} agents x "
                      f"{T} autoreset steps, hashed actions, {dt:.1f} s, {threads} thread(s)"}


def parity_sample(tab, n_envs, steps, device, seed=321):
    """CPU-reference parity rate: the default step kernel and the CPU oracle (the checker,
    oracle/rmx_oracle.c) step the same envs with the same hashed actions; an (env x agent)-step counts as
    exact when pos_x, pos_y, rm_q, flags and the env's t match bit for bit and reward + shaping agree
    within 1e-6 in f64.  Bounded sample of the headline workload, run after the timed region."""
    import numpy as np
    import torch

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from rmx.engine import VecRMEnv

    env = VecRMEnv(tab, n_envs, device=device)
    orc = O.OracleEnv(tab, n_envs)
    A = tab.n_agents
    exact = total = 0
    t0 = time.perf_counter()
    for s in range(steps):
        env.step_hashed(seed, s)
        orc.step(O.hash_actions(seed, s, 1, n_envs, 0, n_envs, A)[0])
        torch.cuda.synchronize()
        ok = np.ones((A, n_envs), bool)
        for k in ("pos_x", "pos_y", "rm_q"):
            ok &= getattr(env, k).cpu().numpy() == getattr(orc, k)
        ok &= env.flags.cpu().numpy().view(np.uint32) == orc.flags
        ok &= (env.t.cpu().numpy() == orc.t)[None, :]
        rg = env.reward.cpu().numpy().astype(np.float64)
        rc = orc.reward.astype(np.float64)
        if env.shaping is not None:
            rg = rg + env.shaping.cpu().numpy()
            rc = rc + orc.shaping
        ok &= np.abs(rg - rc) <= 1e-6
        exact += int(ok.sum())
        total += ok.size
    env.check_errors()
    return {"rate": exact / total, "exact": exact, "instance_steps": total,
            "sample": f"{n_envs} envs x {A} agents x {steps} steps, kernel {KERNEL_NAMES[env.step_variant]} vs the "
                      f"CPU oracle, int state bit-exact and |reward+shaping| diff <= 1e-6 (f64), "
                      f"{time.perf_counter() - t0:.1f} s"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", type=int, default=None, help="BASELINE config (2,3,4,5); default 2 (N=1), 4 (N>1)")
    ap.add_argument("--n-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--graph", type=int, default=1, help="capture the timed steps in a HIP graph")
    ap.add_argument("--parity-steps", type=int, default=200, help="steps of the CPU-reference parity sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="threads of the CPU baseline (16 = the GPU box's CPU share); a 1-thread sample is also reported")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-rollout", action="store_true")
    ap.add_argument("--large-envs", type=int, default=1 << 23,
                    help="envs of the bandwidth-regime measurement (0: skip)")
    ap.add_argument("--seed", type=int, default=0)
    args = ap.parse_args()

    import numpy as np
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    from rmx import dist as RD

    # one process per GPU; RCCL process group when world > 1.  RMX_BENCH_BACKEND=gloo is a rehearsal mode
    # for the multi-rank path on fewer GPUs than ranks (ranks then share devices: local % device_count)
    backend = os.environ.get("RMX_BENCH_BACKEND", "nccl")
    rank, world, local = RD.init(backend)
    local = local % max(1, torch.cuda.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist
    torch.cuda.set_device(local)
    def barrier():
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()

    def timed_run(cfg_id):
        """W untimed warmup steps, then EXACTLY K graph-replayed steps bracketed by barrier + sync, the
        statistics all-reduce inside the window; wall clock max over ranks."""
        tab = T.compile_scenario(T.baseline_scenario(cfg_id))
        # weak scaling: a fixed --n-envs shard per GPU, contiguous in the global env index
        offset, N = RD.shard(world * args.n_envs, world, rank)
        env = VecRMEnv(tab, N, device=local, env_offset=offset, n_envs_global=world * args.n_envs,
                       with_renv=False, with_env_done=True)
        K, W = args.steps, args.warmup
        # inputs resident in HBM before timing: warmup + timed actions from the counter hash
        acts = env.fill_actions(args.seed, 0, W + K)
        stream = torch.cuda.current_stream()
        for s in range(W):
            env.step(acts[s])
        graph = None
        if args.graph:
            graph = torch.cuda.CUDAGraph()
            s0 = torch.cuda.Stream()
            s0.wait_stream(stream)
            with torch.cuda.stream(s0):
                with torch.cuda.graph(graph, stream=s0):
                    for s in range(K):
                        env.step(acts[W + s])
            stream.wait_stream(s0)
            # the capture did not execute: restore the post-warmup state by re-running warmup
            env.reset()
            env.clear_stats()
            for s in range(W):
                env.step(acts[s])
        env.clear_stats()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        barrier()
        t0 = time.perf_counter()
        ev0.record(stream)
        if graph is not None:
            graph.replay()
        else:
            for s in range(K):
                env.step(acts[W + s])
        ev1.record(stream)
        st = env.stats_tensor()
        RD.allreduce_stats(st)  # the one collective: RCCL SUM of (return, episodes, successes, length)
        barrier()
        wall = time.perf_counter() - t0
        ev_ms = ev0.elapsed_time(ev1)
        env.check_errors()
        t_max = torch.tensor([wall], dtype=torch.float64, device="cuda")
        if dist is not None:
            dist.all_reduce(t_max, op=dist.ReduceOp.MAX)
        wall_max = float(t_max.item())
        del graph
        return {"tab": tab, "env": env, "N": N, "A": tab.n_agents, "K": K, "W": W, "wall_max": wall_max,
                "ev_ms": ev_ms, "stats": st.cpu().numpy(), "variant": env.step_variant, "stream": stream,
                "value": world * N * tab.n_agents * K / wall_max}

    # the same per-GPU workload at every N (BASELINE config 2 shape: 65,536 envs x 2 agents per GPU), so
    # the driver's scaling efficiency compares like with like; BASELINE config 4 (4 agents) is reported
    # beside it as `config4`
    cfg_id = args.config or 2
    run = timed_run(cfg_id)
    tab, env, N, A, K, W = run["tab"], run["env"], run["N"], run["A"], run["K"], run["W"]
    wall_max, ev_ms, stats, variant, stream, value = (run[k] for k in ("wall_max", "ev_ms", "stats", "variant",
                                                                        "stream", "value"))

    # roofline of the dominant kernel (the step kernel): algorithmic bytes per launch / avg duration
    B = algorithmic_bytes_per_instance_step(A, tab.shape is not None)
    bytes_per_launch = N * A * B
    launch_s = ev_ms / 1e3 / K
    achieved = bytes_per_launch / launch_s / 1e9
    # HBM bytes per launch from the committed rocprofv3 PMC passes of the same kernel/config/size
    # (profiles/traffic.json, FETCH_SIZE x2 + WRITE_SIZE; see that file for the gfx950 correction)
    traffic = pmc_traffic(cfg_id, N)

    rollout = None
    if not args.no_rollout:
        env.reset()
        env.clear_stats()
        env.rollout(args.seed, 0, 10)  # warm
        torch.cuda.synchronize()
        r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        r0.record(stream)
        env.rollout(args.seed, 10, K)
        r1.record(stream)
        torch.cuda.synchronize()
        rs = r0.elapsed_time(r1) / 1e3
        rollout = {"value": N * A * K / rs * world, "unit": "(env x agent)-steps/s",
                   "note": "fused T-step rollout kernel (state in VGPRs, actions hashed in-kernel), secondary"}

    large = None
    if args.large_envs > 0 and world == 1:  # single-GPU characterisation only
        large = bandwidth_regime(tab, args.large_envs, 20, local, cfg_id)

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(tab, 65536, args.cpu_seconds, args.cpu_threads)
        if args.cpu_threads != 1:
            cpu["single_thread"] = cpu_baseline(tab, 8192, args.cpu_seconds / 2, 1)
        parity = parity_sample(tab, N, args.parity_steps, local)

    config4 = None
    if args.config is None:  # BASELINE config 4 (4 agents per env), same protocol, every rank
        r4 = timed_run(4)
        config4 = {"value": r4["value"], "unit": "(env x agent)-steps/s", "ms_per_step": r4["wall_max"] * 1e3 / K,
                   "workload": WORKLOADS[4], "n_envs_total": world * r4["N"], "n_agents": r4["A"],
                   "kernel": KERNEL_NAMES[r4["variant"]], "scaling": "weak"}
        r4["env"].close()

    if rank == 0:
        out = {
            "metric": METRIC, "value": value, "unit": "(env x agent)-steps/s", "n_gpus": world, "steps": K,
            "warmup": W, "ms_per_step": wall_max * 1e3 / K, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32", "data": "synthetic: counter-hash uniform random actions",
            "config": {"workload": WORKLOADS[cfg_id], "baseline_config": cfg_id, "n_envs_per_gpu": N,
                       "n_envs_total": world * N, "n_agents": A, "rm_states": tab.n_rm_states,
                       "parallelism": f"dp{world} (env shards, no data-path collective)",
                       "graph": bool(args.graph)},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_launch": bytes_per_launch, "bytes_per_instance_step": B,
                         "avg_launch_us": launch_s * 1e6,
                         "floor": copy_floor(N, launch_s * 1e6) if cfg_id == 2 else None,
                         "kernel": KERNEL_NAMES[variant]},
            "roofline_large": large,
            "cpu_baseline": cpu,
            "parity": parity,
            "rollout": rollout,
            "config4": config4,
            "episode_stats": {"episodes": float(stats[1]), "mean_return_per_agent_episode":
                              float(stats[0] / max(stats[1] * A, 1)), "successes": float(stats[2]),
                              "mean_length": float(stats[3] / max(stats[1], 1))},
        }
        print(json.dumps(out))
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
