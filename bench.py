"""bench.py — (env x agent)-steps/s of the rmx step engine on BASELINE.json's workload.

Default workload (N=1): BASELINE config 2 — FrozenLake map1, 65,536 envs x 2 agents, built-in A->B->C RM
(Q=4 states, "3-state RM"), uniform synthetic actions from the SURVEY §8(d) counter hash, pre-generated in
HBM before the timed region.  One "step" = one RMEnvironmentWrapper.step of every env = one launch of the
gfx950 step kernel (state round-trips HBM, autoreset on episode end).

Protocol: per BASELINE config, the K timed steps are one rmx_step_seq call (--dispatch queue, the
default: K kernel-dispatch packets on the engine's own AQL queue, rmx_queue.cpp, returning once they are done) or a
HIP graph of the K launches (--dispatch graph, and for handles whose step is not the thread-per-env fast kernel),
run back to back for --spin-ms (2 s, so the GPU clocks are up before timing; a graph's first replay, which pays a
one-time upload, among them); then for each of 5 windows (action seeds 0, 1, 2, 0, 1): reset, W eager warmup
steps, barrier + sync (at N > 1 every rank then starts at one agreed instant of the node clock), the K steps whose
last one also produces the episode-statistics report (rmx_step_report: inside that step's launch for the default
kernel), device sync; wall clock from the agreed start, max over ranks.  Then, outside the timed steps, the job-wide statistics all-reduce (one RCCL collective of 32 B at
N > 1), timed on its own: `allreduce_us`, and `value_with_allreduce` if every K-step window paid it.  `value` is the
median window's all-rank (env x agent)-steps / wall second.  5 more windows of the same protocol carry HIP events
around a HIP graph of K plain steps (the same kernel, on the stream the events are recorded on) and give the
per-step kernel time that feeds the roofline; they are kept out of `value` because recording the events adds host
time to a short window.

Multi-GPU: `python bench.py --gpus N` starts N fresh ranks itself (torch.distributed.run, before this
process touches the GPU) and exits with their status; under an external launcher WORLD_SIZE must equal
--gpus.  Weak scaling with the same per-GPU workload at every N; every rank owns a contiguous env shard
with no data-path collective; the statistics are summed by ONE all-reduce (4 x f64) per window.
RMX_BENCH_BACKEND=gloo rehearses the multi-rank path on fewer GPUs than ranks (ranks share devices).

Prints ONE JSON line (rank 0) with the driver's contract keys plus `roofline`, `cpu_baseline`, `parity` (the
metric's CPU-ref parity rate) and `configs` (every BASELINE GPU config by the same protocol).
"""
import argparse
import gc
import json
import os
import platform
import socket
import statistics
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))

METRIC = "env×agent steps/sec at 65,536 envs (1/2/4/8 GPU) + CPU-ref parity rate"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
WORKLOADS = {
    2: "FrozenLake map1, 65,536 envs/GPU x 2 agents, built-in A->B->C RM (3-state RM), random actions",
    3: "OfficeWorld map1, 65,536 envs/GPU x 1 agent, A->C->B->D RM (4 RM states), random actions",
    4: "FrozenLake map1, 65,536 envs/GPU x 4 agents, 3-state RM (524,288 envs over 8 GPUs), random actions",
    5: "OfficeWorld map1, 65,536 envs/GPU x 3 agents, exp5 8-state RM + reward shaping, random actions",
}
WINDOW_SEEDS = (0, 1, 2, 0, 1)
BUILD = {}  # rmx_build_info() of the library this run loaded (run_rank)

KERNEL_NAMES = {"fast": "rmx::step_fast_kernel", "fast_lpe": "rmx::step_fast_lpe_kernel",
                "generic": "rmx::step_kernel", "lane_per_agent": "rmx::step_kernel_lpe"}


def algorithmic_bytes_per_instance_step(A, shaping):
    """B = 48 + 9/A (+4 with the shaping column) bytes per (env x agent)-step.
    reads pos_x,pos_y,rm_q,flags 16 + action 4 + ep_ret 4; writes the same 16 + reward 4 + ep_ret 4;
    per env t r/w 8 + env_done 1 (shared by A agents)."""
    return 48.0 + 9.0 / A + (4.0 if shaping else 0.0)


def pmc_entry(cfg_id, n_envs, variant=""):
    """The committed rocprofv3 PMC measurement of the default step kernel at this config / size
    (profiles/traffic.json: FETCH_SIZE x2 + WRITE_SIZE per launch, separate --pmc passes; the file documents the
    gfx950 correction, and each entry the summary and commit it was measured at), or None.  PMC passes cannot
    run inside the timed bench, so `traffic` is this measurement, with its source beside it."""
    tfile = os.environ.get("RMX_TRAFFIC_JSON", os.path.join(ROOT, "profiles", "traffic.json"))
    if os.path.exists(tfile):
        with open(tfile) as f:
            t = json.load(f)
        for key in ((f"config{cfg_id}_{variant}",) if variant else (f"config{cfg_id}", "hbm_diag")):
            v = t.get(key)
            if isinstance(v, dict) and v.get("config") == cfg_id and v.get("n_envs") == n_envs:
                return v
    return None


def pmc_traffic(cfg_id, n_envs, variant=""):
    v = pmc_entry(cfg_id, n_envs, variant)
    return v["bytes_per_launch"] if v else None


def profile_time(cfg_id, n_envs, bytes_per_launch, kern=None):
    """The committed counter pass's per-dispatch time of this config's default step kernel at this size
    (profiles/profile_times.json, scripts/profile_times.py): `avg_launch_us_sq` = SQ_BUSY_CYCLES per dispatch /
    the 32 shader engines / the in-kernel shader clock (the time the kernel's waves occupy the chip, without the
    dispatch set-up and end-of-pipe that the event time per step includes), `frac_sq` the algorithmic bytes over
    it, `trace_launch_us` the same dispatch's traced duration (serialized by the profiler: an idle-GPU dispatch, an
    upper bound).  None when no entry matches.  (The roofline's `avg_launch_us_profile` is this run's own dispatch
    stamps: cp_dispatch_times.)"""
    f = os.path.join(ROOT, "profiles", "profile_times.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        v = json.load(fh).get(f"config{cfg_id}")
    if not v or v.get("n_envs") != n_envs:
        return None
    return {"avg_launch_us_sq": v["sq_busy_us"], "frac_sq": bytes_per_launch / (v["sq_busy_us"] * 1e-6) / 1e9 /
            HBM_PEAK_GBS, "trace_launch_us": v["trace_us_median"], "sq_source": v.get("source"),
            "sq_same_kernels": (v.get("kern") == kern) if kern and v.get("kern") else None}


def cp_dispatch_times(env, run, K, prep, reps=3, every=50):
    """This run's per-dispatch time of the step kernel on the command processor's own clock: `reps` more reported
    windows (`run`: the bench's rmx_step_seq window, each after `prep(seed)`: the timed windows' own refill of the
    action buffer, reset and warmup) with the queue's dispatch timing on (rmx_queue_timing), after the timed windows
    and outside the timed region.  Packets 0, every, 2*every, ... and the last are stamped (start, end);
    a stamped packet costs ~1.2 us more than an unstamped one, so the sparse stride keeps the bench's cadence.  The
    dispatch time at cadence = (start of the last packet - start of packet 0) / (K - 1): the window's back-to-back
    dispatches on the CP clock, the last one (the fused report) excluded; median over the windows.  Also the stamped
    dispatches' own end - start and the windows' wall per step with timing on.  None without a queue window or K < 3."""
    import numpy as np
    import torch

    if run is None or K < 3:
        return None
    spans, stamped, walls, n_st = [], [], [], 0
    env.queue_timing(every)
    try:
        for i in range(reps):
            prep(WINDOW_SEEDS[i % len(WINDOW_SEEDS)])
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run()
            torch.cuda.synchronize()
            walls.append((time.perf_counter() - t0) / K)
            ts = env.queue_times().astype(np.int64)
            if len(ts) < 2 or ts[0, 0] != 0 or ts[-1, 0] != K - 1:
                return None
            spans.append((ts[-1, 1] - ts[0, 1]) / (K - 1))
            stamped.extend((ts[:-1, 2] - ts[:-1, 1]).tolist())
            n_st = len(ts)
    finally:
        env.queue_timing(0)
    return {"dispatch_us": statistics.median(spans) / 1e3, "stamped_dispatch_us": statistics.median(stamped) / 1e3,
            "wall_us_per_step_timed": statistics.median(walls) * 1e6, "stamps_per_window": n_st, "every": every,
            "windows": reps,
            "source": "command-processor dispatch stamps (rmx_queue_timing / hsa_amd_profiling_get_dispatch_time) of "
                      "this run's K-step queue windows: the span from packet 0's start to the last packet's start / "
                      "(K - 1)"}


def frac_counter(traffic_bytes, launch_s):
    """The counter-measured bandwidth fraction: PMC traffic per launch (FETCH_SIZE x2 + WRITE_SIZE, the HBM/fabric
    bytes the kernel really moved) / the kernel's time per launch / the 8 TB/s peak.  Beside `frac` (algorithmic
    bytes, which count the rm_q / ep_ret stores the kernel skips when unchanged): `frac` is the §8(d) figure, this one
    says how close the bytes actually moved come to the peak (profiles/README.md)."""
    if not traffic_bytes or not launch_s:
        return None
    return traffic_bytes / launch_s / 1e9 / HBM_PEAK_GBS


def pmc_source(cfg_id, n_envs, variant="", src=None, kern=None):
    """Where `traffic` comes from: the summary, the commit it was measured at and the digests of the library that ran
    (rmx_build_info); `same_build` says whether its source digest is the one of the library timed here,
    `same_kernels` whether its kernels' code-object digest is (host-side changes leave that one unchanged)."""
    v = pmc_entry(cfg_id, n_envs, variant)
    if not v:
        return None
    return {"summary": v.get("source"), "commit": v.get("commit"), "src": v.get("src"), "kern": v.get("kern"),
            "same_build": (v.get("src") == src) if src and v.get("src") else None,
            "same_kernels": (v.get("kern") == kern) if kern and v.get("kern") else None}


def copy_floor(n_envs, launch_us, cfg_id=2, chain_us=None):
    """The achievable floor of the step's access pattern at this size (profiles/floors.json, measured by
    scripts/floor_bench): an empty launch and a pure copy of exactly the default step kernel's I/O for this
    config's shape, each timed as a graph-replayed chain of 500 dependent launches on one fixed action buffer.
    frac_of_copy_floor = copy time / the step's per-launch time in the SAME form (chain_launch_s: 500 graph-replayed
    steps); frac_of_copy_floor_window = copy time / the K-step event window's per-step time, which also carries the
    graph launch's own latency spread over K steps (≈0.2 us per step at K = 20)."""
    f = os.path.join(ROOT, "profiles", "floors.json")
    if not os.path.exists(f):
        return None
    with open(f) as fh:
        v = json.load(fh).get(str(n_envs))
    if not v:
        return None
    copy = v.get("copy_cfg", {}).get(str(cfg_id), v["copy_step_io_us"] if cfg_id == 2 else None)
    if copy is None:
        return None
    out = {"null_us": v["null_us"], "copy_step_io_us": copy, "source": v["source"]}
    gather = v.get("gather_cfg", {}).get(str(cfg_id))
    if gather:  # the copy + the one dependent record lookup the step cannot avoid
        out["copy_gather_us"] = gather
    if chain_us:
        out.update(frac_of_copy_floor=copy / chain_us, chain_launch_us=chain_us)
        if gather:
            out["frac_of_gather_floor"] = gather / chain_us
    out["frac_of_copy_floor_window"] = copy / launch_us
    if not chain_us:
        out["frac_of_copy_floor"] = copy / launch_us
    return out


def chain_launch_s(env, act, stream, n=500, reps=5):
    """Per-launch time of the default step kernel in the floors' own form: a graph of n dependent steps on one
    fixed action slice, replayed once untimed, then `reps` times between HIP events on the launch stream; the
    fastest replay (floor_bench takes the same).  Runs after the timed windows, outside the timed region."""
    import torch

    s0 = torch.cuda.Stream()
    s0.wait_stream(stream)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s0):
        with torch.cuda.graph(g, stream=s0):
            for _ in range(n):
                env.step(act)
    stream.wait_stream(s0)
    g.replay()
    best = None
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        g.replay()
        e1.record(stream)
        torch.cuda.synchronize()
        t = e0.elapsed_time(e1) / 1e3 / n
        best = t if best is None else min(best, t)
    del g
    return best


def pin_host_thread(torch, dev):
    """Restrict the launching (main) thread to the CPUs of its GPU's NUMA node (sysfs local_cpulist of the GPU's
    PCI function); returns the CPU list or None when sysfs does not tell."""
    pr = torch.cuda.get_device_properties(dev)
    path = f"/sys/bus/pci/devices/{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}.0/local_cpulist"
    try:
        spec = open(path).read().strip()
    except OSError:
        return None
    cpus = set()
    for part in spec.split(","):
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    cpus &= os.sched_getaffinity(0)
    if not cpus:
        return None
    os.sched_setaffinity(0, cpus)
    return spec


def host_cpu():
    """What the CPU baseline ran on: logical CPUs of the machine, the CPUs this process may use, the box's
    thread budget (OMP_NUM_THREADS) and the lscpu model name."""
    model = platform.processor() or ""
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for ln in out.splitlines():
            if ln.startswith("Model name:"):
                model = ln.split(":", 1)[1].strip()
    except Exception:
        pass
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count()
    omp = os.environ.get("OMP_NUM_THREADS")
    return {"cpu_count": os.cpu_count(), "affinity_cpus": affinity, "omp_num_threads": int(omp) if omp else None,
            "model": model}


def baseline_threads(info):
    """Every host core this process may use, capped by the box's declared thread budget (OMP_NUM_THREADS: the
    GPU box shares its host between GPUs and sets 16 per GPU)."""
    n = info["affinity_cpus"] or 1
    if info["omp_num_threads"]:
        n = min(n, info["omp_num_threads"])
    return max(1, n)


def cpu_baseline(tab, n_envs, seconds, threads, info):
    """The CPU oracle (scalar C restatement, 'port', OpenMP over envs) on a bounded sample of the same
    workload."""
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
            "kind": "port", "host": info,
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


def python_speed_probe(n=100_000, reps=5):
    """us per iteration of a FIXED pure-Python workload shaped like the reference's per-step Python (per-agent dict
    copies and rebuilds, attribute access, small-int arithmetic, dict comprehensions; ma_frozen_lake.py:96-154).
    Timed here and, by tests/golden/time_reference.py, in the build container beside the reference's own loop: the
    ratio scales the container-measured reference loop to this host's CPU (best of `reps`)."""
    class Ag:
        def __init__(self, name):
            self.name = name
            self.state = {"pos_x": 0, "pos_y": 0}

        def get_state(self):
            return self.state

    ags = [Ag("a1"), Ag("a2")]
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        for i in range(n):
            infos = {a.name: {} for a in ags}
            rewards = {a.name: 0 for a in ags}
            for a in ags:
                cur = a.get_state().copy()
                x = (cur["pos_x"] + (i & 1)) % 10
                a.state = {"pos_x": x, "pos_y": cur["pos_y"]}
                infos[a.name]["prev_s"] = cur
                infos[a.name]["s"] = a.state.copy()
                rewards[a.name] += 0.0 if x else 1.0
            terms = {a.name: rewards[a.name] > 0 for a in ags}
            if all(terms.values()):
                infos.clear()
        best = min(best, (time.perf_counter() - t0) / n * 1e6)
    return best


def dict_api_leg(device, seconds, parity_steps=2000):
    """BASELINE config 1 (FrozenLake map1, 1 env, 2 agents, built-in A->B->C RM: the reference's CPU-runnable case,
    "CPU reference path, no GPU") through the drop-in dict API, rmx.compat.RMEnvironmentWrapper, on the engine's host
    path (device="cpu": a host handle, csrc/rmx_hoststep.cpp — no GPU and no PCIe round trip per call): the loop
    tests/golden/time_reference.py times for the reference (pre-generated uniform actions, reset(0) when every agent
    terminated or truncated, ActionRL objects in, the five dicts out), ~`seconds` of it.  Beside it: the same loop on
    the GPU (the resident workgroup behind rmx_step_sync, `gpu_sync`, with the one-launch-per-call form), the reference's
    own loop measured in the build container (profiles/reference_cpu_container.json; the reference cannot travel to
    the GPU box) scaled to this host by a fixed Python probe, and a parity sample of the host path against the CPU
    oracle on the same actions."""
    import ctypes as C

    import numpy as np

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    from rmx import compat as CP
    from rmx import tables as T

    desc = T.baseline_scenario(1)
    A = len(desc["agents"])
    pre = np.random.default_rng(0).integers(0, 4, size=(400_000, A)).tolist()
    acts = [CP.ActionRL(n) for n in ("up", "down", "left", "right")]

    def loop(w, names, secs):
        steps = t = 0
        need = True
        t0 = time.perf_counter()
        while True:
            if need:
                w.reset(0)
                need = False
            row = pre[t % len(pre)]
            _, _, terms, truncs, _ = w.step({names[i]: acts[row[i]] for i in range(A)})
            steps += 1
            t += 1
            if all(terms.values()) or all(truncs.values()):
                need = True
            if steps % 2000 == 0 and time.perf_counter() - t0 > secs:
                return steps, time.perf_counter() - t0

    def wrapper(dev):
        env, agents = CP.scenario_objects(desc)
        return CP.RMEnvironmentWrapper(env, agents, device=dev), [ag.name for ag in agents]

    def call_us(w, M=20000):  # the synchronous C call alone (rmx_step_sync, N = 1, autoreset) from a ctypes loop
        t0 = time.perf_counter()
        for _ in range(M):
            w._step_fn(w._h, w._act_p, 1, w._bufs_p, None)
        return (time.perf_counter() - t0) / M * 1e6

    def timed(dev, secs):
        w, names = wrapper(dev)
        loop(w, names, 0.3)  # warm: first call, first table compile
        steps, dt = loop(w, names, secs)
        return w, names, steps, dt, call_us(w)

    w, names, steps, dt, host_call = timed("cpu", seconds)
    assert w._engine.step_variant == "host"
    # parity sample: the host path's dict API vs the CPU oracle (1 env, autoreset = the loop's reset(0)) on the same
    # actions
    orc = O.OracleEnv(T.compile_scenario(desc), 1)
    orc.reset(seed=0)
    w.reset(0)
    exact = 0
    for s in range(parity_steps):
        row = pre[s]
        obs, rew, terms, truncs, infos = w.step({names[i]: acts[row[i]] for i in range(A)})
        orc.step(np.array(row, np.int32).reshape(A, 1))
        for i, n in enumerate(names):
            exact += int(obs[n]["pos_x"] == orc.pos_x[i, 0] and obs[n]["pos_y"] == orc.pos_y[i, 0]
                         and w.tables.rms[i].get_state_index(infos[n]["q"]) == orc.rm_q[i, 0]
                         and abs(rew[n] - float(orc.reward[i, 0])) <= 1e-6
                         and terms[n] == bool(orc.flags[i, 0] & 0x4) and truncs[n] == bool(orc.flags[i, 0] & 0x8))
        if all(terms.values()) or all(truncs.values()):
            w.reset(0)  # the oracle autoresets the env at its next step: the same start state
    w._engine.close()
    gpu = None
    if device != "cpu":  # the same loop through the GPU (the resident workgroup), then one launch per call
        wg, _, gsteps, gdt, gcall = timed(device, seconds / 2)
        wg._engine.close()
        os.environ["RMX_SYNC"] = "launch"
        try:
            w2, names2 = wrapper(device)
            loop(w2, names2, 0.2)
            steps2, dt2 = loop(w2, names2, seconds / 4)
            w2._engine.close()
        finally:
            del os.environ["RMX_SYNC"]
        gpu = {"value": gsteps * A / gdt, "us_per_env_step": gdt / gsteps * 1e6, "us_per_sync_call": gcall,
               "value_launch_per_call": steps2 * A / dt2, "us_per_env_step_launch_per_call": dt2 / steps2 * 1e6,
               "engine": "gfx950 resident workgroup (rmx_step_sync)"}
    ref = None
    rfile = os.path.join(ROOT, "profiles", "reference_cpu_container.json")
    probe_here = python_speed_probe()
    if os.path.exists(rfile):
        with open(rfile) as f:
            rj = json.load(f)
        r = next((x for x in rj["runs"] if x["config"] == "fl2"), None)
        if r:
            ref = {"value": r["value"], "unit": r["unit"], "cores": r["cores"], "kind": "reference",
                   "where": "build container (no GPU): the reference's own RMEnvironmentWrapper loop, "
                            "tests/golden/time_reference.py; the reference cannot run on the GPU box",
                   "source": "profiles/reference_cpu_container.json"}
            probe_there = rj.get("python_probe_us")
            if probe_there:  # the same fixed Python workload in both places scales the reference to this CPU
                ref["python_probe_us_container"] = probe_there
                ref["python_probe_us_here"] = probe_here
                ref["value_scaled_to_this_host"] = r["value"] * probe_there / probe_here
            h2h = rj.get("head_to_head")
            if h2h:  # the same loop through this host path and the reference's, alternating on the container's core
                ref["head_to_head_container_ratio"] = h2h["median_ratio"]
    value = steps * A / dt
    return {"config": 1, "workload": "FrozenLake map1, 1 env x 2 agents, built-in A->B->C RM, uniform random actions, "
                                     "through the dict API rmx.compat.RMEnvironmentWrapper on the engine's host path "
                                     "(device=\"cpu\", no GPU)",
            "engine": "host", "n_envs_per_gpu": 1, "n_agents": A, "value": value, "unit": "(env x agent)-steps/s",
            "us_per_env_step": dt / steps * 1e6, "env_steps": steps, "seconds": dt,
            "us_per_sync_call": host_call, "us_python_dicts": dt / steps * 1e6 - host_call,
            "gpu_sync": gpu,
            "reference_loop": ref, "vs_reference_loop": value / ref["value"] if ref else None,
            "vs_reference_loop_scaled": value / ref["value_scaled_to_this_host"]
            if ref and ref.get("value_scaled_to_this_host") else None,
            "parity": {"rate": exact / (parity_steps * A), "exact": exact, "instance_steps": parity_steps * A,
                       "sample": f"1 env x {A} agents x {parity_steps} dict-API steps on the host path vs the CPU "
                                 "oracle: positions, RM state, terminations, truncations exact, reward within 1e-6"}}


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
    g.replay()  # the first replay uploads the graph
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
           "frac_counter": frac_counter(pmc_traffic(cfg_id, n_envs), launch_s),
           "traffic_source": pmc_source(cfg_id, n_envs, "", BUILD.get("src"), BUILD.get("kern")),
           "floor": copy_floor(n_envs, launch_s * 1e6) if cfg_id == 2 else None,
           "avg_launch_us": launch_s * 1e6, "value": n_envs * tab.n_agents / launch_s,
           "note": "same kernel at an HBM-resident size (bandwidth regime); secondary"}
    del g, env, acts
    torch.cuda.empty_cache()
    return out


HIP_DEVICE_SCHEDULE_SPIN = 1  # hip_runtime_api.h hipDeviceScheduleSpin


def set_device_flags(device, flags):
    """hipSetDeviceFlags on the HIP runtime torch loaded, before the device's context exists: the host thread
    spin-waits in synchronise instead of HIP's default (which may yield / sleep between polls)."""
    import ctypes

    import torch
    torch.zeros(1)  # loads torch's HIP runtime without initialising a device
    path = next(ln.split()[-1] for ln in open("/proc/self/maps") if "libamdhip64" in ln)
    hip = ctypes.CDLL(path)
    if hip.hipSetDevice(ctypes.c_int(device)) != 0 or hip.hipSetDeviceFlags(ctypes.c_uint(flags)) != 0:
        raise RuntimeError("hipSetDeviceFlags failed (the device was initialised already?)")


START_MARGIN_S = 5e-4  # aligned window start: the latest rank's "now" + this (covers one small collective)


def aligned_start(device, margin_s=START_MARGIN_S):
    """Start line of a timed window at N > 1, after the barrier: every rank spins until the same instant of the
    node's monotonic clock (time.perf_counter is CLOCK_MONOTONIC, shared by the node's processes): the latest
    rank's clock + margin, agreed by one MAX all-reduce on the collective device (rmx.dist.collective_device: the
    rank's GPU under RCCL, the host under gloo — the same call either way).  Host wake-up skew after the barrier
    then stays out of the max-over-ranks window; a rank that arrives after the instant starts at once, and the
    others' closing collective waits for it, so its lateness is still counted."""
    from rmx import dist as RD

    target = RD.max_over_ranks([time.perf_counter() + margin_s], device)[0]
    while time.perf_counter() < target:
        pass
    return target


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def device_identity(torch, local):
    """What this rank runs on: its GPU's PCI domain / bus / device numbers and UUID (torch's device properties)."""
    pr = torch.cuda.get_device_properties(local)
    return {"pci": f"{pr.pci_domain_id:04x}:{pr.pci_bus_id:02x}:{pr.pci_device_id:02x}", "uuid": str(getattr(pr, "uuid", "")),
            "name": pr.name}


def collective_block(dist, backend, rank, world, local, ident, offset, n, strict, device):
    """Proof of what an N-rank job ran on, for the detail file (rank 0's line keeps backend, world, distinct devices
    and every_rank_on_queue): the backend, the RCCL version, the world size and, per rank (one all_gather on the
    collective device), LOCAL_RANK, the device's PCI address and UUID, and the env shard.  strict (the "nccl" =
    RCCL backend, one GPU per rank): two ranks on one device is an error — every rank raises, so the job exits
    non-zero instead of reporting a scaling number that shares a GPU.  Rehearsals on fewer GPUs than ranks (gloo)
    report the sharing instead."""
    import hashlib

    import torch
    key = f"{ident['pci']}|{ident['uuid']}"
    h = int.from_bytes(hashlib.sha256(key.encode()).digest()[:7], "little")
    row = torch.tensor([rank, local, offset, n, h], dtype=torch.int64)
    dev = device
    rows = [torch.zeros(5, dtype=torch.int64, device=dev) for _ in range(world)]
    if world > 1:
        dist.all_gather(rows, row.to(dev))
    else:
        rows = [row]
    rows = [r.cpu().tolist() for r in rows]
    idents = [None] * world
    if world > 1:
        dist.all_gather_object(idents, ident)
    else:
        idents = [ident]
    try:
        import torch.cuda.nccl as nccl
        ver = ".".join(str(v) for v in nccl.version()) if backend == "nccl" else None
    except Exception:
        ver = None
    ranks = [{"rank": r[0], "local_rank": r[1], "env_offset": r[2], "n_envs": r[3], "device_pci": idents[i]["pci"],
              "device_uuid": idents[i]["uuid"], "device_name": idents[i].get("name"),
              "device_index": idents[i].get("device_index")} for i, r in enumerate(rows)]
    hashes = [r[4] for r in rows]
    distinct = len(set(hashes))
    out = {"backend": backend, "rccl_version": ver, "world": world,
           "distinct_devices": distinct, "ranks": ranks}
    if strict and distinct != world:
        dup = sorted({i["pci"] for i in idents if sum(j["pci"] == i["pci"] and j["uuid"] == i["uuid"] for j in idents) > 1})
        raise RuntimeError(f"{world} ranks on {distinct} distinct devices under the {backend} backend "
                           f"(shared: {', '.join(dup)}): not one GPU per rank")
    return out


def attach_rank_dispatch(dist, world, coll, mine):
    """After the timed windows: every rank's per-config dispatch (how its reported windows ran: "queue", "graph",
    "eager") and its queue counters over those windows, gathered (one all_gather_object) into the collective block's
    per-rank rows, so an N > 1 line shows that every rank's windows went through its own queue."""
    rows = [None] * world
    if world > 1:
        dist.all_gather_object(rows, mine)
    else:
        rows = [mine]
    for r, row in zip(coll["ranks"], rows):
        r["dispatch"] = row
    coll["every_rank_on_queue"] = all(c.get("dispatch") == "queue" and c.get("queue_counters", {}).get("packets", 0) > 0
                                      for row in rows for c in row.values())
    return coll


def launch_ranks(n):
    """Start n fresh ranks of this script (torch.distributed.run, one process per GPU) as a CHILD process —
    this process has not touched the GPU and never re-execs — and return their exit status.  Every rank records
    how it ended (rank_status); when the job fails, the ranks that failed, and those that never finished (killed
    by the launcher after another rank failed, or hung), are named on stderr."""
    import tempfile

    status_dir = tempfile.mkdtemp(prefix="rmx_ranks_")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"),
               RMX_RANK_STATUS_DIR=status_dir)
    # stdout carries only rank 0's JSON line: anything else the ranks or their libraries print there (gloo's
    # connection messages, say) is passed on to stderr, line by line as it arrives
    proc = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, text=True, bufsize=1)
    for line in proc.stdout:
        if line.startswith("{") and '"metric"' in line:
            sys.stdout.write(line)
            sys.stdout.flush()
        else:
            sys.stderr.write(line)
            sys.stderr.flush()
    rc = proc.wait()
    report = rank_report(status_dir, n)
    if rc != 0 or report["failed"] or report["missing"]:
        print(f"bench.py: {n} ranks, torch.distributed.run exit status {rc}; failed: "
              + (", ".join(f"rank {r} ({m})" for r, m in report["failed"]) or "none")
              + "; no status (killed or hung): " + (", ".join(f"rank {r}" for r in report["missing"]) or "none"),
              file=sys.stderr)
        rc = rc or 1
    import shutil
    shutil.rmtree(status_dir, ignore_errors=True)
    return rc


def rank_status(rank, ok, msg=""):
    """Record how this rank ended (launch_ranks reads it after the job)."""
    d = os.environ.get("RMX_RANK_STATUS_DIR")
    if d:
        with open(os.path.join(d, f"rank{rank}.status"), "w") as f:
            f.write(("ok" if ok else "failed") + (f": {msg}" if msg else ""))


def rank_report(status_dir, n):
    failed, missing = [], []
    for r in range(n):
        p = os.path.join(status_dir, f"rank{r}.status")
        if not os.path.exists(p):
            missing.append(r)
            continue
        txt = open(p).read().strip()
        if not txt.startswith("ok"):
            failed.append((r, txt.partition(": ")[2] or txt))
    return {"failed": failed, "missing": missing}


def assemble_detail(args, world, head_cfg, head, others, rs_legs, coll, cpu, parity, rollout, large, pinned):
    """Everything the run measured (per-window arrays, event windows, floors, per-rank dispatch rows): the detail
    file.  The stdout line (compact_line) is a summary of it."""
    N, A = head["n_envs_per_gpu"], head["n_agents"]
    return {
        "metric": METRIC, "value": head["value"], "unit": "(env x agent)-steps/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": head["ms_per_step"], "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "int32", "data": "synthetic: counter-hash uniform random actions",
        "config": {"workload": head["workload"], "baseline_config": head_cfg, "n_envs_per_gpu": N,
                   "n_envs_total": world * N, "n_agents": A, "rm_states": head["rm_states"],
                   "parallelism": f"dp{world} (env shards, no data-path collective)", "graph": bool(args.graph),
                   "dispatch": head["dispatch"], "windows": len(head["windows"]),
                   "window_seeds": [w["seed"] for w in head["windows"]],
                   "value_is": "median window, wall clock from the agreed start to the last rank's synchronised "
                               "K-th step (barrier+sync both sides, max over ranks); the statistics all-reduce "
                               "is timed separately (allreduce_us, value_with_allreduce)",
                   "host_pin": pinned, "host_sync": args.sync},
        "us_per_step_event": head["us_per_step_event"],
        "windows": head["windows"],
        "event_windows": head["event_windows"],
        "allreduce_us": head["allreduce_us"], "value_with_allreduce": head["value_with_allreduce"],
        "roofline": head["roofline"],
        "roofline_large": large,
        "cpu_baseline": cpu,
        "parity": parity,
        "rollout": rollout,
        "configs": others,
        "configs_random_starts": rs_legs,
        "collective": coll,
        "build": dict(BUILD),
        "episode_stats": head["episode_stats"],
    }


def write_detail(detail, path, world):
    """The detail JSON next to the run (default gpurun_out/bench_detail_n<N>.json); returns the path written, or
    None when it cannot be written (the line still carries every contract key)."""
    path = path or os.path.join(ROOT, "gpurun_out", f"bench_detail_n{world}.json")
    try:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        with open(path, "w") as f:
            json.dump(detail, f, indent=1)
    except OSError as e:
        print(f"bench.py: detail file not written ({e})", file=sys.stderr)
        return None
    path = os.path.abspath(path)
    return os.path.relpath(path, ROOT) if path.startswith(ROOT + os.sep) else path


LINE_MAX_BYTES = 8000  # the driver's stdout tail: the final line must fit in it whole


def _g(v, digits=5):
    """A float rounded to `digits` significant digits (the line's numbers); anything else as is."""
    if isinstance(v, float):
        return float(f"{v:.{digits}g}")
    return v


def _pick(d, keys):
    return {k: _g(d.get(k)) for k in keys if d is not None and d.get(k) is not None}


ROOF_KEYS = ("bound", "achieved", "peak", "unit", "frac", "frac_counter", "traffic", "bytes_per_launch",
             "avg_launch_us", "avg_launch_us_profile", "frac_profile", "avg_launch_us_sq", "frac_sq",
             "trace_launch_us", "chain_launch_us")


def _roofline_summary(rf):
    if not rf:
        return None
    out = _pick(rf, ROOF_KEYS)
    ts = rf.get("traffic_source") or {}
    if ts:
        out["traffic_source"] = f"{ts.get('summary')} (same_kernels={ts.get('same_kernels')})"
    fl = rf.get("floor") or {}
    if fl.get("frac_of_gather_floor") is not None:
        out["frac_of_gather_floor"] = _g(fl["frac_of_gather_floor"])
    return out


def config_summary(o):
    """One entry of the line's `configs`: the config's value, ms_per_step, roofline fraction(s) and parity rate (its
    full record is in the detail file)."""
    if o is None:
        return None
    if o.get("config") == 1:  # the dict API: per-call time, the reference loop beside it
        ref = o.get("reference_loop") or {}
        s = _pick(o, ("value", "us_per_env_step", "vs_reference_loop", "vs_reference_loop_scaled", "engine"))
        s["reference_loop"] = _g(ref.get("value"))
        s["head_to_head_container_ratio"] = _g(ref.get("head_to_head_container_ratio"))
        gpu = o.get("gpu_sync") or {}
        if gpu:
            s["gpu_sync"] = _pick(gpu, ("value", "us_per_env_step"))
    else:
        rf = o.get("roofline") or {}
        s = _pick(o, ("value", "ms_per_step", "us_per_step_event", "dispatch"))
        s.update(_pick(rf, ("frac", "frac_counter", "frac_profile", "chain_launch_us")))
        fl = rf.get("floor") or {}
        if fl.get("frac_of_gather_floor") is not None:
            s["frac_of_gather_floor"] = _g(fl["frac_of_gather_floor"])
    s["parity"] = _g((o.get("parity") or {}).get("rate"))
    return s


def compact_line(detail, detail_path):
    """rank 0's stdout line: the driver's contract keys, `roofline`, `cpu_baseline`, `parity`, one summary per other
    config and the collective's identity — at most LINE_MAX_BYTES at any world size (the per-rank rows, window arrays
    and floors stay in the detail file, named in `detail`)."""
    cpu = detail.get("cpu_baseline")
    par = detail.get("parity")
    coll = detail.get("collective") or {}
    line = {k: _g(detail.get(k)) for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                            "higher_is_better", "scaling", "vs_baseline", "dtype", "data")}
    c = detail.get("config") or {}
    line["config"] = {k: c.get(k) for k in ("workload", "baseline_config", "n_envs_per_gpu", "n_envs_total", "n_agents",
                                            "rm_states", "parallelism", "dispatch", "windows")}
    line["us_per_step_event"] = _g(detail.get("us_per_step_event"))
    line["allreduce_us"] = _g(detail.get("allreduce_us"))
    line["value_with_allreduce"] = _g(detail.get("value_with_allreduce"))
    line["roofline"] = _roofline_summary(detail.get("roofline"))
    line["cpu_baseline"] = None if cpu is None else dict(
        _pick(cpu, ("value", "unit", "cores", "kind", "sample")),
        host=(cpu.get("host") or {}).get("model"),
        single_thread=_g((cpu.get("single_thread") or {}).get("value")))
    line["parity"] = None if par is None else _pick(par, ("rate", "exact", "instance_steps"))
    line["configs"] = {k: config_summary(v) for k, v in (detail.get("configs") or {}).items()}
    line["configs"].update({"rs" + k: config_summary(v) for k, v in (detail.get("configs_random_starts") or {}).items()})
    lg = detail.get("roofline_large")
    line["roofline_large"] = None if lg is None else _pick(lg, ("n_envs", "frac", "frac_counter", "avg_launch_us"))
    line["collective"] = {k: coll.get(k) for k in ("backend", "rccl_version", "world", "distinct_devices",
                                                   "every_rank_on_queue")}
    b = detail.get("build") or {}
    line["build"] = {k: b.get(k) for k in ("src", "kern")}
    line["detail"] = detail_path
    s = json.dumps(line)
    if len(s.encode()) > LINE_MAX_BYTES:  # never expected (tests/test_bench_cpu.py): drop the summaries, keep the contract
        for k in ("configs", "roofline_large", "build"):
            line.pop(k, None)
    return line


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--config", type=int, default=None,
                    help="time only this BASELINE config (2,3,4,5); default: config 2 headline + every other config")
    ap.add_argument("--n-envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--graph", type=int, default=1, help="capture the timed steps in a HIP graph")
    ap.add_argument("--dispatch", choices=["queue", "graph"], default="queue",
                    help="the reported windows' K steps: queue = one rmx_step_seq (the engine's own AQL queue, where "
                         "the handle's step is the thread-per-env fast kernel), graph = a HIP graph replay")
    ap.add_argument("--windows", type=int, default=len(WINDOW_SEEDS), help="timed windows per config (median)")
    ap.add_argument("--chain", type=int, default=1, help="also time a 500-step graph chain per config (the floors' form)")
    ap.add_argument("--sync", choices=["auto", "spin"], default="auto",
                    help="host wait of torch.cuda.synchronize: HIP's default or hipDeviceScheduleSpin")
    ap.add_argument("--pin", choices=["none", "numa"], default="none",
                    help="numa: run the launching thread on its GPU's NUMA-node CPUs")
    ap.add_argument("--spin-ms", type=float, default=2000.0, help="untimed back-to-back steps before each config's "
                    "timed windows (clock spin-up), in ms")
    ap.add_argument("--parity-steps", type=int, default=200, help="steps of the CPU-reference parity sample")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the CPU baseline (0: every usable host core, capped by OMP_NUM_THREADS)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-rollout", action="store_true")
    ap.add_argument("--large-envs", type=int, default=1 << 23,
                    help="envs of the bandwidth-regime measurement (0: skip)")
    ap.add_argument("--slip", action="store_true",
                    help="characterisation only: the BASELINE scenarios with their env's slip switch on")
    ap.add_argument("--random-starts", action="store_true",
                    help="characterisation only: the FrozenLake BASELINE scenarios with random_start_positions on")
    ap.add_argument("--rs-configs", default="2,4",
                    help="default run: the FrozenLake configs also timed with random_start_positions on (empty: none)")
    ap.add_argument("--dict-seconds", type=float, default=2.0,
                    help="seconds of the BASELINE config 1 dict-API loop (0: skip)")
    ap.add_argument("--detail", default=None,
                    help="the detail JSON (every window, floor and per-rank row; default gpurun_out/bench_detail_n<N>.json)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher / process-group / reporting path only, no GPU work (CPU tests)")
    ap.add_argument("--dry-run-same-device", action="store_true",
                    help="--dry-run only: every rank reports the same fake device, checked as RCCL would be (CPU tests "
                         "of the one-GPU-per-rank refusal)")
    ap.add_argument("--fail-rank", type=int, default=-1,
                    help="--dry-run only: this rank exits with status 3 in the middle of its window (CPU tests of the "
                         "failure path)")
    return ap.parse_args(argv)


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))

    from rmx import dist as RD

    rank, world, local = RD.env_rank()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)", file=sys.stderr)
        sys.exit(2)
    try:
        if args.dry_run:
            dry_run(args, rank, world)
        else:
            run_rank(args)
    except SystemExit as e:
        rank_status(rank, e.code in (0, None), f"exit status {e.code}")
        raise
    except BaseException as e:
        rank_status(rank, False, f"{type(e).__name__}: {e}"[:300])
        print(f"bench.py rank {rank}: {type(e).__name__}: {e}", file=sys.stderr)
        raise
    rank_status(rank, True)


def run_rank(args):
    """One rank of the timed benchmark (the module docstring's protocol)."""
    import numpy as np  # noqa: F401  (loaded before torch, as before the split)
    import torch

    from rmx import dist as RD

    from rmx import _capi
    from rmx import tables as T
    from rmx.engine import VecRMEnv

    BUILD.update(_capi.build_info(_capi.load_library()))  # the source digest of the library timed here
    # one process per GPU; RCCL process group when world > 1.  RMX_BENCH_BACKEND=gloo is a rehearsal mode
    # for the multi-rank path on fewer GPUs than ranks (ranks then share devices: local % device_count)
    backend = os.environ.get("RMX_BENCH_BACKEND", "nccl")
    rank, world, local = RD.env_rank()
    if args.sync == "spin":
        set_device_flags(local % max(1, torch.cuda.device_count()), HIP_DEVICE_SCHEDULE_SPIN)
    rank, world, local = RD.init(backend)
    local_rank = local  # LOCAL_RANK as launched (the rehearsal maps several onto one device)
    local = local % max(1, torch.cuda.device_count())
    dist = None
    if world > 1:
        import torch.distributed as dist
    torch.cuda.set_device(local)
    pinned = pin_host_thread(torch, local) if args.pin == "numa" else None
    # every collective's tensors live here: this rank's GPU under RCCL, the host under the gloo rehearsal
    coll_dev = RD.collective_device(backend if world > 1 else "none", local)

    def barrier():
        """Opening barrier of a window; returns the window's start instant (at N > 1 the instant every rank agreed
        on, so a rank that starts late is charged its lateness)."""
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
            torch.cuda.synchronize()
            return aligned_start(coll_dev)
        return time.perf_counter()

    K, W = args.steps, args.warmup

    def timed_config(cfg_id, random_starts=False, windows=None):
        """The protocol of the module docstring for one BASELINE config; returns per-window samples."""
        desc = T.baseline_scenario(cfg_id)
        if args.slip:  # characterisation: the env's own slip switch on (frozen_lake_stochastic / stochastic)
            desc = dict(desc, stochastic=True)
        random_starts = random_starts or (args.random_starts and desc["kind"] == "frozen_lake")
        if random_starts:  # FrozenLake random_start_positions (ma_frozen_lake.py:37-39), the runner's seed schedule
            desc = dict(desc, random_start_positions=True)
        variant = "_".join(v for v, on in (("slip", args.slip), ("randstart", random_starts)) if on)
        n_windows = windows or args.windows
        tab = T.compile_scenario(desc)
        # weak scaling: a fixed --n-envs shard per GPU, contiguous in the global env index
        offset, N = RD.shard(world * args.n_envs, world, rank)
        env = VecRMEnv(tab, N, device=local, env_offset=offset, n_envs_global=world * args.n_envs,
                       with_renv=False, with_env_done=True)
        stream = torch.cuda.current_stream()
        # inputs resident in HBM before timing: warmup + timed actions from the counter hash, one buffer
        # refilled per window seed (the graph captures its address)
        acts = env.fill_actions(WINDOW_SEEDS[0], 0, W + K)
        for s in range(W):
            env.step(acts[s])
        # the statistics report of a window: fused into the K-th step's launch (rmx_step_report) where the
        # handle's kernel allows it, else that step then the stats launch; the event windows time K plain steps
        report = torch.zeros(4, dtype=torch.float64, device=f"cuda:{local}")

        def steps(reported):
            for s in range(K - 1 if reported else K):
                env.step(acts[W + s])
            if reported:
                env.step_report(acts[W + K - 1], out=report)

        # the reported windows: one rmx_step_seq (K dispatch packets on the engine's own AQL queue, blocking) where
        # the handle's step allows it, else a HIP graph replay; the event windows always replay a graph of K plain
        # steps on the stream (HIP events time the same kernel there)
        use_queue = args.dispatch == "queue" and env.step_variant == "fast"
        win_acts = acts[W:W + K]  # a view: refilled in place per window seed, same address
        seq, queue_error = None, None
        if use_queue:
            try:  # one untimed window: a queue that cannot start is reported (queue_error), the graph then runs
                seq = env.seq_window(win_acts, out=report)  # checked once, bound
                seq()
            except RuntimeError as e:
                seq, use_queue, queue_error = None, False, str(e)[:300]
                print(f"bench.py: the engine's queue failed, windows through a HIP graph: {e}", file=sys.stderr)
        graph = graph_ev = None
        if args.graph:
            s0 = torch.cuda.Stream()
            s0.wait_stream(stream)
            graph, graph_ev = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.stream(s0):
                if not use_queue:
                    with torch.cuda.graph(graph, stream=s0):
                        steps(True)
                with torch.cuda.graph(graph_ev, stream=s0):
                    steps(False)
            stream.wait_stream(s0)
            if use_queue:
                graph = None
            else:
                graph.replay()  # untimed: the first replay of a graph pays its upload (+1.5 us per step at K=20)
            graph_ev.replay()


        def reported_steps():
            if seq is not None:
                seq()
            elif graph is not None:
                graph.replay()
            else:
                steps(True)

        torch.cuda.synchronize()
        # no collector pause inside a ~70-us window (as timeit does); collected before the spin-up, so the GPU is
        # not left idle (clocking down) between the spin-up and the first window
        gc.collect()
        gc.disable()
        # untimed spin-up: ~--spin-ms of back-to-back steps so the timed windows do not start on an idle-clocked
        # GPU (after an idle gap the first 20-step windows ran at 4.7-5.5 us per step instead of 3.6)
        t_spin = time.perf_counter() + args.spin_ms / 1e3
        while time.perf_counter() < t_spin:
            reported_steps()
            torch.cuda.synchronize()
        RD.allreduce_stats(env.stats_tensor(), coll_dev)  # untimed: the collective's first call sets up its channels
        torch.cuda.synchronize()
        q0 = env.queue_counters()

        def prep(seed):
            """A window's inputs and state: this seed's actions in the one buffer, a reset, the W warmup steps."""
            env.fill_actions(seed, 0, W + K, out=acts)
            env.reset()
            env.clear_stats()
            for s in range(W):
                env.step(acts[s])

        def window(seed, events):
            """One timed window.  The wall-clock windows carry no HIP events: recording them around the graph
            adds ~15 us of host time to a 20-step window (round-2 window probe); the event windows that
            time the steps alone for the roofline are separate."""
            prep(seed)
            if events:
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0 = barrier()
            if events:  # K plain steps between the events, then the report as its own launch
                ev0.record(stream)
                if graph_ev is not None:
                    graph_ev.replay()
                else:
                    steps(False)
                ev1.record(stream)
                st = env.stats_tensor()
            else:  # the K-th step carries the episode-statistics report (rmx_step_report)
                reported_steps()
                st = report
            torch.cuda.synchronize()
            wall = time.perf_counter() - t0  # from the agreed start to this rank's last step (and its report)
            # the job-wide statistic: ONE RCCL all-reduce of the 4 x f64 vector per window, after the K steps are
            # timed and timed on its own (a training loop logs every >= 1,000 steps; at K = 20 a
            # collective inside every window would stand for 50x its share); then the max over ranks
            ta = time.perf_counter()
            RD.allreduce_stats(st, coll_dev)
            torch.cuda.synchronize()
            t_ar = time.perf_counter() - ta
            wall_max, ar_max = RD.max_over_ranks([wall, t_ar], coll_dev)
            return {"seed": seed, "wall_s": wall_max, "allreduce_s": ar_max,
                    "ev_steps_s": ev0.elapsed_time(ev1) / 1e3 if events else None, "stats": st.cpu().numpy()}

        try:
            window(WINDOW_SEEDS[0], False)  # discarded: the first window after the spin-up often ran slow
            samples = [window(WINDOW_SEEDS[w % len(WINDOW_SEEDS)], False) for w in range(n_windows)]
            ev_samples = [window(WINDOW_SEEDS[w % len(WINDOW_SEEDS)], True) for w in range(n_windows)]
        finally:
            gc.enable()
        q1 = env.queue_counters()
        q_state = env.queue_info()["state"]
        chain_s = chain_launch_s(env, acts[W], stream) if args.graph and args.chain > 0 else None
        cp = cp_dispatch_times(env, seq, K, prep) if use_queue else None
        env.check_errors()
        del graph, graph_ev
        walls = [x["wall_s"] for x in samples]
        med = sorted(range(len(walls)), key=lambda i: walls[i])[len(walls) // 2]
        m = samples[med]
        A = tab.n_agents
        # + the env's PCG64 state with slip (32 B read, 16 B written per env-step), + the cached start cells with
        # random starts (4 B per two agents per env; the fixed-start cache)
        B = (algorithmic_bytes_per_instance_step(A, tab.shape is not None) + (48.0 / A if args.slip else 0.0)
             + (4.0 * ((A + 1) // 2) / A if random_starts else 0.0))
        launch_s = statistics.median(x["ev_steps_s"] for x in ev_samples) / K
        achieved = N * A * B / launch_s / 1e9
        st = m["stats"]
        out = {
            "config": cfg_id, "workload": WORKLOADS[cfg_id] + (", slip dynamics" if args.slip else "")
            + (", random start positions (seed schedule (1, 1, 0): reset(seed) every episode)" if random_starts else ""),
            "n_envs_per_gpu": N, "n_envs_total": world * N,
            "n_agents": A, "rm_states": tab.n_rm_states, "kernel": KERNEL_NAMES[env.step_variant],
            "value": world * N * A * K / m["wall_s"], "unit": "(env x agent)-steps/s",
            "ms_per_step": m["wall_s"] * 1e3 / K, "us_per_step_event": launch_s * 1e6,
            # the window's statistics all-reduce (N > 1: one RCCL collective of 32 B), timed on its own, and the
            # throughput if every K-step window also paid it
            "allreduce_us": statistics.median(x["allreduce_s"] for x in samples) * 1e6,
            "value_with_allreduce": world * N * A * K / statistics.median(x["wall_s"] + x["allreduce_s"] for x in samples),
            "report_fused": env.report_fused,  # the window's statistics report ran inside the K-th step launch
            # how the reported windows' K launches were issued; the queue's counters over this config's timed windows
            # (uploads: kernel-argument copies to the device, 0 when every window re-runs the same buffers)
            "dispatch": "queue" if use_queue else ("graph" if args.graph else "eager"), "queue_error": queue_error,
            "queue_counters": {k: q1[k] - q0[k] for k in q0}, "queue_state": q_state,
            "windows": [{"seed": x["seed"], "us_per_step_wall": x["wall_s"] * 1e6 / K, "allreduce_us": x["allreduce_s"] * 1e6}
                        for x in samples],
            "event_windows": [{"seed": x["seed"], "us_per_step_event": x["ev_steps_s"] * 1e6 / K,
                               "us_per_step_wall": x["wall_s"] * 1e6 / K} for x in ev_samples],
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": pmc_traffic(cfg_id, N, variant),
                         "frac_counter": frac_counter(pmc_traffic(cfg_id, N, variant), launch_s),
                         "traffic_source": pmc_source(cfg_id, N, variant, BUILD.get("src"), BUILD.get("kern")),
                         "bytes_per_launch": N * A * B, "bytes_per_instance_step": B,
                         "avg_launch_us": launch_s * 1e6,
                         "chain_launch_us": chain_s * 1e6 if chain_s else None,
                         "floor": None if variant else copy_floor(N, launch_s * 1e6, cfg_id,
                                                                    chain_s * 1e6 if chain_s else None),
                         "kernel": KERNEL_NAMES[env.step_variant]},
            "episode_stats": {"episodes": float(st[1]), "mean_return_per_agent_episode": float(st[0] / max(st[1] * A, 1)),
                              "successes": float(st[2]), "mean_length": float(st[3] / max(st[1], 1))},
        }
        if not variant:  # the committed counter pass's per-dispatch time of this kernel (profiles/profile_times.json)
            out["roofline"].update(profile_time(cfg_id, N, N * A * B, BUILD.get("kern")) or {})
        if cp:  # the profile time of this run: the command processor's stamps of the same windows' dispatches
            out["roofline"].update(avg_launch_us_profile=cp["dispatch_us"],
                                   frac_profile=N * A * B / (cp["dispatch_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS,
                                   profile_source=cp["source"], cp_timing=cp)
        return tab, env, out

    # what the job runs on (one all_gather before any timing; strict under RCCL: one GPU per rank)
    off0, n0 = RD.shard(world * args.n_envs, world, rank)
    ident = dict(device_identity(torch, local), device_index=local)
    coll = collective_block(dist, backend if world > 1 else "none", rank, world, local_rank, ident, off0, n0,
                            strict=world > 1 and backend == "nccl", device=coll_dev)

    head_cfg = args.config or 2
    tab, env, head = timed_config(head_cfg)
    N, A = head["n_envs_per_gpu"], head["n_agents"]
    stream = torch.cuda.current_stream()

    rollout = None
    if not args.no_rollout:
        env.reset()
        env.clear_stats()
        env.rollout(0, 0, 10)  # warm
        torch.cuda.synchronize()
        # T >= 1,000 steps per launch and the median of 3 launches: one 20-step launch (~10 us) after an idle gap
        # measured 67-134 G across boxes (clock ramp), which says nothing about the kernel
        T_r, times = max(K, 1000), []
        for i in range(3):
            r0, r1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            r0.record(stream)
            env.rollout(0, 10 + i * T_r, T_r)
            r1.record(stream)
            torch.cuda.synchronize()
            times.append(r0.elapsed_time(r1) / 1e3)
        rs = statistics.median(times)
        rollout = {"value": N * A * T_r / rs * world, "unit": "(env x agent)-steps/s", "steps_per_launch": T_r,
                   "note": "fused T-step rollout kernel (state in VGPRs, actions hashed in-kernel), secondary"}
    env.close()

    others = {}
    if args.config is None:  # every other BASELINE GPU config by the same protocol, on every rank
        for c in (3, 4, 5):
            t_c, e_c, o_c = timed_config(c)
            e_c.close()
            if rank == 0 and world == 1 and not args.no_cpu_baseline:  # the metric's parity rate for this config too
                o_c["parity"] = parity_sample(t_c, o_c["n_envs_per_gpu"], args.parity_steps, local)
            others[str(c)] = o_c
        if rank == 0 and world == 1 and args.dict_seconds > 0:  # BASELINE config 1: the dict API at N = 1
            others["1"] = dict_api_leg(local, args.dict_seconds)
    rs_legs = {}
    if args.config is None and not args.random_starts and args.rs_configs:
        # the FrozenLake configs with random_start_positions on (the reference runner's schedule): characterisation
        for c in (int(x) for x in args.rs_configs.split(",")):
            t_c, e_c, o_c = timed_config(c, random_starts=True)
            e_c.close()
            det = head if c == head_cfg else others.get(str(c))
            if det:
                o_c["vs_deterministic_event"] = o_c["us_per_step_event"] / det["us_per_step_event"]
            if rank == 0 and world == 1 and not args.no_cpu_baseline:
                o_c["parity"] = parity_sample(t_c, o_c["n_envs_per_gpu"], args.parity_steps, local)
            rs_legs[str(c)] = o_c

    # every rank's dispatch per config, into the collective block (one all_gather_object, after all timing)
    mine = {name: {"dispatch": o["dispatch"], "queue_counters": o["queue_counters"], "queue_state": o["queue_state"]}
            for name, o in [(str(head_cfg), head)] + list(others.items()) + [("rs" + k, v) for k, v in rs_legs.items()]
            if "dispatch" in o}
    attach_rank_dispatch(dist, world, coll, mine)

    large = None
    if args.large_envs > 0 and world == 1:  # single-GPU characterisation only
        large = bandwidth_regime(tab, args.large_envs, 20, local, head_cfg)

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        info = host_cpu()
        threads = args.cpu_threads or baseline_threads(info)
        cpu = cpu_baseline(tab, 65536, args.cpu_seconds, threads, info)
        if threads != 1:
            cpu["single_thread"] = cpu_baseline(tab, 8192, args.cpu_seconds / 2, 1, info)
        parity = parity_sample(tab, N, args.parity_steps, local)

    if rank == 0:
        detail = assemble_detail(args, world, head_cfg, head, others, rs_legs, coll, cpu, parity, rollout, large,
                                 pinned)
        print(json.dumps(compact_line(detail, write_detail(detail, args.detail, world))), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def _dry_result(cfg_id, n, A, world, wall_s, ar_s, K):
    """A timed_config-shaped record for the dry run (no GPU: the window is the collective sequence itself)."""
    B = algorithmic_bytes_per_instance_step(A, cfg_id == 5)
    wall_s = max(wall_s, 1e-9)
    per = wall_s / max(K, 1)
    roof = {"bound": "hbm", "achieved": n * A * B / per / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": n * A * B / per / 1e9 / HBM_PEAK_GBS, "traffic": None, "frac_counter": None,
            "traffic_source": {"summary": "dry-run", "commit": None, "src": None, "kern": None, "same_build": None,
                               "same_kernels": None},
            "bytes_per_launch": n * A * B, "bytes_per_instance_step": B, "avg_launch_us": per * 1e6,
            "avg_launch_us_profile": per * 1e6, "frac_profile": n * A * B / per / 1e9 / HBM_PEAK_GBS,
            "avg_launch_us_sq": None, "frac_sq": None, "chain_launch_us": per * 1e6,
            "floor": {"null_us": 0.0, "copy_step_io_us": 0.0, "copy_gather_us": 0.0, "frac_of_gather_floor": 0.0,
                      "source": "dry-run"}, "kernel": "dry-run"}
    return {"config": cfg_id, "workload": WORKLOADS.get(cfg_id, "dry-run"), "n_envs_per_gpu": n,
            "n_envs_total": world * n, "n_agents": A, "rm_states": 4, "kernel": "dry-run",
            "value": world * n * A / per, "unit": "(env x agent)-steps/s", "ms_per_step": per * 1e3,
            "us_per_step_event": per * 1e6, "allreduce_us": ar_s * 1e6,
            "value_with_allreduce": world * n * A * K / (wall_s + ar_s), "report_fused": True, "dispatch": "dry-run",
            "queue_error": None, "queue_counters": {}, "queue_state": "unused",
            "windows": [{"seed": s, "us_per_step_wall": per * 1e6, "allreduce_us": ar_s * 1e6} for s in WINDOW_SEEDS],
            "event_windows": [{"seed": s, "us_per_step_event": per * 1e6, "us_per_step_wall": per * 1e6}
                              for s in WINDOW_SEEDS],
            "roofline": roof, "episode_stats": {"episodes": 0.0, "mean_return_per_agent_episode": 0.0,
                                                "successes": 0.0, "mean_length": 0.0},
            "parity": {"rate": None, "exact": 0, "instance_steps": 0, "sample": "dry-run"}}


def dry_run(args, rank, world):
    """The launcher / process-group / reporting path without any GPU work, through the calls the GPU run makes:
    collective_block (all_gather), barrier, aligned_start (MAX), the statistics all-reduce (rmx.dist.allreduce_stats)
    and the window's max over ranks (rmx.dist.max_over_ranks), every tensor on the collective device as the RCCL run
    has it on its GPU (here gloo's: the host, so no copy is made, exactly as under RCCL); then the per-rank dispatch
    rows, the detail file and the compact line of a full run (every config, random-start legs, collective), marked
    dry_run with `value` null."""
    import torch
    import torch.distributed as dist

    from rmx import dist as RD

    if world > 1:
        RD.init("gloo")
    dev = RD.collective_device("gloo" if world > 1 else "none", 0)
    offset, n = RD.shard(world * args.n_envs, world, rank)
    # fake devices: one per rank (or all the same with --dry-run-same-device, checked as under RCCL)
    fake = {"pci": "0000:00:00" if args.dry_run_same_device else f"0000:{0x10 + rank:02x}:00",
            "uuid": "fake-0" if args.dry_run_same_device else f"fake-{rank}", "name": "dry-run", "device_index": rank}
    coll = collective_block(dist if world > 1 else None, "gloo" if world > 1 else "none", rank, world, rank, fake,
                            offset, n, strict=args.dry_run_same_device, device=dev)
    st = torch.tensor([1.0, float(rank + 1), 0.0, float(n)], dtype=torch.float64, device=dev)
    skew = None
    if world > 1:
        dist.barrier()
        target = aligned_start(dev)
        skew = time.perf_counter() - target  # how late after the agreed instant this rank started
    t0 = time.perf_counter()
    if rank == args.fail_rank:
        print(f"bench.py rank {rank}: --fail-rank: exiting mid-window", file=sys.stderr, flush=True)
        rank_status(rank, False, "--fail-rank")
        os._exit(3)  # dies without leaving the process group, as a crashed rank would
    wall = time.perf_counter() - t0
    ta = time.perf_counter()
    RD.allreduce_stats(st, dev)
    t_ar = time.perf_counter() - ta
    wall, t_ar = RD.max_over_ranks([wall, t_ar], dev)
    # the per-rank dispatch rows as the GPU run gathers them, one per config leg (no queue here: marked dry-run)
    q0 = {"windows": 0, "uploads": 0, "packets": 0, "stream_windows": 0, "recordings": 0}
    attach_rank_dispatch(dist if world > 1 else None, world, coll, {
        k: {"dispatch": "dry-run", "queue_counters": dict(q0), "queue_state": "unused"}
        for k in ("2", "3", "4", "5", "rs2", "rs4")})
    shards = [torch.zeros(2, dtype=torch.int64, device=dev) for _ in range(world)]
    if world > 1:
        dist.all_gather(shards, torch.tensor([offset, n], dtype=torch.int64, device=dev))
    else:
        shards = [torch.tensor([offset, n])]
    if rank == 0:
        K = args.steps
        head = _dry_result(2, n, 2, world, wall, t_ar, K)
        others = {str(c): _dry_result(c, n, A, world, wall, t_ar, K) for c, A in ((3, 1), (4, 4), (5, 3))}
        others["1"] = {"config": 1, "value": 0.0, "us_per_env_step": 0.0, "vs_reference_loop": None,
                       "vs_reference_loop_scaled": None, "engine": "dry-run", "reference_loop": {"value": None},
                       "gpu_sync": {"value": 0.0, "us_per_env_step": 0.0}, "parity": {"rate": None}}
        rs = {c: dict(_dry_result(int(c), n, A, world, wall, t_ar, K), vs_deterministic_event=1.0)
              for c, A in (("2", 2), ("4", 4))}
        cpu = {"value": 0.0, "unit": "(env x agent)-steps/s", "cores": 1, "kind": "port",
               "host": host_cpu(), "sample": "dry-run", "single_thread": {"value": 0.0}}
        detail = assemble_detail(args, world, 2, head, others, rs, coll, cpu, head["parity"], None, None, None)
        line = compact_line(detail, write_detail(detail, args.detail, world))
        line.update(value=None, dry_run=True, shards=[s.tolist() for s in shards], stats_allreduced=st.tolist(),
                    aligned_start_late_s=skew)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
