"""Cost of the one-launch statistics report inside bench.py's short window (diagnostic, GPU box).
Config 2, 65,536 envs, K graph-replayed steps, then per window (21 windows, medians printed):
  wall     graph(K steps); stats launch; device sync                  (bench.py's wall window)
  ev       the same with HIP events around the steps and around the report
  chain    one event pair around 20 back-to-back reports (latency of one report in a dependent chain)
Run once per library build (RMX_LIB=...) for a same-box A/B."""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))
import torch  # noqa: E402

from rmx import tables as T  # noqa: E402
from rmx.engine import VecRMEnv  # noqa: E402


def set_device_flags(flags):
    """hipSetDeviceFlags on the HIP runtime torch loaded, before the device is initialised (1 = spin-wait,
    2 = yield, 4 = blocking sync); returns the library path used."""
    import ctypes
    torch.zeros(1)  # loads torch's HIP runtime without initialising a device
    path = next(l.split()[-1] for l in open("/proc/self/maps") if "libamdhip64" in l)
    rc = ctypes.CDLL(path).hipSetDeviceFlags(ctypes.c_uint(flags))
    assert rc == 0, rc
    return path


def main():
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    if os.environ.get("RMX_PROBE_DEVFLAGS"):
        print(json.dumps({"device_flags": int(os.environ["RMX_PROBE_DEVFLAGS"]),
                          "hip": set_device_flags(int(os.environ["RMX_PROBE_DEVFLAGS"]))}), flush=True)
    W = 5
    tab = T.compile_scenario(T.baseline_scenario(2))
    env = VecRMEnv(tab, 65536, device=0, with_renv=False, with_env_done=True)
    st = torch.cuda.current_stream()
    acts = env.fill_actions(0, 0, W + K)
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()
    s0.wait_stream(st)
    with torch.cuda.stream(s0):
        with torch.cuda.graph(g, stream=s0):
            for s in range(K):
                env.step(acts[W + s])
    st.wait_stream(s0)
    g.replay()
    torch.cuda.synchronize()
    ref = None
    walls, evs_steps, evs_stats, chains = [], [], [], []
    for w in range(21):
        for events in (False, True):
            env.reset()
            env.clear_stats()
            for s in range(W):
                env.step(acts[s])
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if events:
                ev[0].record(st)
            g.replay()
            if events:
                ev[1].record(st)
            out = env.stats_tensor()
            if events:
                ev[2].record(st)
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e6
            if events:
                evs_steps.append(ev[0].elapsed_time(ev[1]) * 1e3)
                evs_stats.append(ev[1].elapsed_time(ev[2]) * 1e3)
            else:
                walls.append(wall)
            v = out.cpu().numpy().tolist()
            ref = ref or v
            assert v == ref, (v, ref)  # every window replays the same actions: the same report, bit for bit
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(20):
            env.stats_tensor()
        e1.record(st)
        torch.cuda.synchronize()
        chains.append(e0.elapsed_time(e1) * 1e3 / 20)
    env.check_errors()
    print(json.dumps({"lib": os.path.basename(os.environ.get("RMX_LIB", "librmx.so")), "K": K,
                      "devflags": os.environ.get("RMX_PROBE_DEVFLAGS", ""),
                      "wall_us": statistics.median(walls), "wall_us_per_step": statistics.median(walls) / K,
                      "ev_steps_us": statistics.median(evs_steps), "ev_stats_us": statistics.median(evs_stats),
                      "chain_stats_us": statistics.median(chains), "stats": ref}), flush=True)


if __name__ == "__main__":
    main()
