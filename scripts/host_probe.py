"""Where the host time of a 20-step window goes: graph.replay() call time, synchronise latency, and alternatives
(hipGraphLaunch through ctypes on the raw exec handle, stream vs device synchronise).  Config 2, 65,536 envs."""
import ctypes
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "multiagent-rl-rm_amd"))


def main():
    import torch

    from rmx import tables as T
    from rmx.engine import VecRMEnv

    K, reps = 20, 41
    tab = T.compile_scenario(T.baseline_scenario(2))
    env = VecRMEnv(tab, 65536, with_renv=False)
    acts = env.fill_actions(0, 0, K)
    out = torch.zeros(4, dtype=torch.float64, device="cuda")
    g = torch.cuda.CUDAGraph()
    s0 = torch.cuda.Stream()
    s0.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s0):
        with torch.cuda.graph(g, stream=s0):
            for s in range(K - 1):
                env.step(acts[s])
            env.step_report(acts[K - 1], out=out)
    torch.cuda.current_stream().wait_stream(s0)
    g.replay()
    torch.cuda.synchronize()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipGraphLaunch.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    hip.hipStreamSynchronize.argtypes = [ctypes.c_void_p]
    hip.hipDeviceSynchronize.argtypes = []
    stream = torch.cuda.current_stream()
    sptr = ctypes.c_void_p(stream.cuda_stream)
    exec_h = None
    try:
        exec_h = ctypes.c_void_p(g.raw_cuda_graph_exec())
    except Exception as ex:  # noqa: BLE001
        print("no raw exec:", ex, file=sys.stderr)
    t_end = time.perf_counter() + 0.3
    while time.perf_counter() < t_end:
        g.replay()
        torch.cuda.synchronize()

    def measure(launch, sync):
        walls, calls = [], []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            launch()
            t1 = time.perf_counter()
            sync()
            t2 = time.perf_counter()
            walls.append((t2 - t0) * 1e6)
            calls.append((t1 - t0) * 1e6)
        return {"wall_us": round(statistics.median(walls), 2), "launch_call_us": round(statistics.median(calls), 2)}

    res = {}
    for rnd in range(2):
        res[f"torch_replay+torch_sync#{rnd}"] = measure(g.replay, torch.cuda.synchronize)
        res[f"torch_replay+stream_sync#{rnd}"] = measure(g.replay, stream.synchronize)
        res[f"torch_replay+hipDeviceSync#{rnd}"] = measure(g.replay, hip.hipDeviceSynchronize)
        if exec_h is not None:
            res[f"hipGraphLaunch+torch_sync#{rnd}"] = measure(lambda: hip.hipGraphLaunch(exec_h, sptr),
                                                             torch.cuda.synchronize)
            res[f"hipGraphLaunch+hipStreamSync#{rnd}"] = measure(lambda: hip.hipGraphLaunch(exec_h, sptr),
                                                                lambda: hip.hipStreamSynchronize(sptr))
        # an empty window: the synchronise round trip alone
        res[f"sync_only#{rnd}"] = measure(lambda: None, torch.cuda.synchronize)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
